# C5 with the first-tile precompute on the production stream: T-segments 3,
# the drain hold, paired with the default
set -u
O=gpurun_out/${OUT:-r6v}; mkdir -p $O
run() {  # name, env, args
  n=$1; shift; e=$1; shift
  env $e timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-serialized > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));s=d['stages'];print('$n', round(d['value']/1e6,3), s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), s.get('steady_ms_per_step'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"
}
run c5 X=0 --config C5
run c5_s3 X=0 --config C5 --segments 3
run c5_drain ASR_PIPELINE_DRAIN=-1 --config C5
run c5_s3_drain ASR_PIPELINE_DRAIN=-1 --config C5 --segments 3
run c5b X=0 --config C5
