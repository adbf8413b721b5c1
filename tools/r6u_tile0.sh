# C5: the wide decoder's first-tile precompute on the production stream
# (default) vs ahead of each decode launch (ASR_PIPELINE_TILE0_PROD=0), paired;
# then the pipeline / full-config / wide GPU tests
set -u
O=gpurun_out/${OUT:-r6u}; mkdir -p $O
run() {  # name, env, args
  n=$1; shift; e=$1; shift
  env $e timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-serialized > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));s=d['stages'];print('$n', round(d['value']/1e6,3), s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), s.get('steady_ms_per_step'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"
}
run c5_prod X=0 --config C5
run c5_dec ASR_PIPELINE_TILE0_PROD=0 --config C5
run c5_prod2 X=0 --config C5
run c5_dec2 ASR_PIPELINE_TILE0_PROD=0 --config C5
run c5_prod_d4 X=0 --config C5 --inflight 4
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_pipeline_gpu.py tests/test_full_configs_gpu.py tests/test_ctc_wide_gpu.py tests/test_ctc_segment_gpu.py > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -2 $O/pt.log
