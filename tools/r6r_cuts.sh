# 256 per GPU / C2 / 512 per GPU: T-segment boundaries (ASR_PIPELINE_CUTS), paired on one box
set -u
O=gpurun_out/${OUT:-r6r}; mkdir -p $O
run() {  # name, env, args
  n=$1; shift; e=$1; shift
  env $e timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-serialized > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));s=d['stages'];print('$n', round(d['value']/1e6,1), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"
}
run g256_s2 X=0 --batch 256
run g256_s3 X=0 --batch 256 --segments 3
run g256_c25_75 ASR_PIPELINE_CUTS=0.25,0.75 --batch 256 --segments 3
run g256_c2_8 ASR_PIPELINE_CUTS=0.2,0.8 --batch 256 --segments 3
run g256_c3_7 ASR_PIPELINE_CUTS=0.3,0.7 --batch 256 --segments 3
run g256_s4 X=0 --batch 256 --segments 4
run g256_c4 ASR_PIPELINE_CUTS=0.15,0.5,0.85 --batch 256 --segments 4
run g256_s2b X=0 --batch 256
run g256_c25_75b ASR_PIPELINE_CUTS=0.25,0.75 --batch 256 --segments 3
run c2_s2 X=0 --config C2
run c2_c25_75 ASR_PIPELINE_CUTS=0.25,0.75 --config C2 --segments 3
run g512_s4 X=0 --batch 512
run g512_c4 ASR_PIPELINE_CUTS=0.15,0.45,0.8 --batch 512 --segments 4
