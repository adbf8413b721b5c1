# The one-launch recurrence at two workgroups per CU (ASR_RP_PER_CU=2, 64 KB
# LDS each): alone, its fault tests, and C5 with three / four decode groups
set -u
O=gpurun_out/${OUT:-r6aa}; mkdir -p $O
timeout -k 10 200 python -u tools/step_time.py 32:1024:2000 64:1024:1000 > $O/step1.log 2>&1 || { tail $O/step1.log; exit 1; }
ASR_RP_PER_CU=2 timeout -k 10 200 python -u tools/step_time.py 32:1024:2000 64:1024:1000 > $O/step2.log 2>&1 || { tail $O/step2.log; exit 1; }
echo "1 per CU"; grep '^{' $O/step1.log; echo "2 per CU"; grep '^{' $O/step2.log
ASR_RP_PER_CU=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_gpu.py tests/test_pipeline_gpu.py -k "persist" > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
run() {  # name, env, args
  n=$1; shift; e=$1; shift
  env $e timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-serialized > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));s=d['stages'];print('$n', round(d['value']/1e6,3), s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), s.get('steady_ms_per_step'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"
}
run c5 X=0 --config C5
run c5_rp2 ASR_RP_PER_CU=2 --config C5
run c5_rp2_d4 ASR_RP_PER_CU=2 --config C5 --inflight 4
run c5_rp2_d5 ASR_RP_PER_CU=2 --config C5 --inflight 5
run c5b X=0 --config C5
