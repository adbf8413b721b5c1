# Decoder prefetch by buffer loads: parity, probe, C4 bench; decode-partition scan at 256 / 512 per GPU.
O=gpurun_out/${OUT:-sd}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_ctc_gpu.py tests/test_ctc_list_gpu.py tests/test_ctc_segment_gpu.py tests/test_pipeline_gpu.py > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/decode_cu_probe.py --T 300 --per-cu 8,16,32 > $O/probe.jsonl 2>&1; echo "probe rc=$?"; cat $O/probe.jsonl | grep per_cu
run() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d['stages'];print('$n', d['value'], d['ms_per_step'], s['steady_ms_per_step'], s['first_decode_start_ms'], s['last_production_end_ms'], s['last_decode_end_ms'], d['config']['inflight_decodes'], d['config']['production_streams'])" || echo "$n rc=$rc"; }
run c4
run c4b
run b256 --batch 256
run b256p144 --batch 256 --decode-partition 144
run b256p160 --batch 256 --decode-partition 160
run b512 --batch 512
run b512p144 --batch 512 --decode-partition 144
run b1024 --batch 1024
