# One-launch recurrence and T-segments (wide decoder) in the pipeline: segment tests, pipeline / full-config / dense tests, C5 at the default 20 / 5 with its
# parity witness, and C5 at 10 / 3 (the earlier lines' shape).
O=gpurun_out/${OUT:-sw}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_ctc_segment_gpu.py tests/test_pipeline_gpu.py tests/test_full_configs_gpu.py tests/test_dense_gpu.py tests/test_bench_pipeline_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; echo pytest rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config C5 > $O/c5.json 2> $O/c5.err; python -c "import json;d=json.load(open('$O/c5.json'));c=d['config'];s=d.get('stages') or {};print('c5', d['value'], d['ms_per_step'], c.get('inflight_decodes'), (d.get('parity') or {}).get('match'), (d.get('cpu_baseline') or {}).get('value'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline --no-serialized > $O/c5_10.json 2> $O/c5_10.err; python -c "import json;d=json.load(open('$O/c5_10.json'));print('c5_10', d['value'], d['ms_per_step'], d['config'].get('inflight_decodes'))"
