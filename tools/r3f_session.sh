set -u
mkdir -p gpurun_out/r3f
timeout -k 10 200 python -u -m pytest tests/test_ctc_cu_semantics.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3f/pytest.log; [ $rc -le 1 ] || exit $rc
ASR_PIPELINE_TRACE=1 ASR_BENCH_HOSTLOG=gpurun_out/r3f/hostlog_c2n.txt timeout -k 10 200 python bench.py --config C2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3f/bench_c2n.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r3f/bench_c2n.log | grep -v '^{' | tail -40; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3f/bench_c2n.log
