set -u
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py tests/test_bench_pipeline_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/occupancy_sweep.py --T 300 --k 1,2,3,4,6,8,12,16 --waves -1 > $O/sweep.log 2>&1 || exit $?; grep '^{' $O/sweep.log | cut -c1-160
OUT=r3j RUNS='c4||--steps 20 --warmup 5 --no-cpu-baseline;g1024||--global-batch 1024 --steps 20 --warmup 5 --no-cpu-baseline;g512||--global-batch 512 --steps 20 --warmup 5 --no-cpu-baseline;g256||--global-batch 256 --steps 20 --warmup 5 --no-cpu-baseline;g256d6||--global-batch 256 --steps 20 --warmup 5 --no-cpu-baseline --inflight 6;c2||--config C2 --steps 20 --warmup 5 --no-cpu-baseline' bash tools/ab_runs.sh
