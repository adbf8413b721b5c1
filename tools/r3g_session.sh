set -u
mkdir -p gpurun_out/r3g
OUT=r3g PYTEST_LIMIT=700 bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python -u tools/occupancy_sweep.py --T 300 --k 1,2,4,6,8,12,16 --waves -1 > gpurun_out/r3g/sweep.log 2>&1 || exit $?; grep '^{' gpurun_out/r3g/sweep.log | cut -c1-200
OUT=r3g RUNS='c4||--steps 20 --warmup 5 --no-cpu-baseline;c2||--config C2 --steps 20 --warmup 5 --no-cpu-baseline;g1024||--global-batch 1024 --steps 20 --warmup 5 --no-cpu-baseline;g512||--global-batch 512 --steps 20 --warmup 5 --no-cpu-baseline;g256||--global-batch 256 --steps 20 --warmup 5 --no-cpu-baseline;g256w|ASR_CTC_WAVES=-1|--global-batch 256 --steps 20 --warmup 5 --no-cpu-baseline' bash tools/ab_runs.sh
