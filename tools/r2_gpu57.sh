#!/bin/bash
# Round-2 closing pass: smoke, pytest -m gpu, the driver's bench shape
# (20 steps / warmup 5, CPU baseline included), 100-step line, rocprofv3
# kernel trace + stats of the driver shape.
set -u
O=gpurun_out/r2g57
mkdir -p $O
BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" PYTEST_LIMIT=600 bash tools/gpu_check.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/bench.log $O/
tail -1 $O/bench.log > $O/bench_C2_driver_shape.json
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > $O/bench_100.log 2>&1 || { echo "100-step bench failed"; exit 1; }
tail -1 $O/bench_100.log > $O/bench_C2_100.json; cut -c1-120 $O/bench_C2_100.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
python3 -c "
import csv
for r in csv.reader(open('$O/trace/run_kernel_stats.csv')): print(r[0][:50], r[1], r[3])"
