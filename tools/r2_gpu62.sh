#!/bin/bash
# Final-tree check: smoke, pytest -m gpu, the driver's bench command.
set -u
O=gpurun_out/r2g62
mkdir -p $O
BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" PYTEST_LIMIT=600 bash tools/gpu_check.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/bench.log $O/
