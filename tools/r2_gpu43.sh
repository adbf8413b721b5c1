#!/bin/bash
# Final round-2 pass: smoke, pytest -m gpu, default bench (CPU baseline), short
# bench (driver-like small warmup), C3/C4/C5/BL lines, rocprofv3 trace + PMC.
set -u
O=gpurun_out/r2g43
mkdir -p $O
BENCH_ARGS=" " PYTEST_LIMIT=600 bash tools/gpu_check.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/bench.log $O/
tail -1 $O/bench.log > $O/bench_C2.json
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_short.log 2>&1 || { echo "short bench failed"; exit 1; }
echo "short :: $(tail -1 $O/bench_short.log | cut -c1-160)"
for c in C5 C4 BL C3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --steps 30 > $O/bench_$c.log 2>&1 || { echo "bench $c failed $?"; tail -5 $O/bench_$c.log; exit 1; }
  tail -1 $O/bench_$c.log > $O/bench_$c.json
done
PROF_OUT=r2g43prof BENCH_ARGS="--no-cpu-baseline" bash tools/profile_r02.sh
