#!/bin/bash
# Full pass at the split-production / in-flight bench: smoke, pytest -m gpu,
# default bench (CPU baseline included), C3/C4/C5/BL lines, rocprofv3 trace +
# PMC passes of the default C2 bench.
set -u
O=gpurun_out/r2g38
mkdir -p $O
BENCH_ARGS=" " PYTEST_LIMIT=600 bash tools/gpu_check.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/bench.log $O/
tail -1 $O/bench.log > $O/bench_C2.json
for c in "C5" "C5 --prod-split all" "C4" "BL" "C3"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --steps 30 > $O/bench_$n.log 2>&1 || { echo "bench $c failed $?"; tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log > $O/bench_$n.json; echo "$c :: $(cut -c1-100 $O/bench_$n.json | cut -d, -f2,6)"
done
