#!/bin/bash
# Re-entry GPU pass at HEAD: smoke + pytest -m gpu + default bench, then the
# C4/C5/BL bench lines as JSON under gpurun_out/r2g30/.
set -u
O=gpurun_out/r2g30
mkdir -p $O
PYTEST_LIMIT=600 bash tools/gpu_check.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/bench.log $O/ 2>/dev/null
for c in C4 C5 BL; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} > $O/bench_$c.log 2>&1 || { echo "bench $c failed $?"; tail -5 $O/bench_$c.log; exit 1; }
  tail -1 $O/bench_$c.log > $O/bench_$c.json; echo "$c :: $(cut -c1-160 $O/bench_$c.json)"
done
