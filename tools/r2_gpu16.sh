#!/bin/bash
set -u
O=gpurun_out/r2g16
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-400
timeout -k 10 300 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { echo "bench c4 failed"; tail -5 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-300
echo done
