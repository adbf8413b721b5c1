#!/bin/bash
set -u
O=gpurun_out/r2g14
mkdir -p $O
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default_$i.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_default_$i.log; exit 1; }
tail -1 $O/bench_default_$i.log | cut -c1-230
timeout -k 10 300 python bench.py --no-cpu-baseline --overlap-results > $O/bench_overlap_$i.log 2>&1 || { echo "bench overlap failed"; tail -5 $O/bench_overlap_$i.log; exit 1; }
tail -1 $O/bench_overlap_$i.log | cut -c1-230
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --warmup 5 --overlap-results > $O/bench_overlap_long.log 2>&1 || exit 1
tail -1 $O/bench_overlap_long.log | cut -c1-230
echo done
