#!/bin/bash
# rocprofv3 kernel trace + stats of the packed-decode bench (100 steps, warmup 30).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g59
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --packed > $O/bench.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 $O/bench.log > $O/bench_c2_packed.json; cut -c1-140 $O/bench_c2_packed.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --packed > $O/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
python3 -c "
import csv
for r in csv.reader(open('$O/trace/run_kernel_stats.csv')): print(r[0][:50], r[1], r[3])"
