#!/bin/bash
# C5 kernel trace (wide decoder + tile0 precompute under the CU groups).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g44
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --config C5 --steps 10 --warmup 3 > $O/trace.log 2>&1 || { echo "trace failed $?"; tail -5 $O/trace.log; exit 1; }
python3 -c "
import csv
for r in csv.reader(open('$O/trace/run_kernel_stats.csv')): print(r[0][:60], r[1], r[3])"
