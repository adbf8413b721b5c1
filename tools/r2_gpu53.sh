#!/bin/bash
# Kernel trace of the packed bench at the driver shape (first timed run slow).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g53
mkdir -p $O
ASR_BENCH_REPEAT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --packed --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace failed $?"; tail -5 $O/trace.log; exit 1; }
grep -E "repeat|^\{" $O/trace.log | cut -c1-200
