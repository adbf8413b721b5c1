#!/bin/bash
# Two 4-wave decode workgroups per CU (--waves 4, 32-CU decode groups) x D groups.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g47
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -8 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["inflight_decodes"], d["gather"]["digest"])')"; }
run
run --waves 4
run --waves 4 --decode-cus 32 --inflight 3
run --waves 4 --decode-cus 32 --inflight 4
run --waves 4 --decode-cus 32 --inflight 6
run --waves 4 --decode-cus 32 --inflight 5
run --decode-cus 32 --inflight 6
