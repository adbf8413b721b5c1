#!/bin/bash
# 2 decode workgroups per CU (--waves 4, 32-CU groups): D x production split.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g48
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -8 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["inflight_decodes"], d["gather"]["digest"])')"; }
W="--waves 4 --decode-cus 32"
run $W --inflight 4 --prod-split norec
run $W --inflight 5 --prod-split norec
run $W --inflight 4 --prod-split all
run $W --inflight 4 --prod-split prod
run $W --inflight 5 --prod-split prod
run $W --inflight 6 --prod-split norec
