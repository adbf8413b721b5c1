#!/bin/bash
# C5 with production D+P-1 batches ahead: D = 2 / 3 / 4.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g60
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -8 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], c["inflight_decodes"], c["production_streams"], d["gather"]["digest"])')"; }
run --config C5 --steps 20
run --config C5 --steps 20 --inflight 3
run --config C5 --steps 20 --inflight 4
run --config C5 --steps 20 --inflight 3 --prod-streams 3
run --steps 20 --warmup 5
