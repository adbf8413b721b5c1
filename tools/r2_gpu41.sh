#!/bin/bash
# C5: production replayed from HIP graphs (no per-launch host queueing).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g42
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -8 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["inflight_decodes"], d["config"]["production_streams"], d["gather"]["digest"])')"; }
run --config C5 --steps 20
run --config C5 --steps 20 --inflight 2 --prod-streams 1 --graph-production off
run --config C5 --steps 20 --inflight 3
run --config C5 --steps 20 --inflight 3 --prod-streams 3
run --config C5 --steps 20 --inflight 4 --prod-streams 3
run --config C5 --steps 20 --inflight 2 --prod-streams 1
run --steps 100
echo "GPU_MAX_HW_QUEUES in the box env: ${GPU_MAX_HW_QUEUES:-unset}"
