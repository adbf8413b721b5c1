#!/bin/bash
# Default 8-wave D=3: production split all vs prod (after the recurrence fix).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g55
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -8 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], c["inflight_decodes"], c["decode_waves"])')"; }
run --steps 20 --warmup 5 --prod-split all
run --steps 20 --warmup 5 --prod-split prod
run --steps 100 --prod-split all
run --steps 100 --prod-split prod
run --steps 20 --warmup 5 --inflight 2
