#!/bin/bash
# In-flight decode groups (bench --inflight D): C2 / C5 sweeps.
set -u
O=gpurun_out/r2g31
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -5 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["gather"]["digest"])')"; }
run --inflight 1
run --inflight 2
run --inflight 3
run --inflight 3 --steps 300
run --config C5 --inflight 1 --steps 20
run --config C5 --inflight 2 --steps 20
run --config C5 --inflight 3 --steps 20
run --config C5 --inflight 4 --steps 20
