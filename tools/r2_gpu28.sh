#!/bin/bash
# Bench after queueing each decode before the next batch's production.
set -u
O=gpurun_out/r2g28
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -5 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"; }
run --cu-split fit
run --cu-split half
run --cu-split fit --overlap-results
run --cu-split half --overlap-results
run --config C5 --cu-split half --steps 20
run --config C5 --cu-split fit --steps 20
run --config C4 --cu-split fit
run --config C4 --cu-split half
run --config BL --cu-split fit
run --config BL --cu-split half
