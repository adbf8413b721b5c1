#!/bin/bash
# Where the fixed cost of a short timed run goes: the same run(20) repeated.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g50
mkdir -p $O
run() { ASR_BENCH_REPEAT=4 timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2> $O/e.log || { echo "bench $* failed"; tail -8 $O/e.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], c["inflight_decodes"], c["decode_waves"])') | $(grep repeat $O/e.log | tr '\n' ' ')"; }
run --steps 20 --warmup 5
run --steps 20 --warmup 5 --inflight 3
run --steps 20 --warmup 5 --inflight 1
run --steps 100 --warmup 5
