#!/bin/bash
# Packed first-run penalty: idle before the timed region / longer warmups.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g58
mkdir -p $O
run() { ASR_BENCH_REPEAT=1 timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2> $O/e.log || { echo "bench $* failed"; tail -8 $O/e.log; exit 1; }; echo "${ASR_BENCH_SLEEP:-0} $* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])') | $(grep repeat $O/e.log | tr '\n' ' ')"; }
run --packed --steps 20 --warmup 5
ASR_BENCH_SLEEP=0.1 run --packed --steps 20 --warmup 5
ASR_BENCH_SLEEP=0.5 run --packed --steps 20 --warmup 5
run --packed --steps 20 --warmup 10
run --packed --steps 20 --warmup 20
run --packed --steps 40 --warmup 5
