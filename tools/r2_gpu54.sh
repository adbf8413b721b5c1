#!/bin/bash
# Driver shape with GC off in the timed region: packed vs default.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g54
mkdir -p $O
run() { ASR_BENCH_REPEAT=1 timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2> $O/e.log || { echo "bench $* failed"; tail -8 $O/e.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], c["inflight_decodes"], c["decode_waves"])') | $(grep repeat $O/e.log | tr '\n' ' ')"; }
run --packed --steps 20 --warmup 5
run --packed --steps 20 --warmup 5
run --steps 20 --warmup 5
run --packed --steps 100 --warmup 5
