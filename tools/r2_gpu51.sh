#!/bin/bash
# Packed decode: first timed run vs priming length (driver shape: 20 steps, warmup 5).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g51
mkdir -p $O
run() { ASR_BENCH_REPEAT=2 timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2> $O/e.log || { echo "bench $* failed"; tail -8 $O/e.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], c["inflight_decodes"], c["decode_waves"])') | $(grep repeat $O/e.log | tr '\n' ' ')"; }
run --steps 20 --warmup 5
ASR_BENCH_PRIME=30 run --steps 20 --warmup 5
ASR_BENCH_PRIME=60 run --steps 20 --warmup 5
run --steps 20 --warmup 40
run --steps 20 --warmup 5 --inflight 4 --waves 4 --decode-cus 32 --prod-split norec
run --steps 20 --warmup 5 --inflight 3 --waves 4 --decode-cus 32 --prod-split norec
