#!/bin/bash
# Driver-shape bench (20 steps, warmup 5) at the default config, packed opt-in, pipeline parity test.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g52
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -8 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], c["inflight_decodes"], c["decode_waves"], d["gather"]["digest"])')"; }
run --gpus 1 --steps 20 --warmup 5
run --gpus 1 --steps 20 --warmup 5
run --packed --steps 100
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bench_pipeline_gpu.py > $O/pipe.log 2>&1 || { echo "pipe test failed"; tail -20 $O/pipe.log; exit 1; }
tail -1 $O/pipe.log
