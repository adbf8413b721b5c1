#!/bin/bash
# Split production (recurrence stream + GEMM stream one batch ahead), 8 HW queues.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g34
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dense_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed $?"; tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -5 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["inflight_decodes"], d["gather"]["digest"])')"; }
run --warmup 30 --prod-split off
run --warmup 30 --prod-split prod
run --warmup 30 --prod-split all
run --warmup 30 --prod-split prod --inflight 2
run --config C5 --steps 20 --inflight 3
run --config C5 --steps 20 --inflight 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --warmup 30 > $O/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
echo done
