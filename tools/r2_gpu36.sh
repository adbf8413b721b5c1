#!/bin/bash
# Recurrence with buffer loads/stores (no wait on the h_t store per step).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g36
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dense_gpu.py tests/test_dropin.py > $O/pytest.log 2>&1 || { echo "pytest failed $?"; tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -5 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["inflight_decodes"], d["gather"]["digest"])')"; }
run
run --inflight 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
python3 -c "
import csv
for r in csv.reader(open('$O/trace/run_kernel_stats.csv')): print(r[0][:40], r[1], r[3])"
