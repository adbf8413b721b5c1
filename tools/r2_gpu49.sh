#!/bin/bash
# Packed decode auto policy: default bench x2, short bench, pipeline parity test, trace.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g49
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -8 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], c["inflight_decodes"], c["decode_waves"], c["decode_cus_per_batch"], d["gather"]["digest"])')"; }
run
run
run --steps 20 --warmup 3
run --steps 300
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bench_pipeline_gpu.py > $O/pipe.log 2>&1 || { echo "pipe test failed"; tail -20 $O/pipe.log; exit 1; }
tail -1 $O/pipe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
python3 -c "
import csv
for r in csv.reader(open('$O/trace/run_kernel_stats.csv')): print(r[0][:50], r[1], r[3])"
