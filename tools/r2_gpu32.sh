#!/bin/bash
# In-flight decode groups with primed handles: C2 / C5 lines + rocprofv3 stats of C2.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g32
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -5 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["inflight_decodes"], d["gather"]["digest"])')"; }
run
run --steps 10
run --steps 300
run --inflight 2
run --config C5 --steps 20
run --config C3 --steps 20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
find $O -name "*stats*.csv" | while read f; do echo "== $f"; cut -d, -f1-8 "$f" | head -12; done
