#!/bin/bash
# Decoder wave-0 issue priority A/B (libasr_amd_prio{1,3}.so vs the product).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g56
mkdir -p $O
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -8 $O/b.log; exit 1; }; echo "${ASR_LIB:-prod} $* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["gather"]["digest"])')"; }
for L in libasr_amd.so libasr_amd_prio1.so libasr_amd_prio3.so; do
  export ASR_LIB=$L
  run --inflight 1 --steps 40
  run --steps 100
  run --config C3 --steps 10
done
