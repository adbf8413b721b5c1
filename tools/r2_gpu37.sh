#!/bin/bash
# Narrow-output streaming GEMM (emission projection): parity + A/B timing.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g37
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dense_gpu.py tests/test_dropin.py > $O/pytest.log 2>&1 || { echo "pytest failed $?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -5 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["gather"]["digest"], d["mfma"])')"; }
run
ASR_GEMM_NARROW=0 run
run --config BL --steps 20
ASR_GEMM_NARROW=0 run --config BL --steps 20
