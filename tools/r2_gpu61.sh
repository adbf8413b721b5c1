#!/bin/bash
# 8-wave decoder under a 4-waves-per-SIMD register budget (128 VGPRs, 13 spilled):
# two 8-wave workgroups per CU (--decode-cus 32) x D groups.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g61
mkdir -p $O
export ASR_LIB=libasr_amd_wpe4.so
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "bench $* failed"; tail -8 $O/b.log; exit 1; }; echo "$* :: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], c["inflight_decodes"], d["gather"]["digest"])')"; }
run --inflight 1 --steps 40
run --steps 100
run --decode-cus 32 --inflight 4 --prod-split norec --steps 100
run --decode-cus 32 --inflight 5 --prod-split norec --steps 100
run --decode-cus 32 --inflight 5 --prod-split norec --steps 20 --warmup 5
