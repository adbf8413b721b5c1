#!/bin/bash
# V=4096 parity: current library, without the tile-0 precompute, previous commit.
set -u
O=gpurun_out/r2g25
mkdir -p $O
T="tests/test_ctc_wide_gpu.py -k 4096"
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread $T -m gpu > $O/cur.log 2>&1; echo "cur rc=$?"; tail -2 $O/cur.log
ASR_CTC_TILE0=0 timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread $T -m gpu > $O/t0off.log 2>&1; echo "t0off rc=$?"; tail -2 $O/t0off.log
ASR_LIB=libasr_amd_prev.so timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread $T -m gpu > $O/prev.log 2>&1; echo "prev rc=$?"; tail -2 $O/prev.log
ASR_LIB=libasr_amd_prev.so ASR_CTC_TILE0=0 timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread $T -m gpu > $O/prevoff.log 2>&1; echo "prevoff rc=$?"; tail -2 $O/prevoff.log
