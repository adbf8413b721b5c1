#!/bin/bash
# One-wave decoder (ctc_wave_kernel.inc v2): parity, then throughput vs the 4-wave kernel.
set -u
O=gpurun_out/${OUT:-r3d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ctc_list_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_list.log 2>&1; rc=$?; tail -15 $O/pytest_list.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/occupancy_sweep.py --T 300 --k ${SWEEP_K:-1,2,4,8,12} --waves ${SWEEP_W:-4,-1} > $O/sweep.log 2>&1; rc=$?; grep '^{' $O/sweep.log; exit $rc
