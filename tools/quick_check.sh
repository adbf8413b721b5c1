#!/bin/bash
# Decoder iteration on the GPU box: parity tests of the register kernel, then
# C2/C3 decode timings.  Each GPU step under its own limit; stop on failure.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ctc_gpu.py tests/test_ctc_batch_gpu.py tests/test_ctc_cu_semantics.py -m gpu -x -q --timeout 120 --timeout-method thread ${QC_PYTEST:-} > gpurun_out/qc_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/qc_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ctc_profile.py --waves ${QC_WAVES:-0,8} --cases ${QC_CASES:-c2,c3} --reps 3 > gpurun_out/qc_timing.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/qc_timing.log; exit $rc
