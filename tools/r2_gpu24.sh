#!/bin/bash
# Wide kernel: parity, C5 timing and phase clocks.
set -u
O=gpurun_out/r2g24
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ctc_wide_gpu.py tests/test_ctc_cu_semantics.py tests/test_ctc_timesteps_gpu.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/ctc_profile.py --waves 8 --cases c5 --sigmas bench,3,0.5 --reps 2 > $O/c5.log 2>&1 || { echo "c5 failed"; tail -5 $O/c5.log; exit 1; }
grep -v amdgpu $O/c5.log
ASR_LIB=libasr_amd_stamps.so timeout -k 10 300 python tools/ctc_profile.py --stamps --waves 8 --cases c5 --sigmas bench --reps 1 > $O/st.log 2>&1 || { echo "stamps failed"; tail -5 $O/st.log; exit 1; }
grep -v amdgpu $O/st.log
