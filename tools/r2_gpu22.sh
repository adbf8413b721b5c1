#!/bin/bash
# Wide kernel with the precomputed first-tile threshold: parity, C5 timing
# and phase clocks with/without it; then the bench overlap comparison.
set -u
O=gpurun_out/r2g22
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ctc_wide_gpu.py tests/test_ctc_cu_semantics.py tests/test_ctc_timesteps_gpu.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for F in 1 0; do
  ASR_CTC_TILE0=$F timeout -k 10 300 python tools/ctc_profile.py --waves 8 --cases c5 --sigmas bench,3 --reps 2 > $O/c5_t$F.log 2>&1 || { echo "c5 $F failed"; tail -5 $O/c5_t$F.log; exit 1; }
  echo "tile0=$F"; grep -v amdgpu $O/c5_t$F.log
  ASR_CTC_TILE0=$F ASR_LIB=libasr_amd_stamps.so timeout -k 10 300 python tools/ctc_profile.py --stamps --waves 8 --cases c5 --sigmas bench --reps 1 > $O/st_t$F.log 2>&1 || { echo "stamps $F failed"; tail -5 $O/st_t$F.log; exit 1; }
  grep -v amdgpu $O/st_t$F.log
done
bash tools/r2_gpu20.sh
