#!/bin/bash
# Wide-kernel (C5) phase clocks from the stamps build.
set -u
O=gpurun_out/r2g21
mkdir -p $O
ASR_LIB=libasr_amd_stamps.so timeout -k 10 300 python tools/ctc_profile.py --stamps --waves 8 --cases c5 --sigmas bench,3 --reps 1 > $O/stamps.log 2>&1 || { echo "stamps failed"; tail -5 $O/stamps.log; exit 1; }
grep -v amdgpu $O/stamps.log
