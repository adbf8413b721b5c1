#!/bin/bash
# Marginal phase costs by ablation builds (timing only; results are wrong):
#   abl2 no orphan tables, abl4 selection run twice, abl16 candidates (P1) twice.
set -u
O=gpurun_out/${R2OUT:-r2abl}
mkdir -p $O
for L in libasr_amd.so libasr_amd_abl2.so libasr_amd_abl4.so libasr_amd_abl16.so; do
  ASR_LIB=$L timeout -k 10 200 python tools/ctc_profile.py --waves 8 --cases c2,c3 --sigmas bench --reps 3 > $O/timing_$L.log 2>&1 || { echo "timing $L failed"; tail -5 $O/timing_$L.log; exit 1; }
  grep -hv amdgpu $O/timing_$L.log | cut -c1-150 | sed "s/^/$L /"
done
echo done
