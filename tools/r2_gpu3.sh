#!/bin/bash
# Selection A/B (0 one-decider, 1 list, 2 all-wave 64-bin histogram) with the
# wave index made uniform; parity of mode 2; timings; stamps; bench.
set -u
O=gpurun_out/r2g3
mkdir -p $O
ASR_CTC_SEL=2 timeout -k 10 600 python -u -m pytest tests/test_ctc_gpu.py tests/test_ctc_batch_gpu.py tests/test_ctc_list_gpu.py tests/test_full_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_sel2.log 2>&1 || { echo "pytest sel2 failed"; tail -30 $O/pytest_sel2.log; exit 1; }
tail -1 $O/pytest_sel2.log
for S in 0 2 1; do
  ASR_CTC_SEL=$S timeout -k 10 200 python tools/ctc_profile.py --waves 8 --cases c2,c3 --sigmas bench,3 --reps 3 > $O/timing_sel$S.log 2>&1 || { echo "timing $S failed"; tail -5 $O/timing_sel$S.log; exit 1; }
done
for S in 0 2; do
  ASR_CTC_SEL=$S ASR_LIB=libasr_amd_wstamps.so timeout -k 10 200 python tools/ctc_profile.py --wstamps --waves 8 --cases c2 --sigmas bench --reps 2 > $O/wstamps_sel$S.log 2>&1 || { echo "wstamps $S failed"; tail -5 $O/wstamps_sel$S.log; exit 1; }
  ASR_CTC_SEL=$S ASR_LIB=libasr_amd_stamps.so timeout -k 10 200 python tools/ctc_profile.py --stamps --waves 8 --cases c2 --sigmas bench --reps 2 > $O/stamps_sel$S.log 2>&1 || { echo "stamps $S failed"; tail -5 $O/stamps_sel$S.log; exit 1; }
done
for S in 0 2 1; do grep -hv amdgpu $O/timing_sel$S.log | cut -c1-150 | sed "s/^/sel$S /"; done
ASR_CTC_SEL=2 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_sel2.log 2>&1 || { echo "bench 2 failed"; tail -5 $O/bench_sel2.log; exit 1; }
tail -1 $O/bench_sel2.log | cut -c1-200
echo done
