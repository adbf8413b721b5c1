#!/bin/bash
# GEMM K-stage change + list selection A/B: parity of both selections, decoder
# timings, critical-path wave stamps and selection counters, bench lines.
set -u
O=gpurun_out/r2g2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_ctc_gpu.py tests/test_ctc_batch_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_sel0.log 2>&1 || { echo "pytest sel0 failed"; tail -30 $O/pytest_sel0.log; exit 1; }
tail -1 $O/pytest_sel0.log
ASR_CTC_SEL=1 timeout -k 10 600 python -u -m pytest tests/test_ctc_gpu.py tests/test_ctc_batch_gpu.py tests/test_full_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_sel1.log 2>&1 || { echo "pytest sel1 failed"; tail -30 $O/pytest_sel1.log; exit 1; }
tail -1 $O/pytest_sel1.log
for S in 0 1; do
  ASR_CTC_SEL=$S timeout -k 10 200 python tools/ctc_profile.py --waves 8 --cases c2,c3 --sigmas bench,3 --reps 3 > $O/timing_sel$S.log 2>&1 || { echo "timing $S failed"; tail -5 $O/timing_sel$S.log; exit 1; }
  ASR_CTC_SEL=$S ASR_LIB=libasr_amd_wstamps.so timeout -k 10 200 python tools/ctc_profile.py --wstamps --waves 8 --cases c2 --sigmas bench --reps 2 > $O/wstamps_sel$S.log 2>&1 || { echo "wstamps $S failed"; tail -5 $O/wstamps_sel$S.log; exit 1; }
  ASR_CTC_SEL=$S ASR_LIB=libasr_amd_stamps.so timeout -k 10 200 python tools/ctc_profile.py --stamps --waves 8 --cases c2 --sigmas bench --reps 2 > $O/stamps_sel$S.log 2>&1 || { echo "stamps $S failed"; tail -5 $O/stamps_sel$S.log; exit 1; }
done
grep -hv amdgpu $O/timing_sel*.log | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_sel0.log 2>&1 || { echo "bench 0 failed"; tail -5 $O/bench_sel0.log; exit 1; }
ASR_CTC_SEL=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_sel1.log 2>&1 || { echo "bench 1 failed"; tail -5 $O/bench_sel1.log; exit 1; }
tail -1 $O/bench_sel0.log | cut -c1-200; tail -1 $O/bench_sel1.log | cut -c1-200
echo done
