#!/bin/bash
# Round-2 stage 1 on the GPU box: new full-size config tests, bench lines
# (C2 headline, C4 strong at N=1), decoder statistics on the bench's
# emissions, then the rocprofv3 passes.  Each GPU step has its own limit.
set -u
O=gpurun_out/r2s1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_full_configs_gpu.py tests/test_ctc_gpu.py tests/test_dense_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed $?"; tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
grep -E "PASSED|FAILED" $O/pytest.log | grep -E "full_configs|overflow_retry|h2048" 
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -5 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log
timeout -k 10 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { echo "bench c4 failed"; tail -5 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log
ASR_LIB=libasr_amd_stamps.so timeout -k 10 200 python tools/ctc_profile.py --stamps --waves 8 --cases c2 --sigmas bench,3 --reps 2 > $O/stamps.log 2>&1 || { echo "stamps failed"; tail -5 $O/stamps.log; exit 1; }
grep -v amdgpu $O/stamps.log
PROF_OUT=r2s1/prof bash tools/profile_r02.sh > $O/prof.log 2>&1 || { echo "profile failed"; tail -5 $O/prof.log; exit 1; }
echo done
