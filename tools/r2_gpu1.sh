#!/bin/bash
# Round-2 GPU pass 1: the whole -m gpu suite (incl. the full-size C3/C4/C5/BL
# tests), bench lines (C2 headline, C4 strong at N=1, C5, BL), then the
# rocprofv3 passes of the C2 bench.  Each GPU step has its own limit; the
# script stops at the first failure.
set -u
O=gpurun_out/r2g1
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed $?"; tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -5 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log
timeout -k 10 300 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { echo "bench c4 failed"; tail -5 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.log 2>&1 || { echo "bench c5 failed"; tail -5 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log
timeout -k 10 300 python bench.py --config BL --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_bl.log 2>&1 || { echo "bench bl failed"; tail -5 $O/bench_bl.log; exit 1; }
tail -1 $O/bench_bl.log
ASR_LIB=libasr_amd_wstamps.so timeout -k 10 200 python tools/ctc_profile.py --wstamps --waves 8 --cases c2,c3 --sigmas bench,3 --reps 2 > $O/wstamps.log 2>&1 || { echo "wstamps failed"; tail -5 $O/wstamps.log; exit 1; }
PROF_OUT=r2g1/prof bash tools/profile_r02.sh > $O/prof.log 2>&1 || { echo "profile failed"; tail -5 $O/prof.log; exit 1; }
echo done
