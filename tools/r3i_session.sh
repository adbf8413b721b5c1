set -u
O=gpurun_out/${OUT:-r3i}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ctc_list_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
ASR_LIB=libasr_amd_stamps.so timeout -k 10 200 python tools/ctc_profile.py --stamps --waves -1 --cases s64,s4096 --sigmas bench --reps 1 > $O/stamps.log 2>&1; grep '^{' $O/stamps.log | cut -c 150-900
timeout -k 10 300 python -u tools/occupancy_sweep.py --T 300 --k 8,16 --waves -1 > $O/sweep.log 2>&1 || exit $?; grep '^{' $O/sweep.log | cut -c1-220
OUT=${OUT:-r3i} RUNS='c4||--steps 20 --warmup 5 --no-cpu-baseline' bash tools/ab_runs.sh
