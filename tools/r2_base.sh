set -u
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1 || { echo "pytest failed $?"; tail -20 gpurun_out/r2a/pytest.log; exit 1; }
tail -2 gpurun_out/r2a/pytest.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/r2a/bench.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 gpurun_out/r2a/bench.log
ASR_LIB=libasr_amd_wstamps.so timeout -k 10 200 python tools/ctc_profile.py --wstamps --waves 8 --cases c2,c3 --reps 2 > gpurun_out/r2a/wstamps.log 2>&1
grep -v amdgpu gpurun_out/r2a/wstamps.log
