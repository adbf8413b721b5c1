set -u
mkdir -p gpurun_out/r3ad
for L in libasr_amd.so libasr_amd_wnl6.so libasr_amd_wnl4.so libasr_amd_wnl3.so; do
  ASR_LIB=$L timeout -k 10 200 python tools/ctc_profile.py --waves -1 --cases s4096 --sigmas bench,3 --reps 3 > gpurun_out/r3ad/prof_$L.log 2>&1 || exit $?
  echo "$L $(grep '^{' gpurun_out/r3ad/prof_$L.log | python3 -c 'import sys,json; print([ (json.loads(l)["sigma"], json.loads(l)["kernel_ms_min"]) for l in sys.stdin])')"
done
ASR_LIB=libasr_amd_wnl4.so timeout -k 10 400 python -u -m pytest tests/test_ctc_list_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r3ad/pytest_wnl4.log 2>&1
echo "pytest wnl4 rc=$?"; tail -2 gpurun_out/r3ad/pytest_wnl4.log
A="--steps 20 --warmup 5 --no-cpu-baseline"
export OUT=r3ad SKIP="smoke pytest"
export RUNS="c4:$A|c4wnl4@ASR_LIB=libasr_amd_wnl4.so:$A|c4wnl3@ASR_LIB=libasr_amd_wnl3.so:$A|c4b:$A|c4wnl4b@ASR_LIB=libasr_amd_wnl4.so:$A"
bash tools/gpu_check.sh
