set -u
mkdir -p gpurun_out/r3ai
for L in libasr_amd.so libasr_amd_wf1.0_0.25.so libasr_amd_wf0.9_0.2.so libasr_amd_wf1.3_0.5.so; do
  ASR_LIB=$L timeout -k 10 200 python tools/ctc_profile.py --waves -1 --cases s4096 --sigmas bench,3 --reps 3 > gpurun_out/r3ai/prof_$L.log 2>&1 || exit $?
  echo "$L $(grep '^{' gpurun_out/r3ai/prof_$L.log | python3 -c 'import sys,json; print([ (json.loads(l)["sigma"], json.loads(l)["kernel_ms_min"]) for l in sys.stdin])')"
done
A="--steps 20 --warmup 5 --no-cpu-baseline"
export OUT=r3ai SKIP="smoke pytest"
export RUNS="c4:$A|c4wf10@ASR_LIB=libasr_amd_wf1.0_0.25.so:$A|c4wf09@ASR_LIB=libasr_amd_wf0.9_0.2.so:$A|c4wf13@ASR_LIB=libasr_amd_wf1.3_0.5.so:$A"
bash tools/gpu_check.sh
