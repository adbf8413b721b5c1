set -u
mkdir -p gpurun_out/r3r
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_pipeline_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3r/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r3r/pytest.log
[ $rc -le 1 ] || exit $rc
for rb in 1 2; do
  ASR_RNN_RB=$rb timeout -k 10 120 python tools/emit_profile.py --B 2048 >> gpurun_out/r3r/emit.log 2>&1 || exit $?
  ASR_RNN_RB=$rb timeout -k 10 120 python tools/emit_profile.py --B 256 >> gpurun_out/r3r/emit.log 2>&1 || exit $?
done
cat gpurun_out/r3r/emit.log
A="--steps 20 --warmup 5 --no-cpu-baseline"
export OUT=r3r SKIP="smoke pytest"
export RUNS="c4rb1@ASR_RNN_RB=1:$A|c4rb2@ASR_RNN_RB=2:$A|g256rb2@ASR_RNN_RB=2:--global-batch 256 $A|g1024rb2@ASR_RNN_RB=2:--global-batch 1024 $A"
bash tools/gpu_check.sh
