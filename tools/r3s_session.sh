set -u
mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py -k "emit or mfma" -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3s/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3s/pytest.log
[ $rc -le 1 ] || exit $rc
for e in 0 1; do
  ASR_RNN_EMIT_EARLY=$e timeout -k 10 120 python tools/emit_profile.py --B 2048 >> gpurun_out/r3s/emit.log 2>&1 || exit $?
done
ASR_RNN_EMIT_EARLY=1 timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py -k "emit" -m gpu -q -x --timeout 120 --timeout-method thread >> gpurun_out/r3s/pytest.log 2>&1 || exit $?
cat gpurun_out/r3s/emit.log
A="--steps 20 --warmup 5 --no-cpu-baseline"
export OUT=r3s SKIP="smoke pytest"
export RUNS="c4:$A|c4early@ASR_RNN_EMIT_EARLY=1:$A"
bash tools/gpu_check.sh
