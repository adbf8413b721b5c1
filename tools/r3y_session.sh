set -u
mkdir -p gpurun_out/r3y
timeout -k 10 400 python -u -m pytest tests/test_dense_gpu.py -k "step or h2048 or c5_hidden or graph" -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r3y/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3y/pytest.log
[ $rc -le 1 ] || exit $rc
for nt in 1 2 4; do ASR_RNN_STEP_NT=$nt timeout -k 10 120 python tools/rnn_profile.py --T 200 --B 256 --H 2048 --reps 3 >> gpurun_out/r3y/rnn_bl.log 2>&1 || exit $?; done
for nt in 1 2; do ASR_RNN_STEP_NT=$nt timeout -k 10 120 python tools/rnn_profile.py --T 2000 --B 32 --H 1024 --reps 3 >> gpurun_out/r3y/rnn_c5.log 2>&1 || exit $?; done
cat gpurun_out/r3y/rnn_bl.log gpurun_out/r3y/rnn_c5.log | grep rnn_fwd
A="--steps 10 --warmup 3 --no-cpu-baseline"
export OUT=r3y SKIP="smoke pytest"
export RUNS="bl:--config BL $A|c5:--config C5 --steps 30 --warmup 3 --no-cpu-baseline|c5nt2@ASR_RNN_STEP_NT=2:--config C5 --steps 30 --warmup 3 --no-cpu-baseline|c5d3nt2@ASR_RNN_STEP_NT=2:--config C5 --inflight 3 --prod-streams 3 --steps 30 --warmup 3 --no-cpu-baseline"
bash tools/gpu_check.sh
