set -u
mkdir -p gpurun_out/r3c
OUT=r3c bash tools/r3d_session.sh || exit $?
timeout -k 10 300 python -u -m pytest tests/test_ctc_cu_semantics.py tests/test_dense_gpu.py tests/test_ctc_wide_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3c/pytest.log; [ $rc -le 1 ] || exit $rc
for pk in 0 1; do ASR_RNN_PK=$pk timeout -k 10 120 python tools/rnn_recur_sweep.py --T 500 --B 64,256 > gpurun_out/r3c/rnn_pk$pk.log 2>&1 || exit $?; grep '^{' gpurun_out/r3c/rnn_pk$pk.log; done
OUT=r3c RUNS='c2n||--config C2 --steps 20 --warmup 5 --no-cpu-baseline;c2m|ASR_PIPELINE_MASKALL=1|--config C2 --steps 20 --warmup 5 --no-cpu-baseline;c2py||--config C2 --py-pipeline --steps 20 --warmup 5 --no-cpu-baseline' bash tools/ab_runs.sh || exit $?
OUT=c2n BENCH_ARGS='--config C2 --steps 20 --warmup 5 --no-cpu-baseline' PASSES=trace bash tools/profile_bench.sh
