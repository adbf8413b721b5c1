set -u
mkdir -p gpurun_out/r3x
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3x/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3x/pytest.log
[ $rc -le 1 ] || exit $rc
A="--steps 20 --warmup 5 --no-cpu-baseline"
export OUT=r3x SKIP="smoke pytest"
export RUNS="c3:--config C3 $A|c3nofuse@ASR_PIPELINE_FUSE=0:--config C3 $A|c3p1:--config C3 --prod-streams 1 $A|bl:--config BL --steps 10 --warmup 3 --no-cpu-baseline|blp1:--config BL --prod-streams 1 --steps 10 --warmup 3 --no-cpu-baseline"
bash tools/gpu_check.sh
OUT=r3x_bl BENCH_ARGS="--config BL --steps 6 --warmup 2 --no-cpu-baseline" PASSES="trace" bash tools/profile_bench.sh || exit $?
OUT=r3x_c3 BENCH_ARGS="--config C3 --steps 10 --warmup 3 --no-cpu-baseline" PASSES="trace" bash tools/profile_bench.sh || exit $?
