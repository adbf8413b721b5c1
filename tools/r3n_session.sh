set -u
export OUT=r3n SKIP="smoke" PYTEST_ARGS="tests/test_dense_gpu.py tests/test_pipeline_gpu.py tests/test_bench_pipeline_gpu.py"
export RUNS="c4:--steps 20 --warmup 5 --no-cpu-baseline|c4nofuse@ASR_PIPELINE_FUSE=0:--steps 20 --warmup 5 --no-cpu-baseline|c4g2@ASR_PIPELINE_GSPLIT=0.2:--steps 20 --warmup 5 --no-cpu-baseline|c4g3@ASR_PIPELINE_GSPLIT=0.3:--steps 20 --warmup 5 --no-cpu-baseline|c4g4@ASR_PIPELINE_GSPLIT=0.4:--steps 20 --warmup 5 --no-cpu-baseline"
bash tools/gpu_check.sh
