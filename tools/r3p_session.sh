set -u
A="--steps 20 --warmup 5 --no-cpu-baseline"
export OUT=r3p SKIP="smoke" PYTEST_ARGS="tests/test_dense_gpu.py tests/test_pipeline_gpu.py"
export RUNS="c4:$A|c4g2@ASR_PIPELINE_GSPLIT=0.2:$A|c4g4@ASR_PIPELINE_GSPLIT=0.4:$A|g256:--global-batch 256 $A|g256p4:--global-batch 256 --prod-streams 4 $A|g256g0@ASR_PIPELINE_GSPLIT=0:--global-batch 256 $A|g512:--global-batch 512 $A|g1024:--global-batch 1024 $A|g1024g0@ASR_PIPELINE_GSPLIT=0:--global-batch 1024 $A"
bash tools/gpu_check.sh
