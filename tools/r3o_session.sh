set -u
A="--steps 20 --warmup 5 --no-cpu-baseline"
export OUT=r3o SKIP="smoke" PYTEST_ARGS="tests/test_dense_gpu.py tests/test_pipeline_gpu.py"
export RUNS="c4:$A|c4g3@ASR_PIPELINE_GSPLIT=0.3:$A|c4g4@ASR_PIPELINE_GSPLIT=0.4:$A|c4g5@ASR_PIPELINE_GSPLIT=0.5:$A|c4g6@ASR_PIPELINE_GSPLIT=0.6:$A|g256:--global-batch 256 $A|g256q16@GPU_MAX_HW_QUEUES=16:--global-batch 256 $A|g256g4q16@GPU_MAX_HW_QUEUES=16,ASR_PIPELINE_GSPLIT=0.4:--global-batch 256 $A|g512q16@GPU_MAX_HW_QUEUES=16:--global-batch 512 $A|g1024g4@ASR_PIPELINE_GSPLIT=0.4:--global-batch 1024 $A"
bash tools/gpu_check.sh
