set -u
A="--steps 20 --warmup 5 --no-cpu-baseline"
export OUT=r3u SKIP="smoke pytest"
export RUNS="g256w0@ASR_GEMM_WIDE=0:--global-batch 256 $A|g256w0d6@ASR_GEMM_WIDE=0:--global-batch 256 --inflight 6 --decode-partition 96 $A|g256w0g5@ASR_GEMM_WIDE=0,ASR_PIPELINE_GSPLIT=0.5:--global-batch 256 $A|g512w0@ASR_GEMM_WIDE=0:--global-batch 512 $A|g1024w0@ASR_GEMM_WIDE=0:--global-batch 1024 $A|c4w0@ASR_GEMM_WIDE=0:$A|g256:--global-batch 256 $A"
bash tools/gpu_check.sh
