# One A/B sweep on the GPU box (edit RUNS per experiment; the runs and their
# results are recorded in profiles/<round>/bench_scan.md).
set -u
A="--steps 20 --warmup 5 --no-cpu-baseline"
export OUT=${OUT:-ab} SKIP="smoke pytest"
export RUNS=${RUNS:-"c4:$A|c4g35@ASR_PIPELINE_GSPLIT=0.35:$A|c4g4@ASR_PIPELINE_GSPLIT=0.4:$A|c4g25@ASR_PIPELINE_GSPLIT=0.25:$A|c4b:$A|g256:--global-batch 256 $A|g512:--global-batch 512 $A|g1024:--global-batch 1024 $A"}
bash tools/gpu_check.sh
