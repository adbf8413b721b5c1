set -u
A="--steps 20 --warmup 5 --no-cpu-baseline"
export OUT=r3q SKIP="smoke pytest"
export RUNS="g256:--global-batch 256 $A|g256d7:--global-batch 256 --inflight 7 --decode-partition 112 $A|g256d6:--global-batch 256 --inflight 6 --decode-partition 96 $A|g512:--global-batch 512 $A|g512d3:--global-batch 512 --inflight 3 --decode-partition 96 $A|g512d3p6:--global-batch 512 --inflight 3 --prod-streams 6 --decode-partition 96 $A|g1024:--global-batch 1024 $A|g1024p4:--global-batch 1024 --prod-streams 4 $A|c4g25@ASR_PIPELINE_GSPLIT=0.25:$A|c4g35@ASR_PIPELINE_GSPLIT=0.35:$A"
bash tools/gpu_check.sh
mkdir -p gpurun_out/r3q
ASR_LIB=libasr_amd_stamps.so timeout -k 10 200 python tools/ctc_profile.py --stamps --waves -1 --cases s4096 --sigmas bench --reps 2 > gpurun_out/r3q/stamps_s4096.log 2>&1
echo "stamps rc=$?"
