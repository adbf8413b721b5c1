set -u
A="--steps 60 --warmup 5 --no-cpu-baseline"
export OUT=r3v SKIP="smoke pytest"
export RUNS="g256a:--global-batch 256 $A|g256d6a:--global-batch 256 --inflight 6 --decode-partition 96 $A|g256d5a:--global-batch 256 --inflight 5 --decode-partition 80 $A|g256b:--global-batch 256 $A|g256d6b:--global-batch 256 --inflight 6 --decode-partition 96 $A|g256d5b:--global-batch 256 --inflight 5 --decode-partition 80 $A|g512a:--global-batch 512 $A|g512d3a:--global-batch 512 --inflight 3 --decode-partition 96 $A|g512b:--global-batch 512 $A|g512d3b:--global-batch 512 --inflight 3 --decode-partition 96 $A"
bash tools/gpu_check.sh
