set -u
export OUT=r3w PYTEST_LIMIT=900
export RUNS="c4:--steps 20 --warmup 5|c4s60:--steps 60 --warmup 5 --no-cpu-baseline|g256:--global-batch 256 --steps 20 --warmup 5 --no-cpu-baseline|g512:--global-batch 512 --steps 20 --warmup 5 --no-cpu-baseline|g1024:--global-batch 1024 --steps 20 --warmup 5 --no-cpu-baseline|c2:--config C2 --steps 20 --warmup 5 --no-cpu-baseline|c3:--config C3 --steps 20 --warmup 5 --no-cpu-baseline|c5:--config C5 --steps 10 --warmup 3 --no-cpu-baseline|bl:--config BL --steps 10 --warmup 3 --no-cpu-baseline"
bash tools/gpu_check.sh
