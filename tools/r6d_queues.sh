# Round 6: the whole GPU suite and the bench lines at the environment's
# hardware-queue count (no override: HIP's default 4 on the box)
set -u
O=gpurun_out/${OUT:-r6d}; mkdir -p $O
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
A="--no-cpu-baseline --no-serialized"
OUT=${OUT:-r6d} BENCH_LIMIT=240 RUNS="c4:$A|g256:--batch 256 $A|g512:--batch 512 $A|g1024:--batch 1024 $A|c2:--config C2 $A|c3:--config C3 $A|c3d5:--config C3 --inflight 5 --prod-streams 5 $A|c5:--config C5 $A|bl:--config BL $A" bash tools/bench_matrix.sh
