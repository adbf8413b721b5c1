#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench on one GPU (ranks wrap around):
# weak scaling (C2) and C4 strong scaling, host gather + 1-GPU verification.
set -u
O=gpurun_out/r2g18
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 2 > $O/bench_n2.log 2>&1 || { echo "n2 failed"; tail -20 $O/bench_n2.log; exit 1; }
grep '"metric"' $O/bench_n2.log | cut -c1-300
grep -o '"gather": {[^}]*}' $O/bench_n2.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c4_n2.log 2>&1 || { echo "c4 n2 failed"; tail -20 $O/bench_c4_n2.log; exit 1; }
grep '"metric"' $O/bench_c4_n2.log | cut -c1-300
grep -o '"gather": {[^}]*}' $O/bench_c4_n2.log
echo done
