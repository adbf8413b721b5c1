#!/bin/bash
# 2-rank rehearsal on one GPU (ranks wrap around) of the in-flight bench
# (C2 weak, C4 strong with host gather verified against a 1-GPU decode),
# then rocprofv3 kernel trace + stats of the default C2 bench.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g39
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 30 > $O/bench_n2.log 2>&1 || { echo "n2 failed"; tail -20 $O/bench_n2.log; exit 1; }
grep '^{' $O/bench_n2.log | tail -1 > $O/rehearsal_c2.json; cut -c1-200 $O/rehearsal_c2.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c4_n2.log 2>&1 || { echo "c4 n2 failed"; tail -20 $O/bench_c4_n2.log; exit 1; }
grep '^{' $O/bench_c4_n2.log | tail -1 > $O/rehearsal_c4.json; cut -c1-200 $O/rehearsal_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
tail -1 $O/trace.log | cut -c1-120
python3 -c "
import csv
for r in csv.reader(open('$O/trace/run_kernel_stats.csv')): print(r[0][:50], r[1], r[3])"
