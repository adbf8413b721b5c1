#!/bin/bash
# rocprofv3 evidence for bench.py on the GPU box (run from the repo root):
#   1. kernel trace + stats of a short bench run
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate: TCC slot limits)
#   4. SQ instruction/issue pass (8 SQ counters), 5. GRBM pass (clock)
# Each step under its own time limit; stop on the first failure.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_OUT:-r02prof}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || { echo "fetch pass failed $?"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || { echo "write pass failed $?"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 || { echo "sq pass failed $?"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/grbm -o run -- python3 bench.py $ARGS > $OUT/grbm.log 2>&1 || { echo "grbm pass failed $?"; exit 1; }
find $OUT -name "*.csv"
