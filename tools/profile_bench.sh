#!/bin/bash
# rocprofv3 evidence for one bench.py workload (run on the GPU box from the
# repo root).  Passes, each a separate run under its own time limit (counters
# never share a run with tracing; one block's slots per pass):
#   trace  kernel trace + stats
#   fetch  FETCH_SIZE            write  WRITE_SIZE
#   sq     8 SQ issue counters   grbm   GRBM_GUI_ACTIVE GRBM_COUNT
#   valu   VALU mix (fp64)       mfma   MFMA busy / instruction counters + GRBM
#   list   rocprofv3 -L (the counters this box offers)
# Stops at the first failing pass.  Summaries are made on the dev side:
#   tools/traffic_from_pmc.py, tools/issue_from_pmc.py -> profiles/<round>/
#
#   OUT=c4 BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline" PASSES="trace fetch write sq" \
#       bash tools/profile_bench.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_${OUT:-run}
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline --no-serialized"}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
# the decoder's VALU mix (fp64 share, VALU issue cycles) and the scalar unit
VALU="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES"
# matrix-core evidence of the dense kernels (+ the clock)
# (fp32 MFMAs: the fp32 kernels and the emission GEMM; bf16 MFMAs: the split-bf16 kernels, dense_x3.hip)
# where the decoder's waits go: LDS / VMEM / SMEM instruction
# cycles and LDS bank conflicts; then the issue side
WAIT="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_LDS_BANK_CONFLICT"
ISSUE="SQ_IFETCH SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_BUSY_CYCLES"
MFMA="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
for pass in ${PASSES:-trace fetch write}; do
    case $pass in
        trace) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
                   -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1 ;;
        fetch) timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
                   -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1 ;;
        write) timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
                   -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1 ;;
        sq)    timeout -s KILL 180 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/sq" -o run \
                   -- python3 bench.py $ARGS > "$OUT/sq.log" 2>&1 ;;
        list)  timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1 ;;
        valu)  timeout -s KILL 180 rocprofv3 --pmc $VALU --output-format csv -d "$OUT/valu" -o run \
                   -- python3 bench.py $ARGS > "$OUT/valu.log" 2>&1 ;;
        mfma)  timeout -s KILL 180 rocprofv3 --pmc $MFMA --output-format csv -d "$OUT/mfma" -o run \
                   -- python3 bench.py $ARGS > "$OUT/mfma.log" 2>&1 ;;
        wait)  timeout -s KILL 180 rocprofv3 --pmc $WAIT --output-format csv -d "$OUT/wait" -o run \
                   -- python3 bench.py $ARGS > "$OUT/wait.log" 2>&1 ;;
        issue) timeout -s KILL 180 rocprofv3 --pmc $ISSUE --output-format csv -d "$OUT/issue" -o run \
                   -- python3 bench.py $ARGS > "$OUT/issue.log" 2>&1 ;;
        grbm)  timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/grbm" -o run \
                   -- python3 bench.py $ARGS > "$OUT/grbm.log" 2>&1 ;;
        *) echo "unknown pass $pass"; exit 2 ;;
    esac
    rc=$?
    echo "pass $pass rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
find "$OUT" -name "*.csv"
