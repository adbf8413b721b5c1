# Counter passes of the split-bf16 production kernels alone (tools/gemm_probe.py) on 128 CUs.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-sq5}; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS"
P3="SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/gemm_probe.py 3 both > $O/trace.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/p1 -o run -- python3 tools/gemm_probe.py 3 both > $O/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $O/p2 -o run -- python3 tools/gemm_probe.py 3 both > $O/p2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $P3 --output-format csv -d $O/p3 -o run -- python3 tools/gemm_probe.py 3 both > $O/p3.log 2>&1
echo rc=$?
