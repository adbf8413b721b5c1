# Round 6: fragment-major A tile in the K <= 256 split GEMM vs the row-major (padded) tile
set -u
O=gpurun_out/${OUT:-r6i}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dense_x3_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/dense_time.py base rowmajor base rowmajor > $O/dense_time.log 2>&1
rc=$?; grep -v amdgpu.ids $O/dense_time.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
A="--no-cpu-baseline --no-serialized"
OUT=${OUT:-r6i} BENCH_LIMIT=200 RUNS="c4:$A|c4row@ASR_LIB=libasr_amd_dv_rowmajor.so:$A|g256:--batch 256 $A|g256row@ASR_LIB=libasr_amd_dv_rowmajor.so:--batch 256 $A|c4b:$A|c4rowb@ASR_LIB=libasr_amd_dv_rowmajor.so:$A" bash tools/bench_matrix.sh
