# Round 6: large-K split-bf16 GEMM — accuracy / M-independence tests, timing vs fp32, then C5 / BL lines
set -u
O=gpurun_out/${OUT:-r6c}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dense_x3_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_x3.log 2>&1
rc=$?; tail -3 $O/pytest_x3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/gemm_largek_time.py > $O/gemm_time.log 2>&1
rc=$?; grep -v amdgpu.ids $O/gemm_time.log; [ $rc -eq 0 ] || exit $rc
A="--no-cpu-baseline --no-serialized"
OUT=${OUT:-r6c} BENCH_LIMIT=240 RUNS="c5:--config C5 $A|bl:--config BL $A" bash tools/bench_matrix.sh
