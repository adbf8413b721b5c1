# Round 6: large-K split GEMM, three-stage ring with fragments a chunk ahead vs two stages
set -u
O=gpurun_out/${OUT:-r6j}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dense_x3_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in libasr_amd.so libasr_amd_dv_x3k2.so libasr_amd.so libasr_amd_dv_x3k2.so; do
  echo $lib; ASR_LIB=$lib timeout -k 10 120 python tools/gemm_largek_time.py 2>&1 | grep -v amdgpu.ids || exit 1
done
A="--no-cpu-baseline --no-serialized"
OUT=${OUT:-r6j} BENCH_LIMIT=240 RUNS="c5:--config C5 $A|c5s2@ASR_LIB=libasr_amd_dv_x3k2.so:--config C5 $A|bl:--config BL $A|bls2@ASR_LIB=libasr_amd_dv_x3k2.so:--config BL $A" bash tools/bench_matrix.sh
