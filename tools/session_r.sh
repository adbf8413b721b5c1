# A/B: s_setprio forms in the split-bf16 GEMM / recurrence (dvariants p1, p2); the decoder's two-copy
# selection histogram (cvariant h2): decoder timing at 16 per CU, its parity tests, C4 lines.
O=gpurun_out/${OUT:-sr}; mkdir -p $O
timeout -k 10 300 python tools/dense_time.py base p1 p2 > $O/dense.jsonl 2>&1; cat $O/dense.jsonl | cut -c1-400
for lib in libasr_amd.so libasr_amd_cv_h2.so; do
  ASR_LIB=$lib timeout -k 10 200 python tools/ctc_profile.py --waves -1 --cases s4096,s768 --sigmas bench,3 --reps 3 > $O/ctc_$lib.jsonl 2>&1; echo $lib; cat $O/ctc_$lib.jsonl
done
ASR_LIB=libasr_amd_cv_h2.so timeout -k 10 600 python -u -m pytest tests/test_ctc_gpu.py tests/test_ctc_list_gpu.py tests/test_ctc_segment_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_h2.log 2>&1; tail -2 $O/pytest_h2.log
for rep in a b; do
  for lib in libasr_amd.so libasr_amd_cv_h2.so; do
    ASR_LIB=$lib timeout -k 10 200 python bench.py --no-serialized > $O/c4_${lib}_$rep.json 2> $O/c4_${lib}_$rep.err
    python -c "import json;d=json.load(open('$O/c4_${lib}_$rep.json'));print('c4 $lib $rep', d['value'], d['parity']['match'], d['stages']['decode_span_ms_per_batch'], d['stages']['production_ms_per_batch'])"
  done
done
