# Round-5 A/B session: dense kernel variants, decoder lse variants, parity tests, bench.
O=gpurun_out/${OUT:-sa}; mkdir -p $O
echo "== dense variants"; timeout -k 10 400 python tools/dense_time.py ${DV_LIST:-base pf pfsgb tanh pack tp} > $O/dense.jsonl 2>&1; echo rc=$?; cat $O/dense.jsonl | cut -c1-400
echo "== decoder probe"
for lib in libasr_amd.so libasr_amd_cv_ocml.so; do
  ASR_LIB=$lib timeout -k 10 200 python tools/decode_cu_probe.py --T 300 --per-cu 16,32 > $O/probe_$lib.jsonl 2>&1; echo "$lib rc=$?"; cat $O/probe_$lib.jsonl
done
echo "== ctc parity tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_ctc_gpu.py tests/test_ctc_list_gpu.py tests/test_ctc_segment_gpu.py tests/test_ctc_wide_gpu.py tests/test_ctc_batch_gpu.py tests/test_ctc_timesteps_gpu.py tests/test_ctc_cu_semantics.py > $O/pytest_ctc.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_ctc.log
[ $rc -le 1 ] || exit $rc
echo "== bench"
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err; echo "bench rc=$?"
python -c "import json;d=json.load(open('$O/bench.json'));s=d['stages'];print(d['value'], d['ms_per_step'], d['parity']['match'], s['production_ms_per_batch'], s['decode_span_ms_per_batch'], s['steady_ms_per_step'], d['clock']['gfxclk_mhz'])"
