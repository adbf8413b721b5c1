# Fragment-major P (ASR_PIPELINE_PFRAG) A/B: pipeline parity tests, C4 and 256 per GPU.
O=gpurun_out/${OUT:-se}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_pipeline_gpu.py tests/test_dense_x3_gpu.py tests/test_bench_pipeline_gpu.py > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -le 1 ] || exit $rc
run() { n=$1; shift; env $ENVV timeout -k 10 200 python bench.py "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d['stages'];print('$n', d['value'], d['ms_per_step'], s['production_ms_per_batch'], s['decode_span_ms_per_batch'], s['steady_ms_per_step'], (d.get('parity') or {}).get('match'))" || echo "$n rc=$rc"; }
ENVV="ASR_PIPELINE_PFRAG=1" run on1
ENVV="ASR_PIPELINE_PFRAG=0" run off1 --no-cpu-baseline
ENVV="ASR_PIPELINE_PFRAG=1" run on2 --no-cpu-baseline
ENVV="ASR_PIPELINE_PFRAG=0" run off2 --no-cpu-baseline
ENVV="ASR_PIPELINE_PFRAG=1" run on256 --batch 256 --no-cpu-baseline
ENVV="ASR_PIPELINE_PFRAG=0" run off256 --batch 256 --no-cpu-baseline
