# C2 on the chip-filling schedule by default: pipeline + bench-pipeline tests, C2 and C4 lines with parity.
O=gpurun_out/${OUT:-si}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pipeline_gpu.py tests/test_bench_pipeline_gpu.py > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --config C2 > $O/c2.json 2> $O/c2.err; echo "c2 rc=$?"
python -c "import json;d=json.load(open('$O/c2.json'));print('c2', d['value'], d['ms_per_step'], d['parity'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py > $O/c4.json 2> $O/c4.err; echo "c4 rc=$?"
python -c "import json;d=json.load(open('$O/c4.json'));print('c4', d['value'], d['ms_per_step'], d['parity']['match'], d['roofline']['serialized']['ms_per_launch'])"
