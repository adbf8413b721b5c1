# final validation: smoke, the whole GPU suite, the default bench line, C2
set -e
out=gpurun_out/${RUN:-fin6}
mkdir -p $out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python bench.py > $out/bench_c4.json 2> $out/bench_c4.err
python -c "import json;d=json.load(open('$out/bench_c4.json'));print('c4', d['value'], d['parity']['match'], d['cpu_baseline']['value'])"
timeout -k 10 150 python bench.py --config C2 > $out/bench_c2.json 2> $out/bench_c2.err
python -c "import json;d=json.load(open('$out/bench_c2.json'));print('c2', d['value'], d['parity']['match'])"
timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err
python -c "import json;d=json.load(open('$out/bench_c5.json'));print('c5', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --config BL --no-cpu-baseline > $out/bench_bl.json 2> $out/bench_bl.err
python -c "import json;d=json.load(open('$out/bench_bl.json'));print('bl', d['value'], d['ms_per_step'])"
