# Round 6 final lines: smoke, the default bench line (CPU baseline + parity witness), C2, 256 per GPU
set -u
O=gpurun_out/${OUT:-r6k}; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c4.json 2> $O/bench_c4.err || { tail $O/bench_c4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c4.json'));print('c4', d['value'], d['parity'], d['cpu_baseline']['value'], d['roofline']['frac'], d['roofline']['serialized'])"
timeout -k 10 200 python bench.py --config C2 > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', d['value'], d['parity']['match'])"
timeout -k 10 200 python bench.py --batch 256 --no-cpu-baseline > $O/bench_g256.json 2> $O/bench_g256.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_g256.json'));print('g256', d['value'])"
