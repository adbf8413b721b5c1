# Round 6 final evidence on the final tree: smoke, the whole GPU suite, the
# default bench line (CPU baseline + parity witness + serialized decode), C5,
# C2 and the 256-per-GPU shard
set -u
O=gpurun_out/${OUT:-r6bb}; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_c4.json 2> $O/bench_c4.err || { tail $O/bench_c4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c4.json'));r=d['roofline'];print('c4', d['value'], d['parity']['match'], d['cpu_baseline']['value'], r['frac'], r.get('serialized',{}).get('ms_per_launch'), r.get('serialized',{}).get('frac'))"
for a in "c5:--config C5 --no-cpu-baseline" "c2:--config C2" "g256:--batch 256 --no-cpu-baseline" "c3:--config C3 --no-cpu-baseline --no-serialized" "bl:--config BL --no-cpu-baseline --no-serialized"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python bench.py $args > $O/bench_$n.json 2> $O/bench_$n.err || { tail $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n', d['value'], (d.get('parity') or {}).get('match'))"
done
