# C2 fill / drain: T-segments 2 / 3 / 4 / 5 and decodes in flight 10 / 12 (20 / 5), each twice.
O=gpurun_out/${OUT:-sp}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 150 python bench.py --config C2 --no-cpu-baseline --no-serialized "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d.get('stages') or {};c=d['config'];print('$n', d['value'], d['ms_per_step'], s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'), c.get('segments'), c.get('inflight_decodes'), c.get('production_streams'))" || { echo "$n rc=$rc"; tail -3 $O/b_$n.err; }; }
for rep in a b; do
  run s2$rep
  run s3$rep --segments 3
  run s4$rep --segments 4
  run s5$rep --segments 5
  run s4d12$rep --segments 4 --inflight 12
done
# C4 at 3 T-segments (2 is the default)
c4() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized "$@" > $O/c4_$n.json 2> $O/c4_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/c4_$n.json'));s=d.get('stages') or {};c=d['config'];print('c4 $n', d['value'], d['ms_per_step'], s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'), c.get('segments'))" || { echo "c4 $n rc=$rc"; tail -3 $O/c4_$n.err; }; }
for rep in a b; do c4 s2$rep; c4 s3$rep --segments 3; done
