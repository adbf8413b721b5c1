# C5 with the one-launch recurrence and T-segments: the default 20 / 5 line, decodes in flight 3 / 4; BL.
O=gpurun_out/${OUT:-sy}; mkdir -p $O
c5() { n=$1; shift; timeout -k 10 600 python bench.py --config C5 "$@" > $O/c5_$n.json 2> $O/c5_$n.err; python -c "import json;d=json.load(open('$O/c5_$n.json'));c=d['config'];s=d.get('stages') or {};print('c5 $n', d['value'], d['ms_per_step'], c.get('segments'), c.get('inflight_decodes'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'), (d.get('cpu_baseline') or {}).get('value'))"; }
c5 def
c5 d4 --inflight 4 --no-cpu-baseline --no-serialized
c5 d4s4 --inflight 4 --segments 4 --no-cpu-baseline --no-serialized
c5 s4 --segments 4 --no-cpu-baseline --no-serialized
timeout -k 10 300 python bench.py --config BL --no-cpu-baseline > $O/bl.json 2> $O/bl.err; python -c "import json;d=json.load(open('$O/bl.json'));print('bl', d['value'], d['ms_per_step'])"
