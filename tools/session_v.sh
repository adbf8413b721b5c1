# C5 with the one-launch recurrence: decodes in flight / production streams scan, and the step-launch A/B.
O=gpurun_out/${OUT:-sv}; mkdir -p $O
c5() { n=$1; shift; env $ENVV timeout -k 10 300 python bench.py --no-cpu-baseline --no-serialized --config C5 "$@" > $O/c5_$n.json 2> $O/c5_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/c5_$n.json'));c=d['config'];s=d.get('stages') or {};print('c5 $n', d['value'], d['ms_per_step'], c.get('inflight_decodes'), c.get('production_streams'), c.get('decode_cus'), s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))" || { echo "c5 $n rc=$rc"; tail -3 $O/c5_$n.err; }; }
ENVV=ASR_RNN_PERSIST=0 c5 off_d2 --steps 10 --warmup 3
ENVV= c5 on_d2 --steps 10 --warmup 3
ENVV= c5 on_d3 --steps 10 --warmup 3 --inflight 3
ENVV= c5 on_d4 --steps 10 --warmup 3 --inflight 4
ENVV= c5 on_d3p3 --steps 10 --warmup 3 --inflight 3 --prod-streams 3
ENVV= c5 on_d4p3 --steps 10 --warmup 3 --inflight 4 --prod-streams 3
ENVV= c5 on_d5 --steps 10 --warmup 3 --inflight 5
