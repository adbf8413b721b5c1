# C2 chip-filling schedule: decodes in flight, decode partition, hardware queues.
O=gpurun_out/${OUT:-sh}; mkdir -p $O
run() { n=$1; shift; env $ENVV timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized --config C2 "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d.get('stages') or {};c=d['config'];print('$n', d['value'], d['ms_per_step'], s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'), c.get('inflight_decodes'), c.get('production_streams'), c.get('decode_cus'), c.get('streams'), c.get('hw_queues'))" || { echo "$n rc=$rc"; tail -3 $O/b_$n.err; }; }
export ASR_PIPELINE_MODE=1
run d16p8 --inflight 16 --prod-streams 8
run d16p8c192 --inflight 16 --prod-streams 8 --decode-partition 192
run d12p8c192 --inflight 12 --prod-streams 8 --decode-partition 192
run d20p10q32 --inflight 20 --prod-streams 10 --hw-queues 32
run d20p10c192q32 --inflight 20 --prod-streams 10 --decode-partition 192 --hw-queues 32
run d22p8c192q32 --inflight 22 --prod-streams 8 --decode-partition 192 --hw-queues 32
ASR_PIPELINE_MODE=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized --hw-queues 32 > $O/b_c4q32.json 2>&1; python -c "import json;print('c4q32', json.load(open('$O/b_c4q32.json'))['value'])"
