# C2 on the chip-filling schedule (one-wave decoder, many batches in flight) vs CU groups.
O=gpurun_out/${OUT:-sg}; mkdir -p $O
run() { n=$1; shift; env $ENVV timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized --config C2 "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d.get('stages') or {};c=d['config'];print('$n', d['value'], d['ms_per_step'], s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'), c.get('inflight_decodes'), c.get('production_streams'), c.get('segments'), c.get('decode_waves'))" || { echo "$n rc=$rc"; tail -3 $O/b_$n.err; }; }
ENVV= run groups
ENVV=ASR_PIPELINE_MODE=1 run shared
ENVV=ASR_PIPELINE_MODE=1 run shared_d6 --inflight 6
ENVV=ASR_PIPELINE_MODE=1 run shared_d12 --inflight 12 --prod-streams 10
ENVV=ASR_PIPELINE_MODE=1 run shared_s1 --segments 1
ENVV=ASR_PIPELINE_MODE=1 run shared_st60 --steps 60
