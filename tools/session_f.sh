# 256-per-GPU shard schedule scan (production streams, decodes in flight, segments, tiled production GEMM) + C2.
O=gpurun_out/${OUT:-sf}; mkdir -p $O
run() { n=$1; shift; env $ENVV timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d.get('stages') or {};c=d['config'];print('$n', d['value'], d['ms_per_step'], s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'), c.get('inflight_decodes'), c.get('production_streams'), c.get('segments'))" || echo "$n rc=$rc"; }
ENVV= run base --batch 256
ENVV= run p6 --batch 256 --prod-streams 6
ENVV= run p8 --batch 256 --prod-streams 8
ENVV= run p14 --batch 256 --prod-streams 14
ENVV= run d12 --batch 256 --inflight 12
ENVV= run d8 --batch 256 --inflight 8
ENVV= run s4 --batch 256 --segments 4
ENVV=ASR_PIPELINE_PTILED=4 run t4 --batch 256
ENVV=ASR_PIPELINE_PTILED=16 run t16 --batch 256
ENVV=ASR_PIPELINE_PTILED=16 run c4t16
ENVV= run c2 --config C2
