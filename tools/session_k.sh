# C4 decode partition scan on the current tree (decode CUs [0, N), production on the rest).
O=gpurun_out/${OUT:-sk}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d.get('stages') or {};c=d['config'];print('$n', d['value'], d['ms_per_step'], s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'), c.get('inflight_decodes'), c.get('production_streams'))" || { echo "$n rc=$rc"; tail -3 $O/b_$n.err; }; }
run p128a
run p120 --decode-partition 120
run p112 --decode-partition 112
run p136 --decode-partition 136
run p128b
run p120b --decode-partition 120
run p120d5 --decode-partition 120 --inflight 5
c5() { n=$1; shift; env $ENVV timeout -k 10 300 python bench.py --no-cpu-baseline --no-serialized --config C5 --steps 10 --warmup 3 "$@" > $O/c5_$n.json 2> $O/c5_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/c5_$n.json'));c=d['config'];print('c5 $n', d['value'], d['ms_per_step'], c.get('inflight_decodes'), c.get('production_streams'), c.get('decode_cus'))" || { echo "c5 $n rc=$rc"; tail -3 $O/c5_$n.err; }; }
ENVV=ASR_PIPELINE_PSLICE=0 c5 shared
ENVV= c5 slice
ENVV= c5 slice_d3 --inflight 3
ENVV= c5 slice_d4 --inflight 4
ENVV= c5 slice_d3p3 --inflight 3 --prod-streams 3
