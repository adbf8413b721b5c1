# (ASR_PIPELINE_FILL was an A/B knob, removed after this run: fill on every CU 163 M vs 217-223 M at 256 per GPU)
# (ASR_PIPELINE_XCD was an A/B knob, removed: an XCD left out of a CU mask gets every CU, so both roles ran chip-wide)
# Fill phase on every CU at 32 hardware queues (256 per GPU needs 30 streams), and the
# whole-XCD decode / production split (ASR_PIPELINE_XCD=1), C4 and 256 per GPU.
O=gpurun_out/${OUT:-sm}; mkdir -p $O
run() { n=$1; shift; env $ENVV ASR_BENCH_TIMELINE=$O/tl_$n.txt timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d.get('stages') or {};c=d['config'];p=d.get('cu_placement') or {};print('$n', d['value'], d['ms_per_step'], s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'), c.get('streams'), c.get('hw_queues'), p.get('decode_cus_per_xcd'), p.get('production_cus_per_xcd'))" || { echo "$n rc=$rc"; tail -3 $O/b_$n.err; }; }
ENVV= run g0 --batch 256 --hw-queues 32
ENVV=ASR_PIPELINE_FILL=10 run g10 --batch 256 --hw-queues 32
ENVV=ASR_PIPELINE_FILL=20 run g20 --batch 256 --hw-queues 32
ENVV=ASR_PIPELINE_XCD=1 run gx --batch 256
ENVV=ASR_PIPELINE_XCD=1 run c4x
ENVV= run c4
ENVV= run g0b --batch 256 --hw-queues 32
ENVV=ASR_PIPELINE_FILL=10 run g10b --batch 256 --hw-queues 32
