# (ASR_PIPELINE_FILL was an A/B knob, removed after this run: fill on every CU 163 M vs 217-223 M at 256 per GPU)
# Fill phase on every CU (ASR_PIPELINE_FILL=F: the first F batches after the pipeline was empty
# produce on full-chip streams): 256 per GPU and C4, with timelines.
O=gpurun_out/${OUT:-sl}; mkdir -p $O
run() { n=$1; shift; env $ENVV ASR_BENCH_TIMELINE=$O/tl_$n.txt timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d.get('stages') or {};c=d['config'];print('$n', d['value'], d['ms_per_step'], s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'), c.get('streams'), c.get('hw_queues'))" || { echo "$n rc=$rc"; tail -3 $O/b_$n.err; }; }
ENVV= run g0 --batch 256
ENVV=ASR_PIPELINE_FILL=10 run g10 --batch 256
ENVV=ASR_PIPELINE_FILL=5 run g5 --batch 256
ENVV=ASR_PIPELINE_FILL=20 run g20 --batch 256
ENVV= run g0b --batch 256
ENVV=ASR_PIPELINE_FILL=10 run g10b --batch 256
ENVV=ASR_PIPELINE_FILL=6 run h6 --batch 512
ENVV= run h0 --batch 512
ENVV=ASR_PIPELINE_FILL=4 run c4f4
ENVV= run c4f0
