# C5: T-segments 1 / 2 with timelines (regression check), 10 / 3 steps.
O=gpurun_out/${OUT:-sx}; mkdir -p $O
c5() { n=$1; shift; ASR_BENCH_TIMELINE=$O/tl_$n.txt timeout -k 10 300 python bench.py --no-cpu-baseline --no-serialized --config C5 --steps 10 --warmup 3 "$@" > $O/c5_$n.json 2> $O/c5_$n.err; python -c "import json;d=json.load(open('$O/c5_$n.json'));c=d['config'];s=d.get('stages') or {};print('c5 $n', d['value'], d['ms_per_step'], c.get('segments'), s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"; cat $O/tl_$n.txt; }
c5 s1 --segments 1
c5 s2 --segments 2
