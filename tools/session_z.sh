# (result: 128 decode CUs stay best at 256 / 512 per GPU: 112 / 120 lose 4-13 %)
# Small shards: fewer decode CUs (production is the pole at 256 per GPU), paired with the default.
O=gpurun_out/${OUT:-sz}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized "$@" > $O/b_$n.json 2> $O/b_$n.err; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d.get('stages') or {};c=d['config'];print('$n', d['value'], d['ms_per_step'], c.get('decode_cus'), s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"; }
for rep in a b; do
  run g128$rep --batch 256
  run g112$rep --batch 256 --decode-partition 112
  run g120$rep --batch 256 --decode-partition 120
  run h128$rep --batch 512
  run h120$rep --batch 512 --decode-partition 120
done
