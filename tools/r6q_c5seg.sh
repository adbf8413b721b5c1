# C5 (decode-bound since the recurrence fixes): T-segments 2 / 3 / 4
set -u
O=gpurun_out/${OUT:-r6q}; mkdir -p $O
for a in "--segments 2" "--segments 3" "--segments 4" "--segments 2" "--segments 4"; do
  n=$(echo $a | tr -d ' -'); n=${n}_$RANDOM
  timeout -k 10 300 python bench.py --config C5 $a --no-cpu-baseline --no-serialized > $O/c5_$n.json 2> $O/c5_$n.err || { tail $O/c5_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c5_$n.json'));s=d['stages'];print('c5 $a', d['value'], s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), s.get('steady_ms_per_step'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"
done
