# The one-launch recurrence's wait polls the abort word / clock every 16th
# poll only: recurrence alone (C5 shape and 64 x 1024), the persist tests,
# C5 lines
set -u
O=gpurun_out/${OUT:-r6l}; mkdir -p $O
timeout -k 10 200 python -u tools/step_time.py 32:1024:2000 64:1024:1000 32:512:1000 > $O/step.log 2>&1 || { tail $O/step.log; exit 1; }
cat $O/step.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_gpu.py -k "persist" > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -2 $O/pt.log
for i in 1 2; do
timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline --no-serialized > $O/c5_$i.json 2> $O/c5_$i.err || { tail $O/c5_$i.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5_$i.json'));print('c5', d['value'], d['stages'].get('production_ms_per_batch'), d['stages'].get('decode_span_ms_per_batch'), d['stages'].get('steady_ms_per_step'))"
done
