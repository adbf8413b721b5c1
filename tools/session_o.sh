# Queue fit "production streams down to half the decodes, then both": C2 / 256 per GPU at 4 / 8 / 16 queues,
# C4 at 4; and the H > 256 recurrence step alone (C5, BL shapes).
O=gpurun_out/${OUT:-so}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));c=d['config'];print('$n', d['value'], d['ms_per_step'], c.get('streams'), c.get('hw_queues'), c.get('inflight_decodes'), c.get('production_streams'))" || { echo "$n rc=$rc"; tail -3 $O/b_$n.err; }; }
timeout -k 10 300 python tools/step_time.py 32:1024:2000 256:2048:200 64:1024:500 > $O/step.jsonl 2> $O/step.err; cat $O/step.jsonl
for q in 4 8 16; do
  run c2_q$q --config C2 --hw-queues $q
  run g256_q$q --batch 256 --hw-queues $q
done
run c4_q4 --hw-queues 4
