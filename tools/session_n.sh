# GPU_MAX_HW_QUEUES a C-ABI server needs: C4, C2 and 256 per GPU at 4 / 8 / 16 / 24 / 32 hardware queues
# (the library fits its schedule to the queues it finds; bench --hw-queues sets the variable before HIP starts).
O=gpurun_out/${OUT:-sn}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));c=d['config'];print('$n', d['value'], d['ms_per_step'], c.get('streams'), c.get('hw_queues'), c.get('inflight_decodes'), c.get('production_streams'))" || { echo "$n rc=$rc"; tail -3 $O/b_$n.err; }; }
for q in ${QS:-4 8 16 24 32}; do
  run c4_q$q --hw-queues $q
  run c2_q$q --config C2 --hw-queues $q
  run g256_q$q --batch 256 --hw-queues $q
done
