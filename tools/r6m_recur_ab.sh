# A/B of the one-launch recurrence alone: round-5 tree (worktree _wt_r05,
# built in-tree), this tree with the h_{t-1} loads all in flight (default)
# and without (ASR_RP_HOIST=0), alternating on one box; then the persist
# tests and C5 lines
set -u
O=$PWD/gpurun_out/${OUT:-r6m}; mkdir -p $O
S="32:1024:2000 64:1024:1000 32:512:1000"
for i in 1 2; do
  ( cd _wt_r05 && timeout -k 10 200 python -u tools/step_time.py $S ) > $O/r05_$i.log 2>&1 || { tail $O/r05_$i.log; exit 1; }
  ASR_RP_HOIST=0 timeout -k 10 200 python -u tools/step_time.py $S > $O/nohoist_$i.log 2>&1 || { tail $O/nohoist_$i.log; exit 1; }
  timeout -k 10 200 python -u tools/step_time.py $S > $O/hoist_$i.log 2>&1 || { tail $O/hoist_$i.log; exit 1; }
  for v in r05 nohoist hoist; do echo "$v $i"; grep '^{' $O/${v}_$i.log; done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_gpu.py -k "persist" > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for i in 1 2; do
timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline --no-serialized > $O/c5_$i.json 2> $O/c5_$i.err || { tail $O/c5_$i.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5_$i.json'));print('c5', d['value'], d['stages'].get('production_ms_per_batch'), d['stages'].get('decode_span_ms_per_batch'), d['stages'].get('steady_ms_per_step'))"
done
for d in 4; do
timeout -k 10 300 python bench.py --config C5 --inflight $d --no-cpu-baseline --no-serialized > $O/c5_d$d.json 2> $O/c5_d$d.err || { tail $O/c5_d$d.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5_d$d.json'));print('c5 d$d', d['value'], d['stages'].get('production_ms_per_batch'), d['stages'].get('decode_span_ms_per_batch'), d['stages'].get('steady_ms_per_step'))"
done
