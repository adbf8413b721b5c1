# bench priming (--prime-s) A/B at C4, alternating, and the 256-per-GPU shard.
O=gpurun_out/${OUT:-ss}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d.get('stages') or {};c=d.get('clock') or {};print('$n', d['value'], d['ms_per_step'], s.get('production_ms_per_batch'), s.get('decode_span_ms_per_batch'), (c.get('gfxclk_mhz') or {}).get('mean'), c.get('socket_power_w'))" || { echo "$n rc=$rc"; tail -3 $O/b_$n.err; }; }
for rep in a b c; do run p0$rep --prime-s 0; run p3$rep; done
run g0 --batch 256 --prime-s 0; run g3 --batch 256
