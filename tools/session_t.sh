# (ASR_PIPELINE_SEGFRAC was an A/B knob, removed after this run: every uneven split slower, the drain unchanged)
# Uneven T-segments (ASR_PIPELINE_SEGFRAC = frames in the first segment / T): C4, 256 per GPU, C2.
O=gpurun_out/${OUT:-st5}; mkdir -p $O
run() { n=$1; shift; env $ENVV timeout -k 10 200 python bench.py --no-cpu-baseline --no-serialized "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d.get('stages') or {};print('$n', d['value'], d['ms_per_step'], s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))" || { echo "$n rc=$rc"; tail -3 $O/b_$n.err; }; }
for rep in a b; do
  ENVV= run c4_50$rep
  ENVV=ASR_PIPELINE_SEGFRAC=0.6 run c4_60$rep
  ENVV=ASR_PIPELINE_SEGFRAC=0.7 run c4_70$rep
  ENVV=ASR_PIPELINE_SEGFRAC=0.8 run c4_80$rep
done
for rep in a b; do
  ENVV= run g_50$rep --batch 256
  ENVV=ASR_PIPELINE_SEGFRAC=0.65 run g_65$rep --batch 256
  ENVV= run c2_50$rep --config C2
  ENVV=ASR_PIPELINE_SEGFRAC=0.65 run c2_65$rep --config C2
done
