# Round 6: the 20-per-CU decoder variant (ip5) in the pipeline vs the product (same box)
set -u
A="--no-cpu-baseline --no-serialized"
OUT=${OUT:-r6h} BENCH_LIMIT=200 RUNS="c4:$A|c4ip5@ASR_LIB=libasr_amd_cv_ip5.so:$A|g256:--batch 256 $A|g256ip5@ASR_LIB=libasr_amd_cv_ip5.so:--batch 256 $A|c2:--config C2 $A|c2ip5@ASR_LIB=libasr_amd_cv_ip5.so:--config C2 $A|g512:--batch 512 $A|g512ip5@ASR_LIB=libasr_amd_cv_ip5.so:--batch 512 $A|c4b:$A|c4ip5b@ASR_LIB=libasr_amd_cv_ip5.so:$A" bash tools/bench_matrix.sh
for f in gpurun_out/${OUT:-r6h}/bench_*.json; do python3 -c "
import json
d=json.load(open('$f')); c=d['config']
print('$f'.split('/')[-1], round(d['value']/1e6,1), 'D', c.get('inflight_decodes'), 'P', c.get('production_streams'), 'launch', d['roofline']['avg_launch_ms'])
"; done
