# Round 6: the one-wave decoder at 5 waves per SIMD (96 VGPRs, spills) with the in-place LDS layout
# (7.6 KB: 20 per CU) vs the product at 16 per CU — decode alone on the bench's emissions
set -u
O=gpurun_out/${OUT:-r6g}; mkdir -p $O
for lib in libasr_amd.so libasr_amd_cv_ip4.so libasr_amd_cv_ip5.so; do
  ASR_LIB=$lib timeout -k 10 200 python tools/occupancy_sweep.py --T 300 --k 8,16,20,24 --waves -1 --beam 50 > $O/sweep50_$lib.jsonl 2>$O/sweep50_$lib.err || exit 1
done
for f in $O/sweep*.jsonl; do echo $f; python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); print(d['per_cu'], d['kernel_ms'], d['utt_frames_per_us_per_cu'], d['lds'], d['same_as_first_schedule'])
"; done
