# Round 6: one-wave decoder before / after the in-place LDS layout (decode alone, bench emissions)
set -u
O=gpurun_out/${OUT:-r6e}; mkdir -p $O
for lib in libasr_amd.so libasr_amd_cv_oldwave.so; do
  ASR_LIB=$lib timeout -k 10 200 python tools/occupancy_sweep.py --T 300 --k 4,8,11,12 --waves -1 --beam 100 > $O/sweep100_$lib.jsonl 2>$O/sweep100_$lib.err || exit 1
  ASR_LIB=$lib timeout -k 10 200 python tools/occupancy_sweep.py --T 300 --k 8,16 --waves -1 --beam 50 > $O/sweep50_$lib.jsonl 2>$O/sweep50_$lib.err || exit 1
done
for f in $O/sweep*.jsonl; do echo $f; python3 -c "
import json,sys
for l in open('$f'):
    d=json.loads(l); print(d['per_cu'], d['kernel_ms'], d['utt_frames_per_us_per_cu'], d['lds'])
"; done
