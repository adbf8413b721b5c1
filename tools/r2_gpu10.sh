#!/bin/bash
set -u
O=gpurun_out/r2g10
mkdir -p $O
timeout -k 10 200 python tools/ctc_profile.py --waves 8 --cases c2,c3 --sigmas bench,3 --reps 3 > $O/timing.log 2>&1 || exit 1; grep -hv amdgpu $O/timing.log | cut -c1-160
ASR_LIB=libasr_amd_stamps.so timeout -k 10 200 python tools/ctc_profile.py --stamps --waves 8 --cases c2,c3 --sigmas bench --reps 2 > $O/stamps.log 2>&1 || { echo "stamps failed"; tail -5 $O/stamps.log; exit 1; }
grep -hv amdgpu $O/stamps.log | python3 -c "import json,sys; [print(json.loads(l)['kernel_ms_min'], json.dumps(json.loads(l)['events_per_frame']), json.dumps(json.loads(l)['cycles_per_step'])) for l in sys.stdin]"
echo done
