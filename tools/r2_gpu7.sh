#!/bin/bash
set -u
O=gpurun_out/${R2OUT:-r2g7}
mkdir -p $O
ASR_LIB=libasr_amd_wstamps.so timeout -k 10 200 python tools/ctc_profile.py --wstamps --waves 8 --cases c2 --sigmas bench --reps 2 > $O/wstamps.log 2>&1 || { echo "wstamps failed"; tail -5 $O/wstamps.log; exit 1; }
grep -v amdgpu $O/wstamps.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(json.dumps(d['last_wave_arrival']))
    for k,v in d['arrival_cycles_by_wave'].items(): print(k.ljust(22), v)"
echo done
