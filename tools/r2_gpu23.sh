#!/bin/bash
# C5 wide-kernel phase split and LDS counters.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g23
mkdir -p $O
ASR_LIB=libasr_amd_stamps.so timeout -k 10 300 python tools/ctc_profile.py --stamps --waves 8 --cases c5 --sigmas bench --reps 1 > $O/st.log 2>&1 || { echo "stamps failed"; tail -5 $O/st.log; exit 1; }
grep -v amdgpu $O/st.log
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d $O/sq -o run -- python3 tools/ctc_profile.py --waves 8 --cases c5 --sigmas bench --reps 1 > $O/sq.log 2>&1 || { echo "sq pass failed $?"; tail -5 $O/sq.log; exit 1; }
python3 - <<'PY'
import csv,glob,collections
f=glob.glob("gpurun_out/r2g23/sq/**/*counter_collection.csv",recursive=True)
print(f)
acc=collections.defaultdict(float)
for fn in f:
    for r in csv.DictReader(open(fn)):
        if "ctc_wide" in r.get("Kernel_Name",""):
            acc[r["Counter_Name"]]+=float(r["Counter_Value"])
print(dict(acc))
PY
