# Kernel trace of the one-launch recurrence alone, round-5 tree vs this tree
set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6o}; mkdir -p $O
( cd $R/_wt_r05 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05 -o run -- python3 tools/step_time.py 32:1024:2000 ) > $O/r05.log 2>&1 || { tail $O/r05.log; exit 1; }
( cd $R && ASR_RP_HOIST=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r06 -o run -- python3 tools/step_time.py 32:1024:2000 ) > $O/r06.log 2>&1 || { tail $O/r06.log; exit 1; }
for v in r05 r06; do echo $v; grep '^{' $O/$v.log; f=$(find $O/$v -name '*kernel_stats.csv' | head -1); cut -c1-150 $f | head -6; t=$(find $O/$v -name '*kernel_trace.csv' | head -1); python3 - "$t" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
for r in rows[-8:]:
    print(r["Kernel_Name"][:50], int(r["Start_Timestamp"]), (int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3)
PY
done
