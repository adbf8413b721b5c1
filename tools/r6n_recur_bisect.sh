# Bisect of the one-launch recurrence's per-frame time against the round-5
# kernel: variants of dense.hip (make rvariant): b = no start-of-launch abort
# read, bc = b + round 5's wait loop; all without the load hoist
set -u
O=$PWD/gpurun_out/${OUT:-r6n}; mkdir -p $O
S="32:1024:2000 64:1024:1000 32:512:1000"
for i in 1 2; do
  ( cd _wt_r05 && timeout -k 10 200 python -u tools/step_time.py $S ) > $O/r05_$i.log 2>&1 || { tail $O/r05_$i.log; exit 1; }
  for v in libasr_amd.so libasr_amd_rv_b.so libasr_amd_rv_bc.so; do
    ASR_RP_HOIST=0 ASR_LIB=$v timeout -k 10 200 python -u tools/step_time.py $S > $O/${v}_$i.log 2>&1 || { tail $O/${v}_$i.log; exit 1; }
  done
  for v in r05 libasr_amd.so libasr_amd_rv_b.so libasr_amd_rv_bc.so; do echo "$v $i"; grep '^{' $O/${v}_$i.log; done
done
