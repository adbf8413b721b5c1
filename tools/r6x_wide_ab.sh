# Wide-decoder variants against the product library: time and bit-identity of
# the ranked beams (C5-like bench emissions, V = 1000, beam = 200)
set -u
O=gpurun_out/${OUT:-r6x}; mkdir -p $O
for T in 500 2000; do
for v in libasr_amd.so ${VARIANTS:-libasr_amd_cv_wlist.so} libasr_amd.so; do
  ASR_LIB=$v timeout -k 10 300 python -u tools/wide_ab.py --T $T --out $O/${v}_$T.json > $O/${v}_$T.log 2>&1 || { tail $O/${v}_$T.log; exit 1; }
  echo "$v T=$T $(cat $O/${v}_$T.json)"
done
done
