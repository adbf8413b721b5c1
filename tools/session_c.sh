# Default bench line (full) on the current tree, then the rocprofv3 passes for profiles/r05.
O=gpurun_out/${OUT:-sc}; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_c4.json 2> $O/bench_c4.err; echo "bench rc=$?"
python -c "import json;d=json.load(open('$O/bench_c4.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], d['parity']['match'], r['frac'], r['serialized'], r['chip_level']['frac'])"
OUT=${OUT:-sc} PASSES="${PASSES:-trace fetch write sq wait issue valu mfma}" bash tools/profile_bench.sh
