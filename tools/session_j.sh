# Round-5 evidence on the current tree: config lines (C3, C5, BL, shards) and the C4 rocprofv3 passes.
O=gpurun_out/${OUT:-sj}; mkdir -p $O
line() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err; rc=$?; python -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'], (d.get('parity') or {}).get('match'), (d.get('parity') or {}).get('checked'))" || echo "$n rc=$rc"; }
line c3 --config C3
line c5 --config C5 --steps 10 --warmup 3
line bl --config BL --steps 10 --warmup 3
line s1024 --batch 1024 --no-cpu-baseline
line s512 --batch 512 --no-cpu-baseline
line s256 --batch 256 --no-cpu-baseline
OUT=${OUT:-sj} PASSES="trace fetch write sq wait issue valu mfma" bash tools/profile_bench.sh
