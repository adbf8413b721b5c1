# Fresh-box reproducibility: the default bench line first (cold GPU), then
# the same command twice more in the same session (warm GPU).
set -e
O=gpurun_out/${OUT:-cw}
mkdir -p $O
for i in 1 2 3; do
    timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/b$i.json 2> $O/b$i.err
    python -c "import json;d=json.load(open('$O/b$i.json'));print('run $i', d['value'], d['ms_per_step'])"
done
