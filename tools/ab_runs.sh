#!/bin/bash
# A/B bench lines with per-run environment (run on the GPU box from the repo root):
#   OUT=r3b RUNS="name|ENV=1 OTHER=2|--config C2 --steps 20;name2||--config C4" bash tools/ab_runs.sh
# RUNS: ';'-separated name|env|args triples.  Each run has its own time limit
# (BENCH_LIMIT, default 300 s); the first failure ends the call.
set -u
O=gpurun_out/${OUT:-ab}
mkdir -p "$O"
IFS=';' read -ra items <<< "${RUNS:?RUNS is required}"
for it in "${items[@]}"; do
    IFS='|' read -r name envs args <<< "$it"
    env $envs timeout -k 10 ${BENCH_LIMIT:-300} python bench.py $args > "$O/bench_$name.log" 2>&1
    rc=$?
    grep '^{' "$O/bench_$name.log" | tail -1 > "$O/bench_$name.json"
    echo "$name rc=$rc $(python3 -c "import json,sys; d=json.load(open('$O/bench_$name.json')); print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('avg_launch_ms'))" 2>/dev/null)"
    [ $rc -eq 0 ] || { tail -20 "$O/bench_$name.log"; exit $rc; }
done
