#!/bin/bash
# Several bench.py lines in one GPU-box call (run from the repo root).
#   OUT=r3a RUNS="c4:--steps 20 --warmup 5|c2:--config C2 --steps 20 --warmup 5" bash tools/bench_matrix.sh
# RUNS: '|'-separated name:args pairs; name@VAR=v,VAR2=w sets environment
# variables for that run (A/B knobs).  Each run has its own time limit
# (BENCH_LIMIT, default 300 s); the first failure ends the call.
set -u
O=gpurun_out/${OUT:-bench}
mkdir -p "$O"
IFS='|' read -ra items <<< "${RUNS:?RUNS is required}"
for it in "${items[@]}"; do
    name=${it%%:*}
    args=${it#*:}
    envs=""
    case $name in *@*) envs=${name#*@}; envs=${envs//,/ }; name=${name%%@*} ;; esac
    timeout -k 10 ${BENCH_LIMIT:-300} env $envs python bench.py $args > "$O/bench_$name.log" 2>&1
    rc=$?
    grep '^{' "$O/bench_$name.log" | tail -1 > "$O/bench_$name.json"
    echo "$name rc=$rc $(python3 -c "import json,sys; d=json.load(open('$O/bench_$name.json')); print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('avg_launch_ms'))" 2>/dev/null)"
    [ $rc -eq 0 ] || { tail -20 "$O/bench_$name.log"; exit $rc; }
done
