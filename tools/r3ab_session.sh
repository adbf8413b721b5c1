set -u
A="--config C5 --steps 30 --warmup 3 --no-cpu-baseline"
export OUT=r3ab SKIP="smoke pytest"
export RUNS="c5g0@ASR_RNN_GRAPH=0:$A|c5d3g0@ASR_RNN_GRAPH=0:--inflight 3 --prod-streams 3 $A|c5d3p4g0@ASR_RNN_GRAPH=0:--inflight 3 --prod-streams 4 $A|c5d4p4g0@ASR_RNN_GRAPH=0:--inflight 4 --prod-streams 4 $A"
bash tools/gpu_check.sh
OUT=r3ab_c5d3g0 BENCH_ARGS="--config C5 --inflight 3 --prod-streams 3 --steps 12 --warmup 2 --no-cpu-baseline" PASSES="trace" ASR_RNN_GRAPH=0 bash tools/profile_bench.sh || exit $?
