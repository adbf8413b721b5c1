set -u
OUT=r3ac_c5d3p1 BENCH_ARGS="--config C5 --inflight 3 --prod-streams 1 --steps 12 --warmup 2 --no-cpu-baseline" PASSES="trace" bash tools/profile_bench.sh || exit $?
