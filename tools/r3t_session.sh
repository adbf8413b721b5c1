set -u
OUT=r3t_c4 BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline" PASSES="trace" bash tools/profile_bench.sh || exit $?
OUT=r3t_g256 BENCH_ARGS="--global-batch 256 --steps 30 --warmup 5 --no-cpu-baseline" PASSES="trace" bash tools/profile_bench.sh || exit $?
