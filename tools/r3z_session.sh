set -u
OUT=r3z_c4 BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline" PASSES="trace fetch write sq" bash tools/profile_bench.sh || exit $?
OUT=r3z_g256 BENCH_ARGS="--global-batch 256 --steps 10 --warmup 2 --no-cpu-baseline" PASSES="trace" bash tools/profile_bench.sh || exit $?
