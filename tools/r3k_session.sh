set -u
OUT=r3k_c4 BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline" PASSES="trace fetch write sq" bash tools/profile_bench.sh
