# rocprofv3 kernel traces of the dynamic-batching lines (C2 at ten submits
# per launch, 256 per GPU at two)
set -u
OUT=r6kk_c2 BENCH_ARGS="--config C2 --steps 20 --warmup 5 --no-cpu-baseline --no-serialized" PASSES="trace" bash tools/profile_bench.sh || exit 1
OUT=r6kk_g256 BENCH_ARGS="--batch 256 --steps 20 --warmup 5 --no-cpu-baseline --no-serialized" PASSES="trace" bash tools/profile_bench.sh || exit 1
