# Round 6 rocprofv3 evidence: C4 (all passes) and a C5 / 256-per-GPU kernel trace
set -u
OUT=r6c4 PASSES="trace fetch write sq wait issue valu mfma" bash tools/profile_bench.sh || exit 1
OUT=r6c5 BENCH_ARGS="--config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-serialized" PASSES="trace" bash tools/profile_bench.sh || exit 1
OUT=r6g256 BENCH_ARGS="--batch 256 --steps 5 --warmup 2 --no-cpu-baseline --no-serialized" PASSES="trace" bash tools/profile_bench.sh || exit 1
