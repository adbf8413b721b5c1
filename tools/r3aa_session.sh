set -u
OUT=r3aa_c5d3 BENCH_ARGS="--config C5 --inflight 3 --prod-streams 3 --steps 12 --warmup 2 --no-cpu-baseline" PASSES="trace" bash tools/profile_bench.sh || exit $?
OUT=r3aa_c5d2 BENCH_ARGS="--config C5 --steps 12 --warmup 2 --no-cpu-baseline" PASSES="trace" bash tools/profile_bench.sh || exit $?
mkdir -p gpurun_out/r3aa
ASR_PIPELINE_TRACE=1 timeout -k 10 200 python bench.py --config C5 --inflight 3 --prod-streams 3 --steps 12 --warmup 2 --no-cpu-baseline > gpurun_out/r3aa/c5d3_hosttrace.log 2>&1
echo "hosttrace rc=$?"
