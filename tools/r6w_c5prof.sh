# C5 evidence on the current tree: a rocprofv3 kernel trace of the bench
# (5 / 2 steps) and the wide decoder's per-phase clocks (stamps build, bench
# emissions, 8 waves)
set -u
OUT=r6w_c5 BENCH_ARGS="--config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-serialized" PASSES="trace" bash tools/profile_bench.sh || exit 1
O=gpurun_out/r6w; mkdir -p $O
ASR_LIB=libasr_amd_stamps.so timeout -k 10 400 python -u tools/ctc_profile.py --stamps --cases c5 --sigmas bench --waves 8 --reps 1 > $O/stamps.jsonl 2> $O/stamps.err || { tail $O/stamps.err; exit 1; }
cat $O/stamps.jsonl
