set -u
mkdir -p gpurun_out/r3e
for lib in libasr_amd_r3old.so libasr_amd.so; do ASR_LIB=$lib timeout -k 10 120 python tools/diag/wide_tie_diag.py >> gpurun_out/r3e/tie.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/r3e/tie.log
ASR_BENCH_HOSTLOG=gpurun_out/r3e/hostlog_c2n.txt timeout -k 10 200 python bench.py --config C2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3e/bench_c2n.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3e/bench_c2n.log
OUT=r3e RUNS='c4||--steps 20 --warmup 5 --no-cpu-baseline;c4w|ASR_CTC_WAVES=-1|--steps 20 --warmup 5 --no-cpu-baseline;c4wd2|ASR_CTC_WAVES=-1|--steps 20 --warmup 5 --no-cpu-baseline --inflight 2;g512w|ASR_CTC_WAVES=-1|--global-batch 512 --steps 20 --warmup 5 --no-cpu-baseline' bash tools/ab_runs.sh
