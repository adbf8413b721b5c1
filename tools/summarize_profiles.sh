# Summaries of a tools/profile_bench.sh run of the default C4 bench into profiles/<round>/:
#   RUN=prof_sj ROUND=r05 bash tools/summarize_profiles.sh
set -e
P=gpurun_out/${RUN:?}; R=${ROUND:-r05}
mkdir -p profiles/$R
SRC="gpurun_out/$RUN (rocprofv3 passes of bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-serialized: C4, two 1024-utterance pipeline batches per step, 4 decodes in flight, 2 T-segments; ${R} tree at commit $(git rev-parse --short HEAD))"
python tools/traffic_from_pmc.py $P/fetch/run_counter_collection.csv $P/write/run_counter_collection.csv C4 "$SRC" $R | tail -3
python tools/issue_from_pmc.py $P/sq/run_counter_collection.csv --kernel ctc_wave_kernel --T 500 --B 1024 --workload C4 --cus 128 --source "$SRC" --round $R | tail -5
python tools/wait_from_pmc.py $P/wait/run_counter_collection.csv $P/issue/run_counter_collection.csv $P/sq/run_counter_collection.csv --T 500 --B 1024 --source "$SRC" --round $R | tail -5
python tools/mfma_from_pmc.py --mfma $P/mfma/run_counter_collection.csv --valu $P/valu/run_counter_collection.csv --workload C4 --cus "gemm_x3_kernel<8,8>=128" --cus gemm_x3_kernel=256 --cus rnn_recur_x3_kernel=128 --cus gemm_narrow_kernel=256 --T 500 --B 1024 --decoder ctc_wave_kernel --decoder-cus 128 --source "$SRC" --round $R > /dev/null
cp $P/trace/run_kernel_trace.csv profiles/$R/c4_final_kernel_trace.csv
cp $P/trace/run_kernel_stats.csv profiles/$R/c4_final_kernel_stats.csv
for p in fetch write sq wait issue valu mfma; do cp $P/$p/run_counter_collection.csv profiles/$R/c4_final_${p}_counters.csv; done
ls -la profiles/$R | head -30
