# Fill order A/B (ASR_PIPELINE_GEMM_ORDER), C4 and the 256-per-GPU shard, with timelines; decoder phase stamps at 16 per CU.
O=gpurun_out/${OUT:-sb}; mkdir -p $O
run() { n=$1; shift; env $ENVV ASR_BENCH_TIMELINE=$O/tl_$n.txt timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d['stages'];print('$n', d['value'], d['ms_per_step'], s['steady_ms_per_step'], s['first_decode_start_ms'], s['last_production_end_ms'], s['last_decode_end_ms'], d['clock']['gfxclk_mhz']['mean'])" || echo "$n rc=$rc"; }
ENVV="ASR_PIPELINE_GEMM_ORDER=1" run on1
ENVV="ASR_PIPELINE_GEMM_ORDER=0" run off1
ENVV="ASR_PIPELINE_GEMM_ORDER=1" run on2
ENVV="ASR_PIPELINE_GEMM_ORDER=1" run on256 --batch 256
ENVV="ASR_PIPELINE_GEMM_ORDER=0" run off256 --batch 256
ENVV="ASR_PIPELINE_GEMM_ORDER=1" run on512 --batch 512
echo "== stamps"
ASR_LIB=libasr_amd_stamps.so timeout -k 10 200 python tools/ctc_profile.py --stamps --waves -1 --cases s4096 --sigmas bench --reps 2 > $O/stamps.jsonl 2>&1; echo rc=$?; cat $O/stamps.jsonl | tail -2
