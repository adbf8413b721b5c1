# Bench lines with the per-batch timeline dumped (ASR_BENCH_TIMELINE): default, 4 segments, 60 steps, 256 per GPU.
set -e
O=gpurun_out/${OUT:-g3}; mkdir -p $O
run() { n=$1; shift; ASR_BENCH_TIMELINE=$O/tl_$n.txt timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/b_$n.json 2> $O/b_$n.err; python -c "import json;d=json.load(open('$O/b_$n.json'));s=d['stages'];print('$n', d['value'], d['ms_per_step'], s['steady_ms_per_step'], s['first_decode_start_ms'], s['last_production_end_ms'], s['last_decode_end_ms'], d['clock']['gfxclk_mhz']['mean'])"; }
run def
run s4 --segments 4
run st60 --steps 60
run b256 --batch 256
run b256s4 --batch 256 --segments 4
