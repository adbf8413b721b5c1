set -e
mkdir -p gpurun_out/xp
run() { # name, env, args...
  n=$1; shift; e=$1; shift
  env $e timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify "$@" > gpurun_out/xp/$n.json 2>gpurun_out/xp/$n.err
  python -c "import json;d=json.load(open('gpurun_out/xp/$n.json'));c=d['config'];print('$n', round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
run c4_x0a ASR_PIPELINE_XPERM=0 --config C4
run c4_x1a ASR_PIPELINE_XPERM=1 --config C4
run c4_x0b ASR_PIPELINE_XPERM=0 --config C4
run c4_x1b ASR_PIPELINE_XPERM=1 --config C4
run c4_x1_144 ASR_PIPELINE_XPERM=1 --config C4 --decode-partition 144
run g512_x1 ASR_PIPELINE_XPERM=1 --config C4 --global-batch 512
run c2_x1 ASR_PIPELINE_XPERM=1 --config C2
