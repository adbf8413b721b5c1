set -e
mkdir -p gpurun_out/c4f
run() { # name, args...
  n=$1; shift
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify "$@" > gpurun_out/c4f/$n.json 2>gpurun_out/c4f/$n.err
  python -c "import json;d=json.load(open('gpurun_out/c4f/$n.json'));c=d['config'];print('$n', round(d['value']/1e6,2), d['ms_per_step'], c.get('segments'), c.get('inflight_decodes'))"
}
run g1024_s2d4 --config C4 --global-batch 1024
run g1024_s4d4 --config C4 --global-batch 1024 --segments 4
run g1024_s4d5 --config C4 --global-batch 1024 --segments 4 --inflight 5
run g1024_s4d6 --config C4 --global-batch 1024 --segments 4 --inflight 6
run g256_s2d10 --config C4 --global-batch 256
run g256_s3d10 --config C4 --global-batch 256 --segments 3
run g256_s4d11 --config C4 --global-batch 256 --segments 4 --inflight 11
run c4_s4d5 --config C4 --segments 4 --inflight 5
