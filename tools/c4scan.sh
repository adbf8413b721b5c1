set -e
mkdir -p gpurun_out/c4s
run() { # name, args...
  n=$1; shift
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify "$@" > gpurun_out/c4s/$n.json 2>gpurun_out/c4s/$n.err
  python -c "import json;d=json.load(open('gpurun_out/c4s/$n.json'));c=d['config'];print('$n', round(d['value']/1e6,2), d['ms_per_step'], c.get('segments'), c.get('inflight_decodes'))"
}
run c4_s2 --config C4
run c4_s3 --config C4 --segments 3
run c4_s4 --config C4 --segments 4
run c4_s2_i5 --config C4 --inflight 5
run g1024_s4 --config C4 --global-batch 1024 --segments 4
run g512_s4 --config C4 --global-batch 512 --segments 4
run g512_s2 --config C4 --global-batch 512
run g1024_s3 --config C4 --global-batch 1024 --segments 3
