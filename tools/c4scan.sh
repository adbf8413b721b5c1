set -e
mkdir -p gpurun_out/c4p
run() { # name, args...
  n=$1; shift
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify "$@" > gpurun_out/c4p/$n.json 2>gpurun_out/c4p/$n.err
  python -c "import json;d=json.load(open('gpurun_out/c4p/$n.json'));c=d['config'];print('$n', round(d['value']/1e6,2), d['ms_per_step'], c.get('decode_cus'), c.get('inflight_decodes'), c.get('production_streams'))"
}
run c4_128 --config C4
run c4_144 --config C4 --decode-partition 144
run c4_160 --config C4 --decode-partition 160
run c4_120 --config C4 --decode-partition 120
run g1024_144 --config C4 --global-batch 1024 --decode-partition 144
run g1024_128 --config C4 --global-batch 1024
run g512_144 --config C4 --global-batch 512 --decode-partition 144
