set -e
mkdir -p gpurun_out/c3s
run() { # name, args...
  n=$1; shift
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify "$@" > gpurun_out/c3s/$n.json 2>gpurun_out/c3s/$n.err
  python -c "import json;d=json.load(open('gpurun_out/c3s/$n.json'));c=d['config'];print('$n', round(d['value']/1e6,2), d['ms_per_step'], c.get('segments'), c.get('inflight_decodes'))"
}
run c3_def --config C3
run c3_s1 --config C3 --segments 1
run c3_s4 --config C3 --segments 4
run c3_d5 --config C3 --inflight 5
run c3_d6 --config C3 --inflight 6
run c3_s4d6 --config C3 --segments 4 --inflight 6
