# Dynamic batching, repeats: 256 per GPU with 1 / 2 submits per launch, C2 at
# the bench's automatic choice
set -u
O=gpurun_out/${OUT:-r6dd}; mkdir -p $O
run() {  # name, args
  n=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-serialized > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));s=d['stages'];c=d['config'];print('$n', round(d['value']/1e6,1), c.get('coalesce'), c.get('inflight_decodes'), c.get('production_streams'), (d.get('parity') or {}).get('match'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"
}
run g256_c1a --batch 256 --coalesce 1 --no-cpu-baseline
run g256_c2a --batch 256 --coalesce 2 --no-cpu-baseline
run g256_c1b --batch 256 --coalesce 1 --no-cpu-baseline
run g256_c2b --batch 256 --coalesce 2 --no-cpu-baseline
run c2_auto --config C2
run c2_auto2 --config C2
run c2_c5 --config C2 --coalesce 5
run g128 --batch 128 --no-cpu-baseline
run g128_c4 --batch 128 --coalesce 4 --no-cpu-baseline
