# 256 per GPU and C2: decode CUs (the production half is the pole at 256 per GPU)
set -u
O=gpurun_out/${OUT:-r6s}; mkdir -p $O
run() {  # name, args
  n=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-serialized > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));s=d['stages'];c=d['config'];print('$n', round(d['value']/1e6,1), c.get('decode_cus'), c.get('inflight_decodes'), c.get('production_streams'), s.get('production_busy_frac'), s.get('decode_busy_frac'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"
}
run g256 --batch 256
run g256_p12 --batch 256 --prod-streams 12
run g256_p14 --batch 256 --prod-streams 14
run g256_p16 --batch 256 --prod-streams 16
run g256_d112 --batch 256 --decode-partition 112
run g256_d112p12 --batch 256 --decode-partition 112 --prod-streams 12
run g256_d144 --batch 256 --decode-partition 144
run g256b --batch 256
run g256_p12b --batch 256 --prod-streams 12
run c2 --config C2
run c2_p12 --config C2 --prod-streams 12
run c2_p14 --config C2 --prod-streams 14
run c2_d112 --config C2 --decode-partition 112
run g512 --batch 512
run g512_p9 --batch 512 --prod-streams 9
