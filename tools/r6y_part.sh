# 256 per GPU / C4: decode partition with the default stream counts held fixed
set -u
O=gpurun_out/${OUT:-r6y}; mkdir -p $O
run() {  # name, args
  n=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-serialized > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));s=d['stages'];c=d['config'];print('$n', round(d['value']/1e6,1), c.get('decode_cus'), c.get('inflight_decodes'), c.get('production_streams'), s.get('production_busy_frac'), s.get('decode_busy_frac'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"
}
run g256 --batch 256
run g256_d112 --batch 256 --decode-partition 112 --inflight 10 --prod-streams 10
run g256_d120 --batch 256 --decode-partition 120 --inflight 10 --prod-streams 10
run g256_d136 --batch 256 --decode-partition 136 --inflight 10 --prod-streams 10
run g256b --batch 256
run c4 --config C4
run c4_d120 --config C4 --decode-partition 120 --inflight 5 --prod-streams 5
run c4_d136 --config C4 --decode-partition 136 --inflight 5 --prod-streams 5
run c4b --config C4
