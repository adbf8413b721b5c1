# 256 per GPU at two submits per launch: decodes / productions in flight
set -u
O=gpurun_out/${OUT:-r6ii}; mkdir -p $O
for a in "d:" "i8:--inflight 8 --prod-streams 8" "i6:--inflight 6 --prod-streams 6" "i9:--inflight 9 --prod-streams 9" "d2:"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python bench.py --batch 256 --no-cpu-baseline --no-serialized $args > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));c=d['config'];print('$n', round(d['value']/1e6,1), c.get('coalesce'), c.get('inflight_decodes'), c.get('production_streams'))"
done
