# C3 (beam 100, 256 per submit): one vs two submits per launch, paired
set -u
O=gpurun_out/${OUT:-r6hh}; mkdir -p $O
for a in "c3_1:--coalesce 1" "c3_2:--coalesce 2" "c3_1b:--coalesce 1" "c3_2b:--coalesce 2"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline --no-serialized $args > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));c=d['config'];print('$n', round(d['value']/1e6,1), c.get('coalesce'), c.get('inflight_decodes'), c.get('production_streams'))"
done
