# 512-utterance batches (256 per GPU at two per launch; 512 per GPU): 5 / 6 / 7 decodes in flight
set -u
O=gpurun_out/${OUT:-r6jj}; mkdir -p $O
for a in "g256_i6:--batch 256 --inflight 6 --prod-streams 6" "g256_d:--batch 256" "g256_i5:--batch 256 --inflight 5 --prod-streams 5" "g256_i6b:--batch 256 --inflight 6 --prod-streams 6" "g512_d:--batch 512" "g512_i6:--batch 512 --inflight 6 --prod-streams 6" "g512_i5:--batch 512 --inflight 5 --prod-streams 5"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-serialized $args > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));c=d['config'];print('$n', round(d['value']/1e6,1), c.get('coalesce'), c.get('inflight_decodes'), c.get('production_streams'))"
done
