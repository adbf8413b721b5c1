# Dynamic batching with the vectorized staging copy: tests, 256 per GPU, C2
set -u
O=gpurun_out/${OUT:-r6ll}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py tests/test_bench_pipeline_gpu.py -k "coalesced or c2_chip" > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for a in "g256:--batch 256 --no-cpu-baseline" "g256b:--batch 256 --no-cpu-baseline" "c2:--config C2"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python bench.py --no-serialized $args > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));c=d['config'];print('$n', round(d['value']/1e6,1), c.get('coalesce'), (d.get('parity') or {}).get('match'))"
done
