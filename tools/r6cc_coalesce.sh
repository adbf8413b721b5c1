# Dynamic batching (asr_pipeline_create_coalesced): the GPU test, then small
# shards and C2 with `--coalesce G` against the per-submit pipeline
set -u
O=gpurun_out/${OUT:-r6cc}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py -k "coalesced or segmented_handoff or matches_sequential" > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
run() {  # name, args
  n=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-serialized > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));s=d['stages'];c=d['config'];print('$n', round(d['value']/1e6,1), c.get('coalesce'), c.get('inflight_decodes'), c.get('production_streams'), (d.get('parity') or {}).get('match'), s.get('first_decode_start_ms'), s.get('last_production_end_ms'), s.get('last_decode_end_ms'))"
}
run g256 --batch 256 --no-cpu-baseline
run g256_c2 --batch 256 --coalesce 2 --no-cpu-baseline
run g256_c4 --batch 256 --coalesce 4 --no-cpu-baseline
run g512 --batch 512 --no-cpu-baseline
run g512_c2 --batch 512 --coalesce 2 --no-cpu-baseline
run c2 --config C2
run c2_c4 --config C2 --coalesce 4
run c2_c10 --config C2 --coalesce 10
run c2_c20 --config C2 --coalesce 20
