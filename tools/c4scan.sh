set -e
mkdir -p gpurun_out/c4e
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_ctc_segment_gpu.py tests/test_full_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c4e/pytest.log 2>&1
tail -1 gpurun_out/c4e/pytest.log
for n in 512 1024; do
timeout -k 10 150 python bench.py --steps 20 --warmup 5 --config C4 --global-batch $n > gpurun_out/c4e/g$n.json 2>gpurun_out/c4e/g$n.err
python -c "import json;d=json.load(open('gpurun_out/c4e/g$n.json'));c=d['config'];print('g$n', round(d['value']/1e6,2), d['ms_per_step'], c.get('segments'), c.get('inflight_decodes'), (d.get('parity') or {}).get('match'))"
done
