set -e
mkdir -p gpurun_out/c2s
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_full_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c2s/pytest.log 2>&1
tail -2 gpurun_out/c2s/pytest.log
for n in a b; do
timeout -k 10 120 python bench.py --config C2 --steps 20 --warmup 5 > gpurun_out/c2s/c2_$n.json 2>gpurun_out/c2s/c2_$n.err
python -c "import json;d=json.load(open('gpurun_out/c2s/c2_$n.json'));print('c2', round(d['value']/1e6,2), d['ms_per_step'], d['config']['streams'], d['parity'])"
done
