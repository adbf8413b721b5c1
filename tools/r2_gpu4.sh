#!/bin/bash
# Prefix-score (L0) candidate keys: parity (all decoder tests + full configs),
# decoder timings, critical-path stamps, bench.
set -u
O=gpurun_out/${R2OUT:-r2g4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ctc_gpu.py tests/test_ctc_batch_gpu.py tests/test_ctc_cu_semantics.py tests/test_ctc_list_gpu.py tests/test_ctc_wide_gpu.py tests/test_dropin.py tests/test_full_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/ctc_profile.py --waves 8 --cases c2,c3 --sigmas bench,3 --reps 3 > $O/timing.log 2>&1 || { echo "timing failed"; tail -5 $O/timing.log; exit 1; }
grep -hv amdgpu $O/timing.log | cut -c1-160
ASR_LIB=libasr_amd_wstamps.so timeout -k 10 200 python tools/ctc_profile.py --wstamps --waves 8 --cases c2 --sigmas bench --reps 2 > $O/wstamps.log 2>&1 || { echo "wstamps failed"; tail -5 $O/wstamps.log; exit 1; }
grep -v amdgpu $O/wstamps.log | python3 -c "import json,sys; [print(json.dumps(json.loads(l)['last_wave_arrival'])) for l in sys.stdin]"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
echo done
