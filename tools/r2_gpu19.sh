#!/bin/bash
set -u
O=gpurun_out/r2g19
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ctc_cu_semantics.py tests/test_ctc_wide_gpu.py tests/test_ctc_timesteps_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/ctc_profile.py --waves 8 --cases c5 --sigmas bench --reps 2 > $O/timing.log 2>&1 || { echo "timing failed"; tail -5 $O/timing.log; exit 1; }
grep -hv amdgpu $O/timing.log | cut -c1-160
echo done
