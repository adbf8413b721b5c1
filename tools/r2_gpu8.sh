#!/bin/bash
set -u
O=gpurun_out/${R2OUT:-r2g8}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ctc_gpu.py tests/test_ctc_batch_gpu.py tests/test_ctc_cu_semantics.py tests/test_full_configs_gpu.py::test_c3_full_size -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/ctc_profile.py --waves 8 --cases c2,c3 --sigmas bench,3 --reps 3 > $O/timing.log 2>&1 || { echo "timing failed"; tail -5 $O/timing.log; exit 1; }
grep -hv amdgpu $O/timing.log | cut -c1-160
ASR_LIB=libasr_amd_stamps.so timeout -k 10 200 python tools/ctc_profile.py --stamps --waves 8 --cases c2,c3 --sigmas bench --reps 2 > $O/stamps.log 2>&1 || { echo "stamps failed"; tail -5 $O/stamps.log; exit 1; }
grep -hv amdgpu $O/stamps.log | python3 -c "import json,sys; [print(json.dumps(json.loads(l)['events_per_frame']), json.dumps(json.loads(l)['per_frame'])) for l in sys.stdin]"
echo done
