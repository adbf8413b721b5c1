#!/bin/bash
set -u
O=gpurun_out/${R2OUT:-r2g6}
mkdir -p $O
timeout -k 10 60 ./gpu-accelerated-speech-recognition_amd/build/scan_test || { echo "scan test failed"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_ctc_gpu.py tests/test_ctc_batch_gpu.py tests/test_ctc_cu_semantics.py tests/test_ctc_wide_gpu.py tests/test_full_configs_gpu.py::test_c3_full_size -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/ctc_profile.py --waves 4,8 --cases c2,c3 --sigmas bench,3 --reps 3 > $O/timing.log 2>&1 || { echo "timing failed"; tail -5 $O/timing.log; exit 1; }
grep -hv amdgpu $O/timing.log | cut -c1-160
ASR_LIB=libasr_amd_abl4.so timeout -k 10 200 python tools/ctc_profile.py --waves 8 --cases c2 --sigmas bench --reps 3 > $O/timing_abl4.log 2>&1 || { echo "abl4 failed"; exit 1; }
grep -hv amdgpu $O/timing_abl4.log | cut -c1-160 | sed 's/^/abl4 /'
ASR_LIB=libasr_amd_wstamps.so timeout -k 10 200 python tools/ctc_profile.py --wstamps --waves 8 --cases c2 --sigmas bench --reps 2 > $O/wstamps.log 2>&1 || { echo "wstamps failed"; tail -5 $O/wstamps.log; exit 1; }
grep -v amdgpu $O/wstamps.log | python3 -c "import json,sys; [print(json.dumps(json.loads(l)['last_wave_arrival'])) for l in sys.stdin]"
echo done
