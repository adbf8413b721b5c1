# Round 6 A/B: drain schedule (ASR_PIPELINE_DRAIN / ASR_PIPELINE_SEG0) and
# the hardware-queue fit (CU-masked streams at GPU_MAX_HW_QUEUES=4 with the
# 24-queue schedule forced by explicit inflight / prod_streams).
set -u
O=gpurun_out/${OUT:-r6b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ctc_list_gpu.py tests/test_ctc_segment_gpu.py tests/test_ctc_gpu.py tests/test_pipeline_gpu.py tests/test_full_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
A="--no-cpu-baseline --no-serialized"
OUT=${OUT:-r6b} BENCH_LIMIT=200 RUNS="c3:--config C3 $A|g256:--batch 256 $A|g256d@ASR_PIPELINE_DRAIN=-1:--batch 256 $A|g256ds@ASR_PIPELINE_DRAIN=-1,ASR_PIPELINE_SEG0=0.3:--batch 256 $A|g256s@ASR_PIPELINE_SEG0=0.3:--batch 256 $A|g512:--batch 512 $A|g512d@ASR_PIPELINE_DRAIN=-1:--batch 512 $A|c2:--config C2 $A|c2d@ASR_PIPELINE_DRAIN=-1:--config C2 $A|c2ds@ASR_PIPELINE_DRAIN=-1,ASR_PIPELINE_SEG0=0.3:--config C2 $A|c4:$A|c4d@ASR_PIPELINE_DRAIN=-1:$A|q4c4:--hw-queues 4 $A|q4c4f:--hw-queues 4 --inflight 4 --prod-streams 4 $A|q4g256:--hw-queues 4 --batch 256 $A|q4g256f:--hw-queues 4 --inflight 10 --prod-streams 10 --batch 256 $A|q4c2f:--hw-queues 4 --inflight 10 --prod-streams 10 --config C2 $A|g256b:--batch 256 $A|g256db@ASR_PIPELINE_DRAIN=-1:--batch 256 $A|c5:--config C5 $A|c5f32@ASR_DENSE=f32:--config C5 $A|c5b:--config C5 $A" bash tools/bench_matrix.sh
