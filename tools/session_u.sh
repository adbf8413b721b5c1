# The one-launch H > 256 recurrence: bit-equality / torch tests, step timing with and without it, kernel names.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-su}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "persistent or step or h_gt_256 or bidirectional or c5_hidden or h2048 or recur_stage" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; echo pytest rc=$rc
[ $rc -eq 0 ] || exit $rc
ASR_RNN_PERSIST=0 timeout -k 10 120 python tools/step_time.py 32:1024:2000 64:1024:500 32:512:1000 > $O/step_off.jsonl 2>&1; cat $O/step_off.jsonl
timeout -k 10 120 python tools/step_time.py 32:1024:2000 64:1024:500 32:512:1000 > $O/step_on.jsonl 2>&1; cat $O/step_on.jsonl
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/step_time.py 32:1024:2000 > $O/trace.log 2>&1; echo trace rc=$?
