#!/bin/bash
# One GPU-box session: smoke -> pytest -m gpu -> short bench.  Each GPU step
# has its own time limit; a crash/abort/timeout ends the session (no retries).
set -u
mkdir -p gpurun_out
stop_if_fatal() {  # $1 = exit code, $2 = step
    case "$1" in
        0|1) return 0 ;;    # ok / ordinary test failures
        *) echo "FATAL: $2 exited $1; stopping" | tee -a gpurun_out/session.log; exit "$1" ;;
    esac
}
echo "== smoke" | tee gpurun_out/session.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/session.log; tail -3 gpurun_out/smoke.log
stop_if_fatal $rc smoke
echo "== pytest -m gpu" | tee -a gpurun_out/session.log
timeout -k 10 ${PYTEST_LIMIT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/session.log; tail -15 gpurun_out/pytest_gpu.log
stop_if_fatal $rc pytest
echo "== bench" | tee -a gpurun_out/session.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/session.log; tail -5 gpurun_out/bench.log
exit $rc
