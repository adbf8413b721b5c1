#!/bin/bash
# One GPU-box session (run from the repo root): smoke -> pytest -m gpu ->
# bench lines (tools/bench_matrix.sh) -> rocprofv3 passes (tools/profile_bench.sh).
# Each GPU step has its own time limit; a crash / abort / timeout ends the
# session (no retries); ordinary test failures (pytest rc 1) do not.
#   OUT=r3a PYTEST_ARGS="tests/test_full_configs_gpu.py" RUNS="c4:--steps 20 --warmup 5" \
#       PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline" PASSES="trace" bash tools/gpu_check.sh
# SKIP="smoke pytest" skips steps.
set -u
export OUT=${OUT:-check}
O=gpurun_out/$OUT
mkdir -p "$O"
stop_if_fatal() {  # $1 = exit code, $2 = step
    case "$1" in
        0|1) return 0 ;;
        *) echo "FATAL: $2 exited $1; stopping" | tee -a "$O/session.log"; exit "$1" ;;
    esac
}
skip() { case " ${SKIP:-} " in *" $1 "*) return 0 ;; *) return 1 ;; esac; }
if ! skip smoke; then
    echo "== smoke" | tee -a "$O/session.log"
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
    rc=$?; echo "smoke rc=$rc" | tee -a "$O/session.log"; tail -3 "$O/smoke.log"
    [ $rc -eq 0 ] || exit $rc
fi
if ! skip pytest; then
    echo "== pytest -m gpu ${PYTEST_ARGS:-tests}" | tee -a "$O/session.log"
    timeout -k 10 ${PYTEST_LIMIT:-600} python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -q -rf --timeout 240 \
        --timeout-method thread > "$O/pytest_gpu.log" 2>&1
    rc=$?; echo "pytest rc=$rc" | tee -a "$O/session.log"; tail -15 "$O/pytest_gpu.log"
    stop_if_fatal $rc pytest
fi
if [ -n "${RUNS:-}" ]; then
    echo "== bench" | tee -a "$O/session.log"
    bash tools/bench_matrix.sh 2>&1 | tee -a "$O/session.log"
    rc=${PIPESTATUS[0]}
    [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${EXTRA:-}" ]; then   # one more GPU command (e.g. a tools/ sweep), its own limit
    echo "== extra: $EXTRA" | tee -a "$O/session.log"
    timeout -k 10 ${EXTRA_LIMIT:-300} bash -c "$EXTRA" > "$O/extra.log" 2>&1
    rc=$?; echo "extra rc=$rc" | tee -a "$O/session.log"; tail -30 "$O/extra.log"
    stop_if_fatal $rc extra
fi
if [ -n "${PASSES:-}" ]; then
    echo "== rocprofv3 ${PASSES}" | tee -a "$O/session.log"
    BENCH_ARGS="${PROF_ARGS:---steps 5 --warmup 2 --no-cpu-baseline}" OUT="$OUT" bash tools/profile_bench.sh \
        2>&1 | tee -a "$O/session.log"
    exit ${PIPESTATUS[0]}
fi
