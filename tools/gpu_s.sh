#!/bin/bash
# One GPU-box session of round 3: parity tests (all -m gpu), then the kernel
# timings the session is about.  Every GPU step has its own time limit and
# the script stops at the first crash / abort / timeout.
#   OUT=gpurun_out/<tag> [PYTEST_K=expr] [SKIP_TESTS=1] tools/gpu_s.sh [extra command...]
set -u
OUT=${OUT:-gpurun_out/s}
mkdir -p "$OUT"
if [ -z "${SKIP_TESTS:-}" ]; then
    timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 300 \
        --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest.log" 2>&1
    rc=$?
    echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ $# -gt 0 ]; then
    timeout -k 10 ${STEP_TIMEOUT:-400} "$@" > "$OUT/step.log" 2>&1
    rc=$?
    echo "step rc=$rc"; tail -12 "$OUT/step.log"
    exit $rc
fi
