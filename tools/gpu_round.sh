#!/bin/bash
# One GPU-box session: parity tests, then (only if they ran to completion,
# pass or fail) the benchmark.  Stops at the first crash/timeout.
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-700} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"
tail -3 gpurun_out/bench.log
exit $rc
