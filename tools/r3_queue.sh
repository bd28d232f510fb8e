#!/bin/bash
# Queue session: GPU queue tests, then queue_bench saturation runs (copy,
# zero copy, copy-only) twice each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r3q}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_queue.py tests/test_c_caller_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for extra in "" "--zerocopy 1" "--copy-only 1"; do
    echo "== $round $extra"
    timeout -k 10 120 tools/queue_bench --alg 1 --packets 2097152 --size 1024 --threads 8 $extra 2>&1 | tail -1 || exit 1
  done
done
