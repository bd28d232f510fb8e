#!/bin/bash
# Round-2 GPU session: smoke, parity tests, bench (weak N=1 default and
# strong C5 on one GPU), rocprofv3 kernel trace of the bench.  Every GPU step
# has its own time limit; the script stops at the first crash/timeout.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r2a}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log
  return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
if [ -z "$SKIP_TESTS" ]; then
  step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS}
  rc=$?; [ $rc -ne 0 ] && exit $rc
fi
[ -n "$SKIP_BENCH" ] && exit 0
step bench 400 python bench.py ${BENCH_ARGS} || exit $?
step bench_c5 300 python bench.py --scaling strong --no-extras --no-cpu --steps 50 --warmup 20 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 $R/bench.py --no-cpu --no-extras > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"
exit $rc
