#!/bin/bash
# Round-end style GPU session: smoke, parity tests, bench, rocprofv3 trace of
# the bench command, PMC passes (FETCH_SIZE, WRITE_SIZE, SQ group) on the
# bench workload for every digest.  Stops at the first crash/timeout.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r1}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.json | cut -c1-400
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 $R/bench.py --no-cpu --no-extras > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 $R/tools/kbench.py --alg md5,sha1,sha224,sha256,sha384,sha512,gost256,gost512 --reps 3 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
