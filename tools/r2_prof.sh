#!/bin/bash
# Round-2 profiling session: bench (N=1 default), rocprofv3 kernel trace of
# the bench, PMC passes (HBM bytes and VALU counts) over every algorithm on
# the bench workload, and the C4 workload's HBM bytes.  Each step has its own
# time limit; stop at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r2p}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/bench.json; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 $R/bench.py --no-cpu --no-extras > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 $R/tools/kbench.py --alg md5,sha1,sha224,sha256,sha384,sha512,gost256,gost512 --reps 3 --warmup 5 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_c4 -o run --output-format csv -- python3 $R/tools/c4bench.py --alg md5 --reps 3 > $OUT/pmc_c4.log 2>&1
rc=$?; echo "pmc c4 rc=$rc"
exit $rc
