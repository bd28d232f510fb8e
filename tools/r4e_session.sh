#!/bin/bash
# Closing GPU session of the resident-grid MD5 build: the SHA-384/512 line-
# stream A/B (when build_exp/nolines exists), smoke, GPU tests, the
# PMC passes (tools/pmc_session.sh) collected into the stamped counter files
# on the box, then the bench (which reads them) and its kernel trace.
# Stops at the first failure.   TAG=r4e bash tools/r4e_session.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4e}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
# AB_LIBS=product,<build_exp name> AB_WORK=... AB_ALG=...: a same-process A/B first.
if [ -n "$AB_LIBS" ]; then
  timeout -k 10 300 python -u tools/ab_inproc.py --libs $AB_LIBS --work ${AB_WORK:-fixed} --alg ${AB_ALG:-md5} --rounds ${AB_ROUNDS:-12} > $O/ab.txt 2>&1
  rc=$?; echo "ab rc=$rc"; grep -v amdgpu $O/ab.txt | cut -c1-330; [ $rc -ne 0 ] && exit $rc
elif [ -d build_exp/nolines ]; then
  timeout -k 10 300 python -u tools/ab_inproc.py --libs product,nolines --work c4,r1k,pkt --alg sha512,sha384 --rounds 10 > $O/ab_lines.txt 2>&1
  rc=$?; echo "ab rc=$rc"; grep -v amdgpu $O/ab_lines.txt | cut -c1-330; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
TAG=$TAG bash $R/tools/pmc_session.sh
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd $R
python3 tools/pmc_collect.py $O $TAG > $O/pmc_collect.log 2>&1
rc=$?; echo "collect rc=$rc"; tail -3 $O/pmc_collect.log; [ $rc -ne 0 ] && exit $rc
mkdir -p $O/profiles && cp profiles/pmc_*.json profiles/valu_counts.json $O/profiles/
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.json | cut -c1-300; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 $R/bench.py --no-cpu --no-extras > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
