set -o pipefail
O=gpurun_out/s20; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab_inproc.py --libs product,lp0 --work fixed,c4 --alg sha512,gost256 --rounds 6 > $O/ab_lp.txt 2>&1; rc=$?; grep -v amdgpu $O/ab_lp.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?; tail -2 $O/smoke.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 300 $O/bench.json; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-extras --no-cpu > $GRAFT_REPO_ROOT/$O/kt_bench.json 2>&1; rc=$?; echo "kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/ktp -o pkt --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pkt_bench.py --steps 10 --no-layouts > $GRAFT_REPO_ROOT/$O/ktp.log 2>&1; rc=$?; echo "ktp rc=$rc"; exit $rc
