set -o pipefail
O=gpurun_out/s19; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_packets.py tests/test_radius_gpu.py tests/test_queue.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab_inproc.py --libs product,skip2,skipoff --work pkt,r1k,c4 --alg md5 --rounds 10 > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu $O/ab.txt; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $GRAFT_REPO_ROOT/$O/kt_pkt_$grp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pkt_bench.py --steps 3 --no-layouts --no-c4 > $GRAFT_REPO_ROOT/$O/kt_pkt_$grp.log 2>&1; rc=$?; echo "pmc $grp rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
