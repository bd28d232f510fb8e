set -o pipefail
O=gpurun_out/s16; mkdir -p $O
LCB_HASH_GPU_LIB=build_exp/skip/liblcb_hash_gpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_packets.py tests/test_radius_gpu.py tests/test_queue.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_skip.txt 2>&1; rc=$?; tail -1 $O/pytest_skip.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab_inproc.py --libs product,noprio,skip --work c4,pkt,r1k --alg md5 --rounds 8 > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu $O/ab.txt; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for v in product skip; do
  L=$GRAFT_REPO_ROOT/liblcb_amd/liblcb_hash_gpu.so; [ $v = skip ] && L=$GRAFT_REPO_ROOT/build_exp/skip/liblcb_hash_gpu.so
  for grp in FETCH_SIZE WRITE_SIZE; do
    LCB_HASH_GPU_LIB=$L timeout -s KILL 150 rocprofv3 --pmc $grp -d $GRAFT_REPO_ROOT/$O/kt_pkt_${v}_$grp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pkt_bench.py --steps 3 --no-layouts --no-c4 > $GRAFT_REPO_ROOT/$O/kt_pkt_${v}_$grp.log 2>&1; rc=$?; echo "pmc $v $grp rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
