# s12: tile/fixed traces (occupancy per CU), then the ingestion queue under a
# kernel + memory-copy trace, copying vs zero copy.
set -o pipefail
O=gpurun_out/s12; mkdir -p $O
LCB_HASH_GPU_LIB=build_exp/trace/liblcb_hash_gpu.so timeout -k 10 300 python -u tools/tile_trace.py --work fixed,r1k,pkt --out $O/tr4 > $O/trace4.txt 2>&1; rc=$?; grep -v amdgpu $O/trace4.txt | cut -c1-400; [ $rc -ne 0 ] && exit $rc
LCB_HASH_GPU_LIB=build_exp/trace_fw2/liblcb_hash_gpu.so timeout -k 10 200 python -u tools/tile_trace.py --work fixed --out $O/tr2 > $O/trace2.txt 2>&1; rc=$?; grep -v amdgpu $O/trace2.txt | cut -c1-400; [ $rc -ne 0 ] && exit $rc
for zc in 0 1; do
  timeout -k 10 120 tools/queue_bench --alg 1 --packets 2097152 --size 1024 --threads 8 --zerocopy $zc > $O/q_zc$zc.json 2> $O/q_zc$zc.err; rc=$?; cut -c1-300 $O/q_zc$zc.json; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
for zc in 0 1; do
  timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/qprof_zc$zc -o q --output-format csv -- $GRAFT_REPO_ROOT/tools/queue_bench --alg 1 --packets 2097152 --size 1024 --threads 8 --zerocopy $zc > $GRAFT_REPO_ROOT/$O/qprof_zc$zc.log 2>&1; rc=$?; echo "qprof zc=$zc rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
