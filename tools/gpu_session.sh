set -o pipefail
O=gpurun_out/s23; mkdir -p $O
for v in a16 pp; do
LCB_HASH_GPU_LIB=build_exp/$v/liblcb_hash_gpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_packets.py tests/test_radius_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ragged or packets or c4 or keyed or radius or bucketed" > $O/pytest_$v.txt 2>&1; rc=$?; tail -1 $O/pytest_$v.txt; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u tools/ab_inproc.py --libs product,a16,pp --work pkt,r1k,c4 --alg md5 --rounds 8 > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu $O/ab.txt; exit $rc
