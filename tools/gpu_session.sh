set -o pipefail
O=gpurun_out/s26; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
LCB_HASH_GPU_LIB=build_exp/cxcd/liblcb_hash_gpu.so timeout -k 10 300 python -u -m pytest tests/test_crc32_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_cxcd.txt 2>&1; rc=$?; tail -1 $O/pytest_cxcd.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_inproc.py --libs product,cxcd --work fixed --alg crc32b,crc32a,crc32c --rounds 12 > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu $O/ab.txt; exit $rc
