set -o pipefail
O=gpurun_out/s25; mkdir -p $O
LCB_HASH_GPU_LIB=build_exp/fxcd/liblcb_hash_gpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3 or fixed or kat or golden or properties" > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_inproc.py --libs product,fxcd --work fixed --alg md5,sha1 --rounds 14 > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu $O/ab.txt; exit $rc
