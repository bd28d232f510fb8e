# Resident-grid fixed-stride variants: same-process A/B, then the parity
# suite on the first variant (LCB_HASH_GPU_LIB).
set -o pipefail
timeout -k 10 300 python -u tools/ab_inproc.py --libs product,p4p,p4pi,p4i --work fixed --alg md5,sha1,sha256 --rounds 12 --launches 40 > gpurun_out/ab_pers2.txt 2>&1 &&
LCB_HASH_GPU_LIB=build_exp/p4pi/liblcb_hash_gpu.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/par_p4pi.txt 2>&1
