#!/bin/bash
# A/B session: GPU parity of the changed kernels, then kernel timings of the
# main library against the build_exp/ variants.  Stops at the first failure.
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_crc32_gpu.py tests/test_chacha_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ab/tests.log
[ $rc -ne 0 ] && exit $rc
for v in main ${VARIANTS:-old nt}; do
  if [ $v = main ]; then L=""; else L=$PWD/build_exp/lib_$v.so; fi
  echo "== $v"
  LCB_HASH_GPU_LIB=$L timeout -k 10 120 python3 tools/kbench.py --alg ${ALGS:-md5,gost256,gost512} --reps 30 || exit 1
  LCB_HASH_GPU_LIB=$L timeout -k 10 120 python3 tools/crc_bench.py --variants 1,4,6 --reps 30 || exit 1
  LCB_HASH_GPU_LIB=$L timeout -k 10 120 python3 tools/cha_bench.py --rounds 20,8 --reps 30 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab/bench.log
