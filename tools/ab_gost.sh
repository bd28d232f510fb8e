#!/bin/bash
# A/B of GOST kernel variants (build_exp/lib_<v>.so): GPU parity of each
# variant, then its kernel timings.  Stops at the first failure.
mkdir -p gpurun_out/abg
for v in main ${VARIANTS}; do
  if [ $v = main ]; then L=""; else L=$PWD/build_exp/lib_$v.so; fi
  LCB_HASH_GPU_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abg/tests_$v.log 2>&1
  rc=$?; echo "== $v tests rc=$rc $(tail -1 gpurun_out/abg/tests_$v.log)"
  [ $rc -ne 0 ] && exit $rc
  LCB_HASH_GPU_LIB=$L timeout -k 10 120 python3 tools/kbench.py --alg ${ALGS:-gost256,gost512} --reps 50 2>&1 | grep -v amdgpu.ids || exit 1
done 2>&1 | tee gpurun_out/abg/bench.log
