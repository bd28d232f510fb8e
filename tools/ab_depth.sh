#!/bin/bash
# LDS line-stream depth x waves-per-workgroup sweep for the fixed-stride
# MD5/SHA kernel: parity of each variant on the fixed-stride tests, then
# interleaved kernel timings.  Stops at the first failure.
mkdir -p gpurun_out/ab
V=${VARIANTS:-D1W4 D2W2 D2W4 D2W1 D3W1}
for v in $V; do
  LCB_HASH_GPU_LIB=$PWD/build_exp/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "fixed or golden or c3 or kat" > gpurun_out/ab/tests_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc $(tail -1 gpurun_out/ab/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for i in 1 2; do for v in $V; do
  echo "== $v"
  LCB_HASH_GPU_LIB=$PWD/build_exp/$v.so timeout -k 10 120 python3 tools/kbench.py --alg ${ALGS:-md5,sha1,sha256} --reps 50 || exit 1
done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab/depth.log
