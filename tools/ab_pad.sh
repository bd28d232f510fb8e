#!/bin/bash
# A/B session for the scalar pad-block schedule (LCB_UNIFORM_PAD): GPU parity
# of the main library, then kernel timings of build_exp/G.so (off) and
# build_exp/L.so (on), interleaved twice.  Stops at the first failure.
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ab/tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do for v in G L; do
  echo "== $v"
  LCB_HASH_GPU_LIB=$PWD/build_exp/$v.so timeout -k 10 120 python3 tools/kbench.py --alg ${ALGS:-md5,sha1,sha256,sha512} --reps 50 || exit 1
done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab/pad_bench.log
