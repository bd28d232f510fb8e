#!/bin/bash
# Ragged LDS line-stream gather kernel: GPU parity of the main library, then
# the C4 mixed-length workload (bench.bench_c4) with build_exp/G0.so (per-lane
# loads) and build_exp/G1.so (gather line stream), interleaved twice.
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests_gather.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ab/tests_gather.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do for v in G0 G1; do
  echo "== $v"
  LCB_HASH_GPU_LIB=$PWD/build_exp/$v.so timeout -k 10 200 python3 -c "
import bench
for alg in (1, 2, 4):
    print(alg, bench.bench_c4(alg, 3, 8))
" || exit 1
done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab/gather.log
