#!/bin/bash
# Time split of the fixed-stride LDS-DMA kernel: main (L), no loads (S1:
# compression of register data only), no compression (S2: DMA stream only).
mkdir -p gpurun_out/ab
for i in 1 2; do for v in L S1 S2; do
  echo "== $v"
  LCB_HASH_GPU_LIB=$PWD/build_exp/$v.so timeout -k 10 120 python3 tools/kbench.py --alg ${ALGS:-md5,sha1,sha256} --reps 50 || exit 1
done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab/split.log
