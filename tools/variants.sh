#!/bin/bash
# Time every build_exp/*.so variant with tools/kbench.py (one process each).
ALGS=${ALGS:-md5,sha1,sha256,sha512,gost256}
mkdir -p gpurun_out
for so in ${VARIANTS:-build_exp/*.so}; do
  echo "== $so"
  LCB_HASH_GPU_LIB=$PWD/$so timeout -k 10 120 python3 tools/kbench.py --alg $ALGS --reps ${REPS:-10} || exit $?
done
