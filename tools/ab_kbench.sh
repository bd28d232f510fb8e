#!/bin/bash
# Kernel A/B on the GPU box: tools/kbench.py (1M x 1 KiB, fixed stride) for
# the algorithms KALGS over the product library and the variants
# build_exp/<v>/liblcb_hash_gpu.so listed in VARIANTS, ROUNDS alternating
# rounds; each run time-limited, the script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
lib() { [ $1 = product ] && echo liblcb_amd/liblcb_hash_gpu.so || echo build_exp/$1/liblcb_hash_gpu.so; }
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in product $VARIANTS; do
    echo "== $v round $round"
    LCB_HASH_GPU_LIB=$(lib $v) timeout -k 10 120 python tools/kbench.py --alg ${KALGS:-md5} --reps ${REPS:-30} --warmup 20 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
