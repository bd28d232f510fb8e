#!/bin/bash
# GOST layout/spill A/B (round 3): kbench over 1M x 1 KiB for each build
# variant in build_exp/, two alternating rounds on one box.
set -u
for round in 1 2; do
  for v in r2 P4 P2 P8 P4u; do
    echo "== $v round $round"
    LCB_HASH_GPU_LIB=build_exp/$v/liblcb_hash_gpu.so timeout -k 10 120 \
        python tools/kbench.py --alg gost256,gost512 --reps 20 --warmup 10 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
