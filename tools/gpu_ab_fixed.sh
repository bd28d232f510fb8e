# Fixed-stride kernel A/B: tools/kbench.py (1M x 1 KiB, back-to-back launches,
# HIP-event median/min) per build; builds in build_exp/ ("" = product).
# usage: bash tools/gpu_ab_fixed.sh ALGS lib1.so lib2.so ...
set -o pipefail
algs=$1; shift
for r in 1 2 3; do
  for lib in "$@"; do
    echo "== ${lib:-product}"
    LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python tools/kbench.py --alg $algs --reps 100 || exit 1
  done
done
