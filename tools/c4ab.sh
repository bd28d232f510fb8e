# C4 A/B: experiment builds in build_exp/ against the product build
# (tools/c4bench.py: HIP-event median per pass, bucketing included, digest-of-
# digests checked; tools/stride_bench.py: 64 KiB records at a given pad).
# usage: bash tools/c4ab.sh lib1.so lib2.so ...   (empty string = product build)
set -o pipefail
for r in 1 2; do
  for lib in "$@"; do
    echo "== ${lib:-product}"
    LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python tools/c4bench.py --alg md5 --reps 20 || exit 1
    LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python tools/stride_bench.py --len 65536 --count 349525 --reps 10 --pad 64 || exit 1
  done
done
