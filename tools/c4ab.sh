# C4 A/B: experiment builds in build_exp/ (tools/c4bench.py, tools/stride_bench.py).
set -o pipefail
for r in 1 2; do
  for lib in build_exp/liblcb_notiles.so build_exp/liblcb_wg4aux0.so build_exp/liblcb_w6aux0.so build_exp/liblcb_w5aux0.so; do
    echo "== ${lib:-default}"
    LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python tools/c4bench.py --alg md5 --reps 20 || exit 1
    LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python tools/stride_bench.py --len 65536 --count 349525 --reps 10 --pad 64 || exit 1
  done
done
