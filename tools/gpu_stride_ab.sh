# Fixed-stride cache-policy A/B: tools/stride_bench.py at aligned and unaligned strides, per build
# ("" = product).  usage: bash tools/gpu_stride_ab.sh lib1.so lib2.so ...
set -o pipefail
for r in 1 2; do
  for lib in "$@"; do
    echo "== ${lib:-product}"
    for args in "--len 1024 --count 1048576 --pad 0" "--len 1024 --count 1048576 --pad 16" "--len 1024 --count 1048576 --pad 64" "--len 65536 --count 349525 --pad 64"; do
      LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python tools/stride_bench.py $args --reps 10 || exit 1
    done
  done
done
