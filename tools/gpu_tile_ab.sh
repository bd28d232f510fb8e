# Tile-kernel A/B: C4 (tools/c4bench.py) and 1M x 1 KiB ragged at aligned / 16-B / 1-B strides
# (tools/stride_bench.py, ragged rows), per build ("" = product).
set -o pipefail
for r in 1 2; do
  for lib in "$@"; do
    echo "== ${lib:-product}"
    LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python tools/c4bench.py --alg md5 --reps 20 || exit 1
    for p in 0 16 1; do
      LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python tools/stride_bench.py --len 1024 --count 1048576 --pad $p --reps 10 | grep ragged || exit 1
    done
  done
done
