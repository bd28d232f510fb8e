# Sustained clock A/B of library builds: for each build, in a fresh process,
# the MD5 per-algorithm row six times in a row (10 warm + 5 timed launches
# each; tools/alg_clock_order.py) -- the later rows hold the kernel's own
# sustained clock.  Builds alternate twice.
# usage: bash tools/sustained_ab.sh <out dir> <lib.so>...
O=$1; shift
mkdir -p $O
for r in 1 2; do
  for lib in "$@"; do
    tag=$(basename $(dirname $lib))
    LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python3 -u tools/alg_clock_order.py --order md5,md5,md5,md5,md5,md5 --reps 1 \
      > $O/${tag}_$r.txt 2>/dev/null || exit 1
  done
done
