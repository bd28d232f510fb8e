set -o pipefail
for lib in "" build_exp/liblcb_notiles.so; do
echo "== ${lib:-default}"
for args in "--len 1024 --count 4194304" "--len 65536 --count 65536" "--len 65536 --count 65536 --pad 1088" "--len 16384 --count 262144" "--len 4096 --count 1048576"; do
LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python tools/stride_bench.py $args || exit 1
done; done
