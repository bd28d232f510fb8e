R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/c4p
cd /tmp && export TMPDIR=/tmp
for v in product prev; do
  lib=$R/liblcb_amd/liblcb_hash_gpu.so; [ $v = prev ] && lib=$R/build_exp/prev/liblcb_hash_gpu.so
  LCB_HASH_GPU_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4p/$v -o run --output-format csv -- python3 $R/tools/c4bench.py --alg md5 --reps 5 > $R/gpurun_out/c4p/$v.log 2>&1 || exit 1
  echo "== $v"; cut -d, -f1-4 $R/gpurun_out/c4p/$v/run_kernel_stats.csv | head -8
done
