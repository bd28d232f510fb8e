#!/bin/bash
# Session r3 s3: gather-layout ragged tile stream -- every GPU test, then the
# ragged A/B lines (packets, 1 KiB at three strides, C4), then GOST against
# the round-2 library.
set -u
mkdir -p gpurun_out/s3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/s3/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/pkt_bench.py --steps 10 > gpurun_out/s3/pkt.log 2>&1 || { tail -5 gpurun_out/s3/pkt.log; exit 1; }
grep -v amdgpu gpurun_out/s3/pkt.log
for round in 1 2; do
  for v in r2 product; do
    lib=build_exp/$v/liblcb_hash_gpu.so; [ $v = product ] && lib=liblcb_amd/liblcb_hash_gpu.so
    echo "== $v round $round"
    LCB_HASH_GPU_LIB=$lib timeout -k 10 120 python tools/kbench.py --alg gost256,gost512 --reps 20 --warmup 10 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
