#!/bin/bash
# Driver-shaped bench runs (--steps 20 --warmup 5: the round-end command)
# alternating the product library and the one-generation MD5 kernel
# (build_exp/nopers, LCB_FIXED_PERSIST=0), then one default-length run each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4h
mkdir -p $O
cd $R
for i in 1 2 3; do
  for v in product nopers; do
    if [ $v = product ]; then L=""; else L=build_exp/nopers/liblcb_hash_gpu.so; fi
    LCB_HASH_GPU_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu > $O/short_${v}_$i.json 2> $O/short_${v}_$i.err
    rc=$?; [ $rc -ne 0 ] && { echo "$v $i rc=$rc"; exit $rc; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['roofline']['kernel_ms'])" $O/short_${v}_$i.json $v
  done
done
for v in product nopers; do
  if [ $v = product ]; then L=""; else L=build_exp/nopers/liblcb_hash_gpu.so; fi
  LCB_HASH_GPU_LIB=$L timeout -k 10 200 python bench.py --no-extras --no-cpu > $O/long_${v}.json 2> $O/long_${v}.err
  rc=$?; [ $rc -ne 0 ] && { echo "$v long rc=$rc"; exit $rc; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], 'long', d['value'], d['roofline']['kernel_ms'])" $O/long_${v}.json $v
done
