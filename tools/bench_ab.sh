#!/bin/bash
# Driver-shaped bench A/B (GPU box): `bench.py --steps 20 --warmup 5` (the
# round-end command) alternating library builds, N rounds; one JSON line per
# run under gpurun_out/$TAG.  LIBS: "product" = the in-tree library, else a
# build_exp/<name> from tools/build_variant.sh.
#   TAG=ab LIBS="product r4" N=3 bash tools/bench_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-bench_ab}
LIBS=${LIBS:-product}
N=${N:-3}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for i in $(seq 1 $N); do
  for v in $LIBS; do
    if [ $v = product ]; then L=""; else L=$R/build_exp/$v/liblcb_hash_gpu.so; fi
    LCB_HASH_GPU_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu > $O/${v}_$i.json 2> $O/${v}_$i.err
    rc=$?; [ $rc -ne 0 ] && { echo "$v $i rc=$rc"; exit $rc; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['roofline']['kernel_ms'])" $O/${v}_$i.json $v
  done
done
exit 0
