#!/bin/bash
# A/B session: library variants under build_exp/<name> against the product
# build (kbench fixed-stride MD5, the ragged-packet rows), then the parity
# tests on the first variant.  VARIANTS="a b" ; each step time-limited.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r3ab}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
V=${VARIANTS:-md5asm}
lib() { [ $1 = product ] && echo liblcb_amd/liblcb_hash_gpu.so || echo build_exp/$1/liblcb_hash_gpu.so; }
first=${PYTEST_VARIANT:-product}
if [ -z "$SKIP_PYTEST" ]; then
LCB_HASH_GPU_LIB=$(lib $first) timeout -k 10 300 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_$first.log 2>&1
rc=$?; echo "pytest $first rc=$rc"; tail -2 $OUT/pytest_$first.log; [ $rc -ne 0 ] && exit $rc
fi
[ -n "$LIST_COUNTERS" ] && (cd /tmp && TMPDIR=/tmp timeout -k 5 60 rocprofv3 -L > $OUT/counters.txt 2>&1)
for round in 1 2; do
  for v in product $V; do
    echo "== $v round $round"
    LCB_HASH_GPU_LIB=$(lib $v) timeout -k 10 120 python tools/kbench.py --alg ${KALGS:-md5} --reps 50 --warmup 30 2>&1 | grep -v amdgpu.ids || exit 1
    LCB_HASH_GPU_LIB=$(lib $v) timeout -k 10 200 python tools/pkt_bench.py --steps 20 ${PKT_ARGS:---no-c4} > $OUT/pkt_${v}_$round.log 2>&1 || { tail -3 $OUT/pkt_${v}_$round.log; exit 1; }
    python3 - $OUT/pkt_${v}_$round.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    j = json.loads(l)
    if "ragged_packets" in j:
        print("   packets", {k: (v["ms_per_pass"], v["hbm_frac"], v["dod_equals_reference"]) for k, v in j["ragged_packets"].items() if isinstance(v, dict)})
    elif "c4" in j:
        print("   c4", j.get("alg", ""), j["c4"]["ms_per_pass"], j["c4"]["hbm_frac"], j["c4"].get("dod_equals_reference"))
    else:
        print("  ", j)
PY
  done
done
