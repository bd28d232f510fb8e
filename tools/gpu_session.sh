set -o pipefail
O=gpurun_out/s11; mkdir -p $O
lib() { [ $1 = product ] && echo liblcb_amd/liblcb_hash_gpu.so || echo build_exp/$1/liblcb_hash_gpu.so; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -3 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for v in product head; do
    LCB_HASH_GPU_LIB=$(lib $v) timeout -k 10 200 python tools/pkt_bench.py --steps 20 > $O/pkt_${v}_$round.log 2>&1 || { tail -3 $O/pkt_${v}_$round.log; exit 1; }
    python3 tools/pkt_summary.py $v $O/pkt_${v}_$round.log
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 90 rocprofv3 -L > $GRAFT_REPO_ROOT/$O/counters_avail.txt 2>&1; echo "list rc=$?"
