set -o pipefail
O=gpurun_out/s8; mkdir -p $O
lib() { [ $1 = product ] && echo liblcb_amd/liblcb_hash_gpu.so || echo build_exp/$1/liblcb_hash_gpu.so; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_packets.py tests/test_queue.py tests/test_radius_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for v in product dpp; do
    LCB_HASH_GPU_LIB=$(lib $v) timeout -k 10 200 python tools/pkt_bench.py --steps 20 --no-layouts > $O/pkt_${v}_$round.log 2>&1 || { tail -3 $O/pkt_${v}_$round.log; exit 1; }
    python3 tools/pkt_summary.py $v $O/pkt_${v}_$round.log
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o pkt --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pkt_bench.py --steps 10 --no-layouts --no-c4 > $GRAFT_REPO_ROOT/$O/kt.log 2>&1; rc=$?; echo "kt rc=$rc"; exit $rc
cd $GRAFT_REPO_ROOT
