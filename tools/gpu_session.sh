set -o pipefail
O=gpurun_out/s10; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -3 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  timeout -k 10 200 python tools/pkt_bench.py --steps 20 > $O/pkt_product_$round.log 2>&1 || { tail -3 $O/pkt_product_$round.log; exit 1; }
  python3 tools/pkt_summary.py product $O/pkt_product_$round.log
done
