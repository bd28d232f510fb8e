set -o pipefail
O=gpurun_out/s15; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/pkt_bench.py --steps 20 > $O/pkt.log 2>&1 || { tail -3 $O/pkt.log; exit 1; }
python3 tools/pkt_summary.py product $O/pkt.log
