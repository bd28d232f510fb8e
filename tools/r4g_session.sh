#!/bin/bash
# Kernel trace of the ragged rows (packets + C4, tools/pkt_bench.py) on the
# final round-4 library, and a short bench run (20 steps) beside the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4g
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-extras > $O/bench_short.json 2> $O/bench_short.err
rc=$?; echo "bench short rc=$rc"; tail -1 $O/bench_short.json | cut -c1-200; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pkt -o pkt --output-format csv -- python3 $R/tools/pkt_bench.py --steps 20 > $O/pkt.log 2>&1
rc=$?; echo "pkt trace rc=$rc"; tail -5 $O/pkt.log; exit $rc
