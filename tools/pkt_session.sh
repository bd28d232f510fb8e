#!/bin/bash
# Packet-path session (GPU box): per-kernel trace of the 1M-packet rows
# (bucketing + tile kernel, plain / HMAC / keyed) and one occupancy/VALU
# counter pass per library build given in LIBS (product = the in-tree
# library, or build_exp/<name>/liblcb_hash_gpu.so), over tools/pkt_bench.py.
#   TAG=r5c LIBS="product head" bash tools/pkt_session.sh
# Every step runs under its own time limit; the script stops at the first
# failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-pkt}
LIBS=${LIBS:-product}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for lib in $LIBS; do
  if [ "$lib" = product ]; then unset LCB_HASH_GPU_LIB; else export LCB_HASH_GPU_LIB=$R/build_exp/$lib/liblcb_hash_gpu.so; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt_$lib -o run --output-format csv -- python3 $R/tools/pkt_bench.py --steps 10 --no-layouts --no-c4 > $O/kt_$lib.log 2>&1
  rc=$?; echo "trace $lib rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_$lib -o run --output-format csv -- python3 $R/tools/pkt_bench.py --steps 3 --no-layouts --no-c4 > $O/pmc_$lib.log 2>&1
  rc=$?; echo "pmc $lib rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
