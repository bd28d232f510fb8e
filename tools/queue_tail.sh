#!/bin/bash
# Latency-tail hunt for the ingestion queue (GPU box): N open-loop runs at a
# fixed offered rate of tools/queue_bench, zero copy and copying alternating,
# one JSON line each (queue stage maxima included).
#   TAG=r5h N=6 RATE=14000000 PACKETS=2097152 bash tools/queue_tail.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-qtail}
N=${N:-6}
RATE=${RATE:-14000000}
PACKETS=${PACKETS:-2097152}
O=$R/gpurun_out/$TAG
mkdir -p $O
for i in $(seq 1 $N); do
  for zc in 1 0; do
    LCB_QUEUE_TRACE=1 timeout -k 10 120 $R/tools/queue_bench --alg 1 --packets $PACKETS --size 1024 --threads 8 --zerocopy $zc --rate $RATE >> $O/queue_tail.jsonl 2>> $O/queue_tail.err
    rc=$?; [ $rc -ne 0 ] && { echo "queue_bench rc=$rc"; exit $rc; }
  done
done
exit 0
