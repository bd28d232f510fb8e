#!/bin/bash
# Ingestion-queue sweep (no pytest): producer threads x slots x callbacks.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-qs}
mkdir -p $OUT
cd $R
while read -r cfg; do
  [ -z "$cfg" ] && continue
  timeout -k 10 120 ./tools/queue_bench $cfg >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
  rc=$?; [ $rc -ne 0 ] && { echo "FAILED rc=$rc: $cfg"; exit $rc; }
done <<CFGS
${CFGS:---threads 8
--threads 8 --cb 0
--threads 16 --slots 8
--threads 16 --slots 8 --cb 0
--threads 8 --slots 8 --flush-us 100
--threads 8 --size 64 --packets 4194304 --slots 8}
CFGS
cat $OUT/sweep.jsonl
