#!/bin/bash
# GPU session: parity tests, then ingestion-queue throughput/latency sweeps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-q1}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for cfg in "--threads 1" "--threads 4" "--threads 8" "--threads 16" "--threads 8 --flush-us 50 --batch-msgs 8192" \
           "--threads 8 --batch-msgs 262144 --batch-bytes 268435456" "--threads 8 --size 64 --packets 4194304" \
           "--threads 8 --size 4096 --packets 262144"; do
  timeout -k 10 120 ./tools/queue_bench $cfg >> $OUT/queue_bench.jsonl 2>> $OUT/queue_bench.err
  rc=$?; echo "queue_bench $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
cat $OUT/queue_bench.jsonl
exit 0
