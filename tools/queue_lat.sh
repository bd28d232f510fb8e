#!/bin/bash
# Ingestion-queue latency under an offered load (open loop, tools/queue_bench
# --rate): 1 KiB MD5 packets from 8 producer threads at rates from 1 M/s up
# to saturation, then the closed-loop saturation run for reference.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-qlat}
mkdir -p $OUT
cd $R
: > $OUT/lat.jsonl
for rate in ${RATES:-1000000 2000000 5000000 10000000 15000000 20000000}; do
  timeout -k 10 120 ${QB:-./tools/queue_bench} --threads 8 --packets 2097152 --rate $rate ${EXTRA} >> $OUT/lat.jsonl 2>> $OUT/lat.err
  rc=$?; echo "rate $rate rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
for k in ${SATRUNS:-1 2 3}; do
  timeout -k 10 120 ${QB:-./tools/queue_bench} --threads 8 --packets 2097152 ${EXTRA} >> $OUT/lat.jsonl 2>> $OUT/lat.err
  rc=$?; echo "saturated rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 -c "
import json
for l in open('$OUT/lat.jsonl'):
    j = json.loads(l)
    print('rate %9.0f  got %9.0f pkt/s  p50 %7.1f  p99 %7.1f  p999 %7.1f  max %7.1f us (at %.3f)  2nd half p99 %7.1f max %7.1f  batches %d  waits %d  max fill/launch/gpu/cb/wait %.0f/%.0f/%.0f/%.0f/%.0f us' % (j['rate'], j['packets_per_s'], j['lat_us_p50'], j['lat_us_p99'], j['lat_us_p999'], j['lat_us_max'], j['worst_at'], j['late_half_p99'], j['late_half_max'], j['batches'], j['submit_waits'], j['max_fill_us'], j['max_launch_us'], j['max_gpu_us'], j['max_callback_us'], j['max_submit_wait_us']))
"
exit $rc
