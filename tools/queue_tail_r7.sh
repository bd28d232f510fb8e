mkdir -p gpurun_out/r7m
Q=tools/queue_bench
timeout -k 10 120 $Q --alg 1 --packets 2097152 --size 1024 --threads 8 > gpurun_out/r7m/sat.json 2> gpurun_out/r7m/sat.err || exit 1
RATE=$(python3 -c "import json;print(int(json.load(open('gpurun_out/r7m/sat.json'))['packets_per_s']/2))")
for i in 1 2 3; do
  LCB_QUEUE_TRACE=1 timeout -k 10 120 $Q --alg 1 --packets 2097152 --size 1024 --threads 8 --rate $RATE > gpurun_out/r7m/half_$i.json 2> gpurun_out/r7m/half_$i.err || exit 1
done
