# Hunt the blocking enqueue of the zero-copy path (r7x: one launch's run
# copies took 9 ms to enqueue): zero-copy saturation, then eight open-loop
# runs at half its rate with LCB_QUEUE_TRACE=2 (the queue's watchdog samples
# the flusher's stack while one launch's enqueues take over 2 ms), and three
# copying-path runs the same way.
# usage: bash tools/queue_stall_stacks.sh <out dir under gpurun_out>
O=${1:-gpurun_out/qs}
mkdir -p $O
Q=tools/queue_bench
for zc in 1 0; do
  timeout -k 10 120 $Q --alg 1 --packets 2097152 --size 1024 --threads 8 --zerocopy $zc > $O/zc${zc}_sat.json 2> $O/zc${zc}_sat.err || exit 1
  RATE=$(python3 -c "import json;print(int(json.load(open('$O/zc${zc}_sat.json'))['packets_per_s']/2))")
  N=8; [ $zc = 0 ] && N=3
  for i in $(seq 1 $N); do
    LCB_QUEUE_TRACE=2 timeout -k 10 120 $Q --alg 1 --packets 2097152 --size 1024 --threads 8 --zerocopy $zc --rate $RATE > $O/zc${zc}_half_$i.json 2> $O/zc${zc}_half_$i.err || exit 1
  done
done
