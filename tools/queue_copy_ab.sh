# A/B of the queue's host -> device moves (round 7): one gather-copy kernel
# per batch (default) against hipMemcpyAsync per range (LCB_QUEUE_COPY=api).
# Copying and zero-copy paths, saturation then three open-loop runs at half
# its rate each, LCB_QUEUE_TRACE=1 (stalls over 1 ms on stderr).
# usage: bash tools/queue_copy_ab.sh <out dir under gpurun_out>
O=${1:-gpurun_out/qc}
mkdir -p $O
Q=tools/queue_bench
for mode in kernel api; do
  for zc in 0 1; do
    LCB_QUEUE_COPY=$mode timeout -k 10 120 $Q --alg 1 --packets 2097152 --size 1024 --threads 8 --zerocopy $zc > $O/${mode}_zc${zc}_sat.json 2> $O/${mode}_zc${zc}_sat.err || exit 1
    RATE=$(python3 -c "import json;print(int(json.load(open('$O/${mode}_zc${zc}_sat.json'))['packets_per_s']/2))")
    for i in 1 2 3; do
      LCB_QUEUE_TRACE=1 LCB_QUEUE_COPY=$mode timeout -k 10 120 $Q --alg 1 --packets 2097152 --size 1024 --threads 8 --zerocopy $zc --rate $RATE > $O/${mode}_zc${zc}_half_$i.json 2> $O/${mode}_zc${zc}_half_$i.err || exit 1
    done
  done
done
