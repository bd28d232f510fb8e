# Copying-path half-load tail: a saturation run, then six open-loop runs at
# half its rate with LCB_QUEUE_TRACE=1 (stall trace points: late completer
# pick-ups, flusher waits for a free slot, submits waiting for an open slot),
# the cgroup's CPU throttling counters read around each run.
# usage: bash tools/queue_tail_r8.sh <out dir under gpurun_out>
O=${1:-gpurun_out/qt}
mkdir -p $O
Q=tools/queue_bench
cg() { for f in /sys/fs/cgroup/cpu.stat /sys/fs/cgroup/cpu/cpu.stat /sys/fs/cgroup/cpu,cpuacct/cpu.stat; do [ -r $f ] && { tr "\n" " " < $f; echo; return; }; done; echo "no cpu.stat"; }
timeout -k 10 120 $Q --alg 1 --packets 2097152 --size 1024 --threads 8 > $O/sat.json 2> $O/sat.err || exit 1
RATE=$(python3 -c "import json;print(int(json.load(open('$O/sat.json'))['packets_per_s']/2))")
for i in 1 2 3 4 5 6; do
  echo "before $i: $(cg)" >> $O/cpu_stat.txt
  LCB_QUEUE_TRACE=1 timeout -k 10 120 $Q --alg 1 --packets 2097152 --size 1024 --threads 8 --rate $RATE > $O/half_$i.json 2> $O/half_$i.err || exit 1
  echo "after $i: $(cg)" >> $O/cpu_stat.txt
done
