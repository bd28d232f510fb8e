R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5i; mkdir -p $O
for zc in 1 0 1 0; do
  LCB_QUEUE_TRACE=1 timeout -k 10 120 $R/tools/queue_bench --alg 1 --packets 6291456 --size 1024 --threads 8 --zerocopy $zc --rate 14000000 >> $O/q.jsonl 2>> $O/q.err
  rc=$?; [ $rc -ne 0 ] && exit $rc
  echo "=== end zc=$zc" >> $O/q.err
done
