# s15: queue slots 4 vs 8 (copying and zero copy), then the round-4 PMC session.
set -o pipefail
O=gpurun_out/s15; mkdir -p $O
for sl in 4 8; do for zc in 0 1; do
  timeout -k 10 120 tools/queue_bench --alg 1 --packets 2097152 --size 1024 --threads 8 --slots $sl --zerocopy $zc > $O/q_s${sl}_zc$zc.json 2> $O/q_s${sl}_zc$zc.err; rc=$?; cut -c1-200 $O/q_s${sl}_zc$zc.json; [ $rc -ne 0 ] && exit $rc
done; done
TAG=r4a bash tools/pmc_session.sh
