#!/bin/bash
# Round-3 profiling session: the ragged-packet rows (tools/pkt_bench.py), their
# kernel trace, PMC passes over the packet rows (HBM bytes, VALU/LDS/SALU
# instruction counts, wave/busy/wait cycles, shader clock), and GOST's HBM
# bytes and kernel time (kbench).  Each step has its own limit; the script
# stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r3d}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python tools/pkt_bench.py --steps 20 > $OUT/pkt.log 2>&1
rc=$?; echo "pkt rc=$rc"; grep -v amdgpu $OUT/pkt.log | tail -6; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o pkt --output-format csv -- python3 $R/tools/pkt_bench.py --steps 5 --no-c4 > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for grp in FETCH_SIZE WRITE_SIZE \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 $R/tools/pkt_bench.py --steps 3 --no-c4 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 $R/tools/kbench.py --alg gost256,gost512 --reps 3 --warmup 5 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 120 python3 $R/tools/kbench.py --alg gost256,gost512,md5 --reps 20 --warmup 10 > $OUT/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu $OUT/kbench.log
exit $rc
