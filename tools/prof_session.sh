#!/bin/bash
# rocprofv3 session: kernel trace + stats, then one PMC pass per counter group.
# Counters in their own passes (no sys/runtime trace with --pmc).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_TAG:-prof}
ALGS=${ALGS:-md5,sha1,sha256,sha512,gost256}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/tools/kbench.py --alg $ALGS --reps 10 > $OUT/trace.log 2>&1 || exit $?
i=0
for grp in ${PMC_GROUPS:-"FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 $R/tools/kbench.py --alg $ALGS --reps 3 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc group $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc$i.log; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
