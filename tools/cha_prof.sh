#!/bin/bash
# rocprofv3 on the ChaCha microbenchmark: kernel trace + stats, then PMC
# passes (one counter group per run, no trace domains with --pmc).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_TAG:-chaprof}
ARGS=${CHA_ARGS:-"--rounds 20 --reps 3 --warmup 2"}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/tools/cha_bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
i=0
for grp in ${PMC_GROUPS:-"FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 $R/tools/cha_bench.py $ARGS > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc group $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc$i.log; exit $rc; fi
done
exit 0
