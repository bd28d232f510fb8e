#!/bin/bash
# PMC passes over tools/gost_lanes_ab (build_exp/gost_lanes_ab): VALU / LDS
# instruction counts, busy and wait cycles, LDS bank conflicts, and the
# shader clock (GRBM_GUI_ACTIVE over the kernel time) per layout.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gost_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- $R/build_exp/gost_lanes_ab 1048576 2 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
