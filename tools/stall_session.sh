#!/bin/bash
# Stall counters of the fixed-stride kernels (SHA-1 runs
# ~8 % under its VALU floor at its clock; MD5 and SHA-256 do not): three
# rocprofv3 --pmc passes (8 SQ counters at most each) over tools/kbench.py
# md5,sha1,sha256, then tools/stall_summary.py <dir> on the build host.
#   TAG=r7s bash tools/stall_session.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r7s}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_IFETCH_LEVEL SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/st_$i -o run --output-format csv -- python3 $R/tools/kbench.py --alg md5,sha1,sha256 --reps 5 --warmup 20 > $O/st_$i.log 2>&1
  rc=$?; echo "stall pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
