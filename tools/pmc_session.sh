#!/bin/bash
# Counter session (GPU box): rocprofv3 --pmc passes, one counter group per
# run (FETCH_SIZE and WRITE_SIZE never together: TCC slots), over
#   kb_<i>      tools/kbench.py, every algorithm on the bench workload;
#   kt_pkt_<i>  the 1M-packet workload (plain MD5: md_tiles_kernel<Md5, 0>);
#   kt_c4_<i>   the C4 workload (MD5, the same kernel);
# then tools/pmc_collect.py <dir> <tag> on the build host writes the stamped
# profiles/pmc_*.json and valu_counts.json.  Each pass has its own limit; the
# script stops at the first failure.   TAG=r4p bash tools/pmc_session.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4c}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $O/kb_$i -o run --output-format csv -- python3 $R/tools/kbench.py --alg md5,sha1,sha224,sha256,sha384,sha512,gost256,gost512 --reps 3 --warmup 3 > $O/kb_$i.log 2>&1
  rc=$?; echo "kb $i ($grp) rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
# MD5 fixed-stride kernel only: wave occupancy and clock (SQ_WAVE_CYCLES /
# SQ_BUSY_CYCLES), and why the dispatcher could not place a workgroup
# (SPI resource-allocation stalls: LDS full, workgroup limit).
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS -d $O/kb_occ -o run --output-format csv -- python3 $R/tools/kbench.py --alg md5,sha1,sha256,sha512,gost256 --reps 5 --warmup 5 > $O/kb_occ.log 2>&1
rc=$?; echo "kb occ rc=$rc"; [ $rc -ne 0 ] && exit $rc
# GOST: LDS-array cycles, bank-conflict cycles, LDS instructions of the
# plain kernel and of its bare LPS chain (the probe), with the clock.
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES SQ_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $O/kb_lds -o run --output-format csv -- python3 $R/tools/kbench.py --alg gost256,gost512 --reps 5 --warmup 3 --gost-probe > $O/kb_lds.log 2>&1
rc=$?; echo "kb lds rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 90 rocprofv3 --pmc SPI_RA_LDS_CU_FULL_CSN SPI_RA_TGLIM_CU_FULL_CSN -d $O/kb_spi -o run --output-format csv -- python3 $R/tools/kbench.py --alg md5 --reps 5 --warmup 5 > $O/kb_spi.log 2>&1
rc=$?; echo "kb spi rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VALU -d $O/kt_pktocc -o run --output-format csv -- python3 $R/tools/pkt_bench.py --steps 3 --no-layouts --no-c4 > $O/kt_pktocc.log 2>&1
rc=$?; echo "kt pkt occ rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $O/kt_pkt_$i -o run --output-format csv -- python3 $R/tools/pkt_bench.py --steps 3 --no-layouts --no-c4 > $O/kt_pkt_$i.log 2>&1
  rc=$?; echo "kt_pkt $i ($grp) rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $O/kt_c4_$i -o run --output-format csv -- python3 $R/tools/pkt_bench.py --steps 3 --no-layouts --no-packets > $O/kt_c4_$i.log 2>&1
  rc=$?; echo "kt_c4 $i ($grp) rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
