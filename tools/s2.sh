#!/bin/bash
# Session r3 s2: GOST persistent-grid A/B, the new ragged tile kernel (packets,
# C4, ragged 1 KiB; reference dods checked), then every GPU test.
set -u
mkdir -p gpurun_out/s2
timeout -k 10 400 tools/ab_gost3.sh > gpurun_out/s2/gost_ab.log 2>&1 || exit $?
tail -2 gpurun_out/s2/gost_ab.log
timeout -k 10 300 python tools/pkt_bench.py --steps 10 > gpurun_out/s2/pkt.log 2>&1 || { tail -5 gpurun_out/s2/pkt.log; exit 1; }
cat gpurun_out/s2/pkt.log | grep -v amdgpu
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/s2/pytest.log; exit $rc
