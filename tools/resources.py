#!/usr/bin/env python3
"""Per-kernel resource usage (VGPRs, AGPRs, scratch, occupancy, LDS) of a
HIP source, from hipcc's kernel-resource-usage remarks, one line per kernel.

usage: python3 tools/resources.py [liblcb_amd/csrc/lcb_kernels.hip] [-Dextra ...]"""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "liblcb_amd/csrc/lcb_kernels.hip"
extra = [a for a in sys.argv[1:] if a.startswith("-")]
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "-o", "/dev/null",
                    "-Rpass-analysis=kernel-resource-usage", src] + extra, capture_output=True, text=True)
if r.returncode:
    sys.exit(r.stderr[-3000:])
cur = None
rows = {}
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = cur.replace("lcbgpu::", "").replace("(KArgs)", "")
        rows[cur] = {}
        continue
    m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|SGPRs): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    print("%-60s vgpr %3s agpr %3s sgpr %3s scratch %4s occ %s lds %6s" % (
        k[:60], v.get("VGPRs"), v.get("AGPRs"), v.get("SGPRs"), v.get("ScratchSize"), v.get("Occupancy"), v.get("LDS")))
