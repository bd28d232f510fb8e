#!/usr/bin/env python3
"""Per-launch stall counters of the fixed-stride kernels from
tools/stall_session.sh (median over the profiled launches of each kernel),
with the ratios that name a stall: VALU-issue cycles per wave cycle, wait
cycles (any / instruction dependency / LDS) per wave cycle, instruction
fetch per VALU instruction, and the engine clock (GRBM_GUI_ACTIVE / 8 /
dispatch time is not available here: SQ_BUSY_CYCLES per XCD).  SQ_*_CYCLES
and SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md).

usage: stall_summary.py gpurun_out/<tag>"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "st_*", "run_counter_collection.csv"))):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].replace("void ", "").split("(")[0].strip().replace("lcbgpu::", "")
            per[(k, row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        for (k, _), cs in per.items():
            for c, v in cs.items():
                acc[k][c].append(v)
    out = {}
    for k, cs in acc.items():
        if "md_fixed" not in k:
            continue
        m = {c: statistics.median(v) for c, v in cs.items()}
        r = {"counters": {c: int(v) for c, v in sorted(m.items())}}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC"):
                if c in m:
                    r[c + "_per_wave_cycle"] = round(m[c] / wc, 4)
        if m.get("SQ_INSTS_VALU"):
            for c in ("SQ_IFETCH", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
                if c in m:
                    r[c + "_per_valu"] = round(m[c] / m["SQ_INSTS_VALU"], 4)
        out[k] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
