#!/usr/bin/env python3
"""Per-pass timeline of the 1M-packet rows from a rocprofv3 kernel trace of
tools/pkt_bench.py (tools/pkt_session.sh): for the last pass of each row
(plain / HMAC / keyed HMAC / keyed suffix tile kernels), every operation
since the previous pass's tile kernel with its duration and the idle gap
before it.

usage: pkt_gaps.py gpurun_out/<tag>/kt_<lib>/run_kernel_trace.csv"""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("lcbgpu::", ""),
            int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "gen_kernel" not in r["Kernel_Name"]]
    for mode, name in (("0>", "plain"), ("1>", "hmac"), ("2>", "keyed_hmac"), ("3>", "keyed_suffix")):
        idx = [i for i, (n, _, _) in enumerate(seq) if "md_tiles_kernel<" in n and n.endswith(mode)]
        if len(idx) < 2:
            continue
        i, j = idx[-1], idx[-2]
        ops = seq[j + 1:i + 1]
        gaps = sum(s - e for (_, s, _), (_, _, e) in zip(ops, [seq[j]] + ops[:-1])) / 1e3
        print("%-13s pass %.1f us (tile kernel %.1f, other ops %.1f, idle %.1f)" % (
            name, (seq[i][2] - seq[j][2]) / 1e3, (seq[i][2] - seq[i][1]) / 1e3,
            sum(e - s for _, s, e in ops[:-1]) / 1e3, gaps))
        prev = seq[j][2]
        for n, s, e in ops:
            print("    %-45s dur %6.1f  gap %6.1f" % (n[:45], (e - s) / 1e3, (s - prev) / 1e3))
            prev = e


if __name__ == "__main__":
    main(sys.argv[1])
