#!/usr/bin/env python3
"""Median durations of the bucketing kernels (and the batch kernel after
them) in a rocprofv3 --kernel-trace rocpd database of tools/bucket_ab.py.

usage: python3 tools/bucket_trace.py <results.db>"""
import re
import sqlite3
import statistics as st
import sys
from collections import defaultdict


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    dur = defaultdict(list)
    for name, s, e in rows:
        m = re.match(r"(?:void )?(?:lcbgpu::)?([A-Za-z_0-9]+(?:<[^>]*>)?)", name)
        dur[m.group(1) if m else name[:40]].append((e - s) / 1000.0)
    for k, v in sorted(dur.items(), key=lambda kv: -len(kv[1])):
        if "bucket" in k or "tiles" in k:
            print("%-48s n=%4d median %8.2f us  min %8.2f" % (k[:48], len(v), st.median(v), min(v)))


if __name__ == "__main__":
    main()
