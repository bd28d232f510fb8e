#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc -save-temps .s file.
usage: isa_stats.py file.s kernel-substring"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
m = [x for x in re.finditer(r"\n(_Z\w+):", s) if pat in x.group(1)]
start = m[0].end()
end = s.find(".Lfunc_end", start)
body = s[start:end].splitlines()
blocks, cur, name = [], [], "entry"
for l in body:
    if re.match(r"^\.LBB\w+:", l):
        blocks.append((name, cur)); name, cur = l.split(":")[0], []
    elif l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;") and l.strip():
        cur.append(l.split()[0])
blocks.append((name, cur))
for name, ins in blocks:
    if len(ins) < 40:
        continue
    c = collections.Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print("%s: %d instr, %d VALU, %d vmem, %d waitcnt" % (name, len(ins), valu,
          sum(v for k, v in c.items() if k.startswith(("global_", "buffer_", "flat_"))),
          c.get("s_waitcnt", 0)))
    print("   ", sorted(c.items(), key=lambda x: -x[1])[:14])
