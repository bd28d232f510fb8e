#!/usr/bin/env python3
"""Instruction mix of the loops of one kernel in a hipcc -S (.s) file.

A loop is taken as the layout range [header, latch] of every backward branch
(latch -> header); its VALU count is the sum over the range's blocks (an
upper bound for loops with side branches, exact for the straight-line line
loops of the stream kernels).  Used to compare the VALU per streamed line of
md_tiles_kernel against md_fixed_* (VERDICT r4 item 1).

usage: isa_loops.py file.s kernel-substring [--min-valu 300]"""
import argparse
import collections
import re


def blocks_of(text, pat):
    m = [x for x in re.finditer(r"\n(_Z\w+):", text) if pat in x.group(1)]
    if not m:
        raise SystemExit("kernel %r not found" % pat)
    start = m[0].end()
    end = text.find(".Lfunc_end", start)
    out, cur, name = [], [], "entry"
    for line in text[start:end].splitlines():
        if re.match(r"^\.LBB\w+:", line):
            out.append((name, cur))
            name, cur = line.split(":")[0], []
        elif line.startswith("\t") and not line.startswith(("\t.", "\t;")) and line.strip():
            cur.append(line.strip())
    out.append((name, cur))
    return m[0].group(1), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--min-valu", type=int, default=300)
    a = ap.parse_args()
    name, blocks = blocks_of(open(a.asm).read(), a.kernel)
    pos = {b: i for i, (b, _) in enumerate(blocks)}
    print(name)
    for i, (b, ins) in enumerate(blocks):
        for x in ins:
            if not x.startswith(("s_cbranch", "s_branch")):
                continue
            tgt = x.split()[-1]
            if tgt in pos and pos[tgt] <= i:
                rng = blocks[pos[tgt]:i + 1]
                c = collections.Counter(y.split()[0] for _, bi in rng for y in bi)
                valu = sum(v for k, v in c.items() if k.startswith("v_"))
                if valu < a.min_valu:
                    continue
                keys = ("v_alignbyte_b32", "v_mov_b32_e32", "v_cndmask_b32_e64", "v_cndmask_b32_e32",
                        "v_xor_b32_e32", "ds_read_b128", "global_load_lds_dwordx4", "s_nop")
                print("loop %s..%s (%d blocks): %d VALU; %s" % (tgt, b, len(rng), valu,
                      ", ".join("%s %d" % (k, c[k]) for k in keys if c[k])))


if __name__ == "__main__":
    main()
