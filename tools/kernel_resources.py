#!/usr/bin/env python3
"""Per-kernel resources of the BUILT library (liblcb_amd/liblcb_hash_gpu.so):
VGPRs, SGPRs, scratch bytes per lane, LDS bytes per workgroup, read from the
gfx950 code objects' AMDHSA metadata notes (what the GPU actually loads, not
a recompile).  The offload bundles of every translation unit are found in
the .so, the gfx950 ELF of each is cut out and `llvm-readelf --notes`
prints its kernel table.

usage: python3 tools/kernel_resources.py [--spills] [path/to/lib.so]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_SO = os.path.join(ROOT, "liblcb_amd", "liblcb_hash_gpu.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(so_path, arch="gfx950"):
    """The `arch` device ELFs of every offload bundle in the shared object."""
    data = open(so_path, "rb").read()
    out, i = [], 0
    while True:
        i = data.find(MAGIC, i)
        if i < 0:
            return out
        n = struct.unpack_from("<Q", data, i + len(MAGIC))[0]
        p = i + len(MAGIC) + 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl]
            p += tl
            if arch.encode() in triple and size:
                out.append(data[i + off:i + off + size])
        i += len(MAGIC)


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.split("\n")[:len(names)] if r.returncode == 0 else names


def kernels(so_path=DEFAULT_SO):
    """[{name, mangled, vgpr, sgpr, scratch, lds}] for every kernel."""
    rows = []
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(so_path)):
            path = os.path.join(td, "%d.co" % k)
            open(path, "wb").write(co)
            txt = subprocess.run([READELF, "--notes", path], capture_output=True, text=True,
                                 check=True).stdout
            # one YAML mapping per kernel inside amdhsa.kernels
            for blk in re.split(r"\n\s+- \.", txt)[1:]:
                blk = "." + blk
                m = re.search(r"\.name:\s+(\S+)", blk)
                if not m:
                    continue
                def num(key):
                    mm = re.search(r"\." + key + r":\s+(\d+)", blk)
                    return int(mm.group(1)) if mm else None
                rows.append({"mangled": m.group(1), "vgpr": num("vgpr_count"), "sgpr": num("sgpr_count"),
                             "scratch": num("private_segment_fixed_size"),
                             "lds": num("group_segment_fixed_size")})
    for r, d in zip(rows, demangle([r["mangled"] for r in rows])):
        r["name"] = d.replace("lcbgpu::", "")
    return rows


def main(argv):
    spills = "--spills" in argv
    args = [a for a in argv if not a.startswith("--")]
    rows = kernels(args[0] if args else DEFAULT_SO)
    for r in sorted(rows, key=lambda r: r["name"]):
        if spills and not r["scratch"]:
            continue
        print("%-90s vgpr %3s sgpr %3s scratch %4s lds %6s" % (r["name"][:90], r["vgpr"], r["sgpr"],
                                                              r["scratch"], r["lds"]))
    print("%d kernels, %d with scratch" % (len(rows), sum(1 for r in rows if r["scratch"])))


if __name__ == "__main__":
    main(sys.argv[1:])
