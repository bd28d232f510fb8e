#!/usr/bin/env python3
"""Code-size record of the built library: the .so size,
the gfx950 code objects' total size and the sorted list of kernel symbols
(demangled), written to tests/golden/codesize.json.  tests/test_codesize.py
fails when the library grows more than 10 % past the record or gains a
kernel the record does not list (DESIGN.md 9 finding 12: a 33 MB library
ran the headline's first timed steps 7 % slower than an 18 MB one).

usage: python3 tools/codesize.py [--write]"""
import json
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "liblcb_amd", "liblcb_hash_gpu.so")
OUT = os.path.join(ROOT, "tests", "golden", "codesize.json")


def measure(so=SO):
    kr = runpy.run_path(os.path.join(ROOT, "tools", "kernel_resources.py"))
    cos = kr["code_objects"](so)
    # kernel names with their template arguments, without the parameter list
    names = sorted(set(r["name"].split("(")[0] for r in kr["kernels"](so)))
    return {"so_bytes": os.path.getsize(so), "code_object_bytes": sum(len(c) for c in cos),
            "kernels": names}


def main(argv):
    rec = measure()
    print(json.dumps({k: v for k, v in rec.items() if k != "kernels"} | {"kernels": len(rec["kernels"])}))
    if "--write" in argv:
        json.dump(rec, open(OUT, "w"), indent=1)
        print("wrote", OUT)


if __name__ == "__main__":
    main(sys.argv[1:])
