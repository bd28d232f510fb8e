#!/usr/bin/env python3
"""Stamps that tie a committed counter file (profiles/pmc_<alg>.json,
profiles/valu_counts.json) to the kernel code it was measured on.

The stamp of a kernel is the sha256 of its machine code: the bytes of its
function symbol in the gfx950 code object inside the built library (found
through the offload bundles, as tools/kernel_resources.py does; ELF parsed
here, no external tool).  bench.py recomputes the stamp of the kernel a
counter file names from the library it loaded and uses the file only when
the stamps agree, so a counter measured on an earlier build is never
reported against a later kernel.

usage: codestamp.py [lib.so] [symbol-substring ...]   (lists matching kernels)"""
import hashlib
import os
import struct
import sys

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


def functions(elf):
    """{symbol name: machine-code bytes} of the STT_FUNC symbols of an ELF64."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        return {}
    shoff = struct.unpack_from("<Q", elf, 0x28)[0]
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    secs = []
    for k in range(shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, shoff + k * shentsize)
        secs.append((typ, addr, off, size, link, entsize))
    out = {}
    for typ, addr, off, size, link, entsize in secs:
        if typ != 2 or not entsize:          # SHT_SYMTAB
            continue
        stroff = secs[link][2]
        for j in range(size // entsize):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from(
                "<IBBHQQ", elf, off + j * entsize)
            if (st_info & 0xF) != 2 or st_shndx >= len(secs) or not st_size:   # STT_FUNC
                continue
            end = elf.index(b"\0", stroff + st_name)
            name = elf[stroff + st_name:end].decode()
            s_addr, s_off = secs[st_shndx][1], secs[st_shndx][2]
            out[name] = elf[s_off + (st_value - s_addr):s_off + (st_value - s_addr) + st_size]
    return out


def kernel_stamps(so_path):
    """{mangled kernel symbol: sha256 of its machine code} over the library."""
    out = {}
    for elf in code_objects(so_path):
        for name, code in functions(elf).items():
            out[name] = hashlib.sha256(code).hexdigest()
    return out


def stamp_of(so_path, symbol, _cache={}):
    key = (os.path.abspath(so_path), os.path.getmtime(so_path))
    if key not in _cache:
        _cache[key] = kernel_stamps(so_path)
    return _cache[key].get(symbol)


def find(so_path, *parts):
    """Mangled kernel symbols containing every substring of `parts`."""
    return sorted(n for n in kernel_stamps(so_path) if all(p in n for p in parts))


if __name__ == "__main__":
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "liblcb_amd", "liblcb_hash_gpu.so")
    st = kernel_stamps(so)
    for n in sorted(st):
        if all(p in n for p in sys.argv[2:]):
            print(st[n][:16], n)
