#!/usr/bin/env python3
"""Generate tests/golden/crc32.json (run ONLY in the build container).

Pure data fixtures for the CRC-32 family of include/math/crc32.h:

kat
    The reference's own known-answer table, extracted as data from
    crc32_self_test() (crc32.h:581-657: three strings x crc32a/b/c/d/q) and
    the catalogue check values in the variant comments (crc32.h:501-576,
    "check=0x..." = CRC of "123456789"), each re-derived by the compiled
    reference (oracle/_ref/libref_hash.so) before it is written.
batches
    CRCs computed by the compiled reference over synthetic batches from the
    SURVEY.md 8d generator: ragged lengths 0..1100 (every CRC kept), byte-
    misaligned starts, the X_update form with per-buffer initial values, and
    65536 / 1048576 x 1 KiB ("crc of crcs": SHA-256 over the packed LE u32
    array, so the GPU box can check a full 1 GiB pass).

Usage:  python3 tests/golden/make_golden_crc32.py   (needs `make -C oracle`)
"""
import hashlib
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle.pyoracle import CRC_VARIANTS, SEED, Ref, gen_stream  # noqa: E402

REF_HDR = "/root/reference/include/math/crc32.h"
VID = {v: k for k, v in CRC_VARIANTS.items()}


def extract_kat():
    src = open(REF_HDR).read()
    body = src[src.index("crc32_self_test(void)"):]
    strings = re.findall(r'"((?:[^"\\]|\\.)*)"', body[:body.index("data_size")])
    sizes = [int(x) for x in re.search(r"data_size\[\]\s*=\s*\{([^}]*)\}", body).group(1).split(",")]
    assert [len(s) for s in strings] == sizes, (strings, sizes)
    cases = []
    for name in ("a", "b", "c", "d", "q"):
        vals = re.search(r"result_crc32%s\[\]\s*=\s*\{([^}]*)\}" % name, body).group(1)
        vals = [int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]+", vals)]
        for s, v in zip(strings, vals):
            cases.append({"variant": "crc32" + name, "msg": s.encode().hex(), "crc": "%08x" % v,
                          "source": "crc32.h:581-657"})
    # catalogue check values: the comment block above each macro pair
    for m in re.finditer(r"check=0x([0-9a-fA-F]{8}).*?\n#define (crc32\w+)_update", src, re.S):
        cases.append({"variant": m.group(2), "msg": b"123456789".hex(), "crc": m.group(1).lower(),
                      "source": "crc32.h:501-576 (catalogue check)"})
    return cases


def main():
    ref = Ref()
    assert ref.crc32_self_test() == 0
    kat = extract_kat()
    assert len(kat) == 15 + 8, len(kat)
    for c in kat:
        m = np.frombuffer(bytes.fromhex(c["msg"]), np.uint8)
        got = ref.crc32_batch(VID[c["variant"]], m, np.zeros(1, np.uint64), np.array([m.size], np.uint32))
        assert "%08x" % got[0] == c["crc"], c
    batches = []

    def add(name, data_seed, lens, offs, dod=False, init=None, extra=None):
        total = int((offs + lens).max()) if len(lens) else 1
        data = gen_stream(data_seed, max(total, 1))
        e = {"name": name, "seed": data_seed, "crcs": {}}
        if extra:
            e.update(extra)
        for v, vn in CRC_VARIANTS.items():
            crc = ref.crc32_batch(v, data, offs, lens, init=init)
            e["crcs"][vn] = ("sha256:" + hashlib.sha256(crc.astype("<u4").tobytes()).hexdigest()) if dod \
                else crc.astype("<u4").tobytes().hex()
        batches.append(e)

    lens = np.arange(0, 1101, dtype=np.uint32)
    offs = np.zeros(len(lens), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    add("ragged_0_1100", SEED ^ 0xC3C, lens, offs, extra={"layout": "packed lengths 0..1100"})
    # byte-misaligned: message i at 4099*i + (i % 16), length 1 + (i*37 % 1500)
    n = 512
    lens = np.array([1 + (i * 37) % 1500 for i in range(n)], np.uint32)
    offs = np.array([4099 * i + (i % 16) for i in range(n)], np.uint64)
    add("misaligned_512", SEED ^ 0xC3D, lens, offs,
        extra={"layout": "offset 4099*i + i%16, length 1 + (37*i % 1500)"})
    # X_update form: init[i] = (i * 2654435761) mod 2^32, lengths 0..299
    lens = np.arange(0, 300, dtype=np.uint32)
    offs = np.zeros(len(lens), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    init = (np.arange(len(lens), dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32)
    add("update_0_299", SEED ^ 0xC3E, lens, offs, init=init,
        extra={"layout": "packed lengths 0..299", "init": "i * 2654435761 mod 2^32"})
    for count, name in ((1 << 16, "C2_64k_x_1k"), (1 << 20, "C3_1M_x_1k")):
        lens = np.full(count, 1024, np.uint32)
        offs = np.arange(count, dtype=np.uint64) * 1024
        add(name, SEED, lens, offs, dod=True, extra={"layout": "fixed stride 1024", "count": count})
    json.dump({"source": "include/math/crc32.h compiled from /root/reference (oracle/_ref)",
               "kat": kat, "batches": batches}, open(os.path.join(HERE, "crc32.json"), "w"), indent=0)
    print("crc32.json: %d kat, %d batches" % (len(kat), len(batches)))


if __name__ == "__main__":
    main()
