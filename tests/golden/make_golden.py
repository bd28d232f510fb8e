#!/usr/bin/env python3
"""Generate the committed golden fixtures (run ONLY in the build container).

Two kinds of fixture, both pure data (inputs + expected outputs):

kat.json
    The reference's own known-answer tables, extracted as data from the
    self-test functions of /root/reference/include/crypto/hash/*.h
    (md5.h:440-512, sha1.h:990-1077, sha2.h:915-1132,
    gost3411-2012.h:2026-2257), plus chunked-update cases that mirror
    sha1.h:1059-1062 ("million a") and gost3411-2012.h:2162-2230 (every
    chunk size).  Every extracted digest is re-derived by the compiled
    reference (oracle/_ref/libref_hash.so) before it is written.

batches.json
    Digests computed by the compiled reference over synthetic batches from
    the counter-based generator: the packed input stream is the
    little-endian u64 words mix64(seed ^ k), k = 0, 1, ...  Small batches keep
    every digest; large ones (BASELINE configs C2/C3) keep SHA-256 over the
    packed digest array ("digest of digests") so the GPU box can check a full
    1M x 1 KiB pass without shipping megabytes.  MD/SHA batches are also
    cross-checked against Python hashlib/hmac (OpenSSL).

Usage:  python3 tests/golden/make_golden.py   (needs `make -C oracle` first)
"""
import ctypes
import hashlib
import hmac as pyhmac
import json
import os
import re
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_HDR = "/root/reference/include/crypto/hash"
REF_SO = os.path.join(REPO, "oracle", "_ref", "libref_hash_simd.so")
REF_SO_GENERIC = os.path.join(REPO, "oracle", "_ref", "libref_hash.so")

ALGS = {"md5": 1, "sha1": 2, "sha224": 3, "sha256": 4, "sha384": 5,
        "sha512": 6, "gost256": 7, "gost512": 8}
DSIZE = {1: 16, 2: 20, 3: 28, 4: 32, 5: 48, 6: 64, 7: 32, 8: 64}
PYNAME = {1: "md5", 2: "sha1", 3: "sha224", 4: "sha256", 5: "sha384", 6: "sha512"}
SEED = 0x6C62636861736821

M64 = (1 << 64) - 1


def gen_stream(seed, nbytes):
    """Packed synthetic input: u64 words mix64(seed ^ k), little-endian."""
    nw = (nbytes + 7) // 8
    k = np.arange(nw, dtype=np.uint64)
    z = (k ^ np.uint64(seed)) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:nbytes]


# ------------------------------------------------------------ KAT parsing
def _block(src, name):
    i = src.index(name)
    j = src.index("};", i)
    return src[i:j]


def _strings(block):
    out = []
    for m in re.finditer(r'"((?:[^"\\]|\\.)*)"', block):
        out.append(m.group(1).encode().decode("unicode_escape").encode("latin-1"))
    return out


def _ints(block):
    body = block[block.index("{") + 1:]
    return [int(x) for x in re.findall(r"\b\d+\b", body)]


def kat_md_sha(fname, prefix):
    src = open(os.path.join(REF_HDR, fname)).read()
    fn = src[src.index(prefix + "_self_test(void)"):]
    data = _strings(_block(fn, "*data[]"))
    sizes = _ints(_block(fn, "data_size[]"))
    rep = _ints(_block(fn, "repeat_count[]")) if "repeat_count[]" in fn else [1] * len(data)
    assert len(data) == len(sizes) == len(rep)
    msgs = [d[:s] for d, s in zip(data, sizes)]
    return fn, msgs, rep


def build_kat():
    cases = []
    # MD5 (md5.h:440-512): digests, then HMAC with key = message.
    fn, msgs, rep = kat_md_sha("md5.h", "md5")
    dig = _strings(_block(fn, "*result_digest[]"))
    hdig = _strings(_block(fn, "*result_hdigest[]"))
    for m, d, h in zip(msgs, dig, hdig):
        cases.append(dict(alg="md5", msg=m.hex(), repeat=1, digest=d.decode()))
        cases.append(dict(alg="md5", key=m.hex(), msg=m.hex(), repeat=1, digest=h.decode()))
    # SHA-1 (sha1.h:990-1077): repeat counts apply to the digest test only.
    fn, msgs, rep = kat_md_sha("sha1.h", "sha1")
    dig = _strings(_block(fn, "*result_digest[]"))
    hdig = _strings(_block(fn, "*result_hdigest[]"))
    for m, r, d, h in zip(msgs, rep, dig, hdig):
        c = dict(alg="sha1", msg=m.hex(), repeat=r, digest=d.decode())
        if r > 1:  # sha1.h:1059-1062 feeds each repetition as its own update
            c["chunks"] = [len(m)]
        cases.append(c)
        cases.append(dict(alg="sha1", key=m.hex(), msg=m.hex(), repeat=1, digest=h.decode()))
    # SHA-2 (sha2.h:915-1132): 224/256/384/512 digests, HMAC 256/384/512.
    fn, msgs, rep = kat_md_sha("sha2.h", "sha2")
    for bits in (224, 256, 384, 512):
        dig = _strings(_block(fn, "*result_digest%d[]" % bits))
        assert len(dig) == len(msgs)
        for m, d in zip(msgs, dig):
            cases.append(dict(alg="sha%d" % bits, msg=m.hex(), repeat=1,
                              digest=d.decode()[:2 * DSIZE[ALGS["sha%d" % bits]]]))
    for bits in (256, 384, 512):
        hdig = _strings(_block(fn, "*result_hdigest%d[]" % bits))
        assert len(hdig) == len(msgs)
        for m, d in zip(msgs, hdig):
            cases.append(dict(alg="sha%d" % bits, key=m.hex(), msg=m.hex(), repeat=1,
                              digest=d.decode()[:2 * DSIZE[ALGS["sha%d" % bits]]]))
    # GOST (gost3411-2012.h:2026-2131).
    src = open(os.path.join(REF_HDR, "gost3411-2012.h")).read()
    arrays = {}
    for name in ("gost3411_2012_hash_m2", "gost3411_2012_hash_m4",
                 "gost3411_2012_hmac_k1", "gost3411_2012_hmac_m1"):
        blk = _block(src, "%s[] = {" % name)
        arrays[name] = bytes(int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", blk))
    tbl = _block(src, "gost3411_2012_hash_tst[] = {")
    tbl = src[src.index("gost3411_2012_hash_tst[] = {"):src.index("#define GOST3411_2012_TEST_IDX")]
    for ent in re.split(r"\},\s*\{", tbl):
        mm = re.search(r"\.msg =\*/\s*(.*?),\s*\n", ent)
        if not mm:
            continue
        expr = mm.group(1).strip()
        am = re.search(r"\(const char\*\)(\w+)", expr)
        msg = arrays[am.group(1)] if am else _strings(expr)[0]
        size = re.search(r"\.msg_size =\*/\s*(\w+\(?\w*\)?)", ent).group(1)
        size = len(msg) if size.startswith("sizeof") else int(size)
        msg = msg[:size]
        for bits in (256, 512):
            hm = re.search(r"\.hash%d =\*/\s*(\"[0-9a-f]+\"|NULL)" % bits, ent)
            if hm and hm.group(1) != "NULL":
                d = hm.group(1).strip('"')
                cases.append(dict(alg="gost%d" % bits, msg=msg.hex(), repeat=1, digest=d))
                # gost3411-2012.h:2162-2230: every update chunk size 1..len-1.
                cases.append(dict(alg="gost%d" % bits, msg=msg.hex(), repeat=1, digest=d,
                                  chunks=list(range(1, len(msg)))))
    htbl = src[src.index("gost3411_2012_hmac_tst[] = {"):]
    htbl = htbl[:htbl.index("};")]
    for bits in (256, 512):
        d = re.search(r"\.hmac%d =\*/\s*\"([0-9a-f]+)\"" % bits, htbl).group(1)
        cases.append(dict(alg="gost%d" % bits, key=arrays["gost3411_2012_hmac_k1"].hex(),
                          msg=arrays["gost3411_2012_hmac_m1"].hex(), repeat=1, digest=d))
    return cases


# -------------------------------------------------------- reference calls
class Ref:
    def __init__(self, path):
        self.lib = ctypes.CDLL(path)
        self.lib.ref_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
        self.lib.ref_chunked.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                         ctypes.c_size_t, ctypes.c_char_p]

    def batch(self, alg, base, offsets=None, lengths=None, count=1, stride=0, fixed_len=0, key=None):
        base = np.ascontiguousarray(base, dtype=np.uint8)
        out = np.zeros(count * DSIZE[alg], dtype=np.uint8)
        kb = ctypes.c_char_p(key) if key is not None else None
        off = offsets.ctypes.data if offsets is not None else None
        ln = lengths.ctypes.data if lengths is not None else None
        rc = self.lib.ref_batch(alg, kb, len(key) if key else 0, base.ctypes.data, off, ln,
                                count, stride, fixed_len, out.ctypes.data)
        assert rc == 0
        return out

    def batch_mt(self, alg, base, count, stride, fixed_len, key=None, threads=8):
        """Fixed-stride batch split over threads (ctypes drops the GIL)."""
        out = np.zeros(count * DSIZE[alg], dtype=np.uint8)
        per = (count + threads - 1) // threads
        kb = ctypes.c_char_p(key) if key is not None else None

        def work(t):
            lo, hi = t * per, min(count, (t + 1) * per)
            if lo >= hi:
                return
            self.lib.ref_batch(alg, kb, len(key) if key else 0, base.ctypes.data + lo * stride,
                               None, None, hi - lo, stride, fixed_len,
                               out.ctypes.data + lo * DSIZE[alg])
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(work, range(threads)))
        return out

    def chunked(self, alg, msg, chunk):
        out = ctypes.create_string_buffer(64)
        assert self.lib.ref_chunked(alg, msg, len(msg), chunk, out) == 0
        return out.raw[:DSIZE[alg]]


def dod(digests):
    return hashlib.sha256(digests.tobytes()).hexdigest()


def pycheck(alg, msgs, digests, key=None):
    if alg not in PYNAME:
        return
    ds = DSIZE[alg]
    for i, m in enumerate(msgs):
        if key is None:
            exp = hashlib.new(PYNAME[alg], m).digest()
        else:
            exp = pyhmac.new(key, m, PYNAME[alg]).digest()
        assert exp == digests[i * ds:(i + 1) * ds].tobytes(), (alg, i)


def mixed_lengths(seed, count):
    """C4 length rule: {64, 1024, 65536}[mix64(seed + i) % 3]."""
    out = []
    for i in range(count):
        z = (seed + i + 0x9E3779B97F4A7C15) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        z ^= z >> 31
        out.append((64, 1024, 65536)[z % 3])
    return out


HMAC_KEYS = {  # key lengths around the 64 / 128 byte block boundaries
    "k0": b"", "k16": bytes(range(16)), "k64": bytes(range(64)),
    "k65": bytes(range(65)), "k128": bytes(range(128)), "k129": bytes(range(129)),
    "k200": bytes((7 * i) & 0xFF for i in range(200)),
}


def build_batches(ref, full):
    out = {"seed": SEED, "generator": "u64 words mix64(seed ^ k), little-endian", "batches": []}
    B = out["batches"]

    # 1) ragged packed batch, lengths 0..4159, contiguous.
    lens = np.arange(4160, dtype=np.uint32)
    offs = np.zeros(len(lens), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(lens.sum())
    data = gen_stream(SEED, total)
    msgs = [data[int(o):int(o) + int(n)].tobytes() for o, n in zip(offs, lens)]
    for name, alg in ALGS.items():
        d = ref.batch(alg, data, offs, lens, len(lens))
        pycheck(alg, msgs, d)
        B.append(dict(name="ragged_0_4159", alg=name, layout="packed", lengths="0..4159",
                      count=len(lens), dod=dod(d), first=d[:8 * DSIZE[alg]].tobytes().hex()))
        for kname, key in HMAC_KEYS.items():
            d = ref.batch(alg, data, offs, lens, len(lens), key=key)
            pycheck(alg, msgs, d, key)
            B.append(dict(name="ragged_0_4159", alg=name, layout="packed", lengths="0..4159",
                          count=len(lens), key=kname, key_hex=key.hex(), dod=dod(d)))

    # 2) misaligned: 2048 messages, lengths 0..300, 0..15 byte gaps (any alignment).
    rng = np.random.RandomState(1234)
    lens = rng.randint(0, 301, size=2048).astype(np.uint32)
    gaps = rng.randint(0, 16, size=2048).astype(np.uint64)
    offs = np.zeros(2048, dtype=np.uint64)
    pos = 0
    for i in range(2048):
        pos += int(gaps[i])
        offs[i] = pos
        pos += int(lens[i])
    data = gen_stream(SEED ^ 0x5A5A, pos)
    msgs = [data[int(o):int(o) + int(n)].tobytes() for o, n in zip(offs, lens)]
    for name, alg in ALGS.items():
        d = ref.batch(alg, data, offs, lens, 2048)
        pycheck(alg, msgs, d)
        B.append(dict(name="misaligned_2048", alg=name, layout="rng1234", seed_xor=0x5A5A,
                      count=2048, lengths=lens.tolist(), offsets=offs.tolist(), dod=dod(d)))

    # 3) one big buffer each: 64 KiB and 64 KiB + 1.
    for n in (65536, 65537):
        data = gen_stream(SEED, n)
        for name, alg in ALGS.items():
            d = ref.batch(alg, data, None, None, 1, 0, n)
            B.append(dict(name="big_%d" % n, alg=name, count=1, fixed_len=n, digest=d.tobytes().hex()))

    # 4) C4-like mixed lengths {64, 1 KiB, 64 KiB}, 512 buffers, packed.
    lens = np.array(mixed_lengths(SEED, 512), dtype=np.uint32)
    offs = np.zeros(512, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = gen_stream(SEED, int(lens.sum()))
    for name, alg in ALGS.items():
        d = ref.batch(alg, data, offs, lens, 512)
        B.append(dict(name="mixed_512", alg=name, layout="packed", lengths="mix64(seed+i)%3",
                      count=512, dod=dod(d)))

    # 4b) larger mixed batch: above the bucketing threshold (4096) of the GPU
    #     path, so the length-bucketed ordering is exercised at C4's mix.
    lens = np.array(mixed_lengths(SEED ^ 0xC4, 16384), dtype=np.uint32)
    offs = np.zeros(16384, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = gen_stream(SEED ^ 0xC4, int(lens.sum()))
    for name, alg in ALGS.items():
        d = ref.batch(alg, data, offs, lens, 16384)
        B.append(dict(name="mixed_16384", alg=name, layout="packed", lengths="mix64(seed^0xc4+i)%3",
                      seed_xor=0xC4, count=16384, dod=dod(d)))
        if name in ("md5", "sha256"):
            dk = ref.batch(alg, data, offs, lens, 16384, key=HMAC_KEYS["k65"])
            B.append(dict(name="mixed_16384", alg=name, layout="packed", seed_xor=0xC4,
                          count=16384, key="k65", key_hex=HMAC_KEYS["k65"].hex(), dod=dod(dk)))

    # 5) fixed-stride 1 KiB batches: 1024 (full digests kept for MD5), C2 64K, C3 1M.
    sizes = [(1024, "fixed1k_1024"), (65536, "C2_64k_x_1k")]
    if full:
        sizes.append((1 << 20, "C3_1M_x_1k"))
    for count, tag in sizes:
        data = gen_stream(SEED, count * 1024)
        for name, alg in ALGS.items():
            d = ref.batch_mt(alg, data, count, 1024, 1024)
            if count == 1024:
                pycheck(alg, [data[i * 1024:(i + 1) * 1024].tobytes() for i in range(count)], d)
            ent = dict(name=tag, alg=name, count=count, stride=1024, fixed_len=1024, dod=dod(d))
            if count == 1024:
                ent["first"] = d[:16 * DSIZE[alg]].tobytes().hex()
            B.append(ent)
            if count <= 65536:
                dk = ref.batch_mt(alg, data, count, 1024, 1024, key=HMAC_KEYS["k16"])
                B.append(dict(name=tag, alg=name, count=count, stride=1024, fixed_len=1024,
                              key="k16", key_hex=HMAC_KEYS["k16"].hex(), dod=dod(dk)))
            print("  %s %s done" % (tag, name), flush=True)
    return out


def main():
    if not os.path.isdir(REF_HDR):
        sys.exit("reference headers absent: fixtures can only be regenerated in the build container")
    ref = Ref(REF_SO_GENERIC)
    assert ref.lib.ref_self_test() == 0, "reference self test failed"
    cases = build_kat()
    # Re-derive every KAT digest with the compiled reference.
    for c in cases:
        alg = ALGS[c["alg"]]
        msg = bytes.fromhex(c["msg"]) * c.get("repeat", 1)
        if "key" in c:
            got = ref.batch(alg, np.frombuffer(msg, dtype=np.uint8) if msg else np.zeros(1, np.uint8),
                            None, None, 1, 0, len(msg), key=bytes.fromhex(c["key"])).tobytes()
        else:
            got = ref.chunked(alg, msg, 0)
        assert got.hex() == c["digest"], c
        for ch in c.get("chunks", []):
            assert ref.chunked(alg, msg, ch).hex() == c["digest"], (c["alg"], ch)
    json.dump({"source": "reference self tests (md5.h, sha1.h, sha2.h, gost3411-2012.h)",
               "cases": cases}, open(os.path.join(HERE, "kat.json"), "w"), indent=0)
    print("kat.json: %d cases" % len(cases))
    refs = Ref(REF_SO)
    b = build_batches(refs, full="--no-full" not in sys.argv)
    json.dump(b, open(os.path.join(HERE, "batches.json"), "w"), indent=0)
    print("batches.json: %d entries" % len(b["batches"]))


if __name__ == "__main__":
    main()
