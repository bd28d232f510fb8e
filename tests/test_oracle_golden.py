"""Pin the oracle (oracle/lcb_oracle.c) before trusting it as the checker.

* every known-answer vector of the reference's own self tests
  (tests/golden/kat.json, extracted from md5.h / sha1.h / sha2.h /
  gost3411-2012.h), including the chunked-update variants;
* digests the compiled reference produced over synthetic batches
  (tests/golden/batches.json: ragged, misaligned, 64 KiB, mixed, 1 KiB x N);
* the compiled reference itself (oracle/_ref), when it has been built here.
"""
import hashlib

import numpy as np
import pytest

from oracle.pyoracle import Oracle, Ref, gen_stream
from tests.golden_util import check_entry, layout

ALG = {"md5": 1, "sha1": 2, "sha224": 3, "sha256": 4, "sha384": 5, "sha512": 6,
       "gost256": 7, "gost512": 8}


def test_kat_count(kat):
    # md5 14+14, sha1 16+16, sha2 19*4 + 19*3, gost 11 (+11 chunked) + 2 HMAC
    assert len(kat) == 217


def test_oracle_kat(kat, oracle):
    for c in kat:
        alg = ALG[c["alg"]]
        msg = bytes.fromhex(c["msg"]) * c.get("repeat", 1)
        if "key" in c:
            got = oracle.batch(alg, np.frombuffer(msg, np.uint8), lengths=[len(msg)], offsets=[0],
                               key=bytes.fromhex(c["key"]))[0].tobytes()
            assert got.hex() == c["digest"], c
        elif "chunks" in c:
            for ch in c["chunks"]:
                assert oracle.chunked(alg, msg, ch).hex() == c["digest"], (c["alg"], ch)
        else:
            got = oracle.batch(alg, np.frombuffer(msg, np.uint8), lengths=[len(msg)],
                               offsets=[0])[0].tobytes()
            assert got.hex() == c["digest"], c


SMALL = ("ragged_0_4159", "misaligned_2048", "big_65536", "big_65537", "mixed_512",
         "fixed1k_1024")


def test_oracle_batches(batches, oracle):
    n = 0
    for e in batches["batches"]:
        if e["name"] not in SMALL:
            continue
        if e["alg"].startswith("gost") and e["name"] == "mixed_512":
            continue  # 11 MB through the bit-serial LPS: covered by the GPU tests
        L = layout(e)
        data = gen_stream(L["seed"], L["nbytes"])
        d = oracle.batch(ALG[e["alg"]], data, L["offsets"], L["lengths"], L["count"],
                         L["stride"], L["fixed_len"], key=L["key"])
        check_entry(e, d)
        n += 1
    assert n > 100


@pytest.mark.parametrize("alg", ["md5", "sha1", "sha256", "sha512"])
def test_oracle_c2(batches, oracle, alg):
    """BASELINE config C2 (64K x 1 KiB) digest-of-digests, fast algorithms."""
    e = [x for x in batches["batches"] if x["name"] == "C2_64k_x_1k" and x["alg"] == alg
         and "key" not in x][0]
    data = gen_stream(batches["seed"], 65536 * 1024)
    d = oracle.batch_fixed_mt(ALG[alg], data, 65536, 1024, 1024)
    check_entry(e, d)


def test_hashlib_cross_check(oracle):
    """Second, independent oracle for the MD/SHA family (OpenSSL via hashlib)."""
    rng = np.random.RandomState(7)
    names = {1: "md5", 2: "sha1", 3: "sha224", 4: "sha256", 5: "sha384", 6: "sha512"}
    lens = rng.randint(0, 700, size=200).astype(np.uint32)
    offs = np.zeros(200, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = rng.randint(0, 256, size=int(lens.sum())).astype(np.uint8)
    for alg, nm in names.items():
        d = oracle.batch(alg, data, offs, lens)
        for i in range(200):
            m = data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
            assert d[i].tobytes() == hashlib.new(nm, m).digest()


@pytest.mark.skipif(not Ref.available(), reason="oracle/_ref not built (reference absent)")
def test_oracle_vs_reference_random():
    o, r = Oracle(), Ref()
    rng = np.random.RandomState(11)
    lens = rng.randint(0, 3000, size=300).astype(np.uint32)
    offs = np.zeros(300, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = rng.randint(0, 256, size=int(lens.sum())).astype(np.uint8)
    for alg in range(1, 9):
        for key in (None, b"", b"k" * 70, bytes(range(130))):
            assert np.array_equal(o.batch(alg, data, offs, lens, key=key),
                                  r.batch(alg, data, offs, lens, key=key)), (alg, key)
