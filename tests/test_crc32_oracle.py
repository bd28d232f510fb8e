"""CRC-32 oracle pinned against the reference (include/math/crc32.h):
KATs extracted from crc32_self_test and the catalogue check values, batch
fixtures computed by the compiled reference, the byte tables, and zlib for the
ISO-HDLC variant."""
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

from oracle.pyoracle import CRC_VARIANTS, Oracle, Ref, gen_stream

HERE = os.path.dirname(os.path.abspath(__file__))
VID = {v: k for k, v in CRC_VARIANTS.items()}


@pytest.fixture(scope="module")
def crc_golden():
    return json.load(open(os.path.join(HERE, "golden", "crc32.json")))


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def batch_layout(e):
    if e["name"].startswith("ragged") or e["name"].startswith("update"):
        hi = 1101 if e["name"].startswith("ragged") else 300
        lens = np.arange(0, hi, dtype=np.uint32)
        offs = np.zeros(len(lens), np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    elif e["name"].startswith("misaligned"):
        n = 512
        lens = np.array([1 + (i * 37) % 1500 for i in range(n)], np.uint32)
        offs = np.array([4099 * i + (i % 16) for i in range(n)], np.uint64)
    else:
        lens = np.full(e["count"], 1024, np.uint32)
        offs = np.arange(e["count"], dtype=np.uint64) * 1024
    init = None
    if e["name"].startswith("update"):
        init = (np.arange(len(lens), dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32)
    total = int((offs + lens).max())
    return gen_stream(e["seed"], total), offs, lens, init


def check_crcs(crc, want):
    packed = crc.astype("<u4").tobytes()
    if want.startswith("sha256:"):
        return hashlib.sha256(packed).hexdigest() == want[7:]
    return packed.hex() == want


def test_kat(orc, crc_golden):
    assert len(crc_golden["kat"]) == 23
    for c in crc_golden["kat"]:
        m = np.frombuffer(bytes.fromhex(c["msg"]), np.uint8)
        got = orc.crc32_batch(VID[c["variant"]], m, np.zeros(1, np.uint64), np.array([m.size], np.uint32))
        assert "%08x" % got[0] == c["crc"], c


def test_partial_updates(orc, crc_golden):
    """crc32_self_test's second half: byte-at-a-time X_update chains
    (crc32.h:636-653) give the one-shot value."""
    for c in crc_golden["kat"]:
        v = VID[c["variant"]]
        m = bytes.fromhex(c["msg"])
        a = np.frombuffer(m, np.uint8)
        crc = orc.crc32_batch(v, a[:1], np.zeros(1, np.uint64), np.array([1], np.uint32))[0]
        for j in range(1, len(m)):
            crc = orc.crc32_batch(v, a[j:j + 1], np.zeros(1, np.uint64), np.array([1], np.uint32),
                                  init=np.array([crc], np.uint32))[0]
        assert "%08x" % crc == c["crc"], c


@pytest.mark.parametrize("name", ["ragged_0_1100", "misaligned_512", "update_0_299", "C2_64k_x_1k"])
def test_batches(orc, crc_golden, name):
    e = next(b for b in crc_golden["batches"] if b["name"] == name)
    data, offs, lens, init = batch_layout(e)
    for vn, want in e["crcs"].items():
        crc = orc.crc32_batch(VID[vn], data, offs, lens, init=init)
        assert check_crcs(crc, want), (name, vn)


def test_tables_match_reference(orc):
    if not Ref.available():
        pytest.skip("oracle/_ref not built")
    ref = Ref()
    for v in CRC_VARIANTS:
        assert np.array_equal(orc.crc32_table(v), ref.crc32_table(v)), v


def test_iso_hdlc_is_zlib(orc):
    d = gen_stream(7, 5000)
    lens = np.arange(0, 100, dtype=np.uint32) * 47 % 5000
    offs = np.zeros(len(lens), np.uint64)
    got = orc.crc32_batch(VID["crc32b"], d, offs, lens)
    assert [int(x) for x in got] == [zlib.crc32(d[:n].tobytes()) for n in lens]


def test_random_vs_reference(orc):
    if not Ref.available():
        pytest.skip("oracle/_ref not built")
    ref = Ref()
    rng = np.random.default_rng(3)
    d = rng.integers(0, 256, 300000, dtype=np.uint8)
    lens = rng.integers(0, 3000, 400).astype(np.uint32)
    offs = rng.integers(0, 300000 - 3000, 400).astype(np.uint64)
    init = rng.integers(0, 1 << 32, 400, dtype=np.uint64).astype(np.uint32)
    for v in CRC_VARIANTS:
        assert np.array_equal(orc.crc32_batch(v, d, offs, lens), ref.crc32_batch(v, d, offs, lens))
        assert np.array_equal(orc.crc32_batch(v, d, offs, lens, init=init),
                              ref.crc32_batch(v, d, offs, lens, init=init))
