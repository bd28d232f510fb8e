"""ChaCha oracle (oracle/chacha_oracle.c) pinned against the reference
(include/crypto/cipher/chacha.h): its self-test vectors, the self test's
xchacha/chacha one-shot outputs, reference-computed batch fixtures, and a
random comparison with the compiled reference."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle.pyoracle import Oracle, Ref, gen_stream

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def cg():
    return json.load(open(os.path.join(HERE, "golden", "chacha.json")))


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def kat_args(v):
    n = len(v["output"]) // 2
    c = np.frombuffer(bytes.fromhex(v["counter"]), np.uint8) if v["counter"] else None
    iv = np.frombuffer(bytes.fromhex(v["iv"]), np.uint8) if v["iv"] else None
    src = np.frombuffer(bytes.fromhex(v["plain"]), np.uint8) if v["plain"] else None
    return bytes.fromhex(v["key"]), n, c, iv, src


def batch_inputs(e):
    """Inputs of a chacha.json batch entry (see make_golden_chacha.py)."""
    if e["name"].startswith("C2"):
        cnt = e["count"]
        src = gen_stream(e["seed"], cnt * 1024)
        ivs = np.arange(cnt, dtype="<u8").view(np.uint8)
        return src, None, None, cnt, 1024, 1024, None, ivs
    rng = np.random.default_rng(11)
    lens = rng.integers(0, 1200, 300).astype(np.uint32)
    offs = np.zeros(300, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    src = gen_stream(e["seed"], int((offs + lens).max()))
    counters = np.frombuffer(bytes.fromhex(e["counters"]), np.uint8)
    ivs = np.frombuffer(bytes.fromhex(e["ivs"]), np.uint8)
    return src, offs, lens, None, 0, 0, counters, ivs


def test_kat(orc, cg):
    assert len(cg["kat"]) == 22
    for v in cg["kat"]:
        key, n, c, iv, src = kat_args(v)
        out = orc.chacha_batch(key, v["key_size"], v["rounds"], src, offsets=[0], lengths=[n], counters=c,
                               ivs=iv, nbytes=n)
        assert out[:n].tobytes().hex() == v["output"], v


def test_selftest_xchacha(orc, cg):
    from tests.golden.make_golden_chacha import selftest_plain
    sx = cg["selftest_x"]
    key = bytes.fromhex(sx["key"])
    iv = np.frombuffer(bytes.fromhex(sx["iv"]), np.uint8)
    plain = np.frombuffer(selftest_plain(), np.uint8)
    x = orc.chacha_batch(key, 256, 8, plain, [0], [2048], ivs=iv, x=True)
    assert x.tobytes().hex() == sx["xchacha"]
    c = orc.chacha_batch(key, 256, 8, plain, [0], [2048], ivs=iv[:8])
    assert c.tobytes().hex() == sx["chacha"]


@pytest.mark.parametrize("i", range(13))
def test_batches(orc, cg, i):
    e = cg["batches"][i]
    src, offs, lens, cnt, stride, flen, counters, ivs = batch_inputs(e)
    key = bytes.fromhex(e["key"])
    out = orc.chacha_batch(key, e["key_size"], e["rounds"], src, offs, lens, count=cnt, stride=stride,
                           fixed_len=flen, counters=counters, ivs=ivs, x=e["x"])
    assert hashlib.sha256(out.tobytes()).hexdigest() == e["out_sha256"], e["name"]
    if "keystream_sha256" in e:
        ks = orc.chacha_batch(key, e["key_size"], e["rounds"], None, offs, lens, counters=counters, ivs=ivs,
                              x=e["x"], nbytes=src.size)
        assert hashlib.sha256(ks.tobytes()).hexdigest() == e["keystream_sha256"], e["name"]


def test_random_vs_reference(orc):
    if not Ref.available():
        pytest.skip("oracle/_ref not built")
    ref = Ref()
    assert ref.chacha_self_test() == 0
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, 200000, dtype=np.uint8)
    lens = rng.integers(0, 2500, 150).astype(np.uint32)
    offs = rng.integers(0, 200000 - 2500, 150).astype(np.uint64)
    offs.sort()
    keep = np.concatenate([[True], offs[1:] >= offs[:-1] + lens[:-1]])  # non-overlapping outputs
    offs, lens = offs[keep], lens[keep]
    for x in (False, True):
        for ksz in (32, 256, 16, 7):
            key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
            cnt = rng.integers(0, 256, 8 * len(lens), dtype=np.uint8)
            ivs = rng.integers(0, 256, (24 if x else 8) * len(lens), dtype=np.uint8)
            for rounds in (8, 20):
                a = orc.chacha_batch(key, ksz, rounds, src, offs, lens, counters=cnt, ivs=ivs, x=x)
                b = ref.chacha_batch(key, ksz, rounds, src, offs, lens, counters=cnt, ivs=ivs, x=x)
                assert np.array_equal(a, b), (x, ksz, rounds)
