"""GPU parity of the batched ChaCha / XChaCha (include/lcb_chacha_gpu.h)
through the C-ABI: bit-exact against the reference's own self-test vectors,
the reference-computed fixtures of tests/golden/chacha.json (incl. the 64K x
1 KiB C2 pass) and the oracle (oracle/chacha_oracle.c, pinned by
tests/test_chacha_oracle.py) on misaligned / ragged / gapped / in-place /
keystream-only batches with odd round counts and 64-bit counter carries, in
device and host mode; plus size-independent properties at 1M x 1 KiB."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from oracle.pyoracle import SEED, Oracle, gen_stream
from tests.test_chacha_oracle import batch_inputs, kat_args

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cg():
    return json.load(open(os.path.join(HERE, "golden", "chacha.json")))


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def dev(a, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def run_dev(x, key, ksz, rounds, src, offs, lens, counters=None, ivs=None, count=None, stride=None,
            fixed_len=None, nbytes=None, dst_init=None):
    from liblcb_amd.chacha import chacha_batch, xchacha_batch
    fn = xchacha_batch if x else chacha_batch
    n = src.size if src is not None else nbytes
    dst = dev(dst_init) if dst_init is not None else torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
    out = fn(key, dev(src) if src is not None else None, dst=dst, key_size=ksz, rounds=rounds,
             counters=dev(counters) if counters is not None else None,
             ivs=dev(ivs) if ivs is not None else None,
             offsets=dev(offs.astype(np.int64)) if offs is not None else None,
             lengths=dev(lens.astype(np.int32)) if lens is not None else None,
             count=count, stride=stride, fixed_len=fixed_len)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def test_kat_device_and_host(gpu, cg):
    from liblcb_amd.chacha import chacha_batch
    for v in cg["kat"]:
        key, n, c, iv, src = kat_args(v)
        d = run_dev(False, key, v["key_size"], v["rounds"], src, np.zeros(1, np.uint64), np.array([n], np.uint32),
                    counters=c, ivs=iv, nbytes=n)
        assert d[:n].tobytes().hex() == v["output"], v
        h = chacha_batch(key, src, key_size=v["key_size"], rounds=v["rounds"], counters=c, ivs=iv,
                         offsets=[0], lengths=[n], nbytes=n)
        assert h[:n].tobytes().hex() == v["output"], v


def test_selftest_xchacha(gpu, cg):
    from tests.golden.make_golden_chacha import selftest_plain
    sx = cg["selftest_x"]
    key = bytes.fromhex(sx["key"])
    iv = np.frombuffer(bytes.fromhex(sx["iv"]), np.uint8)
    plain = np.frombuffer(selftest_plain(), np.uint8)
    one = (np.zeros(1, np.uint64), np.array([2048], np.uint32))
    assert run_dev(True, key, 256, 8, plain, *one, ivs=iv).tobytes().hex() == sx["xchacha"]
    assert run_dev(False, key, 256, 8, plain, *one, ivs=iv[:8].copy()).tobytes().hex() == sx["chacha"]


@pytest.mark.parametrize("i", range(13))
def test_golden_batches(gpu, cg, i):
    e = cg["batches"][i]
    src, offs, lens, cnt, stride, flen, counters, ivs = batch_inputs(e)
    key = bytes.fromhex(e["key"])
    kw = dict(counters=counters, ivs=ivs, count=cnt, stride=stride or None, fixed_len=flen or None)
    out = run_dev(e["x"], key, e["key_size"], e["rounds"], src, offs, lens, **kw)
    assert hashlib.sha256(out.tobytes()).hexdigest() == e["out_sha256"], e["name"]
    if "keystream_sha256" in e:
        ks = run_dev(e["x"], key, e["key_size"], e["rounds"], None, offs, lens, nbytes=src.size, **kw)
        assert hashlib.sha256(ks.tobytes()).hexdigest() == e["keystream_sha256"], e["name"]


def gapped_layout(rng, n, hi, total_pad=64):
    """Random lengths (incl. 0 and exact block multiples) at random byte
    offsets with random gaps (so buffers are misaligned and non-adjacent)."""
    lens = rng.integers(0, hi, n).astype(np.uint32)
    lens[::7] = 0
    lens[3::11] = (lens[3::11] // 64) * 64
    gaps = rng.integers(0, 40, n).astype(np.uint64)
    offs = np.zeros(n, np.uint64)
    pos = np.uint64(rng.integers(0, 16))
    for i in range(n):
        pos += gaps[i]
        offs[i] = pos
        pos += np.uint64(lens[i])
    return offs, lens, int(pos) + total_pad


def expected_with_sentinel(full, offs, lens, sentinel):
    exp = sentinel.copy()
    for o, l in zip(offs.tolist(), lens.tolist()):
        exp[o:o + l] = full[o:o + l]
    return exp


@pytest.mark.parametrize("x", [False, True])
@pytest.mark.parametrize("rounds", [20, 8, 12, 7, 0, 1, 33])
def test_misaligned_ragged_vs_oracle(gpu, orc, x, rounds):
    """Gapped, misaligned ragged buffers; bytes outside buffers untouched."""
    rng = np.random.default_rng(100 + rounds + (1000 if x else 0))
    n = 257
    offs, lens, total = gapped_layout(rng, n, 700)
    src = rng.integers(0, 256, total, dtype=np.uint8)
    for ksz in (32, 16):
        key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        counters = rng.integers(0, 256, 8 * n, dtype=np.uint8)
        counters[0:4 * 8:8] = 0xf0  # low word near 2^32: carry into word 13 inside the buffer
        for b in range(1, 4):
            counters[b:4 * 8:8] = 0xff
        ivs = rng.integers(0, 256, (24 if x else 8) * n, dtype=np.uint8)
        full = orc.chacha_batch(key, ksz, rounds, src, offs, lens, counters=counters, ivs=ivs, x=x)
        sentinel = np.full(total, 0xA5, np.uint8)
        exp = expected_with_sentinel(full, offs, lens, sentinel)
        got = run_dev(x, key, ksz, rounds, src, offs, lens, counters=counters, ivs=ivs, dst_init=sentinel)
        assert np.array_equal(got, exp), (x, rounds, ksz)
        ks_full = orc.chacha_batch(key, ksz, rounds, None, offs, lens, counters=counters, ivs=ivs, x=x,
                                   nbytes=total)
        ks = run_dev(x, key, ksz, rounds, None, offs, lens, counters=counters, ivs=ivs, dst_init=sentinel)
        assert np.array_equal(ks, expected_with_sentinel(ks_full, offs, lens, sentinel)), (x, rounds, ksz)


def test_host_mode_vs_oracle(gpu, orc):
    """Host (pageable) memory: staging, packing and scatter back to gapped offsets."""
    from liblcb_amd.chacha import chacha_batch, xchacha_batch
    rng = np.random.default_rng(9)
    n = 3000
    offs, lens, total = gapped_layout(rng, n, 3000)
    src = rng.integers(0, 256, total, dtype=np.uint8)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    for x, fn in ((False, chacha_batch), (True, xchacha_batch)):
        ivs = rng.integers(0, 256, (24 if x else 8) * n, dtype=np.uint8)
        counters = rng.integers(0, 256, 8 * n, dtype=np.uint8)
        full = orc.chacha_batch(key, 32, 20, src, offs, lens, counters=counters, ivs=ivs, x=x)
        sentinel = np.full(total, 0x3C, np.uint8)
        dst = sentinel.copy()
        fn(key, src, dst=dst, rounds=20, counters=counters, ivs=ivs, offsets=offs, lengths=lens)
        assert np.array_equal(dst, expected_with_sentinel(full, offs, lens, sentinel)), x
        # in place
        buf = src.copy()
        fn(key, buf, dst=buf, rounds=20, counters=counters, ivs=ivs, offsets=offs, lengths=lens)
        assert np.array_equal(buf, expected_with_sentinel(full, offs, lens, src)), x
        # fixed stride, dense and strided
        exp = orc.chacha_batch(key, 32, 12, src, count=n // 10, stride=300, fixed_len=300, ivs=ivs, x=x)
        got = fn(key, src, rounds=12, ivs=ivs, count=n // 10, stride=300, fixed_len=300)
        assert np.array_equal(got, exp), x
        exp = orc.chacha_batch(key, 32, 12, src, count=n // 10, stride=301, fixed_len=250, x=x)
        got = fn(key, src, rounds=12, count=n // 10, stride=301, fixed_len=250)
        assert np.array_equal(got[:(n // 10) * 301], exp[:(n // 10) * 301]), x


def test_pointer_alignments(gpu, orc):
    """Device buffers whose base pointers are misaligned, equal and different
    between src and dst (the byte path), fixed and ragged layouts."""
    rng = np.random.default_rng(4)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    n, L = 50, 333
    src = rng.integers(0, 256, n * L + 64, dtype=np.uint8)
    exp = orc.chacha_batch(key, 32, 20, src[:n * L], count=n, stride=L, fixed_len=L)
    from liblcb_amd.chacha import chacha_batch
    for ss in range(0, 5):
        s_full = torch.zeros(n * L + 32, dtype=torch.uint8, device="cuda")
        s_full[ss:ss + n * L] = torch.as_tensor(src[:n * L]).cuda()
        s_t = s_full[ss:ss + n * L]
        for ds in (0, 1, 2, 3, 8):
            d_full = torch.zeros(n * L + 32, dtype=torch.uint8, device="cuda")
            d_t = d_full[ds:ds + n * L]
            chacha_batch(key, s_t, dst=d_t, rounds=20, count=n, stride=L, fixed_len=L)
            torch.cuda.synchronize()
            got = d_full.cpu().numpy()
            assert np.array_equal(got[ds:ds + n * L], exp[:n * L]), (ss, ds)
            assert not got[:ds].any() and not got[ds + n * L:].any(), (ss, ds)


def test_large_buffers_and_empty(gpu, orc):
    rng = np.random.default_rng(8)
    lens = np.array([0, 65536, 1, 0, 65535, 200000, 63, 64, 65], np.uint32)
    offs = np.zeros(len(lens), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    src = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    key = bytes(range(32))
    counters = np.zeros(8 * len(lens), np.uint8)
    counters[8:16] = [0xff] * 4 + [0x01, 0, 0, 0]  # counter 0x1_ffffffff
    for x in (False, True):
        exp = orc.chacha_batch(key, 32, 20, src, offs, lens, counters=counters, x=x)
        got = run_dev(x, key, 32, 20, src, offs, lens, counters=counters)
        assert np.array_equal(got, exp), x
    # all-empty ragged batch and zero fixed_len: nothing written, no error
    z = run_dev(False, key, 32, 20, src[:64], np.zeros(4, np.uint64), np.zeros(4, np.uint32),
                dst_init=np.full(64, 7, np.uint8))
    assert (z == 7).all()
    z = run_dev(False, key, 32, 20, src[:64], None, None, count=4, stride=16, fixed_len=0,
                dst_init=np.full(64, 7, np.uint8))
    assert (z == 7).all()


def test_c3_scale_properties(gpu, orc):
    """BASELINE C3 shape, 1M x 1 KiB generated on the device: decrypt(encrypt)
    is the identity, ciphertext ^ keystream == plaintext, and sampled buffers
    equal the oracle."""
    import liblcb_amd
    from liblcb_amd.chacha import chacha_batch
    n = 1 << 20
    data = liblcb_amd.gen_synthetic(SEED, n * 1024)
    ivs = torch.arange(n, dtype=torch.int64, device="cuda").view(torch.uint8)
    key = bytes(range(32))
    ct = chacha_batch(key, data, rounds=20, ivs=ivs, count=n, stride=1024, fixed_len=1024)
    pt = chacha_batch(key, ct, rounds=20, ivs=ivs, count=n, stride=1024, fixed_len=1024)
    ks = chacha_batch(key, None, dst=torch.empty_like(data), rounds=20, ivs=ivs, count=n, stride=1024,
                      fixed_len=1024)
    torch.cuda.synchronize()
    assert torch.equal(pt, data)
    assert torch.equal(ct ^ ks, data)
    host = data.cpu().numpy()
    ivh = ivs.cpu().numpy()
    sample = [0, 1, 4095, 65536, 777777, n - 1]
    ct_h = ct.cpu().numpy()
    for i in sample:
        e = orc.chacha_batch(key, 32, 20, host[i * 1024:(i + 1) * 1024], [0], [1024], ivs=ivh[8 * i:8 * i + 8])
        assert np.array_equal(ct_h[i * 1024:(i + 1) * 1024], e), i
