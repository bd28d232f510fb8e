"""Parity of the MI355X kernels (through the C-ABI) with the reference.

Checkers: the reference's KAT tables (kat.json), digests the compiled
reference produced (batches.json), and the oracle restatement (full digest
arrays, same seeded inputs).  Bar: bit-exact.  Every test runs through
liblcb_hash_gpu.so; nothing here computes a digest on the CPU except the
oracle it compares against.
"""
import errno

import numpy as np
import pytest
import torch

from oracle.pyoracle import gen_stream
from tests.golden_util import check_entry, dod, layout

pytestmark = pytest.mark.gpu

ALG = {"md5": 1, "sha1": 2, "sha224": 3, "sha256": 4, "sha384": 5, "sha512": 6,
       "gost256": 7, "gost512": 8}


def dev(x, dtype=None):
    return torch.as_tensor(np.ascontiguousarray(x), device="cuda") if dtype is None else \
        torch.as_tensor(np.ascontiguousarray(x).astype(dtype), device="cuda")


def run_entry(gpu, e, mode="device"):
    L = layout(e)
    alg = ALG[e["alg"]]
    if mode == "device":
        data = gpu.gen_synthetic(L["seed"], L["nbytes"])
        offs = dev(L["offsets"], np.int64) if L["offsets"] is not None else None
        lens = dev(L["lengths"], np.int32) if L["lengths"] is not None else None
        d = gpu.hash_batch(alg, data, offsets=offs, lengths=lens, count=L["count"],
                           stride=L["stride"], fixed_len=L["fixed_len"], key=L["key"])
        torch.cuda.synchronize()
        return d.cpu().numpy()
    data = gen_stream(L["seed"], L["nbytes"])
    return gpu.hash_batch(alg, data, offsets=L["offsets"], lengths=L["lengths"], count=L["count"],
                          stride=L["stride"], fixed_len=L["fixed_len"], key=L["key"])


def test_device_generator_matches_host(gpu):
    for start, n in ((0, 4096), (3, 1000), (8, 77), (12345, 1 << 16)):
        d = gpu.gen_synthetic(0x1234, n, start=start).cpu().numpy()
        assert np.array_equal(d, gen_stream(0x1234, n, start)), (start, n)


@pytest.mark.parametrize("mode", ["device", "host"])
def test_kat(gpu, kat, mode):
    """Every vector of the reference self tests (tests/hash/main.c path)."""
    for c in kat:
        alg = ALG[c["alg"]]
        msg = bytes.fromhex(c["msg"]) * c.get("repeat", 1)
        key = bytes.fromhex(c["key"]) if "key" in c else None
        arr = np.frombuffer(msg, np.uint8) if msg else np.zeros(1, np.uint8)
        if mode == "device":
            d = gpu.hash_batch(alg, dev(arr), count=1, fixed_len=len(msg), key=key).cpu().numpy()
        else:
            d = gpu.hash_batch(alg, arr, count=1, fixed_len=len(msg), key=key)
        assert d[0].tobytes().hex() == c["digest"], (c["alg"], len(msg), "key" in c)


def test_kat_as_one_ragged_batch(gpu, kat):
    """All KAT messages of one algorithm in ONE ragged batch (mixed lanes)."""
    for name, alg in ALG.items():
        cases = [c for c in kat if c["alg"] == name and "key" not in c]
        msgs = [bytes.fromhex(c["msg"]) * c.get("repeat", 1) for c in cases]
        lens = np.array([len(m) for m in msgs], np.uint32)
        offs = np.zeros(len(msgs), np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        blob = np.frombuffer(b"".join(msgs) or b"\0", np.uint8)
        d = gpu.hash_batch(alg, dev(blob), offsets=dev(offs, np.int64), lengths=dev(lens, np.int32))
        d = d.cpu().numpy()
        for i, c in enumerate(cases):
            assert d[i].tobytes().hex() == c["digest"], (name, i)


SMALL = ("ragged_0_4159", "misaligned_2048", "big_65536", "big_65537", "mixed_512",
         "mixed_16384", "fixed1k_1024", "C2_64k_x_1k")


def test_golden_batches_device(gpu, batches):
    n = 0
    for e in batches["batches"]:
        if e["name"] in SMALL:
            check_entry(e, run_entry(gpu, e))
            n += 1
    assert n >= 120


def test_golden_batches_host(gpu, batches):
    for e in batches["batches"]:
        if e["name"] in ("ragged_0_4159", "misaligned_2048", "big_65537", "mixed_16384") and "key" not in e:
            check_entry(e, run_entry(gpu, e, mode="host"))


@pytest.mark.parametrize("alg", list(ALG))
def test_c3_full_size(gpu, batches, alg):
    """BASELINE config C3 (1M x 1 KiB, the bench workload): digest-of-digests
    from the compiled reference."""
    e = [x for x in batches["batches"] if x["name"] == "C3_1M_x_1k" and x["alg"] == alg][0]
    check_entry(e, run_entry(gpu, e))


def test_full_digests_vs_oracle(gpu, oracle):
    """Full digest arrays (not hashes of them) against the oracle on a ragged,
    misaligned batch with HMAC keys around the block boundary."""
    rng = np.random.RandomState(3)
    lens = rng.randint(0, 600, size=700).astype(np.uint32)
    gaps = rng.randint(0, 9, size=700)
    offs = np.zeros(700, np.uint64)
    pos = 5
    for i in range(700):
        offs[i] = pos
        pos += int(lens[i]) + int(gaps[i])
    data = gen_stream(99, pos)
    ddata = dev(data)
    for alg in range(1, 9):
        for key in (None, b"", b"secret", bytes(range(64)), bytes(range(65)), bytes(range(128)),
                    bytes(range(129)), bytes(300)):
            exp = oracle.batch(alg, data, offs, lens, key=key)
            got = gpu.hash_batch(alg, ddata, offsets=dev(offs, np.int64), lengths=dev(lens, np.int32),
                                 key=key).cpu().numpy()
            assert np.array_equal(got, exp), (alg, None if key is None else len(key))


def test_every_alignment_and_tail_length(gpu, oracle):
    """Start offsets 0..15 x lengths 0..200: every tail/padding branch and every
    load path (16-B aligned, 4-B aligned, byte-misaligned)."""
    lens, offs = [], []
    pos = 0
    for a in range(16):
        for n in range(0, 201):
            pos = (pos + 15) // 16 * 16 + a
            offs.append(pos)
            lens.append(n)
            pos += n
    lens = np.array(lens, np.uint32)
    offs = np.array(offs, np.uint64)
    data = gen_stream(5, pos + 16)
    for alg in range(1, 9):
        exp = oracle.batch(alg, data, offs, lens)
        got = gpu.hash_batch(alg, dev(data), offsets=dev(offs, np.int64), lengths=dev(lens, np.int32))
        assert np.array_equal(got.cpu().numpy(), exp), alg


@pytest.mark.parametrize("stride_pad", [0, 16, 3])
def test_fixed_whole_block_lengths(gpu, oracle, stride_pad):
    """Fixed-length batches whose length is a whole number of blocks end in a
    pad-only block built from the wave-uniform length (md_pad_only: scalar
    schedule).  Lengths 0..4096 in 64-B steps x plain/HMAC; stride padding 0
    and 16 take the LDS line-stream kernel where eligible, 3 the generic one;
    300 records so the last wave is partial."""
    n = 300
    for L in (0, 64, 128, 192, 256, 320, 448, 512, 1024, 1088, 2048, 4096):
        stride = L + stride_pad
        data = gen_stream(1000 + L, max(1, n * stride))
        for alg in range(1, 9):
            for key in (None, b"k" * 20, bytes(range(200))):
                exp = oracle.batch(alg, data, count=n, stride=stride, fixed_len=L, key=key)
                got = gpu.hash_batch(alg, dev(data), count=n, stride=stride, fixed_len=L, key=key)
                assert np.array_equal(got.cpu().numpy(), exp), (alg, L, stride, key is not None)


@pytest.mark.parametrize("count", [63, 64, 65, 127, 1000, 4096 + 7])
def test_fixed_stride_partial_last_wave(gpu, oracle, count):
    """Fixed-stride LDS-stream kernels cover whole 64-record waves: a partial
    last wave moves back over its predecessor's records and stores only its
    own (63 records: the per-lane kernel).  Lengths of whole lines and with a
    ragged tail, every MD algorithm plus CRC-32 and HMAC-MD5."""
    from liblcb_amd.crc32 import crc32_batch
    for stride, flen in ((1024, 1024), (1040, 1000), (256, 130)):
        data = gen_stream(count * 7 + flen, count * stride)
        dd = dev(data)
        for alg in range(1, 9):
            for key in ((None, b"k") if alg == 1 else (None,)):
                exp = oracle.batch(alg, data, count=count, stride=stride, fixed_len=flen, key=key)
                got = gpu.hash_batch(alg, dd, count=count, stride=stride, fixed_len=flen, key=key).cpu().numpy()
                assert np.array_equal(got, exp), (alg, count, stride, flen, key)
        exp = oracle.crc32_batch(3, data, count=count, stride=stride, fixed_len=flen)
        got = crc32_batch(3, dd, count=count, stride=stride, fixed_len=flen).cpu().numpy().view(np.uint32)
        assert np.array_equal(got, np.asarray(exp).view(np.uint32)), ("crc", count, stride, flen)


@pytest.mark.parametrize("layout", ["aligned64", "aligned16", "packed"])
def test_sha512_ragged_line_stream(gpu, oracle, layout):
    """Bucketed ragged SHA-384/512 batches (count >= 16,384) take
    md_lines_kernel: waves whose records all start 16-B aligned stream their
    common whole lines through LDS, then finish per lane; other waves (packed:
    most) take the per-lane loop from line 0.  Lengths 0..3000, runs of equal
    lengths (C4-like), some 64 KiB records, a partial last wave; plain and
    HMAC vs the oracle."""
    rng = np.random.default_rng(7 + len(layout))
    n = 20000 + 37
    lens = rng.integers(0, 3001, n).astype(np.uint32)
    lens[: n // 4] = 1024
    lens[rng.integers(0, n, 60)] = 65536
    lens[rng.integers(0, n, 60)] = 128 * rng.integers(1, 9, 60)
    align = {"aligned64": 64, "aligned16": 16, "packed": 1}[layout]
    offs = np.zeros(n, np.uint64)
    pos = 0
    for k in range(n):
        pos = (pos + align - 1) // align * align
        offs[k] = pos
        pos += int(lens[k]) + (int(rng.integers(0, 3)) if layout == "packed" else 0)
    data = gen_stream(123 + align, pos + 16)
    dd, dl, do = dev(data), dev(lens, np.int32), dev(offs, np.int64)
    for alg in (5, 6):
        for key in (None, b"radius-secret"):
            exp = oracle.batch(alg, data, offs, lens, key=key)
            got = gpu.hash_batch(alg, dd, offsets=do, lengths=dl, key=key).cpu().numpy()
            assert np.array_equal(got, exp), (layout, alg, key)


@pytest.mark.parametrize("count", [4 * 256 * 256 + 1, 4 * 256 * 256 + 64 * 8 * 3 + 37, 300000])
def test_fixed_stride_resident_grid(gpu, oracle, count):
    """MD5 batches larger than one resident grid (4 workgroups x 256 CUs x
    256 records) take md_fixed_persist_kernel: every wave hashes several
    64-record chunks of its XCD's eighth, the partial last chunk moved back.
    Uneven chunk counts per XCD and per wave, both line-stream policies
    (128-B aligned stride: nt; 16-B: default), whole-line and ragged tails,
    plain and HMAC, all digests vs the oracle."""
    for stride, flen in ((256, 256), (208, 200)):
        data = gen_stream(count + flen, count * stride)
        dd = dev(data)
        for key in (None, b"radius-secret"):
            exp = oracle.batch(1, data, count=count, stride=stride, fixed_len=flen, key=key)
            got = gpu.hash_batch(1, dd, count=count, stride=stride, fixed_len=flen, key=key).cpu().numpy()
            assert np.array_equal(got, exp), (count, stride, flen, key)


def test_bit_length_high_word(gpu, oracle):
    """A message of 512 MiB + 67 B: its bit length no longer fits 32 bits, so
    the high word of MD5's LE length field (md5.h:282) and of SHA-512's
    128-bit BE one (sha2.h:725-731) are exercised; the message starts
    unaligned.  One lane walks 8M blocks (latency-bound, ~25 s per
    algorithm), so this is the slowest GPU test."""
    n = (1 << 29) + 67
    data = gpu.gen_synthetic(0x4242, n + 5)
    host = data.cpu().numpy()
    offs, lens = np.array([5], np.uint64), np.array([n], np.uint32)
    do, dl = dev(offs, np.int64), dev(lens, np.int32)
    for alg in (1, 6):
        exp = oracle.batch(alg, host, offs, lens)
        got = gpu.hash_batch(alg, data, offsets=do, lengths=dl).cpu().numpy()
        assert np.array_equal(got, exp), alg
    del data
    torch.cuda.empty_cache()


def test_unaligned_digest_output(gpu, oracle):
    data = gen_stream(1, 64 * 100)
    for alg in (1, 2, 6, 7):
        D = gpu.DIGEST_SIZE[alg]
        out = torch.zeros(100 * D + 3, dtype=torch.uint8, device="cuda")
        view = out[3:]
        gpu.lib().lcb_hash_batch(alg, None, 0, dev(data).data_ptr(), None, None, 100, 64, 64,
                                 view.data_ptr(), 1, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        exp = oracle.batch(alg, data, count=100, stride=64, fixed_len=64)
        assert np.array_equal(view.cpu().numpy().reshape(100, D), exp)
        assert out[:3].sum().item() == 0


def test_reference_named_entry_points(gpu, oracle):
    data = gen_stream(2, 1024 * 300)
    d = dev(data)
    kw = dict(count=300, stride=1024, fixed_len=1000)
    for fn, alg in ((gpu.md5_get_digest_batch, 1), (gpu.sha1_get_digest_batch, 2)):
        assert np.array_equal(fn(d, **kw).cpu().numpy(), oracle.batch(alg, data, **kw))
    for bits, alg in ((224, 3), (28, 3), (256, 4), (32, 4), (384, 5), (48, 5), (512, 6), (64, 6)):
        assert np.array_equal(gpu.sha2_get_digest_batch(bits, d, **kw).cpu().numpy(),
                              oracle.batch(alg, data, **kw))
        assert np.array_equal(gpu.sha2_hmac_get_digest_batch(bits, b"k", d, **kw).cpu().numpy(),
                              oracle.batch(alg, data, key=b"k", **kw))
    for bits, alg in ((256, 7), (32, 7), (512, 8), (64, 8), (1, 8), (0, 8)):
        assert np.array_equal(gpu.gost3411_2012_get_digest_batch(bits, d, **kw).cpu().numpy(),
                              oracle.batch(alg, data, **kw))
    assert np.array_equal(gpu.md5_hmac_get_digest_batch(b"radius-secret", d, **kw).cpu().numpy(),
                          oracle.batch(1, data, key=b"radius-secret", **kw))
    assert np.array_equal(gpu.sha1_hmac_get_digest_batch(b"", d, **kw).cpu().numpy(),
                          oracle.batch(2, data, key=b"", **kw))
    assert np.array_equal(gpu.gost3411_2012_hmac_get_digest_batch(256, b"x" * 70, d, **kw).cpu().numpy(),
                          oracle.batch(7, data, key=b"x" * 70, **kw))
    with pytest.raises(gpu.LcbHashError) as ei:
        gpu.sha2_get_digest_batch(100, d, **kw)
    assert ei.value.errno == errno.EINVAL


def test_empty_and_zero_count(gpu, oracle):
    d = dev(np.zeros(16, np.uint8))
    for alg in range(1, 9):
        got = gpu.hash_batch(alg, d, count=5, stride=0, fixed_len=0).cpu().numpy()
        exp = oracle.batch(alg, np.zeros(1, np.uint8), count=5, stride=0, fixed_len=0)
        assert np.array_equal(got, exp)
        assert gpu.hash_batch(alg, d, count=0, fixed_len=4).shape == (0, gpu.DIGEST_SIZE[alg])


def test_properties_full_size(gpu):
    """Size-independent properties at the bench size (1M x 1 KiB): identical
    messages give identical digests; a one-byte change flips exactly that
    message's digest; the host pipeline equals the device path."""
    n = 1 << 20
    data = gpu.gen_synthetic(7, n * 1024)
    base = gpu.hash_batch(1, data, count=n, stride=1024, fixed_len=1024)
    data[1024 * 12345 + 17] ^= 1
    flip = gpu.hash_batch(1, data, count=n, stride=1024, fixed_len=1024)
    diff = (base != flip).any(dim=1).nonzero().flatten().tolist()
    assert diff == [12345]
    same = torch.zeros(1024 * 64, dtype=torch.uint8, device="cuda")
    z = gpu.hash_batch(4, same, count=64, stride=1024, fixed_len=1024)
    assert (z == z[0]).all()
    host = gpu.hash_batch(1, data[:1 << 26].cpu().numpy(), count=1 << 16, stride=1024, fixed_len=1024)
    assert np.array_equal(host, flip[:1 << 16].cpu().numpy())


def test_bucketed_equals_unbucketed(gpu, oracle):
    """A ragged batch above the bucketing threshold (length-sorted lanes) gives
    the same digests, in input order, as the same messages hashed in small
    (unbucketed) batches."""
    from tests.golden_util import mixed_lengths
    n = 12000
    lens = np.array(mixed_lengths(17, n), np.uint32) // np.array([1, 3, 7], np.uint32)[np.arange(n) % 3]
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = gpu.gen_synthetic(17, int(lens.sum()))
    dl, do = dev(lens, np.int32), dev(offs, np.int64)
    for alg in (1, 4, 7):
        whole = gpu.hash_batch(alg, data, offsets=do, lengths=dl).cpu().numpy()
        parts = [gpu.hash_batch(alg, data, offsets=do[i:i + 1000], lengths=dl[i:i + 1000]).cpu().numpy()
                 for i in range(0, n, 1000)]
        assert np.array_equal(whole, np.concatenate(parts)), alg


@pytest.mark.parametrize("layout", ["aligned16", "packed", "mostly_aligned"])
def test_ragged_line_stream(gpu, oracle, layout):
    """Bucketed ragged batches (count above the bucketing threshold) take the
    tile kernel (md_tiles_kernel): tiles whose records all start
    16-B aligned with equal line counts stream their lines through LDS, the
    others load per lane.  Lengths 0..3000 plus a few 64 KiB records, so waves
    mix records with and without whole lines; plain and HMAC."""
    rng = np.random.default_rng(len(layout))
    n = 6000
    lens = rng.integers(0, 3001, n).astype(np.uint32)
    lens[rng.integers(0, n, 40)] = 65536
    lens[rng.integers(0, n, 40)] = 128 * rng.integers(1, 9, 40)
    offs = np.zeros(n, np.uint64)
    pos = 0
    for k in range(n):
        if layout == "aligned16" or (layout == "mostly_aligned" and k % 997 != 5):
            pos = (pos + 15) // 16 * 16
        offs[k] = pos
        pos += int(lens[k]) + int(rng.integers(0, 3))
    data = gen_stream(99, pos + 16)
    dd, dl, do = dev(data), dev(lens, np.int32), dev(offs, np.int64)
    for alg in range(1, 7):
        for key in (None, b"radius-secret"):
            exp = oracle.batch(alg, data, offs, lens, key=key)
            got = gpu.hash_batch(alg, dd, offsets=do, lengths=dl, key=key).cpu().numpy()
            assert np.array_equal(got, exp), (alg, layout, key is not None)


@pytest.mark.parametrize("mix", ["halves", "all64", "any16"])
def test_ragged_half_line_phase(gpu, oracle, mix):
    """Bucketed ragged batches whose records start 0 or 64 B into a 128-B line
    (packed 64-B multiples, as C4): the bucketing groups each length class by
    that half-line phase and the tile kernel streams a 64-B-phase tile as the
    whole cache lines its records overlap (first and last line half
    discarded).  Lengths of whole lines, whole lines + 64 and ragged tails;
    the last record ends at the end of the buffer; other 16-B phases ("any16")
    keep the record-relative stream.  MD5 plain and HMAC (the tile kernel's
    algorithm) plus SHA-256 and GOST through the same bucketing."""
    rng = np.random.default_rng({"halves": 1, "all64": 2, "any16": 3}[mix])
    n = 6000
    lines = rng.integers(1, 40, n)
    tail = rng.choice([0, 64, 0, 17, 100], n)
    lens = (128 * lines + tail).astype(np.uint32)
    lens[rng.integers(0, n, 30)] = 65536
    lens[-1] = 128 * 7
    offs = np.zeros(n, np.uint64)
    pos = 64 if mix == "all64" else 0
    for k in range(n):
        if mix == "all64":
            pos = (pos + 63) // 128 * 128 + 64
        elif mix == "halves":
            pos = (pos + 63) // 64 * 64
        else:
            pos = (pos + 15) // 16 * 16
        offs[k] = pos
        pos += int(lens[k])
    data = gen_stream(5, pos)
    dd, dl, do = dev(data), dev(lens, np.int32), dev(offs, np.int64)
    for alg, key in ((1, None), (1, b"radius-secret"), (4, None), (7, None)):
        exp = oracle.batch(alg, data, offs, lens, key=key)
        got = gpu.hash_batch(alg, dd, offsets=do, lengths=dl, key=key).cpu().numpy()
        assert np.array_equal(got, exp), (alg, mix, key is not None)


def test_host_mode_pinned_direct_dma(gpu, batches):
    """Host mode from page-locked input (direct DMA, rebased offsets for ragged
    chunks) and from pageable input (parallel gather), multi-chunk sizes."""
    for e in batches["batches"]:
        if e["name"] not in ("ragged_0_4159", "mixed_16384", "C2_64k_x_1k", "misaligned_2048"):
            continue
        if "key" in e and e["name"] != "mixed_16384":
            continue
        L = layout(e)
        host = gen_stream(L["seed"], L["nbytes"])
        pinned = torch.empty(max(len(host), 1), dtype=torch.uint8).pin_memory()
        pinned.numpy()[:len(host)] = host
        d = gpu.hash_batch(ALG[e["alg"]], pinned.numpy(), offsets=L["offsets"], lengths=L["lengths"],
                           count=L["count"], stride=L["stride"], fixed_len=L["fixed_len"], key=L["key"])
        check_entry(e, d)


@pytest.fixture(scope="module")
def large():
    import json
    import os
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", "large.json")))


def test_c5_full_size_one_gpu(gpu, large):
    """BASELINE config C5 (8M x 1 KiB = 8 GiB) on ONE MI355X, every
    algorithm: the whole digest array and each of the 8 per-GPU shards of
    the weak-scaling bench against the reference's digest-of-digests
    (tests/golden/large.json)."""
    import hashlib
    fx = large["C5_8M_x_1k"]
    n, sh = fx["count"], fx["shard"]
    data = gpu.gen_synthetic(large["seed"], n * 1024)
    for name, alg in ALG.items():
        d = gpu.hash_batch(alg, data, count=n, stride=1024, fixed_len=1024).cpu().numpy()
        assert dod(d) == fx["algs"][name]["dod"], name
        shards = [hashlib.sha256(d[k * sh:(k + 1) * sh].tobytes()).hexdigest() for k in range(n // sh)]
        assert shards == fx["algs"][name]["shard_dod"], name
    del data
    torch.cuda.empty_cache()


def test_c4_full_size(gpu, large):
    """BASELINE config C4 (1M buffers of {64 B, 1 KiB, 64 KiB}, 21.7 GiB
    packed, the bench's ragged_c4 workload), every algorithm, against the
    reference's digest-of-digests."""
    from tests.golden_util import mixed_lengths_np
    fx = large["C4_1M_mixed"]
    lens = mixed_lengths_np(large["seed"], fx["count"])
    offs = np.zeros(lens.size, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    assert int(lens.sum()) == fx["total_bytes"]
    data = gpu.gen_synthetic(large["seed"], fx["total_bytes"])
    dl, do = dev(lens, np.int32), dev(offs, np.int64)
    for name, alg in ALG.items():
        d = gpu.hash_batch(alg, data, offsets=do, lengths=dl).cpu().numpy()
        assert dod(d) == fx["algs"][name]["dod"], name
    del data
    torch.cuda.empty_cache()


@pytest.mark.parametrize("alg", [1, 2, 3, 4], ids=["md5", "sha1", "sha224", "sha256"])
@pytest.mark.parametrize("shape", ["short", "lines"])
def test_ragged_every_line_phase(gpu, oracle, shape, alg):
    """The tile kernel's whole-cache-line stream (md_tiles.hpp): records start
    at every one of the 128 byte offsets inside a 128-B line (off = 64 h + 16 m
    + 4 R + sh: the tile's dword phase R from the bucketing, the lane's chunk
    rotation m applied by the DMA addresses and merged into the carry, its
    half-line h offsetting its block numbering, its byte shift sh), so every
    tile of a key mixes all (h, m, sh).  Lengths 1..700 ("short": records of
    1-6 lines, tails of every size) or whole lines +- a few bytes ("lines"),
    a few 4 KiB records, the last record ending at the buffer's end.  Every
    hash with a tile kernel (MD5, SHA-1, SHA-224/256): plain, HMAC, keyed HMAC
    and keyed suffix (the tile kernel's modes) digest by digest against the
    oracle."""
    rng = np.random.default_rng({"short": 11, "lines": 12}[shape])
    n = 8192
    if shape == "short":
        lens = rng.integers(1, 701, n)
    else:
        lens = 128 * rng.integers(1, 12, n) + rng.integers(-3, 4, n)
    lens[rng.integers(0, n, 50)] = 4096
    lens = lens.astype(np.uint32)
    phase = rng.permutation(np.arange(n) % 128)
    offs = np.zeros(n, np.uint64)
    pos = 0
    for k in range(n):
        pos = pos + (int(phase[k]) - pos) % 128
        offs[k] = pos
        pos += int(lens[k])
    data = gen_stream(17, pos)
    dd, dl, do = dev(data), dev(lens, np.int32), dev(offs, np.int64)
    exp = oracle.batch(alg, data, offs, lens)
    assert np.array_equal(gpu.hash_batch(alg, dd, offsets=do, lengths=dl).cpu().numpy(), exp), shape
    exp = oracle.batch(alg, data, offs, lens, key=b"radius-secret")
    got = gpu.hash_batch(alg, dd, offsets=do, lengths=dl, key=b"radius-secret").cpu().numpy()
    assert np.array_equal(got, exp), shape
    keys = [bytes(range(7 + 13 * k)) for k in range(5)]
    kidx = rng.integers(0, len(keys), n).astype(np.uint32)
    for mode in (1, 3):   # LCB_HASH_KEY_HMAC, LCB_HASH_KEY_SUFFIX
        exp = oracle.batch_keyed(alg, mode, keys, data, kidx, offs, lens)
        got = gpu.hash_batch_keyed(alg, mode, keys, dd, key_index=dev(kidx, np.int32), offsets=do,
                                   lengths=dl).cpu().numpy()
        assert np.array_equal(got, exp), (shape, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 3])
def test_tiles_pad_heavy(gpu, oracle, mode):
    """Regression for the round-4 fault (a readfirstlane under
    a per-lane select read a pad entry): tiles whose lanes 1..63 are pads
    (a key with ONE record), and a key run of 64k + 1 records (its last
    tile: 1 record + 63 pads), in plain, keyed-HMAC and keyed-suffix form,
    vs the oracle."""
    import torch
    from tests.test_radius_gpu import KEYS
    n = 4097 + 3
    lens = np.full(n, 100, np.uint32)
    lens[17] = 1000                 # a key of its own (class 16)
    lens[2222] = 3000               # another lone record (class 47)
    lens[4000] = 65                 # class 2, alone at its phase below
    offs = np.arange(n, dtype=np.uint64) * 3072 + 16
    offs[4000] += 4                 # dword phase 1: a one-record key
    data = gen_stream(0xBAD0, int(offs[-1]) + 3072)
    dd = torch.as_tensor(data, device="cuda")
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    kidx = (np.arange(n) % len(KEYS)).astype(np.uint32)
    for alg in (1, 2, 4):
        if mode == 0:
            got = gpu.hash_batch(alg, dd, offsets=do, lengths=dl).cpu().numpy()
            exp = oracle.batch(alg, data, offs, lens)
        else:
            got = gpu.hash_batch_keyed(alg, mode, KEYS, dd, key_index=torch.as_tensor(kidx.astype(np.int32),
                                       device="cuda"), offsets=do, lengths=dl).cpu().numpy()
            exp = oracle.batch_keyed(alg, mode, KEYS, data, kidx, offs, lens)
        assert np.array_equal(got, exp), (alg, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("alg,key", [(1, None), (1, b"seg-key"), (2, None), (4, None), (6, None), (5, b"k")])
def test_segmented_long_tiles(gpu, oracle, alg, key, monkeypatch):
    """Segmented long tiles (md_tiles.hpp TileSeg): a batch whose longest
    class (32-64 KiB records) fills 1.25 generations of the tile kernel's
    wave slots or more, and whose tile count leaves the SIMDs unevenly
    loaded, runs each such tile as three jobs handing the state on through
    memory.  Records of
    32,704..40,000 bytes at every byte phase: the digests equal the same
    batch with segmenting off (LCB_TILE_SEGS=0) and, on 400 samples, the
    oracle.  SHA-384/512 run md_lines_kernel's segmented jobs."""
    # 5.33 (MD5, 4 waves per SIMD) and 2.67 (SHA, 2) generations of wave
    # slots, where thirds fill the SIMDs and whole tiles do not (the bucketing
    # cuts only then: lcb_kernels.hip bucket_place_kernel)
    tiles = 2726 if alg in (2, 3, 4) else 5456   # SHA-384/512: md_lines_kernel, 4 waves per SIMD
    n = tiles * 64
    rng = np.random.default_rng(60 + alg)
    lens = rng.integers(32704, 40001, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 16, n - 1).astype(np.uint64))
    total = int(offs[-1] + lens[-1]) + 64
    data = gpu.gen_synthetic(0x5E6 + alg, total)
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    seg = gpu.hash_batch(alg, data, offsets=do, lengths=dl, key=key).cpu().numpy()
    monkeypatch.setenv("LCB_TILE_SEGS", "0")
    whole = gpu.hash_batch(alg, data, offsets=do, lengths=dl, key=key).cpu().numpy()
    monkeypatch.delenv("LCB_TILE_SEGS")
    assert np.array_equal(seg, whole), alg
    pick = np.sort(rng.choice(n, 400, replace=False))
    parts, soff, pos = [], np.zeros(len(pick), np.uint64), 0
    for j, i in enumerate(pick):
        o, ln = int(offs[i]), int(lens[i])
        parts.append(data[o:o + ln].cpu().numpy())
        soff[j] = pos
        pos += ln
    host = np.concatenate(parts)
    exp = oracle.batch(alg, host, soff, lens[pick], key=key)
    assert np.array_equal(seg[pick], exp), alg
    del data
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("alg,key", [(1, None), (1, b"seg-hmac-key"), (2, None), (2, b"seg-hmac-key" * 7),
                                     (3, None), (3, b"224"), (4, None), (4, b"k"), (6, None), (7, None),
                                     (8, None)])
def test_segmented_takeover(gpu, alg, key, monkeypatch):
    """the take-over path of segmented jobs (seg_jobs.hpp
    seg_wait): with LCB_SEG_TAKEOVER=1 the jobs of every cut wave run in
    reverse segment order with no wait, so each wave's last segment starts
    first, finds its predecessors not done and takes the wave over (flag
    kSegTaken, the whole wave from line 0); the middle segment sees the flag
    and leaves, the first one's publish fails.  The digests equal the same
    batch with segmenting off, and the flags read back
    (lcb_hash_gpu_seg_last) show the waves taken over."""
    import ctypes
    # lengths within 7/8 of each other (61,440..65,536 B), so a tile's
    # whole-block lines are most of it and it is cut (md_tiles.hpp); GOST:
    # gost_seg_kernel, 4 waves per SIMD like MD5's tiles
    tiles = 2726 if alg in (2, 3, 4) else 5456
    n = tiles * 64
    rng = np.random.default_rng(160 + alg)
    lens = rng.integers(61440, 65537, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    # SHA-384/512 (md_lines_kernel) stream only 16-B aligned records
    gap = rng.integers(0, 16, n - 1).astype(np.uint64)
    step = lens[:-1].astype(np.uint64) + gap
    if alg in (5, 6):
        step = (step + 15) // 16 * 16
    offs[1:] = np.cumsum(step)
    total = int(offs[-1] + lens[-1]) + 64
    data = gpu.gen_synthetic(0x7A6 + alg, total)
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    monkeypatch.setenv("LCB_TILE_SEGS", "0")
    whole = gpu.hash_batch(alg, data, offsets=do, lengths=dl, key=key).cpu().numpy()
    monkeypatch.delenv("LCB_TILE_SEGS")
    monkeypatch.setenv("LCB_SEG_TAKEOVER", "1")
    taken = gpu.hash_batch(alg, data, offsets=do, lengths=dl, key=key).cpu().numpy()
    st = (ctypes.c_uint32 * 4)()
    assert gpu.lib().lcb_hash_gpu_seg_last(st) == 0
    monkeypatch.delenv("LCB_SEG_TAKEOVER")
    nseg, ntaken, inorder, other = list(st)
    print("alg %d: cut waves %d, taken over %d, in order %d, other %d" % (alg, nseg, ntaken, inorder, other))
    assert np.array_equal(taken, whole), alg
    assert nseg > 0 and ntaken >= 0.9 * nseg and inorder == 0, list(st)
    # and the normal order again (the knob is per call)
    again = gpu.hash_batch(alg, data, offsets=do, lengths=dl, key=key).cpu().numpy()
    assert np.array_equal(again, whole), alg
    if key is not None or alg in (7, 8):   # HMAC tiles and GOST segments against the oracle, sampled
        from oracle.pyoracle import Oracle
        pick = np.sort(rng.choice(n, 64, replace=False))
        parts, soff, pos = [], np.zeros(len(pick), np.uint64), 0
        for j, i in enumerate(pick):
            o, ln = int(offs[i]), int(lens[i])
            parts.append(data[o:o + ln].cpu().numpy())
            soff[j] = pos
            pos += ln
        exp = Oracle().batch(alg, np.concatenate(parts), soff, lens[pick], key=key)
        assert np.array_equal(again[pick], exp)
    del data
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("alg", [7, 8])
def test_gost_segmented_mixed_lengths(gpu, alg, monkeypatch):
    """Plain GOST's segmented long waves (gost_seg_kernel) in the normal
    order, on lengths that vary inside a wave: 300K records of 32..160 KiB
    at random lengths (not multiples of 64; two to three length classes, so
    a cut wave's lanes hold different block counts and each lane cuts its own
    chain in thirds) after 60K short records (the bucketing puts the long
    class first either way).  Digests equal the same batch unsegmented
    (LCB_TILE_SEGS=0) and a sample equals the oracle."""
    from oracle.pyoracle import Oracle
    rng = np.random.default_rng(700 + alg)
    n_long, n_short = 5200 * 64, 60000
    lens = np.concatenate([rng.integers(0, 2000, n_short), rng.integers(32768, 163841, n_long)]).astype(np.uint32)
    rng.shuffle(lens)
    offs = np.zeros(len(lens), np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 8, len(lens) - 1).astype(np.uint64))
    total = int(offs[-1] + lens[-1]) + 64
    data = gpu.gen_synthetic(0x6057 + alg, total)
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    seg = gpu.hash_batch(alg, data, offsets=do, lengths=dl).cpu().numpy()
    monkeypatch.setenv("LCB_TILE_SEGS", "0")
    whole = gpu.hash_batch(alg, data, offsets=do, lengths=dl).cpu().numpy()
    monkeypatch.delenv("LCB_TILE_SEGS")
    assert np.array_equal(seg, whole), alg
    pick = np.sort(rng.choice(len(lens), 48, replace=False))
    parts, soff, pos = [], np.zeros(len(pick), np.uint64), 0
    for j, i in enumerate(pick):
        o, ln = int(offs[i]), int(lens[i])
        parts.append(data[o:o + ln].cpu().numpy())
        soff[j] = pos
        pos += ln
    exp = Oracle().batch(alg, np.concatenate(parts), soff, lens[pick])
    assert np.array_equal(seg[pick], exp), alg
    del data
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("alg", [1, 6])
def test_bucketing_one_kernel_form(gpu, alg, monkeypatch):
    """The one-kernel bucketing (LCB_BUCKET_FUSED=1, lcb_kernels.hip
    bucket_fused_kernel: ticket-ordered count and place phases) gives the
    same digests as the default three-kernel form: the 1M-packet layout
    (tile kernel, padded runs; MD5) and a 300K-message mix with segmented
    long waves (SHA-512, unpadded), three passes each (its sync words reset
    between uses), and a keyed batch (the fused key-index check)."""
    from tests.golden_util import packet_layout
    offs, lens, total = packet_layout()
    data = gpu.gen_synthetic(0xB0C, total)
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    ref = gpu.hash_batch(alg, data, offsets=do, lengths=dl).cpu().numpy()
    monkeypatch.setenv("LCB_BUCKET_FUSED", "1")
    for rep in range(3):
        got = gpu.hash_batch(alg, data, offsets=do, lengths=dl).cpu().numpy()
        assert np.array_equal(got, ref), (alg, rep)
    kidx = torch.as_tensor((np.arange(len(lens)) % 5).astype(np.int32), device="cuda")
    keys = [bytes([k]) * (7 * k + 1) for k in range(5)]
    kf = gpu.hash_batch_keyed(alg, 1, keys, data, key_index=kidx, offsets=do, lengths=dl).cpu().numpy()
    monkeypatch.delenv("LCB_BUCKET_FUSED")
    kr = gpu.hash_batch_keyed(alg, 1, keys, data, key_index=kidx, offsets=do, lengths=dl).cpu().numpy()
    assert np.array_equal(kf, kr), alg
    del data
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_bucketing_large_chunks(gpu, oracle):
    """ragged batches above 4M messages bucket in chunks of
    4097..8192 messages (two unrolled steps per thread, ~1,000 blocks), a
    path the other tests never reach.  4.5M short messages of many lengths:
    the whole batch (chunk 4,395) against its two halves (chunk 4,096) and
    2,000 sampled digests against the oracle, MD5 (tile form, padded runs)
    and SHA-512 (unpadded form)."""
    n = 4_500_000
    rng = np.random.default_rng(45)
    lens = rng.integers(0, 180, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 3)
    total = int(offs[-1] + lens[-1]) + 64
    data = gpu.gen_synthetic(0x4545, total)
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    pick = rng.choice(n, 2000, replace=False)
    host = None
    for alg in (1, 6):
        whole = gpu.hash_batch(alg, data, offsets=do, lengths=dl).cpu().numpy()
        h = n // 2
        a = gpu.hash_batch(alg, data, offsets=do[:h], lengths=dl[:h]).cpu().numpy()
        b = gpu.hash_batch(alg, data, offsets=do[h:], lengths=dl[h:]).cpu().numpy()
        assert np.array_equal(whole, np.concatenate([a, b])), alg
        if host is None:
            host = data.cpu().numpy()
        exp = oracle.batch(alg, host, offs[pick], lens[pick])
        assert np.array_equal(whole[pick], exp), alg
    del data
    torch.cuda.empty_cache()
