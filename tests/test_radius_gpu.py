"""Keyed batches (lcb_hash_batch_keyed) and the RADIUS shapes built on them.

GPU, against the oracle: every algorithm x {HMAC, H(K || m), H(m || K)}
with a per-message key index into a 7-key table (key lengths 0, 1, 15, 64,
65, 128, 200: empty, short, one block, multi-block, longer than the HMAC
block), ragged misaligned messages of 0..300 bytes, device and host mode.

GPU, against the REFERENCE: tests/golden/radius.json holds 481 packets the
reference's own radius.h built and signed (radius_pkt_sign) and verified
(radius_pkt_verify), plus its User-Password encodings.  liblcb_amd.radius
re-signs the unsigned packets and verifies the signed ones with every MD5 /
HMAC-MD5 on the GPU: byte-identical packets, identical verification results,
and tampered packets rejected.
"""
import errno
import json
import os

import numpy as np
import pytest

from oracle.pyoracle import gen_stream

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "radius.json")
KEYS = [b"", b"k", bytes(range(15)), bytes(range(64)), bytes(range(1, 66)), bytes(range(128)),
        bytes((3 * i) & 0xFF for i in range(200))]


@pytest.fixture(scope="module")
def rad():
    j = json.load(open(GOLDEN))
    j["secrets"] = [bytes.fromhex(s) for s in j["secrets"]]
    return j


def _ragged(seed, n):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 301, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    pos = 1
    for i in range(n):
        offs[i] = pos
        pos += int(lens[i]) + int(rng.integers(0, 7))
    kidx = rng.integers(0, len(KEYS), n).astype(np.uint32)
    return gen_stream(seed, pos + 8), offs, lens, kidx


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2, 3])
def test_keyed_vs_oracle_device(gpu, oracle, mode):
    import torch
    data, offs, lens, kidx = _ragged(10 + mode, 3000)
    dd = torch.as_tensor(data, device="cuda")
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    dk = torch.as_tensor(kidx.astype(np.int32), device="cuda")
    for alg in range(1, 9):
        got = gpu.hash_batch_keyed(alg, mode, KEYS, dd, key_index=dk, offsets=do, lengths=dl).cpu().numpy()
        exp = oracle.batch_keyed(alg, mode, KEYS, data, kidx, offs, lens)
        assert np.array_equal(got, exp), (alg, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 3])
def test_keyed_tiles_every_key_length(gpu, oracle, mode):
    """Device mode above the bucketing threshold: the tile kernel of every
    64-B-block hash, keyed HMAC and secret suffix, with the 7 keys (0..200
    bytes: a suffix that ends in the message's last block, spans the next
    ones, or is empty) at every start byte phase and tail length."""
    import torch
    data, offs, lens, kidx = _ragged(40 + mode, 9000)
    dd = torch.as_tensor(data, device="cuda")
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    dk = torch.as_tensor(kidx.astype(np.int32), device="cuda")
    for alg in (1, 2, 3, 4):
        got = gpu.hash_batch_keyed(alg, mode, KEYS, dd, key_index=dk, offsets=do, lengths=dl).cpu().numpy()
        exp = oracle.batch_keyed(alg, mode, KEYS, data, kidx, offs, lens)
        assert np.array_equal(got, exp), (alg, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2, 3])
def test_keyed_vs_oracle_host_and_fixed(gpu, oracle, mode):
    data, offs, lens, kidx = _ragged(20 + mode, 6000)   # above the bucketing threshold
    for alg in (1, 2, 4, 6, 7):
        got = gpu.hash_batch_keyed(alg, mode, KEYS, data, key_index=kidx, offsets=offs, lengths=lens)
        assert np.array_equal(got, oracle.batch_keyed(alg, mode, KEYS, data, kidx, offs, lens)), (alg, mode)
    # fixed stride, one key for every message (key_index NULL)
    fx = gen_stream(30 + mode, 500 * 200)
    for alg in (1, 5, 8):
        got = gpu.hash_batch_keyed(alg, mode, [KEYS[4]], fx, count=500, stride=200, fixed_len=190)
        exp = oracle.batch_keyed(alg, mode, [KEYS[4]], fx, None, count=500, stride=200, fixed_len=190)
        assert np.array_equal(got, exp), (alg, mode)


@pytest.mark.gpu
def test_keyed_hmac_equals_single_key_hmac(gpu):
    """KEY_HMAC with one key == the single-key HMAC of lcb_hash_batch."""
    import torch
    data = gpu.gen_synthetic(3, 4096 * 1024)
    for alg in (1, 4, 7):
        a = gpu.hash_batch(alg, data, count=4096, stride=1024, fixed_len=1024, key=b"radius-secret")
        b = gpu.hash_batch_keyed(alg, gpu.KEY_HMAC, [b"radius-secret"], data, count=4096, stride=1024,
                                 fixed_len=1024)
        assert bool((a == b).all()), alg
        torch.cuda.synchronize()


def test_keyed_argument_errors():
    import liblcb_amd
    try:
        L = liblcb_amd.lib()
    except RuntimeError as e:
        pytest.skip(str(e))
    buf = np.zeros(64, np.uint8)
    out = np.zeros(64, np.uint8)
    kl = np.array([4], np.uint32)
    k = np.frombuffer(b"abcd", np.uint8)
    args = (k.ctypes.data, None, kl.ctypes.data, 1, None, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 0,
            None)
    assert L.lcb_hash_batch_keyed(1, 0, *args) == errno.EINVAL          # mode
    assert L.lcb_hash_batch_keyed(1, 4, *args) == errno.EINVAL
    assert L.lcb_hash_batch_keyed(9, 1, *args) == errno.EINVAL          # alg
    assert L.lcb_hash_batch_keyed(1, 1, k.ctypes.data, None, kl.ctypes.data, 0, None, buf.ctypes.data, None, None,
                                  1, 0, 8, out.ctypes.data, 0, None) == errno.EINVAL   # no keys
    assert L.lcb_hash_batch_keyed(1, 1, None, None, kl.ctypes.data, 1, None, buf.ctypes.data, None, None,
                                  1, 0, 8, out.ctypes.data, 0, None) == errno.EINVAL   # key bytes missing
    bad = np.array([1], np.uint32)                                         # index >= nkeys (host mode)
    import torch
    if not torch.cuda.is_available():
        assert L.lcb_hash_batch_keyed(1, 1, k.ctypes.data, None, kl.ctypes.data, 1, bad.ctypes.data,
                                      buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 0, None) == \
            errno.EINVAL


# ----------------------------------------------------------------- RADIUS
@pytest.mark.gpu
@pytest.mark.parametrize("device", [False, True])
def test_sign_matches_reference(gpu, rad, device):
    from liblcb_amd.radius import radius_pkt_sign_batch
    P = rad["packets"]
    err, got = radius_pkt_sign_batch([bytes.fromhex(p["pre"]) for p in P], rad["secrets"],
                                     [p["key"] for p in P], device=device)
    assert err.tolist() == [0] * len(P)
    bad = [i for i, p in enumerate(P) if got[i].hex() != p["signed"]]
    assert not bad, (len(bad), [P[i]["code"] for i in bad[:10]])


@pytest.mark.gpu
@pytest.mark.parametrize("device", [False, True])
def test_verify_matches_reference(gpu, rad, device):
    from liblcb_amd.radius import radius_pkt_verify_batch
    P = rad["packets"]
    reqs = [bytes.fromhex(p["request"]) if p["kind"] == "reply" else None for p in P]
    err, out = radius_pkt_verify_batch([bytes.fromhex(p["signed"]) for p in P], rad["secrets"],
                                       [p["key"] for p in P], reqs, device=device)
    assert err.tolist() == [0] * len(P)
    assert [o.hex() for o in out] == [p["verified"] for p in P]
    # passwords decoded back to the plaintext the reference encoded
    n = 0
    for p, o in zip(P, out):
        if p["kind"] == "request" and p.get("password"):
            pw = bytes.fromhex(p["password"])
            from liblcb_amd.radius import find_attr
            a = find_attr(o, 2)
            assert o[a + 2:a + 2 + len(pw)] == pw
            n += 1
    assert n > 50


@pytest.mark.gpu
def test_verify_rejects_tampering(gpu, rad):
    """One flipped byte in a signed packet (attribute data, or the
    authenticator) makes the check the reference would fail fail here."""
    from liblcb_amd.radius import RANDOM_AUTH, find_attr, radius_pkt_verify_batch
    P = [p for p in rad["packets"] if p["msg_authr"] or p["code"] not in RANDOM_AUTH]
    pk, reqs = [], []
    for p in P:
        b = bytearray.fromhex(p["signed"])
        if p["msg_authr"]:
            b[find_attr(b, 80) + 5] ^= 1            # inside the Message-Authenticator
        else:
            b[7] ^= 1                               # inside the authenticator
        pk.append(bytes(b))
        reqs.append(bytes.fromhex(p["request"]) if p["kind"] == "reply" else None)
    err, _ = radius_pkt_verify_batch(pk, rad["secrets"], [p["key"] for p in P], reqs)
    assert (err == errno.EBADMSG).all(), np.unique(err)


@pytest.mark.gpu
def test_password_encode_vectors(gpu, rad):
    """radius_pkt_attr_password_encode (radius.h:745-790) for every password
    length 1..128 through the KEY_PREFIX chain."""
    from liblcb_amd.radius import radius_pkt_sign_batch
    pk, ki, want = [], [], []
    for v in rad["password_encode"]:
        pw = bytes.fromhex(v["password"])
        tm = (len(pw) + 15) // 16 * 16
        attr = bytes([2, 2 + tm]) + pw + bytes(tm - len(pw))
        hdr = bytes([1, 0]) + (20 + len(attr)).to_bytes(2, "big") + bytes.fromhex(v["authenticator"])
        pk.append(hdr + attr)
        ki.append(v["key"])
        want.append(v["encoded"])
    err, got = radius_pkt_sign_batch(pk, rad["secrets"], ki)
    assert [g[22:].hex() for g in got] == want


# ------------------------------------------- host logic, CPU (oracle backend)
@pytest.fixture
def oracle_keyed(monkeypatch, oracle):
    """liblcb_amd.radius with its keyed batches served by the oracle: checks
    the host-side packet logic (field substitution, chaining, XOR) on CPU."""
    import liblcb_amd.radius as R

    def fake(alg, mode, keys, data, key_index=None, offsets=None, lengths=None, **kw):
        return oracle.batch_keyed(alg, mode, keys, data, key_index, offsets, lengths)
    monkeypatch.setattr(R, "hash_batch_keyed", fake)
    return R


def test_radius_host_logic_sign_verify(oracle_keyed, rad):
    R = oracle_keyed
    P = rad["packets"]
    err, got = R.radius_pkt_sign_batch([bytes.fromhex(p["pre"]) for p in P], rad["secrets"],
                                       [p["key"] for p in P])
    assert err.tolist() == [0] * len(P)
    assert [g.hex() for g in got] == [p["signed"] for p in P]
    reqs = [bytes.fromhex(p["request"]) if p["kind"] == "reply" else None for p in P]
    err, out = R.radius_pkt_verify_batch(got, rad["secrets"], [p["key"] for p in P], reqs)
    assert err.tolist() == [0] * len(P)
    assert [o.hex() for o in out] == [p["verified"] for p in P]
    # a reply without its request: EINVAL, as radius_pkt_verify returns
    i = [k for k, p in enumerate(P) if p["kind"] == "reply" and p["code"] in R.REPLY_AUTH][0]
    err, _ = R.radius_pkt_verify_batch([got[i]], rad["secrets"], [P[i]["key"]], [None])
    assert err.tolist() == [errno.EINVAL]


# --------------------------------------------------- edge cases
@pytest.fixture(scope="module")
def rad_edge():
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", "radius_edge.json")))["cases"]


def _check_edge(R, rad, cases, device=False):
    """radius_pkt_sign_batch against the reference's radius_pkt_sign on
    packets with bytes past their Length and on User-Passwords it refuses:
    the same error (EOVERFLOW / EINVAL, packet untouched) or the same signed
    packet over [0, Length) with the extra bytes left as they were; the
    signed packets (with their tails) then verify."""
    pk = [bytes.fromhex(c["pre"]) for c in cases]
    err, got = R.radius_pkt_sign_batch(pk, rad["secrets"], [c["key"] for c in cases], device=device)
    assert err.tolist() == [c["rc"] for c in cases]
    for c, p, g in zip(cases, pk, got):
        if c["rc"]:
            assert g == p, c["what"]
        else:
            n = R.pkt_len(p)
            assert g[:n].hex() == c["signed"], c["what"]
            assert g[n:] == p[n:]
    # requests verify on their own (replies would need their request)
    req = [(c, g) for c, g in zip(cases, got)
           if c["rc"] == 0 and g[0] not in R.REPLY_AUTH and g[0] != R.ACCOUNTING_RESPONSE]
    assert len(req) > 20
    e, _ = R.radius_pkt_verify_batch([g for _, g in req], rad["secrets"], [c["key"] for c, _ in req],
                                     device=device)
    assert (e == 0).all(), e


def test_radius_edge_host_logic(oracle_keyed, rad, rad_edge):
    _check_edge(oracle_keyed, rad, rad_edge)


@pytest.mark.gpu
@pytest.mark.parametrize("device", [False, True])
def test_radius_edge_gpu(gpu, rad, rad_edge, device):
    import liblcb_amd.radius as R
    _check_edge(R, rad, rad_edge, device)


# ------------------------------------- keyed-batch arguments
@pytest.mark.gpu
@pytest.mark.parametrize("device", [False, True])
def test_keyed_bad_index_is_einval(gpu, device):
    """A key index >= nkeys is EINVAL in host AND device mode, and no digest
    is written (device mode checks on the device before the batch runs)."""
    import torch
    from liblcb_amd._lib import LcbHashError
    n = 5000                                   # large enough to be bucketed (tile kernel)
    data = gen_stream(0x5EED, n * 100)
    lens = np.full(n, 97, np.uint32)
    offs = np.arange(n, dtype=np.uint64) * 100
    kidx = np.zeros(n, np.uint32)
    kidx[1234] = len(KEYS)                     # one out of range
    for mode in (1, 2, 3):
        if device:
            out = torch.full((n, 16), 0x5A, dtype=torch.uint8, device="cuda")
            args = dict(key_index=torch.as_tensor(kidx.astype(np.int32), device="cuda"),
                        offsets=torch.as_tensor(offs.astype(np.int64), device="cuda"),
                        lengths=torch.as_tensor(lens.astype(np.int32), device="cuda"), out=out)
            d = torch.as_tensor(data, device="cuda")
        else:
            out = np.full((n, 16), 0x5A, np.uint8)
            args = dict(key_index=kidx, offsets=offs, lengths=lens, out=out)
            d = data
        with pytest.raises(LcbHashError) as e:
            gpu.hash_batch_keyed(1, mode, KEYS, d, **args)
        assert e.value.errno == errno.EINVAL
        if device:
            torch.cuda.synchronize()
            out = out.cpu().numpy()
        assert (out == 0x5A).all()


@pytest.mark.gpu
def test_wrapper_validation_device(gpu):
    """The device-mode wrappers refuse descriptions the C-ABI would read out
    of range: wrong dtypes, non-contiguous, other device, short
    arrays, a short `out`."""
    import torch
    n = 64
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * 16
    lens = torch.full((n,), 16, dtype=torch.int32, device="cuda")
    kidx = torch.zeros(n, dtype=torch.int32, device="cuda")
    bad = [dict(lengths=lens.to(torch.int64), offsets=offs),          # lengths read as uint32
           dict(lengths=lens, offsets=offs.to(torch.int32)),          # offsets read as uint64
           dict(lengths=lens[::2].repeat(2), offsets=offs[:32]),      # short offsets
           dict(lengths=lens, offsets=offs, key_index=kidx.to(torch.int64)),
           dict(lengths=lens, offsets=offs, key_index=kidx[:10]),
           dict(lengths=lens, offsets=offs, out=torch.empty(n * 16 - 1, dtype=torch.uint8, device="cuda")),
           dict(lengths=lens, offsets=offs, key_index=kidx.cpu())]
    for kw in bad:
        with pytest.raises((TypeError, ValueError)):
            gpu.hash_batch_keyed(1, 1, KEYS, d, **kw)
    with pytest.raises((TypeError, ValueError)):
        gpu.hash_batch_multi([0], 1, d, lengths=lens.to(torch.int64), offsets=offs)
    with pytest.raises((TypeError, ValueError)):
        gpu.hash_batch_multi([0], 1, d, lengths=lens, offsets=offs,
                             out=torch.empty(8, dtype=torch.uint8, device="cuda"))
    with pytest.raises((TypeError, ValueError)):
        gpu.hash_batch(1, d, lengths=lens, offsets=offs[::2])


def test_wrapper_validation_host():
    """Host-mode wrappers: short per-message arrays and a short `out` are
    refused before the C-ABI is called (no GPU needed)."""
    import liblcb_amd
    n = 64
    d = np.zeros(n * 16, np.uint8)
    offs = np.arange(n, dtype=np.uint64) * 16
    lens = np.full(n, 16, np.uint32)
    with pytest.raises(ValueError):
        liblcb_amd.hash_batch_keyed(1, 1, KEYS, d, key_index=np.zeros(10, np.uint32), offsets=offs, lengths=lens)
    with pytest.raises(ValueError):
        liblcb_amd.hash_batch_keyed(1, 1, KEYS, d, offsets=offs, lengths=lens, out=np.empty(10, np.uint8))
    with pytest.raises(ValueError):
        liblcb_amd.hash_batch_multi([0], 1, d, offsets=offs, lengths=lens, out=np.empty(10, np.uint8))
    with pytest.raises(ValueError):
        liblcb_amd.hash_batch(1, d, offsets=offs, lengths=lens, out=np.empty((n, 15), np.uint8))
    with pytest.raises(ValueError):
        liblcb_amd.hash_batch_multi([0], 1, d, offsets=offs, lengths=lens, copy_parts=True)


@pytest.mark.gpu
def test_keyed_check_epochs_same_stream(gpu, oracle):
    """The device-mode key-index check writes the call's epoch into the
    stream scratch's flag word (lcb_hash_gpu.cpp, r5): bad, good, bad, good
    batches back to back on ONE stream -- every bad one is EINVAL with no
    digest written, every good one right.  Tile kernel (5000 messages,
    bucketed), per-lane keyed kernel (KEY_PREFIX) and GOST, and a key table
    that changes between calls (the key cache must not hand one table's
    mid-states to another)."""
    import torch
    from liblcb_amd._lib import LcbHashError
    data, offs, lens, kidx = _ragged(77, 5000)
    dd = torch.as_tensor(data, device="cuda")
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    bad = kidx.copy()
    bad[4321] = len(KEYS) + 3
    dk_good = torch.as_tensor(kidx.astype(np.int32), device="cuda")
    dk_bad = torch.as_tensor(bad.astype(np.int32), device="cuda")
    keys2 = [k[::-1] + b"x" for k in KEYS]           # a second table, same shape
    for alg, mode in ((1, 1), (1, 3), (4, 1), (1, 2), (7, 1)):
        for rep in range(2):
            for keys in (KEYS, keys2):
                out = torch.full((len(lens), gpu.DIGEST_SIZE[alg]), 0x5A, dtype=torch.uint8, device="cuda")
                with pytest.raises(LcbHashError) as e:
                    gpu.hash_batch_keyed(alg, mode, keys, dd, key_index=dk_bad, offsets=do, lengths=dl, out=out)
                assert e.value.errno == errno.EINVAL
                got = gpu.hash_batch_keyed(alg, mode, keys, dd, key_index=dk_good, offsets=do, lengths=dl)
                assert np.array_equal(got.cpu().numpy(), oracle.batch_keyed(alg, mode, keys, data, kidx, offs, lens)), \
                    (alg, mode, rep)
                torch.cuda.synchronize()
                assert (out.cpu().numpy() == 0x5A).all(), (alg, mode, rep)


@pytest.mark.gpu
def test_hmac_key_cache_distinct_keys(gpu, oracle):
    """Single-key HMAC mid-states come from the per-device key cache: many
    different keys (more than the cache holds) and repeats, every result vs
    the oracle (short, block-sized and long keys)."""
    import torch
    n = 300
    data = gen_stream(91, n * 130)
    dd = torch.as_tensor(data, device="cuda")
    offs = np.arange(n, dtype=np.uint64) * 130
    lens = (np.arange(n) % 129).astype(np.uint32)
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    keys = [bytes([i]) * (i * 7 % 150) for i in range(24)]
    for rep in range(2):
        for i, k in enumerate(keys):
            alg = (1, 2, 4, 6, 7)[i % 5]
            got = gpu.hash_batch(alg, dd, offsets=do, lengths=dl, key=k).cpu().numpy()
            assert np.array_equal(got, oracle.batch(alg, data, offs, lens, key=k)), (alg, i, rep)


@pytest.mark.gpu
def test_key_cache_lru_flush_and_off(gpu, oracle, monkeypatch):
    """ADVICE r5 (the key cache holds secrets): more distinct key tables than
    the cache holds, repeated, stay right (least recently used evicted and
    zeroed, re-prepared on return); lcb_hash_key_cache_flush drops every
    entry; LCB_HASH_KEY_CACHE=0 adds none and stays right (per-call buffers)."""
    import torch
    L = gpu.lib()
    data, offs, lens, kidx = _ragged(17, 600)
    dd = torch.as_tensor(data, device="cuda")
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    dk = torch.as_tensor(kidx.astype(np.int32), device="cuda")
    tables = [[k + bytes([t]) for k in KEYS] for t in range(20)]
    for rep in range(2):
        for t, keys in enumerate(tables):
            got = gpu.hash_batch_keyed(1, 1, keys, dd, key_index=dk, offsets=do, lengths=dl).cpu().numpy()
            assert np.array_equal(got, oracle.batch_keyed(1, 1, keys, data, kidx, offs, lens)), (rep, t)
            assert L.lcb_hash_key_cache_entries() <= 16
    assert L.lcb_hash_key_cache_entries() == 16
    torch.cuda.synchronize()
    assert L.lcb_hash_key_cache_flush() == 0
    assert L.lcb_hash_key_cache_entries() == 0
    monkeypatch.setenv("LCB_HASH_KEY_CACHE", "0")
    for t in (0, 5):
        got = gpu.hash_batch_keyed(4, 3, tables[t], dd, key_index=dk, offsets=do, lengths=dl).cpu().numpy()
        assert np.array_equal(got, oracle.batch_keyed(4, 3, tables[t], data, kidx, offs, lens)), t
        got = gpu.hash_batch(1, dd, offsets=do, lengths=dl, key=b"per-call key").cpu().numpy()
        assert np.array_equal(got, oracle.batch(1, data, offs, lens, key=b"per-call key"))
    assert L.lcb_hash_key_cache_entries() == 0


@pytest.mark.gpu
def test_keyed_unfused_check_bad_then_good(gpu, oracle):
    """the unfused key-index check (key_index_check_kernel: a
    fixed-stride keyed batch, and a ragged one under 4096 messages) counts
    its blocks on a host-tracked counter; a bad index then a good one, back
    to back on ONE stream, several times: EINVAL with no digest, then right
    digests (a miscounted counter would make every later call EIO)."""
    import torch
    from liblcb_amd._lib import LcbHashError
    n = 3000
    data = gen_stream(0xF1, n * 128)
    dd = torch.as_tensor(data, device="cuda")
    kidx = (np.arange(n) % len(KEYS)).astype(np.uint32)
    bad = kidx.copy()
    bad[n - 7] = len(KEYS)
    dk_good = torch.as_tensor(kidx.astype(np.int32), device="cuda")
    dk_bad = torch.as_tensor(bad.astype(np.int32), device="cuda")
    offs = np.arange(n, dtype=np.uint64) * 128
    lens = (np.arange(n) % 120).astype(np.uint32)
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    shapes = (("fixed", dict(count=n, stride=128, fixed_len=100), offs, np.full(n, 100, np.uint32)),
              ("ragged", dict(offsets=do, lengths=dl), offs, lens))
    for rep in range(3):
        for name, shape, eo, el in shapes:
            out = torch.full((n, 16), 0x5A, dtype=torch.uint8, device="cuda")
            with pytest.raises(LcbHashError) as e:
                gpu.hash_batch_keyed(1, 1, KEYS, dd, key_index=dk_bad, out=out, **shape)
            assert e.value.errno == errno.EINVAL, (name, rep)
            got = gpu.hash_batch_keyed(1, 1, KEYS, dd, key_index=dk_good, **shape)
            assert np.array_equal(got.cpu().numpy(), oracle.batch_keyed(1, 1, KEYS, data, kidx, eo, el)), (name, rep)
            torch.cuda.synchronize()
            assert (out.cpu().numpy() == 0x5A).all(), (name, rep)
