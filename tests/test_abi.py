"""The C-ABI library: builds, loads, exports every declared symbol, and fails
loudly (never silently on the CPU) where no MI355X is visible."""
import errno
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDRS = [os.path.join(ROOT, "include", h) for h in ("lcb_hash_gpu.h", "lcb_hash_queue.h", "lcb_crc32_gpu.h", "lcb_chacha_gpu.h")]
SO = os.path.join(ROOT, "liblcb_amd", "liblcb_hash_gpu.so")


def declared_functions():
    names = set()
    for h in HDRS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b([a-z_0-9]+)\(", src)) - {"defined", "sizeof"}
    return sorted(names)


@pytest.fixture(scope="module")
def L():
    import liblcb_amd
    return liblcb_amd.lib()


def test_exports_every_declared_symbol(L):
    names = declared_functions()
    assert len(names) == 26 + 9 + 10 + 3, names   # gpu + queue + crc + chacha
    out = subprocess.check_output(["nm", "-D", "--defined-only", SO]).decode()
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    from liblcb_amd._lib import CHACHA_SIGNATURES, CRC_SIGNATURES, QUEUE_SIGNATURES, SIGNATURES
    sigs = SIGNATURES + QUEUE_SIGNATURES + CRC_SIGNATURES + CHACHA_SIGNATURES
    assert sorted(n for n, _, _ in sigs) == names


def test_info_calls(L):
    assert L.lcb_hash_gpu_abi_version() == 6
    assert [L.lcb_hash_digest_size(a) for a in range(0, 10)] == [0, 16, 20, 28, 32, 48, 64, 32, 64, 0]
    assert [L.lcb_hash_block_size(a) for a in range(1, 9)] == [64, 64, 64, 64, 128, 128, 64, 64]
    assert L.lcb_hash_strerror(errno.EINVAL) == b"invalid argument"


def test_argument_errors(L):
    buf = np.zeros(64, np.uint8)
    out = np.zeros(64, np.uint8)
    # unknown algorithm / flags / null buffers -> EINVAL before touching HIP
    assert L.lcb_hash_batch(0, None, 0, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 0, None) == errno.EINVAL
    assert L.lcb_hash_batch(9, None, 0, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 0, None) == errno.EINVAL
    assert L.lcb_hash_batch(1, None, 0, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 0x10, None) == errno.EINVAL
    assert L.lcb_hash_batch(1, None, 0, None, None, None, 1, 0, 8, out.ctypes.data, 0, None) == errno.EINVAL
    assert L.lcb_hash_batch(1, None, 5, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 0, None) == errno.EINVAL
    # sha2 bits outside sha2_init's table (sha2.h:217-241) -> EINVAL
    ds = np.zeros(1, np.uint64)
    assert L.sha2_get_digest_batch(100, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data,
                                   ds.ctypes.data, 0, None) == errno.EINVAL
    # empty batch is a no-op
    assert L.lcb_hash_batch(1, None, 0, buf.ctypes.data, None, None, 0, 0, 8, out.ctypes.data, 0, None) == 0


def test_digest_size_outparam(L):
    """sha2/gost *_batch report the digest size like the reference's
    digest_size out-parameter, including gost's 'any other bits -> 512'."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    buf = np.zeros(64, np.uint8)
    out = np.zeros(64, np.uint8)
    ds = np.zeros(1, np.uint64)
    L.sha2_get_digest_batch(28, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, ds.ctypes.data, 0, None)
    assert ds[0] == 28
    L.gost3411_2012_get_digest_batch(100, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data,
                                     ds.ctypes.data, 0, None)
    assert ds[0] == 64


def test_fails_loudly_without_gpu(L):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    buf = np.zeros(64, np.uint8)
    out = np.zeros(16, np.uint8)
    assert L.lcb_hash_batch(1, None, 0, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 0, None) == errno.ENODEV
    import liblcb_amd
    with pytest.raises(liblcb_amd.LcbHashError):
        liblcb_amd.md5_get_digest_batch(np.zeros(64, np.uint8), count=1, fixed_len=8)


def test_gost_table_matches_reference(L):
    """The compile-time generated LPS table equals gost3411_2012_Ax."""
    t = np.zeros(2048, np.uint64)
    assert L.lcb_hash_gpu_gost_table(t.ctypes.data) == 0
    from oracle.pyoracle import Ref
    if Ref.available():
        assert np.array_equal(t, Ref().gost_ax())
    # Independently: LPS of 0 through the table equals the first column.
    assert t[0] == t[256 * 0 + 0] and len(set(t[:256].tolist())) == 256


def test_crc32_argument_errors(L):
    buf = np.zeros(64, np.uint8)
    out = np.zeros(4, np.uint32)
    assert L.lcb_crc32_batch(0, None, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 0, None) == errno.EINVAL
    assert L.lcb_crc32_batch(9, None, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 0, None) == errno.EINVAL
    assert L.lcb_crc32_batch(1, None, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data + 1, 0, None) == errno.EINVAL
    assert L.lcb_crc32_batch(1, None, None, None, None, 1, 0, 8, out.ctypes.data, 0, None) == errno.EINVAL
    assert L.lcb_crc32_batch(1, None, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 4, None) == errno.EINVAL
    assert L.crc32c_batch(None, buf.ctypes.data, None, None, 0, 0, 8, out.ctypes.data, 0, None) == 0
    # the digest entry point does not take CRC ids
    assert L.lcb_hash_batch(101, None, 0, buf.ctypes.data, None, None, 1, 0, 8, out.ctypes.data, 0, None) == errno.EINVAL


def test_crc32_fails_loudly_without_gpu(L):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    import liblcb_amd.crc32 as c
    with pytest.raises(liblcb_amd_error()):
        c.crc32c_batch(np.zeros(64, np.uint8), count=1, fixed_len=8)


def liblcb_amd_error():
    import liblcb_amd
    return liblcb_amd.LcbHashError


def test_crc32_tables_match_reference(L):
    """Table 0 of every variant == the reference's crc32_tbl256_*; table k is
    table k-1 advanced by one zero byte."""
    from oracle.pyoracle import Oracle, Ref
    ref = Ref() if Ref.available() else Oracle()
    for v in range(1, 9):
        t = np.zeros(8 * 256, np.uint32)
        assert L.lcb_crc32_gpu_tables(v, t.ctypes.data) == 0
        t = t.reshape(8, 256)
        assert np.array_equal(t[0], ref.crc32_table(v)), v
        refl = v in (4, 5, 6, 7)
        for k in range(1, 8):
            p = t[k - 1].astype(np.uint64)
            if refl:
                want = (p >> 8) ^ t[0][(p & 255).astype(np.int64)]
            else:
                want = ((p << 8) & 0xffffffff) ^ t[0][(p >> 24).astype(np.int64)]
            assert np.array_equal(t[k], want.astype(np.uint32)), (v, k)


def test_chacha_argument_errors(L):
    key = np.zeros(32, np.uint8)
    buf = np.zeros(64, np.uint8)
    k, b = key.ctypes.data, buf.ctypes.data
    # null key / dst, unknown flags, unbounded rounds -> EINVAL before touching HIP
    assert L.lcb_chacha_batch(0, None, 32, None, None, 20, b, b, None, None, 1, 0, 8, 0, None) == errno.EINVAL
    assert L.lcb_chacha_batch(0, k, 32, None, None, 20, b, None, None, None, 1, 0, 8, 0, None) == errno.EINVAL
    assert L.lcb_chacha_batch(0, k, 32, None, None, 20, b, b, None, None, 1, 0, 8, 0x10, None) == errno.EINVAL
    assert L.chacha_batch(k, 32, None, None, 1 << 20, b, b, None, None, 1, 0, 8, 0, None) == errno.EINVAL
    # empty batch is a no-op
    assert L.xchacha_batch(k, 32, None, None, 20, b, b, None, None, 0, 0, 8, 0, None) == 0


def test_chacha_fails_loudly_without_gpu(L):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    key = np.zeros(32, np.uint8)
    buf = np.zeros(64, np.uint8)
    assert L.chacha_batch(key.ctypes.data, 32, None, None, 20, buf.ctypes.data, buf.ctypes.data, None, None,
                          1, 0, 64, 0, None) == errno.ENODEV
    import liblcb_amd.chacha as c
    with pytest.raises(liblcb_amd_error()):
        c.chacha_batch(bytes(32), np.zeros(64, np.uint8), count=1, fixed_len=64)
