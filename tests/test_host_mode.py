"""Host-memory mode of the C-ABI (lcb_hash_batch with flags = 0) at its
staging limits, and the Python mirror's argument validation.

GPU: fixed-length pageable batches whose packed size exceeds the 64 MiB
pinned staging buffer with stride 0 (one message repeated) and with
overlapping records (stride = fixed_len / 2); checked against the oracle.
CPU: out-of-range buffer descriptions raise ValueError before any native
call reads memory.
"""
import numpy as np
import pytest

from oracle.pyoracle import gen_stream


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [0, 512])
@pytest.mark.parametrize("pinned", [False, True])
def test_fixed_overlapping_records_beyond_staging(gpu, oracle, stride, pinned):
    import torch
    n, L = 300_000, 1024          # 300K x 1 KiB packed = 293 MiB > 64 MiB staging
    nbytes = (n - 1) * stride + L
    host = gen_stream(41 + stride, nbytes)
    if pinned:
        t = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        t.numpy()[:] = host
        host = t.numpy()
    got = gpu.hash_batch(1, host, count=n, stride=stride, fixed_len=L)
    if stride == 0:
        exp = np.repeat(oracle.batch(1, host[:L], count=1, stride=0, fixed_len=L), n, axis=0)
    else:
        exp = oracle.batch_fixed_mt(1, host, n, stride, L, threads=8)
    assert np.array_equal(got, exp)


@pytest.mark.gpu
def test_host_ragged_hmac_overlapping(gpu, oracle):
    """Ragged host batch whose records overlap (offsets step 100, length 700):
    the gather path packs more bytes than the span."""
    n = 120_000
    offs = np.arange(n, dtype=np.uint64) * 100
    lens = np.full(n, 700, np.uint32)
    data = gen_stream(9, int(offs[-1]) + 700)
    got = gpu.hash_batch(4, data, offsets=offs, lengths=lens, key=b"radius")
    exp = oracle.batch(4, data, offs, lens, key=b"radius")
    assert np.array_equal(got, exp)


def _lib_or_skip():
    import liblcb_amd
    try:
        liblcb_amd.lib()
    except RuntimeError as e:
        pytest.skip(str(e))
    return liblcb_amd


@pytest.mark.parametrize("kw", [
    dict(count=5, stride=1024, fixed_len=1024),                       # 5 KiB of a 4 KiB buffer
    dict(count=4, stride=1024, fixed_len=1025),
    dict(offsets=np.array([0, 4000], np.uint64), lengths=np.array([10, 97], np.uint32)),
    dict(offsets=np.array([0], np.uint64), lengths=np.array([1, 2], np.uint32), count=2),
])
def test_extent_is_validated(kw):
    lcb = _lib_or_skip()
    data = np.zeros(4096, np.uint8)
    from liblcb_amd.chacha import chacha_batch
    from liblcb_amd.crc32 import crc32_batch
    with pytest.raises(ValueError):
        lcb.hash_batch(1, data, **kw)
    with pytest.raises(ValueError):
        crc32_batch(1, data, **kw)
    with pytest.raises(ValueError):
        chacha_batch(bytes(32), data, **kw)


def test_extent_in_range_passes_validation():
    from liblcb_amd.hash import _check_extent
    _check_extent(4096, 4, None, None, 1024, 1024)
    _check_extent(4096, 3, np.array([0, 100, 4000], np.uint64), np.array([0, 5, 96], np.uint32), 0, 0)
    _check_extent(0, 0, None, None, 0, 0)
    _check_extent(10, 1000, None, None, 0, 10)      # stride 0: one message repeated
