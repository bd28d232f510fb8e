"""Host-side mirror of liblcb's include/math/crc32.h macros, batched.

crc32X_batch(data, ...) returns, per buffer, the value of the reference macro
crc32X(data, size); with `init=` it returns crc32X_update(init[i], data, size)
(crc32.h:501-576).  Buffer description and memory modes as liblcb_amd.hash:
torch CUDA tensors run in device mode on torch's current stream, numpy /
bytes in host mode through pinned staging.  All CRCs are computed by the HIP
kernels of liblcb_hash_gpu.so; there is no CPU path.
"""
import numpy as np
import torch

from ._lib import F_DEVICE, check, lib
from .hash import _check_extent, _is_dev, _layout

CRC32A, CRC32CKSUM, CRC32MPEG2, CRC32B, CRC32JAMCRC, CRC32C, CRC32D, CRC32Q = range(1, 9)
CRC_NAMES = {CRC32A: "crc32a", CRC32CKSUM: "crc32cksum", CRC32MPEG2: "crc32mpeg2",
             CRC32B: "crc32b", CRC32JAMCRC: "crc32jamcrc", CRC32C: "crc32c", CRC32D: "crc32d",
             CRC32Q: "crc32q"}
CRC_IDS = {v: k for k, v in CRC_NAMES.items()}

__all__ = ["crc32_batch", "CRC_NAMES", "CRC_IDS"] + ["%s_batch" % n for n in CRC_NAMES.values()]


def crc32_batch(variant, data, *, offsets=None, lengths=None, count=None, stride=None,
                fixed_len=None, init=None, out=None):
    """CRC of every buffer; returns uint32 (count,) in the memory kind of `data`."""
    if isinstance(variant, str):
        variant = CRC_IDS[variant]
    L = lib()
    if _is_dev(data):
        assert data.dtype == torch.uint8 and data.is_contiguous()
        count, stride, fixed_len = _layout(count, offsets, lengths, stride, fixed_len, data.numel())
        for t, dt in ((offsets, (torch.int64, torch.uint64)), (lengths, (torch.int32, torch.uint32)),
                      (init, (torch.int32, torch.uint32))):
            if t is not None:
                assert _is_dev(t) and t.dtype in dt and t.is_contiguous() and t.device == data.device
        _check_extent(data.numel(), count, offsets, lengths, stride, fixed_len)
        if init is not None:
            assert init.numel() >= count
        if out is None:
            out = torch.empty(count, dtype=torch.int32, device=data.device)
        assert out.numel() >= count
        with torch.cuda.device(data.device):
            stream = torch.cuda.current_stream(data.device).cuda_stream
            check(L.lcb_crc32_batch(variant, init.data_ptr() if init is not None else None,
                                    data.data_ptr(),
                                    offsets.data_ptr() if offsets is not None else None,
                                    lengths.data_ptr() if lengths is not None else None,
                                    count, stride, fixed_len, out.data_ptr(), F_DEVICE, stream))
        return out
    if isinstance(data, (bytes, bytearray, memoryview)):
        data = np.frombuffer(bytes(data), dtype=np.uint8)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    nbytes = data.size
    if data.size == 0:
        data = np.zeros(1, dtype=np.uint8)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    if lengths is not None:
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    if init is not None:
        init = np.ascontiguousarray(init, dtype=np.uint32)
    count, stride, fixed_len = _layout(count, offsets, lengths, stride, fixed_len, data.size)
    _check_extent(nbytes, count, offsets, lengths, stride, fixed_len)
    if init is not None:
        assert init.size >= count
    if out is None:
        out = np.empty(count, dtype=np.uint32)
    assert out.dtype == np.uint32 and out.flags.c_contiguous and out.size >= count
    check(L.lcb_crc32_batch(variant, init.ctypes.data if init is not None else None, data.ctypes.data,
                            offsets.ctypes.data if offsets is not None else None,
                            lengths.ctypes.data if lengths is not None else None,
                            count, stride, fixed_len, out.ctypes.data, 0, None))
    return out


def _named(variant):
    name = CRC_NAMES[variant]

    def fn(data, **kw):
        return crc32_batch(variant, data, **kw)
    fn.__name__ = name + "_batch"
    fn.__doc__ = "Batch %s / %s_update (include/math/crc32.h)." % (name, name)
    return fn


crc32a_batch = _named(CRC32A)
crc32cksum_batch = _named(CRC32CKSUM)
crc32mpeg2_batch = _named(CRC32MPEG2)
crc32b_batch = _named(CRC32B)
crc32jamcrc_batch = _named(CRC32JAMCRC)
crc32c_batch = _named(CRC32C)
crc32d_batch = _named(CRC32D)
crc32q_batch = _named(CRC32Q)
