"""Host-side mirror of liblcb's include/crypto/cipher/chacha.h one-shot
functions, batched.

chacha_batch(key, src, ...) returns dst where buffer i holds exactly what the
reference's chacha(key, key_size, counter_i, iv_i, rounds, src_i, len_i,
dst_i) writes (chacha.h:662-674); xchacha_batch the same for xchacha()
(chacha.h:681-693, 24-byte ivs).  src None gives the keystream itself.
Buffer description as liblcb_amd.hash (offsets/lengths or stride/fixed_len).
torch CUDA tensors run in device mode on torch's current stream; numpy /
bytes run in host mode through page-locked staging.  Every byte is produced
by the HIP kernels of liblcb_hash_gpu.so; there is no CPU path.
"""
import ctypes

import numpy as np
import torch

from ._lib import F_DEVICE, check, lib
from .hash import _check_extent, _is_dev, _layout

__all__ = ["chacha_batch", "xchacha_batch"]


def _dev_u8(t, n_per, count, name):
    if t is None:
        return None
    assert _is_dev(t) and t.dtype == torch.uint8 and t.is_contiguous(), name
    assert t.numel() >= n_per * count, name
    return t


def _crypt(x, key, src, dst, key_size, counters, ivs, rounds, offsets, lengths, count, stride,
           fixed_len, nbytes):
    key = bytes(key)
    if key_size is None:
        key_size = len(key)
    kbuf = (ctypes.c_uint8 * max(32, len(key))).from_buffer_copy(key.ljust(max(32, len(key)), b"\0"))
    ivl = 24 if x else 8
    L = lib()
    ref = src if src is not None else dst
    if ref is not None and _is_dev(ref):  # device mode
        dev = ref.device
        total = ref.numel()
        count, stride, fixed_len = _layout(count, offsets, lengths, stride, fixed_len, total)
        for t, dt in ((offsets, (torch.int64, torch.uint64)), (lengths, (torch.int32, torch.uint32))):
            if t is not None:
                assert _is_dev(t) and t.dtype in dt and t.is_contiguous() and t.device == dev
        if src is not None:
            assert src.dtype == torch.uint8 and src.is_contiguous()
        counters = _dev_u8(counters, 8, count, "counters")
        ivs = _dev_u8(ivs, ivl, count, "ivs")
        _check_extent(total, count, offsets, lengths, stride, fixed_len)
        if dst is None:
            dst = torch.zeros(max(total, 1), dtype=torch.uint8, device=dev)
        assert dst.dtype == torch.uint8 and dst.is_contiguous() and dst.device == dev
        _check_extent(dst.numel(), count, offsets, lengths, stride, fixed_len)
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev).cuda_stream
            check(L.lcb_chacha_batch(1 if x else 0, kbuf, key_size,
                                     counters.data_ptr() if counters is not None else None,
                                     ivs.data_ptr() if ivs is not None else None, rounds,
                                     src.data_ptr() if src is not None else None, dst.data_ptr(),
                                     offsets.data_ptr() if offsets is not None else None,
                                     lengths.data_ptr() if lengths is not None else None,
                                     count, stride, fixed_len, F_DEVICE, stream))
        return dst
    # host mode
    if src is not None:
        if isinstance(src, (bytes, bytearray, memoryview)):
            src = np.frombuffer(bytes(src), dtype=np.uint8)
        src = np.ascontiguousarray(src, dtype=np.uint8)
        total = src.size
    else:
        total = dst.size if dst is not None else int(nbytes)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    if lengths is not None:
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    count, stride, fixed_len = _layout(count, offsets, lengths, stride, fixed_len, total)
    _check_extent(total, count, offsets, lengths, stride, fixed_len)
    if dst is None:
        dst = np.zeros(max(total, 1), dtype=np.uint8)
    assert dst.dtype == np.uint8 and dst.flags.c_contiguous
    _check_extent(dst.size, count, offsets, lengths, stride, fixed_len)
    if counters is not None:
        counters = np.ascontiguousarray(np.frombuffer(bytes(counters), np.uint8)
                                        if isinstance(counters, (bytes, bytearray)) else counters, dtype=np.uint8)
    if ivs is not None:
        ivs = np.ascontiguousarray(np.frombuffer(bytes(ivs), np.uint8)
                                   if isinstance(ivs, (bytes, bytearray)) else ivs, dtype=np.uint8)
    assert counters is None or counters.size >= 8 * count, "counters"
    assert ivs is None or ivs.size >= ivl * count, "ivs"
    check(L.lcb_chacha_batch(1 if x else 0, kbuf, key_size,
                             counters.ctypes.data if counters is not None else None,
                             ivs.ctypes.data if ivs is not None else None, rounds,
                             src.ctypes.data if src is not None and src.size else None, dst.ctypes.data,
                             offsets.ctypes.data if offsets is not None else None,
                             lengths.ctypes.data if lengths is not None else None,
                             count, stride, fixed_len, 0, None))
    return dst


def chacha_batch(key, src=None, *, dst=None, key_size=None, counters=None, ivs=None, rounds=20,
                 offsets=None, lengths=None, count=None, stride=None, fixed_len=None, nbytes=None):
    """Batched chacha() (chacha.h:662).  key: 16/32 bytes (key_size defaults
    to len(key); 256/32 select a 256-bit key, anything else 128-bit);
    counters: 8 bytes per buffer (LE block counter), ivs: 8 bytes per buffer;
    src None -> keystream (give dst or nbytes).  Returns dst."""
    return _crypt(False, key, src, dst, key_size, counters, ivs, rounds, offsets, lengths, count, stride,
                  fixed_len, nbytes)


def xchacha_batch(key, src=None, *, dst=None, key_size=None, counters=None, ivs=None, rounds=20,
                  offsets=None, lengths=None, count=None, stride=None, fixed_len=None, nbytes=None):
    """Batched xchacha() (chacha.h:681): ivs are 24 bytes per buffer."""
    return _crypt(True, key, src, dst, key_size, counters, ivs, rounds, offsets, lengths, count, stride,
                  fixed_len, nbytes)
