"""Host-side mirror of liblcb's include/crypto/hash one-shot API, batched.

Each function below is the batch counterpart of the reference function named
in its docstring and returns, per message, exactly the bytes that function
writes.  Arguments keep the reference's meaning (`bits` as sha2_init /
gost3411_2012_init, `key`/`key_size` as the *_hmac_* functions); the batch
adds the buffer description of include/lcb_hash_gpu.h.

Memory modes
  * torch CUDA (ROCm) tensors -> device mode: the kernels run on the tensor's
    device, enqueued on torch's current stream; the call does not synchronise.
  * numpy arrays / bytes      -> host mode: pinned staging, H2D, kernel, D2H.

Errors raise LcbHashError (liblcb errno codes).  There is no CPU fallback.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import (ALG_IDS, DIGEST_SIZE, F_COPY_PARTS, F_DEVICE, GOST256, KEY_HMAC, KEY_PREFIX, KEY_SUFFIX, GOST512, MD5, SHA1, SHA224,
                   SHA256, SHA384, SHA512, check, lib)

__all__ = [
    "hash_batch", "md5_get_digest_batch", "md5_hmac_get_digest_batch",
    "sha1_get_digest_batch", "sha1_hmac_get_digest_batch", "sha2_get_digest_batch",
    "sha2_hmac_get_digest_batch", "gost3411_2012_get_digest_batch",
    "gost3411_2012_hmac_get_digest_batch", "gen_synthetic", "sha2_alg", "gost_alg",
    "partition", "hash_batch_multi", "multi_stats", "hash_batch_keyed", "KEY_HMAC", "KEY_PREFIX", "KEY_SUFFIX",
]


def sha2_alg(bits):
    """sha2_init's bits-or-bytes convention (sha2.h:217-241); None if invalid."""
    return {224: SHA224, 28: SHA224, 256: SHA256, 32: SHA256,
            384: SHA384, 48: SHA384, 512: SHA512, 64: SHA512}.get(int(bits))


def gost_alg(bits):
    """gost3411_2012_init (gost3411-2012.h:1715-1729): 256/32 -> 256, else 512."""
    return GOST256 if int(bits) in (256, 32) else GOST512


def _is_dev(t):
    return isinstance(t, torch.Tensor) and t.is_cuda


def _layout(count, offsets, lengths, stride, fixed_len, nbytes):
    if count is None:
        if lengths is not None:
            count = int(lengths.shape[0])
        elif offsets is not None:
            count = int(offsets.shape[0])
        elif stride:
            count = nbytes // int(stride)
        else:
            raise ValueError("count is required for a fixed-length batch without stride")
    if lengths is None and fixed_len is None:
        fixed_len = int(stride or 0)
    return int(count), int(stride or 0), int(fixed_len or 0)


def _check_extent(nbytes, count, offsets, lengths, stride, fixed_len):
    """Every described message must lie inside the `nbytes` of `data`: the
    C-ABI trusts the description (out-of-range host reads would leak or
    crash; out-of-range device reads fault the GPU).  Works on numpy arrays
    and on device tensors (one reduction, one synchronisation)."""
    if count == 0:
        return
    for name, t in (("offsets", offsets), ("lengths", lengths)):
        if t is not None and int(t.shape[0]) < count:
            raise ValueError("%s has %d entries, count is %d" % (name, int(t.shape[0]), count))
    if offsets is None and lengths is None:
        end = (count - 1) * stride + fixed_len
    elif isinstance(offsets if offsets is not None else lengths, torch.Tensor):
        o = offsets[:count].to(torch.int64) if offsets is not None else \
            torch.arange(count, dtype=torch.int64, device=lengths.device) * stride
        n = lengths[:count].to(torch.int64) & 0xFFFFFFFF if lengths is not None else fixed_len
        end = int((o + n).max().item())
        if int(o.min().item()) < 0:
            raise ValueError("negative offset")
    else:
        o = offsets[:count].astype(np.uint64) if offsets is not None else \
            np.arange(count, dtype=np.uint64) * np.uint64(stride)
        n = lengths[:count].astype(np.uint64) if lengths is not None else np.uint64(fixed_len)
        end = int((o + n).max())
    if end > nbytes:
        raise ValueError("messages extend to byte %d of a %d-byte buffer" % (end, nbytes))


def _dev_batch(data, count, offsets, lengths, stride, fixed_len, out, D, per_msg=()):
    """Validate a device-mode batch description and return (count, stride,
    fixed_len, out): data uint8 and contiguous; offsets int64/uint64 and
    lengths int32/uint32 (the C-ABI reads them as uint64 / uint32), per-message
    uint32 arrays (`per_msg`: (name, tensor) pairs, e.g. key_index) int32 /
    uint32, all contiguous, on data's device and with >= count entries;
    `out` (allocated if None) uint8, contiguous, on data's device, >= count x D
    bytes; every message inside data (_check_extent)."""
    if data.dtype != torch.uint8 or not data.is_contiguous():
        raise TypeError("data must be a contiguous uint8 tensor")
    count, stride, fixed_len = _layout(count, offsets, lengths, stride, fixed_len, data.numel())
    for name, t, dts in (("offsets", offsets, (torch.int64, torch.uint64)),
                         ("lengths", lengths, (torch.int32, torch.uint32))) + \
            tuple((n, t, (torch.int32, torch.uint32)) for n, t in per_msg):
        if t is None:
            continue
        if not _is_dev(t) or t.device != data.device:
            raise ValueError("%s must be a tensor on %s" % (name, data.device))
        if t.dtype not in dts or not t.is_contiguous():
            raise TypeError("%s must be a contiguous %s tensor" % (name, " / ".join(str(d) for d in dts)))
        if int(t.numel()) < count:
            raise ValueError("%s has %d entries, count is %d" % (name, int(t.numel()), count))
    _check_extent(data.numel(), count, offsets, lengths, stride, fixed_len)
    if out is None:
        out = torch.empty((count, D), dtype=torch.uint8, device=data.device)
    elif not _is_dev(out) or out.device != data.device or out.dtype != torch.uint8 or not out.is_contiguous():
        raise TypeError("out must be a contiguous uint8 tensor on %s" % data.device)
    if int(out.numel()) < count * D:
        raise ValueError("out holds %d bytes, %d x %d needed" % (int(out.numel()), count, D))
    return count, stride, fixed_len, out


def _host_batch(data, count, offsets, lengths, stride, fixed_len, out, D, per_msg=()):
    """Host-mode counterpart of _dev_batch: -> (data, offsets, lengths,
    per_msg arrays, count, stride, fixed_len, out, nbytes) as contiguous
    numpy arrays of the dtypes the C-ABI reads."""
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
    count, stride, fixed_len = _layout(count, offsets, lengths, stride, fixed_len, data.size)
    arrs = []
    for name, t in per_msg:
        if t is not None:
            t = np.ascontiguousarray(t, dtype=np.uint32)
            if t.size < count:
                raise ValueError("%s has %d entries, count is %d" % (name, t.size, count))
        arrs.append(t)
    _check_extent(nbytes, count, offsets, lengths, stride, fixed_len)
    if out is None:
        out = np.empty((count, D), dtype=np.uint8)
    elif not isinstance(out, np.ndarray) or out.dtype != np.uint8 or not out.flags.c_contiguous:
        raise TypeError("out must be a C-contiguous uint8 numpy array")
    if out.size < count * D:
        raise ValueError("out holds %d bytes, %d x %d needed" % (out.size, count, D))
    return data, offsets, lengths, arrs, count, stride, fixed_len, out, nbytes


def hash_batch(alg, data, *, offsets=None, lengths=None, count=None, stride=None,
               fixed_len=None, key=None, out=None):
    """Digest (or HMAC when `key` is given) of every message of a batch.

    data     uint8 torch CUDA tensor (device mode) or numpy uint8 / bytes (host)
    offsets  int64/uint64 per-message start offsets, or None (i * stride)
    lengths  int32/uint32 per-message lengths, or None (fixed_len)
    returns  packed digests, shape (count, D), same kind of memory as `data`
    """
    if isinstance(alg, str):
        alg = ALG_IDS[alg]
    if alg not in DIGEST_SIZE:
        raise _lib.LcbHashError(22, "liblcb_hash_gpu: invalid argument (unknown alg)")
    D = DIGEST_SIZE[alg]
    kb = None if key is None else bytes(key)
    kptr = ctypes.c_char_p(kb) if kb is not None else None
    klen = len(kb) if kb is not None else 0
    L = lib()
    if _is_dev(data):
        count, stride, fixed_len, out = _dev_batch(data, count, offsets, lengths, stride, fixed_len, out, D)
        with torch.cuda.device(data.device):
            stream = torch.cuda.current_stream(data.device).cuda_stream
            check(L.lcb_hash_batch(alg, kptr, klen, data.data_ptr(),
                                   offsets.data_ptr() if offsets is not None else None,
                                   lengths.data_ptr() if lengths is not None else None,
                                   count, stride, fixed_len, out.data_ptr(), F_DEVICE, stream))
        return out
    data, offsets, lengths, _, count, stride, fixed_len, out, _ = _host_batch(
        data, count, offsets, lengths, stride, fixed_len, out, D)
    check(L.lcb_hash_batch(alg, kptr, klen, data.ctypes.data,
                           offsets.ctypes.data if offsets is not None else None,
                           lengths.ctypes.data if lengths is not None else None,
                           count, stride, fixed_len, out.ctypes.data, 0, None))
    return out


# ----------------------------------------------- reference-named wrappers
def md5_get_digest_batch(data, **kw):
    """Batch md5_get_digest (md5.h:396-402)."""
    return hash_batch(MD5, data, **kw)


def md5_hmac_get_digest_batch(key, data, **kw):
    """Batch md5_hmac_get_digest (md5.h:419-425)."""
    return hash_batch(MD5, data, key=key, **kw)


def sha1_get_digest_batch(data, **kw):
    """Batch sha1_get_digest (sha1.h:946-954)."""
    return hash_batch(SHA1, data, **kw)


def sha1_hmac_get_digest_batch(key, data, **kw):
    """Batch sha1_hmac_get_digest (sha1.h:969-975)."""
    return hash_batch(SHA1, data, key=key, **kw)


def _sha2(bits):
    alg = sha2_alg(bits)
    if alg is None:  # sha2_init leaves an unknown size undefined; we refuse it
        raise _lib.LcbHashError(22, "liblcb_hash_gpu: invalid argument (sha2 bits %r)" % (bits,))
    return alg


def sha2_get_digest_batch(bits, data, **kw):
    """Batch sha2_get_digest (sha2.h:854-865); bits as sha2_init."""
    return hash_batch(_sha2(bits), data, **kw)


def sha2_hmac_get_digest_batch(bits, key, data, **kw):
    """Batch sha2_hmac_get_digest (sha2.h:887-894)."""
    return hash_batch(_sha2(bits), data, key=key, **kw)


def gost3411_2012_get_digest_batch(bits, data, **kw):
    """Batch gost3411_2012_get_digest (gost3411-2012.h:1962-1973)."""
    return hash_batch(gost_alg(bits), data, **kw)


def gost3411_2012_hmac_get_digest_batch(bits, key, data, **kw):
    """Batch gost3411_2012_hmac_get_digest (gost3411-2012.h:1996-2004)."""
    return hash_batch(gost_alg(bits), data, key=key, **kw)


def gen_synthetic(seed, nbytes, start=0, device="cuda", out=None):
    """Device tensor holding bytes [start, start+nbytes) of the synthetic stream
    (u64 word k = mix64(seed ^ k), little-endian)."""
    if out is None:
        out = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
    with torch.cuda.device(out.device):
        stream = torch.cuda.current_stream(out.device).cuda_stream
        check(lib().lcb_hash_gen_synthetic(seed, start, out.data_ptr(), int(nbytes), stream))
    return out[:int(nbytes)]


def partition(nparts, *, lengths=None, count=None, fixed_len=0):
    """lcb_hash_partition: contiguous message ranges of balanced work
    (bytes + one 64-B padding block per message) -> uint64 array `first` of
    nparts + 1 entries; part p = messages [first[p], first[p+1])."""
    if lengths is not None:
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        count = int(lengths.size) if count is None else int(count)
        assert lengths.size >= count
    first = np.zeros(int(nparts) + 1, np.uint64)
    check(lib().lcb_hash_partition(lengths.ctypes.data if lengths is not None else None, int(count),
                                   int(fixed_len), int(nparts), first.ctypes.data))
    return first


def hash_batch_multi(devs, alg, data, *, offsets=None, lengths=None, count=None, stride=None,
                     fixed_len=None, key=None, out=None, copy_parts=False):
    """lcb_hash_batch_multi: the batch split by `partition` over the HIP
    devices `devs` (repeats allowed) and hashed on all of them at once.
    Device tensors must live on devs[0]; the call is ordered after torch's
    current stream on devs[0] (passed as the ABI's `stream`).  numpy input
    runs in host mode."""
    if isinstance(alg, str):
        alg = ALG_IDS[alg]
    D = DIGEST_SIZE[alg]
    kb = None if key is None else bytes(key)
    kptr = ctypes.c_char_p(kb) if kb is not None else None
    klen = len(kb) if kb is not None else 0
    dv = (ctypes.c_int * len(devs))(*devs)
    if _is_dev(data):
        if data.device.index != devs[0]:
            raise ValueError("device tensors must live on devs[0] = %d" % devs[0])
        count, stride, fixed_len, out = _dev_batch(data, count, offsets, lengths, stride, fixed_len, out, D)
        stream = torch.cuda.current_stream(data.device).cuda_stream
        check(lib().lcb_hash_batch_multi(dv, len(devs), alg, kptr, klen, data.data_ptr(),
                                         offsets.data_ptr() if offsets is not None else None,
                                         lengths.data_ptr() if lengths is not None else None,
                                         count, stride, fixed_len, out.data_ptr(),
                                         F_DEVICE | (F_COPY_PARTS if copy_parts else 0), stream))
        return out
    if copy_parts:
        raise ValueError("copy_parts is a device-mode option")
    data, offsets, lengths, _, count, stride, fixed_len, out, _ = _host_batch(
        data, count, offsets, lengths, stride, fixed_len, out, D)
    check(lib().lcb_hash_batch_multi(dv, len(devs), alg, kptr, klen, data.ctypes.data,
                                     offsets.ctypes.data if offsets is not None else None,
                                     lengths.ctypes.data if lengths is not None else None,
                                     count, stride, fixed_len, out.ctypes.data, 0, None))
    return out


def multi_stats():
    """lcb_hash_multi_stats as a dict: device-mode lcb_hash_batch_multi calls,
    remote parts, remote parts fully enqueued before the call's first wait,
    device pairs with peer access enabled / unavailable."""
    from ._lib import MultiStats
    st = MultiStats()
    check(lib().lcb_hash_multi_stats(ctypes.byref(st)))
    return {n: int(getattr(st, n)) for n, _ in MultiStats._fields_}


def hash_batch_keyed(alg, mode, keys, data, *, key_index=None, offsets=None, lengths=None, count=None,
                     stride=None, fixed_len=None, out=None):
    """lcb_hash_batch_keyed: message i hashed with key keys[key_index[i]]
    (key 0 without key_index) as HMAC(K, m) (KEY_HMAC), H(K || m)
    (KEY_PREFIX) or H(m || K) (KEY_SUFFIX) — the RADIUS shapes
    (include/proto/radius.h:745-919, 1315-1377).  keys: sequence of bytes.
    key_index lives with the batch: a device tensor in device mode."""
    if isinstance(alg, str):
        alg = ALG_IDS[alg]
    D = DIGEST_SIZE[alg]
    keys = [bytes(k) for k in keys]
    blob = np.frombuffer(b"".join(keys) or b"\0", np.uint8)
    klen = np.array([len(k) for k in keys], np.uint32)
    koff = np.zeros(len(keys), np.uint64)
    if len(keys) > 1:
        koff[1:] = np.cumsum(klen[:-1], dtype=np.uint64)
    L = lib()
    if _is_dev(data):
        count, stride, fixed_len, out = _dev_batch(data, count, offsets, lengths, stride, fixed_len, out, D,
                                                   per_msg=(("key_index", key_index),))
        with torch.cuda.device(data.device):
            stream = torch.cuda.current_stream(data.device).cuda_stream
            check(L.lcb_hash_batch_keyed(alg, mode, blob.ctypes.data, koff.ctypes.data, klen.ctypes.data,
                                         len(keys), key_index.data_ptr() if key_index is not None else None,
                                         data.data_ptr(), offsets.data_ptr() if offsets is not None else None,
                                         lengths.data_ptr() if lengths is not None else None,
                                         count, stride, fixed_len, out.data_ptr(), F_DEVICE, stream))
        return out
    data, offsets, lengths, (key_index,), count, stride, fixed_len, out, _ = _host_batch(
        data, count, offsets, lengths, stride, fixed_len, out, D, per_msg=(("key_index", key_index),))
    check(L.lcb_hash_batch_keyed(alg, mode, blob.ctypes.data, koff.ctypes.data, klen.ctypes.data, len(keys),
                                 key_index.ctypes.data if key_index is not None else None, data.ctypes.data,
                                 offsets.ctypes.data if offsets is not None else None,
                                 lengths.ctypes.data if lengths is not None else None,
                                 count, stride, fixed_len, out.ctypes.data, 0, None))
    return out
