"""ctypes binding of the in-tree C-ABI library liblcb_hash_gpu.so.

The library is the product: every digest computed through this package is
computed by its HIP kernels.  If the library is missing, or no MI355X is
visible, calls raise instead of falling back to anything on the CPU.

torch is imported first on purpose: torch ships its own libamdhip64 (soname
libamdhip64.so.7); loading it before our library makes both share ONE HIP
runtime, so torch tensors, streams and events interoperate with our kernels.
"""
import ctypes
import errno
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
# LCB_HASH_GPU_LIB selects an alternative build (tuning experiments only).
LIB_PATH = os.environ.get("LCB_HASH_GPU_LIB") or os.path.join(HERE, "liblcb_hash_gpu.so")

MD5, SHA1, SHA224, SHA256, SHA384, SHA512, GOST256, GOST512 = range(1, 9)
ALG_NAMES = {MD5: "md5", SHA1: "sha1", SHA224: "sha224", SHA256: "sha256",
             SHA384: "sha384", SHA512: "sha512", GOST256: "gost256", GOST512: "gost512"}
ALG_IDS = {v: k for k, v in ALG_NAMES.items()}
DIGEST_SIZE = {MD5: 16, SHA1: 20, SHA224: 28, SHA256: 32, SHA384: 48, SHA512: 64,
               GOST256: 32, GOST512: 64}
BLOCK_SIZE = {a: (128 if a in (SHA384, SHA512) else 64) for a in DIGEST_SIZE}
F_DEVICE = 0x1
F_COPY_PARTS = 0x100
KEY_HMAC, KEY_PREFIX, KEY_SUFFIX = 1, 2, 3

_lib = None

c_sz = ctypes.c_size_t
c_u64 = ctypes.c_uint64
c_u32 = ctypes.c_uint32
c_vp = ctypes.c_void_p

# (name, restype, argtypes) for every symbol include/lcb_hash_gpu.h declares.
_PLAIN = [c_vp, c_vp, c_vp, c_sz, c_u64, c_u32, c_vp, c_u32, c_vp]
_HMAC = [c_vp, c_sz] + _PLAIN
SIGNATURES = [
    ("lcb_hash_gpu_abi_version", ctypes.c_int, []),
    ("lcb_hash_digest_size", c_sz, [ctypes.c_int]),
    ("lcb_hash_block_size", c_sz, [ctypes.c_int]),
    ("lcb_hash_gpu_device_count", ctypes.c_int, []),
    ("lcb_hash_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("lcb_hash_batch", ctypes.c_int, [ctypes.c_int, c_vp, c_sz] + _PLAIN),
    ("md5_get_digest_batch", ctypes.c_int, _PLAIN),
    ("md5_hmac_get_digest_batch", ctypes.c_int, _HMAC),
    ("sha1_get_digest_batch", ctypes.c_int, _PLAIN),
    ("sha1_hmac_get_digest_batch", ctypes.c_int, _HMAC),
    ("sha2_get_digest_batch", ctypes.c_int,
     [c_sz, c_vp, c_vp, c_vp, c_sz, c_u64, c_u32, c_vp, c_vp, c_u32, c_vp]),
    ("sha2_hmac_get_digest_batch", ctypes.c_int,
     [c_sz, c_vp, c_sz, c_vp, c_vp, c_vp, c_sz, c_u64, c_u32, c_vp, c_vp, c_u32, c_vp]),
    ("gost3411_2012_get_digest_batch", ctypes.c_int,
     [c_sz, c_vp, c_vp, c_vp, c_sz, c_u64, c_u32, c_vp, c_vp, c_u32, c_vp]),
    ("gost3411_2012_hmac_get_digest_batch", ctypes.c_int,
     [c_sz, c_vp, c_sz, c_vp, c_vp, c_vp, c_sz, c_u64, c_u32, c_vp, c_vp, c_u32, c_vp]),
    ("lcb_hash_batch_keyed", ctypes.c_int,
     [ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp, c_sz, c_vp] + _PLAIN),
    ("lcb_hash_partition", ctypes.c_int, [c_vp, c_sz, c_u32, c_sz, c_vp]),
    ("lcb_hash_batch_multi", ctypes.c_int,
     [c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_sz, c_vp, c_vp, c_vp, c_sz, c_u64, c_u32, c_vp, c_u32, c_vp]),
    ("lcb_hash_multi_stats", ctypes.c_int, [c_vp]),
    ("lcb_hash_gen_synthetic", ctypes.c_int, [c_u64, c_u64, c_vp, c_sz, c_vp]),
    ("lcb_hash_gpu_gost_table", ctypes.c_int, [c_vp]),
    ("lcb_hash_gpu_read_probe", ctypes.c_int, [ctypes.c_int, c_vp, c_sz, c_u64, c_u32, c_vp, c_vp]),
    ("lcb_hash_gpu_probe_sink_words", c_sz, [ctypes.c_int, c_sz]),
    ("lcb_hash_gpu_clock_stamp", ctypes.c_int, [c_vp, c_sz, c_vp]),
    ("lcb_hash_key_cache_flush", ctypes.c_int, []),
    ("lcb_hash_key_cache_entries", c_sz, []),
    ("lcb_hash_gpu_seg_last", ctypes.c_int, [c_vp]),
]


_CRC = [c_vp, c_vp, c_vp, c_vp, c_sz, c_u64, c_u32, c_vp, c_u32, c_vp]
# every symbol include/lcb_crc32_gpu.h declares
CRC_SIGNATURES = [("lcb_crc32_batch", ctypes.c_int, [ctypes.c_int] + _CRC),
                  ("lcb_crc32_gpu_tables", ctypes.c_int, [ctypes.c_int, c_vp])] + [
    ("%s_batch" % n, ctypes.c_int, _CRC) for n in
    ("crc32a", "crc32cksum", "crc32mpeg2", "crc32b", "crc32jamcrc", "crc32c", "crc32d", "crc32q")]


_CHA = [c_vp, c_sz, c_vp, c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, c_sz, c_u64, c_u32, c_u32, c_vp]
# every symbol include/lcb_chacha_gpu.h declares
CHACHA_SIGNATURES = [("lcb_chacha_batch", ctypes.c_int, [ctypes.c_int] + _CHA),
                     ("chacha_batch", ctypes.c_int, _CHA),
                     ("xchacha_batch", ctypes.c_int, _CHA)]


class MultiStats(ctypes.Structure):
    """lcb_hash_multi_stats_t (include/lcb_hash_gpu.h)."""
    _fields_ = [(n, c_u64) for n in ("calls", "remote_parts", "parts_enqueued_before_wait", "peer_enabled",
                                     "peer_unavailable", "host_ns", "split_ns", "device_splits")]


class QueueSettings(ctypes.Structure):
    """lcb_hash_queue_settings_t (include/lcb_hash_queue.h)."""
    _fields_ = [("max_batch_msgs", c_sz), ("max_batch_bytes", c_sz), ("flush_usec", c_u32),
                ("batches", c_u32), ("align", c_u32), ("flags", c_u32)]


class QueueStats(ctypes.Structure):
    """lcb_hash_queue_stats_t."""
    _fields_ = [(n, c_u64) for n in ("packets", "bytes", "batches", "sealed_full", "sealed_timer",
                                     "sealed_flush", "max_batch_msgs", "submit_waits",
                                     "flusher_drain_ns", "flusher_launch_ns", "completer_busy_ns",
                                     "gpu_wait_ns", "max_fill_ns", "max_launch_ns", "max_gpu_ns",
                                     "max_callback_ns", "max_submit_wait_ns")] + [
        ("max_launch_steps_ns", c_u64 * 7)]


class Seg(ctypes.Structure):
    """lcb_hash_seg_t."""
    _fields_ = [("data", c_vp), ("size", c_sz)]


# void cb(void *udata, int error, const uint8_t *digest, size_t digest_size)
DONE_CB = ctypes.CFUNCTYPE(None, c_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint8), c_sz)
Q_F_NOWAIT = 0x1
Q_F_ZEROCOPY = 0x2

# every symbol include/lcb_hash_queue.h declares
QUEUE_SIGNATURES = [
    ("lcb_hash_queue_settings_def", None, [ctypes.POINTER(QueueSettings)]),
    ("lcb_hash_queue_create", ctypes.c_int,
     [ctypes.c_int, c_vp, c_sz, ctypes.POINTER(QueueSettings), ctypes.POINTER(c_vp)]),
    ("lcb_hash_queue_destroy", None, [c_vp]),
    ("lcb_hash_queue_submit", ctypes.c_int, [c_vp, c_vp, c_sz, c_vp, DONE_CB, c_vp, c_u32]),
    ("lcb_hash_queue_submitv", ctypes.c_int,
     [c_vp, ctypes.POINTER(Seg), c_sz, c_vp, DONE_CB, c_vp, c_u32]),
    ("lcb_hash_queue_register", ctypes.c_int, [c_vp, c_vp, c_sz]),
    ("lcb_hash_queue_flush", ctypes.c_int, [c_vp]),
    ("lcb_hash_queue_wait", ctypes.c_int, [c_vp]),
    ("lcb_hash_queue_stats", ctypes.c_int, [c_vp, ctypes.POINTER(QueueStats)]),
]


class LcbHashError(OSError):
    """A non-zero liblcb-style errno from the C-ABI."""


def lib():
    """The loaded library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("%s is missing: build it with `python -c 'import __graft_entry__ as g; "
                               "g.build()'` (or `make -C liblcb_amd`)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES + QUEUE_SIGNATURES + CRC_SIGNATURES + CHACHA_SIGNATURES:
            if os.environ.get("LCB_HASH_GPU_LIB") and not hasattr(L, name):
                continue  # an older experiment build: bind what it has
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().lcb_hash_strerror(rc).decode()
        raise LcbHashError(rc, "liblcb_hash_gpu: %s (%s)" % (msg, errno.errorcode.get(rc, rc)))
    return rc
