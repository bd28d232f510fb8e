"""Python mirror of the asynchronous ingestion queue (include/lcb_hash_queue.h).

The reference hashes each received packet inside the thread-pool callback
(src/threadpool/threadpool_task.c:661-725 -> include/proto/radius.h:776-830).
HashQueue is the batching replacement: `submit` copies the packet into the
open page-locked batch and returns; the digest arrives later in `out` and/or
through `cb(error, digest_bytes)`, called on the library's completion thread
(the tpt_msg_send() delivery point, src/threadpool/threadpool_msg_sys.c:279).

All hashing happens in the HIP kernels of liblcb_hash_gpu.so; there is no
CPU path.
"""
import ctypes
import itertools
import threading

import numpy as np

from ._lib import (DIGEST_SIZE, DONE_CB, Q_F_NOWAIT, QueueSettings, QueueStats, Seg, c_vp, check,
                   lib)

__all__ = ["HashQueue"]


def _buf(x):
    """(address, size, keepalive) of a bytes-like / numpy uint8 packet."""
    if isinstance(x, np.ndarray):
        a = np.ascontiguousarray(x).view(np.uint8).reshape(-1)
        return a.ctypes.data, a.size, a
    b = bytes(x)
    if not b:
        return None, 0, b
    cb = ctypes.create_string_buffer(b, len(b))
    return ctypes.addressof(cb), len(b), cb


class HashQueue:
    """One digest algorithm (+ optional HMAC key) fed by any number of threads."""

    def __init__(self, alg, key=None, max_batch_msgs=65536, max_batch_bytes=16 << 20,
                 flush_usec=200, batches=4, align=16):
        L = lib()
        self.alg = alg
        self.D = DIGEST_SIZE[alg]
        s = QueueSettings(max_batch_msgs, max_batch_bytes, flush_usec, batches, align, 0)
        kp, kn, self._key = (None, 0, None) if key is None else _buf(key)
        if key is not None and kp is None:           # empty HMAC key: valid, non-NULL
            self._key = ctypes.create_string_buffer(1)
            kp = ctypes.addressof(self._key)
        q = c_vp()
        check(L.lcb_hash_queue_create(alg, kp, kn, ctypes.byref(s), ctypes.byref(q)))
        self._q = q
        self._lock = threading.Lock()
        self._ids = itertools.count(1)
        self._cbs = {}          # udata id -> python callable
        self._outs = []         # digest arrays kept alive until wait()
        self._trampoline = DONE_CB(self._on_done)

    def _on_done(self, udata, error, digest, size):
        with self._lock:
            fn = self._cbs.pop(udata, None)
        if fn is not None:
            fn(error, bytes(digest[:size]) if error == 0 else None)

    def _submit(self, segs, out, cb, nowait):
        L = lib()
        op = None
        if out is not None:
            if out.dtype != np.uint8 or out.size < self.D or not out.flags.c_contiguous:
                raise ValueError("out must be a contiguous uint8 array of >= %d bytes" % self.D)
            op = out.ctypes.data
        uid = 0
        if cb is not None:
            uid = next(self._ids)
            with self._lock:
                self._cbs[uid] = cb
        arr = (Seg * max(1, len(segs)))()
        keep = []
        for i, x in enumerate(segs):
            p, n, k = _buf(x)
            arr[i].data, arr[i].size = p, n
            keep.append(k)
        rc = L.lcb_hash_queue_submitv(self._q, arr, len(segs), op,
                                      self._trampoline if cb is not None else DONE_CB(),
                                      uid or None, Q_F_NOWAIT if nowait else 0)
        if rc != 0 and uid:
            with self._lock:
                self._cbs.pop(uid, None)
        check(rc)
        if out is not None:
            with self._lock:
                self._outs.append(out)

    def submit(self, data, out=None, cb=None, nowait=False):
        """Queue one packet.  `out` (uint8[D]) receives the digest; `cb(error,
        digest)` is called on the completion thread.  Both stay pending until
        completion (see wait())."""
        self._submit([data], out, cb, nowait)

    def submitv(self, segs, out=None, cb=None, nowait=False):
        """Queue one packet given as segments (hashed as their concatenation)."""
        self._submit(list(segs), out, cb, nowait)

    def flush(self):
        check(lib().lcb_hash_queue_flush(self._q))

    def wait(self):
        """Block until everything submitted so far completed."""
        rc = lib().lcb_hash_queue_wait(self._q)
        with self._lock:
            self._outs.clear()
        check(rc)

    def stats(self):
        st = QueueStats()
        check(lib().lcb_hash_queue_stats(self._q, ctypes.byref(st)))
        return {n: int(getattr(st, n)) for n, _ in QueueStats._fields_}

    def close(self):
        if self._q:
            lib().lcb_hash_queue_destroy(self._q)
            self._q = None
            self._outs.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
