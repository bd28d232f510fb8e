"""Python mirror of the asynchronous ingestion queue (include/lcb_hash_queue.h).

The reference hashes each received packet inside the thread-pool callback
(src/threadpool/threadpool_task.c:661-725 -> include/proto/radius.h:776-830).
HashQueue is the batching replacement: `submit` copies the packet into the
open page-locked batch and returns; the digest arrives later in `out` and/or
through `cb(error, digest_bytes)`, called on the library's completion thread
(the tpt_msg_send() delivery point, src/threadpool/threadpool_msg_sys.c:279).
Zero copy: `register` a page-locked receive area (e.g. a pinned torch tensor's
numpy view) and `submit(..., zerocopy=True)` packets lying in it -- the queue
records where they are and the kernel reads them in place.

All hashing happens in the HIP kernels of liblcb_hash_gpu.so; there is no
CPU path.
"""
import ctypes
import itertools
import threading

import numpy as np

from ._lib import (DIGEST_SIZE, DONE_CB, Q_F_NOWAIT, Q_F_ZEROCOPY, QueueSettings, QueueStats, Seg, c_vp,
                   check, lib)

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
        self._outs = []         # digest arrays (and zero-copy packets) kept alive until wait()
        self._regions = []      # registered page-locked areas
        self._trampoline = DONE_CB(self._on_done)

    def _on_done(self, udata, error, digest, size):
        with self._lock:
            fn = self._cbs.pop(udata, None)
        if fn is not None:
            fn(error, bytes(digest[:size]) if error == 0 else None)

    def register(self, area):
        """Register a page-locked uint8 area (numpy view of pinned memory, or
        a pinned CPU torch tensor) as a zero-copy packet source."""
        if hasattr(area, "data_ptr"):
            if not area.is_pinned():
                raise ValueError("torch tensor must be pinned")
            if not area.is_contiguous():
                raise ValueError("area must be contiguous")   # else numel*size is not its byte extent
            p, n = area.data_ptr(), area.numel() * area.element_size()
        else:
            a = np.asarray(area)
            if not a.flags.c_contiguous:
                raise ValueError("area must be contiguous")
            p, n = a.ctypes.data, a.nbytes
        check(lib().lcb_hash_queue_register(self._q, p, n))
        self._regions.append(area)

    def _submit(self, segs, out, cb, nowait, zerocopy=False):
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
            if zerocopy and not (isinstance(x, np.ndarray) and x.flags.c_contiguous):
                raise ValueError("a zero-copy packet is a contiguous numpy view of a registered area")
            p, n, k = _buf(x)
            arr[i].data, arr[i].size = p, n
            keep.append(k)
        flags = (Q_F_NOWAIT if nowait else 0) | (Q_F_ZEROCOPY if zerocopy else 0)
        rc = L.lcb_hash_queue_submitv(self._q, arr, len(segs), op,
                                      self._trampoline if cb is not None else DONE_CB(),
                                      uid or None, flags)
        if rc != 0 and uid:
            with self._lock:
                self._cbs.pop(uid, None)
        check(rc)
        if out is not None or zerocopy:
            with self._lock:
                if out is not None:
                    self._outs.append(out)
                if zerocopy:
                    self._outs.append(keep)

    def submit(self, data, out=None, cb=None, nowait=False, zerocopy=False):
        """Queue one packet.  `out` (uint8[D]) receives the digest; `cb(error,
        digest)` is called on the completion thread.  Both stay pending until
        completion (see wait()).  zerocopy: `data` lies in a registered area
        and must stay unchanged until completion (LCB_HASH_Q_F_ZEROCOPY)."""
        self._submit([data], out, cb, nowait, zerocopy)

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
        def val(v):
            return [int(x) for x in v] if isinstance(v, ctypes.Array) else int(v)
        return {n: val(getattr(st, n)) for n, _ in QueueStats._fields_}

    def close(self):
        if self._q:
            lib().lcb_hash_queue_destroy(self._q)
            self._q = None
            self._outs.clear()
            self._regions.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
