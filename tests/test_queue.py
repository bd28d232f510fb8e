"""Asynchronous ingestion queue (include/lcb_hash_queue.h).

CPU: settings defaults/validation and the loud ENODEV without a GPU.
GPU: digests delivered through `out` and callbacks equal the oracle's
one-shot digests for packets submitted from several threads, segment
submission (packet || secret, as radius.h:776-789 hashes it), HMAC queues
with short and long keys, the flush_usec timer, EMSGSIZE, empty packets.
"""
import errno
import threading
import time

import numpy as np
import pytest

from liblcb_amd._lib import (MD5, SHA1, SHA256, SHA512, GOST256, QueueSettings, c_vp, lib,
                             LcbHashError)

pytestmark = pytest.mark.timeout(300)   # a lost wake-up must fail, not hang the run


def test_settings_defaults():
    s = QueueSettings()
    lib().lcb_hash_queue_settings_def(s)
    assert (s.max_batch_msgs, s.max_batch_bytes, s.flush_usec, s.batches, s.align, s.flags) == \
        (65536, 16 << 20, 200, 4, 16, 0)


@pytest.mark.parametrize("field,value", [("max_batch_msgs", 0), ("max_batch_msgs", 1 << 23),
                                         ("max_batch_bytes", 0), ("batches", 1), ("batches", 17),
                                         ("align", 3), ("align", 8192), ("flags", 1)])
def test_settings_validation(field, value):
    import ctypes
    s = QueueSettings()
    lib().lcb_hash_queue_settings_def(s)
    setattr(s, field, value)
    q = c_vp()
    assert lib().lcb_hash_queue_create(MD5, None, 0, ctypes.byref(s), ctypes.byref(q)) == errno.EINVAL
    assert not q.value


def test_create_argument_errors():
    import ctypes
    q = c_vp()
    assert lib().lcb_hash_queue_create(0, None, 0, None, ctypes.byref(q)) == errno.EINVAL
    assert lib().lcb_hash_queue_create(MD5, None, 4, None, ctypes.byref(q)) == errno.EINVAL
    from liblcb_amd._lib import DONE_CB
    assert lib().lcb_hash_queue_submit(None, None, 0, None, DONE_CB(), None, 0) == errno.EINVAL


def test_queue_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from liblcb_amd.queue import HashQueue
    with pytest.raises(LcbHashError) as e:
        HashQueue(MD5)
    assert e.value.errno == errno.ENODEV


# ------------------------------------------------------------------ GPU
def _packets(seed, n, lo=0, hi=1500):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi, n)
    return [rng.integers(0, 256, int(k), dtype=np.uint8) for k in lens]


def _oracle_digests(oracle, alg, pkts, key=None):
    lens = np.array([p.size for p in pkts], np.uint32)
    offs = np.zeros(len(pkts), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = np.concatenate(pkts) if lens.sum() else np.zeros(1, np.uint8)
    return oracle.batch(alg, data, offs, lens, key=key)


@pytest.mark.gpu
@pytest.mark.parametrize("alg,key", [(MD5, None), (MD5, b"radius-shared-secret"), (SHA1, None),
                                     (SHA256, bytes(range(100))), (SHA512, None), (GOST256, None)])
def test_multithreaded_submit_out(gpu, oracle, alg, key):
    from liblcb_amd.queue import HashQueue
    from liblcb_amd._lib import DIGEST_SIZE
    pkts = _packets(alg * 7 + (len(key) if key else 0), 4000)
    want = _oracle_digests(oracle, alg, pkts, key)
    got = np.zeros((len(pkts), DIGEST_SIZE[alg]), np.uint8)
    # small batches so many batches (and slot reuse) happen
    with HashQueue(alg, key=key, max_batch_msgs=257, max_batch_bytes=1 << 20, batches=3) as q:
        def producer(t):
            for i in range(t, len(pkts), 4):
                q.submit(pkts[i], out=got[i])
        th = [threading.Thread(target=producer, args=(t,)) for t in range(4)]
        [x.start() for x in th]
        [x.join() for x in th]
        q.wait()
        st = q.stats()
    assert np.array_equal(got, want)
    assert st["packets"] == len(pkts)
    assert st["bytes"] == sum(p.size for p in pkts)
    assert st["batches"] >= len(pkts) // 257
    assert st["max_batch_msgs"] <= 257


@pytest.mark.gpu
def test_callbacks_and_segments(gpu, oracle):
    """submitv(packet, secret) == one-shot md5(packet || secret); callbacks
    deliver every digest exactly once."""
    from liblcb_amd.queue import HashQueue
    secret = b"testing123"
    pkts = _packets(11, 1000, 20, 4096)
    want = _oracle_digests(oracle, MD5, [np.concatenate([p, np.frombuffer(secret, np.uint8)])
                                         for p in pkts])
    got = {}
    lock = threading.Lock()

    def mk(i):
        def cb(err, dig):
            assert err == 0
            with lock:
                assert i not in got
                got[i] = dig
        return cb
    with HashQueue(MD5, max_batch_msgs=100) as q:
        for i, p in enumerate(pkts):
            q.submitv([p, secret], cb=mk(i))
        q.wait()
    assert len(got) == len(pkts)
    for i in range(len(pkts)):
        assert got[i] == want[i].tobytes()


@pytest.mark.gpu
def test_timer_flush(gpu, oracle):
    """A partly filled batch is sealed by flush_usec without flush()/wait()."""
    from liblcb_amd.queue import HashQueue
    done = threading.Event()
    res = []

    def cb(err, dig):
        res.append((err, dig))
        if len(res) == 3:
            done.set()
    with HashQueue(SHA256, flush_usec=2000) as q:
        for m in (b"", b"abc", b"x" * 1000):
            q.submit(m, cb=cb)
        assert done.wait(10.0), "timer did not seal the batch"
        st = q.stats()
    assert st["sealed_timer"] >= 1 and st["packets"] == 3
    want = _oracle_digests(oracle, SHA256, [np.frombuffer(m, np.uint8) for m in
                                            (b"", b"abc", b"x" * 1000)])
    assert [d for _, d in res] == [w.tobytes() for w in want]


@pytest.mark.gpu
def test_msgsize_and_empty(gpu, oracle):
    from liblcb_amd.queue import HashQueue
    with HashQueue(MD5, max_batch_bytes=4096) as q:
        with pytest.raises(LcbHashError) as e:
            q.submit(np.zeros(4097, np.uint8))
        assert e.value.errno == errno.EMSGSIZE
        out = np.zeros(16, np.uint8)
        q.submit(b"", out=out)
        big = np.full(4096, 7, np.uint8)
        out2 = np.zeros(16, np.uint8)
        q.submit(big, out=out2)
        q.wait()
    assert out.tobytes() == bytes.fromhex("d41d8cd98f00b204e9800998ecf8427e")
    assert out2.tobytes() == _oracle_digests(oracle, MD5, [big])[0].tobytes()


@pytest.mark.gpu
def test_full_batches_and_slot_pressure(gpu, oracle):
    """Tiny batches + 2 slots: producers must wait for slots; nothing is lost."""
    from liblcb_amd.queue import HashQueue
    pkts = _packets(5, 3000, 0, 300)
    want = _oracle_digests(oracle, MD5, pkts)
    got = np.zeros((len(pkts), 16), np.uint8)
    t0 = time.time()
    with HashQueue(MD5, max_batch_msgs=8, batches=2, align=1) as q:
        for i, p in enumerate(pkts):
            q.submit(p, out=got[i])
        q.wait()
        st = q.stats()
    assert np.array_equal(got, want)
    assert st["sealed_full"] >= len(pkts) // 8 - 2
    assert time.time() - t0 < 60


@pytest.mark.gpu
@pytest.mark.parametrize("alg,key", [(MD5, ""), (MD5, "00112233445566778899aabbccddeeff")])
def test_native_producers(gpu, oracle, tmp_path, alg, key):
    """tools/queue_bench: 8 native producer threads, 64K x 1 KiB packets of the
    §8d synthetic stream, digests == oracle."""
    import json
    import os
    import subprocess
    from oracle.pyoracle import SEED, gen_stream
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "queue_bench")
    n, size = 1 << 16, 1024
    out = tmp_path / "dig.bin"
    cmd = [exe, "--alg", str(alg), "--packets", str(n), "--size", str(size), "--threads", "8",
           "--batch-msgs", "4096", "--out", str(out)] + (["--key", key] if key else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["packets"] == n and res["batches"] >= n // 4096
    got = np.fromfile(out, np.uint8).reshape(n, 16)
    want = oracle.batch_fixed_mt(alg, gen_stream(SEED, n * size), n, size, size,
                                 key=bytes.fromhex(key) if key else None)
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_native_producers_repeated(gpu, oracle, tmp_path):
    """Regression: 4 slots of 4096-packet batches run concurrently on four
    streams, each bucketed through its own scratch.  With the default
    stream-ordered pool a live bucketing buffer could be handed to a second
    batch on another stream, and 1-3 runs in 20 delivered whole batches of
    another packet's digests; six runs in a row must all be exact."""
    import json
    import os
    import subprocess
    from oracle.pyoracle import SEED, gen_stream
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "queue_bench")
    n, size = 1 << 16, 1024
    want = oracle.batch_fixed_mt(MD5, gen_stream(SEED, n * size), n, size, size)
    out = tmp_path / "dig.bin"
    for it in range(6):
        r = subprocess.run([exe, "--alg", str(MD5), "--packets", str(n), "--size", str(size), "--threads", "8",
                            "--batch-msgs", "4096", "--out", str(out)], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        got = np.fromfile(out, np.uint8).reshape(n, 16)
        bad = np.nonzero((got != want).any(1))[0]
        assert len(bad) == 0, (it, len(bad), bad[:8])


@pytest.mark.gpu
def test_concurrent_ragged_batches_on_streams(gpu, oracle):
    """Device-mode ragged batches (bucketed: >= 4096 messages) launched on four
    streams at once, repeatedly: each batch's scratch stays its own."""
    import torch
    rng = np.random.default_rng(77)
    jobs = []
    for k in range(4):
        n = 6000 + 1000 * k
        lens = rng.integers(0, 1500, n).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        from oracle.pyoracle import gen_stream
        data = gen_stream(100 + k, int(lens.sum()) + 8)
        jobs.append((data, offs, lens, oracle.batch(MD5, data, offs, lens)))
    dev = [(torch.as_tensor(d, device="cuda"), torch.as_tensor(o.astype(np.int64), device="cuda"),
            torch.as_tensor(l.astype(np.int32), device="cuda")) for d, o, l, _ in jobs]
    streams = [torch.cuda.Stream() for _ in jobs]
    for rep in range(10):
        outs = []
        for (dd, do, dl), st in zip(dev, streams):
            with torch.cuda.stream(st):
                outs.append(gpu.hash_batch(MD5, dd, offsets=do, lengths=dl))
        torch.cuda.synchronize()
        for (_, _, _, exp), got in zip(jobs, outs):
            assert np.array_equal(got.cpu().numpy(), exp), rep


@pytest.mark.gpu
def test_stale_lease_across_generations(gpu, oracle):
    """One producer goes idle holding a lease while the others cycle the slots
    through many generations (2 slots, 16-message batches); when it wakes its
    stale lease must neither be written nor disturb the busy count of the
    record's current owner (lease records are reused every generation)."""
    from liblcb_amd.queue import HashQueue
    pkts = _packets(23, 6000, 0, 400)
    want = _oracle_digests(oracle, MD5, pkts)
    got = np.zeros((len(pkts), 16), np.uint8)
    with HashQueue(MD5, max_batch_msgs=64, batches=2, align=1) as q:
        def sleeper():
            for i in range(0, 600, 3):
                q.submit(pkts[i], out=got[i])
                time.sleep(0.002)     # idle while the others reopen the slots
        def busy(t):
            for i in range(600 + t, len(pkts), 2):
                q.submit(pkts[i], out=got[i])
            for i in range(1 + t, 600, 3):
                q.submit(pkts[i], out=got[i])
        th = [threading.Thread(target=sleeper)] + [threading.Thread(target=busy, args=(t,)) for t in range(2)]
        [x.start() for x in th]
        [x.join() for x in th]
        q.wait()
        st = q.stats()
    assert np.array_equal(got, want)
    assert st["packets"] == len(pkts) and st["batches"] > 50


# ------------------------------------------------------------ zero copy
@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["scattered", "ring"])
@pytest.mark.parametrize("alg,key", [(MD5, None), (MD5, b"radius-shared-secret"), (SHA256, None)])
def test_zerocopy_submit(gpu, oracle, alg, key, layout):
    """LCB_HASH_Q_F_ZEROCOPY: packets at byte offsets inside a registered
    pinned area (mixed with copied submits), from several threads, over many
    batches; digests == oracle.  "scattered": random offsets over 8 MiB, so a
    batch's packets are sparse in their span and the kernel reads them in
    host memory; "ring": packets back to back as in a receive ring, so a
    batch's span moves with one H2D copy (lcb_hash_queue.cpp launch)."""
    import torch
    from liblcb_amd.queue import HashQueue
    from liblcb_amd._lib import DIGEST_SIZE
    rng = np.random.default_rng(31 + alg)
    area_t = torch.empty(8 << 20, dtype=torch.uint8, pin_memory=True)
    area = area_t.numpy()
    area[:] = rng.integers(0, 256, area.size, dtype=np.uint8)
    n = 6000
    lens = rng.integers(0, 1600, n)
    if layout == "scattered":
        offs = rng.integers(0, area.size - 1600, n)
        lens[:4] = (0, 1, 64, 1599)
        offs[:4] = (0, area.size - 1, area.size - 64, area.size - 1599)   # ends exactly at the area's end
    else:
        offs = np.zeros(n, np.int64)
        offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 3, n - 1))
        offs += area.size - int(offs[-1] + lens[-1])                      # the last ends at the area's end
    pkts = [area[o:o + l] for o, l in zip(offs, lens)]
    want = _oracle_digests(oracle, alg, [p.copy() for p in pkts], key)
    got = np.zeros((n, DIGEST_SIZE[alg]), np.uint8)
    with HashQueue(alg, key=key, max_batch_msgs=500, max_batch_bytes=1 << 20, batches=3) as q:
        q.register(area_t)
        def producer(t):
            for i in range(t, n, 4):
                q.submit(pkts[i], out=got[i], zerocopy=(i % 5 != 0))
        th = [threading.Thread(target=producer, args=(t,)) for t in range(4)]
        [x.start() for x in th]
        [x.join() for x in th]
        q.wait()
        st = q.stats()
    assert np.array_equal(got, want)
    assert st["packets"] == n and st["batches"] >= n // 500


@pytest.mark.gpu
def test_zerocopy_errors(gpu):
    """EINVAL: zero-copy packet outside every registered area, zero copy with
    two segments, registering pageable memory; ENOMEM past 16 areas."""
    import torch
    from liblcb_amd.queue import HashQueue
    pinned = torch.empty(1 << 16, dtype=torch.uint8, pin_memory=True)
    with HashQueue(MD5) as q:
        with pytest.raises(LcbHashError) as e:
            q.submit(np.zeros(100, np.uint8), zerocopy=True)      # not registered
        assert e.value.errno == errno.EINVAL
        with pytest.raises(LcbHashError) as e:
            q.register(np.zeros(4096, np.uint8))                  # pageable
        assert e.value.errno == errno.EINVAL
        q.register(pinned)
        a = pinned.numpy()
        with pytest.raises(LcbHashError) as e:
            q.submit(np.zeros(10, np.uint8), zerocopy=True)       # still outside
        assert e.value.errno == errno.EINVAL
        from liblcb_amd._lib import DONE_CB, Q_F_ZEROCOPY, Seg
        segs = (Seg * 2)()
        segs[0].data, segs[0].size = a.ctypes.data, 10
        segs[1].data, segs[1].size = a.ctypes.data + 10, 10
        assert lib().lcb_hash_queue_submitv(q._q, segs, 2, None, DONE_CB(), None, Q_F_ZEROCOPY) == errno.EINVAL
        # the area itself works; a packet running past its end does not
        out = np.zeros(16, np.uint8)
        a[:3] = np.frombuffer(b"abc", np.uint8)
        q.submit(a[:3], out=out, zerocopy=True)
        q.wait()
        assert out.tobytes().hex() == "900150983cd24fb0d6963f7d28e17f72"
        assert lib().lcb_hash_queue_submit(q._q, a.ctypes.data + a.size - 8, 16, None, DONE_CB(), None,
                                           Q_F_ZEROCOPY) == errno.EINVAL
        more = [torch.empty(4096, dtype=torch.uint8, pin_memory=True) for _ in range(15)]
        for m in more:
            q.register(m)
        with pytest.raises(LcbHashError) as e:
            q.register(torch.empty(4096, dtype=torch.uint8, pin_memory=True))
        assert e.value.errno == errno.ENOMEM


@pytest.mark.gpu
def test_native_producers_zerocopy(gpu, oracle, tmp_path):
    """tools/queue_bench --zerocopy 1: 8 native producers submit 64K x 1 KiB
    packets of a registered pinned pool in place; digests == oracle."""
    import json
    import os
    import subprocess
    from oracle.pyoracle import SEED, gen_stream
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "queue_bench")
    n, size = 1 << 16, 1024
    out = tmp_path / "dig.bin"
    r = subprocess.run([exe, "--alg", str(MD5), "--packets", str(n), "--size", str(size), "--threads", "8",
                        "--batch-msgs", "4096", "--zerocopy", "1", "--out", str(out)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["zerocopy"] == 1 and res["packets"] == n
    got = np.fromfile(out, np.uint8).reshape(n, 16)
    want = oracle.batch_fixed_mt(MD5, gen_stream(SEED, n * size), n, size, size)
    assert np.array_equal(got, want)
