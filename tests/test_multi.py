"""Multi-device batches (include/lcb_hash_gpu.h: lcb_hash_partition,
lcb_hash_batch_multi).

CPU: the work-balanced split (bytes + one padding block per message) on the
C4 length mix keeps every part within 1 % of the mean; fixed lengths split
into equal counts; degenerate shapes.  GPU (one MI355X on the box): the
multi-device call with devs = {0} equals lcb_hash_batch; devs = {0, 0, 0}
runs three concurrent parts on one device (host mode: three staging
pipelines; device mode: in place, and through the peer-copy scatter/gather
path forced by LCB_HASH_F_COPY_PARTS), all checked against the oracle.
"""
import numpy as np
import pytest

from oracle.pyoracle import gen_stream
from tests.golden_util import SEED, mixed_lengths_np


def _lcb():
    import liblcb_amd
    try:
        liblcb_amd.lib()
    except RuntimeError as e:
        pytest.skip(str(e))
    return liblcb_amd


@pytest.mark.parametrize("nparts", [2, 4, 8])
def test_partition_balances_c4_bytes(nparts):
    lcb = _lcb()
    lens = mixed_lengths_np(SEED, 1 << 20)
    first = lcb.partition(nparts, lengths=lens)
    assert first[0] == 0 and first[-1] == lens.size and np.all(np.diff(first.astype(np.int64)) >= 0)
    cum = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)])
    part_bytes = cum[first[1:].astype(np.int64)] - cum[first[:-1].astype(np.int64)]
    mean = cum[-1] / nparts
    assert part_bytes.max() <= 1.01 * mean, (part_bytes, mean)
    # the rule: first[p] is where the work prefix (bytes + 64 per message) crosses p/N
    w = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 64)])
    for p in range(1, nparts):
        i = int(first[p])
        t = w[-1] * p // nparts
        assert w[i] - (int(lens[i - 1]) + 64) // 2 < t <= w[i] + (int(lens[i]) + 64) // 2


def test_partition_fixed_and_degenerate():
    lcb = _lcb()
    assert lcb.partition(8, count=8 << 20, fixed_len=1024).tolist() == [k << 20 for k in range(9)]
    assert lcb.partition(3, count=10, fixed_len=5).tolist() == [0, 3, 6, 10]
    assert lcb.partition(4, count=2, fixed_len=5).tolist() == [0, 0, 1, 1, 2]
    assert lcb.partition(1, lengths=np.array([5, 6], np.uint32)).tolist() == [0, 2]
    z = lcb.partition(2, lengths=np.zeros(10, np.uint32))      # empty messages still cost a block
    assert z.tolist() == [0, 5, 10]
    assert lcb.partition(3, lengths=np.zeros(0, np.uint32)).tolist() == [0, 0, 0, 0]
    import errno
    with pytest.raises(lcb.LcbHashError) as e:
        lcb.partition(0, count=4)
    assert e.value.errno == errno.EINVAL


def _ragged(seed, n):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 3000, n).astype(np.uint32)
    lens[rng.integers(0, n, 20)] = 65536
    offs = np.zeros(n, np.uint64)
    pos = 3
    for i in range(n):
        offs[i] = pos
        pos += int(lens[i]) + int(rng.integers(0, 5))
    return gen_stream(seed, pos), offs, lens


@pytest.mark.gpu
@pytest.mark.parametrize("devs", [[0], [0, 0, 0]])
def test_multi_host_mode(gpu, oracle, devs):
    data, offs, lens = _ragged(5, 9000)
    for alg, key in ((1, None), (4, b"radius"), (7, None)):
        got = gpu.hash_batch_multi(devs, alg, data, offsets=offs, lengths=lens, key=key)
        assert np.array_equal(got, oracle.batch(alg, data, offs, lens, key=key)), (alg, devs)
    fx = gen_stream(6, 5000 * 1024)
    got = gpu.hash_batch_multi(devs, 2, fx, count=5000, stride=1024, fixed_len=1000)
    assert np.array_equal(got, oracle.batch(2, fx, count=5000, stride=1024, fixed_len=1000))


@pytest.mark.gpu
@pytest.mark.parametrize("devs,copy", [([0], False), ([0, 0, 0], False), ([0, 0, 0], True), ([0, 0], True)])
def test_multi_device_mode(gpu, oracle, devs, copy):
    import torch
    data, offs, lens = _ragged(8, 9000)
    dd = torch.as_tensor(data, device="cuda:0")
    do = torch.as_tensor(offs.astype(np.int64), device="cuda:0")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda:0")
    for alg, key in ((1, None), (6, b"k" * 200), (8, None)):
        got = gpu.hash_batch_multi(devs, alg, dd, offsets=do, lengths=dl, key=key, copy_parts=copy)
        assert np.array_equal(got.cpu().numpy(), oracle.batch(alg, data, offs, lens, key=key)), (alg, devs)
    # lengths without offsets (message i at i * stride) and plain fixed stride
    n = 4000
    fx = gen_stream(9, n * 512)
    fl = (np.arange(n) % 513).astype(np.uint32)
    got = gpu.hash_batch_multi(devs, 4, torch.as_tensor(fx, device="cuda:0"), stride=512,
                               lengths=torch.as_tensor(fl.astype(np.int32), device="cuda:0"), copy_parts=copy)
    exp = oracle.batch(4, fx, None, fl, count=n, stride=512)
    assert np.array_equal(got.cpu().numpy(), exp)
    got = gpu.hash_batch_multi(devs, 1, torch.as_tensor(fx, device="cuda:0"), count=n, stride=512,
                               fixed_len=512, copy_parts=copy)
    assert np.array_equal(got.cpu().numpy(), oracle.batch(1, fx, count=n, stride=512, fixed_len=512))


@pytest.mark.gpu
def test_multi_single_device_equals_batch(gpu):
    """devs = {0}: the same digests as lcb_hash_batch on the bench workload."""
    n = 1 << 18
    data = gpu.gen_synthetic(SEED, n * 1024)
    a = gpu.hash_batch(1, data, count=n, stride=1024, fixed_len=1024)
    b = gpu.hash_batch_multi([0], 1, data, count=n, stride=1024, fixed_len=1024)
    assert bool((a == b).all())


@pytest.mark.gpu
def test_multi_errors(gpu):
    import errno
    import torch
    d = torch.zeros(1024, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(gpu.LcbHashError) as e:
        gpu.hash_batch_multi([0, 99], 1, d, count=1, fixed_len=16)
    assert e.value.errno == errno.ENODEV


@pytest.mark.gpu
def test_multi_c5_eight_parts_copy(gpu):
    """C5 through lcb_hash_batch_multi with devs = {0 x 8} and the peer-copy
    path forced (LCB_HASH_F_COPY_PARTS): 8M x 1 KiB split into 8 parts, each
    remote part's span copied and hashed beside the others, digests gathered
    back in order -- equal to the reference's digest-of-digests
    (tests/golden/large.json C5_8M_x_1k)."""
    import hashlib
    import json
    import os
    import torch
    large = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "large.json")))
    fx = large["C5_8M_x_1k"]
    n = fx["count"]
    data = gpu.gen_synthetic(large["seed"], n * 1024)
    got = gpu.hash_batch_multi([0] * 8, 1, data, count=n, stride=1024, fixed_len=1024, copy_parts=True)
    torch.cuda.synchronize()
    assert hashlib.sha256(got.cpu().numpy().tobytes()).hexdigest() == fx["algs"]["md5"]["dod"]
    del data, got
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_multi_ragged_c4_shape_copies_before_wait(gpu):
    """a C4-shaped ragged batch ({64 B, 1 KiB, 64 KiB}
    lengths, packed) over 8 parts on device 0 with the peer-copy path forced:
    every remote part's copies, batch and digest copy-back are enqueued
    before the call waits for any part (lcb_hash_multi_stats), the parts run
    from pooled slots (repeat calls), and the digests equal the single-device
    batch."""
    import torch
    from tests.golden_util import mixed_lengths
    n = 24000
    lens = np.array(mixed_lengths(0x51, n), dtype=np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = gpu.gen_synthetic(0x51, int(lens.sum()) + 64)
    do = torch.as_tensor(offs.astype(np.int64), device="cuda:0")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda:0")
    for alg in (1, 6):
        ref = gpu.hash_batch(alg, data, offsets=do, lengths=dl).cpu().numpy()
        for rep in range(2):
            before = gpu.multi_stats()
            got = gpu.hash_batch_multi([0] * 8, alg, data, offsets=do, lengths=dl, copy_parts=True)
            after = gpu.multi_stats()
            assert np.array_equal(got.cpu().numpy(), ref), (alg, rep)
            assert after["calls"] - before["calls"] == 1
            assert after["remote_parts"] - before["remote_parts"] == 7
            assert after["device_splits"] - before["device_splits"] == 1


@pytest.mark.gpu
def test_multi_c4_full_size_host_time(gpu):
    """the full C4-shaped batch (1M records of {64 B,
    1 KiB, 64 KiB}, packed, 21.7 GiB) over 8 parts on device 0 with the
    peer-copy path forced.  The split and every part's byte span are
    computed on the device (no copy of the 12 MB of offsets and lengths to
    the host, no host pass over the messages): the host time per call, from
    entry until every part is enqueued (lcb_hash_multi_stats host_ns), stays
    within 0.3 ms once the part slots exist, and the digests equal the
    single-device batch and the reference's digest-of-digests."""
    import hashlib
    import json
    import os
    import torch
    from tests.golden_util import mixed_lengths
    n = 1 << 20
    lens = np.array(mixed_lengths(SEED, n), dtype=np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = gpu.gen_synthetic(SEED, int(lens.sum()))
    do = torch.as_tensor(offs.astype(np.int64), device="cuda:0")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda:0")
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "large.json")))["C4_1M_mixed"]
    ref = gpu.hash_batch(1, data, offsets=do, lengths=dl).cpu().numpy()
    assert hashlib.sha256(ref.tobytes()).hexdigest() == fx["algs"]["md5"]["dod"]
    host_ms, split_ms = [], []
    for rep in range(3):
        before = gpu.multi_stats()
        got = gpu.hash_batch_multi([0] * 8, 1, data, offsets=do, lengths=dl, copy_parts=True)
        after = gpu.multi_stats()
        assert np.array_equal(got.cpu().numpy(), ref), rep
        assert after["device_splits"] - before["device_splits"] == 1
        host_ms.append((after["host_ns"] - before["host_ns"]) / 1e6)
        split_ms.append((after["split_ns"] - before["split_ns"]) / 1e6)
        del got
    print("host ms per call (first: slot allocation):", [round(x, 4) for x in host_ms],
          "of which the split:", [round(x, 4) for x in split_ms])
    assert max(host_ms[1:]) <= 0.3, host_ms
    del data
    torch.cuda.empty_cache()
