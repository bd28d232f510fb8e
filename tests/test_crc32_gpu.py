"""GPU parity of the batched CRC-32 family (include/lcb_crc32_gpu.h) through
the C-ABI: bit-exact against the reference's KATs, the reference-computed
fixtures of tests/golden/crc32.json (incl. the full 1M x 1 KiB pass) and the
oracle on misaligned / ragged / chained (X_update) / bucketed batches, in
device and host mode."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from oracle.pyoracle import CRC_VARIANTS, SEED, gen_stream

HERE = os.path.dirname(os.path.abspath(__file__))
VID = {v: k for k, v in CRC_VARIANTS.items()}
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def crc_golden():
    return json.load(open(os.path.join(HERE, "golden", "crc32.json")))


def dev(a, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def run_dev(v, data, offs, lens, init=None):
    from liblcb_amd.crc32 import crc32_batch
    out = crc32_batch(v, dev(data), offsets=dev(offs.astype(np.int64)), lengths=dev(lens.astype(np.int32)),
                      init=dev(init.astype(np.int32)) if init is not None else None)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def test_kat_device_and_host(gpu, crc_golden):
    from liblcb_amd.crc32 import crc32_batch
    for vn, v in VID.items():
        cases = [c for c in crc_golden["kat"] if c["variant"] == vn]
        msgs = [bytes.fromhex(c["msg"]) for c in cases]
        lens = np.array([len(m) for m in msgs], np.uint32)
        offs = np.zeros(len(msgs), np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        data = np.frombuffer(b"".join(msgs), np.uint8)
        want = ["%08x" % int(c["crc"], 16) for c in cases]
        got_d = run_dev(v, data, offs, lens)
        got_h = crc32_batch(v, data, offsets=offs, lengths=lens)
        assert ["%08x" % x for x in got_d] == want, vn
        assert ["%08x" % x for x in got_h] == want, vn


def _layout(e):
    from tests.test_crc32_oracle import batch_layout
    return batch_layout(e)


@pytest.mark.parametrize("name", ["ragged_0_1100", "misaligned_512", "update_0_299", "C2_64k_x_1k"])
def test_golden_batches(gpu, crc_golden, name):
    from tests.test_crc32_oracle import check_crcs
    e = next(b for b in crc_golden["batches"] if b["name"] == name)
    data, offs, lens, init = _layout(e)
    for vn, want in e["crcs"].items():
        got = run_dev(VID[vn], data, offs, lens, init)
        assert check_crcs(got, want), (name, vn)


def test_c3_full_pass(gpu, crc_golden):
    """BASELINE C3 shape: 1M x 1 KiB generated on the device, fixed stride."""
    import liblcb_amd
    from liblcb_amd.crc32 import crc32_batch
    e = next(b for b in crc_golden["batches"] if b["name"] == "C3_1M_x_1k")
    n = e["count"]
    data = liblcb_amd.gen_synthetic(SEED, n * 1024)
    for vn, want in e["crcs"].items():
        out = crc32_batch(VID[vn], data, count=n, stride=1024, fixed_len=1024)
        torch.cuda.synchronize()
        packed = out.cpu().numpy().view(np.uint32).astype("<u4").tobytes()
        assert "sha256:" + hashlib.sha256(packed).hexdigest() == want, vn
    del data


def test_alignment_sweep_vs_oracle(gpu, oracle):
    """Every start alignment 0..15 x lengths 0..300, with and without init."""
    rng = np.random.default_rng(17)
    offs, lens = [], []
    pos = 0
    for a in range(16):
        for n in range(0, 301, 7):
            pos = (pos + 15) // 16 * 16 + a
            offs.append(pos)
            lens.append(n)
            pos += n
    offs = np.array(offs, np.uint64)
    lens = np.array(lens, np.uint32)
    data = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    init = rng.integers(0, 1 << 32, len(lens), dtype=np.uint64).astype(np.uint32)
    for v in CRC_VARIANTS:
        assert np.array_equal(run_dev(v, data, offs, lens), oracle.crc32_batch(v, data, offs, lens)), v
        assert np.array_equal(run_dev(v, data, offs, lens, init),
                              oracle.crc32_batch(v, data, offs, lens, init=init)), v


def test_bucketed_mixed_lengths(gpu, oracle):
    """>= 4096 ragged buffers take the device length-bucketing path; results
    land at the caller's index regardless of the processing order."""
    from tests.golden_util import mixed_lengths
    lens = np.array(mixed_lengths(SEED ^ 0xC4C, 8192), np.uint32) % 5000  # {64, 1024, 65536 % 5000}
    offs = np.zeros(len(lens), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = gen_stream(SEED ^ 0xC4C, int(lens.sum()))
    for v in (VID["crc32c"], VID["crc32a"]):
        assert np.array_equal(run_dev(v, data, offs, lens), oracle.crc32_batch(v, data, offs, lens))


def test_host_mode_pinned_and_chained(gpu, oracle):
    """Host mode: pageable and page-locked input, chained X_update over two
    halves == one-shot over the whole buffer (crc32.h:636-653 style)."""
    from liblcb_amd.crc32 import crc32_batch
    n, L = 3000, 700
    data = gen_stream(SEED ^ 0x77, n * L)
    pinned = torch.from_numpy(data.copy()).pin_memory()
    for v in CRC_VARIANTS:
        whole = crc32_batch(v, data, count=n, stride=L, fixed_len=L)
        assert np.array_equal(whole, oracle.crc32_batch(v, data, count=n, stride=L, fixed_len=L))
        whole_p = crc32_batch(v, pinned.numpy(), count=n, stride=L, fixed_len=L)
        assert np.array_equal(whole, whole_p)
        first = crc32_batch(v, data, count=n, stride=L, fixed_len=300)
        offs = np.arange(n, dtype=np.uint64) * L + 300
        second = crc32_batch(v, data, offsets=offs, lengths=np.full(n, L - 300, np.uint32), init=first)
        assert np.array_equal(second, whole), v


def test_named_entry_points(gpu, oracle):
    import liblcb_amd.crc32 as c
    msg = np.frombuffer(b"123456789", np.uint8)
    checks = {"crc32a": 0xfc891918, "crc32cksum": 0x765e7680, "crc32mpeg2": 0x0376e6e7,
              "crc32b": 0xcbf43926, "crc32jamcrc": 0x340bc6d9, "crc32c": 0xe3069283,
              "crc32d": 0x87315576, "crc32q": 0x3010bf7f}
    for name, want in checks.items():
        got = getattr(c, name + "_batch")(msg, count=1, fixed_len=9)
        assert int(got[0]) == want, name
    empty = c.crc32c_batch(np.zeros(1, np.uint8), count=3, stride=0, fixed_len=0)
    assert [int(x) for x in empty] == [0, 0, 0]
