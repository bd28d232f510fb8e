"""The network-packet workload (tests/golden/packets.json, make_golden_packets.py):
1M RADIUS-sized packets of 20..4096 bytes packed at byte offsets
(include/proto/radius.h:576, src/threadpool/threadpool_task.c:692-696), plain,
HMAC and per-peer keyed digests, against digest-of-digests computed by the
reference's own code.

CPU: the oracle restatement reproduces the reference's fixtures on the first
4,096 packets.  GPU (-m gpu): the product library on all 1M packets, input
generated on the device, device mode through the C-ABI (bucketed ragged
tiles), and host mode on a pageable buffer for the small scope."""
import json
import os

import numpy as np
import pytest

from tests.golden_util import (PKT_COUNT, SEED, dod, packet_key_index, packet_keys,
                               packet_layout)

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "packets.json")))
ALGS = {"md5": 1, "sha1": 2, "sha224": 3, "sha256": 4, "sha384": 5, "sha512": 6, "gost256": 7, "gost512": 8}
KEY_MODE = {"keyed_hmac": 1, "keyed_prefix": 2, "keyed_suffix": 3}
HMAC_KEY = bytes.fromhex(FIX["hmac_key_hex"])


def _cases():
    for name in sorted(FIX["small"]):
        kind, alg = name.rsplit("_", 1)
        yield name, kind, ALGS[alg]


def _oracle_digests(oracle, kind, alg, data, offs, lens, keys, kidx):
    if kind == "plain":
        return oracle.batch(alg, data, offsets=offs, lengths=lens)
    if kind == "hmac":
        return oracle.batch(alg, data, offsets=offs, lengths=lens, key=HMAC_KEY)
    return oracle.batch_keyed(alg, KEY_MODE[kind], keys, data, key_index=kidx, offsets=offs, lengths=lens)


def test_fixture_shape():
    offs, lens, total = packet_layout()
    assert FIX["count"] == PKT_COUNT and FIX["total_bytes"] == total
    assert lens.min() >= 20 and lens.max() <= 4096
    # every byte alignment occurs (the point of the workload)
    assert len(np.unique(offs % 16)) == 16


@pytest.mark.parametrize("name,kind,alg", list(_cases()))
def test_oracle_matches_reference_small(oracle, name, kind, alg):
    from oracle.pyoracle import gen_stream
    n = 4096
    offs, lens, _ = packet_layout(n)
    data = gen_stream(SEED, int(offs[-1]) + int(lens[-1]))
    d = _oracle_digests(oracle, kind, alg, data, offs, lens, packet_keys(), packet_key_index(n))
    assert dod(d) == FIX["small"][name]["dod"], name
    assert d[:64].tobytes().hex() == FIX["small"][name]["first"]


# ------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def dev_packets(gpu):
    import torch
    offs, lens, total = packet_layout()
    data = gpu.gen_synthetic(SEED, total)
    d_offs = torch.as_tensor(offs.astype(np.int64), device="cuda")
    d_lens = torch.as_tensor(lens.astype(np.int32), device="cuda")
    d_kidx = torch.as_tensor(packet_key_index().astype(np.int32), device="cuda")
    torch.cuda.synchronize()
    yield data, d_offs, d_lens, d_kidx
    del data, d_offs, d_lens, d_kidx
    torch.cuda.empty_cache()


def _gpu_digests(gpu, kind, alg, data, offs, lens, kidx):
    if kind == "plain":
        return gpu.hash_batch(alg, data, offsets=offs, lengths=lens)
    if kind == "hmac":
        return gpu.hash_batch(alg, data, offsets=offs, lengths=lens, key=HMAC_KEY)
    return gpu.hash_batch_keyed(alg, KEY_MODE[kind], packet_keys(), data, key_index=kidx, offsets=offs,
                                lengths=lens)


@pytest.mark.gpu
@pytest.mark.parametrize("name,kind,alg", list(_cases()))
def test_packets_full_size(gpu, dev_packets, name, kind, alg):
    """All 1M packets on the device against the reference's digest-of-digests."""
    import torch
    data, offs, lens, kidx = dev_packets
    d = _gpu_digests(gpu, kind, alg, data, offs, lens, kidx)
    torch.cuda.synchronize()
    h = d.cpu().numpy()
    assert h[:64].tobytes().hex() == FIX["full"][name]["first"], name
    assert dod(h) == FIX["full"][name]["dod"], name


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["plain", "hmac", "keyed_hmac", "keyed_suffix"])
def test_packets_host_mode_small(gpu, kind):
    """Host mode (pageable buffer) over the first 4,096 packets."""
    from oracle.pyoracle import gen_stream
    n = 4096
    offs, lens, _ = packet_layout(n)
    data = gen_stream(SEED, int(offs[-1]) + int(lens[-1]))
    d = _gpu_digests(gpu, kind, 1, data, offs, lens, packet_key_index(n))
    assert dod(d) == FIX["small"]["%s_md5" % kind]["dod"]
