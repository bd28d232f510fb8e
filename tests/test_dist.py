"""Multi-GPU path, exercised on CPU with gloo (world size 2): the weak-scaling
shards of bench.py cover the global batch exactly once, per-rank digests
concatenate to the single-process result, and the job time is the max over
ranks.  The per-rank hashing here is the oracle (CPU); on the GPU box the
same shard bounds feed liblcb_hash_gpu.so."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

PER = 96   # buffers per rank
LEN = 1024


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import bench
    from oracle.pyoracle import Oracle, gen_stream
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port,
                            rank=rank, world_size=world)
    first, n = bench.shard_bounds(rank, world, PER)
    data = gen_stream(bench.SEED, n * LEN, start=first * LEN)
    d = Oracle().batch(1, data, count=n, stride=LEN, fixed_len=LEN)
    parts = [torch.zeros((PER, 16), dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(parts, torch.from_numpy(d))
    t = bench.max_over_ranks(0.5 + rank, world)
    if rank == 0:
        out.put((torch.cat(parts).numpy().tobytes(), t, first))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_weak_shards_cover_batch_once(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, t, first = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from bench import SEED
    from oracle.pyoracle import Oracle, gen_stream
    whole = gen_stream(SEED, world * PER * LEN)
    exp = Oracle().batch(1, whole, count=world * PER, stride=LEN, fixed_len=LEN)
    assert got == exp.tobytes()
    assert t == 0.5 + (world - 1)   # slowest rank
    assert first == 0


def test_shard_bounds():
    import bench
    spans = [bench.shard_bounds(r, 8, 1 << 20) for r in range(8)]
    assert spans[0] == (0, 1 << 20) and spans[7] == (7 << 20, 1 << 20)
    assert all(a + n == b for (a, n), (b, _) in zip(spans, spans[1:]))
