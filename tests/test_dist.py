"""Multi-GPU path, exercised on CPU with gloo (world size 2).

* `bench.py --gpus 2 --plan` run directly (no launcher): bench.py starts the
  two ranks itself, each rank reports the shard the bench would time, and
  the shards are disjoint and cover the global batch (weak and strong).
* A gloo world of 2 in which each rank takes ITS shard from the same
  bench.shard_bounds (lcb_hash_partition) the bench uses, hashes it (the
  oracle stands in for the GPU here; on the box the same bounds feed
  liblcb_hash_gpu.so), and the ranks' digests — gathered to rank 0 the way
  bench.gather_digests pads and trims them — equal the single-process result.
  The job time is the max over ranks.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEN = 1024


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lib_or_skip():
    import liblcb_amd
    try:
        liblcb_amd.lib()
    except RuntimeError as e:
        pytest.skip(str(e))


@pytest.mark.parametrize("scaling,extra", [("weak", ["--count", "96"]), ("strong", ["--global-count", "1001"])])
def test_bench_gpus2_spawns_two_ranks(scaling, extra):
    _lib_or_skip()
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--plan",
                        "--scaling", scaling] + extra, capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    j = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    p = sorted(j["plan"], key=lambda x: x["rank"])
    assert [x["rank"] for x in p] == [0, 1] and all(x["world_size"] == 2 for x in p)
    assert p[0]["pid"] != p[1]["pid"]
    assert p[0]["first"] == 0 and p[0]["first"] + p[0]["count"] == p[1]["first"]
    assert p[1]["first"] + p[1]["count"] == j["total"] == (192 if scaling == "weak" else 1001)


def _worker(rank, world, port, out, scaling, per, gcount):
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from oracle.pyoracle import Oracle, gen_stream
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port,
                            rank=rank, world_size=world)
    total = bench.global_count(scaling, world, per, gcount)
    first, n = bench.shard_bounds(rank, world, per, scaling, gcount)
    data = gen_stream(bench.SEED, n * LEN, start=first * LEN)
    d = Oracle().batch(1, data, count=n, stride=LEN, fixed_len=LEN)
    import liblcb_amd
    fa = liblcb_amd.partition(world, count=total, fixed_len=LEN)
    mx = int(np.max(np.diff(fa.astype(np.int64))))
    buf = torch.zeros((mx, 16), dtype=torch.uint8)
    buf[:n] = torch.from_numpy(d)
    parts = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    t = bench.max_over_ranks(0.5 + rank, world)
    if rank == 0:
        got = torch.cat([parts[r][:int(fa[r + 1] - fa[r])] for r in range(world)])
        out.put((got.numpy().tobytes(), t, first, total))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("scaling,per,gcount", [("weak", 96, None), ("strong", 0, 203)])
def test_shards_cover_batch_once(scaling, per, gcount):
    _lib_or_skip()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, scaling, per, gcount)) for r in range(world)]
    for p in procs:
        p.start()
    got, t, first, total = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from bench import SEED
    from oracle.pyoracle import Oracle, gen_stream
    whole = gen_stream(SEED, total * LEN)
    exp = Oracle().batch(1, whole, count=total, stride=LEN, fixed_len=LEN)
    assert got == exp.tobytes()
    assert t == 0.5 + (world - 1)   # slowest rank
    assert first == 0


def test_shard_bounds():
    _lib_or_skip()
    sys.path.insert(0, ROOT)
    import bench
    spans = [bench.shard_bounds(r, 8, 1 << 20) for r in range(8)]
    assert spans[0] == (0, 1 << 20) and spans[7] == (7 << 20, 1 << 20)
    assert all(a + n == b for (a, n), (b, _) in zip(spans, spans[1:]))
    strong = [bench.shard_bounds(r, 4, 1 << 20, "strong", 8 << 20) for r in range(4)]
    assert strong == [(k << 21, 1 << 21) for k in range(4)]
    odd = [bench.shard_bounds(r, 3, 0, "strong", 10) for r in range(3)]
    assert odd == [(0, 3), (3, 3), (6, 4)]
