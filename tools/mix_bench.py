#!/usr/bin/env python3
"""Ragged batch of a chosen length mix, packed like C4 (records back to back
in a random interleave), timed with LCB_TILE_SEGS settings alternating in
one process: which part of a mix makes segmented long waves lose.

usage: python3 tools/mix_bench.py --alg sha512 --mix 65536:349525,64:349525 --segs 2,0"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import ALG_IDS, DIGEST_SIZE, F_DEVICE, check, lib  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--alg", default="sha512")
p.add_argument("--mix", default="65536:349525,1024:349525,64:349525")
p.add_argument("--segs", default="2,0")
p.add_argument("--rounds", type=int, default=4)
p.add_argument("--reps", type=int, default=3)
a = p.parse_args()
parts = [tuple(int(x) for x in m.split(":")) for m in a.mix.split(",")]
lens = np.concatenate([np.full(n, L, np.uint32) for L, n in parts])
rng = np.random.default_rng(7)
rng.shuffle(lens)
n = len(lens)
offs = np.zeros(n, np.uint64)
offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
total = int(lens.sum())
data = liblcb_amd.gen_synthetic(3, total + 64)
dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
do = torch.as_tensor(offs.astype(np.int64), device="cuda")
s = torch.cuda.current_stream()
alg = ALG_IDS[a.alg]
dig = torch.empty((n, DIGEST_SIZE[alg]), dtype=torch.uint8, device="cuda")


def launch():
    check(lib().lcb_hash_batch(alg, None, 0, data.data_ptr(), do.data_ptr(), dl.data_ptr(), n, 0, 0,
                               dig.data_ptr(), F_DEVICE, s.cuda_stream))


res = {g: [] for g in a.segs.split(",")}
digs = {}
for r in range(a.rounds):
    for g in (list(res) if r % 2 == 0 else list(res)[::-1]):
        os.environ["LCB_TILE_SEGS"] = g
        launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            launch()
        e1.record(s)
        torch.cuda.synchronize()
        res[g].append(e0.elapsed_time(e1) / a.reps)
        digs[g] = dig.cpu().numpy().tobytes()
print(json.dumps({"alg": a.alg, "mix": a.mix, "digests_equal": len(set(digs.values())) == 1,
                  "median_ms": {g: round(sorted(v)[len(v) // 2], 3) for g, v in res.items()}}), flush=True)
