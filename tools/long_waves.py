#!/usr/bin/env python3
"""How the time of a ragged batch of equal long records grows with its wave
count (C4's long class: 5,461 waves of 64 x 64 KiB over 1,024 SIMDs).  The
records are passed with offsets + lengths, so the ragged path runs (bucketing,
then the tile kernel or md_lines_kernel), as in C4.  If time per wave at 5,461
waves is well above that at 4,096 (4 per SIMD), the last wave generation runs
at low occupancy.

usage: python3 tools/long_waves.py [--alg sha512,sha1,md5] [--kib 64]"""
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
p.add_argument("--alg", default="sha512,sha1,md5")
p.add_argument("--kib", type=int, default=64)
p.add_argument("--waves", default="1024,2048,3072,4096,5120,5461,6144,8192")
p.add_argument("--reps", type=int, default=5)
p.add_argument("--phase", type=int, default=0, help="byte offset of every record from a multiple of its length")
p.add_argument("--segs", default="1", help="comma list of LCB_TILE_SEGS settings to run (1: default, 0: off)")
a = p.parse_args()
L = a.kib * 1024
waves = [int(x) for x in a.waves.split(",")]
nmax = max(waves) * 64
data = liblcb_amd.gen_synthetic(1, nmax * L + a.phase)
s = torch.cuda.current_stream()
for name, sg in [(n_, g_) for n_ in a.alg.split(",") for g_ in a.segs.split(",")]:
    if sg == "0":
        os.environ["LCB_TILE_SEGS"] = "0"
    else:
        os.environ.pop("LCB_TILE_SEGS", None)
    alg = ALG_IDS[name]
    D = DIGEST_SIZE[alg]
    for w in waves:
        n = w * 64
        dl = torch.full((n,), L, dtype=torch.int32, device="cuda")
        do = torch.arange(n, dtype=torch.int64, device="cuda") * L + a.phase
        dig = torch.empty((n, D), dtype=torch.uint8, device="cuda")

        def launch():
            check(lib().lcb_hash_batch(alg, None, 0, data.data_ptr(), do.data_ptr(), dl.data_ptr(), n, 0, 0,
                                       dig.data_ptr(), F_DEVICE, s.cuda_stream))
        launch()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for e0, e1 in ev:
            e0.record(s)
            launch()
            e1.record(s)
        torch.cuda.synchronize()
        ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        med = ts[len(ts) // 2]
        print(json.dumps({"alg": name, "segs": sg, "phase": a.phase, "waves": w, "waves_per_simd": round(w / 1024, 3), "median_ms": round(med, 3),
                          "ms_per_1024_waves": round(med / (w / 1024), 3)}), flush=True)
        del dl, do, dig
