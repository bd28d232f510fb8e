#!/usr/bin/env python3
"""BASELINE config C4 microbenchmark: 1M buffers of {64 B, 1 KiB, 64 KiB}
(mix64(seed + i) % 3), packed, device resident; HIP-event time per pass
(bucketing included) and the digest-of-digests check against
tests/golden/large.json.  LCB_HASH_GPU_LIB selects an alternative build.

usage: python3 tools/c4bench.py [--alg md5,sha1] [--reps 20]"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import ALG_IDS, DIGEST_SIZE, F_DEVICE, check, lib  # noqa: E402
from tests.golden_util import SEED, mixed_lengths_np  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--alg", default="md5")
p.add_argument("--reps", type=int, default=20)
p.add_argument("--key", default=None)
p.add_argument("--ab-segs", type=int, default=0,
               help="N rounds alternating segmented long tiles on / off (LCB_TILE_SEGS) in this process")
a = p.parse_args()
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "large.json")))["C4_1M_mixed"]
n = fx["count"]
lens = mixed_lengths_np(SEED, n)
offs = np.zeros(n, np.uint64)
offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
total = int(lens.sum())
data = liblcb_amd.gen_synthetic(SEED, total)
dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
do = torch.as_tensor(offs.astype(np.int64), device="cuda")
s = torch.cuda.current_stream()
key = a.key.encode() if a.key else None
for name in a.alg.split(","):
    alg = ALG_IDS[name]
    D = DIGEST_SIZE[alg]
    dig = torch.empty((n, D), dtype=torch.uint8, device="cuda")

    def launch():
        check(lib().lcb_hash_batch(alg, key, len(key) if key else 0, data.data_ptr(), do.data_ptr(),
                                   dl.data_ptr(), n, 0, 0, dig.data_ptr(), F_DEVICE, s.cuda_stream))
    for _ in range(3):
        launch()
    if a.ab_segs:
        res = {"on": [], "off": []}
        for r in range(a.ab_segs):
            for mode in (("on", "off") if r % 2 == 0 else ("off", "on")):
                if mode == "off":
                    os.environ["LCB_TILE_SEGS"] = "0"
                else:
                    os.environ.pop("LCB_TILE_SEGS", None)
                launch()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.reps):
                    launch()
                e1.record(s)
                torch.cuda.synchronize()
                res[mode].append(e0.elapsed_time(e1) / a.reps)
        os.environ.pop("LCB_TILE_SEGS", None)
        on, off = sorted(res["on"]), sorted(res["off"])
        print(json.dumps({"alg": name, "ab": "segmented long tiles on vs off, alternating rounds",
                          "on_ms_median": round(on[len(on) // 2], 4), "off_ms_median": round(off[len(off) // 2], 4),
                          "on_over_off": round(on[len(on) // 2] / off[len(off) // 2], 4),
                          "on_ms": [round(x, 4) for x in res["on"]], "off_ms": [round(x, 4) for x in res["off"]]}),
              flush=True)
        continue
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
    for e0, e1 in ev:
        e0.record(s)
        launch()
        e1.record(s)
    torch.cuda.synchronize()
    ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    ok = None
    if key is None:
        ok = hashlib.sha256(dig.cpu().numpy().tobytes()).hexdigest() == fx["algs"][name]["dod"]
    ab = total + n * (D + 12)
    print(json.dumps({"alg": name, "median_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4),
                      "GiB_s": round(total / (ts[len(ts) // 2] * 1e-3) / 2**30, 1),
                      "hbm_frac": round(ab / (ts[len(ts) // 2] * 1e-3) / 8e12, 4), "dod_ok": ok}), flush=True)
