#!/usr/bin/env python3
"""Access-pattern microbenchmark: N records of L bytes each, hashed as a
fixed-stride batch (LDS-DMA line stream kernel when eligible) and as a
ragged batch with the same bytes (offsets/lengths: bucketed path).  Prints
HIP-event ms and TB/s per variant.  LCB_HASH_GPU_LIB selects a build.

usage: python3 tools/stride_bench.py --len 65536 --count 349525 [--alg md5]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import ALG_IDS, DIGEST_SIZE, F_DEVICE, check, lib  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--alg", default="md5")
p.add_argument("--len", type=int, default=65536)
p.add_argument("--count", type=int, default=349525)
p.add_argument("--reps", type=int, default=10)
p.add_argument("--pad", type=int, default=0, help="extra bytes between records")
a = p.parse_args()
alg = ALG_IDS[a.alg]
n, L, stride = a.count, a.len, a.len + a.pad
data = liblcb_amd.gen_synthetic(1, n * stride)
dig = torch.empty((n, DIGEST_SIZE[alg]), dtype=torch.uint8, device="cuda")
offs = torch.arange(n, dtype=torch.int64, device="cuda") * stride
lens = torch.full((n,), L, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()


def run(ragged):
    def launch():
        check(lib().lcb_hash_batch(alg, None, 0, data.data_ptr(), offs.data_ptr() if ragged else None,
                                   lens.data_ptr() if ragged else None, n, stride, L, dig.data_ptr(),
                                   F_DEVICE, s.cuda_stream))
    for _ in range(3):
        launch()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
    for e0, e1 in ev:
        e0.record(s)
        launch()
        e1.record(s)
    torch.cuda.synchronize()
    t = sorted(e0.elapsed_time(e1) for e0, e1 in ev)[a.reps // 2]
    return {"variant": "ragged" if ragged else "fixed", "len": L, "stride": stride, "count": n,
            "ms": round(t, 4), "TB_s": round(n * L / (t * 1e-3) / 1e12, 3)}


for ragged in (False, True):
    print(json.dumps(run(ragged)), flush=True)
