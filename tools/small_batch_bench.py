#!/usr/bin/env python3
"""Small / long-message batches (under one wave per SIMD): HIP-event median
ms and GB/s of ragged batches of a few long messages, per algorithm.
LCB_HASH_GPU_LIB selects a build.

usage: python3 tools/small_batch_bench.py [--alg md5,sha1,sha256,sha512] [--reps 5]"""
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
p.add_argument("--alg", default="md5,sha1,sha256,sha512")
p.add_argument("--reps", type=int, default=5)
a = p.parse_args()
s = torch.cuda.current_stream()
for count, ln in ((1, 32 << 20), (64, 4 << 20), (1024, 256 << 10), (4000, 64 << 10)):
    data = liblcb_amd.gen_synthetic(7, count * ln)
    offs = torch.as_tensor((np.arange(count, dtype=np.int64) * ln), device="cuda")
    lens = torch.full((count,), ln, dtype=torch.int32, device="cuda")
    for name in a.alg.split(","):
        alg = ALG_IDS[name]
        dig = torch.empty((count, DIGEST_SIZE[alg]), dtype=torch.uint8, device="cuda")

        def launch():
            check(lib().lcb_hash_batch(alg, None, 0, data.data_ptr(), offs.data_ptr(), lens.data_ptr(), count, 0, 0,
                                       dig.data_ptr(), F_DEVICE, s.cuda_stream))
        launch()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            launch()
            e1.record(s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = sorted(ts)[len(ts) // 2]
        print(json.dumps({"alg": name, "count": count, "len": ln, "ms": round(ms, 3),
                          "GB_s": round(count * ln / (ms * 1e-3) / 1e9, 2)}), flush=True)
    del data
