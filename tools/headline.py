#!/usr/bin/env python3
"""The bench headline alone (bench.py's settle + time_alg on 1M x 1 KiB MD5,
the same steps / warm-up), for comparing library builds process by process:
LCB_HASH_GPU_LIB selects the build.

usage: python3 tools/headline.py [--steps 20 --warmup 5 --reps 3]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import liblcb_amd  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--steps", type=int, default=20)
p.add_argument("--warmup", type=int, default=5)
p.add_argument("--reps", type=int, default=3)
a = p.parse_args()
torch.cuda.set_device(0)
count = bench.MSGS_PER_GPU
data = liblcb_amd.gen_synthetic(bench.SEED, count * bench.MSG_LEN)
dig = torch.empty((count, 16), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
out = []
for _ in range(a.reps):
    bench.settle()
    t, kms, _clk = bench.time_alg(1, data, dig, count, a.steps, a.warmup, 1)
    out.append((round(t / a.steps * 1e3, 4), round(kms, 4)))
print(json.dumps({"lib": os.environ.get("LCB_HASH_GPU_LIB", "product"), "ms_per_step_wall_event": out}), flush=True)
