#!/usr/bin/env python3
"""Per-step overhead of the bench's timed loop (1M x 1 KiB MD5): wall time of
K back-to-back launches with per-launch HIP events (bench.py's loop), with
events only at the ends, and the kernel time the per-launch events report.

usage: python3 tools/step_overhead.py [--steps 200] [--rounds 3]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import F_DEVICE, check, lib  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--steps", type=int, default=200)
p.add_argument("--rounds", type=int, default=3)
a = p.parse_args()
n = 1 << 20
data = liblcb_amd.gen_synthetic(0x6C62636861736821, n * 1024)
dig = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
sp = s.cuda_stream
L = lib()


def launch():
    check(L.lcb_hash_batch(1, None, 0, data.data_ptr(), None, None, n, 1024, 1024, dig.data_ptr(), F_DEVICE, sp))


for _ in range(100):
    launch()
torch.cuda.synchronize()
for r in range(a.rounds):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e0, e1 in ev:
        e0.record(s)
        launch()
        e1.record(s)
    torch.cuda.synchronize()
    t_ev = time.perf_counter() - t0
    kms = sum(e0.elapsed_time(e1) for e0, e1 in ev) / a.steps
    b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    b0.record(s)
    for _ in range(a.steps):
        launch()
    b1.record(s)
    torch.cuda.synchronize()
    t_plain = time.perf_counter() - t0
    print("round %d: per-launch events %.4f ms/step (kernel %.4f)   ends-only %.4f ms/step (event span %.4f)"
          % (r, t_ev / a.steps * 1e3, kms, t_plain / a.steps * 1e3, b0.elapsed_time(b1) / a.steps), flush=True)
