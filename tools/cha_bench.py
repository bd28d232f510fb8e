#!/usr/bin/env python3
"""ChaCha kernel microbenchmark over the bench workload (1M x 1 KiB
device-resident, fixed stride, iv_i = i): HIP-event time per launch for
ChaCha8/12/20 and XChaCha20, encrypt (read + write) and keystream-only
(write) modes; GB/s counts algorithmic bytes (1 KiB read + 1 KiB written +
8 B iv per buffer; keystream mode: 1 KiB written + 8 B).

usage: python3 tools/cha_bench.py [--rounds 20,12,8] [--reps 20] [--warmup 30]
(LCB_HASH_GPU_LIB=<alt .so> selects another build for A/B runs)
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import F_DEVICE, check, lib  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rounds", default="20,12,8")
p.add_argument("--reps", type=int, default=20)
p.add_argument("--warmup", type=int, default=30)
p.add_argument("--count", type=int, default=1 << 20)
p.add_argument("--len", type=int, default=1024)
p.add_argument("--x", action="store_true", help="also XChaCha20")
a = p.parse_args()

data = liblcb_amd.gen_synthetic(0x6C62636861736821, a.count * a.len)
dst = torch.empty_like(data)
ivs = torch.arange(a.count, dtype=torch.int64, device="cuda").view(torch.uint8)
key = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(range(32)))
s = torch.cuda.current_stream()


def launch(x, rounds, src):
    check(lib().lcb_chacha_batch(x, key, 32, None, ivs.data_ptr() if not x else None, rounds,
                                 src.data_ptr() if src is not None else None, dst.data_ptr(), None, None,
                                 a.count, a.len, a.len, F_DEVICE, s.cuda_stream))


cases = [(0, int(r), True) for r in a.rounds.split(",")] + [(0, int(a.rounds.split(",")[0]), False)]
if a.x:
    cases.append((1, 20, True))
for x, rounds, enc in cases:
    src = data if enc else None
    for _ in range(a.warmup):
        launch(x, rounds, src)
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        launch(x, rounds, src)
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    med = ts[len(ts) // 2]
    by = a.count * (a.len * (2 if enc else 1) + 8)
    print("%s%-3d %-9s median %.4f ms  min %.4f ms  %.1f GB/s  %.1f GiB/s payload  hbm_frac %.3f" % (
        "xchacha" if x else "chacha", rounds, "encrypt" if enc else "keystream", med, ts[0], by / med / 1e6,
        a.count * a.len / (med * 1e-3) / 2**30, by / med / 1e6 / 8000), flush=True)
