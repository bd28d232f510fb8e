#!/usr/bin/env python3
"""Kernel time vs. elapsed run time (clock ramp / thermal check): blocks of
30 MD5 passes over 1M x 1 KiB, mean HIP-event ms per block."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import F_DEVICE, check, lib  # noqa: E402

alg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = 1 << 20
data = liblcb_amd.gen_synthetic(1, n * 1024)
dig = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
t0 = time.perf_counter()
for blk in range(int(sys.argv[2]) if len(sys.argv) > 2 else 40):
    ev = []
    for _ in range(30):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        check(lib().lcb_hash_batch(alg, None, 0, data.data_ptr(), None, None, n, 1024, 1024,
                                   dig.data_ptr(), F_DEVICE, s.cuda_stream))
        b.record(s)
        ev.append((a, b))
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in ev]
    print("t=%7.3fs block %2d mean %.4f min %.4f max %.4f" % (time.perf_counter() - t0, blk,
          sum(ms) / len(ms), min(ms), max(ms)), flush=True)
