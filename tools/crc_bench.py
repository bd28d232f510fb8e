#!/usr/bin/env python3
"""CRC-32 kernel microbenchmark: every variant over the bench workload
(1M x 1 KiB device-resident, fixed stride), HIP-event times per launch.

usage: python3 tools/crc_bench.py [--variants 1,4,6] [--reps 20] [--warmup 60]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import F_DEVICE, check, lib  # noqa: E402
from liblcb_amd.crc32 import CRC_NAMES  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--variants", default="1,2,3,4,5,6,7,8")
p.add_argument("--reps", type=int, default=20)
p.add_argument("--warmup", type=int, default=60)
p.add_argument("--count", type=int, default=1 << 20)
p.add_argument("--len", type=int, default=1024)
a = p.parse_args()

data = liblcb_amd.gen_synthetic(0x6C62636861736821, a.count * a.len)
out = torch.empty(a.count, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()


def launch(v):
    check(lib().lcb_crc32_batch(v, None, data.data_ptr(), None, None, a.count, a.len, a.len,
                                out.data_ptr(), F_DEVICE, s.cuda_stream))


for v in [int(x) for x in a.variants.split(",")]:
    for _ in range(a.warmup):
        launch(v)
    ts = []
    for r in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        launch(v)
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    gb = a.count * a.len
    print("%-12s median %.4f ms  min %.4f ms  %.1f GB/s (median)" % (CRC_NAMES[v], ts[len(ts) // 2], ts[0],
                                                                   gb / ts[len(ts) // 2] / 1e6), flush=True)
