#!/usr/bin/env python3
"""Kernel microbenchmark for profiling: N launches of one algorithm over the
bench workload (1M x 1 KiB device-resident), printing HIP-event times.

usage: python3 tools/kbench.py [--alg md5,sha256,...] [--reps 10] [--count N]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import ALG_IDS, DIGEST_SIZE, F_DEVICE, check, lib  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--alg", default="md5")
p.add_argument("--reps", type=int, default=50)
p.add_argument("--count", type=int, default=1 << 20)
p.add_argument("--len", type=int, default=1024)
p.add_argument("--warmup", type=int, default=60, help="untimed launches per algorithm (clock ramp)")
p.add_argument("--gost-probe", action="store_true",
               help="also run the GOST LPS-chain probe (lcb_hash_gpu_read_probe LCB_PROBE_GOST_LPS)")
a = p.parse_args()

data = liblcb_amd.gen_synthetic(0x6C62636861736821, a.count * a.len)
s = torch.cuda.current_stream()
for name in a.alg.split(","):
    alg = ALG_IDS[name]
    dig = torch.empty((a.count, DIGEST_SIZE[alg]), dtype=torch.uint8, device="cuda")
    ts = []
    for _ in range(a.warmup):
        check(lib().lcb_hash_batch(alg, None, 0, data.data_ptr(), None, None, a.count, a.len, a.len,
                                   dig.data_ptr(), F_DEVICE, s.cuda_stream))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
    for e0, e1 in ev:      # back to back, as bench.py times them
        e0.record(s)
        check(lib().lcb_hash_batch(alg, None, 0, data.data_ptr(), None, None, a.count, a.len, a.len,
                                   dig.data_ptr(), F_DEVICE, s.cuda_stream))
        e1.record(s)
    torch.cuda.synchronize()
    ts = [e0.elapsed_time(e1) for e0, e1 in ev]
    ts.sort()
    gb = a.count * a.len
    print("%-8s median %.4f ms  min %.4f ms  %.1f GB/s (min)" % (name, ts[len(ts) // 2], ts[0],
                                                               gb / ts[0] / 1e6), flush=True)

if a.gost_probe:
    sink = torch.empty(a.count, dtype=torch.int32, device="cuda")
    for _ in range(3):
        check(lib().lcb_hash_gpu_read_probe(2, None, a.count, a.len, a.len, sink.data_ptr(), s.cuda_stream))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
    for e0, e1 in ev:
        e0.record(s)
        check(lib().lcb_hash_gpu_read_probe(2, None, a.count, a.len, a.len, sink.data_ptr(), s.cuda_stream))
        e1.record(s)
    torch.cuda.synchronize()
    ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    print("gost_lps_probe median %.4f ms  min %.4f ms" % (ts[len(ts) // 2], ts[0]), flush=True)
