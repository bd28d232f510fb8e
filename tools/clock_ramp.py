#!/usr/bin/env python3
"""Engine clock and kernel time of the bench's timed shape over a run
(which clock each row runs at, and why).  For each
pre-conditioning variant -- `gen` (bench.py settle(): the synthetic-stream
kernel writing 256 MiB for 0.4 s), `md5` (0.4 s of the MD5 batch itself),
`idle` (0.5 s of nothing) -- it runs 5 warm-up launches and then `--windows`
windows of 20 back-to-back launches, each bracketed by bench.ClockWindow,
printing ms per launch and the in-run clock of every window.  Workloads:
`fixed` (the headline: 1M x 1 KiB MD5) and `pkt` (the 1M-packet MD5 pass).

usage: python3 tools/clock_ramp.py [--work fixed,pkt] [--settle gen,md5,idle] [--windows 12]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import F_DEVICE, check, lib  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--work", default="fixed,pkt")
    p.add_argument("--settle", default="gen,md5,idle")
    p.add_argument("--windows", type=int, default=12)
    p.add_argument("--steps", type=int, default=20)
    a = p.parse_args()
    s = torch.cuda.current_stream()
    n = 1 << 20
    fixed = liblcb_amd.gen_synthetic(bench.SEED, n * 1024)
    dig = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    from tests.golden_util import packet_layout
    offs, lens, total = packet_layout()
    pdata = liblcb_amd.gen_synthetic(bench.SEED, total)
    po = torch.as_tensor(offs.astype(np.int64), device="cuda")
    pl = torch.as_tensor(lens.astype(np.int32), device="cuda")

    def launch_fixed():
        check(lib().lcb_hash_batch(1, None, 0, fixed.data_ptr(), None, None, n, 1024, 1024, dig.data_ptr(),
                                   F_DEVICE, s.cuda_stream))

    def launch_pkt():
        check(lib().lcb_hash_batch(1, None, 0, pdata.data_ptr(), po.data_ptr(), pl.data_ptr(), len(lens), 0, 0,
                                   dig.data_ptr(), F_DEVICE, s.cuda_stream))
    works = {"fixed": launch_fixed, "pkt": launch_pkt}
    for work in a.work.split(","):
        launch = works[work]
        for settle in a.settle.split(","):
            if settle == "gen":
                bench.settle()
            elif settle == "md5":
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 0.4:
                    for _ in range(20):
                        launch_fixed()
                    torch.cuda.synchronize()
            else:
                torch.cuda.synchronize()
                time.sleep(0.5)
            for _ in range(5):
                launch()
            rows = []
            for w in range(a.windows):
                ms, clk = bench._event_ms(launch, 0, a.steps, s, clock=True)
                rows.append({"w": w, "ms": round(ms, 4), "GHz": clk["clock_GHz"] if clk else None,
                             "GHz_min": clk["clock_GHz_min"] if clk else None})
            print(json.dumps({"work": work, "settle": settle, "windows": rows}), flush=True)


if __name__ == "__main__":
    main()
