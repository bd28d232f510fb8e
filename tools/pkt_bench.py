#!/usr/bin/env python3
"""Ragged-path A/B driver (GPU box): bench.py's ragged_packets rows (1M packets,
20..4096 B at byte offsets; plain / HMAC / keyed, reference dod checked), the
C4 pass, and 1M x 1 KiB described as a ragged batch at strides 1024 / 1040 /
1025 (aligned, 16-B phase, unaligned).  One JSON line per measurement.

usage: python3 tools/pkt_bench.py [--steps 20] [--algs md5,sha1] [--no-c4]
                                 [--no-layouts] [--c4-algs sha1,sha256]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import F_DEVICE, check, lib  # noqa: E402


def ragged_1k(stride, steps):
    count = 1 << 20
    data = liblcb_amd.gen_synthetic(bench.SEED, count * stride + 64)
    offs = torch.arange(count, dtype=torch.int64, device="cuda") * stride
    lens = torch.full((count,), 1024, dtype=torch.int32, device="cuda")
    dig = torch.empty((count, 16), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()

    def launch():
        check(lib().lcb_hash_batch(1, None, 0, data.data_ptr(), offs.data_ptr(), lens.data_ptr(), count, 0, 0,
                                   dig.data_ptr(), F_DEVICE, s.cuda_stream))
    ms = bench._event_ms(launch, 10, steps, s)
    return {"variant": "ragged_1k", "stride": stride, "ms": round(ms, 4),
            "TB_s": round(count * 1024 / (ms * 1e-3) / 1e12, 3)}


def packets_layout(kind, steps):
    """The packet lengths (tests/golden_util.packet_layout) in other layouts:
    `sorted` packs them in descending length order (a tile's records lie
    close together in memory), `aligned128` starts every packet on a 128-B
    line (no streamed line straddles two cache lines)."""
    from tests.golden_util import packet_layout
    _, lens, _ = packet_layout()
    lens = lens.astype(np.uint64)
    if kind == "sorted":
        lens = np.sort(lens)[::-1].copy()
    span = (lens + 127) // 128 * 128 if kind == "aligned128" else lens
    offs = np.zeros(len(lens), np.uint64)
    offs[1:] = np.cumsum(span[:-1], dtype=np.uint64)
    total = int(offs[-1] + span[-1])
    count = len(lens)
    data = liblcb_amd.gen_synthetic(bench.SEED, total)
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    dig = torch.empty((count, 16), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()

    def launch():
        check(lib().lcb_hash_batch(1, None, 0, data.data_ptr(), do.data_ptr(), dl.data_ptr(), count, 0, 0,
                                   dig.data_ptr(), F_DEVICE, s.cuda_stream))
    ms = bench._event_ms(launch, 10, steps, s)
    nbytes = int(lens.sum())
    return {"variant": "packets_" + kind, "ms": round(ms, 4), "TB_s": round(nbytes / (ms * 1e-3) / 1e12, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--algs", default="md5")
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--no-layouts", action="store_true", help="skip the MD5 layout / 1 KiB rows")
    ap.add_argument("--c4-algs", default="", help="C4 passes of these algorithms (full steps each)")
    ap.add_argument("--no-packets", action="store_true", help="skip the ragged_packets rows")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    bench.settle()
    if not a.no_packets:
        print(json.dumps({"ragged_packets": bench.bench_packets(10, a.steps, tuple(a.algs.split(",")))}),
              flush=True)
    if not a.no_layouts:
        for kind in ("sorted", "aligned128"):
            print(json.dumps(packets_layout(kind, a.steps)), flush=True)
        for st in (1024, 1040, 1025):
            print(json.dumps(ragged_1k(st, a.steps)), flush=True)
    for name in filter(None, a.c4_algs.split(",")):
        alg = bench.ALG_IDS[name]
        print(json.dumps({"c4": bench.bench_c4([alg], 3, max(3, a.steps // 4))[name], "alg": name}), flush=True)
    if not a.no_c4:
        print(json.dumps({"c4": bench.bench_c4([1], 5, a.steps)["md5"]}), flush=True)


if __name__ == "__main__":
    main()
