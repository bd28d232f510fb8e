#!/usr/bin/env python3
"""Per-tile / per-wave timing of the MD5 tile kernel and the fixed-stride
kernel (diagnostic build: tools/build_variant.sh trace k_md5.hip
-DLCB_TILE_TRACE, selected with LCB_HASH_GPU_LIB).  For each workload the
kernel records, per tile (per wave for the fixed kernel), the 100 MHz
real-time clock at start / after the geometry / first take / last take /
end, the hardware id, the line count and the shader cycles; this script
runs the workload (warm), then once traced, and prints a summary JSON line
per workload; raw traces go to --out as .npz.

usage: LCB_HASH_GPU_LIB=build_exp/trace/liblcb_hash_gpu.so \
       python3 tools/tile_trace.py [--out gpurun_out/trace] [--work fixed,r1k,pkt,c4]"""
import argparse
import ctypes
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

TICK_NS = 10.0   # s_memrealtime: 100 MHz


def workloads(names):
    from tests.golden_util import mixed_lengths, packet_layout
    for name in names:
        if name == "fixed":
            count = 1 << 20
            yield name, count, 1024, None, None, count * 1024
        elif name == "r1k":
            count = 1 << 20
            offs = np.arange(count, dtype=np.uint64) * 1024
            lens = np.full(count, 1024, np.uint32)
            yield name, count, 0, offs, lens, count * 1024
        elif name == "pkt":
            offs, lens, total = packet_layout()
            yield name, len(lens), 0, offs.astype(np.uint64), lens.astype(np.uint32), int(total)
        elif name == "c4":
            count = 1 << 20
            lens = np.array(mixed_lengths(bench.SEED, count), dtype=np.uint32)
            offs = np.zeros(count, np.uint64)
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            yield name, count, 0, offs, lens, int(lens.sum())


def summarize(raw, total_bytes):
    t = raw[raw[:, 0] != 0]
    if len(t) == 0:
        return {}
    t0 = t[:, 0].min()
    start, geom, first, last, end = (t[:, i].astype(np.int64) - int(t0) for i in range(5))
    nl = (t[:, 6] & 0xffff).astype(np.int64)
    wave = (t[:, 6] >> 16).astype(np.int64)
    cyc = t[:, 7].astype(np.float64)
    span = int(end.max())
    dur = end - start
    pct = lambda x: [round(float(np.percentile(x, q)) * TICK_NS / 1e3, 3) for q in (5, 50, 95, 99)]  # noqa: E731
    ok = (first > 0) & (nl > 1)
    per_line = (last[ok] - first[ok]) / np.maximum(nl[ok] - 1, 1)
    out = {"tiles": int(len(t)), "span_us": round(span * TICK_NS / 1e3, 2),
           "GBps_over_span": round(total_bytes / (span * TICK_NS * 1e-9) / 1e9, 1),
           "tile_us_p5_50_95_99": pct(dur),
           "geom_us": pct((geom - start)[geom > 0]) if (geom > 0).any() else None,
           "first_line_us": pct((first - np.where(geom > 0, geom, start))[ok]),
           "per_line_us": pct(per_line),
           "after_last_take_us": pct((end - last)[ok]),
           "clock_GHz_median": round(float(np.median(cyc / np.maximum(dur, 1) / TICK_NS)), 3),
           "lines_p50": float(np.median(nl))}
    # gaps between consecutive tiles of one wave, and each wave's finish
    order = np.lexsort((start, wave))
    w, s, e = wave[order], start[order], end[order]
    same = w[1:] == w[:-1]
    gaps = (s[1:] - e[:-1])[same]
    if len(gaps):
        out["gap_us"] = pct(gaps)
    last_end = {}
    first_start = {}
    for wi, si, ei in zip(w, s, e):
        last_end[wi] = max(last_end.get(wi, 0), ei)
        first_start[wi] = min(first_start.get(wi, 1 << 62), si)
    le = np.array(list(last_end.values()))
    fs = np.array(list(first_start.values()))
    out["waves"] = int(len(le))
    out["wave_finish_us_p5_50_95_max"] = [round(float(np.percentile(le, q)) * TICK_NS / 1e3, 2) for q in (5, 50, 95, 100)]
    out["wave_first_start_us_p50_max"] = [round(float(np.percentile(fs, q)) * TICK_NS / 1e3, 2) for q in (50, 100)]
    busy = dur.sum()
    out["busy_frac"] = round(float(busy) / (len(le) * span), 3)
    # in-flight profile: tiles active per 2 us bin
    bins = np.arange(0, span + 200, 200)
    act = np.zeros(len(bins))
    for si, ei in zip(start, end):
        act[si // 200:ei // 200 + 1] += 1
    out["active_tiles_per_2us"] = [int(x) for x in act[::max(1, len(act) // 24)]]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "trace"))
    ap.add_argument("--work", default="fixed,r1k,pkt,c4")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    L = lib()
    fn = L.lcb_debug_tile_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    torch.cuda.set_device(0)
    bench.settle()
    s = torch.cuda.current_stream()
    for name, count, stride, offs, lens, total in workloads(a.work.split(",")):
        data = liblcb_amd.gen_synthetic(bench.SEED, total + 64)
        dig = torch.empty((count, 16), dtype=torch.uint8, device="cuda")
        do = torch.as_tensor(offs.astype(np.int64), device="cuda") if offs is not None else None
        dl = torch.as_tensor(lens.astype(np.int32), device="cuda") if lens is not None else None

        def launch():
            check(L.lcb_hash_batch(1, None, 0, data.data_ptr(), do.data_ptr() if do is not None else None,
                                   dl.data_ptr() if dl is not None else None, count, stride, stride,
                                   dig.data_ptr(), F_DEVICE, s.cuda_stream))
        ntr = (count + 63) // 64 + 4096
        buf = torch.zeros((ntr, 8), dtype=torch.int64, device="cuda")
        check(fn(None, None))
        ms = bench._event_ms(launch, 10, 20, s)        # untraced time
        key = "fixed" if name == "fixed" else "tiles"
        check(fn(buf.data_ptr(), None) if key == "tiles" else fn(None, buf.data_ptr()))
        for _ in range(3):
            buf.zero_()
            launch()
        torch.cuda.synchronize()
        check(fn(None, None))
        raw = buf.cpu().numpy().view(np.uint64)
        np.savez_compressed(os.path.join(a.out, "%s.npz" % name), raw=raw)
        res = {"work": name, "untraced_ms": round(ms, 4), "bytes": total}
        res.update(summarize(raw, total))
        print(json.dumps(res), flush=True)
        del data, dig, do, dl, buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
