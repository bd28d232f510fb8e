#!/usr/bin/env python3
"""Same-process A/B of library builds: every build is dlopen'ed side by side
(own handle, own kernels) and the builds alternate round by round, each
round timing `--launches` back-to-back launches with HIP events at the two
ends only (as bench.py times its steps).  Alternating inside one process
keeps the clock / power state and the data identical between builds, so a
1-2 % difference is visible above the run-to-run noise of separate
processes.

Workloads: `fixed` (1M x 1 KiB, stride 1024: the bench kernel), `pkt` (the
1M-packet ragged batch, bucketing included), `r1k` (1M x 1 KiB as a ragged
batch), `c4` (1M mixed lengths: 64 B / 1 KiB / 64 KiB).

usage: python3 tools/ab_inproc.py --libs product,head [--work fixed,pkt]
                                  [--alg md5] [--rounds 8] [--launches 40]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import ALG_IDS, CRC_SIGNATURES, DIGEST_SIZE, F_DEVICE, SIGNATURES  # noqa: E402
from liblcb_amd.crc32 import CRC_NAMES  # noqa: E402

CRC_IDS = {n: v for v, n in CRC_NAMES.items()}


def load(name):
    path = os.path.join(ROOT, "liblcb_amd", "liblcb_hash_gpu.so") if name == "product" else \
        os.path.join(ROOT, "ab_builds", name, "liblcb_hash_gpu.so")
    L = ctypes.CDLL(path)
    for fn, res, args in SIGNATURES + CRC_SIGNATURES:
        if hasattr(L, fn):
            f = getattr(L, fn)
            f.restype = res
            f.argtypes = args
    return L


def workload(name):
    from tests.golden_util import mixed_lengths, packet_layout
    seed = 0x6C62636861736821
    if name == "fixed":
        n = 1 << 20
        return n, None, None, 1024, n * 1024
    if name == "r1k":
        n = 1 << 20
        return n, np.arange(n, dtype=np.uint64) * 1024, np.full(n, 1024, np.uint32), 0, n * 1024
    if name == "pkt":
        offs, lens, total = packet_layout()
        return len(lens), offs.astype(np.uint64), lens.astype(np.uint32), 0, int(total)
    if name == "c4":
        n = 1 << 20
        lens = np.array(mixed_lengths(seed, n), dtype=np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        return n, offs, lens, 0, int(lens.sum())
    raise SystemExit("unknown workload " + name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="product,head")
    ap.add_argument("--work", default="fixed")
    ap.add_argument("--alg", default="md5")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--mode", default="plain",
                    help="plain | hmac | keyed_hmac | keyed_suffix (keyed: the packet rows' 64 secrets)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    libs = {n: load(n) for n in a.libs.split(",")}
    s = torch.cuda.current_stream()
    bad = []
    for wname in a.work.split(","):
        count, offs, lens, stride, total = workload(wname)
        data = liblcb_amd.gen_synthetic(0x6C62636861736821, total + 64)
        do = torch.as_tensor(offs.astype(np.int64), device="cuda") if offs is not None else None
        dl = torch.as_tensor(lens.astype(np.int32), device="cuda") if lens is not None else None
        for alg_name in a.alg.split(","):
            crc = CRC_IDS.get(alg_name)      # a CRC-32 variant (lcb_crc32_batch) or a hash
            alg = None if crc else ALG_IDS[alg_name]
            dig = torch.empty((count, 4 if crc else DIGEST_SIZE[alg]), dtype=torch.uint8, device="cuda")
            launches = max(4, a.launches if wname in ("fixed", "r1k") else a.launches // (10 if wname == "c4" else 2))

            if a.mode.startswith("keyed"):
                from tests.golden_util import packet_key_index, packet_keys
                keys = packet_keys()
                blob = np.frombuffer(b"".join(keys), np.uint8).copy()
                koff = np.zeros(len(keys), np.uint64)
                koff[1:] = np.cumsum([len(k) for k in keys[:-1]])
                klen = np.array([len(k) for k in keys], np.uint32)
                kidx = torch.as_tensor(packet_key_index(count).astype(np.int32), device="cuda")
                kmode = 1 if a.mode == "keyed_hmac" else 3
            hkey = b"ab-inproc-hmac-key" if a.mode == "hmac" else None

            def run(L, k):
                for _ in range(k):
                    if a.mode.startswith("keyed"):
                        rc = L.lcb_hash_batch_keyed(alg, kmode, blob.ctypes.data, koff.ctypes.data, klen.ctypes.data,
                                                    len(keys), kidx.data_ptr(), data.data_ptr(),
                                                    do.data_ptr() if do is not None else None,
                                                    dl.data_ptr() if dl is not None else None, count, stride, stride,
                                                    dig.data_ptr(), F_DEVICE, s.cuda_stream)
                    elif crc:
                        rc = L.lcb_crc32_batch(crc, None, data.data_ptr(),
                                               do.data_ptr() if do is not None else None,
                                               dl.data_ptr() if dl is not None else None, count, stride, stride,
                                               dig.data_ptr(), F_DEVICE, s.cuda_stream)
                    else:
                        rc = L.lcb_hash_batch(alg, hkey, len(hkey) if hkey else 0, data.data_ptr(),
                                              do.data_ptr() if do is not None else None,
                                              dl.data_ptr() if dl is not None else None, count, stride, stride,
                                              dig.data_ptr(), F_DEVICE, s.cuda_stream)
                    if rc:
                        raise SystemExit("lcb_hash_batch rc=%d" % rc)
            res = {n: [] for n in libs}
            digs = {}
            for n, L in libs.items():      # warm every build (clocks, code load)
                run(L, launches)
                torch.cuda.synchronize()
                digs[n] = dig.cpu().numpy().tobytes()
            same = len(set(digs.values())) == 1
            for _ in range(a.rounds):
                for n, L in libs.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record(s)
                    run(L, launches)
                    e1.record(s)
                    torch.cuda.synchronize()
                    res[n].append(e0.elapsed_time(e1) / launches)
            out = {"work": wname, "alg": alg_name, "mode": a.mode, "launches": launches, "rounds": a.rounds,
                   "digests_equal": same}
            if not same:
                # A faster build with other digests is not a result: mark the
                # row and fail the run.
                out["INVALID"] = "digests differ between builds"
                bad.append((wname, alg_name))
            for n, v in res.items():
                v = sorted(v)
                out[n] = {"median_ms": round(v[len(v) // 2], 4), "min_ms": round(v[0], 4),
                          "max_ms": round(v[-1], 4)}
            base = out[list(libs)[0]]["median_ms"]
            for n in libs:
                out[n]["rel"] = round(out[n]["median_ms"] / base, 4)
            print(json.dumps(out), flush=True)
            del dig
        del data, do, dl
        torch.cuda.empty_cache()
    if bad:
        raise SystemExit("ab_inproc: digests differ between builds for %s" % bad)


if __name__ == "__main__":
    main()
