#!/usr/bin/env python3
"""Generate tests/golden/large.json (run ONLY in the build container).

Digest-of-digests fixtures for the two BASELINE configurations too large
for batches.json, computed by the reference's own code compiled from
/root/reference (oracle/_ref/libref_hash_simd.so, built by oracle/Makefile):

  C5  8,388,608 x 1 KiB, fixed stride, seed SEED (BASELINE.json configs[4]);
      the union of the 8 per-GPU shards of bench.py (rank r owns buffers
      [r * 1M, (r + 1) * 1M)), and the strong-scaling global batch.
  C4  1,048,576 buffers, lengths {64, 1024, 65536}[mix64(SEED + i) % 3],
      packed (BASELINE.json configs[3], bench.py ragged_c4).

The input is the synthetic stream of SURVEY.md 8d (u64 word k =
mix64(seed ^ k), little-endian), generated and hashed in chunks so the
whole input never sits in memory.  dod = SHA-256 over the packed digest
array, like batches.json.  Per shard dods (1M each) are kept for C5 so a
single-GPU box can check one shard without the others.

Usage:  python3 tests/golden/make_golden_large.py [--algs md5,sha256]
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle.pyoracle import REF_SIMD_SO, gen_stream  # noqa: E402
from tests.golden_util import SEED, mixed_lengths_np  # noqa: E402

ALGS = {"md5": 1, "sha1": 2, "sha224": 3, "sha256": 4, "sha384": 5, "sha512": 6,
        "gost256": 7, "gost512": 8}
DSIZE = {1: 16, 2: 20, 3: 28, 4: 32, 5: 48, 6: 64, 7: 32, 8: 64}
THREADS = min(8, os.cpu_count() or 1)
CHUNK = 1 << 20


class Ref:
    def __init__(self, path):
        self.lib = ctypes.CDLL(path)
        self.lib.ref_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]

    def fixed_mt(self, alg, data, count, L):
        out = np.zeros(count * DSIZE[alg], np.uint8)
        per = (count + THREADS - 1) // THREADS

        def work(t):
            lo, hi = t * per, min(count, (t + 1) * per)
            if lo < hi:
                self.lib.ref_batch(alg, None, 0, data.ctypes.data + lo * L, None, None, hi - lo, L, L,
                                   out.ctypes.data + lo * DSIZE[alg])
        with ThreadPoolExecutor(THREADS) as ex:
            list(ex.map(work, range(THREADS)))
        return out

    def ragged_mt(self, alg, data, offs, lens):
        """Messages split over threads at byte quantiles (lengths vary 1000x)."""
        n = len(lens)
        out = np.zeros(n * DSIZE[alg], np.uint8)
        cum = np.cumsum(lens.astype(np.uint64))
        cuts = [0] + [int(np.searchsorted(cum, cum[-1] * t // THREADS)) for t in range(1, THREADS)] + [n]

        def work(t):
            lo, hi = cuts[t], cuts[t + 1]
            if lo < hi:
                self.lib.ref_batch(alg, None, 0, data.ctypes.data, offs[lo:].ctypes.data,
                                   lens[lo:].ctypes.data, hi - lo, 0, 0, out.ctypes.data + lo * DSIZE[alg])
        with ThreadPoolExecutor(THREADS) as ex:
            list(ex.map(work, range(THREADS)))
        return out


def c5(ref, algs, total=8 << 20, shard=1 << 20):
    res = {}
    hs = {a: hashlib.sha256() for a in algs}
    shard_h = {a: [] for a in algs}
    for first in range(0, total, CHUNK):
        data = gen_stream(SEED, CHUNK * 1024, start=first * 1024)
        for a in algs:
            d = ref.fixed_mt(ALGS[a], data, CHUNK, 1024)
            hs[a].update(d.tobytes())
            if first % shard == 0:
                shard_h[a].append(hashlib.sha256())
            shard_h[a][-1].update(d.tobytes())
        print("  C5 %d/%d M" % ((first + CHUNK) >> 20, total >> 20), flush=True)
    for a in algs:
        res[a] = {"dod": hs[a].hexdigest(), "shard_dod": [h.hexdigest() for h in shard_h[a]]}
    return res


def c4(ref, algs, count=1 << 20, step=1 << 16):
    lens_all = mixed_lengths_np(SEED, count)
    offs_all = np.zeros(count, np.uint64)
    offs_all[1:] = np.cumsum(lens_all[:-1], dtype=np.uint64)
    hs = {a: hashlib.sha256() for a in algs}
    for i0 in range(0, count, step):
        i1 = min(count, i0 + step)
        base = int(offs_all[i0])
        nbytes = int(offs_all[i1 - 1]) + int(lens_all[i1 - 1]) - base
        data = gen_stream(SEED, nbytes, start=base)
        offs = np.ascontiguousarray(offs_all[i0:i1] - np.uint64(base))
        lens = np.ascontiguousarray(lens_all[i0:i1])
        for a in algs:
            hs[a].update(ref.ragged_mt(ALGS[a], data, offs, lens).tobytes())
        print("  C4 %d/%d" % (i1, count), flush=True)
    return {a: {"dod": hs[a].hexdigest()} for a in algs}, int(lens_all.sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algs", default=",".join(ALGS))
    ap.add_argument("--c4-algs", default=",".join(ALGS))
    a = ap.parse_args()
    if not os.path.exists(REF_SIMD_SO):
        sys.exit("oracle/_ref not built: make -C oracle (needs /root/reference)")
    ref = Ref(REF_SIMD_SO)
    out = {"source": "reference include/crypto/hash compiled from /root/reference (libref_hash_simd.so)",
           "generator": "u64 words mix64(seed ^ k), little-endian", "seed": SEED}
    t0 = time.time()
    out["C4_1M_mixed"] = {"count": 1 << 20, "lengths": "{64, 1024, 65536}[mix64(seed + i) % 3]",
                          "layout": "packed"}
    r, total = c4(ref, a.c4_algs.split(","))
    out["C4_1M_mixed"]["total_bytes"] = total
    out["C4_1M_mixed"]["algs"] = r
    print("C4 done %.0fs" % (time.time() - t0), flush=True)
    out["C5_8M_x_1k"] = {"count": 8 << 20, "stride": 1024, "fixed_len": 1024, "shard": 1 << 20,
                         "algs": c5(ref, a.algs.split(","))}
    print("C5 done %.0fs" % (time.time() - t0), flush=True)
    json.dump(out, open(os.path.join(HERE, "large.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
