#!/usr/bin/env python3
"""Generate tests/golden/packets.json (run ONLY in the build container).

Digest-of-digests fixtures for the network-packet workload (bench.py
`ragged_packets` / `keyed`, tests/test_packets_gpu.py): 1M packets of 20..4096
bytes packed at byte offsets (tests/golden_util.py packet_layout), computed
by the reference's own code compiled from /root/reference
(oracle/_ref/libref_hash_simd.so, built by oracle/Makefile):

  plain   every algorithm, ref_batch (the reference's *_get_digest)
  hmac    every algorithm, one 16-byte key (the reference's *_hmac_get_digest)
  keyed   64 peer secrets, packet i -> secret packet_key_index[i]:
          HMAC (every algorithm), H(K || m) and H(m || K) (MD5, the RADIUS
          shapes, radius.h:774-789 and :1315-1377) through ref_batch_keyed
          (the reference's init / update / update / final)

plus the first 64 digests of each, and the same for the first 4096 packets
(small enough for the CPU test to re-derive with the oracle).  The input is
the synthetic stream of SURVEY.md 8d (u64 word k = mix64(seed ^ k)).

Usage:  python3 tests/golden/make_golden_packets.py
"""
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
from oracle.pyoracle import REF_SIMD_SO, Ref, gen_stream  # noqa: E402
from tests.golden_util import (PKT_COUNT, PKT_NKEYS, SEED, packet_key_index, packet_keys,  # noqa: E402
                               packet_layout)

ALGS = {"md5": 1, "sha1": 2, "sha224": 3, "sha256": 4, "sha384": 5, "sha512": 6,
        "gost256": 7, "gost512": 8}
HMAC_KEY = bytes(range(16))
THREADS = min(8, os.cpu_count() or 1)


def split_run(fn, count, cum):
    """Run fn(lo, hi) over THREADS byte-balanced contiguous ranges."""
    cuts = [0] + [int(np.searchsorted(cum, cum[-1] * t // THREADS)) for t in range(1, THREADS)] + [count]
    with ThreadPoolExecutor(THREADS) as ex:
        list(ex.map(lambda t: fn(cuts[t], cuts[t + 1]) if cuts[t] < cuts[t + 1] else None, range(THREADS)))


def run(ref, data, offs, lens, alg, key=None, mode=None, keys=None, kidx=None):
    n = len(lens)
    out = np.zeros((n, {1: 16, 2: 20, 3: 28, 4: 32, 5: 48, 6: 64, 7: 32, 8: 64}[alg]), np.uint8)
    cum = np.cumsum(lens.astype(np.uint64))

    def part(lo, hi):
        o = np.ascontiguousarray(offs[lo:hi])
        ln = np.ascontiguousarray(lens[lo:hi])
        if mode:
            out[lo:hi] = ref.batch_keyed(alg, mode, keys, data, key_index=kidx[lo:hi], offsets=o, lengths=ln)
        else:
            out[lo:hi] = ref.batch(alg, data, offsets=o, lengths=ln, key=key)
    split_run(part, n, cum)
    return out


def entry(d):
    return {"dod": hashlib.sha256(np.ascontiguousarray(d).tobytes()).hexdigest(),
            "first": d[:64].tobytes().hex() if len(d) >= 64 else d.tobytes().hex()}


def main():
    if not os.path.exists(REF_SIMD_SO):
        sys.exit("oracle/_ref not built: make -C oracle (needs /root/reference)")
    ref = Ref(REF_SIMD_SO)
    offs, lens, total = packet_layout()
    data = gen_stream(SEED, total)
    keys = packet_keys()
    kidx = packet_key_index()
    out = {"source": "reference include/crypto/hash compiled from /root/reference (libref_hash_simd.so: "
                     "ref_batch, ref_batch_keyed)",
           "generator": "u64 words mix64(seed ^ k), little-endian; tests/golden_util.py packet_layout / "
                        "packet_keys / packet_key_index",
           "seed": SEED, "count": PKT_COUNT, "total_bytes": total, "nkeys": PKT_NKEYS,
           "hmac_key_hex": HMAC_KEY.hex(), "full": {}, "small": {}}
    t0 = time.time()
    for scope, n in (("full", PKT_COUNT), ("small", 4096)):
        o, ln, ki = offs[:n], lens[:n], kidx[:n]
        res = out[scope]
        for name, a in ALGS.items():
            res["plain_" + name] = entry(run(ref, data, o, ln, a))
            res["hmac_" + name] = entry(run(ref, data, o, ln, a, key=HMAC_KEY))
            res["keyed_hmac_" + name] = entry(run(ref, data, o, ln, a, mode=1, keys=keys, kidx=ki))
            print("  %s %s %.0fs" % (scope, name, time.time() - t0), flush=True)
        res["keyed_prefix_md5"] = entry(run(ref, data, o, ln, 1, mode=2, keys=keys, kidx=ki))
        res["keyed_suffix_md5"] = entry(run(ref, data, o, ln, 1, mode=3, keys=keys, kidx=ki))
    json.dump(out, open(os.path.join(HERE, "packets.json"), "w"), indent=1)
    print("packets.json written (%.0fs)" % (time.time() - t0))


if __name__ == "__main__":
    main()
