#!/usr/bin/env python3
"""Generate tests/golden/chacha.json (run ONLY in the build container).

Pure data fixtures for include/crypto/cipher/chacha.h, every expected output
produced by the reference compiled from /root/reference (oracle/_ref, built
with -fno-strict-aliasing: see oracle/Makefile) after its own
chacha_self_test() passed:

kat
    The self test's vector table (chacha.h:709-...), decoded by the
    reference's own hex import helpers (oracle/ref_shim.c ref_chacha_kat).
selftest_x
    The self test's second part (chacha.h:1111-1158): key 192..223, iv
    16..39, the generated 2048-byte plaintext, rounds 8 -> full xchacha() and
    chacha() outputs.
batches
    Synthetic (SURVEY.md 8d stream) ragged batches with per-buffer counters
    and IVs for chacha/xchacha at 8/12/20 rounds and 128/256-bit keys, full
    outputs for small ones, SHA-256 of the output for 64K x 1 KiB.

Usage:  python3 tests/golden/make_golden_chacha.py   (needs `make -C oracle`)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle.pyoracle import SEED, Ref, gen_stream  # noqa: E402


def selftest_plain(n=2048):
    """chacha.h:1115-1119."""
    out, h = bytearray(n), 0
    for i in range(n):
        h = (h + (h + i + 0x55)) & ((1 << 64) - 1)
        h ^= h >> 3
        out[i] = h & 0xff
    return bytes(out)


def ragged(seed, n, hi):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, hi, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return offs, lens


def per_buffer(seed, n, x):
    rng = np.random.default_rng(seed)
    counters = rng.integers(0, 256, 8 * n, dtype=np.uint8)
    counters[4::8] = 0xff  # exercise the 32-bit carry into word 13
    counters[0::8] = np.where(np.arange(n) % 3 == 0, 0xfe, counters[0::8])
    counters[1::8] = np.where(np.arange(n) % 3 == 0, 0xff, counters[1::8])
    counters[2::8] = np.where(np.arange(n) % 3 == 0, 0xff, counters[2::8])
    counters[3::8] = np.where(np.arange(n) % 3 == 0, 0xff, counters[3::8])
    ivs = rng.integers(0, 256, (24 if x else 8) * n, dtype=np.uint8)
    return counters, ivs


def main():
    ref = Ref()
    assert ref.chacha_self_test() == 0, "reference chacha self test fails: check -fno-strict-aliasing"
    kat = ref.chacha_kats()
    key = bytes(range(192, 224))
    iv = np.frombuffer(bytes(range(16, 40)), np.uint8)
    plain = np.frombuffer(selftest_plain(), np.uint8)
    sx = {"key": key.hex(), "key_size": 256, "iv": iv.tobytes().hex(), "rounds": 8,
          "plain": "chacha.h:1115-1119 generator, 2048 bytes"}
    sx["xchacha"] = ref.chacha_batch(key, 256, 8, plain, [0], [2048], ivs=iv, x=True).tobytes().hex()
    sx["chacha"] = ref.chacha_batch(key, 256, 8, plain, [0], [2048], ivs=iv[:8], x=False).tobytes().hex()
    batches = []
    n = 300
    offs, lens = ragged(11, n, 1200)
    total = int((offs + lens).max())
    src = gen_stream(SEED ^ 0xCC, total)
    rng = np.random.default_rng(12)
    for x in (False, True):
        for rounds in (8, 12, 20):
            for ksz in (32, 16):
                k = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
                counters, ivs = per_buffer(rounds * 7 + ksz + (100 if x else 0), n, x)
                out = ref.chacha_batch(k, ksz, rounds, src, offs, lens, counters=counters, ivs=ivs, x=x)
                ks = ref.chacha_batch(k, ksz, rounds, None, offs, lens, counters=counters, ivs=ivs, x=x,
                                      nbytes=total)
                batches.append({"name": "ragged%d_%s%d_k%d" % (n, "x" if x else "", rounds, ksz),
                                "x": x, "rounds": rounds, "key": k.hex(), "key_size": ksz,
                                "counters": counters.tobytes().hex(), "ivs": ivs.tobytes().hex(),
                                "seed": SEED ^ 0xCC, "layout": "ragged(11, 300, 1200)",
                                "out_sha256": hashlib.sha256(out.tobytes()).hexdigest(),
                                "keystream_sha256": hashlib.sha256(ks.tobytes()).hexdigest()})
    # BASELINE C2 shape with chacha20, counter 0 / iv = buffer index (LE)
    cnt = 1 << 16
    src = gen_stream(SEED, cnt * 1024)
    ivs = np.arange(cnt, dtype="<u8").view(np.uint8)
    k = bytes(range(32))
    out = ref.chacha_batch(k, 32, 20, src, count=cnt, stride=1024, fixed_len=1024, ivs=ivs)
    batches.append({"name": "C2_64k_x_1k_chacha20", "x": False, "rounds": 20, "key": k.hex(), "key_size": 32,
                    "counters": None, "ivs": "iv_i = i (u64 LE)", "seed": SEED, "layout": "fixed stride 1024",
                    "count": cnt, "out_sha256": hashlib.sha256(out.tobytes()).hexdigest()})
    json.dump({"source": "include/crypto/cipher/chacha.h compiled from /root/reference (oracle/_ref)",
               "kat": kat, "selftest_x": sx, "batches": batches},
              open(os.path.join(HERE, "chacha.json"), "w"), indent=0)
    print("chacha.json: %d kat, %d batches" % (len(kat), len(batches)))


if __name__ == "__main__":
    main()
