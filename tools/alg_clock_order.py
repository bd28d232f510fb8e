#!/usr/bin/env python3
"""Is an algorithm's in-run engine clock a property of its kernel or of when
it runs?  The bench's per_alg rows (time_alg, 10 warm + 5 timed launches)
in a given order, each with its in-run clock, the whole order repeated.

usage: python3 tools/alg_clock_order.py [--order sha1,md5,sha1,sha256,sha1] [--reps 2]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import liblcb_amd  # noqa: E402
from liblcb_amd._lib import ALG_IDS, DIGEST_SIZE  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--order", default="sha1,md5,sha1,sha256,sha1,sha512,sha1")
    p.add_argument("--reps", type=int, default=2)
    a = p.parse_args()
    count = bench.MSGS_PER_GPU
    data = liblcb_amd.gen_synthetic(bench.SEED, count * bench.MSG_LEN)
    bench.settle()
    for rep in range(a.reps):
        for name in a.order.split(","):
            aid = ALG_IDS[name]
            dg = torch.empty((count, DIGEST_SIZE[aid]), dtype=torch.uint8, device="cuda")
            t, km, ck = bench.time_alg(aid, data, dg, count, 5, 10, 1)
            print(json.dumps({"rep": rep, "alg": name, "kernel_ms": round(km, 4),
                              "clock_GHz": ck["clock_GHz"] if ck else None,
                              "ms_at_2GHz": round(km * ck["clock_GHz"] / 2.0, 4) if ck else None}), flush=True)
            del dg


if __name__ == "__main__":
    main()
