#!/usr/bin/env python3
"""Same-process A/B of the ragged-batch bucketing forms:
the one-kernel ticket-ordered bucketing (LCB_BUCKET_FUSED=1, read per call)
against the three-kernel form (the default), alternating rounds on the 1M-packet
MD5 pass (bench ragged_packets shape) and C4; mean HIP-event ms per pass,
the digests of both forms compared.  (The bucketing's own kernel durations
come from a rocprofv3 kernel trace of the same command.)

usage: python3 tools/bucket_ab.py [--rounds 8] [--launches 20] [--work pkt,c4]"""
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=8)
    p.add_argument("--launches", type=int, default=20)
    p.add_argument("--work", default="pkt,c4")
    a = p.parse_args()
    s = torch.cuda.current_stream()
    from tests.golden_util import mixed_lengths, packet_layout
    works = {}
    offs, lens, total = packet_layout()
    works["pkt"] = (liblcb_amd.gen_synthetic(bench.SEED, total), offs, lens)
    if "c4" in a.work:
        n = 1 << 20
        l4 = np.array(mixed_lengths(bench.SEED, n), dtype=np.uint32)
        o4 = np.zeros(n, np.uint64)
        o4[1:] = np.cumsum(l4[:-1], dtype=np.uint64)
        works["c4"] = (liblcb_amd.gen_synthetic(bench.SEED, int(l4.sum())), o4, l4)
    for w in a.work.split(","):
        data, o, l = works[w]
        do = torch.as_tensor(o.astype(np.int64), device="cuda")
        dl = torch.as_tensor(l.astype(np.int32), device="cuda")
        dig = torch.empty((len(l), 16), dtype=torch.uint8, device="cuda")

        def launch():
            check(lib().lcb_hash_batch(1, None, 0, data.data_ptr(), do.data_ptr(), dl.data_ptr(), len(l), 0, 0,
                                       dig.data_ptr(), F_DEVICE, s.cuda_stream))
        res = {"fused": [], "three": []}
        ref = None
        for r in range(a.rounds):
            for form in ("fused", "three"):
                if form == "fused":
                    os.environ["LCB_BUCKET_FUSED"] = "1"
                else:
                    os.environ.pop("LCB_BUCKET_FUSED", None)
                ms = bench._event_ms(launch, 3, a.launches, s)
                res[form].append(round(ms, 4))
                d = dig.cpu().numpy().tobytes()
                if ref is None:
                    ref = d
                assert d == ref, "digests differ between the bucketing forms"
        os.environ.pop("LCB_BUCKET_FUSED", None)
        print(json.dumps({"work": w, "ms_per_pass": res,
                          "mean": {k: round(float(np.mean(v)), 4) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
