#!/usr/bin/env python3
"""Same-process A/B of a library environment switch read per call (e.g.
LCB_BUCKET_CHUNK=8192 against unset) on the 1M-packet MD5 pass (bench
ragged_packets shape): alternating rounds, mean HIP-event ms per pass, the
digests of both settings compared.  A kernel trace of the same command
(rocprofv3 --kernel-trace) gives the bucketing kernels' own durations
(tools/bucket_trace.py).

usage: python3 tools/env_ab.py NAME VALUE [--rounds 8] [--launches 20]"""
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
    p.add_argument("name")
    p.add_argument("value")
    p.add_argument("--rounds", type=int, default=8)
    p.add_argument("--launches", type=int, default=20)
    a = p.parse_args()
    s = torch.cuda.current_stream()
    from tests.golden_util import packet_layout
    offs, lens, total = packet_layout()
    data = liblcb_amd.gen_synthetic(bench.SEED, total)
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    dig = torch.empty((len(lens), 16), dtype=torch.uint8, device="cuda")

    def launch():
        check(lib().lcb_hash_batch(1, None, 0, data.data_ptr(), do.data_ptr(), dl.data_ptr(), len(lens), 0, 0,
                                   dig.data_ptr(), F_DEVICE, s.cuda_stream))
    res = {"set": [], "unset": []}
    ref = None
    for _ in range(a.rounds):
        for form in ("set", "unset"):
            if form == "set":
                os.environ[a.name] = a.value
            else:
                os.environ.pop(a.name, None)
            res[form].append(round(bench._event_ms(launch, 3, a.launches, s), 4))
            d = dig.cpu().numpy().tobytes()
            ref = ref or d
            assert d == ref, "digests differ between the settings"
    os.environ.pop(a.name, None)
    print(json.dumps({"env": "%s=%s" % (a.name, a.value), "ms_per_pass": res,
                      "mean": {k: round(float(np.mean(v)), 4) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
