#!/usr/bin/env python3
"""Copy a GPU session's rocprofv3 outputs into profiles/ (tracked) and write
profiles/pmc_<alg>.json, the per-launch HBM traffic bench.py reports.

usage: collect_profiles.py gpurun_out/<tag> <round-tag>"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, tag = sys.argv[1], sys.argv[2]
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)
for sub, name in (("trace/bench_kernel_stats.csv", "%s_bench_kernel_stats.csv"),
                  ("trace/bench_kernel_trace.csv", "%s_bench_kernel_trace.csv"),
                  ("bench.json", "%s_bench.json")):
    p = os.path.join(src, sub)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, name % tag))
summ = os.path.join(dst, "%s_pmc_summary.json" % tag)
subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), src,
                       "--json", summ], stdout=subprocess.DEVNULL)
names = {"Md5": "md5", "Sha1": "sha1", "Sha256<true>": "sha224", "Sha256<false>": "sha256",
         "Sha512<true>": "sha384", "Sha512<false>": "sha512", "gost_batch_kernel<true": "gost256",
         "gost_batch_kernel<false": "gost512"}
for k, m in json.load(open(summ)).items():
    alg = next((v for n, v in names.items() if n in k), None)
    if alg is None or "hbm_read_bytes_corrected" not in m or "hbm_write_bytes" not in m:
        continue
    json.dump({"alg": alg, "kernel": k, "count": 1 << 20, "msg_len": 1024, "round": tag,
               "FETCH_SIZE_KiB": m["FETCH_SIZE"], "WRITE_SIZE_KiB": m["WRITE_SIZE"],
               "correction": "read = 2 x FETCH_SIZE (gfx950 wide-stream under-count, "
                             "MI355X_MICROARCH.md HBM section); write = WRITE_SIZE",
               "hbm_bytes_per_launch": m["hbm_read_bytes_corrected"] + m["hbm_write_bytes"],
               "source": os.path.basename(summ)},
              open(os.path.join(dst, "pmc_%s.json" % alg), "w"), indent=1)
    print(alg, m["hbm_read_bytes_corrected"] + m["hbm_write_bytes"])
