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
summary = json.load(open(summ))
# the kernels the bench workload (fixed stride) launches; md_tiles_kernel etc. are other shapes
BENCH_KERNELS = ("md_fixed_lds_kernel", "md_batch_kernel", "gost_batch_kernel")
valu = {}
for k, m in summary.items():
    alg = next((v for n, v in names.items() if n in k), None) if k.startswith(BENCH_KERNELS) else None
    if alg and "<" in k and ", true>" not in k and "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
        valu[alg] = {"kernel": k, "SQ_INSTS_VALU": m["SQ_INSTS_VALU"], "SQ_WAVES": m["SQ_WAVES"],
                     "valu_per_wave": round(m["SQ_INSTS_VALU"] / m["SQ_WAVES"])}
if len(valu) == len(names):
    json.dump({"what": "SQ_INSTS_VALU (wave-instructions) per launch of each algorithm's kernel on the bench "
                       "workload (1M x 1 KiB, fixed stride), rocprofv3 --pmc, mean over dispatches",
               "model": "VALU floor = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x 2.4 GHz): the mixed-stream issue "
                        "rate of DESIGN.md 5 at the MI355X max clock",
               "round": tag, "source": os.path.basename(summ), "count": 1 << 20, "msg_len": 1024,
               "algs": valu}, open(os.path.join(dst, "valu_counts.json"), "w"), indent=1)
    print("valu_counts.json", {a: v["valu_per_wave"] for a, v in valu.items()})
for k, m in summary.items():
    alg = next((v for n, v in names.items() if n in k), None) if k.startswith(BENCH_KERNELS) else None
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
