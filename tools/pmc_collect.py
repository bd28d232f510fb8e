#!/usr/bin/env python3
"""Turn one GPU session's rocprofv3 --pmc passes (tools/pmc_session.sh) into
the committed counter files bench.py reads, each stamped with the machine
code of the kernel it describes (tools/codestamp.py):

  profiles/pmc_<alg>.json   HBM bytes per launch of each algorithm's kernel on
                            the bench workload (1M x 1 KiB, fixed stride):
                            read = 2 x FETCH_SIZE (gfx950 wide-stream
                            correction, MI355X_MICROARCH.md HBM section),
                            write = WRITE_SIZE;
  profiles/valu_counts.json SQ_INSTS_VALU per launch (the VALU floor);
  profiles/pmc_tiles.json   the same counters for the ragged tile kernel on
                            the packet and C4 workloads, against their
                            algorithmic bytes.

usage: pmc_collect.py <session dir> <round tag> [lib.so]"""
import collections
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import codestamp  # noqa: E402

CXXFILT = "c++filt"
# The kernel each algorithm launches on the bench workload (1M x 1 KiB,
# 128-B aligned stride: the nt line stream, aux 2).
BENCH_KERNEL = {
    "md5": "lcbgpu::md_fixed_persist_kernel<lcbgpu::Md5, false, 2>",
    "sha1": "lcbgpu::md_fixed_lds_kernel<lcbgpu::Sha1, false, 2>",
    "sha224": "lcbgpu::md_fixed_lds_kernel<lcbgpu::Sha256<true>, false, 2>",
    "sha256": "lcbgpu::md_fixed_lds_kernel<lcbgpu::Sha256<false>, false, 2>",
    "sha384": "lcbgpu::md_batch_kernel<lcbgpu::Sha512<true>, false, false>",
    "sha512": "lcbgpu::md_batch_kernel<lcbgpu::Sha512<false>, false, false>",
    "gost256": "lcbgpu::gost_plain2_kernel<true>",
    "gost512": "lcbgpu::gost_plain2_kernel<false>",
}
DIGEST = {"md5": 16, "sha1": 20, "sha224": 28, "sha256": 32, "sha384": 48, "sha512": 64, "gost256": 32,
          "gost512": 64}


def demangled_symbols(so):
    names = sorted(codestamp.kernel_stamps(so))
    out = subprocess.run([CXXFILT], input="\n".join(names), capture_output=True, text=True, check=True).stdout
    return {d.replace("void ", "").split("(")[0].strip(): m for m, d in zip(names, out.splitlines())}


def passes(d, pattern):
    """{kernel (demangled, no 'void ', no args): {counter: [values per dispatch]}} of the pmc dirs."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, pattern, "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].replace("void ", "").split("(")[0].strip()
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def mean(v):
    return sum(v) / len(v) if v else None


def median(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def occupancy(d, pattern, kernel, n_sq=32):
    """Clock and issue statistics of `kernel` from an occupancy pass
    (SQ_CYCLES, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES, SQ_ACTIVE_INST_VALU), per
    dispatch, medians: SQ_* counters are summed over the n_sq shader engines
    (8 XCDs x 4); SQ_WAVE_CYCLES counts in units of 4 cycles; clock =
    SQ_CYCLES / n_sq / dispatch duration."""
    per = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, pattern, "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if row["Kernel_Name"].replace("void ", "").split("(")[0].strip() != kernel:
                continue
            dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            per[row["Dispatch_Id"]][row["Counter_Name"]] = float(row["Counter_Value"])
            per[row["Dispatch_Id"]]["dur_ns"] = dur
    clk, wav, util, durs = [], [], [], []
    for c in per.values():
        if not all(k in c for k in ("SQ_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU")):
            continue
        clk.append(c["SQ_CYCLES"] / n_sq / c["dur_ns"])
        wav.append(c["SQ_WAVE_CYCLES"] * 4 / c["SQ_BUSY_CYCLES"] / 8)          # 8 CUs per engine
        util.append(c["SQ_ACTIVE_INST_VALU"] * 4 / (c["SQ_BUSY_CYCLES"] / n_sq * 1024))
        durs.append(c["dur_ns"] / 1e6)
    if not clk:
        return None
    return {"dispatches": len(clk), "clock_GHz_median": round(median(clk), 3),
            "clock_GHz_range": [round(min(clk), 3), round(max(clk), 3)],
            "waves_per_CU_median": round(median(wav), 2), "valu_issue_util_median": round(median(util), 3),
            "kernel_ms_median": round(median(durs), 4),
            "method": "SQ_CYCLES / 32 engines / dispatch time; waves = SQ_WAVE_CYCLES x 4 / SQ_BUSY_CYCLES / 8 "
                      "CUs; VALU issue = SQ_ACTIVE_INST_VALU x 4 cycles / (SQ_BUSY_CYCLES / 32 x 1,024 SIMDs)"}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    so = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "liblcb_amd", "liblcb_hash_gpu.so")
    sym = demangled_symbols(so)
    stamps = codestamp.kernel_stamps(so)

    def stamp(demangled):
        m = sym[demangled]
        return {"kernel": demangled, "kernel_symbol": m, "code_sha256": stamps[m]}

    prof = os.path.join(ROOT, "profiles")
    fixed = passes(src, "kb_*")
    valu = {}
    for alg, k in BENCH_KERNEL.items():
        c = fixed.get(k)
        if not c or not c.get("FETCH_SIZE") or not c.get("WRITE_SIZE"):
            print("missing counters for", alg, k)
            continue
        rd = 2 * mean(c["FETCH_SIZE"]) * 1024
        wr = mean(c["WRITE_SIZE"]) * 1024
        alg_bytes = (1 << 20) * (1024 + DIGEST[alg])
        rec = {"alg": alg, "count": 1 << 20, "msg_len": 1024, "round": tag}
        rec.update(stamp(k))
        rec.update({"FETCH_SIZE_KiB": mean(c["FETCH_SIZE"]), "WRITE_SIZE_KiB": mean(c["WRITE_SIZE"]),
                    "dispatches": len(c["FETCH_SIZE"]),
                    "correction": "read = 2 x FETCH_SIZE (gfx950 wide-stream under-count, MI355X_MICROARCH.md HBM "
                                  "section); write = WRITE_SIZE",
                    "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                    "algorithmic_bytes": alg_bytes, "traffic_over_algorithmic": round((rd + wr) / alg_bytes, 4),
                    "source": os.path.relpath(src, ROOT)})
        json.dump(rec, open(os.path.join(prof, "pmc_%s.json" % alg), "w"), indent=1)
        print(alg, "traffic/algorithmic %.4f" % ((rd + wr) / alg_bytes))
        if c.get("SQ_INSTS_VALU") and c.get("SQ_WAVES"):
            v = {"SQ_INSTS_VALU": mean(c["SQ_INSTS_VALU"]), "SQ_WAVES": mean(c["SQ_WAVES"])}
            v["valu_per_wave"] = round(v["SQ_INSTS_VALU"] / v["SQ_WAVES"])
            if c.get("GRBM_GUI_ACTIVE"):
                v["GRBM_GUI_ACTIVE"] = mean(c["GRBM_GUI_ACTIVE"])
            v.update(stamp(k))
            valu[alg] = v
    # Occupancy / clock pass of the VALU-bound kernels.
    for alg in ("md5", "sha1", "sha256", "sha512", "gost256"):
        occ = occupancy(src, "kb_occ", BENCH_KERNEL[alg])
        if occ and alg in valu:
            valu[alg]["occupancy"] = occ
            print(alg, "occupancy", occ)
    # GOST against the LDS array: LDS-array cycles
    # (SQ_LDS_IDX_ACTIVE), the extra cycles of bank conflicts
    # (SQ_LDS_BANK_CONFLICT), LDS instructions, of the plain kernel and of
    # its bare LPS chain.
    lds = {}
    lp = passes(src, "kb_lds")
    for name, k in (("gost256", BENCH_KERNEL["gost256"]), ("gost512", BENCH_KERNEL["gost512"]),
                    ("lps_probe", "lcbgpu::gost_lps_probe_kernel")):
        c = lp.get(k)
        if not c or not c.get("SQ_LDS_IDX_ACTIVE"):
            print("missing LDS counters for", name)
            continue
        r = {n: mean(v) for n, v in c.items()}
        r["dispatches"] = len(c["SQ_LDS_IDX_ACTIVE"])
        r["bank_conflict_share"] = round(r.get("SQ_LDS_BANK_CONFLICT", 0) / r["SQ_LDS_IDX_ACTIVE"], 4)
        r.update(stamp(k))
        lds[name] = r
        print(name, "LDS bank-conflict share", r["bank_conflict_share"])
    if lds:
        json.dump({"round": tag, "source": os.path.relpath(src, ROOT), "count": 1 << 20, "msg_len": 1024,
                   "what": "rocprofv3 --pmc over tools/kbench.py --alg gost256,gost512 --gost-probe: SQ_LDS_IDX_ACTIVE "
                           "= LDS-array cycles, SQ_LDS_BANK_CONFLICT = their extra cycles from bank conflicts "
                           "(MI355X_MICROARCH.md LDS), SQ_INSTS_LDS, per dispatch means",
                   "kernels": lds}, open(os.path.join(prof, "pmc_gost_lds.json"), "w"), indent=1)
    if valu:
        json.dump({"what": "SQ_INSTS_VALU (wave-instructions) per launch of each algorithm's kernel on the bench "
                           "workload (1M x 1 KiB, fixed stride), rocprofv3 --pmc, mean over dispatches",
                   "model": "VALU floor = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x 2.4 GHz): the mixed-stream issue "
                            "rate of DESIGN.md 5 at the MI355X max clock",
                   "round": tag, "source": os.path.relpath(src, ROOT), "count": 1 << 20, "msg_len": 1024,
                   "algs": valu}, open(os.path.join(prof, "valu_counts.json"), "w"), indent=1)
        print("valu_counts", {a: v["valu_per_wave"] for a, v in valu.items()})
    # The ragged tile kernel (plain MD5 mode) on the packet and C4 workloads.
    tiles = {}
    k = "lcbgpu::md_tiles_kernel<lcbgpu::Md5, 0>"
    sys.path.insert(0, ROOT)
    from tests.golden_util import mixed_lengths, packet_layout
    _, plens, ptotal = packet_layout()
    clens = mixed_lengths(0x6C62636861736821, 1 << 20)
    work = {"packets": ("kt_pkt_*", int(ptotal), len(plens)), "c4": ("kt_c4_*", int(sum(clens)), len(clens))}
    for name, (pat, total, n) in work.items():
        c = passes(src, pat).get(k)
        if not c or not c.get("FETCH_SIZE") or not c.get("WRITE_SIZE"):
            print("missing tile counters for", name)
            continue
        rd = 2 * mean(c["FETCH_SIZE"]) * 1024
        wr = mean(c["WRITE_SIZE"]) * 1024
        # read: every message byte + its offset and length + its `order` entry; write: its digest
        alg_rd, alg_wr = total + 16 * n, 16 * n
        tiles[name] = {"messages": n, "message_bytes": total, "FETCH_SIZE_KiB": mean(c["FETCH_SIZE"]),
                       "WRITE_SIZE_KiB": mean(c["WRITE_SIZE"]), "dispatches": len(c["FETCH_SIZE"]),
                       "hbm_read_bytes": rd, "hbm_write_bytes": wr,
                       "algorithmic_read_bytes": alg_rd, "algorithmic_write_bytes": alg_wr,
                       "read_over_algorithmic": round(rd / alg_rd, 4), "write_over_algorithmic": round(wr / alg_wr, 4)}
        print("tiles", name, "read/alg %.4f write/alg %.4f" % (rd / alg_rd, wr / alg_wr))
    if tiles:
        rec = {"round": tag, "source": os.path.relpath(src, ROOT),
               "correction": "read = 2 x FETCH_SIZE, write = WRITE_SIZE (as pmc_<alg>.json)"}
        rec.update(stamp(k))
        rec["workloads"] = tiles
        occ = occupancy(src, "kt_pktocc", k)
        if occ:
            rec["workloads"].setdefault("packets", {})["occupancy"] = occ
        json.dump(rec, open(os.path.join(prof, "pmc_tiles.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
