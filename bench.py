#!/usr/bin/env python3
"""Benchmark: device-resident GiB/s hashed, 1M x 1 KiB buffers per MI355X.

One step = one pass of the batch digest kernel over the rank's shard of
the global batch of 1,024-byte buffers.  Inputs are generated on the device
by the synthetic-stream kernel before timing (no host traffic in the timed
region).  Shards are independent (no data-path collective); the only
collectives in the timed region are the barrier and the max-over-ranks of
the time.

  --scaling weak    (default) 1,048,576 buffers per GPU (BASELINE configs[2]);
                    at --gpus 8 the union is configs[4], 8M x 1 KiB
  --scaling strong  a fixed global batch (--global-count, default 8M x 1 KiB
                    = configs[4]) split over the N GPUs

Shards come from lcb_hash_partition (include/lcb_hash_gpu.h), the library's
own work-balanced split.  `--gpus N` without a torch.distributed launcher
starts the N ranks itself (a torch.distributed.run child, before any GPU
call); under a launcher WORLD_SIZE must equal N.  After timing, the ranks'
digests are gathered to rank 0 over RCCL (timed separately, never part of
`value`) and checked against the reference's digest-of-digests
(tests/golden/batches.json C3, tests/golden/large.json C5).

Extra fields on the JSON line:
  roofline      dominant kernel vs HBM peak (algorithmic bytes / HIP-event
                kernel time); traffic from a committed rocprofv3 PMC summary
                (profiles/pmc_<alg>.json) when one exists for this workload;
                valu_frac = VALU issue floor (committed SQ_INSTS_VALU count,
                profiles/valu_counts.json, x 4 cycles on 1,024 SIMDs at
                2.4 GHz) / kernel time; `clock` = the engine clock of the
                timed launches themselves (ClockWindow: s_memtime /
                s_memrealtime stamps on the launch stream around them) and
                valu_frac_run_clock the same floor at that clock; every
                per_alg, ragged_packets and ragged_c4 row carries its own
  cpu_baseline  the reference's own include/crypto code (oracle/_ref, built
                from /root/reference) timed on this host's cores, rank 0, N=1
  per_alg       the same measurement for every algorithm (N=1), each with
                hbm_frac, valu_frac and the reference CPU rate beside it
  e2e           host-memory path: pinned input -> H2D -> kernel -> D2H
  crc32/chacha  the CRC-32 family and ChaCha/XChaCha over the same bytes
  verify        GPU digests of the timed workload vs the CPU reference run
"""
import argparse
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import liblcb_amd  # noqa: E402
from liblcb_amd._lib import ALG_IDS, ALG_NAMES, DIGEST_SIZE, F_DEVICE, check, lib  # noqa: E402

SEED = 0x6C62636861736821
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MSG_LEN = 1024
CPU_SAMPLE_S = 1.0  # wall seconds of the CPU baseline sample (x threads of CPU work)
MSGS_PER_GPU = 1 << 20


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--alg", default="md5", choices=sorted(ALG_IDS))
    p.add_argument("--scaling", default="weak", choices=("weak", "strong"))
    p.add_argument("--count", type=int, default=MSGS_PER_GPU, help="buffers per GPU (weak scaling)")
    p.add_argument("--global-count", type=int, default=8 * MSGS_PER_GPU,
                   help="buffers of the whole job (strong scaling)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    p.add_argument("--no-extras", action="store_true", help="skip per_alg / e2e")
    p.add_argument("--no-gather", action="store_true", help="skip the RCCL digest gather + fixture check")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--settle", default="gen", choices=("self", "gen"),
                   help="headline warm-up: the synthetic-stream generator (default) or the measured kernel itself")
    p.add_argument("--plan", action="store_true",
                   help="print every rank's shard (gloo, no GPU use) and exit: launch-path check")
    p.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                   help="process group of the N>1 ranks: nccl (= RCCL over xGMI, one rank per GPU) or gloo "
                        "(timing barrier, max and digest gather on host tensors; ranks share devices "
                        "round-robin, so --gpus 2 runs on a one-GPU box)")
    return p.parse_args(argv)


def spawn_ranks(a, argv):
    """`--gpus N` run directly: start N ranks (one process per GPU) with
    torch.distributed.run as a CHILD process, before this process touches the
    GPU, and exit with its status."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def _free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def global_count(scaling, world, per_gpu, global_count_strong):
    return per_gpu * world if scaling == "weak" else global_count_strong


def shard_bounds(rank, world, per_gpu, scaling="weak", global_count_strong=None):
    """(first buffer, buffers) of rank r: lcb_hash_partition of the global
    batch into `world` work-balanced contiguous parts.  Weak scaling: the
    global batch is world x per_gpu (rank r owns [r*per_gpu, (r+1)*per_gpu));
    strong: a fixed global_count_strong buffers."""
    assert 0 <= rank < world
    total = global_count(scaling, world, per_gpu, global_count_strong)
    first = liblcb_amd.partition(world, count=total, fixed_len=MSG_LEN)
    return int(first[rank]), int(first[rank + 1] - first[rank])


def all_shards(rank, world, first, count):
    """[(first, count)] of every rank (gathered as objects: the launch check)."""
    if world == 1:
        return [[first, count]]
    allp = [None] * world
    dist.all_gather_object(allp, [first, count])
    return allp


def max_over_ranks(t, world):
    """The job time is the slowest rank's (barrier-bracketed) time."""
    if world == 1:
        return t
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    tt = torch.tensor([t], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def settle(seconds=0.4, launch=None):
    """Bring the GPU to a loaded clock/power state before a timed segment:
    `seconds` of back-to-back `launch()` calls, by default the
    synthetic-stream generator writing a 256 MiB scratch buffer (so
    rocprofv3's per-kernel statistics of the measured kernels only hold
    steady-state launches).  Measured on MI355X: the first ~100 launches of
    a cold 0.2 ms kernel swing 205-292 us while the power manager reacts
    (profiles/r1b_bench_kernel_trace.csv).  `--settle self` warms up with the
    measured kernel instead: in fresh processes alternating on one box the
    two gave the same headline (5,185 vs 5,188 GiB/s over three pairs, the
    in-run clock 1.80-1.99 GHz either way; profiles/r7_settle_ab.txt)."""
    scratch = None
    if launch is None:
        scratch = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")

        def launch():
            liblcb_amd.gen_synthetic(1, scratch.numel(), out=scratch)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            launch()
        torch.cuda.synchronize()
    del scratch


CLOCK_SLOTS = 4096        # clock-stamp workgroups: ~16 per CU, so every CU stamps in both grids


class ClockWindow:
    """Engine clock of the timed launches themselves:
    a lcb_hash_gpu_clock_stamp grid is enqueued on the launch stream right
    before the timed region (then synchronised, so the stamp is not inside
    the wall time) and again right after its closing synchronise.  s_memtime
    is a per-CU shader-cycle counter (the CUs' counters differ by arbitrary
    offsets; s_memrealtime is one 100 MHz clock for the chip), so the stamps
    are paired per CU (XCC_ID and HW_ID's CU / SH / SE fields): per CU,
    clock = Δ s_memtime ÷ Δ s_memrealtime × 100 MHz over the window; the
    median over CUs is `clock_GHz` (min / max beside it).  The HIP-event span
    of the launches over the window's real time says how much of the window
    the kernels filled (`busy`).  `counter_residual_cycles`: the largest
    spread of one CU's begin stamps after removing the real time at its
    clock (small: the CU's stamps read one counter)."""

    def __init__(self, stream):
        self.sp = stream.cuda_stream
        self.buf = torch.zeros((2, CLOCK_SLOTS, 3), dtype=torch.int64, device="cuda")

    def _stamp(self, k):
        check(lib().lcb_hash_gpu_clock_stamp(self.buf[k].data_ptr(), CLOCK_SLOTS, self.sp))

    def begin(self):
        self._stamp(0)
        torch.cuda.synchronize()

    def end(self):
        self._stamp(1)
        torch.cuda.synchronize()

    @staticmethod
    def _by_cu(rows):
        key = ((rows[:, 0] >> np.uint64(32)) << np.uint64(8)) | ((rows[:, 0] >> np.uint64(8)) & np.uint64(0xFF))
        out = {}
        for k in np.unique(key):
            out[int(k)] = rows[key == k]
        return out

    def result(self, busy_ms=None):
        s = self.buf.cpu().numpy().view(np.uint64)
        b, e = self._by_cu(s[0]), self._by_cu(s[1])
        clocks, xcds, resid = [], set(), 0.0
        for k in sorted(set(b) & set(e)):
            bt, br = np.median(b[k][:, 1].astype(np.float64)), np.median(b[k][:, 2].astype(np.float64))
            et, er = np.median(e[k][:, 1].astype(np.float64)), np.median(e[k][:, 2].astype(np.float64))
            if er <= br or et <= bt:
                continue
            f = (et - bt) / (er - br) * 0.1          # GHz (100 MHz real-time ticks)
            clocks.append(f)
            xcds.add(k >> 8)
            r = b[k][:, 1].astype(np.float64) - b[k][:, 2].astype(np.float64) * f * 10.0
            resid = max(resid, float(r.max() - r.min()))
        if not clocks:
            return None
        win_ms = float(np.median(s[1, :, 2].astype(np.float64)) - np.median(s[0, :, 2].astype(np.float64))) * 1e-5
        out = {"clock_GHz": round(float(np.median(clocks)), 4), "clock_GHz_min": round(min(clocks), 4),
               "clock_GHz_max": round(max(clocks), 4), "cus": len(clocks), "xcds": len(xcds),
               "window_ms": round(win_ms, 4), "counter_residual_cycles": int(resid)}
        if busy_ms:
            out["busy"] = round(busy_ms / win_ms, 4) if win_ms > 0 else None
        return out


def valu_frac_at(vfloor_ms, clock, kms, cpi=None):
    """The VALU issue floor (valu_floor_ms: 4 cycles per instruction at
    2.4 GHz) at the clock the timed launches ran at, over their kernel time;
    with `cpi` (valu_cpi) the floor at the kernel's own measured cycles per
    VALU instruction instead of the 4-cycle model."""
    if not vfloor_ms or not clock or not clock.get("clock_GHz"):
        return None
    f = vfloor_ms * (VALU_CLOCK_HZ / 1e9) / clock["clock_GHz"] / kms
    if cpi:
        f *= cpi / VALU_CYCLES
    return round(f, 4)


# The kernel each algorithm's occupancy pass measured (sha224 / sha384 /
# gost512 run the same body as their siblings).
_OCC_SIBLING = {"sha224": "sha256", "sha384": "sha512", "gost512": "gost256"}


def valu_cpi(alg):
    """Cycles per VALU instruction of this algorithm's kernel: 4 (the
    mixed-stream model of DESIGN.md 5), or fewer when the PMC occupancy pass
    (profiles/valu_counts.json: SQ_ACTIVE_INST_VALU x 4 over the same pass's
    SQ_BUSY_CYCLES, one run, its own clock) saw the kernel issue faster than
    that -- its mix holds full-rate operations (v_xor / v_bitop3 / v_add_u32
    at 2.2-2.6 cycles alone, profiles/r1_valu_rate.txt): MD5 3.73, GOST 3.82,
    SHA-512 3.91, SHA-256 3.94, SHA-1 4.00 (r7p).  The floor can then not read
    above 1 merely because the model is 4 cycles."""
    name = ALG_NAMES[alg]
    try:
        algs = json.load(open(os.path.join(ROOT, "profiles", "valu_counts.json")))["algs"]
        rec = algs[_OCC_SIBLING.get(name, name)]
        if not counters_current(rec):
            return None
        u = float(rec["occupancy"]["valu_issue_util_median"])
    except (OSError, ValueError, KeyError):
        return None
    return round(VALU_CYCLES / max(1.0, u), 3)


def hash_launch(alg, data, digests, count, stream, key=None):
    return lib().lcb_hash_batch(alg, key, len(key) if key else 0, data.data_ptr(), None, None, count,
                                MSG_LEN, MSG_LEN, digests.data_ptr(), F_DEVICE, stream)


def time_alg(alg, data, digests, count, steps, warmup, world, key=None):
    """Returns (wall seconds for `steps` passes, max over ranks; mean kernel
    ms; this rank's engine clock over the timed launches, ClockWindow).

    The kernel time is the HIP-event span of the timed region on the launch
    stream divided by `steps` (back-to-back launches, so it is the average
    launch duration plus the inter-kernel gap).  Events around every launch
    add ~6 us per step on MI355X (tools/step_overhead.py), so only the two
    ends are recorded.  The clock stamps sit outside the wall-time bracket."""
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    for _ in range(warmup):
        check(hash_launch(alg, data, digests, count, sp, key))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cw = ClockWindow(stream)
    cw.begin()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        check(hash_launch(alg, data, digests, count, sp, key))
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    cw.end()
    span = e0.elapsed_time(e1)
    kms = span / steps
    return max_over_ranks(t, world), kms, cw.result(span)


def counters_current(rec):
    """True when a committed counter record (profiles/pmc_<alg>.json,
    valu_counts.json) was measured on the kernel code the loaded library
    runs: the sha256 of that kernel's machine code in the library
    (tools/codestamp.py) equals the record's stamp.  A record of an earlier
    build (or without a stamp) is never reported against this one."""
    from liblcb_amd._lib import LIB_PATH
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import codestamp
    try:
        return bool(rec.get("kernel_symbol")) and codestamp.stamp_of(LIB_PATH, rec["kernel_symbol"]) == \
            rec.get("code_sha256")
    except (OSError, ValueError):
        return False


def pmc_traffic(alg, count):
    """HBM bytes per launch from a committed rocprofv3 PMC summary, corrected
    as MI355X_MICROARCH.md prescribes (FETCH_SIZE reads 1/2 of a wide
    coalesced stream on gfx950: doubled; WRITE_SIZE exact; both in KiB);
    None unless the record's code stamp matches the loaded kernel."""
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % ALG_NAMES[alg])
    if not os.path.exists(path):
        return None
    try:
        j = json.load(open(path))
        if j.get("count") != count or j.get("msg_len") != MSG_LEN or not counters_current(j):
            return None
        return float(j["hbm_bytes_per_launch"])
    except (ValueError, KeyError):
        return None


VALU_CYCLES = 4.0        # cycles per wave64 VALU instruction in a mixed stream
VALU_SIMDS = 1024        # 256 CUs x 4 SIMDs
VALU_CLOCK_HZ = 2.4e9    # MI355X max engine clock (MI355X_MICROARCH.md)


def valu_floor_ms(alg, count):
    """VALU issue floor of one launch on the bench workload: the committed
    SQ_INSTS_VALU count (profiles/valu_counts.json, rocprofv3 --pmc) x 4
    cycles / (1,024 SIMDs x 2.4 GHz).  None without a count for this shape,
    or when the count's code stamp does not match the loaded kernel."""
    path = os.path.join(ROOT, "profiles", "valu_counts.json")
    try:
        j = json.load(open(path))
        if j.get("count") != count or j.get("msg_len") != MSG_LEN:
            return None
        rec = j["algs"][ALG_NAMES[alg]]
        if not counters_current(rec):
            return None
        n = float(rec["SQ_INSTS_VALU"])
    except (OSError, ValueError, KeyError):
        return None
    return n * VALU_CYCLES / (VALU_SIMDS * VALU_CLOCK_HZ) * 1e3


LDS_BYTES_PER_CLK_CU = 256   # ds_read_b64 array rate per CU (MI355X_MICROARCH.md LDS)
N_CUS = 256


def gost_lds_array(name, count, kernel_ms, clock=None):
    """GOST against the LDS array's peak: the table
    gathers' bytes -- 1 KiB message = 17 g_N + 2 g_0 = 19 g x 25 LPS, each 64
    ds_read_b64 of 8 B: 475 x 512 B -- over the kernel time, as a fraction of
    256 B/clk/CU x 256 CUs at 2.4 GHz and at the timed launches' clock, plus the
    bank-conflict share of the LDS-array cycles from the committed counters
    (profiles/pmc_gost_lds.json, when its code stamp matches)."""
    lps = (MSG_LEN // 64 + 1 + 2) * 25
    gbytes = count * lps * 64 * 8
    out = {"lds_gather_bytes": gbytes,
           "lds_array_frac": round(gbytes / (kernel_ms * 1e-3) / (LDS_BYTES_PER_CLK_CU * N_CUS * VALU_CLOCK_HZ), 4)}
    try:
        rec = json.load(open(os.path.join(ROOT, "profiles", "pmc_gost_lds.json")))["kernels"][name]
        if counters_current(rec):
            out["lds_bank_conflict_share"] = rec["bank_conflict_share"]
    except (OSError, ValueError, KeyError):
        pass
    clk = clock.get("clock_GHz") if clock else None
    if clk:   # at the clock of the timed launches themselves
        out["lds_array_frac_run_clock"] = round(gbytes / (kernel_ms * 1e-3) / (LDS_BYTES_PER_CLK_CU * N_CUS * clk * 1e9), 4)
    return out


def read_probes(data, count, steps=50, warmup=20):
    """Achievable HBM read rate on this box, GB/s: the digest
    kernels' own LDS-DMA line stream over the same records without the
    compression ("records"), and plain coalesced 16-B loads over the same
    bytes ("linear"); lcb_hash_gpu_read_probe, HIP events around each launch."""
    stream = torch.cuda.current_stream()
    out = {}
    for name, mode in (("records", 0), ("linear", 1)):
        sink = torch.empty(max(1, lib().lcb_hash_gpu_probe_sink_words(mode, count)), dtype=torch.int32,
                           device="cuda")

        def launch():
            check(lib().lcb_hash_gpu_read_probe(mode, data.data_ptr(), count, MSG_LEN, MSG_LEN,
                                                sink.data_ptr(), stream.cuda_stream))
        for _ in range(warmup):
            launch()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for e0, e1 in ev:
            e0.record(stream)
            launch()
            e1.record(stream)
        torch.cuda.synchronize()
        ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev]))
        out[name + "_GBps"] = round(count * MSG_LEN / (ms * 1e-3) / 1e9, 1)
        out[name + "_ms"] = round(ms, 4)
        del sink
    return out


def gost_lps_floor_ms(count, steps=10, warmup=3):
    """GOST's real bound on this box: the plain GOST kernel's
    LDS table gathers alone -- lcb_hash_gpu_read_probe LCB_PROBE_GOST_LPS,
    the kernel's grid, LDS image and occupancy running each lane's 475 LPS
    (1 KiB message: 19 g x 25) as one chain with no loads, no Sigma.  Mean
    HIP-event ms per launch."""
    stream = torch.cuda.current_stream()
    sink = torch.empty(count, dtype=torch.int32, device="cuda")

    def launch():
        check(lib().lcb_hash_gpu_read_probe(2, None, count, MSG_LEN, MSG_LEN, sink.data_ptr(), stream.cuda_stream))
    ms = _event_ms(launch, warmup, steps, stream)
    del sink
    return ms


def affinity_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def host_threads():
    """Threads the CPU baseline uses: the CPUs this process may run on
    (sched_getaffinity), capped by the container's CPU quota (cgroup
    cpu.max) when one is set — on the GPU box the affinity mask shows the
    whole machine while the quota is the box's CPU share."""
    n = affinity_cpus()
    q = cgroup_cpus()
    if q:
        n = min(n, max(1, int(q + 0.5)))
    return n


def cgroup_cpus():
    """CPU quota of this container (cgroup v2 cpu.max), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def _ref_rate(r, alg, data, count, threads, min_s):
    """GiB/s of the reference over the first `count` buffers, repeated until
    `min_s` wall seconds; returns (rate, seconds, digests, reps)."""
    r.batch_fixed_mt(alg, data[:MSG_LEN * 256], 256, MSG_LEN, MSG_LEN, threads=threads)
    reps, t0 = 0, time.perf_counter()
    while True:
        d = r.batch_fixed_mt(alg, data, count, MSG_LEN, MSG_LEN, threads=threads)
        reps += 1
        t = time.perf_counter() - t0
        if t >= min_s:
            return reps * count * MSG_LEN / t / 2**30, t, d, reps


def cpu_baseline(alg, count, threads):
    """The reference's include/crypto path (oracle/_ref, compiled from the
    reference headers) on this host's cores, over the same 1M x 1 KiB bytes.
    Falls back to reporting the oracle restatement (kind "port") only if the
    reference build is absent."""
    from oracle.pyoracle import REF_SIMD_SO, REF_SO, Oracle, Ref, gen_stream
    data = gen_stream(SEED, count * MSG_LEN)
    res = {}
    for kind, path in (("reference", REF_SO), ("reference-simd", REF_SIMD_SO)):
        if os.path.exists(path):
            res[kind] = _ref_rate(Ref(path), alg, data, count, threads, CPU_SAMPLE_S)
    if not res:
        o = Oracle()
        t0 = time.perf_counter()
        d = o.batch_fixed_mt(alg, data, count, MSG_LEN, MSG_LEN, threads=threads)
        t = time.perf_counter() - t0
        res["port"] = (count * MSG_LEN / t / 2**30, t, d, 1)
    best = max(res, key=lambda k: res[k][0])
    path = {"reference": REF_SO, "reference-simd": REF_SIMD_SO}.get(best)
    one = t16 = taff = None
    if path:
        r = Ref(path)
        n1 = min(count, 1 << 18)
        one = _ref_rate(r, alg, data, n1, 1, 0.0)[0]               # one pass, one thread
        if threads != 16:
            t16 = _ref_rate(r, alg, data, count, 16, 0.5)[0]       # the box's nominal CPU share
        if affinity_cpus() != threads:
            # every CPU of the affinity mask, whatever the quota allows
            taff = _ref_rate(r, alg, data, count, affinity_cpus(), 0.5)[0]
    return best, res, one, t16, taff, data


def cpu_per_alg(data, threads, best):
    """Reference CPU rate of every algorithm measured exactly as the headline
    cpu_baseline: whole passes over the full workload (all buffers, one
    contiguous shard per thread), repeated for >= 0.3 s wall, the build
    `best` picked for the headline.  (Round 2 timed 64K-buffer samples, so
    the threads' start-up was in every pass and the rates read ~1.5x low.)"""
    from oracle.pyoracle import REF_SIMD_SO, REF_SO, Ref
    path = {"reference": REF_SO, "reference-simd": REF_SIMD_SO}.get(best)
    if not path or not os.path.exists(path):
        return {}
    r = Ref(path)
    out = {}
    n = len(data) // MSG_LEN
    for name, aid in sorted(ALG_IDS.items(), key=lambda x: x[1]):
        rate, t, _, reps = _ref_rate(r, aid, data, n, threads, 0.3)
        out[name] = {"GiB_s": round(rate, 3), "buffers": n * reps, "threads": threads, "seconds": round(t, 3)}
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def fixture_dod(alg, total):
    """Reference digest-of-digests for the global fixed-stride batch of
    `total` x 1 KiB buffers (seed SEED), or None if no fixture covers it."""
    name = ALG_NAMES[alg]
    if total == MSGS_PER_GPU:
        b = json.load(open(os.path.join(ROOT, "tests", "golden", "batches.json")))
        for e in b["batches"]:
            if e["name"] == "C3_1M_x_1k" and e["alg"] == name and "key" not in e:
                return e["dod"]
    if total == 8 * MSGS_PER_GPU:
        j = json.load(open(os.path.join(ROOT, "tests", "golden", "large.json")))
        return j["C5_8M_x_1k"]["algs"][name]["dod"]
    return None


def verify_job(alg, digests, total):
    """The whole job's digests (host array, global order) against the
    reference: the digest-of-digests fixture when one covers `total`, else
    (k x 1M buffers, k <= 8: the 2- and 4-GPU weak-scaling jobs) each 1M
    block against the C5 fixture's per-shard digest-of-digests, which are the
    same bytes (tests/golden/large.json).  True / False / None (no fixture)."""
    exp = fixture_dod(alg, total)
    if exp:
        return hashlib.sha256(digests.tobytes()).hexdigest() == exp
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "large.json")))["C5_8M_x_1k"]
    sh = fx["shard"]
    if total % sh or total // sh > len(fx["algs"][ALG_NAMES[alg]]["shard_dod"]):
        return None
    want = fx["algs"][ALG_NAMES[alg]]["shard_dod"]
    return all(hashlib.sha256(digests[k * sh:(k + 1) * sh].tobytes()).hexdigest() == want[k]
               for k in range(total // sh))


def gather_digests(digests, first, n, total, world, rank):
    """RCCL gather of every rank's digests to rank 0; the
    shards are padded to the largest.  Returns (host array on rank 0, ms)."""
    D = digests.shape[1]
    if world == 1:
        torch.cuda.synchronize()
        return digests.cpu().numpy(), 0.0
    first_all = liblcb_amd.partition(world, count=total, fixed_len=MSG_LEN)
    mx = int(np.max(np.diff(first_all.astype(np.int64))))
    # RCCL gathers device tensors; gloo gathers host tensors.
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    buf = torch.zeros((mx, D), dtype=torch.uint8, device=dev)
    buf[:n] = digests.to(dev)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    dist.gather(buf, parts, dst=0)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    if rank != 0:
        return None, ms
    out = [parts[r][:int(first_all[r + 1] - first_all[r])] for r in range(world)]
    return torch.cat(out).cpu().numpy(), ms


def bench_c4(algs, warmup, steps, count=MSGS_PER_GPU, key=None):
    """BASELINE configs[3]: 1M buffers, lengths {64 B, 1 KiB, 64 KiB} chosen by
    mix64(seed + i) % 3, packed, device resident.  The library
    buckets the ragged batch by length on the device (counted in the time).
    One pass per algorithm of `algs` over the same bytes (the first is the
    headline; MD5, SHA-1 and SHA-224/256 run the tile kernel, SHA-384/512 the
    LDS line stream and GOST the per-lane kernel over the bucketed order),
    each checked against
    the reference's digest-of-digests.  With `key`: HMAC rows (named
    hmac_<alg>), checked against the same batch with segmented waves off
    (LCB_TILE_SEGS=0), which no reference fixture covers."""
    from tests.golden_util import mixed_lengths
    lens = np.array(mixed_lengths(SEED, count), dtype=np.uint32)
    offs = np.zeros(count, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(lens.sum())
    data = liblcb_amd.gen_synthetic(SEED, total)
    dl = torch.as_tensor(lens.astype(np.int32), device="cuda")
    do = torch.as_tensor(offs.astype(np.int64), device="cuda")
    stream = torch.cuda.current_stream()
    try:
        ref = json.load(open(os.path.join(ROOT, "tests", "golden", "large.json")))["C4_1M_mixed"]
        if ref["count"] != count or ref["total_bytes"] != total:
            ref = None
    except (OSError, KeyError, ValueError):
        ref = None
    out = {}
    for alg in algs:
        D = DIGEST_SIZE[alg]
        dig = torch.empty((count, D), dtype=torch.uint8, device="cuda")

        def launch():
            check(lib().lcb_hash_batch(alg, key, len(key) if key else 0, data.data_ptr(), do.data_ptr(),
                                       dl.data_ptr(), count, 0, 0, dig.data_ptr(), F_DEVICE, stream.cuda_stream))
        n = steps if alg == algs[0] else 3
        for _ in range(warmup if alg == algs[0] else 1):
            launch()
        cw = ClockWindow(stream)
        cw.begin()
        t0 = time.perf_counter()
        for _ in range(n):
            launch()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / n
        cw.end()
        ab = total + count * (D + 12)          # bytes read once + digest + (u64 offset, u32 length)
        res = {"GiB_s": round(total / t / 2**30, 2), "ms_per_pass": round(t * 1e3, 3),
               "total_GiB": round(total / 2**30, 2), "buffers": count,
               "hbm_frac": round(ab / t / 1e9 / HBM_PEAK_GBS, 4),
               "clock": cw.result(t * n * 1e3),
               "lengths": "{64, 1024, 65536}[mix64(seed+i) % 3]", "bucketed": True}
        if key is not None:
            got = dig.cpu().numpy().tobytes()
            os.environ["LCB_TILE_SEGS"] = "0"
            launch()
            torch.cuda.synchronize()
            os.environ.pop("LCB_TILE_SEGS", None)
            res["digests_equal_unsegmented"] = got == dig.cpu().numpy().tobytes()
        elif ref is not None:
            res["dod_equals_reference"] = hashlib.sha256(dig.cpu().numpy().tobytes()).hexdigest() == \
                ref["algs"][ALG_NAMES[alg]]["dod"]
        out[("hmac_" if key is not None else "") + ALG_NAMES[alg]] = res
        del dig
    del data
    torch.cuda.empty_cache()
    return out


def _event_ms(launch, warmup, steps, stream, clock=False):
    """Mean HIP-event span per launch over `steps` back-to-back launches on
    `stream` (events at the two ends only), after `warmup` launches; with
    clock=True also the engine clock over those launches (ClockWindow)."""
    for _ in range(warmup):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cw = ClockWindow(stream) if clock else None
    if cw:
        cw.begin()
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(steps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    span = e0.elapsed_time(e1)
    if not cw:
        return span / steps
    cw.end()
    return span / steps, cw.result(span)


def bench_packets(warmup, steps, algs=("md5",), ref_clock=None):
    """The network-packet shape of the reference's caller (SURVEY.md 8(f) row 1,
    VERDICT r2 item 1): 1M RADIUS-sized packets, lengths uniform 20..4096 B
    (include/proto/radius.h:576), packed back to back at byte offsets as in a
    receive buffer (src/threadpool/threadpool_task.c:692-696); device
    resident, ragged batch bucketed by length on the device (counted in the
    time).  Rows: plain digest, HMAC (one key), and keyed batches with 64
    peer secrets (src/proto/radius_client.c:242,885,1025): HMAC
    (Message-Authenticator, radius.h:850-919) and H(m || K) (packet
    authenticator, radius.h:1315-1377); each checked against the reference's
    digest-of-digests (tests/golden/packets.json).  Algorithmic bytes = packet
    bytes + per packet (digest + 8 B offset + 4 B length [+ 4 B key index])."""
    from tests.golden_util import packet_key_index, packet_keys, packet_layout
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "packets.json")))
    offs, lens, total = packet_layout()
    count = len(lens)
    data = liblcb_amd.gen_synthetic(SEED, total)
    d_offs = torch.as_tensor(offs.astype(np.int64), device="cuda")
    d_lens = torch.as_tensor(lens.astype(np.int32), device="cuda")
    d_kidx = torch.as_tensor(packet_key_index().astype(np.int32), device="cuda")
    keys = [bytes(k) for k in packet_keys()]
    blob = np.frombuffer(b"".join(keys), np.uint8)
    klen = np.array([len(k) for k in keys], np.uint32)
    koff = np.zeros(len(keys), np.uint64)
    koff[1:] = np.cumsum(klen[:-1], dtype=np.uint64)
    hkey = bytes.fromhex(fx["hmac_key_hex"])
    stream = torch.cuda.current_stream()
    res = {"packets": count, "total_GiB": round(total / 2**30, 4), "lengths": "uniform 20..4096 B",
           "layout": "packed at byte offsets (%d of 16 alignments)" % len(np.unique(offs % 16)),
           "keys": len(keys), "bucketed": True}
    for alg_name in algs:
        alg = ALG_IDS[alg_name]
        D = DIGEST_SIZE[alg]
        dig = torch.empty((count, D), dtype=torch.uint8, device="cuda")
        rows = [("plain", None, None), ("hmac", hkey, None), ("keyed_hmac", None, 1), ("keyed_suffix", None, 3)]
        for kind, key, mode in rows:
            if mode and "keyed_%s_%s" % ({1: "hmac", 3: "suffix"}[mode], alg_name) not in fx["full"]:
                continue

            def launch():
                if mode:
                    check(lib().lcb_hash_batch_keyed(alg, mode, blob.ctypes.data, koff.ctypes.data,
                                                     klen.ctypes.data, len(keys), d_kidx.data_ptr(),
                                                     data.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(),
                                                     count, 0, 0, dig.data_ptr(), F_DEVICE, stream.cuda_stream))
                else:
                    check(lib().lcb_hash_batch(alg, key, len(key) if key else 0, data.data_ptr(),
                                               d_offs.data_ptr(), d_lens.data_ptr(), count, 0, 0,
                                               dig.data_ptr(), F_DEVICE, stream.cuda_stream))
            ms, clk = _event_ms(launch, warmup, steps, stream, clock=True)
            ab = total + count * (D + 12 + (4 if mode else 0))
            name = "%s_%s" % (kind, alg_name)
            ok = hashlib.sha256(dig.cpu().numpy().tobytes()).hexdigest() == fx["full"][name]["dod"]
            res[name] = {"GiB_s": round(total / (ms * 1e-3) / 2**30, 2), "ms_per_pass": round(ms, 4),
                         "hbm_frac": round(ab / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "clock": clk, "dod_equals_reference": ok}
            if ref_clock and clk and clk.get("clock_GHz"):
                # The row at the headline's clock: the
                # same pass time scaled by this row's clock over the
                # headline's (a VALU-issue-bound pass scales with the clock).
                res[name]["hbm_frac_at_headline_clock"] = round(
                    res[name]["hbm_frac"] * ref_clock / clk["clock_GHz"], 4)
        del dig
    del data, d_offs, d_lens, d_kidx
    torch.cuda.empty_cache()
    return res


def bench_crc(data, count, steps):
    """CRC-32 family (include/math/crc32.h) over the same
    1M x 1 KiB device-resident bytes: per-variant kernel time (HIP events,
    after 3 warm launches) and HBM fraction of the algorithmic bytes
    (count x (1024 + 4))."""
    from liblcb_amd.crc32 import CRC_NAMES
    out_t = torch.empty(count, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    res = {}

    def crc_launch(v):
        check(lib().lcb_crc32_batch(v, None, data.data_ptr(), None, None, count, MSG_LEN, MSG_LEN,
                                    out_t.data_ptr(), F_DEVICE, stream.cuda_stream))
    # HBM-bound after VALU-bound rows: the memory side's clocks ramp back
    # over tens of ms (the variants timed in a row ran 0.51 -> 0.69 of HBM
    # with 10 warm launches each, r8d), so the family is warmed for 150 ms
    # first; then each variant: 10 warm launches and `steps` timed between
    # two events.
    t_end = time.time() + 0.15
    while time.time() < t_end:
        for _ in range(20):
            crc_launch(next(iter(CRC_NAMES)))
        torch.cuda.synchronize()
    for v, name in CRC_NAMES.items():
        for _ in range(10):
            crc_launch(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            crc_launch(v)
        e1.record(stream)
        torch.cuda.synchronize()
        km = e0.elapsed_time(e1) / steps
        res[name] = {"GiB_s": round(count * MSG_LEN / (km * 1e-3) / 2**30, 2), "kernel_ms": round(km, 4),
                     "hbm_frac": round(count * (MSG_LEN + 4) / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    del out_t
    return res


def bench_chacha(data, count, steps):
    """ChaCha / XChaCha (include/crypto/cipher/chacha.h)
    over the same 1M x 1 KiB device-resident bytes, iv_i = i: per-variant
    kernel time (HIP events on the launch stream, after 30 warm launches) and
    HBM fraction of the algorithmic bytes (count x (1024 read + 1024 written
    + 8 B iv); keystream-only: 1024 written + 8)."""
    dst = torch.empty_like(data)
    ivs = torch.arange(count, dtype=torch.int64, device="cuda").view(torch.uint8)
    ivs24 = torch.zeros((count, 24), dtype=torch.uint8, device="cuda")
    ivs24[:, 16:] = ivs.view(count, 8)
    key = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(range(32)))
    stream = torch.cuda.current_stream()
    res = {}
    for name, x, rounds, enc in (("chacha20", 0, 20, True), ("chacha12", 0, 12, True), ("chacha8", 0, 8, True),
                                 ("chacha20_keystream", 0, 20, False), ("xchacha20", 1, 20, True)):
        iv = ivs24 if x else ivs

        def launch():
            check(lib().lcb_chacha_batch(x, key, 32, None, iv.data_ptr(), rounds,
                                         data.data_ptr() if enc else None, dst.data_ptr(), None, None,
                                         count, MSG_LEN, MSG_LEN, F_DEVICE, stream.cuda_stream))
        for _ in range(30):
            launch()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        for e0, e1 in ev:
            e0.record(stream)
            launch()
            e1.record(stream)
        torch.cuda.synchronize()
        km = sum(e0.elapsed_time(e1) for e0, e1 in ev) / steps
        ab = count * (MSG_LEN * (2 if enc else 1) + (24 if x else 8))
        res[name] = {"GiB_s": round(count * MSG_LEN / (km * 1e-3) / 2**30, 2), "kernel_ms": round(km, 4),
                     "hbm_frac": round(ab / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "bound": "valu" if rounds == 20 else "hbm"}
    del dst, ivs24
    return res


def _cgroup_throttle():
    """(throttled periods, throttled us) of this process's cgroup CPU quota,
    or None where no cpu.stat is readable (cgroup v2, then v1)."""
    for f, scale in (("/sys/fs/cgroup/cpu.stat", 1.0), ("/sys/fs/cgroup/cpu/cpu.stat", 1e-3),
                     ("/sys/fs/cgroup/cpu,cpuacct/cpu.stat", 1e-3)):
        try:
            kv = dict(ln.split()[:2] for ln in open(f) if len(ln.split()) >= 2)
        except OSError:
            continue
        us = kv.get("throttled_usec")
        us = float(us) if us is not None else float(kv.get("throttled_time", 0)) * scale
        return int(kv.get("nr_throttled", 0)), us
    return None


def bench_ingest(alg_id, packets=1 << 21, threads=8):
    """Asynchronous ingestion queue (include/lcb_hash_queue.h, SURVEY.md 8f
    row 2): `threads` native producer threads submit 1 KiB packets from host
    memory.  Three runs of tools/queue_bench (a child process): saturation
    (producers as fast as they can: packets/s; its latency is queueing behind
    an overload by construction), open loop at half that rate (packets due
    on a fixed schedule, latency counted from the due time: the latency a
    caller below capacity sees), and the producers' memcpy alone (the
    host-side ceiling)."""
    exe = os.path.join(ROOT, "tools", "queue_bench")
    if not os.path.exists(exe):
        return {"skipped": "tools/queue_bench not built"}
    base = [exe, "--alg", str(alg_id), "--packets", str(packets), "--size", str(MSG_LEN),
            "--threads", str(threads)]

    def run(extra):
        # LCB_QUEUE_TRACE=1: the queue logs every stall over 1 ms (a slow
        # launch step, a batch picked up late by the completion thread, the
        # flusher waiting for a free slot, a submit waiting for an open
        # slot) with its time in the run; the host's CPU throttling (cgroup
        # cpu.stat) is read around the run, so a stall caused by the box's
        # CPU quota shows as such in the record.
        env = dict(os.environ, LCB_QUEUE_TRACE="1")
        t0 = _cgroup_throttle()
        r = subprocess.run(base + extra, capture_output=True, text=True, timeout=300, env=env)
        t1 = _cgroup_throttle()
        if r.returncode != 0:
            raise RuntimeError(r.stderr.strip()[-300:])
        out = json.loads(r.stdout.strip().splitlines()[-1])
        out["stall_trace"] = [ln.strip() for ln in r.stderr.splitlines() if "lcb_hash_queue:" in ln][:12]
        out["cgroup_throttled"] = None if t0 is None or t1 is None else \
            {"periods": t1[0] - t0[0], "us": round(t1[1] - t0[1], 1)}
        return out
    try:
        sat = run([])
        half = run(["--rate", str(int(sat["packets_per_s"] / 2))])
        copy = run(["--copy-only", "1"])
        zc = run(["--zerocopy", "1"])
        zc_half = run(["--zerocopy", "1", "--rate", str(int(zc["packets_per_s"] / 2))])
    except RuntimeError as e:
        return {"error": str(e)}
    def stages(r):
        # The queue's per-stage maxima of the run (lcb_hash_queue_stats), so
        # each run attributes its own latency tail: first
        # packet -> seal, seal -> enqueued, GPU, callbacks, longest blocked
        # submit; where the worst packet sat in the run; blocked submits.
        # The slowest launch's own steps ride along.
        return {k: r.get(k) for k in ("max_fill_us", "max_launch_us", "max_launch_steps_us", "max_gpu_us",
                                      "max_callback_us", "max_submit_wait_us", "submit_waits", "worst_at",
                                      "lat_us_max", "late_half_p99", "stall_trace", "cgroup_throttled")}
    return {"packets_per_s": sat["packets_per_s"], "GiB_s": sat["GiB_s"], "batches": sat["batches"],
            # Zero-copy submit (LCB_HASH_Q_F_ZEROCOPY): packets already in a
            # registered page-locked pool (the io_buf receive buffers,
            # include/utils/io_buf.h:40-47) are recorded by address and DMA'd in
            # place -- no producer memcpy.
            "zerocopy": {"packets_per_s": zc["packets_per_s"], "GiB_s": zc["GiB_s"], "batches": zc["batches"],
                         "saturated_lat_us_p50": zc["lat_us_p50"], "saturated_lat_us_p99": zc["lat_us_p99"],
                         "half_load_lat_us_p50": zc_half["lat_us_p50"], "half_load_lat_us_p99": zc_half["lat_us_p99"],
                         "saturated_stages": stages(zc), "half_load_stages": stages(zc_half),
                         "path": "registered page-locked packet -> bulk H2D run copy (or read in place) -> kernel writes digests to pinned memory -> callback"},
            "saturated_stages": stages(sat), "half_load_stages": stages(half),
            "saturated_lat_us_p50": sat["lat_us_p50"], "saturated_lat_us_p99": sat["lat_us_p99"],
            "half_load_packets_per_s": half["packets_per_s"], "half_load_lat_us_p50": half["lat_us_p50"],
            "half_load_lat_us_p99": half["lat_us_p99"], "half_load_lat_us_p999": half["lat_us_p999"],
            "zerocopy_half_load_lat_us_p999": zc_half["lat_us_p999"],
            "half_load_lat_us_max": half["lat_us_max"], "threads": threads, "packet_bytes": MSG_LEN,
            "settings": "64K packets / 64 MiB / 200 us / 4 slots", "copy_only_GiB_s": copy["GiB_s"],
            "path": "producer memcpy into pinned lease -> H2D -> kernel -> D2H -> per-packet callback"}


def plan(a, world, rank):
    """--plan: the launch and sharding path without the GPU (gloo): every
    rank reports its shard, rank 0 prints them as one JSON line."""
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == a.gpus
    first, count = shard_bounds(rank, world, a.count, a.scaling, a.global_count)
    me = {"rank": rank, "world_size": dist.get_world_size() if world > 1 else 1, "first": first,
          "count": count, "pid": os.getpid()}
    allp = [None] * world
    if world > 1:
        dist.all_gather_object(allp, me)
        dist.destroy_process_group()
    else:
        allp = [me]
    if rank == 0:
        print(json.dumps({"plan": allp, "scaling": a.scaling,
                          "total": global_count(a.scaling, world, a.count, a.global_count)}), flush=True)
    return 0


def main():
    argv = sys.argv[1:]
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(a, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, a.gpus))
    if a.plan:
        return plan(a, world, rank)
    ndev = max(1, torch.cuda.device_count())   # does not initialise the GPU
    if world > 1:
        # One rank per GPU (LOCAL_RANK); with gloo more ranks than GPUs share
        # them round-robin.
        local = local % ndev
        torch.cuda.set_device(local)
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == a.gpus, (dist.get_world_size(), a.gpus)
    else:
        torch.cuda.set_device(0)
    alg = ALG_IDS[a.alg]
    D = DIGEST_SIZE[alg]

    # Rank r hashes its lcb_hash_partition shard of the global synthetic batch.
    total = global_count(a.scaling, world, a.count, a.global_count)
    first, count = shard_bounds(rank, world, a.count, a.scaling, a.global_count)
    data = liblcb_amd.gen_synthetic(SEED, max(count, 1) * MSG_LEN, start=first * MSG_LEN)
    digests = torch.empty((max(count, 1), D), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    sp = torch.cuda.current_stream().cuda_stream
    settle(launch=(lambda: check(hash_launch(alg, data, digests, count, sp))) if a.settle == "self" else None)
    t, kms, clock = time_alg(alg, data, digests, count, a.steps, a.warmup, world)
    value = total * MSG_LEN * a.steps / t / 2**30
    alg_bytes = count * (MSG_LEN + D)      # read every message once + write its digest
    achieved = alg_bytes / (kms * 1e-3) / 1e9
    traffic = pmc_traffic(alg, count)
    vfloor = valu_floor_ms(alg, count)
    out = {
        "metric": "device-resident GiB/s hashed, 1M x 1 KiB buffers per GPU",
        "value": round(value, 3),
        "unit": "GiB/s",
        # Physical devices the ranks ran on: a gloo run with more ranks than
        # GPUs shares them round-robin, and then says so (never a scaling point).
        "n_gpus": min(world, ndev),
        "ranks_share_devices": world > ndev,
        "world_size": dist.get_world_size() if world > 1 else 1,
        "dist_backend": a.dist_backend if world > 1 else None,
        "shards": all_shards(rank, world, first, count),
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(t / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": a.scaling,
        "vs_baseline": None,
        "dtype": "u32" if alg not in (5, 6, 7, 8) else "u64",
        "data": "synthetic (device-generated splitmix64 stream, SURVEY.md 8d)",
        "config": {"workload": "%s digest of %d x %d B buffers over %d GPU(s), %s scaling"
                               % (a.alg, total, MSG_LEN, world, a.scaling),
                   "alg": a.alg, "buffers_per_gpu": count, "buffer_bytes": MSG_LEN,
                   "total_buffers": total, "parallelism": "shard%d" % world + ("" if world <= ndev else
                                                                             " (ranks share %d GPU(s))" % ndev),
                   "split": "lcb_hash_partition (work-balanced contiguous shards)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel_ms": round(kms, 4),
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "valu_floor_ms": round(vfloor, 4) if vfloor else None,
                     "valu_frac": round(vfloor / kms, 4) if vfloor else None,
                     # engine clock of the timed launches (rank 0's), and the
                     # VALU floor at that clock
                     "clock": clock,
                     # the same with a flat 4 cycles per VALU instruction:
                     # a model check, not a fraction (above 1 where the mix
                     # issues faster, hence valu_cpi)
                     "valu_4cycle_model_ratio": valu_frac_at(vfloor, clock, kms),
                     "valu_cpi": valu_cpi(alg),
                     "valu_frac_run_clock": valu_frac_at(vfloor, clock, kms, valu_cpi(alg))},
    }
    from liblcb_amd._lib import LIB_PATH
    out["library_sha256_16"] = hashlib.sha256(open(LIB_PATH, "rb").read()).hexdigest()[:16]
    # (Round 5 scaled the floor by the clock of the separate PMC pass
    # instead, valu_frac_pmc_clock: a different run's clock, which put three
    # of them above 1 -- VERDICT r5.  The floor is now taken at the clock of
    # the timed launches themselves, `clock` above.)

    if rank == 0 and world == 1 and not a.no_extras:
        # Achievable read rate on this box next to the spec peak: the same
        # records through the kernel's line stream without compression, and a
        # plain linear read (not `value`; the fraction against spec stays `frac`).
        pr = read_probes(data, count)
        r = out["roofline"]
        r["achievable"] = pr
        r["frac_of_stream"] = round(achieved / pr["records_GBps"], 4)
        r["frac_of_linear_read"] = round(achieved / pr["linear_GBps"], 4)

    if not a.no_gather:
        # RCCL digest gather to rank 0 (outside the timed region), then the
        # whole job's digests against the reference's digest-of-digests.
        allg, gms = gather_digests(digests[:count], first, count, total, world, rank)
        if rank == 0:
            ok = verify_job(alg, allg, total)
            got = hashlib.sha256(allg.tobytes()).hexdigest()
            out["gather"] = {"ms": round(gms, 3), "bytes": int(allg.nbytes),
                             "collective": ("gather (%s)" % ("RCCL" if a.dist_backend == "nccl" else "gloo"))
                             if world > 1 else "none (1 rank)"}
            out.setdefault("verify", {})["job_digests_equal_reference"] = ok
            out["verify"]["digest_of_digests"] = got

    if rank == 0 and world == 1 and not a.no_extras:
        settle()
        per = {}
        for name, aid in sorted(ALG_IDS.items(), key=lambda x: x[1]):
            dg = torch.empty((count, DIGEST_SIZE[aid]), dtype=torch.uint8, device="cuda")
            tt, km, ck = time_alg(aid, data, dg, count, max(3, a.steps // 4), 10, 1)
            ab = count * (MSG_LEN + DIGEST_SIZE[aid])
            vf = valu_floor_ms(aid, count)
            per[name] = {"GiB_s": round(count * MSG_LEN * max(3, a.steps // 4) / tt / 2**30, 2),
                         "kernel_ms": round(km, 4),
                         "hbm_frac": round(ab / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "valu_frac": round(vf / km, 4) if vf else None,
                         "clock": ck, "valu_cpi": valu_cpi(aid),
                         "valu_4cycle_model_ratio": valu_frac_at(vf, ck, km),
                         "valu_frac_run_clock": valu_frac_at(vf, ck, km, valu_cpi(aid))}
            if name.startswith("gost"):
                # GOST is bound by its LDS table gathers, not HBM or VALU:
                # the gathers alone, same grid and image, beside the kernel.
                if "lps_chain_ms" not in per.get("gost256", {}):
                    lps_ms = gost_lps_floor_ms(count)
                else:
                    lps_ms = per["gost256"]["lps_chain_ms"]
                per[name]["lps_chain_ms"] = round(lps_ms, 4)
                per[name]["lds_frac"] = round(lps_ms / km, 4)
                per[name].update(gost_lds_array(name, count, km, ck))
            del dg
        out["per_alg"] = per
        # Batched HMAC (RADIUS needs HMAC-MD5): per call
        # the ipad/opad mid-states are computed on the device (one tiny prep
        # kernel), then every message costs its blocks + 1 outer compression.
        hm = {}
        key = bytes(range(16))
        for name in ("md5", "sha1", "sha256", "sha512"):
            aid = ALG_IDS[name]
            dg = torch.empty((count, DIGEST_SIZE[aid]), dtype=torch.uint8, device="cuda")
            tt, km, ck = time_alg(aid, data, dg, count, max(3, a.steps // 4), 10, 1, key=key)
            hm["hmac_" + name] = {"GiB_s": round(count * MSG_LEN * max(3, a.steps // 4) / tt / 2**30, 2),
                                  "call_ms": round(km, 4), "key_bytes": len(key),
                                  "clock_GHz": ck["clock_GHz"] if ck else None}
            del dg
        out["hmac"] = hm
        c4 = bench_c4([alg] + [ALG_IDS[n] for n in ("sha1", "sha256", "sha512", "gost256") if ALG_IDS[n] != alg],
                      a.warmup, max(3, a.steps // 4))
        out["ragged_c4"] = c4.pop(ALG_NAMES[alg])
        # The other algorithms on C4 (SHA-1/256: the tile kernel; SHA-512:
        # the LDS line stream over the bucketed order; GOST: the per-lane
        # kernel), with their fixed-stride rate for comparison: VALU-bound, so
        # ragged ~ fixed means the ragged machinery is hidden.  The per-block
        # ratio also counts the compressions each byte costs (C4's padding
        # blocks are ~0.3 % of its bytes, 1 KiB records' 6 % / 12.5 %).
        from tests.golden_util import mixed_lengths_np
        c4_lens = mixed_lengths_np(SEED, MSGS_PER_GPU).astype(np.uint64)
        for name, r in c4.items():
            if name in per:
                r["fixed_stride_GiB_s"] = per[name]["GiB_s"]
                blk = {"sha384": (128, 16), "sha512": (128, 16)}.get(name, (64, 8))

                def blocks_per_byte(lens):
                    if name.startswith("gost"):
                        # Streebog: floor(len / 64) full blocks + 1 padded
                        # block, then the N and Sigma finalisation
                        # compressions (gost3411-2012.h)
                        return float(((lens // 64) + 3).sum() * 64) / float(lens.sum())
                    return float(((lens + 1 + blk[1] + blk[0] - 1) // blk[0]).sum() * blk[0]) / float(lens.sum())
                r["fixed_stride_ratio_per_block"] = round(
                    r["GiB_s"] / per[name]["GiB_s"] * blocks_per_byte(c4_lens) /
                    blocks_per_byte(np.array([MSG_LEN], np.uint64)), 3)
                # the same at equal engine clocks (both passes' in-run
                # clocks: VALU-bound kernels scale with it)
                if r.get("clock") and per[name].get("clock"):
                    r["fixed_stride_ratio_per_block_equal_clock"] = round(
                        r["fixed_stride_ratio_per_block"] * per[name]["clock"]["clock_GHz"] /
                        r["clock"]["clock_GHz"], 3)
        # HMAC on C4 (segmented long waves through the
        # HMAC tile kernel's one copy; MD5, SHA-1, SHA-256), each with its
        # per-compression ratio to the fixed-stride HMAC row above (HMAC: one
        # outer compression more per message).
        c4hs = bench_c4([ALG_IDS[n] for n in ("md5", "sha1", "sha256")], 1, 3, key=key)

        def hmac_blocks_per_byte(lens):
            return float((((lens + 1 + 8 + 63) // 64) + 1).sum() * 64) / float(lens.sum())
        for hname, c4h in c4hs.items():
            fx = hm[hname]
            c4h["fixed_stride_GiB_s"] = fx["GiB_s"]
            c4h["fixed_stride_ratio_per_block"] = round(
                c4h["GiB_s"] / fx["GiB_s"] * hmac_blocks_per_byte(c4_lens) /
                hmac_blocks_per_byte(np.array([MSG_LEN], np.uint64)), 3)
            if c4h.get("clock") and fx.get("clock_GHz"):
                c4h["fixed_stride_ratio_per_block_equal_clock"] = round(
                    c4h["fixed_stride_ratio_per_block"] * fx["clock_GHz"] / c4h["clock"]["clock_GHz"], 3)
            c4[hname] = c4h
        out["ragged_c4_per_alg"] = c4
        out["ragged_packets"] = bench_packets(10, max(3, a.steps // 4),
                                              ref_clock=clock["clock_GHz"] if clock else None)
        out["crc32"] = bench_crc(data, count, max(3, a.steps // 4))
        settle()   # ChaCha20 is VALU-heavy: let the clock settle after the HBM-bound CRC launches
        out["chacha"] = bench_chacha(data, count, max(3, a.steps // 4))
        out["ingest"] = bench_ingest(alg)
        # End-to-end host path on the same bytes (lcb_hash_batch host mode):
        # pinned input is DMA'd straight from the caller's buffer, pageable
        # input is gathered into pinned staging first; 64 MiB chunks on two
        # streams, H2D -> kernel -> D2H digests.
        host = data.cpu().pin_memory()
        hd = np.empty((count, D), dtype=np.uint8)
        e2e = {}
        for kind, arr in (("pinned", host.numpy()), ("pageable", np.array(host.numpy()))):
            liblcb_amd.hash_batch(alg, arr[:64 * MSG_LEN], count=64, stride=MSG_LEN, fixed_len=MSG_LEN)
            best = 1e9
            for _ in range(3):
                t0 = time.perf_counter()
                liblcb_amd.hash_batch(alg, arr, count=count, stride=MSG_LEN, fixed_len=MSG_LEN, out=hd)
                best = min(best, time.perf_counter() - t0)
            e2e[kind + "_GiB_s"] = round(count * MSG_LEN / best / 2**30, 3)
        # The link alone: one pinned 1 GiB host -> device copy (the ceiling of
        # the pinned row above).
        scratch = torch.empty_like(data)
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            scratch.copy_(host, non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        e2e["h2d_copy_only_GiB_s"] = round(host.numel() / best / 2**30, 3)
        del scratch
        e2e["path"] = "host buffer -> 64 MiB chunks, 2 streams, H2D -> kernel -> D2H digests"
        out["e2e"] = e2e
        torch.cuda.synchronize()
        gpu_dig = digests.cpu().numpy()
        out.setdefault("verify", {})["e2e_equals_device"] = bool(np.array_equal(hd, gpu_dig))

    if rank == 0 and world == 1 and not a.no_cpu:
        threads = a.cpu_threads or host_threads()
        best, res, one, t16, taff, cdata = cpu_baseline(alg, count, threads)
        gbs, tcpu, dcpu, reps = res[best]
        gpu_dig = digests[:count].cpu().numpy()
        out["cpu_baseline"] = {
            "value": round(gbs, 3), "unit": "GiB/s", "cores": threads, "kind": "reference"
            if best.startswith("reference") else "port",
            "build": best, "sample": "the full workload (%d x %d B, %s) hashed %d times on %d threads "
            "(min of sched_getaffinity %d and the cgroup CPU quota), one contiguous shard per thread, %.1f s wall"
            % (count, MSG_LEN, a.alg, reps, threads, affinity_cpus(), tcpu),
            "affinity_cpus": affinity_cpus(),
            "all": {k: round(v[0], 3) for k, v in res.items()},
            "one_thread": round(one, 3) if one else None,
            "at_16_threads": round(t16, 3) if t16 else None,
            "at_affinity_threads": round(taff, 3) if taff else None,
            "cgroup_cpus": cgroup_cpus(),
            "cpu_model": cpu_model(),
            "build_flags": {"reference": "gcc -O2 -fPIC, #undef __SSE2__ (as tests/hash/main.c:36)",
                            "reference-simd": "gcc -O2 -fPIC -msse4.1 -mssse3 -msha -mavx2 (cpuid dispatch)"},
            "seconds": round(tcpu, 3)}
        cpa = cpu_per_alg(cdata, threads, best)
        for name, v in cpa.items():
            if name in out.get("per_alg", {}):
                out["per_alg"][name]["cpu_GiB_s"] = v["GiB_s"]
        out["cpu_baseline"]["per_alg"] = cpa
        out.setdefault("verify", {})["gpu_equals_cpu_reference"] = bool(np.array_equal(gpu_dig, dcpu))

    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
