"""bench.py's N>1 path on ONE GPU: `--gpus 2
--dist-backend gloo` spawns two ranks that share device 0, each hashes its
lcb_hash_partition shard of the 2M x 1 KiB weak-scaling job, the slowest
rank's time is the job time, the digests are gathered to rank 0 and checked
block by block against the reference's C5 per-shard digest-of-digests
(bench.verify_job's shard branch).  The RCCL variant of the same code path is
what the driver's 8-GPU node runs.

The 8-rank strong-scaling case runs the driver's C5 split
(8M x 1 KiB over 8 ranks, lcb_hash_partition) with all eight ranks on
device 0: the shards, the per-shard device generation at the shard's offset,
the max-over-ranks timing and the gather are the N=8 code path; the record
says ranks_share_devices, never a scaling point."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _run_bench(args, timeout):
    import torch
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    return json.loads(line), torch.cuda.device_count()


def _check_shards(j, total):
    sh = sorted(j["shards"])
    assert j["config"]["total_buffers"] == total
    assert sh[0][0] == 0 and sh[-1][0] + sh[-1][1] == total       # covering
    assert all(a[0] + a[1] == b[0] for a, b in zip(sh, sh[1:]))   # contiguous, disjoint


def test_bench_two_ranks_gloo_one_gpu():
    j, ndev = _run_bench(["--gpus", "2", "--dist-backend", "gloo", "--steps", "5", "--warmup", "2",
                          "--no-extras", "--no-cpu"], 240)
    assert j["world_size"] == 2 and j["dist_backend"] == "gloo"
    # the physical devices used, not the rank count (ranks share a 1-GPU box)
    assert j["n_gpus"] == min(2, ndev) and j["ranks_share_devices"] == (ndev < 2)
    assert j["verify"]["job_digests_equal_reference"] is True
    assert j["gather"]["collective"] == "gather (gloo)"
    _check_shards(j, 2 << 20)
    assert j["value"] > 0


def test_bench_eight_ranks_strong_c5_one_gpu():
    """C5 (BASELINE configs[4]): 8M x 1 KiB split over 8 ranks, strong scaling."""
    j, ndev = _run_bench(["--gpus", "8", "--dist-backend", "gloo", "--scaling", "strong", "--steps", "3",
                          "--warmup", "1", "--no-extras", "--no-cpu"], 420)
    assert j["world_size"] == 8 and j["scaling"] == "strong"
    assert j["n_gpus"] == min(8, ndev) and j["ranks_share_devices"] == (ndev < 8)
    _check_shards(j, 8 << 20)
    assert sorted(c for _, c in j["shards"]) == [1 << 20] * 8      # equal work: equal counts
    assert j["verify"]["job_digests_equal_reference"] is True      # the C5 fixture's digest-of-digests
