"""bench.py's N>1 path on ONE GPU: `--gpus 2
--dist-backend gloo` spawns two ranks that share device 0, each hashes its
lcb_hash_partition shard of the 2M x 1 KiB weak-scaling job, the slowest
rank's time is the job time, the digests are gathered to rank 0 and checked
block by block against the reference's C5 per-shard digest-of-digests
(bench.verify_job's shard branch).  The RCCL variant of the same code path is
what the driver's 8-GPU node runs."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_bench_two_ranks_gloo_one_gpu():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--steps", "5", "--warmup", "2", "--no-extras", "--no-cpu"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    j = json.loads(line)
    assert j["n_gpus"] == 2 and j["world_size"] == 2 and j["dist_backend"] == "gloo"
    assert j["verify"]["job_digests_equal_reference"] is True
    assert j["gather"]["collective"] == "gather (gloo)"
    sh = sorted(j["shards"])
    total = j["config"]["total_buffers"]
    assert total == 2 << 20
    assert sh[0][0] == 0 and sh[-1][0] + sh[-1][1] == total       # covering
    assert all(a[0] + a[1] == b[0] for a, b in zip(sh, sh[1:]))   # contiguous, disjoint
    assert j["value"] > 0
