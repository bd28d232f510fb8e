import json, subprocess, sys, numpy as np
sys.path.insert(0, ".")
from oracle.pyoracle import SEED, gen_stream, Oracle
o = Oracle()
n, size = 1 << 16, 1024
want = o.batch_fixed_mt(1, gen_stream(SEED, n * size), n, size, size)
exe = sys.argv[1] if len(sys.argv) > 1 else 'tools/queue_bench'
for it in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    r = subprocess.run([exe, "--alg", "1", "--packets", str(n), "--size", str(size), "--threads", "8",
                        "--batch-msgs", "4096", "--out", "gpurun_out/dig.bin"], capture_output=True, text=True, timeout=120)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    got = np.fromfile("gpurun_out/dig.bin", np.uint8).reshape(n, 16)
    bad = np.nonzero((got != want).any(1))[0]
    if len(bad):
        lut = {bytes(want[k]): k for k in range(n)}
        src = [lut.get(bytes(got[k]), -1) for k in bad]
        per_thread = np.bincount(bad // (n // 8), minlength=8).tolist()
        found = [x for x in src if x >= 0]
        print("   per-thread", per_thread, "digest of another packet:", len(found), "of", len(bad),
              "offsets sample", [int(src[k] - bad[k]) if src[k] >= 0 else None for k in range(0, len(bad), max(1, len(bad) // 12))],
              "runs", np.split(bad, np.nonzero(np.diff(bad) != 1)[0] + 1).__len__(), flush=True)
    print(exe, it, "bad", len(bad), bad[:20].tolist(), "zero-digests", int((got == 0).all(1).sum()),
          {k: res[k] for k in ("batches", "sealed_full", "sealed_timer", "submit_waits")}, flush=True)
