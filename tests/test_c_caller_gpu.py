"""The batch C-ABI from a plain C program (tests/c/batch_caller.c, built
with gcc against include/ and liblcb_amd/liblcb_hash_gpu.so): ragged,
misaligned packets in pageable host memory through the reference-named
*_get_digest_batch entry points, every digest equal to the drop-in headers'
single-message call (the CPU path the reference's callers compile)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "liblcb_amd")

pytestmark = pytest.mark.gpu


def test_c_caller_batches_equal_dropin_single_message(tmp_path):
    exe = str(tmp_path / "batch_caller")
    subprocess.check_call(["gcc", "-O2", "-Wall", "-Werror", "-Wno-unused-function",
                           "-I" + os.path.join(ROOT, "include"), "-o", exe,
                           os.path.join(ROOT, "tests", "c", "batch_caller.c"),
                           "-L" + LIBDIR, "-llcb_hash_gpu", "-Wl,-rpath," + LIBDIR])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK 3000 "), r.stdout


def test_c_caller_multi_stream_contract(tmp_path):
    """lcb_hash_batch_multi (ABI v4) ordered after the caller's stream:
    tests/c/multi_stream.c writes the batch asynchronously on a non-default
    stream and calls with no host sync; digests equal md5.h's."""
    exe = str(tmp_path / "multi_stream")
    subprocess.check_call(["gcc", "-O2", "-Wall", "-Werror", "-Wno-unused-function", "-D__HIP_PLATFORM_AMD__",
                           "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include", "-o", exe,
                           os.path.join(ROOT, "tests", "c", "multi_stream.c"),
                           "-L" + LIBDIR, "-llcb_hash_gpu", "-Wl,-rpath," + LIBDIR,
                           "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK 65536"), r.stdout
