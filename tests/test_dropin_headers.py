"""The drop-in headers include/crypto/hash/*.h: same API as the reference,
bit-exact on the reference's KAT tables, usable by the reference's own
callers (proto/radius.h) and its own test driver (tests/hash/main.c)."""
import os
import subprocess

import numpy as np
import pytest

from oracle.pyoracle import Oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
C = os.path.join(ROOT, "tests", "c")
REF = "/root/reference"
ALG = {"md5": 1, "sha1": 2, "sha224": 3, "sha256": 4, "sha384": 5, "sha512": 6,
       "gost256": 7, "gost512": 8}
# What the reference's CMake probes define so include/al/os.h agrees with glibc.
HAVE = ["-DHAVE_EXPLICIT_BZERO", "-DHAVE_MEMRCHR", "-DHAVE_MEMMEM", "-DHAVE_REALLOCARRAY",
        "-DHAVE_PIPE2", "-DHAVE_ACCEPT4", "-DHAVE_STRLCPY=0"]


def build(tmp_path, src, out, extra=(), inc=(INC,)):
    exe = str(tmp_path / out)
    cmd = ["gcc", "-O2", "-Wall", "-Werror", "-Wno-unused-function"] + \
          ["-I" + i for i in inc] + list(extra) + ["-o", exe, src]
    subprocess.check_call(cmd)
    return exe


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    return build(tmp_path_factory.mktemp("dropin"), os.path.join(C, "dropin_driver.c"), "drv")


def run_driver(exe, lines):
    out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         check=True).stdout.split()
    assert len(out) == len(lines)
    return out


def test_selftests(tmp_path):
    exe = build(tmp_path, os.path.join(C, "selftest_main.c"), "st")
    assert subprocess.run([exe]).returncode == 0


def kat_line(c, chunk):
    key = "-" if "key" not in c else (c["key"] or "=")
    return "%s %s %s %d %d" % (c["alg"], key, c["msg"] or "-", c.get("repeat", 1), chunk)


def test_reference_kat_tables(driver, kat):
    """All 217 reference KAT vectors, every chunked-update variant included."""
    lines, want = [], []
    for c in kat:
        for ch in (c.get("chunks") or [0]):
            lines.append(kat_line(c, ch))
            want.append(c["digest"])
    assert run_driver(driver, lines) == want
    assert len(lines) > 600


def test_random_vs_oracle(driver):
    o = Oracle()
    rng = np.random.RandomState(5)
    lines, exp = [], []
    for alg, aid in ALG.items():
        for _ in range(25):
            n = int(rng.randint(0, 600))
            m = rng.randint(0, 256, size=n).astype(np.uint8)
            chunk = int(rng.choice([0, 1, 7, 63, 64, 65, 200]))
            key = None if rng.rand() < 0.5 else rng.randint(0, 256, size=int(rng.randint(1, 200))).astype(np.uint8)
            lines.append("%s %s %s 1 %d" % (alg, key.tobytes().hex() if key is not None else "-",
                                            m.tobytes().hex() or "-", chunk))
            d = o.batch(aid, m if n else np.zeros(1, np.uint8), offsets=[0], lengths=[n],
                        key=None if key is None else key.tobytes())
            exp.append(d[0].tobytes().hex())
    assert run_driver(driver, lines) == exp


def test_sanitizers(tmp_path, kat):
    """Host-side ASan/UBSan build of the drop-in headers over the KAT tables."""
    exe = build(tmp_path, os.path.join(C, "dropin_driver.c"), "asan",
                extra=["-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"])
    cases = [(c, ch) for c in kat if c.get("repeat", 1) == 1 for ch in (c.get("chunks") or [0])[:3]]
    assert run_driver(exe, [kat_line(c, ch) for c, ch in cases]) == [c["digest"] for c, _ in cases]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent")
def test_reference_tests_hash_main_builds_against_dropin(tmp_path):
    """The reference's own KAT driver, unmodified, compiled against our headers."""
    exe = build(tmp_path, os.path.join(REF, "tests", "hash", "main.c"), "ref_main",
                extra=["-Wno-unused-variable", "-Wno-unused-parameter"])
    assert subprocess.run([exe]).returncode == 0


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent")
def test_reference_radius_builds_against_dropin(tmp_path):
    """The only in-tree caller (include/proto/radius.h:53) compiles unchanged,
    taking crypto/hash/md5.h from this repo (our include dir first)."""
    exe = str(tmp_path / "radius")
    subprocess.check_call(["gcc", "-O2", "-w", "-I" + INC, "-I" + os.path.join(REF, "include")] + HAVE +
                          ["-o", exe, os.path.join(C, "radius_dropin.c")])
    assert subprocess.run([exe]).returncode == 0
    # and the preprocessed unit really used our header
    pp = subprocess.check_output(["gcc", "-E", "-I" + INC, "-I" + os.path.join(REF, "include")] + HAVE +
                                 [os.path.join(C, "radius_dropin.c")]).decode()
    assert os.path.join(INC, "crypto/hash/md5.h") in pp
