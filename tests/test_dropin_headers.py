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


SIMD_FLAGS = ["-msse4.1", "-mssse3", "-msha", "-mavx2"]


@pytest.fixture(scope="module", params=["generic", "simd"])
def driver(tmp_path_factory, request):
    """The KAT driver built plain, and with the SHA extensions enabled (the
    reference's SIMD build flags): SHA-224/256 then run on SHA-NI when the
    CPU has it (sha2.h sha2_transform_block64_shani)."""
    return build(tmp_path_factory.mktemp("dropin"), os.path.join(C, "dropin_driver.c"), "drv",
                 extra=SIMD_FLAGS if request.param == "simd" else ())


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
@pytest.mark.parametrize("simd", [False, True])
def test_ctx_layouts_match_reference(tmp_path, simd):
    """sizeof / alignment / offsetof of every context struct equal the
    reference's, in the generic build (as tests/hash) and with SSE4.1 /
    SHA-NI / AVX2 enabled (the reference's build-dependent fields)."""
    flags = ["-DLAYOUT_SIMD", "-msse4.1", "-mssse3", "-msha", "-mavx2"] if simd else []
    outs = []
    for inc in (os.path.join(REF, "include"), INC):
        exe = str(tmp_path / ("lay%d" % len(outs)))
        subprocess.check_call(["gcc", "-O0", "-w"] + flags + ["-I" + inc, "-o", exe, os.path.join(C, "layout.c")])
        outs.append(subprocess.check_output([exe]).decode())
    assert outs[0] == outs[1]
    assert "sha1_ctx_t %d 32" % (480 if simd else 448) in outs[1]


def test_gost_table_is_read_only_data():
    """The drop-in GOST table is static const data (no first-use build, no
    mutable global): SURVEY.md 8(b) threading contract."""
    src = open(os.path.join(INC, "crypto", "hash", "gost3411-2012.h")).read()
    tab = open(os.path.join(INC, "crypto", "hash", "gost3411-2012-lps.h")).read()
    assert "static const uint64_t gost3411_2012_T[8][256]" in tab
    assert "__atomic" not in src and "static uint64_t" not in src and "static int" not in src


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent")
def test_reference_radius_sign_verify_with_dropin(tmp_path):
    """The reference's RADIUS code (oracle/ref_radius.c over include/proto/
    radius.h) built against THIS repo's md5.h signs the packets of
    tests/golden/radius.json to the same bytes the reference-header build
    produced, and its radius_pkt_verify accepts them and decodes the same
    passwords."""
    import ctypes
    import json
    so = str(tmp_path / "libradius_dropin.so")
    subprocess.check_call(["gcc", "-O2", "-w", "-shared", "-fPIC", "-I" + INC, "-I" + os.path.join(REF, "include")] +
                          HAVE + ["-o", so, os.path.join(ROOT, "oracle", "ref_radius.c")])
    pp = subprocess.check_output(["gcc", "-E", "-I" + INC, "-I" + os.path.join(REF, "include")] + HAVE +
                                 [os.path.join(ROOT, "oracle", "ref_radius.c")]).decode()
    assert os.path.join(INC, "crypto/hash/md5.h") in pp
    L = ctypes.CDLL(so)
    sz = ctypes.c_size_t
    L.ref_rad_verify.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.c_char_p, ctypes.c_void_p]
    L.ref_rad_authenticator_calc.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.c_int,
                                             ctypes.c_char_p, ctypes.c_void_p]
    L.ref_rad_msg_authenticator_calc.argtypes = L.ref_rad_authenticator_calc.argtypes
    L.ref_rad_password_encode.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_char_p, sz,
                                          ctypes.c_void_p, sz, ctypes.POINTER(sz)]
    j = json.load(open(os.path.join(ROOT, "tests", "golden", "radius.json")))
    secrets = [bytes.fromhex(s) for s in j["secrets"]]
    L.ref_rad_sign.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.c_void_p, ctypes.POINTER(sz)]
    out = ctypes.create_string_buffer(4096)
    a16 = ctypes.create_string_buffer(16)
    ol = sz()
    for p in j["packets"]:
        pre = bytes.fromhex(p["pre"])
        assert L.ref_rad_sign(pre, len(pre), secrets[p["key"]], len(secrets[p["key"]]), out, ctypes.byref(ol)) == 0
        assert out.raw[:ol.value].hex() == p["signed"]      # radius_pkt_sign on the drop-in md5.h
        pkt = bytes.fromhex(p["signed"])
        k = secrets[p["key"]]
        req = bytes.fromhex(p["request"]) if p["kind"] == "reply" else None
        assert L.ref_rad_verify(pkt, len(pkt), k, len(k), req, out) == 0
        assert out.raw[:len(pkt)].hex() == p["verified"]
        if p["kind"] == "reply":
            assert L.ref_rad_authenticator_calc(pkt, len(pkt), k, len(k), 0, req, a16) == 0
            assert a16.raw.hex() == p["authenticator_calc"]
        if p["msg_authr"]:
            assert L.ref_rad_msg_authenticator_calc(pkt, len(pkt), k, len(k), 0, req, a16) == 0
    el = sz()
    for v in j["password_encode"]:
        pw, k = bytes.fromhex(v["password"]), secrets[v["key"]]
        assert L.ref_rad_password_encode(bytes.fromhex(v["authenticator"]), pw, len(pw), k, len(k), out, 256,
                                         ctypes.byref(el)) == 0
        assert out.raw[:el.value].hex() == v["encoded"]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent")
def test_threadpool_queue_integration_compiles(tmp_path):
    """INTEGRATION.md section 3 as a translation unit (tests/c/threadpool_queue.c):
    a tp_task_pkt_rcvr_cb that submits to lcb_hash_queue and returns the
    digest with tpt_msg_send compiles against the REFERENCE's thread-pool
    headers; its only external references are liblcb's thread-pool calls
    and this repo's queue ABI, which liblcb_hash_gpu.so exports."""
    obj = str(tmp_path / "tpq.o")
    subprocess.check_call(["gcc", "-c", "-O2", "-Wall", "-Werror", "-Wno-unused-function", "-Wno-unused-variable",
                           "-I" + INC, "-I" + os.path.join(REF, "include")] + HAVE +
                          ["-o", obj, os.path.join(C, "threadpool_queue.c")])
    und = set(l.split()[-1] for l in subprocess.check_output(["nm", "-u", obj]).decode().splitlines())
    ours = {"lcb_hash_queue_create", "lcb_hash_queue_settings_def", "lcb_hash_queue_submit"}
    assert ours | {"tpt_get_current", "tpt_msg_send"} <= und
    assert und - ours - {"tpt_get_current", "tpt_msg_send"} <= {"calloc", "free", "malloc", "memcpy",
                                                                 "__stack_chk_fail"}
    so = os.path.join(ROOT, "liblcb_amd", "liblcb_hash_gpu.so")
    if os.path.exists(so):
        exported = subprocess.check_output(["nm", "-D", "--defined-only", so]).decode()
        assert all((" T " + s) in exported for s in ours)
