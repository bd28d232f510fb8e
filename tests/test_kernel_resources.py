"""Guard: no product kernel spills to scratch.

Reads the AMDHSA metadata of the BUILT library's gfx950 code objects
(tools/kernel_resources.py: the offload bundle of every translation unit, its
kernel table via llvm-readelf) -- what the GPU loads, not a recompile -- and
fails on any kernel with a nonzero private (scratch) segment.  Scratch spills
are per-lane stores and reloads through the cache hierarchy: round 2's GOST
kernels moved 1.45-1.58x the algorithmic HBM bytes because of them."""
import os
import runpy

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "liblcb_amd", "liblcb_hash_gpu.so")
KR = runpy.run_path(os.path.join(ROOT, "tools", "kernel_resources.py"))


@pytest.fixture(scope="module")
def rows():
    if not os.path.exists(SO):
        pytest.skip("library not built")
    if not os.path.exists(KR["READELF"]):
        pytest.skip("llvm-readelf not available")
    return KR["kernels"](SO)


def test_every_kernel_listed(rows):
    names = [r["name"] for r in rows]
    for k in ("md_fixed_lds_kernel", "md_fixed_persist_kernel", "md_lines_kernel", "md_batch_kernel", "md_tiles_kernel", "md_keyed_kernel",
              "gost_plain2_kernel", "gost_hmac_kernel", "gost_keyed_kernel", "bucket_place_kernel", "crc_fixed_lds_kernel",
              "chacha_lane_kernel"):
        assert any(k in n for n in names), (k, sorted(names)[:20])
    assert len(rows) > 100


def test_no_scratch(rows):
    bad = ["%s: %d B/lane scratch, %d VGPRs" % (r["name"], r["scratch"], r["vgpr"]) for r in rows if r["scratch"]]
    assert not bad, "\n".join(bad)


def test_stream_kernels_keep_four_waves(rows):
    """The LDS-stream kernels are sized for 4 workgroups (4 waves each) per
    CU: 32 KiB of LDS per workgroup and at most 128 VGPRs (512 / 4 waves per
    SIMD).  More VGPRs would silently halve their occupancy."""
    ks = [r for r in rows if any(k in r["name"] for k in ("md_fixed_lds_kernel", "md_fixed_persist_kernel",
                                                          "md_lines_kernel"))]
    assert ks
    bad = ["%s: %d VGPRs" % (r["name"], r["vgpr"]) for r in ks if r["vgpr"] > 128]
    assert not bad, "\n".join(bad)
