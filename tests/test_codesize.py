"""Guard: the built library's code size and kernel list.

A library with segmented copies of every tile mode (33 MB) ran the
headline's first 20 timed fixed-stride steps 7 % slower than one without
(18 MB), the same kernel in fresh processes (DESIGN.md 9 finding 12,
profiles/r6_codesize_headline.txt).  This test reads the BUILT library
(tools/codesize.py) and fails when it is more than 10 % larger than the
committed record (tests/golden/codesize.json) or holds a kernel the record
does not list.  A deliberate change re-records with
`python3 tools/codesize.py --write` in the same commit."""
import json
import os
import runpy

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = runpy.run_path(os.path.join(ROOT, "tools", "codesize.py"))


@pytest.fixture(scope="module")
def now():
    if not os.path.exists(CS["SO"]):
        pytest.skip("library not built")
    kr = runpy.run_path(os.path.join(ROOT, "tools", "kernel_resources.py"))
    if not os.path.exists(kr["READELF"]):
        pytest.skip("llvm-readelf not available")
    return CS["measure"]()


@pytest.fixture(scope="module")
def rec():
    return json.load(open(CS["OUT"]))


def test_size_within_ten_percent(now, rec):
    assert now["so_bytes"] <= 1.10 * rec["so_bytes"], (now["so_bytes"], rec["so_bytes"])
    assert now["code_object_bytes"] <= 1.10 * rec["code_object_bytes"], \
        (now["code_object_bytes"], rec["code_object_bytes"])


def test_no_unlisted_kernel(now, rec):
    extra = sorted(set(now["kernels"]) - set(rec["kernels"]))
    assert not extra, "kernels not in tests/golden/codesize.json:\n" + "\n".join(extra)
