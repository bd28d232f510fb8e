"""HBM read probes (include/lcb_hash_gpu.h lcb_hash_gpu_read_probe): the
bench's achievable-bandwidth numbers only count if the probes read every byte
they claim to.  Records mode folds each record's whole 128-B lines into one
word (XOR), linear mode folds its grid-stride share per thread; both are
checked against numpy on the same bytes."""
import errno

import numpy as np
import pytest
import torch

from oracle.pyoracle import gen_stream

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import liblcb_amd
    return liblcb_amd.lib()


@pytest.mark.parametrize("count,stride,flen", [(64, 1024, 1024), (1000, 1024, 1024), (777, 1040, 1000),
                                               (4096 + 5, 256, 200)])
def test_records_probe_reads_every_line(L, count, stride, flen):
    host = gen_stream(count + flen, count * stride)
    data = torch.as_tensor(host, device="cuda")
    sink = torch.zeros(count, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert L.lcb_hash_gpu_probe_sink_words(0, count) == count
    assert L.lcb_hash_gpu_read_probe(0, data.data_ptr(), count, stride, flen, sink.data_ptr(), s) == 0
    torch.cuda.synchronize()
    nl = flen // 128
    words = host.reshape(count, stride)[:, :nl * 128].copy().view(np.uint32).reshape(count, -1)
    exp = np.bitwise_xor.reduce(words, axis=1) if nl else np.zeros(count, np.uint32)
    assert np.array_equal(sink.cpu().numpy().view(np.uint32), exp)


def test_linear_probe_reads_every_byte(L):
    n = (3 << 20) + 48
    host = gen_stream(11, n)
    data = torch.as_tensor(host, device="cuda")
    words = L.lcb_hash_gpu_probe_sink_words(1, 1)
    assert words > 0
    sink = torch.zeros(words, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert L.lcb_hash_gpu_read_probe(1, data.data_ptr(), n // 16, 16, 16, sink.data_ptr(), s) == 0
    torch.cuda.synchronize()
    got = np.bitwise_xor.reduce(sink.cpu().numpy().view(np.uint32))
    assert got == np.bitwise_xor.reduce(host.view(np.uint32))


def test_probe_rejects_bad_shapes(L):
    data = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    p, q = data.data_ptr(), sink.data_ptr()
    assert L.lcb_hash_gpu_read_probe(0, p, 63, 1024, 1024, q, s) == errno.EINVAL     # < 64 records
    assert L.lcb_hash_gpu_read_probe(0, p, 64, 1024, 100, q, s) == errno.EINVAL      # no whole line
    assert L.lcb_hash_gpu_read_probe(0, p + 8, 64, 1024, 1024, q, s) == errno.EINVAL  # misaligned
    assert L.lcb_hash_gpu_read_probe(1, p, 3, 5, 5, q, s) == errno.EINVAL            # not 16-B multiple
    assert L.lcb_hash_gpu_read_probe(2, p, 0, 1024, 1024, q, s) == errno.EINVAL      # GOST LPS: no lanes
    assert L.lcb_hash_gpu_read_probe(2, p, 64, 1024, 1024, 0, s) == errno.EINVAL      # GOST LPS: no sink
    assert L.lcb_hash_gpu_read_probe(3, p, 64, 1024, 1024, q, s) == errno.EINVAL     # unknown mode
    assert L.lcb_hash_gpu_read_probe(2, p, 64, 1024, 1024, q, s) == 0                # GOST LPS chain runs
    torch.cuda.synchronize()


def test_clock_stamp(L):
    """lcb_hash_gpu_clock_stamp (bench.py ClockWindow): every XCD appears,
    real time and shader cycles advance over a busy window, and the clock
    they give lies in the MI355X's range (the engine clock tops out at
    2.4 GHz).  Bad shapes are EINVAL."""
    import liblcb_amd
    import bench
    s = torch.cuda.current_stream()
    buf = torch.zeros((4096, 3), dtype=torch.int64, device="cuda")
    assert L.lcb_hash_gpu_clock_stamp(buf.data_ptr(), 63, s.cuda_stream) == errno.EINVAL
    assert L.lcb_hash_gpu_clock_stamp(buf.data_ptr(), 0, s.cuda_stream) == errno.EINVAL
    assert L.lcb_hash_gpu_clock_stamp(None, 64, s.cuda_stream) == errno.EINVAL
    data = liblcb_amd.gen_synthetic(1, 1 << 28)
    cw = bench.ClockWindow(s)
    cw.begin()
    for _ in range(40):
        liblcb_amd.gen_synthetic(2, data.numel(), out=data)
    torch.cuda.synchronize()
    cw.end()
    st = cw.buf.cpu().numpy().view(np.uint64)
    assert len(set(int(v) >> 32 for v in st[0, :, 0])) == 8
    assert (st[1, :, 2] > st[0, :, 2]).all()      # one real-time clock for the chip
    r = cw.result()
    print(r)
    assert r["xcds"] == 8 and r["cus"] >= 200, r   # stamps of (nearly) every CU in both grids
    assert 0.3 < r["clock_GHz_min"] <= r["clock_GHz_max"] < 2.6, r
    assert r["counter_residual_cycles"] < 1e6, r
