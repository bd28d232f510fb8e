"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes access to the CPU checkers:
  * Oracle  — oracle/liblcb_oracle.so, the C restatement (lcb_oracle.c);
  * Ref     — oracle/_ref/libref_hash*.so, the reference's own headers
              compiled from /root/reference (present only if built here).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liblcb_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_hash.so")
REF_SIMD_SO = os.path.join(HERE, "_ref", "libref_hash_simd.so")
DSIZE = {1: 16, 2: 20, 3: 28, 4: 32, 5: 48, 6: 64, 7: 32, 8: 64}
SEED = 0x6C62636861736821

_c = ctypes


def build():
    """Build the oracle (and _ref where /root/reference exists)."""
    subprocess.check_call(["make", "-s", "-C", HERE])


def gen_stream(seed, nbytes, start=0):
    """Bytes [start, start+nbytes) of the synthetic stream: u64 word k is
    mix64(seed ^ k), little-endian."""
    w0 = start // 8
    nw = (start + nbytes + 7) // 8 - w0
    k = np.arange(w0, w0 + nw, dtype=np.uint64)
    z = (k ^ np.uint64(seed)) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    b = z.astype("<u8").view(np.uint8)
    off = start - w0 * 8
    return b[off:off + nbytes]


class _Batch:
    fn_batch = None

    def batch(self, alg, data, offsets=None, lengths=None, count=None, stride=0,
              fixed_len=0, key=None):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, dtype=np.uint8)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if lengths is not None:
            lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        if count is None:
            count = len(lengths) if lengths is not None else len(offsets)
        out = np.zeros((count, DSIZE[alg]), dtype=np.uint8)
        kb = bytes(key) if key is not None else None
        rc = self.fn_batch(alg, kb, len(kb) if kb is not None else 0, data.ctypes.data,
                           offsets.ctypes.data if offsets is not None else None,
                           lengths.ctypes.data if lengths is not None else None,
                           count, stride, fixed_len, out.ctypes.data)
        assert rc == 0, rc
        return out

    def batch_keyed(self, alg, mode, keys, data, key_index=None, offsets=None, lengths=None, count=None,
                    stride=0, fixed_len=0):
        """Keyed batch (or_batch_keyed / ref_batch_keyed): mode 1 HMAC, 2 H(K || m),
        3 H(m || K); keys: list of bytes."""
        blob = np.frombuffer(b"".join(keys) or b"\0", np.uint8)
        klen = np.array([len(k) for k in keys], np.uint32)
        koff = np.zeros(len(keys), np.uint64)
        koff[1:] = np.cumsum(klen[:-1], dtype=np.uint64)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if lengths is not None:
            lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        if key_index is not None:
            key_index = np.ascontiguousarray(key_index, dtype=np.uint32)
        if count is None:
            count = len(lengths) if lengths is not None else len(offsets)
        out = np.zeros((count, DSIZE[alg]), np.uint8)
        rc = self.fn_keyed(alg, mode, blob.ctypes.data, koff.ctypes.data, klen.ctypes.data, len(keys),
                                     key_index.ctypes.data if key_index is not None else None, data.ctypes.data,
                                     offsets.ctypes.data if offsets is not None else None,
                                     lengths.ctypes.data if lengths is not None else None, count, stride,
                                     fixed_len, out.ctypes.data)
        assert rc == 0, rc
        return out

    def batch_fixed_mt(self, alg, data, count, stride, fixed_len, key=None, threads=8):
        """Fixed-stride batch split into `threads` contiguous shards (ctypes
        releases the GIL, so the shards run in parallel)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        out = np.zeros((count, DSIZE[alg]), dtype=np.uint8)
        per = (count + threads - 1) // threads
        kb = bytes(key) if key is not None else None

        def work(t):
            lo, hi = t * per, min(count, (t + 1) * per)
            if lo < hi:
                self.fn_batch(alg, kb, len(kb) if kb is not None else 0,
                              data.ctypes.data + lo * stride, None, None, hi - lo, stride,
                              fixed_len, out.ctypes.data + lo * DSIZE[alg])
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(work, range(threads)))
        return out


_ARGS = [_c.c_int, _c.c_char_p, _c.c_size_t, _c.c_void_p, _c.c_void_p, _c.c_void_p,
         _c.c_size_t, _c.c_uint64, _c.c_uint32, _c.c_void_p]


_KEYED_ARGS = [_c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t,
               _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t,
               _c.c_uint64, _c.c_uint32, _c.c_void_p]

_CRC_ARGS = [_c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t,
             _c.c_uint64, _c.c_uint32, _c.c_void_p]
CRC_VARIANTS = {1: "crc32a", 2: "crc32cksum", 3: "crc32mpeg2", 4: "crc32b", 5: "crc32jamcrc",
                6: "crc32c", 7: "crc32d", 8: "crc32q"}


class _Crc:
    fn_crc = None

    def crc32_batch(self, variant, data, offsets=None, lengths=None, count=None, stride=0,
                    fixed_len=0, init=None):
        """crcs[i] = X(msg i), or X_update(init[i], msg i) (include/math/crc32.h)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, dtype=np.uint8)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if lengths is not None:
            lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        if count is None:
            count = len(lengths) if lengths is not None else len(offsets)
        if init is not None:
            init = np.ascontiguousarray(init, dtype=np.uint32)
        out = np.zeros(count, dtype=np.uint32)
        rc = self.fn_crc(variant, init.ctypes.data if init is not None else None, data.ctypes.data,
                         offsets.ctypes.data if offsets is not None else None,
                         lengths.ctypes.data if lengths is not None else None,
                         count, stride, fixed_len, out.ctypes.data)
        assert rc == 0, rc
        return out


_CHA_ARGS = [_c.c_void_p, _c.c_size_t, _c.c_size_t, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p,
             _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_uint64, _c.c_uint32]


class _Cha:
    fn_cha = None

    def chacha_batch(self, key, key_size, rounds, src, offsets=None, lengths=None, count=None,
                     stride=0, fixed_len=0, counters=None, ivs=None, x=False, nbytes=None):
        """dst with buffer i = chacha()/xchacha() of buffer i (chacha.h:650-679);
        src None -> keystream into a zeroed buffer of nbytes."""
        key = np.frombuffer(bytes(key), np.uint8)
        kbuf = np.zeros(max(32, key.size), np.uint8)
        kbuf[:key.size] = key
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if lengths is not None:
            lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        if count is None:
            count = len(lengths) if lengths is not None else len(offsets)
        if src is not None:
            src = np.ascontiguousarray(src, dtype=np.uint8)
            dst = np.zeros(max(src.size, 1), np.uint8)
        else:
            dst = np.zeros(max(int(nbytes), 1), np.uint8)
        if counters is not None:
            counters = np.ascontiguousarray(counters, dtype=np.uint8)
        if ivs is not None:
            ivs = np.ascontiguousarray(ivs, dtype=np.uint8)
        rc = self.fn_cha(kbuf.ctypes.data, key_size, rounds, 1 if x else 0,
                         counters.ctypes.data if counters is not None else None,
                         ivs.ctypes.data if ivs is not None else None,
                         src.ctypes.data if src is not None and src.size else None, dst.ctypes.data,
                         offsets.ctypes.data if offsets is not None else None,
                         lengths.ctypes.data if lengths is not None else None, count, stride, fixed_len)
        assert rc == 0, rc
        return dst


class Oracle(_Batch, _Crc, _Cha):
    """The C restatement."""

    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            build()
        self.lib = _c.CDLL(path)
        self.lib.or_batch.argtypes = _ARGS
        self.fn_batch = self.lib.or_batch
        self.lib.or_init.argtypes = [_c.c_void_p, _c.c_int]
        self.lib.or_update.argtypes = [_c.c_void_p, _c.c_char_p, _c.c_size_t]
        self.lib.or_final.argtypes = [_c.c_void_p, _c.c_char_p]
        self.lib.or_chacha_batch.argtypes = _CHA_ARGS
        self.fn_cha = self.lib.or_chacha_batch
        self.lib.or_crc32_batch.argtypes = _CRC_ARGS
        self.fn_crc = self.lib.or_crc32_batch
        self.lib.or_batch_keyed.argtypes = _KEYED_ARGS
        self.fn_keyed = self.lib.or_batch_keyed
        self.lib.or_crc32_table.restype = _c.c_uint32
        self.lib.or_crc32_table.argtypes = [_c.c_int, _c.c_int]

    def crc32_table(self, variant):
        return np.array([self.lib.or_crc32_table(variant, i) for i in range(256)], np.uint32)


    def chunked(self, alg, msg, chunks):
        """Streaming digest feeding `msg` in pieces of the given size."""
        ctx = _c.create_string_buffer(512)
        out = _c.create_string_buffer(64)
        assert self.lib.or_init(ctx, alg) == 0
        i = 0
        while i < len(msg):
            n = min(chunks, len(msg) - i)
            self.lib.or_update(ctx, msg[i:i + n], n)
            i += n
        self.lib.or_final(ctx, out)
        return out.raw[:DSIZE[alg]]


class Ref(_Batch, _Crc, _Cha):
    """The reference's own code (compiled from /root/reference into _ref/)."""

    def __init__(self, path=REF_SO):
        self.lib = _c.CDLL(path)
        self.lib.ref_batch.argtypes = _ARGS
        self.fn_batch = self.lib.ref_batch
        self.lib.ref_gost_ax.argtypes = [_c.c_void_p]
        self.lib.ref_chacha_batch.argtypes = _CHA_ARGS
        self.fn_cha = self.lib.ref_chacha_batch
        self.lib.ref_crc32_batch.argtypes = _CRC_ARGS
        self.fn_crc = self.lib.ref_crc32_batch
        self.lib.ref_crc32_table.argtypes = [_c.c_int, _c.c_void_p]
        if hasattr(self.lib, "ref_batch_keyed"):
            self.lib.ref_batch_keyed.argtypes = _KEYED_ARGS
            self.fn_keyed = self.lib.ref_batch_keyed

    def crc32_table(self, variant):
        t = np.zeros(256, np.uint32)
        assert self.lib.ref_crc32_table(variant, t.ctypes.data) == 0
        return t

    def crc32_self_test(self):
        return self.lib.ref_crc32_self_test()

    def chacha_self_test(self):
        return self.lib.ref_chacha_self_test()

    def chacha_kats(self):
        """chacha_self_test's vector table, decoded by the reference's own
        import helpers (chacha.h:968-1040)."""
        out = []
        i = 0
        while True:
            key = _c.create_string_buffer(32)
            cnt = _c.create_string_buffer(8)
            iv = _c.create_string_buffer(8)
            exp = _c.create_string_buffer(2048)
            plain = _c.create_string_buffer(2048)
            ks, rounds, size = _c.c_size_t(), _c.c_size_t(), _c.c_size_t()
            hc, hi, hp = _c.c_int(), _c.c_int(), _c.c_int()
            if self.lib.ref_chacha_kat(_c.c_size_t(i), key, _c.byref(ks), cnt, _c.byref(hc), iv, _c.byref(hi),
                                       _c.byref(rounds), _c.byref(size), exp, plain, _c.byref(hp)) != 0:
                return out
            out.append({"key": key.raw.hex(), "key_size": ks.value,
                        "counter": cnt.raw.hex() if hc.value else None,
                        "iv": iv.raw.hex() if hi.value else None, "rounds": rounds.value,
                        "plain": plain.raw[:size.value].hex() if hp.value else None,
                        "output": exp.raw[:size.value].hex()})
            i += 1

    @staticmethod
    def available(path=REF_SO):
        return os.path.exists(path)

    def gost_ax(self):
        t = np.zeros(2048, dtype=np.uint64)
        self.lib.ref_gost_ax(t.ctypes.data)
        return t
