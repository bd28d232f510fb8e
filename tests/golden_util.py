"""Rebuild the inputs of a tests/golden/batches.json entry (data, layout, key).

The fixtures hold seeds and layout rules, not bytes: the input is the
synthetic stream of oracle.pyoracle.gen_stream (host) or
liblcb_amd.gen_synthetic (device), which produce identical bytes.
"""
import hashlib

import numpy as np

SEED = 0x6C62636861736821
M64 = (1 << 64) - 1


def mixed_lengths(seed, count):
    out = []
    for i in range(count):
        z = (seed + i + 0x9E3779B97F4A7C15) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        z ^= z >> 31
        out.append((64, 1024, 65536)[z % 3])
    return out


def mixed_lengths_np(seed, count):
    """mixed_lengths, vectorised (uint32 array, same values)."""
    with np.errstate(over="ignore"):
        z = np.arange(count, dtype=np.uint64) + np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return np.array([64, 1024, 65536], np.uint32)[(z % np.uint64(3)).astype(np.int64)]


def layout(entry):
    """-> dict(seed, nbytes, offsets|None, lengths|None, count, stride, fixed_len, key)."""
    name = entry["name"]
    key = bytes.fromhex(entry["key_hex"]) if "key_hex" in entry else None
    if name.startswith("ragged_0_4159") or name == "mixed_512":
        lens = (np.arange(4160, dtype=np.uint32) if name.startswith("ragged")
                else np.array(mixed_lengths(SEED, 512), dtype=np.uint32))
        offs = np.zeros(len(lens), dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        return dict(seed=SEED, nbytes=int(lens.sum()), offsets=offs, lengths=lens,
                    count=len(lens), stride=0, fixed_len=0, key=key)
    if name == "mixed_16384":
        seed = SEED ^ entry["seed_xor"]
        lens = np.array(mixed_lengths(seed, entry["count"]), dtype=np.uint32)
        offs = np.zeros(len(lens), dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        return dict(seed=seed, nbytes=int(lens.sum()), offsets=offs, lengths=lens,
                    count=len(lens), stride=0, fixed_len=0, key=key)
    if name == "misaligned_2048":
        lens = np.array(entry["lengths"], dtype=np.uint32)
        offs = np.array(entry["offsets"], dtype=np.uint64)
        return dict(seed=SEED ^ entry["seed_xor"], nbytes=int(offs[-1] + lens[-1]), offsets=offs,
                    lengths=lens, count=len(lens), stride=0, fixed_len=0, key=key)
    if name.startswith("big_"):
        n = entry["fixed_len"]
        return dict(seed=SEED, nbytes=n, offsets=None, lengths=None, count=1, stride=0,
                    fixed_len=n, key=key)
    # fixed-stride 1 KiB batches
    c = entry["count"]
    return dict(seed=SEED, nbytes=c * entry["stride"], offsets=None, lengths=None, count=c,
                stride=entry["stride"], fixed_len=entry["fixed_len"], key=key)


def dod(digests):
    """SHA-256 over the packed digest array (fixture 'digest of digests')."""
    return hashlib.sha256(np.ascontiguousarray(digests).tobytes()).hexdigest()


def check_entry(entry, digests):
    """Assert `digests` (count x D numpy) match every field the fixture keeps."""
    d = np.ascontiguousarray(digests)
    if "dod" in entry:
        assert dod(d) == entry["dod"], (entry["name"], entry["alg"], entry.get("key"))
    if "first" in entry:
        n = len(entry["first"]) // 2
        assert d.tobytes()[:n].hex() == entry["first"], (entry["name"], entry["alg"])
    if "digest" in entry:
        assert d.tobytes().hex() == entry["digest"], (entry["name"], entry["alg"])


# ---------------------------------------------------------------- packets
# The network-packet shape of the reference's in-tree caller: RADIUS packets
# of at most 4 KiB (include/proto/radius.h:576) landing at arbitrary receive-
# buffer offsets (src/threadpool/threadpool_task.c:692-696), one shared
# secret per peer (src/proto/radius_client.c:242,885,1025).  1M packets,
# lengths uniform in [20, 4096] (20 = the RADIUS header), packed back to back
# (byte offsets: every alignment occurs), 64 peer secrets of 8..64 bytes.
PKT_COUNT = 1 << 20
PKT_MIN, PKT_MAX = 20, 4096
PKT_TAG = 0x7061636B65747321      # "packets!": decorrelates the length stream
PKT_NKEYS = 64


def _mix64_np(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def packet_layout(count=PKT_COUNT, seed=SEED):
    """-> (offsets uint64, lengths uint32, total bytes): packed packets."""
    with np.errstate(over="ignore"):
        z = _mix64_np(np.arange(count, dtype=np.uint64) ^ np.uint64(seed ^ PKT_TAG))
    lens = (np.uint64(PKT_MIN) + z % np.uint64(PKT_MAX - PKT_MIN + 1)).astype(np.uint32)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return offs, lens, int(offs[-1]) + int(lens[-1]) if count else 0


def packet_keys(nkeys=PKT_NKEYS, seed=SEED):
    """The peers' shared secrets: key k is the first 8 + (k * 7) % 57 bytes
    (8..64) of eight mix64 words of its own."""
    out = []
    for k in range(nkeys):
        n = 8 + (k * 7) % 57
        w = _mix64_np(np.arange(8, dtype=np.uint64) + np.uint64(k * 8) ^ np.uint64(seed ^ 0x6B657973))
        out.append(w.astype("<u8").view(np.uint8)[:n].tobytes())
    return out


def packet_key_index(count=PKT_COUNT, nkeys=PKT_NKEYS, seed=SEED):
    """Peer of packet i: mix64 stream mod nkeys (uint32)."""
    z = _mix64_np(np.arange(count, dtype=np.uint64) ^ np.uint64(seed ^ 0x70656572))
    return (z % np.uint64(nkeys)).astype(np.uint32)
