"""Batched RADIUS packet signing and verification over the keyed digest
batches of liblcb_hash_gpu.so (lcb_hash_batch_keyed).

The in-tree caller of the reference's hash path is RADIUS
(include/proto/radius.h:53): every packet a client sends is signed by
radius_pkt_sign (radius.h:1487) and every reply verified by
radius_pkt_verify (radius.h:1535), one packet at a time on the CPU.  These
functions do the same for MANY packets at once, each with its own shared
secret (one per peer: src/proto/radius_client.c:242,886,1025); every MD5 and
HMAC-MD5 runs on the GPU through one keyed batch per step:

  User-Password hiding      H(secret || authenticator | c_j)  KEY_PREFIX
                            (radius.h:745-790 encode, 795-830 decode)
  Message-Authenticator     HMAC(secret, packet*)             KEY_HMAC
                            (radius.h:850-919)
  packet authenticator      H(packet* || secret)              KEY_SUFFIX
                            (radius.h:1315-1377)

(packet* = the packet with the fields the reference zeroes or substitutes.)
The host side only moves bytes: attribute lookup, field substitution and
the XOR of the password blocks.  Results are byte-identical to the
reference's functions (tests/test_radius_gpu.py, against packets the
reference itself signed: tests/golden/radius.json).

Packet codes and the authenticator each computation uses follow
radius.h:866-904 and 1322-1375 exactly.
"""
import errno

import numpy as np

from .hash import KEY_HMAC, KEY_PREFIX, KEY_SUFFIX, hash_batch_keyed

MD5 = 1
ATTR_USER_PASSWORD = 2        # radius.h:70
ATTR_MSG_AUTHENTIC = 80       # radius.h:232
ACCESS_REQUEST, ACCESS_ACCEPT, ACCESS_REJECT = 1, 2, 3
ACCOUNTING_REQUEST, ACCOUNTING_RESPONSE = 4, 5
ACCESS_CHALLENGE, STATUS_SERVER, STATUS_CLIENT = 11, 12, 13
DISCONNECT_REQUEST, DISCONNECT_ACK, DISCONNECT_NAK = 40, 41, 42
COA_REQUEST, COA_ACK, COA_NAK = 43, 44, 45
RANDOM_AUTH = (ACCESS_REQUEST, STATUS_SERVER, STATUS_CLIENT)
ZERO_AUTH = (ACCOUNTING_REQUEST, DISCONNECT_REQUEST, COA_REQUEST)
REPLY_AUTH = (ACCESS_ACCEPT, ACCESS_REJECT, ACCESS_CHALLENGE, DISCONNECT_ACK, DISCONNECT_NAK, COA_ACK, COA_NAK)

__all__ = ["radius_pkt_sign_batch", "radius_pkt_verify_batch", "find_attr", "pkt_len"]


def find_attr(pkt, attr_type):
    """Offset of the first attribute of `attr_type` (radius.h:696-735), or None."""
    end = int.from_bytes(pkt[2:4], "big")
    i = 20
    while i + 2 <= end:
        t, n = pkt[i], pkt[i + 1]
        if n < 2 or i + n > end:
            return None
        if t == attr_type:
            return i
        i += n
    return None


def pkt_len(pkt):
    """The packet's own Length field (RADIUS_PKT_HDR_LEN_GET, radius.h): the
    reference hashes [0, Length) and ignores buffer bytes past it
    (radius.h:913 RADIUS_PKT_END, :1333)."""
    return int.from_bytes(pkt[2:4], "big")


def _pw_check(n):
    """radius_pkt_attr_password_encode's checks for a User-Password of n data
    bytes encoded in place (radius.h:752-765): 0 or the error it returns."""
    if n > 128:
        return errno.EINVAL
    aligned = ((n + 15) & ~15) if n else 16
    if aligned > n:          # buf_size = n: not a nonzero multiple of 16
        return errno.EOVERFLOW
    return 0


def _pack(msgs):
    lens = np.array([len(m) for m in msgs], np.uint32)
    offs = np.zeros(len(msgs), np.uint64)
    if len(msgs) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = np.frombuffer(b"".join(msgs) or b"\0", np.uint8)
    return blob, offs, lens


def _keyed(mode, keys, msgs, kidx, device):
    """One keyed MD5 batch; returns a list of 16-byte digests."""
    if not msgs:
        return []
    blob, offs, lens = _pack(msgs)
    kidx = np.asarray(kidx, np.uint32)
    if device:
        import torch
        d = hash_batch_keyed(MD5, mode, keys, torch.as_tensor(blob, device="cuda"),
                             key_index=torch.as_tensor(kidx.astype(np.int32), device="cuda"),
                             offsets=torch.as_tensor(offs.astype(np.int64), device="cuda"),
                             lengths=torch.as_tensor(lens.astype(np.int32), device="cuda")).cpu().numpy()
    else:
        d = hash_batch_keyed(MD5, mode, keys, blob, key_index=kidx, offsets=offs, lengths=lens)
    return [bytes(r) for r in d]


def _password_encode(pkts, keys, key_index, err, device):
    """radius.h:745-790 on every packet's User-Password, in place: block j
    of all packets in one KEY_PREFIX batch (the chain is serial per packet).
    A password the reference refuses (_pw_check) sets err[n] and leaves the
    packet untouched, as radius_pkt_sign returns before writing."""
    jobs = []
    for n, p in enumerate(pkts):
        o = find_attr(p, ATTR_USER_PASSWORD)
        if o is None:
            continue
        e = _pw_check(p[o + 1] - 2)
        if e:
            err[n] = e
            continue
        jobs.append((n, o + 2, p[o + 1] - 2))
    prev = {n: bytes(pkts[n][4:20]) for n, _, _ in jobs}          # the authenticator
    j = 0
    while True:
        live = [(n, s, l) for n, s, l in jobs if j * 16 < l]
        if not live:
            return
        digs = _keyed(KEY_PREFIX, keys, [prev[n] for n, _, _ in live], [key_index[n] for n, _, _ in live], device)
        for (n, s, l), d in zip(live, digs):
            a = s + 16 * j
            c = bytes(x ^ y for x, y in zip(pkts[n][a:a + 16], d))
            pkts[n][a:a + 16] = c
            prev[n] = c
        j += 1


def radius_pkt_sign_batch(packets, keys, key_index=None, device=False):
    """radius_pkt_sign(pkt, ..., key, key_len, add_msg_authr = 0) of every
    packet (radius.h:1487-1531): User-Password encoded, an existing
    Message-Authenticator and the authenticator updated with the packet's
    authenticator inside, each over the packet's [0, Length) only.  packets:
    sequence of bytes (a reply already holds its request's authenticator,
    radius_pkt_reply_init; bytes past Length are kept as they are); keys: the
    shared secrets; key_index[i]: packet i's secret (default 0).  Returns
    (errors, packets): errors[i] is 0 or the error radius_pkt_sign returns
    (EINVAL / EOVERFLOW for a User-Password it refuses), and a failed packet
    is returned unchanged."""
    n = len(packets)
    key_index = np.zeros(n, np.uint32) if key_index is None else np.asarray(key_index, np.uint32)
    pkts = [bytearray(p) for p in packets]
    err = np.zeros(n, np.int64)
    _password_encode(pkts, keys, key_index, err, device)
    # Message-Authenticator, authenticator inside (radius.h:866-872, 906-916):
    # HMAC over the packet with the attribute's 16 data bytes zeroed.
    ma = [(i, find_attr(p, ATTR_MSG_AUTHENTIC)) for i, p in enumerate(pkts) if not err[i]]
    ma = [(i, o) for i, o in ma if o is not None]
    msgs = []
    for i, o in ma:
        pkts[i][o + 2:o + 18] = bytes(16)
        msgs.append(bytes(pkts[i][:pkt_len(pkts[i])]))
    for (i, o), d in zip(ma, _keyed(KEY_HMAC, keys, msgs, [key_index[i] for i, _ in ma], device)):
        pkts[i][o + 2:o + 18] = d
    # Authenticator, inside: MD5(packet || secret) except for the codes whose
    # authenticator is random (radius.h:1322-1336, 1404-1421).
    au = [i for i, p in enumerate(pkts) if not err[i] and p[0] not in RANDOM_AUTH]
    for i, d in zip(au, _keyed(KEY_SUFFIX, keys, [bytes(pkts[i][:pkt_len(pkts[i])]) for i in au],
                               [key_index[i] for i in au], device)):
        pkts[i][4:20] = d
    return err, [bytes(p) if not err[i] else bytes(packets[i]) for i, p in enumerate(pkts)]


def _ma_authenticator(code, req):
    """The authenticator radius_pkt_attr_msg_authenticator_calc hashes with
    pkt_authenticator_inside = 0 (radius.h:866-904): None = keep the
    packet's own; EINVAL / EBADMSG as the reference returns."""
    if code in RANDOM_AUTH:
        return None
    if code == ACCOUNTING_RESPONSE and req is not None and req[0] == STATUS_SERVER:
        return bytes(req[4:20])
    if code in ZERO_AUTH or code == ACCOUNTING_RESPONSE:
        return bytes(16)
    if code in REPLY_AUTH:
        return errno.EINVAL if req is None else bytes(req[4:20])
    return errno.EBADMSG


def _auth_authenticator(code, req):
    """The authenticator radius_pkt_authenticator_calc hashes with
    pkt_authenticator_inside = 0 (radius.h:1337-1375)."""
    if code in ZERO_AUTH:
        return bytes(16)
    if code in REPLY_AUTH or code == ACCOUNTING_RESPONSE:
        return errno.EINVAL if req is None else bytes(req[4:20])
    return errno.EINVAL


def radius_pkt_verify_batch(packets, keys, key_index=None, requests=None, device=False):
    """radius_pkt_verify(pkt, key, key_len, pkt_req) of every packet
    (radius.h:1535-1568): Message-Authenticator check, authenticator check,
    then the User-Password decoded in place.  requests[i]: the request a
    reply answers (None for requests).  Returns (errors, packets): errors[i]
    is 0, EBADMSG or EINVAL as the reference returns; packets[i] as the
    reference leaves the buffer (password decoded only when the checks
    pass)."""
    n = len(packets)
    key_index = np.zeros(n, np.uint32) if key_index is None else np.asarray(key_index, np.uint32)
    requests = [None] * n if requests is None else list(requests)
    pkts = [bytearray(p) for p in packets]
    err = np.zeros(n, np.int64)
    # 1. Message-Authenticator (radius.h:922-953, inside = 0).
    jobs, msgs = [], []
    for i, p in enumerate(pkts):
        o = find_attr(p, ATTR_MSG_AUTHENTIC)
        if o is None:
            continue
        if p[o + 1] != 18:
            err[i] = errno.EBADMSG
            continue
        a = _ma_authenticator(p[0], requests[i])
        if isinstance(a, int):
            err[i] = a
            continue
        q = bytearray(p[:pkt_len(p)])
        if a is not None:
            q[4:20] = a
        q[o + 2:o + 18] = bytes(16)
        jobs.append((i, o))
        msgs.append(bytes(q))
    for (i, o), d in zip(jobs, _keyed(KEY_HMAC, keys, msgs, [key_index[i] for i, _ in jobs], device)):
        if d != bytes(pkts[i][o + 2:o + 18]):
            err[i] = errno.EBADMSG
    # 2. Authenticator (radius.h:1380-1402), skipped for random authenticators.
    jobs, msgs = [], []
    for i, p in enumerate(pkts):
        if err[i] or p[0] in RANDOM_AUTH:
            continue
        a = _auth_authenticator(p[0], requests[i])
        if isinstance(a, int):
            err[i] = a
            continue
        q = bytearray(p[:pkt_len(p)])
        q[4:20] = a
        jobs.append(i)
        msgs.append(bytes(q))
    for i, d in zip(jobs, _keyed(KEY_SUFFIX, keys, msgs, [key_index[i] for i in jobs], device)):
        if d != bytes(pkts[i][4:20]):
            err[i] = errno.EBADMSG
    # 3. User-Password decode (radius.h:795-830): every block at once,
    #    b_0 = MD5(secret || authenticator), b_j = MD5(secret || c_{j-1}).
    jobs, msgs, kk = [], [], []
    for i, p in enumerate(pkts):
        o = find_attr(p, ATTR_USER_PASSWORD)
        if err[i] or o is None:
            continue
        l = p[o + 1] - 2
        if l == 0 or l % 16 or l > 128:
            err[i] = errno.EINVAL
            continue
        for j in range(l // 16):
            msgs.append(bytes(p[4:20]) if j == 0 else bytes(p[o + 2 + 16 * (j - 1):o + 2 + 16 * j]))
            kk.append(key_index[i])
            jobs.append((i, o + 2 + 16 * j))
    digs = _keyed(KEY_PREFIX, keys, msgs, kk, device)
    dec = {}
    for (i, a), d in zip(jobs, digs):
        dec.setdefault(i, []).append((a, d))
    for i, blocks in dec.items():   # the digests came from the ENCODED blocks: XOR now
        for a, d in blocks:
            pkts[i][a:a + 16] = bytes(x ^ y for x, y in zip(pkts[i][a:a + 16], d))
    return err, [bytes(p) for p in pkts]
