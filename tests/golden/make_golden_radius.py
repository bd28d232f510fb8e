#!/usr/bin/env python3
"""Generate tests/golden/radius.json (run ONLY in the build container).

RADIUS packets built and signed by the REFERENCE's own packet code
(include/proto/radius.h, compiled from /root/reference into
oracle/_ref/libref_radius.so by oracle/Makefile; wrapper oracle/ref_radius.c):

  requests  Access-Request (random authenticator, User-Password, optional
            Message-Authenticator), Accounting-Request, Status-Server,
            Disconnect-Request, CoA-Request: radius_pkt_init + attributes +
            radius_pkt_sign (radius.h:1487)
  replies   Access-Accept/-Reject/-Challenge, Accounting-Response,
            Disconnect-ACK/-NAK, CoA-ACK/-NAK to a signed request:
            radius_pkt_reply_init + attributes + radius_pkt_sign

Each packet keeps: the secret's index into a 5-secret table (lengths
10, 1, 16, 64 and 100 bytes: short, one-block and multi-block keys), the
packet before and after signing, for replies the request, and the
reference's radius_pkt_verify result (0) with the packet it leaves (User-
Password decoded in place).  Also independent spot values of
radius_pkt_authenticator_calc / radius_pkt_attr_msg_authenticator_calc /
radius_pkt_attr_password_encode for the GPU tests to pin.  Pure data:
packet bytes as hex.

Usage:  python3 tests/golden/make_golden_radius.py   (needs `make -C oracle`)
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SO = os.path.join(REPO, "oracle", "_ref", "libref_radius.so")

SECRETS = [b"testing123", b"s", bytes(range(16)), bytes((7 * i + 3) & 0xFF for i in range(64)),
           bytes((5 * i + 1) & 0xFF for i in range(100))]
REQ_CODES = {1: "Access-Request", 4: "Accounting-Request", 12: "Status-Server", 40: "Disconnect-Request",
             43: "CoA-Request"}
REPLY_CODES = {1: (2, 3, 11), 4: (5,), 12: (2, 5), 40: (41, 42), 43: (44, 45)}
ATTR_TYPES = (1, 18, 24, 25, 32)   # User-Name, Reply-Message, State, Class, NAS-Identifier


def lib():
    L = ctypes.CDLL(SO)
    u8p, sz = ctypes.c_char_p, ctypes.c_size_t
    L.ref_rad_request.argtypes = [ctypes.c_uint8, ctypes.c_uint8, u8p, u8p, sz, u8p, sz, u8p, sz, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.POINTER(sz), ctypes.c_void_p, ctypes.POINTER(sz)]
    L.ref_rad_reply.argtypes = [ctypes.c_uint8, u8p, u8p, sz, u8p, sz, ctypes.c_int,
                                ctypes.c_void_p, ctypes.POINTER(sz), ctypes.c_void_p, ctypes.POINTER(sz)]
    L.ref_rad_verify.argtypes = [u8p, sz, u8p, sz, u8p, ctypes.c_void_p]
    L.ref_rad_authenticator_calc.argtypes = [u8p, sz, u8p, sz, ctypes.c_int, u8p, ctypes.c_void_p]
    L.ref_rad_msg_authenticator_calc.argtypes = [u8p, sz, u8p, sz, ctypes.c_int, u8p, ctypes.c_void_p]
    L.ref_rad_password_encode.argtypes = [u8p, u8p, sz, u8p, sz, ctypes.c_void_p, sz, ctypes.POINTER(sz)]
    L.ref_rad_sign.argtypes = [u8p, sz, u8p, sz, ctypes.c_void_p, ctypes.POINTER(sz)]
    return L


def tlvs(rng):
    out = b""
    for _ in range(int(rng.integers(0, 6))):
        t = int(rng.choice(ATTR_TYPES))
        n = int(rng.integers(1, 61))
        out += bytes([t, n]) + rng.integers(0x20, 0x7F, n, dtype=np.uint8).tobytes()
    return out


def _tlv_starts(t):
    i, out = 0, []
    while i + 2 <= len(t):
        out.append(i)
        i += 2 + t[i + 1]
    return out


def main():
    if not os.path.exists(SO):
        sys.exit("oracle/_ref/libref_radius.so missing: make -C oracle (needs /root/reference)")
    L = lib()
    rng = np.random.default_rng(2865)
    pre = ctypes.create_string_buffer(4096)
    out = ctypes.create_string_buffer(4096)
    pl, ol = ctypes.c_size_t(), ctypes.c_size_t()
    packets = []
    skipped = 0
    while len(packets) < 480:
        code = int(rng.choice([1, 1, 1, 4, 12, 40, 43]))
        k = int(rng.integers(0, len(SECRETS)))
        auth = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        pwd = None
        if code == 1 and rng.random() < 0.85:
            pwd = rng.integers(0x21, 0x7F, int(rng.integers(1, 129)), dtype=np.uint8).tobytes()
        add_ma = 1 if (code == 12 or rng.random() < 0.7) else 0
        t = tlvs(rng)
        if code == 1:   # radius_pkt_chk wants a User-Name in an Access-Request
            n = int(rng.integers(1, 40))
            t = bytes([1, n]) + rng.integers(0x61, 0x7B, n, dtype=np.uint8).tobytes() + \
                b"".join(t[i:i + 2 + t[i + 1]] for i in _tlv_starts(t) if t[i] != 1)
        rc = L.ref_rad_request(code, int(rng.integers(0, 256)), auth, pwd, len(pwd) if pwd else 0, t, len(t),
                               SECRETS[k], len(SECRETS[k]), add_ma, pre, ctypes.byref(pl), out, ctypes.byref(ol))
        if rc != 0:
            continue
        req_pre, req = pre.raw[:pl.value], out.raw[:ol.value]
        chk = ctypes.create_string_buffer(4096)
        vr = L.ref_rad_verify(req, len(req), SECRETS[k], len(SECRETS[k]), None, chk)
        if vr != 0:   # radius_pkt_chk rejects some attribute mixes for this code: not a hash case
            skipped += 1
            continue
        packets.append({"kind": "request", "code": code, "key": k, "msg_authr": add_ma,
                        "password": pwd.hex() if pwd else None, "pre": req_pre.hex(), "signed": req.hex(),
                        "verified": chk.raw[:len(req)].hex()})
        if rng.random() < 0.5:
            rcode = int(rng.choice(REPLY_CODES[code]))
            add_ma = 1 if rng.random() < 0.6 else 0
            t = tlvs(rng)
            rc = L.ref_rad_reply(rcode, req, t, len(t), SECRETS[k], len(SECRETS[k]), add_ma, pre, ctypes.byref(pl),
                                 out, ctypes.byref(ol))
            if rc != 0:
                continue
            rep = out.raw[:ol.value]
            vr = L.ref_rad_verify(rep, len(rep), SECRETS[k], len(SECRETS[k]), req, chk)
            if vr != 0:
                skipped += 1
                continue
            a16 = ctypes.create_string_buffer(16)
            assert L.ref_rad_authenticator_calc(rep, len(rep), SECRETS[k], len(SECRETS[k]), 0, req, a16) == 0
            assert a16.raw == rep[4:20]
            packets.append({"kind": "reply", "code": rcode, "key": k, "msg_authr": add_ma, "request": req.hex(),
                            "pre": pre.raw[:pl.value].hex(), "signed": rep.hex(),
                            "verified": chk.raw[:len(rep)].hex(), "authenticator_calc": a16.raw.hex()})
    # Password hiding spot values (radius.h:745-790), every length 1..128.
    pw = []
    enc = ctypes.create_string_buffer(256)
    el = ctypes.c_size_t()
    for n in range(1, 129):
        k = n % len(SECRETS)
        auth = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        p = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert L.ref_rad_password_encode(auth, p, n, SECRETS[k], len(SECRETS[k]), enc, 256, ctypes.byref(el)) == 0
        pw.append({"key": k, "authenticator": auth.hex(), "password": p.hex(), "encoded": enc.raw[:el.value].hex()})
    json.dump({"source": "reference include/proto/radius.h compiled from /root/reference (oracle/ref_radius.c)",
               "secrets": [s.hex() for s in SECRETS], "packets": packets, "password_encode": pw},
              open(os.path.join(HERE, "radius.json"), "w"), indent=0)
    print("radius.json: %d packets (%d replies), %d password vectors; %d built packets failed "
          "radius_pkt_chk and were dropped" % (len(packets), sum(p["kind"] == "reply" for p in packets), len(pw),
                                               skipped))


def edge():
    """tests/golden/radius_edge.json: radius_pkt_sign (ref_rad_sign) on
    (a) signed-able packets followed by bytes past their Length field (a
    receive buffer longer than the packet: the reference hashes [0, Length)),
    (b) Access-Requests whose User-Password data is 0, unaligned or over 128
    bytes long (radius_pkt_attr_password_encode refuses them,
    radius.h:752-765, and radius_pkt_sign returns that error)."""
    L = lib()
    rad = json.load(open(os.path.join(HERE, "radius.json")))
    rng = np.random.default_rng(1315)
    out = ctypes.create_string_buffer(4096)
    ol = ctypes.c_size_t()
    cases = []
    for p in rad["packets"][:120]:
        pre = bytes.fromhex(p["pre"])
        tail = rng.integers(0, 256, int(rng.integers(1, 200)), dtype=np.uint8).tobytes()
        k = p["key"]
        rc = L.ref_rad_sign(pre + tail, len(pre) + len(tail), SECRETS[k], len(SECRETS[k]), out, ctypes.byref(ol))
        cases.append({"what": "trailing", "key": k, "pre": (pre + tail).hex(), "rc": rc,
                      "signed": out.raw[:ol.value].hex() if rc == 0 else None})
    for n in (0, 1, 5, 15, 17, 33, 129, 130, 144, 160):
        k = n % len(SECRETS)
        auth = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        user = b"\x01\x06user"
        attr = bytes([2, 2 + n]) + rng.integers(0x21, 0x7F, n, dtype=np.uint8).tobytes()
        body = user + attr
        hdr = bytes([1, int(rng.integers(0, 256))]) + (20 + len(body)).to_bytes(2, "big") + auth
        pkt = hdr + body
        rc = L.ref_rad_sign(pkt, len(pkt), SECRETS[k], len(SECRETS[k]), out, ctypes.byref(ol))
        cases.append({"what": "password_len_%d" % n, "key": k, "pre": pkt.hex(), "rc": rc,
                      "signed": out.raw[:ol.value].hex() if rc == 0 else None})
    json.dump({"source": "reference radius_pkt_sign (oracle/ref_radius.c ref_rad_sign)", "cases": cases},
              open(os.path.join(HERE, "radius_edge.json"), "w"), indent=0)
    print("radius_edge.json: %d cases, rcs %s" % (len(cases), sorted({c["rc"] for c in cases})))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--edge":
        edge()
    else:
        main()
