"""Seeded frames for the leaf parsers whose fields the host renders and whose
cursor the walk keeps (nsd_leaf.h): ARP, DCCP, IGMP (v0-v3,
RGMP, query source lists, report group records), LLDP (TLV sequences in and
out of order, every TLV type, bad lengths, the END TLV) and the ICMPv6
130-154 bodies (MLDv2 lists, Neighbor Discovery option chains of every
option type, bad option lengths).  Each structured frame is also cut at
random capture lengths, and IPv4 tot_len is sometimes shorter than the
frame (the trim moves the leaf's tail).  Data only: tests/golden/leaves.*
hold the reference objects' text for them (make_golden.py), the parity
tests compare device records and host walks with the oracle."""
import random

from edge_cases import be16, be32, eth, ipv4, ipv6

A = [bytes.fromhex(h) for h in ("fe800000000000000211223344556677", "ff020000000000000000000000000001",
                                "20010db8000000000000000000000042")]


def _rb(r, n):
    return bytes(r.randrange(256) for _ in range(n))


def _arp(r):
    hrd = r.choice([1, 6, 7, 16, 20, 24, r.randrange(65536)])
    pro = r.choice([0x0800, 0x86DD, r.randrange(65536)])
    op = r.choice([1, 2, 3, 4, 8, 9, r.randrange(65536)])
    return eth(0x0806) + be16(hrd) + be16(pro) + bytes([6, 4]) + be16(op) + _rb(r, 20) + _rb(r, r.randrange(0, 12))


def _dccp_hdr(r):
    x = r.randrange(2)
    typ = r.randrange(16)
    h = be16(r.randrange(65536)) + be16(r.randrange(65536)) + bytes([r.randrange(256), r.randrange(256)]) + \
        be16(r.randrange(65536)) + bytes([(typ << 1) | x | (r.randrange(8) << 5)]) + _rb(r, 3)
    return h + _rb(r, r.choice([0, 2, 4, 6, 8, 12, 16, 24]))


def _igmp_msg(r):
    t = r.choice([1, 2, 3, 4, 5, 6, 7, 8, 0x11, 0x11, 0x12, 0x16, 0x17, 0x22, 0x22, 0xFC, 0xFD, 0xFE, 0xFF,
                  r.randrange(256)])
    if t == 0x11 and r.random() < 0.7:
        n = r.choice([0, 1, 2, 3, 7, r.randrange(300)])
        have = min(n, r.randrange(0, 6))
        return bytes([t, r.randrange(256)]) + be16(0) + be32(0xE0000001) + \
            bytes([r.randrange(256), r.randrange(256)]) + be16(n) + b"".join(be32(0x0A000000 + i) for i in range(have)) + \
            _rb(r, r.choice([0, 0, 1, 2, 3]))
    if t == 0x22 and r.random() < 0.8:
        nrec = r.choice([0, 1, 2, 3, r.randrange(100)])
        body = b""
        for _ in range(min(nrec, r.randrange(0, 4))):
            n = r.choice([0, 1, 2, r.randrange(20)])
            body += bytes([r.randrange(1, 8), 0]) + be16(n) + be32(0xEF000000 + r.randrange(256)) + \
                b"".join(be32(0xC0A80000 + i) for i in range(min(n, r.randrange(0, 4))))
        return bytes([t, 0]) + be16(0) + be16(0) + be16(nrec) + body + _rb(r, r.choice([0, 0, 2, 5]))
    ln = r.choice([8, 8, 20, 20, 12, 4, 9, 24, r.randrange(0, 40)])
    return bytes([t]) + _rb(r, ln - 1) if ln else b""


def _tlv(t, payload):
    return be16((t << 9) | (len(payload) & 0x1FF)) + payload


def _lldp_body(r):
    tl = []
    ordered = r.random() < 0.7
    seq = [1, 2, 3] if ordered else r.sample([1, 2, 3, 4, 7], r.randrange(1, 4))
    seq += [r.choice([4, 5, 6, 7, 8, 8, 127, 9, 12, 126, 0]) for _ in range(r.randrange(0, 6))]
    for t in seq:
        if t in (1, 2):
            sub = r.choice([1, 2, 3, 4, 5, 6, 7, 0, 9])
            if sub == (4 if t == 1 else 3):
                p = bytes([sub]) + _rb(r, r.choice([6, 6, 3]))
            elif sub == (5 if t == 1 else 4):
                af = r.choice([1, 2, 6, 9])
                p = bytes([sub, af]) + _rb(r, r.choice([4, 16, 6, 2, 0]))
            else:
                p = bytes([sub]) + b"ifname-" + bytes([0x30 + r.randrange(10)])
            tl.append(_tlv(t, p))
        elif t == 3:
            tl.append(_tlv(3, be16(r.randrange(65536)) if r.random() < 0.85 else _rb(r, 3)))
        elif t in (4, 5, 6):
            tl.append(_tlv(t, b"desc " + _rb(r, r.randrange(0, 12))))
        elif t == 7:
            tl.append(_tlv(7, _rb(r, 4) if r.random() < 0.85 else _rb(r, 2)))
        elif t == 8:
            alen = r.choice([5, 17, 7, 1, 0, 30])
            af = r.choice([1, 2, 6, 3])
            oid = r.choice([0, 0, 3, 9])
            p = bytes([alen, af]) + _rb(r, max(alen - 1, 0)) + bytes([r.choice([1, 2, 3])]) + be32(r.randrange(1 << 32)) + \
                bytes([oid]) + b"1.3.6.1.2.1"[:oid]
            if r.random() < 0.2:
                p = p[:r.randrange(len(p) + 1)]
            tl.append(_tlv(8, p))
        elif t == 127:
            tl.append(_tlv(127, bytes.fromhex("0080c2") + bytes([r.randrange(256)]) + _rb(r, r.choice([0, 2, 6]))))
        elif t == 0:
            tl.append(be16(0))
        else:
            tl.append(_tlv(t, _rb(r, r.randrange(0, 10))))
    body = b"".join(tl)
    if r.random() < 0.6:
        body += be16(0)                                   # END
    if r.random() < 0.2:                                  # a length past the frame
        body += be16((r.randrange(1, 128) << 9) | 0x1FF) + _rb(r, 4)
    return body + _rb(r, r.choice([0, 0, 1, 2, 9]))


def _nd_opts(r, n):
    out = b""
    for _ in range(n):
        t = r.choice([1, 2, 3, 4, 5, 9, 10, 15, 16, 17, 19, 0, 25, 31, 200])
        if t in (1, 2):
            p = _rb(r, 6)
        elif t == 3:
            p = bytes([64, 0xC0]) + be32(86400) + be32(3600) + be32(0) + A[2]
        elif t == 4:
            p = be16(0) + be32(0) + _rb(r, r.choice([0, 8, 16]))
        elif t == 5:
            p = be16(0) + be32(1500)
        elif t in (9, 10):
            p = be16(0) + be32(0) + b"".join(r.sample(A, r.randrange(0, 3)))
        elif t == 15:
            pad = r.choice([0, 1, 2, 3, 90])
            p = bytes([r.choice([1, 2, 3])]) + pad.to_bytes(8, "little") + b"name"[:r.randrange(5)] + bytes(min(pad, 3))
        elif t == 16:
            p = bytes([1, 0]) + _rb(r, r.choice([4, 6, 12]))
        elif t == 17:
            p = bytes([r.randrange(1, 6), 64]) + r.choice([be32(0) + A[2], A[1], _rb(r, 6)])
        elif t == 19:
            p = bytes([r.randrange(10)]) + _rb(r, r.choice([5, 13]))
        else:
            p = _rb(r, r.choice([6, 14]))
        total = 2 + len(p)
        l8 = (total + 7) // 8
        if r.random() < 0.15:
            l8 = r.choice([0, l8 + 1, l8 + 5, 255])
        body = bytes([t, l8]) + p
        body += bytes(max(0, l8 * 8 - len(body))) if l8 * 8 > len(body) and r.random() < 0.9 else b""
        out += body
    return out


def _icmpv6_body(r):
    t = r.randrange(130, 155)
    c = r.choice([0, 0, 1, 2, r.randrange(256)])
    if t == 130:
        b = be16(r.randrange(65536)) + be16(0) + A[1]
        if r.random() < 0.7:
            n = r.choice([0, 1, 2, 3, 0x102, r.randrange(65536)])
            b += bytes([r.randrange(256), r.randrange(256)]) + be16(n) + b"".join(r.sample(A, min(3, r.randrange(0, 4))))
    elif t in (131, 132):
        b = be16(r.randrange(65536)) + be16(0) + A[r.randrange(3)]
    elif t in (133, 141, 142, 147, 148, 154):
        b = _rb(r, 4) + _nd_opts(r, r.randrange(0, 4))
    elif t == 134:
        b = _rb(r, 12) + _nd_opts(r, r.randrange(0, 4))
    elif t in (135, 136):
        b = _rb(r, 4) + A[0] + _nd_opts(r, r.randrange(0, 4))
    elif t == 137:
        b = _rb(r, 4) + A[0] + A[2] + _nd_opts(r, r.randrange(0, 4))
    elif t in (138, 139, 140):
        b = _rb(r, 12) + _rb(r, r.choice([0, 4, 9]))
    elif t == 143:
        nrec = r.choice([0, 1, 2, 3, 300])
        recs = b""
        for _ in range(min(nrec, r.randrange(0, 4))):
            ns = r.choice([0, 1, 2, 258])
            aux = r.choice([0, 0, 1, 2, 60])
            recs += bytes([r.randrange(0, 9), aux]) + be16(ns) + A[1] + b"".join(r.sample(A, min(ns, r.randrange(0, 3)))) + \
                _rb(r, min(aux * 4, r.choice([0, 4, 8, 240])))
        b = be16(0) + be16(nrec) + recs
    elif t == 145:
        b = _rb(r, 4) + b"".join(r.sample(A, r.randrange(0, 3))) + _rb(r, r.choice([0, 5]))
    elif t == 149:
        b = _rb(r, 8) + _nd_opts(r, r.randrange(0, 4))
    else:
        b = _rb(r, r.choice([0, 2, 4, 8]))
    return bytes([t, c]) + be16(0xBEEF) + b


def _cut(r, f):
    """keep the frame, or cut it at a random capture length"""
    return f if r.random() < 0.55 else f[:r.randrange(14, len(f) + 1)]


def cases(n=3000, seed=0x1EAF):
    r = random.Random(seed)
    out = []
    for _ in range(n):
        k = r.randrange(6)
        if k == 0:
            f = _arp(r)
        elif k == 1:                                       # DCCP over IPv4 / IPv6
            h = _dccp_hdr(r)
            f = eth(0x0800) + ipv4(33, len(h)) + h if r.random() < 0.6 else eth(0x86DD) + ipv6(33, len(h)) + h
        elif k == 2:                                       # IGMP (tot_len: exact, short, long)
            m = _igmp_msg(r)
            tl = r.choice([None, None, None, 20 + max(0, len(m) - 4), 20 + len(m) + 8])
            f = eth(0x0800) + ipv4(2, len(m), tot_len=tl) + m
        elif k == 3:
            f = eth(0x88cc) + _lldp_body(r)
        elif k == 4:                                       # behind a VLAN tag
            f = eth(0x8100) + be16(r.randrange(4096)) + be16(0x88cc) + _lldp_body(r) if r.random() < 0.5 else \
                eth(0x8100) + be16(5) + be16(0x0806) + _arp(r)[14:]
        else:
            m = _icmpv6_body(r)
            f = eth(0x86DD) + ipv6(58, len(m)) + m if r.random() < 0.85 else \
                eth(0x0800) + ipv4(41, 40 + len(m)) + ipv6(58, len(m)) + m
        out.append(_cut(r, f))
    return out
