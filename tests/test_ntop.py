"""The formatter's address text (nsd_ntop.h) against the C library's
inet_ntop, which the reference calls (proto_ipv4.c:53-54, proto_ipv6.c:41-42):
IPv6 addresses over every zero / non-zero pattern of the eight words (the
"::" run choice, ties, leading and trailing runs), the IPv4-compatible and
IPv4-mapped forms, random addresses; IPv4 addresses with 0, 9, 10, 99, 100
and 255 bytes.  socket.inet_ntop is glibc's inet_ntop."""
import random
import socket
import struct

import numpy as np

import nsd
import nsd_testlib as T


def _eth(ethertype):
    return bytes(6) + bytes([2, 0, 0, 0, 0, 1]) + struct.pack(">H", ethertype)


def _ipv6_pkt(src, dst):
    # Eth / IPv6 / NoNext (next header 59), payload length 0
    return _eth(0x86DD) + bytes([0x60, 0, 0, 0]) + struct.pack(">HBB", 0, 59, 64) + src + dst


def _ipv4_pkt(src, dst):
    # Eth / IPv4 (no L4 the chain follows: protocol 254), checksum left zero
    return _eth(0x0800) + bytes([0x45, 0]) + struct.pack(">HHHBBH", 20, 0, 0, 64, 254, 0) + src + dst


def _texts(pkts):
    frames, desc = T.batch_from_packets(pkts)
    orec, oext, _, _ = T.oracle_records(frames, desc)
    texts, rc = nsd.format_batch(frames, desc, orec, oext)
    assert all(r == 0 for r in rc)
    return [t.decode() for t in texts]


def _v6_addresses():
    rng = random.Random(5)
    out = []
    for mask in range(256):
        for fill in (1, 0xffff, 0xabc, None):
            w = [(fill if fill is not None else rng.randrange(1, 0x10000)) if mask >> i & 1 else 0 for i in range(8)]
            out.append(struct.pack(">8H", *w))
    for last in (b"\x01\x02\x03\x04", b"\x00\x00\x00\x01", b"\x0a\x00\x00\x00", b"\xff\xff\xff\xff"):
        out.append(bytes(12) + last)                              # IPv4-compatible
        out.append(bytes(10) + b"\xff\xff" + last)                # IPv4-mapped
        out.append(bytes(10) + b"\xff\xfe" + last)                # neither
        out.append(bytes(8) + b"\x00\x01\x00\x00" + last)         # run of 4
    out += [bytes(rng.randrange(256) if rng.random() < 0.5 else 0 for _ in range(16)) for _ in range(400)]
    return out


def test_ipv6_address_text_is_inet_ntop():
    addrs = _v6_addresses()
    pkts = [_ipv6_pkt(addrs[k], addrs[(k * 7 + 3) % len(addrs)]) for k in range(len(addrs))]
    for k, t in enumerate(_texts(pkts)):
        s = socket.inet_ntop(socket.AF_INET6, addrs[k])
        d = socket.inet_ntop(socket.AF_INET6, addrs[(k * 7 + 3) % len(addrs)])
        assert f"IPv6 Addr ({s} => {d})" in t, (addrs[k].hex(), s, t[:200])


def test_ipv4_address_text_is_inet_ntop():
    rng = random.Random(6)
    vals = [0, 9, 10, 99, 100, 199, 200, 255]
    addrs = [bytes(rng.choice(vals) for _ in range(4)) for _ in range(300)] + [bytes(rng.randrange(256) for _ in range(4))
                                                                              for _ in range(300)]
    pkts = [_ipv4_pkt(addrs[k], addrs[-1 - k]) for k in range(len(addrs))]
    for k, t in enumerate(_texts(pkts)):
        s = socket.inet_ntop(socket.AF_INET, addrs[k])
        d = socket.inet_ntop(socket.AF_INET, addrs[-1 - k])
        assert f"IPv4 Addr ({s} => {d})" in t, (s, d, t[:200])
