"""IPv4 / IPv6 / ICMPv4 vectors pinned by the reference's own csum.h,
ipv4.h and ipv6.h (oracle/ref_iphdr.c -> oracle/_ref/libnsdrefip.so, built
from /root/reference as they lie).

make() builds seeded frames; expected() runs the reference unit over them.
tests/golden/ip_vectors.npz holds both (written by
tests/golden/make_golden.py --ip-only), so the GPU box, which has no
/root/reference, checks the device against the same numbers:

  v4_frames / v4_caplen  Eth + random IPv4 headers: every IHL 0..15 (so
                         calc_csum over ihl*4 bytes reaches past the 20-byte
                         header, past the options the frame holds and past
                         the capture, where bytes read as zero), random
                         version / TOS / lengths / flags / TTL / protocol /
                         checksum / addresses, frames cut anywhere from 34
                         to 110 bytes
  v4_fields              nsref_ipv4_fields: version, ihl, tos, tot_len, id,
                         res, nofrag, morefrag, fragoff, ttl, protocol,
                         check, calc_csum(ip, ihl*4), csum_expected, saddr,
                         daddr
  v6_frames / v6_caplen  Eth + random IPv6 fixed headers
  v6_fields              nsref_ipv6_fields: version, traffic class, flow
                         label, payload length, next header, hop limit
  icmp_frames / icmp_caplen  Eth / IPv4 (valid) / ICMPv4 messages of 8..263
                         bytes, odd and even lengths (calc_csum drops an odd
                         last byte, csum.h:26), half with a correct checksum
  icmp_csum              calc_csum(icmp, message length)
"""
import ctypes
import os
import struct

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_IP_SO = os.path.join(ROOT, "oracle", "_ref", "libnsdrefip.so")
FIXTURE = os.path.join(ROOT, "tests", "golden", "ip_vectors.npz")
W = 320
ETH4 = bytes.fromhex("0a0b0c0d0e0f" "020304050607" "0800")
ETH6 = bytes.fromhex("0a0b0c0d0e0f" "020304050607" "86dd")


def _csum16(b):
    if len(b) % 2:
        b = b[:-1]
    s = sum(struct.unpack(">%dH" % (len(b) // 2), b))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def make(seed=0x1C4D, n4=4096, n6=1024, nicmp=1024):
    rng = np.random.default_rng(seed)
    v4 = np.zeros((n4, W), dtype=np.uint8)
    v4c = np.zeros(n4, dtype=np.uint32)
    for k in range(n4):
        h = bytearray(rng.integers(0, 256, 60, dtype=np.uint8).tobytes())
        h[0] = (int(rng.integers(0, 16)) << 4) | (k % 16)
        if k % 3 == 0:
            h[0] = 0x40 | (k % 16)
        cut = int(rng.integers(20, 97))
        body = bytes(h[:min(cut, 60)]) + rng.integers(0, 256, max(0, cut - 60), dtype=np.uint8).tobytes()
        f = bytearray(ETH4 + body)
        ihl4 = 4 * (k % 16)
        if k % 4 == 1 and ihl4 >= 12:
            # a correct checksum over ihl*4 bytes, zeros past the capture
            f[24:26] = b"\0\0"
            row = bytes(f[14:]) + bytes(64)
            f[24:26] = struct.pack(">H", _csum16(row[:ihl4]))
        v4[k, :len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
        v4c[k] = len(f)
    v6 = np.zeros((n6, W), dtype=np.uint8)
    v6c = np.zeros(n6, dtype=np.uint32)
    for k in range(n6):
        h = bytearray(rng.integers(0, 256, 40, dtype=np.uint8).tobytes())
        if k % 2 == 0:
            h[0] = 0x60 | (h[0] & 0x0F)
        f = ETH6 + bytes(h) + rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
        v6[k, :len(f)] = np.frombuffer(f, dtype=np.uint8)
        v6c[k] = len(f)
    ic = np.zeros((nicmp, W), dtype=np.uint8)
    icc = np.zeros(nicmp, dtype=np.uint32)
    for k in range(nicmp):
        L = 8 + (k % 256)
        msg = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        msg[0], msg[1] = (8, 0) if k % 4 else (0, 0)
        if k % 2 == 0:
            msg[2:4] = b"\0\0"
            c = _csum16(bytes(msg))
            msg[2:4] = struct.pack(">H", c)
        ip = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + L, k, 0, 64, 1, 0, bytes([10, 0, 0, 1]),
                                   bytes([10, 0, 0, 2])))
        ip[10:12] = struct.pack(">H", _csum16(bytes(ip)))
        f = ETH4 + bytes(ip) + bytes(msg)
        ic[k, :len(f)] = np.frombuffer(f, dtype=np.uint8)
        icc[k] = len(f)
    return dict(v4_frames=v4, v4_caplen=v4c, v6_frames=v6, v6_caplen=v6c, icmp_frames=ic, icmp_caplen=icc)


def ref_lib():
    lib = ctypes.CDLL(REF_IP_SO)
    lib.nsref_calc_csum.restype = ctypes.c_uint16
    lib.nsref_calc_csum.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.nsref_csum_expected.restype = ctypes.c_uint16
    lib.nsref_csum_expected.argtypes = [ctypes.c_uint16, ctypes.c_uint16]
    lib.nsref_ipv4_fields.restype = None
    lib.nsref_ipv4_fields.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.nsref_ipv6_fields.restype = None
    lib.nsref_ipv6_fields.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return lib


def expected(v):
    """The reference unit's values for the frames of make() (bytes at or
    past caplen are zero in the frames arrays: the parity domain)."""
    lib = ref_lib()
    n4 = len(v["v4_caplen"])
    f4 = np.zeros((n4, 16), dtype=np.uint32)
    for k in range(n4):
        hdr = np.ascontiguousarray(v["v4_frames"][k, 14:14 + 64])
        lib.nsref_ipv4_fields(hdr.ctypes.data, f4[k].ctypes.data)
    n6 = len(v["v6_caplen"])
    f6 = np.zeros((n6, 6), dtype=np.uint32)
    for k in range(n6):
        hdr = np.ascontiguousarray(v["v6_frames"][k, 14:14 + 40])
        lib.nsref_ipv6_fields(hdr.ctypes.data, f6[k].ctypes.data)
    ni = len(v["icmp_caplen"])
    ci = np.zeros(ni, dtype=np.uint32)
    for k in range(ni):
        L = int(v["icmp_caplen"][k]) - 34
        msg = np.ascontiguousarray(v["icmp_frames"][k, 34:34 + L])
        ci[k] = lib.nsref_calc_csum(msg.ctypes.data, L)
    return dict(v4_fields=f4, v6_fields=f6, icmp_csum=ci)


def save():
    v = make()
    v.update(expected(v))
    np.savez_compressed(FIXTURE, **v)


def load():
    with np.load(FIXTURE, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def batch(frames, caplen):
    """Fixed-stride frame rows -> (frames, desc) at 16-byte aligned offsets."""
    import nsd_testlib as T
    return T.batch_from_packets([bytes(frames[k, :caplen[k]]) for k in range(len(caplen))])
