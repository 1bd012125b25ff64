"""IPv4 / IPv6 pinned by the reference's own headers.

proto_ipv4.c and proto_ipv6.c cannot be compiled here (geoip.h ->
config.h), but the checksum code and header layouts they print from can:
oracle/ref_iphdr.c includes /root/reference/csum.h, ipv4.h and ipv6.h as
they lie (oracle/_ref/libnsdrefip.so).  tests/ip_vectors.py draws seeded
frames (every IHL 0..15, checksums over bytes past the capture, random
fields; IPv6 fixed headers; ICMPv4 messages of odd and even lengths) and
tests/golden/ip_vectors.npz keeps the reference unit's values for them.

CPU: the fixture is what the reference unit computes today; the oracle's
records and text, the product's host walk and the product formatter's text
agree with it field by field.  GPU: the device records (both record forms,
both kernel schedules) and the text rendered from them agree with it."""
import os
import re
import socket
import struct

import numpy as np
import pytest

import ip_vectors as IV
import nsd
import nsd_testlib as T

HAVE_REF = os.path.exists(IV.REF_IP_SO)

RE4 = re.compile(rb"\[ IPv4 Addr \(([0-9.]+) => ([0-9.]+)\), Proto \((\d+)\), TTL \((\d+)\), TOS \((\d+)\), "
                 rb"Ver \((\d+)\), IHL \((\d+)\), Tlen \((\d+)\), ID \((\d+)\), Res \((\d+)\), NoFrag \((\d+)\), "
                 rb"MoreFrag \((\d+)\), FragOff \((\d+)\), CSum \(0x([0-9a-f]{4})\) is ([^\n]*)")
RE6 = re.compile(rb"\[ IPv6 Addr \(([^ ]*) => ([^ ]*)\), Version \((\d+)\), TrafficClass \((\d+)\), "
                 rb"FlowLabel \((\d+)\), Len \((\d+)\), NextHdr \((\d+)\), HopLimit \((\d+)\) \]")
REICMP = re.compile(rb"\[ ICMP Type \(\d+\), Code \(\d+\), CSum \(0x[0-9a-f]{4}\) is ([^\]]*)")


@pytest.fixture(scope="module")
def vec():
    return IV.load()


def ip4(v):
    return socket.inet_ntoa(struct.pack("<I", int(v))).encode()


def check_v4_text(text, f):
    m = RE4.search(text)
    assert m, text[:300]
    g = m.groups()
    assert (g[0], g[1]) == (ip4(f[14]), ip4(f[15]))
    # Proto TTL TOS Ver IHL Tlen ID Res NoFrag MoreFrag FragOff
    want = [f[10], f[9], f[2], f[0], f[1], f[3], f[4], f[5], f[6], f[7], f[8]]
    assert [int(x) for x in g[2:13]] == [int(x) for x in want]
    assert int(g[13], 16) == int(f[11])
    rest = g[14]
    if f[12] == 0:
        assert rest.startswith(b"ok")
    else:
        assert b"bogus (!)" in rest
        assert int(re.search(rb"should be 0x([0-9a-f]{4})", rest).group(1), 16) == int(f[13])


def check_v6_text(text, f):
    m = RE6.search(text)
    assert m, text[:300]
    assert [int(x) for x in m.groups()[2:]] == [int(x) for x in f]


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (no /root/reference)")
def test_fixture_is_the_reference_units_output():
    v = IV.make()
    for k, a in v.items():
        assert np.array_equal(a, IV.load()[k]), k
    e = IV.expected(v)
    fx = IV.load()
    for k, a in e.items():
        assert np.array_equal(a, fx[k]), k
    # a known answer through the reference's csum.h: the IPv4 header of
    # RFC 1071's / Wikipedia's example sums to 0xb861 (calc_csum adds
    # little-endian words: the value reads byte-swapped)
    lib = IV.ref_lib()
    buf = np.frombuffer(bytes.fromhex("450000730000400040110000c0a80001c0a800c7"), dtype=np.uint8).copy()
    assert lib.nsref_calc_csum(buf.ctypes.data, 20) == 0x61b8
    buf[10:12] = (0xb8, 0x61)
    assert lib.nsref_calc_csum(buf.ctypes.data, 20) == 0


def test_fixture_covers_the_edges(vec):
    f4 = vec["v4_fields"]
    assert set(f4[:, 1]) == set(range(16))                          # every IHL
    past = (14 + 4 * f4[:, 1]) > vec["v4_caplen"]
    assert past.sum() > 500                                         # ihl*4 past the capture
    assert ((f4[:, 12] == 0).sum() > 0) and ((f4[:, 12] != 0).sum() > 1000)
    L = vec["icmp_caplen"] - 34
    assert (L % 2 == 1).sum() > 400 and (vec["icmp_csum"] == 0).sum() > 400


def test_oracle_and_host_walk_vs_reference(vec):
    frames, desc = IV.batch(vec["v4_frames"], vec["v4_caplen"])
    rec, ext, _, _ = T.oracle_records(frames, desc, mode=T.PRINT_NORM)
    assert (rec["chain"] >> 5 & 31 == 7).all()                      # layer 1 = ipv4
    assert np.array_equal(rec["ip_csum"], vec["v4_fields"][:, 12].astype(np.uint16))
    hrec = nsd.walk_cpu(frames, desc, mode=T.PRINT_NORM)[0]
    assert np.array_equal(hrec["ip_csum"], vec["v4_fields"][:, 12].astype(np.uint16))
    ora = T.oracle_text_packets(frames, desc, mode=T.PRINT_NORM)
    texts, rc = nsd.format_batch(frames, desc, rec, ext, mode=T.PRINT_NORM)
    assert not any(rc)
    for k in range(len(desc)):
        check_v4_text(ora[k][0], vec["v4_fields"][k])
        check_v4_text(texts[k], vec["v4_fields"][k])


def test_ipv6_text_vs_reference(vec):
    frames, desc = IV.batch(vec["v6_frames"], vec["v6_caplen"])
    rec, ext, _, _ = T.oracle_records(frames, desc, mode=T.PRINT_NORM)
    ora = T.oracle_text_packets(frames, desc, mode=T.PRINT_NORM)
    texts, rc = nsd.format_batch(frames, desc, rec, ext, mode=T.PRINT_NORM)
    assert not any(rc)
    for k in range(len(desc)):
        check_v6_text(ora[k][0], vec["v6_fields"][k])
        check_v6_text(texts[k], vec["v6_fields"][k])


def test_icmp_checksum_vs_reference(vec):
    frames, desc = IV.batch(vec["icmp_frames"], vec["icmp_caplen"])
    rec, ext, _, _ = T.oracle_records(frames, desc, mode=T.PRINT_NORM)
    bad = (rec["nflags"] & nsd.F_ICMP_BAD) != 0
    assert np.array_equal(bad, vec["icmp_csum"] != 0)
    hrec = nsd.walk_cpu(frames, desc, mode=T.PRINT_NORM)[0]
    assert np.array_equal((hrec["nflags"] & nsd.F_ICMP_BAD) != 0, vec["icmp_csum"] != 0)
    texts, rc = nsd.format_batch(frames, desc, rec, ext, mode=T.PRINT_NORM)
    for k in range(len(desc)):
        m = REICMP.search(texts[k])
        assert m and (m.group(1).startswith(b"ok") == (vec["icmp_csum"][k] == 0))


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["full", "compact"])
def test_device_vs_reference(vec, schedule, form):
    """Device IPv4 header checksums and ICMPv4 verdicts == the reference's
    csum.h over the same bytes; the text rendered from the device records
    prints the reference's fields."""
    import torch
    for key in ("v4", "icmp"):
        frames, desc = IV.batch(vec[f"{key}_frames"], vec[f"{key}_caplen"])
        f = torch.from_numpy(frames).cuda()
        d = torch.from_numpy(desc.view(np.int64)).cuda()
        if form == "full":
            rec, ext, _, _ = nsd.dissect_device(f, d, mode=T.PRINT_NORM)
            drec = rec.cpu().numpy().view(nsd.REC_DTYPE)
            dext = ext.cpu().numpy().view(np.uint32)
            texts, rc = nsd.format_batch(frames, desc, drec, dext, mode=T.PRINT_NORM)
        else:
            crec, ext, _, _ = nsd.dissect_device_compact(f, d, mode=T.PRINT_NORM)
            drec = crec.cpu().numpy().view(nsd.CREC_DTYPE)
            dext = ext.cpu().numpy().view(np.uint32)
            texts, rc = nsd.format_batch_compact(frames, desc, drec, dext, mode=T.PRINT_NORM)
        assert not any(rc)
        if key == "v4":
            assert np.array_equal(drec["ip_csum"], vec["v4_fields"][:, 12].astype(np.uint16))
            for k in range(len(desc)):
                check_v4_text(texts[k], vec["v4_fields"][k])
        else:
            assert np.array_equal((drec["nflags"] & nsd.F_ICMP_BAD) != 0, vec["icmp_csum"] != 0)
