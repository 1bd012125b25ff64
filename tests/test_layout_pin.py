"""Line layout of the printers whose sources cannot compile here, pinned by
the reference's own format strings (CPU).

proto_ipv4.c, proto_ipv6.c, show_frame_hdr (dissector.h) and the SLL head
(dissector_sll.c) need the configure-generated config.h, so
their text is not printed by reference code anywhere in this build.  Their
printf format strings are: tests/ref_formats.py reads every `tprintf` call
in those functions out of the source text (with the colorize macros and
literal arguments, e.g. the checksum's "ok" / "bogus (!)" choice) into
tests/golden/ref_formats.json.  Here the oracle's and the product
formatter's text for each layer must be exactly the concatenation of those
strings along a control-flow path of the reference function - literals,
order, spacing and colour escapes - with only the conversions (%u, %s, %x
...) filled in; the values themselves are pinned by test_ip_pin.py
(csum.h / ipv4.h / ipv6.h) and test_sll.py (dev.c tables).

Known-answer-only (not pinned by reference code): which path a packet
takes - the trailer condition and window, the options loop's length rules,
the total-length trim, the frame header's VLAN condition - checked by the
packets below against the paths the reference's code takes for them (read
from the source), by SURVEY's known answers and by the edge goldens'
downstream text.
"""
import json
import os
import re
import struct

import numpy as np
import pytest

import nsd
import nsd_testlib as T
import ref_formats

FIX = os.path.join(T.GOLDEN, "ref_formats.json")
with open(FIX) as _f:
    REF = json.load(_f)
CALLS = {(c["file"], c["line"]): c for c in REF["calls"]}

CONV = re.compile(r"%(%|[-+ #0]*\d*(?:\.\d+)?(?:hh|h|ll|l|z|j|t)?[diouxXcsp])")


def conv_regex(spec):
    t = spec[-1]
    if spec == "%":
        return "%"
    if t == "s":
        return "(.*?)"
    if t in "di":
        return "(-?[0-9]+)"
    if t == "u":
        return "([0-9]+)"
    if t in "xX":
        m = re.search(r"\.(\d+)", spec)
        return "([0-9a-f]{%d,})" % int(m.group(1)) if m else "([0-9a-f]+)"
    if t == "c":
        return "(.)"
    raise ValueError(spec)


def call_regex(file, line, choice=None):
    """One tprintf call as a regex: its literal text escaped, each conversion
    a capture, or the argument's literal text when the argument is literal
    (`choice` picks a ?: alternative)."""
    c = CALLS[(file, line)]
    out, pos, k = [], 0, 0
    for m in CONV.finditer(c["fmt"]):
        out.append(re.escape(c["fmt"][pos:m.start()]))
        spec = m.group(1)
        if spec == "%":
            out.append("%")
        else:
            a = c["args"][k] if k < len(c["args"]) else None
            if isinstance(a, list):
                out.append(re.escape(a[choice]))
            elif isinstance(a, str) and spec[-1] == "s":
                out.append(re.escape(a))
            else:
                out.append(conv_regex(spec))
            k += 1
        pos = m.end()
    out.append(re.escape(c["fmt"][pos:]))
    return "".join(out)


def path_regex(file, items):
    """items: line numbers, (line, '*') for a call repeated in a loop, or
    (line, choice) for a call whose literal argument takes alternative
    `choice`."""
    parts = []
    for it in items:
        if isinstance(it, tuple) and it[1] == "*":
            parts.append("(?:" + call_regex(file, it[0]) + ")*")
        elif isinstance(it, tuple):
            parts.append(call_regex(file, it[0], it[1]))
        else:
            parts.append(call_regex(file, it))
    return "".join(parts)


V4 = "proto_ipv4.c"
V4_HEAD = [69, 70, 71, 72, 73, 74, 75, 76, 77, 78]
V4_OK = V4_HEAD + [(83, 1), 89]                                  # csum ok, no trailer
V4_TRAILER_BAD = [62, (64, "*"), 66] + V4_HEAD + [(83, 0), 87, 89]
OPT_1B = [137, 144]                                              # EOOL / NOP
OPT_OK = [137, 161, 163, (165, "*"), 166]
OPT_BAD = [137, 158]
V6 = [44, 45, 46, 47, 48, 49, 50, 51, 52]


def _csum(h):
    s = sum(struct.unpack(">%dH" % (len(h) // 2), h))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def eth(t):
    return bytes.fromhex("0a0b0c0d0e0f020304050607") + struct.pack(">H", t)


def ipv4(payload, proto=17, opts=b"", tot=None, good=True):
    ihl = 5 + len(opts) // 4
    tot = 20 + len(opts) + len(payload) if tot is None else tot
    h = bytearray(struct.pack(">BBHHHBBH4s4s", 0x40 | ihl, 0x10, tot, 0x1234, 0x4000, 61, proto, 0,
                              bytes([10, 1, 2, 3]), bytes([192, 168, 7, 9])) + opts)
    c = _csum(bytes(h))
    h[10:12] = struct.pack(">H", c if good else c ^ 0x0101)
    return bytes(h) + payload


UDP = struct.pack(">HHHH", 1024, 53, 12, 0) + b"abcd"


def ipv6(payload, nh=17):
    return (bytes([0x61, 0x23, 0x45, 0x67]) + struct.pack(">HBB", len(payload), nh, 63)
            + bytes(range(16)) + bytes(range(16, 32)) + payload)


# (name, frame, mode, path regex of the layer after Ethernet)
CASES = [
    ("v4_ok", eth(0x800) + ipv4(UDP), nsd.PRINT_NORM, path_regex(V4, V4_OK)),
    ("v4_trailer_bad", eth(0x800) + ipv4(UDP, tot=26, good=False) + b"\x01\x02", nsd.PRINT_NORM,
     path_regex(V4, V4_TRAILER_BAD)),
    # NOP, EOOL, record route (len 7), NOP: options walked to the end
    ("v4_opts", eth(0x800) + ipv4(UDP, opts=bytes([1, 0, 7, 7, 4, 10, 0, 0, 1, 1, 1, 1])), nsd.PRINT_NORM,
     path_regex(V4, V4_OK + OPT_1B + OPT_1B + OPT_OK + OPT_1B + OPT_1B + OPT_1B)),
    # NOP then an option whose length runs past the options: "invalid", out
    ("v4_opt_bad", eth(0x800) + ipv4(UDP, opts=bytes([1, 68, 9, 5])), nsd.PRINT_NORM,
     path_regex(V4, V4_OK + OPT_1B + OPT_BAD)),
    ("v4_less", eth(0x800) + ipv4(UDP), nsd.PRINT_LESS, path_regex(V4, [192])),
    ("v6", eth(0x86DD) + ipv6(UDP), nsd.PRINT_NORM, path_regex("proto_ipv6.c", V6)),
    ("v6_less", eth(0x86DD) + ipv6(UDP), nsd.PRINT_LESS, path_regex("proto_ipv6.c", [109])),
]

ETH_NORM = re.compile(rb"(?s)\A \[ Eth [^\n]*\n \[ Vendor [^\n]*\n")
ETH_LESS = re.compile(rb"\A [^\n]*? => [^\n]*? \x1b\[1m\(null\)\x1b\[0m")
NEXT = re.compile(rb"\A(?: \[ (?:UDP|TCP|ICMP|Chr|Hex)| UDP | TCP |\n)")


def _texts(frames, desc, mode, linktype=1, sll=None):
    rec, chains, _ = nsd.walk_cpu(frames, desc, mode=mode, linktype=linktype, sll=sll)
    assert not chains
    prod, rc = nsd.format_batch(frames, desc, rec, mode=mode, linktype=linktype, sll=sll)
    assert not rc.any()
    orc = [t for t, _ in T.oracle_text_packets(frames, desc, linktype=linktype, mode=mode, sll=sll)]
    return prod, orc


def test_fixture_is_current():
    """The committed strings are what the reference's sources hold (build
    container only; the GPU boxes have no /root/reference)."""
    if not os.path.isdir(ref_formats.REF):
        pytest.skip("no /root/reference")
    assert ref_formats.extract_all() == REF


def test_fixture_covers_the_printers():
    funcs = {c["func"] for c in REF["calls"]}
    assert funcs == {"ipv4", "ipv4_less", "ipv6", "ipv6_less", "__show_frame_hdr", "sll_print_full",
                     "sll_print_less"}
    assert CALLS[(V4, 83)]["args"][1] == ["\x1b[30;41mbogus (!)\x1b[0m", "ok"]


@pytest.mark.parametrize("name,frame,mode,rx", CASES, ids=[c[0] for c in CASES])
def test_ip_layer_is_the_reference_format_sequence(name, frame, mode, rx):
    frames, desc = T.batch_from_packets([frame])
    prod, orc = _texts(frames, desc, mode)
    eth_rx = ETH_NORM if mode == nsd.PRINT_NORM else ETH_LESS
    for who, text in (("product", prod[0]), ("oracle", orc[0])):
        m = eth_rx.match(text)
        assert m, (who, text[:200])
        rest = text[m.end():].decode("latin-1")
        lm = re.match(rx, rest, re.S)
        assert lm, f"{who}: {rest[:400]!r} is not the reference's format sequence"
        after = rest[lm.end():].encode("latin-1")
        assert NEXT.match(after), f"{who}: layer text continues past the path: {after[:120]!r}"
    assert prod[0] == orc[0]


def test_geo_lines_never_print():
    """GeoIP is off without a database (geoip.h:43): the Geo lines
    of proto_ipv4.c / proto_ipv6.c are outside the parity domain and must
    not appear."""
    frames, desc = T.batch_from_packets([c[1] for c in CASES])
    for mode in (nsd.PRINT_NORM, nsd.PRINT_LESS):
        prod, orc = _texts(frames, desc, mode)
        for t in prod + orc:
            assert b"Geo (" not in t


FH = "dissector.h"


def _fh_regex(mode, vlan=False, ts=None):
    if mode == nsd.PRINT_LESS:
        return path_regex(FH, [80])
    rx = path_regex(FH, [87])
    if vlan:
        rx += path_regex(FH, [99, 100, 101, 102, 103, 104])
    return rx


def test_frame_header_is_the_reference_format_sequence():
    """show_frame_hdr's lines (dissector.h:53-108) for every packet type,
    the v2 timestamp sources, the VLAN line, and PRINT_LESS; the packet
    type and timestamp-source strings are the reference's tables."""
    types = dict(REF["tables"]["packet_types"])
    order = ["PACKET_HOST", "PACKET_BROADCAST", "PACKET_MULTICAST", "PACKET_OTHERHOST", "PACKET_OUTGOING",
             None, "PACKET_USER", "PACKET_KERNEL"]
    ts = [t for _, t in REF["tables"]["ts_source"]]   # raw hw, sys hw, sw, none
    fh = np.zeros(1, dtype=nsd.FH_DTYPE)[0]
    fh["len"], fh["sec"], fh["nsec"] = 98, 1700000000, 12
    sll = np.zeros(1, dtype=nsd.SLL_DTYPE)[0]
    for mode in (nsd.PRINT_NORM, nsd.PRINT_LESS):
        for t in range(10):
            sll["pkttype"] = t
            for st, src in ((1 << 31, ts[0]), (1 << 30, ts[1]), (1 << 29, ts[2]), (0, ts[3])):
                fh["status"] = st
                for nsec, vlan in ((12, False), (16, True)):
                    fh["nsec"] = nsec
                    got = [nsd.format_frame_hdr(fh, sll=sll, mode=mode, count=t + 5),
                           T.oracle_frame_hdr(fh, sll, mode=mode, count=t + 5)]
                    rx = _fh_regex(mode, vlan=vlan)
                    for g in got:
                        m = re.fullmatch(rx, g.decode("latin-1"), re.S)
                        assert m, (mode, t, st, g)
                        name = types.get(order[t]) if t < len(order) and order[t] else "?"
                        assert m.group(1) == name and m.group(2) == "?"
                        if mode == nsd.PRINT_NORM:
                            assert m.group(7) == src
                    assert got[0] == got[1]


SLL_F = "dissector_sll.c"


def test_sll_head_is_the_reference_format_sequence():
    """The LINKTYPE_LINUX_SLL head (dissector_sll.c:39-82): the full line
    (then the Ethernet chain, or " [ Unknown protocol ]" for a hatype that
    maps to no link type) and the less line, pkt_type2str's strings."""
    names = dict(REF["tables"]["pkt_type2str"])
    order = ["PACKET_HOST", "PACKET_BROADCAST", "PACKET_MULTICAST", "PACKET_OTHERHOST", "PACKET_OUTGOING",
             None, "PACKET_USER", "PACKET_KERNEL"]
    frames_l, slls = [], []
    for t in (0, 1, 4, 6, 7, 9):
        for hatype, proto in ((1, 0x0800), (0xFFFE, 0x0800)):
            s = np.zeros(1, dtype=nsd.SLL_DTYPE)[0]
            s["family"], s["protocol"], s["ifindex"], s["hatype"] = 17, proto, 1, hatype
            s["pkttype"], s["halen"] = t, 6
            s["addr"][:6] = [2, 3, 4, 5, 6, 7]
            slls.append(s)
            frames_l.append(ipv4(UDP))
    sll = np.array(slls, dtype=nsd.SLL_DTYPE)
    frames, desc = T.batch_from_packets(frames_l)
    full = path_regex(SLL_F, [44, 45, 47, 49, 50, 52, 53])
    less = path_regex(SLL_F, [74, 76, 78, 79, 81])
    unk = call_regex(SLL_F, 65)
    for mode, rx in ((nsd.PRINT_NORM, full), (nsd.PRINT_LESS, less)):
        prod, orc = _texts(frames, desc, mode, linktype=nsd.LINKTYPE_LINUX_SLL, sll=sll)
        for k in range(len(slls)):
            for who, text in (("product", prod[k]), ("oracle", orc[k])):
                s = text.decode("latin-1")
                m = re.match(rx, s, re.S)
                assert m, (who, mode, k, s[:300])
                t = int(slls[k]["pkttype"])
                want = names.get(order[t]) if t < len(order) and order[t] else dict(names)[None]
                assert m.group(2) == want, (who, m.group(2), want)
                rest = s[m.end():]
                if mode == nsd.PRINT_NORM and int(slls[k]["hatype"]) == 0xFFFE:
                    assert re.match(unk, rest), (who, rest[:100])
                elif mode == nsd.PRINT_NORM:
                    assert rest.startswith(" [ IPv4 "), (who, rest[:100])
            assert prod[k] == orc[k]
