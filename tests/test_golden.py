"""CPU tests against the committed golden fixtures (tests/golden/, produced by
the reference's own parser objects via oracle/_ref/nsref, make_golden.py):

  - the oracle restatement reproduces the golden text (pins the oracle);
  - the PRODUCT host formatter, fed the oracle's records, reproduces it too;
  - the product tprintf wrap emulation reproduces the 80-column text;
  - names-on flavour (conf files) where /root/reference exists.
"""
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

import nsd
import nsd_testlib as T

G = T.GOLDEN
MODES = [T.PRINT_NORM, T.PRINT_LESS, T.PRINT_HEX, T.PRINT_ASCII, T.PRINT_HEX_ASCII]
REF_CONF = "/root/reference"


def load_golden(base):
    with gzip.open(os.path.join(G, base + ".txt.gz"), "rb") as f:
        data = f.read()
    with open(os.path.join(G, base + ".ends.json")) as f:
        ends = json.load(f)
    out, prev = [], 0
    for e in ends:
        out.append(data[prev:e])
        prev = e
    return out


def batch(name):
    lt, pkts = T.read_pcap(os.path.join(G, name + ".pcap"))
    frames, desc = T.batch_from_packets(pkts)
    return lt, pkts, frames, desc


ICMPV6 = 11   # NSD_OPS_ICMPV6


def host_only(texts_unsupported):
    """Packets whose text the oracle does not restate (host-rendered leaves)."""
    return {i for i, (_, u) in enumerate(texts_unsupported) if u}


def last_layer(r):
    n = int(r["nflags"]) & 7
    return (int(r["chain"]) >> (5 * (n - 1))) & 31 if 0 < n < 7 else -1


@pytest.mark.parametrize("name", ["tiny", "edge"])
@pytest.mark.parametrize("mode", MODES)
def test_oracle_matches_golden(name, mode):
    lt, pkts, frames, desc = batch(name)
    gold = load_golden(f"{name}.m{mode}.w65535")
    ora = T.oracle_text_packets(frames, desc, linktype=lt, mode=mode)
    assert len(gold) == len(pkts)
    bad = [i for i, (t, unsup) in enumerate(ora) if not unsup and t != gold[i]]
    assert not bad, f"oracle text differs at {bad[:10]}"
    if name == "tiny":
        assert not host_only(ora)


@pytest.mark.parametrize("name", ["tiny", "edge"])
@pytest.mark.parametrize("mode", MODES)
def test_formatter_matches_golden(name, mode):
    """Product formatter (record + raw bytes -> text) vs reference text."""
    lt, pkts, frames, desc = batch(name)
    gold = load_golden(f"{name}.m{mode}.w65535")
    rec, ext, _, _ = T.oracle_records(frames, desc, linktype=lt, mode=mode)
    texts, rc = nsd.format_batch(frames, desc, rec, ext, mode=mode, linktype=lt)
    ora = T.oracle_text_packets(frames, desc, linktype=lt, mode=mode)
    hosted = host_only(ora)
    rendered_leaves = icmpv6_bodies = 0
    for i in range(len(pkts)):
        if rec[i]["nflags"] & 0x20:          # overflow: the record holds no full chain
            assert rc[i] != 0
            continue
        assert rc[i] == 0, f"packet {i}: status {rc[i]}"
        assert texts[i] == gold[i], f"packet {i} differs"
        rendered_leaves += i in hosted
        icmpv6_bodies += i in hosted and last_layer(rec[i]) == ICMPV6
    if name == "tiny":
        assert not hosted
    elif mode in (T.PRINT_NORM, T.PRINT_LESS):
        assert rendered_leaves >= 4          # ARP, LLDP, IGMP, DCCP: text from the host leaves
    if name == "edge" and mode == T.PRINT_NORM:
        assert icmpv6_bodies >= 40           # ICMPv6 130-154 bodies (nsd_format_icmpv6.h)


@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_formatter_leaves_match_golden(mode):
    """The leaf frames (tests/leaf_cases.py): the oracle's records carry each
    leaf's end cursor (where the exit op's dump starts), the formatter checks
    its renderer's pulls end there, and the text equals the reference's."""
    lt, pkts, frames, desc = batch("leaves")
    gold = load_golden(f"leaves.m{mode}.w65535")
    rec, ext, _, _ = T.oracle_records(frames, desc, linktype=lt, mode=mode)
    texts, rc = nsd.format_batch(frames, desc, rec, ext, mode=mode, linktype=lt)
    host = moved = 0
    for i in range(len(pkts)):
        assert rc[i] == 0, f"packet {i}: status {rc[i]}"
        assert texts[i] == gold[i], f"packet {i} differs"
        if rec[i]["nflags"] & 0x10:
            host += 1
            n = int(rec[i]["nflags"]) & 7
            start = int(rec[i]["off2"][n - 2]) * 2 if 1 < n < 7 else -1
            moved += int(rec[i]["data_off"]) > start >= 0
    # most leaves pull something (PRINT_LESS: no ICMPv6 bodies, IGMP pulls nothing)
    assert host >= (2500 if mode == T.PRINT_NORM else 2000) and moved >= 1200, (host, moved)


@pytest.mark.parametrize("name", ["tiny", "edge", "leaves"])
@pytest.mark.parametrize("mode", MODES)
def test_formatter_compact_matches_golden(name, mode):
    """Compact 8-byte records (no cursors: each layer starts where the
    previous print left the cursor) render the reference's text too."""
    if name == "leaves" and mode not in (T.PRINT_NORM, T.PRINT_LESS):
        pytest.skip("leaf goldens exist for NORM / LESS")
    lt, pkts, frames, desc = batch(name)
    gold = load_golden(f"{name}.m{mode}.w65535")
    rec, ext, _, _ = T.oracle_records(frames, desc, linktype=lt, mode=mode)
    crec, pool = nsd.compact_of(rec, ext)
    texts, rc = nsd.format_batch_compact(frames, desc, crec, pool, mode=mode, linktype=lt)
    for i in range(len(pkts)):
        if rec[i]["nflags"] & 0x20:          # overflow: no chain in the record
            assert rc[i] != 0
            continue
        assert rc[i] == 0, f"packet {i}: status {rc[i]}"
        assert texts[i] == gold[i], f"packet {i} differs"


@pytest.mark.parametrize("key,cfg", [("udp64", T.SYN_UDP64), ("imix", T.SYN_IMIX), ("ipv6x", T.SYN_IPV6X)])
def test_prefix_text_formatter_compact(key, cfg):
    """Compact records of 64K prefixes render the nsref text digests."""
    with open(os.path.join(G, "prefix.json")) as f:
        want = json.load(f)
    frames, desc = T.make_batch(cfg, 65536)
    for m in (T.PRINT_NORM, T.PRINT_LESS):
        rec, ext, _, _ = T.oracle_records(frames, desc, mode=m)
        crec, pool = nsd.compact_of(rec, ext)
        texts, rc = nsd.format_batch_compact(frames, desc, crec, pool, mode=m)
        assert (rc == 0).all()
        assert hashlib.sha256(b"".join(texts)).hexdigest() == want[f"{key}:m{m}"]["text_sha256"]


@pytest.mark.parametrize("name", ["tiny", "edge"])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_wrap_matches_golden(name, mode):
    """tprintf's 80-column wrapping (tprintf.c:65-103) over the unwrapped
    stream, carrying the line counter across packets."""
    unwrapped = load_golden(f"{name}.m{mode}.w65535")
    wrapped = load_golden(f"{name}.m{mode}.w80")
    lt, pkts, frames, desc = batch(name)
    ora = T.oracle_text_packets(frames, desc, linktype=lt, mode=mode)
    state = 0
    for i, (u, w) in enumerate(zip(unwrapped, wrapped)):
        got, state = nsd.tprintf_wrap(u, cols=80, state=state)
        if ora[i][1]:
            state = 0 if w.endswith(b"\n") else state
            continue
        assert got == w, f"packet {i}: wrap differs"


@pytest.mark.skipif(not os.path.isdir(REF_CONF), reason="conf files live in /root/reference")
@pytest.mark.parametrize("name", ["tiny", "edge"])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_names_on(name, mode):
    lt, pkts, frames, desc = batch(name)
    gold = load_golden(f"{name}.names.m{mode}.w65535")
    try:
        assert nsd.lookup_init(REF_CONF) == 4
        assert T.oracle().nsor_lookup_init(REF_CONF.encode()) == 4
        rec, ext, _, _ = T.oracle_records(frames, desc, linktype=lt, mode=mode)
        texts, rc = nsd.format_batch(frames, desc, rec, ext, mode=mode, linktype=lt)
        ora = T.oracle_text_packets(frames, desc, linktype=lt, mode=mode)
    finally:
        nsd.lookup_cleanup()
        T.oracle().nsor_lookup_init(None)
    for i in range(len(pkts)):
        if rec[i]["nflags"] & 0x20:
            continue
        if not ora[i][1]:
            assert ora[i][0] == gold[i], f"oracle packet {i}"
        assert rc[i] == 0, f"formatter packet {i}: {rc[i]}"
        assert texts[i] == gold[i], f"formatter packet {i}"


def test_line_floor_golden():
    """lines.json (bench.py's line floor) is the restatement's: shard 0 of C3
    and C4 recomputed (distinct 128-byte lines of [off, off + W) per packet),
    and the floor is at least the algorithmic bytes W (a line holds at most
    128 of them)."""
    import ctypes
    L = T.oracle()
    L.nsor_line_floor_mt.restype = ctypes.c_uint64
    L.nsor_line_floor_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int]
    with open(os.path.join(G, "lines.json")) as f:
        lines = json.load(f)
    with open(os.path.join(G, "wsum.json")) as f:
        wsum = json.load(f)
    n = 1 << 24
    for key, cfg in (("imix", T.SYN_IMIX), ("ipv6x", T.SYN_IPV6X)):
        frames, desc = T.make_batch(cfg, n)
        got = int(L.nsor_line_floor_mt(frames.ctypes.data, desc.ctypes.data, n, 1, T.PRINT_NORM, 8))
        del frames, desc
        assert got == lines[f"{key}:0:{n}"], key
        assert 128 * got >= wsum[f"{key}:0:{n}"], key
    assert lines[f"udp64:0:{n}"] == n // 2   # 64-byte frames, two to a line


def test_prefix_digests():
    """64K-packet prefixes of C2/C3/C4: oracle records + counters + ΣW match
    the committed digests (text digests were taken from nsref)."""
    import make_golden_shim as mg
    with open(os.path.join(G, "prefix.json")) as f:
        want = json.load(f)
    for key, cfg in (("udp64", T.SYN_UDP64), ("imix", T.SYN_IMIX), ("ipv6x", T.SYN_IPV6X)):
        frames, desc = T.make_batch(cfg, 65536)
        for m in (T.PRINT_NORM, T.PRINT_LESS):
            rec, ext, cnt, sw = T.oracle_records(frames, desc, mode=m)
            w = want[f"{key}:m{m}"]
            assert mg.rec_digest(rec, ext) == w["records_sha256"], key
            assert [int(x) for x in cnt] == w["counters"], key
            assert sw == w["wsum"], key


@pytest.mark.parametrize("key,cfg", [("udp64", T.SYN_UDP64), ("imix", T.SYN_IMIX)])
def test_prefix_text_formatter(key, cfg):
    """Product formatter over 64K prefixes reproduces the nsref text digest."""
    with open(os.path.join(G, "prefix.json")) as f:
        want = json.load(f)
    frames, desc = T.make_batch(cfg, 65536)
    for m in (T.PRINT_NORM, T.PRINT_LESS):
        rec, ext, _, _ = T.oracle_records(frames, desc, mode=m)
        texts, rc = nsd.format_batch(frames, desc, rec, ext, mode=m)
        assert (rc == 0).all()
        assert hashlib.sha256(b"".join(texts)).hexdigest() == want[f"{key}:m{m}"]["text_sha256"]
