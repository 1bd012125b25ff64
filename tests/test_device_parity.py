"""GPU parity: device records (through the C ABI -> HIP kernel) vs the CPU
oracle on the same inputs, bit-exact.  Runs on an MI355X (-m gpu)."""
import numpy as np
import pytest

import edge_cases
import nsd
import nsd_testlib as T

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("schedule_small")]

MODES = [T.PRINT_NORM, T.PRINT_LESS, T.PRINT_HEX]


def _chain(rec, ext, i):
    """(ids, offsets) of packet i, resolving the ext slot."""
    r = rec[i]
    n = int(r["nflags"]) & 7
    if n == 7:
        slot = int.from_bytes(bytes(r["off2"][:4]), "little")
        if slot == 0xFFFFFFFF:
            return ("overflow",)
        pkt, ids, offs = nsd.ext_entry(ext, slot)
        assert pkt == i
        return ids, offs
    ids = tuple((int(r["chain"]) >> (5 * k)) & 31 for k in range(n))
    offs = tuple([0] + [2 * int(x) for x in r["off2"][:max(n - 1, 0)]])
    return ids, offs[:n]


def assert_same_records(dev, ora, dext, oext):
    n = len(ora)
    assert len(dev) == n
    for f in ("data_off", "tail_off", "ip_csum", "nflags"):
        bad = np.nonzero(dev[f] != ora[f])[0]
        assert len(bad) == 0, f"{f} differs at {bad[:10]}: dev={dev[f][bad[:5]]} ora={ora[f][bad[:5]]}"
    nonext = (ora["nflags"] & 7) != 7
    assert np.array_equal(dev["chain"], ora["chain"]), "chain ids differ"
    assert np.array_equal(dev["off2"][nonext], ora["off2"][nonext]), "layer offsets differ"
    for i in np.nonzero(~nonext)[0]:
        assert _chain(dev, dext, i) == _chain(ora, oext, i), f"ext chain differs at {i}"


def _check(frames, desc, mode):
    rec, ext, cnt = nsd.entry_batch(frames, desc, mode=mode)
    orec, oext, ocnt, _ = T.oracle_records(frames, desc, mode=mode)
    assert_same_records(rec, orec, ext, oext)
    assert np.array_equal(cnt, ocnt), f"counters differ: {nsd.unpack_counters(cnt)} vs {nsd.unpack_counters(ocnt)}"
    return rec, ext


@pytest.mark.parametrize("mode", MODES)
def test_edge_cases(mode):
    frames, desc = T.batch_from_packets(edge_cases.cases())
    _check(frames, desc, mode)


@pytest.mark.parametrize("align", [1, 16])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_leaf_walks(mode, align):
    """The device walks of the host-rendered leaves (nsd_leaf.h): ARP, DCCP,
    IGMP, LLDP and ICMPv6 130-154 frames (tests/golden/leaves.pcap, whose
    reference text pins the end cursors through the exit-op dump); every
    record's data_off is the leaf's end, as the oracle's."""
    _, pkts = T.read_pcap(T.GOLDEN + "/leaves.pcap")
    frames, desc = T.batch_from_packets(pkts, align=align)
    rec, _ = _check(frames, desc, mode)
    host = rec["nflags"] & 0x10 != 0
    assert host.sum() >= 2000


@pytest.mark.parametrize("align", [1, 2, 16])
def test_edge_cases_unaligned(align):
    frames, desc = T.batch_from_packets(edge_cases.cases(), align=align)
    _check(frames, desc, T.PRINT_NORM)


@pytest.mark.parametrize("cfg,n", [(T.SYN_UDP64, 1000), (T.SYN_UDP64, 65536),
                                   (T.SYN_IMIX, 65536), (T.SYN_IPV6X, 65536)])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_synthetic_configs(cfg, n, mode):
    frames, desc = T.make_batch(cfg, n)
    _check(frames, desc, mode)


def _check_compact(frames, desc, mode):
    """Compact device records == the oracle's records minus the cursors
    (nsd.compact_of): ids inline or in the side words, longer chains
    compared by their entries; counters equal.  Returns (crec, pool)."""
    import torch
    f = torch.from_numpy(frames).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    crec, ext, used, cnt = nsd.dissect_device_compact(f, d, mode=mode)
    torch.cuda.synchronize()
    return _compare_compact(crec, ext, used, cnt, frames, desc, mode)


def _compare_compact(crec, ext, used, cnt, frames, desc, mode):
    n = len(desc)
    got = crec.cpu().numpy().view(nsd.CREC_DTYPE)[:n]
    dpool = ext.cpu().numpy().view(np.uint32)[:n + int(used.item())]
    orec, oext, ocnt, _ = T.oracle_records(frames, desc, mode=mode)
    want, wpool = nsd.compact_of(orec, oext)
    for fld in ("ip_csum", "nflags", "nlayers"):
        bad = np.nonzero(got[fld] != want[fld])[0]
        assert len(bad) == 0, f"{fld} differs at {bad[:10]}"
    deep = ((want["nflags"] & 7) == 7) & (want["nlayers"] == 0)
    assert np.array_equal(got["chain"][~deep], want["chain"][~deep]), "chain ids differ"
    # side words: ids 6.. of 7..12-layer chains, or a host leaf's end (NSD_F_LEAF_END)
    leaf = (want["nflags"] & nsd.F_LEAF_END) != 0
    side = (want["nlayers"] != 0) | (leaf & ~deep)
    assert np.array_equal(dpool[:n][side], wpool[:n][side]), "side words differ"
    for i in np.nonzero(deep)[0]:
        if want[i]["chain"] == 0xFFFFFFFF:      # no entry (pool full)
            assert got[i]["chain"] == 0xFFFFFFFF
            continue
        gp, gids, goffs = nsd.ext_entry(dpool, int(got[i]["chain"]))
        _, oids, _ = nsd.ext_entry(wpool, int(want[i]["chain"]))
        assert gp == i and gids == oids and not any(goffs), f"ext chain differs at {i}"
        if leaf[i]:
            assert dpool[int(got[i]["chain"]) + 2] == wpool[int(want[i]["chain"]) + 2], f"leaf end differs at {i}"
    assert np.array_equal(cnt.cpu().numpy().view(np.uint64), ocnt)
    return got, dpool


@pytest.mark.parametrize("mode", MODES)
def test_compact_edge_and_leaves(mode):
    """Compact records of the edge cases and the leaf set: the host-rendered
    leaves' ends (NSD_F_LEAF_END in side words / entries) equal the oracle's
    data_off, which the reference text pins (tests/golden/leaves.*), and the
    formatter renders every record with its leaf end checked."""
    _, leaves = T.read_pcap(T.GOLDEN + "/leaves.pcap")
    frames, desc = T.batch_from_packets(edge_cases.cases() + leaves, align=2)
    got, pool = _check_compact(frames, desc, mode)
    if mode in (T.PRINT_NORM, T.PRINT_LESS):
        assert ((got["nflags"] & nsd.F_LEAF_END) != 0).sum() >= 2000
        texts, rc = nsd.format_batch_compact(frames, desc, got, pool, mode=mode)
        assert ((rc == 0) | ((got["nflags"] & nsd.F_OVERFLOW) != 0)).all()   # overflow: per-packet path
        # a wrong leaf end is refused
        k = int(np.nonzero(((got["nflags"] & nsd.F_LEAF_END) != 0) & ((got["nflags"] & 7) != 7))[0][0])
        bad = pool.copy()
        bad[k] ^= 1
        _, rc2 = nsd.format_batch_compact(frames, desc, got, bad, mode=mode)
        assert rc2[k] != 0


@pytest.mark.parametrize("cfg", [T.SYN_UDP64, T.SYN_IMIX, T.SYN_IPV6X])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_compact_synthetic_text(cfg, mode):
    """Device compact records of 64K-packet prefixes -> the host formatter
    -> the reference text digest (tests/golden/prefix.json)."""
    import hashlib
    import json
    key = {T.SYN_UDP64: "udp64", T.SYN_IMIX: "imix", T.SYN_IPV6X: "ipv6x"}[cfg]
    frames, desc = T.make_batch(cfg, 65536)
    crec, ext = _check_compact(frames, desc, mode)
    texts, rc = nsd.format_batch_compact(frames, desc, crec, ext, mode=mode)
    assert (rc == 0).all()
    with open(T.GOLDEN + "/prefix.json") as fh:
        want = json.load(fh)[f"{key}:m{mode}"]["text_sha256"]
    assert hashlib.sha256(b"".join(texts)).hexdigest() == want


def _long_chains(n, seed=11):
    """IPv6 with 2..7 Hop-by-Hop / DestOpts headers of 8..128 bytes each: most
    chains run past several 128-byte continuation windows and past the
    record's 6 layers (ext entries from the per-wave chunks)."""
    import random
    rnd = random.Random(seed)
    E = edge_cases
    pkts = []
    for _ in range(n):
        k = rnd.randint(2, 7)
        kinds = [rnd.choice([0, 60]) for _ in range(k)]
        body = b""
        for j in range(k):
            nh = kinds[j + 1] if j + 1 < k else 17
            hl = rnd.randint(0, 15)
            body += bytes([nh, hl]) + bytes(rnd.randrange(256) for _ in range((hl + 1) * 8 - 2))
        body += E.udp(payload=bytes(rnd.randrange(8)))
        pkts.append(E.eth(0x86DD) + E.ipv6(kinds[0], len(body)) + body)
    return pkts


@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_long_ext_chains(mode):
    frames, desc = T.batch_from_packets(_long_chains(30000), align=2)
    rec, _ = _check(frames, desc, mode)
    assert ((rec["nflags"] & 7) == 7).mean() > 0.3      # many chains past 6 layers


def test_imix_odd_alignment():
    frames, desc = T.make_batch(T.SYN_IMIX, 20000, align=1)
    _check(frames, desc, T.PRINT_NORM)


def test_device_resident_torch():
    """The device-resident entry (torch tensors, current stream) gives the
    same records as the host batch path."""
    import torch
    frames, desc = T.make_batch(T.SYN_IMIX, 50000)
    f = torch.from_numpy(frames).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    rec, ext, ext_used, counters = nsd.dissect_device(f, d, mode=T.PRINT_NORM)
    torch.cuda.synchronize()
    drec = rec.cpu().numpy().view(nsd.REC_DTYPE)
    orec, oext, ocnt, _ = T.oracle_records(frames, desc)
    dext = ext.cpu().numpy().view(np.uint32)[:int(ext_used.item())]
    assert_same_records(drec, orec, dext, oext)
    assert np.array_equal(counters.cpu().numpy().view(np.uint64), ocnt)


def test_empty_batch_and_caplen_limit():
    rec, ext, cnt = nsd.entry_batch(np.zeros(64, np.uint8), np.zeros(0, np.uint64))
    assert len(rec) == 0
    with pytest.raises(nsd.NsdError):
        nsd.entry_batch(np.zeros(70000, np.uint8), np.array([T.desc_pack(0, 66000)], np.uint64))


@pytest.mark.parametrize("words", [0, 68, 200])
def test_ext_pool_full(words):
    """A pool too small for every ext chain: the packets holding an entry
    match the oracle's chain, every entry lies inside the pool and no two
    overlap, the rest carry NSD_F_OVERFLOW with slot 0xFFFFFFFF."""
    frames, desc = T.batch_from_packets(edge_cases.cases())
    rec, ext, cnt = nsd.entry_batch(frames, desc, ext_words=words)
    orec, oext, _, _ = T.oracle_records(frames, desc)          # full-capacity reference
    need = np.nonzero((orec["nflags"] & 7) == 7)[0]
    assert len(need) > 2
    assert np.array_equal(np.nonzero((rec["nflags"] & 7) == 7)[0], need)
    spans = []
    for i in need:
        slot = int.from_bytes(bytes(rec[i]["off2"][:4]), "little")
        if slot == 0xFFFFFFFF:
            assert rec[i]["nflags"] & 0x20
        else:
            ids, _ = _chain(orec, oext, i)
            spans.append((slot, slot + nsd.ext_words(len(ids))))
            assert spans[-1][1] <= words
            assert _chain(rec, ext, i) == _chain(orec, oext, i)
    assert (len(spans) >= 1) == (words >= 68)
    spans.sort()
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
    assert int(cnt[nsd.CNT_OVERFLOW]) >= len(need) - len(spans)


@pytest.mark.parametrize("depth", [1, 3])
def test_pipe_batches(depth):
    """The pipelined host-batch path (nsd_pipe_*): batches of different
    sizes and configs in flight together; every batch's records, ext and
    counters equal the oracle's for that batch."""
    specs = [(T.SYN_IMIX, 20000, 0), (T.SYN_IPV6X, 7000, 0), (T.SYN_UDP64, 1, 5),
             (T.SYN_IMIX, 15000, 20000), (T.SYN_IPV6X, 9000, 7000), (T.SYN_IMIX, 3, 99)]
    batches = [T.make_batch(cfg, n, lo=lo) for cfg, n, lo in specs]
    max_pkts = max(len(d) for _, d in batches)
    max_bytes = max(f.nbytes for f, _ in batches)
    words = nsd.ext_pool_words(max_pkts)
    pipe = nsd.Pipe(max_pkts, max_bytes, ext_words=words, depth=depth)
    outs = []
    for frames, desc in batches:
        rec = np.zeros(len(desc), dtype=nsd.REC_DTYPE)
        ext = np.zeros(words, dtype=np.uint32)
        ec = np.zeros(1, np.uint32)
        cnt = np.zeros(nsd.NCOUNTERS, np.uint64)
        st = np.full(1, -99, np.int32)
        pipe.submit(frames, desc, rec, ext, ec, cnt, st)
        outs.append((rec, ext, ec, cnt, st))
    assert pipe.drain() == 0
    for (frames, desc), (rec, ext, ec, cnt, st) in zip(batches, outs):
        assert st[0] == 0
        orec, oext, ocnt, _ = T.oracle_records(frames, desc)
        assert_same_records(rec, orec, ext[:int(ec[0])], oext)
        assert np.array_equal(cnt, ocnt)
    assert pipe.wait() == 1
    pipe.close()


@pytest.mark.parametrize("depth", [1, 3])
def test_pipe_batches_compact(depth):
    """The compact-record pipe (nsd_pipe_create_compact / _submit_compact):
    batches of different sizes and configs in flight together (the deep
    IPv6 chains need side words and entries, IMIX none); each batch's
    records, side words / entries and counters equal compact_of(oracle)."""
    specs = [(T.SYN_IMIX, 20000, 0), (T.SYN_IPV6X, 7000, 0), (T.SYN_UDP64, 1, 5),
             (T.SYN_IPV6X, 9000, 7000), (T.SYN_IMIX, 3, 99)]
    batches = [T.make_batch(cfg, n, lo=lo) for cfg, n, lo in specs]
    batches.append(T.batch_from_packets(_long_chains(3000), align=2))
    max_pkts = max(len(d) for _, d in batches)
    max_bytes = max(f.nbytes for f, _ in batches)
    words = max_pkts + nsd.ext_pool_words(max_pkts)
    pipe = nsd.Pipe(max_pkts, max_bytes, ext_words=words, depth=depth, compact=True)
    outs = []
    for frames, desc in batches:
        rec = np.zeros(len(desc), dtype=nsd.CREC_DTYPE)
        ext = np.zeros(words, dtype=np.uint32)
        ec = np.zeros(1, np.uint32)
        cnt = np.zeros(nsd.NCOUNTERS, np.uint64)
        st = np.full(1, -99, np.int32)
        pipe.submit(frames, desc, rec, ext, ec, cnt, st)
        outs.append((rec, ext, ec, cnt, st))
    assert pipe.drain() == 0
    for (frames, desc), (rec, ext, ec, cnt, st) in zip(batches, outs):
        assert st[0] == 0
        n = len(desc)
        orec, oext, ocnt, _ = T.oracle_records(frames, desc)
        want, wpool = nsd.compact_of(orec, oext)
        assert np.array_equal(cnt, ocnt)
        for fld in ("ip_csum", "nflags", "nlayers"):
            assert np.array_equal(rec[fld], want[fld]), fld
        deep = ((want["nflags"] & 7) == 7) & (want["nlayers"] == 0)
        assert np.array_equal(rec["chain"][~deep], want["chain"][~deep])
        side = want["nlayers"] != 0
        assert np.array_equal(ext[:n][side], wpool[:n][side])
        for i in np.nonzero(deep)[0]:
            gp, gids, _ = nsd.ext_entry(ext, int(rec[i]["chain"]))
            _, oids, _ = nsd.ext_entry(wpool, int(want[i]["chain"]))
            assert gp == i and gids == oids
        texts, rc = nsd.format_batch_compact(frames, desc, rec, ext)
        assert (rc == 0).all()
    pipe.close()


def _icmp_sweep(seed=7):
    """ICMPv4 messages of every length class the checksum paths split on
    (inside the staged window, just past it, 1-2 KiB, > 2 KiB), good and
    bad sums, odd lengths, VLAN-shifted and IPv4-trimmed (trailer) frames."""
    import random
    rnd = random.Random(seed)
    E = edge_cases
    pkts = []
    for plen in list(range(0, 80)) + list(range(80, 3000, 37)) + [4000, 8000, 9000]:
        body = bytes(rnd.randrange(256) for _ in range(plen))
        for good in (True, False):
            for vlan in (False, True):
                l2 = E.eth(0x8100) + E.be16(5) + E.be16(0x0800) if vlan else E.eth(0x0800)
                msg = E.icmp(payload=body, good=good)
                trailer = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 0, 3, 17])))
                pkts.append(l2 + E.ipv4(1, len(msg)) + msg + trailer)
    return pkts


@pytest.mark.parametrize("align", [1, 2, 16])
def test_icmp_checksum_sweep(align):
    frames, desc = T.batch_from_packets(_icmp_sweep(), align=align)
    _check(frames, desc, T.PRINT_NORM)


def _packets_of(frames, desc):
    offs, caps = T.desc_off(desc), T.desc_caplen(desc)
    return [bytes(frames[o:o + c]) for o, c in zip(offs, caps)]


def _mixed_tiles(seed=5):
    """64-packet tiles of different kinds in a fixed order: C4 tiles (nearly
    every packet to the walkers: busy walkers, L2 touches of the next tiles),
    C2 tiles (none), long chains (walkers suspended at several windows and
    carried into the next tiles), edge cases (MPLS / SLL-less restarts,
    leaves, ICMP pending) and IMIX at odd offsets."""
    import random
    rnd = random.Random(seed)
    c4 = _packets_of(*T.make_batch(T.SYN_IPV6X, 64 * 42))
    c2 = _packets_of(*T.make_batch(T.SYN_UDP64, 64 * 18))
    c3 = _packets_of(*T.make_batch(T.SYN_IMIX, 64 * 6))
    lc = _long_chains(64 * 12, seed=seed)
    ed = edge_cases.cases()
    src = {"c4": c4, "c2": c2, "c3": c3, "lc": lc}
    order = ["c4", "c4", "c4", "c2", "lc", "c4", "c3", "c4", "c4", "lc", "c2", "c2", "c4", "ed"] * 6
    pkts = []
    for k in order:
        if k == "ed":
            pkts += [ed[rnd.randrange(len(ed))] for _ in range(64)]
        else:
            pkts += [src[k].pop() for _ in range(64)]
    return pkts


@pytest.mark.parametrize("grid", [1, 3, 0])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_walker_pool_mixed_tiles(grid, mode):
    """The general walk's walker pool under few blocks (grid 1: four waves
    walk every tile, so walkers carry across many fast walks, refill mid
    session and drain at the end) over tiles that alternate between
    walker-heavy, walker-free and deep-chain kinds: records, ext chains and
    counters equal the oracle's, for both record forms."""
    import torch
    frames, desc = T.batch_from_packets(_mixed_tiles(), align=2)
    orec, oext, ocnt, _ = T.oracle_records(frames, desc, mode=mode)
    f = torch.from_numpy(frames).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    rec, ext, ext_used, counters = nsd.dissect_device(f, d, mode=mode, grid=grid)
    torch.cuda.synchronize()
    drec = rec.cpu().numpy().view(nsd.REC_DTYPE)
    dext = ext.cpu().numpy().view(np.uint32)[:int(ext_used.item())]
    assert_same_records(drec, orec, dext, oext)
    assert np.array_equal(counters.cpu().numpy().view(np.uint64), ocnt)
    if grid == 0:
        _check_compact(frames, desc, mode)


def _plain_tiles(seed=9, n=64 * 48):
    """Ethernet / IPv4 (no options) / TCP or UDP frames only, so whole tiles
    take the split fast kernel's plain path (plain_walk): frame lengths 42..
    120, total lengths below the header, inside the frame (trimmed) and past
    it, good and bad header checksums, TCP / UDP bodies shorter than their
    headers."""
    import random
    rnd = random.Random(seed)
    pkts = []
    for k in range(n):
        cap = rnd.choice([42, 43, 53, 54, 55, 60, 64, 64, 64, 90, 120])
        proto = rnd.choice([6, 17])
        r = rnd.random()
        totlen = (rnd.randrange(0, 20) if r < 0.15 else rnd.randrange(cap - 14, cap + 30) if r < 0.4
                  else rnd.randrange(20, cap - 14 + 1))
        hdr = bytearray([0x45, rnd.randrange(256)]) + totlen.to_bytes(2, "big") + \
            bytes(rnd.randrange(256) for _ in range(4)) + bytes([rnd.randrange(256), proto, 0, 0]) + \
            bytes(rnd.randrange(256) for _ in range(8))
        if rnd.random() < 0.5:
            s = sum(int.from_bytes(hdr[i:i + 2], "big") for i in range(0, 20, 2))
            while s >> 16:
                s = (s & 0xFFFF) + (s >> 16)
            hdr[10:12] = (~s & 0xFFFF).to_bytes(2, "big")
        else:
            hdr[10:12] = rnd.randrange(65536).to_bytes(2, "big")
        eth = bytes(rnd.randrange(256) for _ in range(12)) + b"\x08\x00"
        body = bytes(rnd.randrange(256) for _ in range(cap - 34))
        pkts.append(eth + bytes(hdr) + body)
    return pkts


@pytest.mark.parametrize("align", [1, 2, 16])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_plain_tiles(mode, align):
    """Tiles of plain IPv4 TCP / UDP frames (the split fast kernel's plain
    path; the fused kernel's fast walk) at odd and even alignments: records
    of both forms and counters equal the oracle's."""
    frames, desc = T.batch_from_packets(_plain_tiles(), align=align)
    _check(frames, desc, mode)
    _check_compact(frames, desc, mode)


def _not_plain(rnd, pkt):
    """One frame the plain path must refuse, made from a plain one: IHL 6
    (an options word), an 802.1Q tag, ICMP, or a frame one byte too short."""
    kind = rnd.randrange(4)
    if kind == 0:
        ip = bytearray(pkt[14:34])
        ip[0] = 0x46
        return pkt[:14] + bytes(ip) + b"\x01\x01\x01\x00" + pkt[34:]
    if kind == 1:
        return pkt[:12] + b"\x81\x00\x00\x05" + pkt[12:]
    if kind == 2:
        return pkt[:23] + b"\x01" + pkt[24:]
    return pkt[:41]


@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_plain_tiles_partial_and_mixed(mode):
    """The plain path's wave-level edges: a partial last tile (64 * 48 + 17
    frames: invalid lanes with clamped descriptors stay out of the ballot),
    and tiles of plain frames where one random lane holds a frame that is not
    plain (the whole tile then goes through fast_walk); both record forms,
    under both schedules (the module's schedule fixture)."""
    import random
    rnd = random.Random(23)
    pkts = _plain_tiles(seed=5, n=64 * 48 + 17)
    frames, desc = T.batch_from_packets(pkts, align=2)
    _check(frames, desc, mode)
    _check_compact(frames, desc, mode)
    for t in range(0, 48, 3):   # one non-plain lane in every third tile
        k = 64 * t + rnd.randrange(64)
        pkts[k] = _not_plain(rnd, pkts[k])
    frames, desc = T.batch_from_packets(pkts, align=1)
    _check(frames, desc, mode)
    _check_compact(frames, desc, mode)


def _imix_tiles(seed=11, n=64 * 48):
    """Ethernet / [one 802.1Q tag] / IPv4 (no options) / TCP, UDP or ICMPv4
    frames only, whole tiles of C3's chains through fast_walk (both
    schedules; the straight-line plain4 walk of r05 is removed): frame
    lengths 38 .. 1500, total lengths
    below the header, inside the frame (trimmed) and past it, good and bad
    header checksums, ICMPv4 messages inside the window and past it with
    good and bad sums, odd and even lengths, L4 bodies shorter than their
    headers."""
    import random
    rnd = random.Random(seed)
    pkts = []
    for k in range(n):
        vlan = rnd.random() < 0.5
        v = 4 if vlan else 0
        cap = rnd.choice([38, 41, 42, 45, 46, 53, 58, 62, 63, 64, 64, 64, 65, 66, 77, 90, 128, 200, 576, 1500])
        cap = max(cap, 34 + v)
        proto = rnd.choice([1, 1, 6, 17])
        r = rnd.random()
        room = cap - 14 - v
        totlen = (rnd.randrange(0, 20) if r < 0.1 else rnd.randrange(room, room + 30) if r < 0.3
                  else rnd.randrange(20, room + 1))
        hdr = bytearray([0x45, rnd.randrange(256)]) + totlen.to_bytes(2, "big") + \
            bytes(rnd.randrange(256) for _ in range(4)) + bytes([rnd.randrange(256), proto, 0, 0]) + \
            bytes(rnd.randrange(256) for _ in range(8))
        s = sum(int.from_bytes(hdr[i:i + 2], "big") for i in range(0, 20, 2))
        while s >> 16:
            s = (s & 0xFFFF) + (s >> 16)
        hdr[10:12] = ((~s & 0xFFFF) if rnd.random() < 0.7 else rnd.randrange(65536)).to_bytes(2, "big")
        body = bytearray(rnd.randrange(256) for _ in range(cap - 34 - v))
        if proto == 1 and rnd.random() < 0.6:
            # a good ICMPv4 sum over the post-trim message (odd trailing byte dropped)
            x = totlen - 20   # the trim (proto_ipv4.c:174-175)
            mlen = x if 0 <= x < len(body) else len(body)
            if mlen >= 4:
                body[2:4] = b"\0\0"
                w = mlen & ~1
                s = sum(int.from_bytes(body[i:i + 2], "little") for i in range(0, w, 2))
                while s >> 16:
                    s = (s & 0xFFFF) + (s >> 16)
                body[2:4] = (~s & 0xFFFF).to_bytes(2, "little")
        eth = bytes(rnd.randrange(256) for _ in range(12))
        eth += (b"\x81\x00" + rnd.randrange(65536).to_bytes(2, "big") + b"\x08\x00") if vlan else b"\x08\x00"
        pkts.append(eth + bytes(hdr) + bytes(body))
    return pkts


def _not_imix(rnd, pkt):
    """One frame the IMIX path must refuse: IHL 6, a second tag, protocol 2
    (IGMP), a frame too short for the IPv4 header, a QinQ outer tag."""
    kind = rnd.randrange(5)
    v = 4 if pkt[12:14] == b"\x81\x00" else 0
    if kind == 0:
        ip = bytearray(pkt[14 + v:34 + v])
        ip[0] = 0x46
        return pkt[:14 + v] + bytes(ip) + b"\x01\x01\x01\x00" + pkt[34 + v:]
    if kind == 1:
        return pkt[:12] + b"\x81\x00\x00\x05\x81\x00\x00\x06" + pkt[12 + v:]
    if kind == 2:
        return pkt[:23 + v] + b"\x02" + pkt[24 + v:]
    if kind == 3:
        return pkt[:33 + v]
    return pkt[:12] + b"\x88\xa8\x00\x07" + pkt[12 + v:]


@pytest.mark.parametrize("align", [1, 2, 16])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_imix_tiles(mode, align):
    """Tiles of IMIX chains only at odd and even alignments, a partial last
    tile, and tiles with one other frame: records of both forms and counters
    equal the oracle's, under both schedules."""
    import random
    rnd = random.Random(31 + align)
    pkts = _imix_tiles(seed=align, n=64 * 40 + 9)
    frames, desc = T.batch_from_packets(pkts, align=align)
    _check(frames, desc, mode)
    _check_compact(frames, desc, mode)
    for t in range(0, 40, 3):
        k = 64 * t + rnd.randrange(64)
        pkts[k] = _not_imix(rnd, pkts[k])
    frames, desc = T.batch_from_packets(pkts, align=align)
    _check(frames, desc, mode)
    _check_compact(frames, desc, mode)


@pytest.mark.parametrize("compact", [False, True])
def test_graph_capture_and_replay(compact, schedule_small):
    """nsd_dissect_device_ws / _compact captured into a HIP graph (torch.cuda
    graph on the launch stream): the walk of a fixed-size batch replayed
    over new frames in the same buffers gives the oracle's records and
    counters each time (C2, C3, C4 batches through one graph), under both
    schedules (an adaptive launch under capture keeps the plan it has and is
    never the sample: no event query or host copy inside the graph)."""
    import torch
    n = 8192
    batches = [T.make_batch(cfg, n, seed=T.SEED + k) for k, cfg in
               enumerate((T.SYN_UDP64, T.SYN_IMIX, T.SYN_IPV6X, T.SYN_IMIX))]
    cap = max(len(f) for f, _ in batches)
    dev = torch.device("cuda", 0)
    frames = torch.zeros(cap, dtype=torch.uint8, device=dev)
    desc = torch.zeros(n, dtype=torch.int64, device=dev)
    rb = nsd.CREC_BYTES if compact else nsd.REC_BYTES
    rec = torch.empty(n * rb, dtype=torch.uint8, device=dev)
    ext = torch.empty(nsd.ext_pool_words(n), dtype=torch.int32, device=dev)
    used = torch.zeros(1, dtype=torch.int32, device=dev)
    cnt = torch.zeros(nsd.NCOUNTERS, dtype=torch.int64, device=dev)
    ws = torch.empty(nsd.lib().nsd_workspace_bytes(n), dtype=torch.uint8, device=dev)

    def walk():
        used.zero_()
        cnt.zero_()
        if compact:
            nsd.dissect_device_compact(frames, desc, mode=T.PRINT_NORM, crec=rec, ext=ext, ext_used=used,
                                       counters=cnt, workspace=ws)
        else:
            nsd.dissect_device(frames, desc, mode=T.PRINT_NORM, rec=rec, ext=ext, ext_used=used, counters=cnt,
                               workspace=ws)

    def load(k):
        f, d = batches[k]
        frames.zero_()
        frames[:len(f)].copy_(torch.from_numpy(f))
        desc.copy_(torch.from_numpy(d.view(np.int64)))

    load(0)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        walk()   # warm-up outside the capture (occupancy queries, first-use state)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        walk()
    for k in range(len(batches)):
        load(k)
        g.replay()
        torch.cuda.synchronize()
        f, d = batches[k]
        if compact:
            _compare_compact(rec, ext, used, cnt, f, d, T.PRINT_NORM)
        else:
            drec = rec.cpu().numpy().view(nsd.REC_DTYPE)
            dext = ext.cpu().numpy().view(np.uint32)[:int(used.item())]
            orec, oext, ocnt, _ = T.oracle_records(f, d, mode=T.PRINT_NORM)
            assert_same_records(drec, orec, dext, oext)
            assert np.array_equal(cnt.cpu().numpy().view(np.uint64), ocnt)


def _cut_sweep(align=16):
    """Every packet of the edge set, 64 C4 and 32 IMIX samples, each cut at
    every capture length up to 160 bytes (and a few past): the batch holds
    the WHOLE original packet at each offset with the descriptor's caplen
    set to the cut, so the bytes right past caplen are exactly the headers a
    walk that ignored caplen would go on to parse.  The device's
    continuation windows are not zeroed past caplen and its 4-byte layer
    reads do not mask them (nsd_kernels.hip LSrc::dword_at: every use is
    gated by the layer's pull); this is the test of that argument."""
    base = [p for p in edge_cases.cases() if 0 < len(p) <= 600]
    for cfg, n in ((T.SYN_IPV6X, 64), (T.SYN_IMIX, 32)):
        fr, de = T.make_batch(cfg, n)
        base += [bytes(fr[int(d) & 0xFFFFFFFFFF:(int(d) & 0xFFFFFFFFFF) + (int(d) >> 40)]) for d in de]
    offs, lens, off = [], [], 0
    for p in base:
        cuts = list(range(0, min(len(p), 160) + 1)) + [c for c in (200, 300, 400) if c < len(p)]
        for c in cuts:
            off = (off + align - 1) & ~(align - 1)
            offs.append((off, p))
            lens.append(c)
            off += len(p)
    frames = np.zeros(off + 64, dtype=np.uint8)
    desc = np.zeros(len(offs), dtype=np.uint64)
    for i, ((o, p), c) in enumerate(zip(offs, lens)):
        frames[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
        desc[i] = T.desc_pack(o, c)
    return frames, desc


@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_cut_sweep_live_tails(mode):
    frames, desc = _cut_sweep()
    assert len(desc) > 20000
    _check(frames, desc, mode)
    _check_compact(frames, desc, mode)
