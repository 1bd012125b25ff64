"""The frame header line `netsniff-ng --in` prints before every packet
(show_frame_hdr / __show_frame_hdr, dissector.h:31-116; read_pcap
netsniff-ng.c:727-737; walk_t3_block :1021).

Pinning: oracle/_ref/nsref -F / -f runs read_pcap's record loop over the
REFERENCE's own pcap objects (pcap_rw.c, pcap_validate_header and
pcap_pkthdr_to_tpacket_hdr from pcap_io.h, compiled as they lie) and prints
the line through a restatement of dissector.h (which needs config.h).  The
committed tests/golden/*.fh.* texts come from it (make_golden.py).

CPU: the oracle's record loop / line (nsor_pcap_meta, nsor_frame_hdr) and
the product's (nsd_pcap_read_batch_fh, nsd_format_frame_hdr) against nsref
on every record format, print mode, packet type, interface index and the
nlmon pkttype rule; the TPACKET_V3 form against the oracle.  GPU: the whole
replay (reader -> device walk -> formatter with frame headers) against the
goldens."""
import os
import struct

import numpy as np
import pytest

import nsd
import nsd_testlib as T
import pcap_formats as PF
import test_golden as TG

G = T.GOLDEN
HAVE_REF = os.path.exists(T.REF_BIN)
MODES = [T.PRINT_NORM, T.PRINT_LESS, T.PRINT_HEX, T.PRINT_ASCII, T.PRINT_HEX_ASCII, T.PRINT_NONE]


def edge_frames():
    _, pkts = T.read_pcap(os.path.join(G, "edge.pcap"))
    return [p for p in pkts if p]


def variant(tmp_path, name, frames=None, **kw):
    path = str(tmp_path / (name + ".pcap"))
    PF.write(path, frames if frames is not None else edge_frames(), **(kw or PF.VARIANTS[name]))
    return path


def product_lines(path, mode):
    lt, pkts, fh, sll = nsd.pcap_frame_hdrs(path, max_n=64)
    return [nsd.format_frame_hdr(fh[i], pkts[i], sll[i], linktype=lt, mode=mode, count=i + 1)
            for i in range(len(pkts))]


def oracle_lines(path, mode):
    lt = nsd.pcap_frame_hdrs(path)[0]
    fh, sll, cl = T.oracle_pcap_meta(path)
    _, pkts, _, _ = nsd.pcap_frame_hdrs(path)
    return [T.oracle_frame_hdr(fh[i], sll[i], pkts[i], linktype=lt, mode=mode, count=i + 1)
            for i in range(len(fh))]


@pytest.mark.parametrize("name", sorted(PF.VARIANTS))
def test_reader_fields_match_oracle(tmp_path, name):
    """nsd_pcap_read_batch_fh's frame header fields and sockaddr_ll (small
    batches, so records cross batch ends) == the restated read_pcap loop."""
    path = variant(tmp_path, name)
    lt, pkts, fh, sll = nsd.pcap_frame_hdrs(path, max_n=16)
    ofh, osll, ocl = T.oracle_pcap_meta(path)
    assert len(pkts) == len(ofh) == len(edge_frames())
    assert [len(p) for p in pkts] == [int(c) for c in ocl]
    assert fh.tobytes() == ofh.tobytes()
    assert sll.tobytes() == osll.astype(nsd.SLL_DTYPE).tobytes()


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (no /root/reference)")
@pytest.mark.parametrize("name", sorted(PF.VARIANTS) + ["netlink"])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS, T.PRINT_HEX_ASCII, T.PRINT_NONE])
def test_lines_match_reference(tmp_path, name, mode):
    """The line for every record: reference pcap code + restated dissector.h
    (nsref -F) == the oracle == the product."""
    if name == "netlink":
        # nlmon capture: *_LL records of link type 253; PACKET_OUTGOING
        # packets show kernel / user by nlmsg_pid (dissector.h:71-75)
        frames = [struct.pack("<IHHII", 16 + i, 0, 0, i, pid) + bytes(i % 5)
                  for i, pid in enumerate([0, 7, 0, 123, 0, 0, 99, 0, 0, 5] * 3)]
        frames += [bytes(15), bytes(8)]    # < 16 bytes: no nlmsghdr
        path = variant(tmp_path, name, frames, fmt="usec", linktype=253, ll=True)
    else:
        path = variant(tmp_path, name)
    want = T.run_ref(path, mode=mode, cols=65535, frames="F")
    assert oracle_lines(path, mode) == want
    assert product_lines(path, mode) == want
    if mode == T.PRINT_NORM and name != "netlink":
        assert any(b"tpacketv3 VLAN" in w for w in want) and not all(b"tpacketv3 VLAN" in w for w in want)


def test_line_fields():
    """Known answers: every packet type name, the ts source text of a v2
    header's status, the v3 VLAN line (tci / tpid; no ts source text)."""
    fh = np.zeros(1, dtype=nsd.FH_DTYPE)[0]
    fh["len"], fh["sec"], fh["nsec"] = 1514, 1700000000, 12  # 12: bits 2, 3
    sll = np.zeros(1, dtype=nsd.SLL_DTYPE)[0]
    names = ["<", "B", "M", "P", ">", "?", "K->U", "U->K", "?", "?"]
    for t, nm in enumerate(names):
        sll["pkttype"] = t
        got = nsd.format_frame_hdr(fh, sll=sll, count=t + 1)
        assert got == f"{nm} ? 1514 1700000000s.12ns #{t + 1} \n".encode()
        assert got == T.oracle_frame_hdr(fh, sll, count=t + 1)
    sll["pkttype"] = 0
    for st, src in ((1 << 29, "(sw ts)"), (1 << 30, "(sys hw ts)"), (1 << 31, "(raw hw ts)"),
                    ((1 << 29) | (1 << 31), "(raw hw ts)")):
        fh["status"] = st
        assert nsd.format_frame_hdr(fh, sll=sll) == f"< ? 1514 1700000000s.12ns #1 {src}\n".encode()
    fh["status"] = 0
    # v2: the VLAN line follows tp_nsec bits 4 / 6 (the tpacket3_hdr view)
    for ns, vl in ((16, True), (64, True), (80, True), (32, False), (1000, True), (0, False)):
        fh["nsec"] = ns
        got = nsd.format_frame_hdr(fh, sll=sll)
        assert (b" [ tpacketv3 VLAN Prio (0), CFI (0), ID (0), Proto (0x0000) ]\n" in got) == vl
        assert got == T.oracle_frame_hdr(fh, sll)
    # v3: status bits, the tci's fields, the tpid; never a ts source
    fh["v3"], fh["nsec"], fh["vlan_tci"], fh["vlan_tpid"] = 1, 5, 0xB123, 0x88A8
    for st in (0x10, 0x40, 0x50, 1 << 29, 0):
        fh["status"] = st
        got = nsd.format_frame_hdr(fh, sll=sll)
        line = b"< ? 1514 1700000000s.5ns #1 \n"
        if st & 0x50:
            line += b" [ tpacketv3 VLAN Prio (5), CFI (1), ID (291), Proto (0x88a8) ]\n"
        assert got == line
        assert got == T.oracle_frame_hdr(fh, sll)
    assert nsd.format_frame_hdr(fh, sll=sll, mode=T.PRINT_LESS, count=7) == b"< ? 1514 #7"
    assert nsd.format_frame_hdr(fh, sll=sll, mode=T.PRINT_NONE) == b""
    sll["ifindex"] = 1
    assert nsd.format_frame_hdr(fh, sll=sll, mode=T.PRINT_LESS) == T.oracle_frame_hdr(fh, sll, mode=T.PRINT_LESS)


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (no /root/reference)")
def test_committed_goldens_are_current(tmp_path):
    """The committed fh_* pcaps are what pcap_formats writes today, and
    their .fh. texts what nsref -f prints for them."""
    for name in PF.VARIANTS:
        path = variant(tmp_path, name)
        assert open(path, "rb").read() == open(os.path.join(G, name + ".pcap"), "rb").read()
    gold = TG.load_golden("fh_kuz.fh.m0.w65535")
    assert T.run_ref(os.path.join(G, "fh_kuz.pcap"), mode=T.PRINT_NORM, cols=65535, frames="f") == gold


def test_t3_block_frame_headers():
    """TPACKET_V3 block walk: each kept frame's tpacket3_hdr fields
    (nsd_t3_block_desc_fh) and its line == the restated v3 form."""
    import test_ring as TR
    pkts = edge_frames()[:40]
    hv1 = [((0x10, 0x40, 0x50, 0x1, 1 << 29 | 0x10)[i % 5], 0x10000 * i + 0x2000 * (i % 8) + i, 0x8100 + i)
           for i in range(len(pkts))]
    block, _ = TR.make_block(pkts, pkttypes=[i % 9 for i in range(len(pkts))],
                             ifindex=[(0, 1, 77777)[i % 3] for i in range(len(pkts))], hv1=hv1)
    desc, sll, fh = nsd.t3_block_desc(block, sll=True, fh=True)
    assert len(desc) == len(pkts)
    for i, (status, tci, tpid) in enumerate(hv1):
        f = fh[i]
        assert (int(f["sec"]), int(f["nsec"]), int(f["status"]), int(f["vlan_tci"]), int(f["vlan_tpid"]),
                int(f["v3"]), int(f["len"])) == (1000 + i, 7 * i, status, tci, tpid, 1, len(pkts[i]) + 4)
        for mode in (T.PRINT_NORM, T.PRINT_LESS):
            got = nsd.format_frame_hdr(f, pkts[i], sll[i], mode=mode, count=i + 1)
            assert got == T.oracle_frame_hdr(f, sll[i], pkts[i], mode=mode, count=i + 1)


# ---- the whole replay on the device ------------------------------------------
def fh_golden_cases():
    out = [("tiny", m, 65535) for m in range(5)] + [("big", m, 65535) for m in range(5)]
    out += [("leaves", m, 65535) for m in (0, 1)] + [("tiny", m, 80) for m in (0, 1)]
    for name in sorted(PF.VARIANTS):
        out += [(name, m, 65535) for m in ((0, 1, 2, 3, 4) if name == "fh_usec" else (0, 1))]
        if name in ("fh_usec", "fh_kuz"):
            out += [(name, m, 80) for m in (0, 1)]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode,cols", fh_golden_cases())
def test_replay_matches_reference_replay(name, mode, cols):
    """`netsniff-ng --in` on the device == the reference's read_pcap loop
    (frame headers, every record format, 80-column wrap included)."""
    gold = TG.load_golden(f"{name}.fh.m{mode}.w{cols}")
    cnt = np.zeros(nsd.NCOUNTERS, dtype=np.uint64)
    n, text = nsd.replay_pcap(os.path.join(G, name + ".pcap"), mode=mode, counters=cnt, cols=cols,
                              threads=1 if name == "leaves" else 4)
    assert n == len(gold)
    assert text == b"".join(gold)
    assert int(cnt[nsd.CNT_PKTS]) == n
