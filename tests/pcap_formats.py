"""pcap files in every record format read_pcap accepts (pcap_io.h:27-141),
with per-record timestamps, lengths and link-layer metadata chosen to reach
every branch of pcap_pkthdr_to_tpacket_hdr (pcap_io.h:594-709) and
show_frame_hdr (dissector.h:53-108): usec values whose ns product has bit 4
or 6 set (the tpacketv3 VLAN line of the v2 view), usec values past 2^31 /
1000 (32-bit products), wire lengths above the caplen, every packet type
0..8 (named, "?" ones), interface indexes 0 / 1 (lo) / one no interface
has.  Used by tests/golden/make_golden.py (committed fixtures) and the
frame header tests."""
import struct

MAGIC = {"usec": 0xA1B2C3D4, "nsec": 0xA1B23C4D, "kuz": 0xA1B2CD34, "bkm": 0xA1E2CB12}
IFINDEX = [0, 1, 0x7FFFFFF0, 0, 2_000_000]


def record_fields(i):
    """(sec, frac, extra_len, pkttype, ifindex, protocol, hatype) of record i."""
    sec = (1_400_000_000 + 7919 * i) & 0xFFFFFFFF
    frac = (104_729 * i + 13) % 1_000_000
    if i % 11 == 5:
        frac = 4_300_000 + 977 * i          # usec * 1000 wraps in 32 bits
    return sec, frac, i % 3, i % 9, IFINDEX[i % len(IFINDEX)], (0x0800, 0x86DD, 0x0806, 0x1234)[i % 4], \
        (1, 772, 768, 0xFFFF, 0)[i % 5]


def write(path, pkts, fmt="usec", endian="<", linktype=1, ll=False, nsec_scale=True):
    """Write pkts as a pcap of record format fmt ("usec" / "nsec" / "kuz" /
    "bkm"), byte order endian; ll=True adds the 16-byte struct pcap_ll after
    each record header (the *_LL form of SLL / netlink files: caplen and len
    count it)."""
    e = endian
    with open(path, "wb") as f:
        f.write(struct.pack(e + "IHHiIII", MAGIC[fmt], 2, 4, 0, 0, 65535, linktype))
        for i, p in enumerate(pkts):
            sec, frac, extra, pkttype, ifindex, proto, hatype = record_fields(i)
            if fmt in ("nsec", "bkm") and nsec_scale:
                frac = (frac * 1000 + i) % 1_000_000_000
            cooked = b""
            if ll:
                cooked = struct.pack(">HHH8sH", pkttype, hatype, (6, 0, 8, 4)[i % 4],
                                     bytes([0xde, 0xad, 0xbe, 0xef, i & 0xFF, 2, 3, 4]), proto)
            cl = len(p) + len(cooked)
            hdr = struct.pack(e + "IIII", sec, frac, cl, cl + extra)
            if fmt == "kuz":
                # struct pcap_pkthdr_kuz: ifindex u32, protocol u16, pkttype u8, pad
                hdr += struct.pack(e + "IH", ifindex & 0xFFFFFFFF, proto) + bytes([pkttype, 0])
            elif fmt == "bkm":
                # struct pcap_pkthdr_bkm: tsource, ifindex, protocol u16; hatype, pkttype u8
                hdr += struct.pack(e + "HHH", i % 4, ifindex & 0xFFFF, proto) + bytes([hatype & 0xFF, pkttype])
            f.write(hdr + cooked + bytes(p))


# the committed frame-header fixtures: name -> write() arguments
VARIANTS = {
    "fh_usec": dict(fmt="usec"),
    "fh_usec_be": dict(fmt="usec", endian=">"),
    "fh_nsec_be": dict(fmt="nsec", endian=">"),
    "fh_kuz": dict(fmt="kuz"),
    "fh_bkm_be": dict(fmt="bkm", endian=">"),
    "fh_sll": dict(fmt="usec", linktype=113, ll=True),
    "fh_sll_be": dict(fmt="nsec", endian=">", linktype=113, ll=True),
}
