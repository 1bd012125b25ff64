"""Hand-built frames covering every quirk of SURVEY §8a (and the parser
branches the synthetic configs do not reach).  Used for the edge golden
(tests/golden/edge.pcap) and the device parity tests."""
import struct


def be16(v):
    return struct.pack(">H", v & 0xFFFF)


def be32(v):
    return struct.pack(">I", v & 0xFFFFFFFF)


DST = bytes.fromhex("3cfdfe000002")
SRC = bytes.fromhex("001b21000001")


def eth(etype, dst=DST, src=SRC):
    return dst + src + be16(etype)


def csum16(b):
    if len(b) & 1:
        b += b"\0"
    s = sum(struct.unpack(">%dH" % (len(b) // 2), b))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def ipv4(proto, payload_len, ihl=5, opts=b"", tot_len=None, good=True, ttl=64,
         src=0x0A000001, dst=0xC0A80001, frag=0x4000, tos=0):
    if tot_len is None:
        tot_len = ihl * 4 + payload_len
    h = bytes([0x40 | (ihl & 15), tos]) + be16(tot_len) + be16(0x1234) + be16(frag) + \
        bytes([ttl, proto]) + b"\0\0" + be32(src) + be32(dst) + opts
    hl = max(ihl * 4, 20)
    h = h[:hl] if len(h) >= hl else h + b"\0" * (hl - len(h))
    c = csum16(h[:ihl * 4] if ihl >= 5 else h[:20]) if good else 0xBEEF
    return h[:10] + be16(c) + h[12:]


def ipv6(nh, plen, src=None, dst=None, tc=0, flow=0, hlim=64):
    w0 = (6 << 28) | ((tc & 0xFF) << 20) | (flow & 0xFFFFF)
    src = src or bytes.fromhex("20010db8000000000000000000000001")
    dst = dst or bytes.fromhex("fe800000000000000000000000000002")
    return be32(w0) + be16(plen) + bytes([nh, hlim]) + src + dst


def udp(sport=1024, dport=53, length=None, payload=b"", check=0):
    if length is None:
        length = 8 + len(payload)
    return be16(sport) + be16(dport) + be16(length) + be16(check) + payload


def tcp(sport=80, dport=443, flags=0x18, doff=5, res=0, seq=1, ack=2, win=1024):
    return be16(sport) + be16(dport) + be32(seq) + be32(ack) + bytes([(doff << 4) | res, flags]) + \
        be16(win) + be16(0xABCD) + be16(7)


def icmp(typ=8, code=0, payload=b"", good=True):
    h = bytes([typ, code]) + b"\0\0" + be16(1) + be16(2) + payload
    c = csum16(h) if good else 0x1111
    return h[:2] + be16(c) + h[4:]


def pad(b, n=64):
    return b + bytes(range(n - len(b))) if len(b) < n else b


def cases():
    P = []
    add = P.append
    payload = bytes(range(32, 96))
    # --- plain paths
    add(pad(eth(0x0800) + ipv4(17, 30) + udp(payload=bytes(22))))
    add(eth(0x0800) + ipv4(6, 20 + 10) + tcp(flags=0xFF) + b"hello tcp!")
    add(eth(0x0800) + ipv4(6, 20) + tcp(flags=0x91))            # FIN ACK CWR -> "FIN ACKCWR"
    add(eth(0x0800) + ipv4(6, 20) + tcp(flags=0x00, doff=15, res=9))
    add(eth(0x0800) + ipv4(1, 8 + 40) + icmp(payload=payload[:40]))
    add(eth(0x0800) + ipv4(1, 8 + 41) + icmp(payload=payload[:41]))           # odd length: byte dropped
    add(eth(0x0800) + ipv4(1, 8 + 40) + icmp(payload=payload[:40], good=False))
    # --- IPv4 quirks
    add(eth(0x0800) + ipv4(17, 30, good=False) + udp(payload=bytes(22)))      # bogus + should be
    add(eth(0x0800) + ipv4(17, 12) + udp(payload=b"abcd") + b"TRAILERBYTES")  # trailer (short)
    add(eth(0x0800) + ipv4(17, 12) + udp(payload=b"abcd") + bytes(range(40)))  # trailer > 20 B
    add(eth(0x0800) + ipv4(17, 8 + 8, ihl=6, opts=b"\x01\x00\x00\x00") + udp(payload=bytes(8)))
    add(eth(0x0800) + ipv4(17, 8, ihl=8, opts=b"\x01\x83\x07\x04\x0a\x00\x00\x01\x00\x00\x00\x00") +
        udp())                                                                 # NOP, LSRR, EOOL
    add(eth(0x0800) + ipv4(17, 8, ihl=7, opts=b"\x83\x0f\x04\x0a\x00\x00\x00\x00") + udp())  # bad opt len
    add(eth(0x0800) + ipv4(17, 8, ihl=6, opts=b"\x01\x01\x01\x44") + udp())   # len byte past opts
    add(eth(0x0800) + ipv4(17, 8, ihl=15, opts=bytes(40)) + udp())           # max IHL
    add(eth(0x0800) + ipv4(17, 8, ihl=3) + udp())                           # ihl < 5
    add(eth(0x0800) + ipv4(17, 8, ihl=15) + udp())                          # options pull fails
    add(eth(0x0800) + ipv4(17, 8, tot_len=10) + udp(payload=bytes(20)))      # tot_len < ihl*4: no trim
    add(eth(0x0800) + ipv4(17, 8, tot_len=1500) + udp())                    # tot_len > frame
    add(eth(0x0800) + ipv4(17, 8, frag=0xE123) + udp())                     # all frag bits
    add(eth(0x0800) + ipv4(0, 8) + bytes([17, 0]) + bytes(6) + udp())        # IPv4 proto 0 -> HBH
    add(eth(0x0800) + ipv4(41, 40 + 8) + ipv6(17, 8) + udp())               # 6in4
    add(eth(0x0800) + ipv4(41, 40 + 40 + 8) + ipv6(41, 48) + ipv6(17, 8) + udp())  # 6in4 in 6
    add(eth(0x0800) + ipv4(99, 10) + bytes(10))                             # unknown proto
    # --- UDP length quirks
    add(eth(0x0800) + ipv4(17, 12) + udp(length=100, payload=b"abcd"))      # len > pkt_len
    add(eth(0x0800) + ipv4(17, 12) + udp(length=4, payload=b"abcd"))        # negative data len
    # --- L2
    add(eth(0x8100) + be16(0xE00A) + be16(0x0800) + ipv4(17, 8) + udp())    # VLAN prio 7 id 10
    add(eth(0x88a8) + be16(0x3064) + be16(0x8100) + be16(0x0005) + be16(0x86DD) + ipv6(59, 0))
    add(eth(0x8100) + be16(1) + be16(0x8100) + be16(2) + be16(0x8100) + be16(3) + be16(0x8100) +
        be16(4) + be16(0x8100) + be16(5) + be16(0x8100) + be16(6) + be16(0x0800) + ipv4(6, 20) + tcp())
    add(eth(0x8847) + be32((100 << 12) | (3 << 9) | 64) + be32((200 << 12) | (1 << 8) | 63) +
        ipv4(17, 8) + udp())                                                 # MPLS x2 -> IPv4
    add(eth(0x8847) + be32((5 << 12) | (1 << 8) | 1) + ipv6(58, 8) + icmp(128))  # MPLS -> IPv6
    add(eth(0x8847) + be32((5 << 12) | (1 << 8) | 1) + b"\x12\x34\x56")     # unknown nibble
    add(eth(0x8847) + be32((5 << 12) | 1) + b"\x00\x00")                    # truncated label stack
    add(eth(0x8847) + be32((5 << 12) | (1 << 8) | 1))                        # S=1, no payload
    add(eth(0x1234) + b"unknown ethertype payload")
    add(eth(0x0800, dst=b"\xff" * 6) + ipv4(17, 8) + udp())                 # broadcast
    add(eth(0x0800, dst=bytes.fromhex("01005e000001"), src=bytes.fromhex("020000000001")) +
        ipv4(17, 8) + udp())                                                 # multicast / local
    add(b"\x01\x02\x03")                                                     # runt
    add(eth(0x0800))                                                         # header only
    add(eth(0x0800) + b"\x45\x00")                                            # truncated IPv4
    add(eth(0x8100) + b"\x00")                                                # truncated VLAN
    add(b"")                                                                 # empty
    # --- IPv6
    add(eth(0x86DD) + ipv6(17, 8, tc=0xAB, flow=0x12345) + udp())           # flow label quirk (885)
    add(eth(0x86DD) + ipv6(6, 20, src=bytes(15) + b"\x01", dst=bytes(10) + b"\xff\xff\x0a\x00\x00\x01") + tcp())
    add(eth(0x86DD) + ipv6(1, 8) + icmp())                                  # nexthdr 1 -> ICMPv4 ops
    add(eth(0x86DD) + ipv6(0, 16) + bytes([17, 1]) + bytes(14) + udp())      # HBH with options
    add(eth(0x86DD) + ipv6(0, 8) + bytes([17, 0]) + bytes(6) + udp())        # HBH no options
    add(eth(0x86DD) + ipv6(0, 8) + bytes([17, 9]) + bytes(6))                # HBH invalid len
    add(eth(0x86DD) + ipv6(60, 8) + bytes([59, 0]) + bytes(6))               # DestOpts -> NoNext
    add(eth(0x86DD) + ipv6(60, 8) + bytes([59, 5]) + bytes(6))               # DestOpts invalid
    add(eth(0x86DD) + ipv6(43, 40) + bytes([17, 4, 0, 2]) + be32(0x11223344) +
        bytes.fromhex("20010db8000000000000000000000001") + bytes.fromhex("20010db8000000000000000000000002") +
        udp())                                                               # routing type 0, 2 addrs
    add(eth(0x86DD) + ipv6(43, 24) + bytes([17, 2, 0, 0]) + be32(7) + bytes(16) + udp())
    add(eth(0x86DD) + ipv6(43, 16) + bytes([17, 1, 4, 3]) + bytes(12) + udp())  # type 4 unknown
    add(eth(0x86DD) + ipv6(43, 8) + bytes([17, 7, 0, 1]) + bytes(4))         # routing invalid
    add(eth(0x86DD) + ipv6(43, 0) + bytes([17, 0]))                           # routing truncated
    add(eth(0x86DD) + ipv6(44, 16) + bytes([17, 0]) + be16((1234 << 3) | 5) + be32(0xDEADBEEF) + udp())
    add(eth(0x86DD) + ipv6(51, 24) + bytes([17, 2]) + be16(0x1) + be32(0x100) + be32(0x200) + bytes(4) + udp())
    add(eth(0x86DD) + ipv6(51, 12) + bytes([17, 0]) + be16(0) + be32(1) + be32(2) + udp())  # hdr_len 8
    add(eth(0x86DD) + ipv6(51, 12) + bytes([17, 40]) + be16(0) + be32(1) + be32(2))        # AH invalid
    add(eth(0x86DD) + ipv6(50, 8) + be32(0xAABBCCDD) + be32(0x01020304) + b"encrypted")
    add(eth(0x86DD) + ipv6(59, 0) + b"ignored tail")
    for mt, hl in [(0, 0), (1, 1), (2, 1), (3, 2), (4, 2), (5, 1), (6, 1), (8, 0)]:
        body = bytes([17, hl, mt, 0]) + be16(0x5A5A) + bytes(range(1, (hl + 1) * 8 - 5))
        add(eth(0x86DD) + ipv6(135, len(body) + 8) + body + udp())
    # mobility quirks: subtype larger than the message (modes differ)
    add(eth(0x86DD) + ipv6(135, 8) + bytes([17, 0, 1, 0, 0, 0, 9, 9]) + bytes(12) + udp())
    add(eth(0x86DD) + ipv6(135, 8) + bytes([17, 0, 3, 0, 0, 0, 9, 9]) + bytes(20) + udp())
    add(eth(0x86DD) + ipv6(135, 8) + bytes([17, 0, 6, 0, 0, 0, 9, 9]))        # type 6, pull fails
    add(eth(0x86DD) + ipv6(135, 8) + bytes([17, 0, 6, 0, 0, 0, 9, 9]) + bytes(8))
    add(eth(0x86DD) + ipv6(135, 8) + bytes([17, 3, 0, 0, 0, 0, 9, 9]))        # invalid len
    for t, c in [(1, 4), (1, 9), (2, 0), (3, 1), (4, 2), (128, 0), (129, 0), (100, 0), (127, 0),
                 (155, 0x8A), (155, 7), (200, 1), (255, 0), (77, 3)]:
        add(eth(0x86DD) + ipv6(58, 8) + bytes([t, c]) + be16(0x1234) + be32(0x00050006) + b"data")
    add(eth(0x86DD) + ipv6(58, 4) + bytes([128, 0]) + be16(0x1234) + b"\x01")  # body pull fails
    add(eth(0x86DD) + ipv6(58, 2) + bytes([128, 0]))                           # header pull fails
    # deep chain -> ext record (8 ext headers)
    chain = b""
    for k in range(8):
        chain += bytes([60 if k < 7 else 17, 0]) + bytes(6)
    add(eth(0x86DD) + ipv6(60, len(chain) + 8) + chain + udp())
    # layer start past byte 510 -> ext record
    add(eth(0x86DD) + ipv6(0, 8 + 8 * 70) + bytes([17, 69]) + bytes(8 * 70 - 2) + udp(payload=b"far"))
    # > 64 layers -> overflow
    add(eth(0x8100) + (be16(7) + be16(0x8100)) * 70 + be16(7) + be16(0x0800) + ipv4(17, 8) + udp())
    # host-rendered leaves (records only)
    add(eth(0x0806) + bytes(28))                                             # ARP
    add(eth(0x88cc) + bytes(20))                                             # LLDP
    add(eth(0x0800) + ipv4(2, 8) + bytes(8))                                 # IGMP
    add(eth(0x0800) + ipv4(33, 16) + bytes(16))                              # DCCP
    add(eth(0x86DD) + ipv6(58, 24) + bytes([135, 0]) + bytes(22))            # ICMPv6 NDP
    return P


# cases whose TEXT is outside this round's host renderer (ARP, LLDP, IGMP,
# DCCP, ICMPv6 130-154) or outside the parity domain; records still compared
HOST_ONLY_TEXT = {"arp", "lldp", "igmp", "dccp", "icmpv6-ndp"}
