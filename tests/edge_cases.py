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
    icmpv6_bodies(add)
    return P


def icmpv6_bodies(add):
    """ICMPv6 types 130-154 (proto_icmpv6.c:1023-1474) and the Neighbor
    Discovery options (:372-911): host-rendered bodies, every branch."""
    A1 = bytes.fromhex("fe800000000000000211223344556677")
    A2 = bytes.fromhex("ff020000000000000000000000000001")
    A3 = bytes.fromhex("20010db8000000000000000000000042")

    def i6(t, c, body):
        add(eth(0x86DD) + ipv6(58, 4 + len(body)) + bytes([t, c]) + be16(0xBEEF) + body)

    def opt(t, l8, payload):
        return bytes([t, l8]) + payload

    # MLD (130-132): v1, v2 (exponential delay, source list; nr_src is a
    # uint8_t in print_ipv6_addr_list), short body
    i6(130, 0, be16(1000) + be16(0) + A2)
    i6(130, 0, be16(0x9123) + be16(7) + A2 + bytes([0x2A, 125]) + be16(2) + A1 + A3)
    i6(130, 0, be16(10) + be16(0) + A2 + bytes([0x08, 1]) + be16(3) + A1)          # sources missing
    i6(130, 0, be16(10) + be16(0) + A2 + bytes([0x00, 1]) + be16(0x0102) + A1 + A3 + b"xyz")
    i6(130, 0, be16(10) + bytes(10))                                               # body pull fails
    i6(131, 0, be16(0) + be16(0x55) + A2)
    i6(132, 1, be16(3) + be16(0) + A2 + b"tail")
    # Router / Neighbor Discovery with options
    i6(133, 0, be32(0) + opt(1, 1, bytes.fromhex("001b21000001")) + opt(200, 1, bytes(6)))
    i6(134, 0, bytes([64, 0xC0]) + be16(1800) + be32(30000) + be32(1000) +
       opt(3, 4, bytes([64, 0xC0]) + be32(86400) + be32(14400) + be32(0) + A3) +
       opt(5, 1, be16(0) + be32(1500)) + opt(25, 2, bytes(14)) + opt(31, 1, bytes(6)))
    i6(135, 0, be32(0) + A1 + opt(1, 1, bytes.fromhex("3cfdfe000002")) + opt(2, 0, b""))   # len 0: invalid
    i6(136, 0, be32(0xE0000005) + A1 + opt(2, 1, bytes.fromhex("3cfdfe000002")))
    i6(137, 0, be32(0x01020304) + A1 + A3 + opt(4, 2, be16(0) + be32(0) + bytes(range(8))))
    i6(134, 0, bytes([64, 0x40]) + be16(0) + be32(0) + be32(0) + opt(3, 2, bytes(14)) + bytes(20))  # opt 3 short
    i6(133, 0, be32(0) + opt(1, 1, bytes(6)) + b"\x01")                          # option header pull fails
    i6(133, 0, be32(0) + opt(9, 4, bytes(6)))                                    # option past the end
    # Router Renumbering, Node Information
    i6(138, 1, be32(77) + bytes([3, 0xA9]) + be16(500) + be32(0) + b"body")
    i6(138, 7, be32(78) + bytes([0, 0x17]) + be16(0) + be32(9))
    i6(139, 0, be16(2) + be16(0x1234) + bytes(range(1, 9)) + b"data")
    i6(140, 2, be16(9) + be16(0) + bytes(8))
    i6(139, 5, be16(4) + be16(1) + bytes(8))
    # Inverse ND with address lists
    i6(141, 0, be32(0) + opt(9, 5, be16(1) + be32(2) + A1 + A3))
    i6(142, 0, be32(0) + opt(10, 3, be16(0) + be32(0) + A2) + opt(1, 1, bytes(6)))
    # MLDv2 report: records, unknown record type, aux data, invalid aux length
    i6(143, 0, be16(0) + be16(2) +
       bytes([1, 1]) + be16(1) + A2 + A1 + b"\xaa\x0b\xcc\x0d" +
       bytes([9, 0]) + be16(0) + A2)
    i6(143, 0, be16(5) + be16(1) + bytes([0, 0]) + be16(0) + A2)
    i6(143, 0, be16(0) + be16(1) + bytes([4, 9]) + be16(0) + A2 + bytes(8))
    i6(143, 0, be16(0) + be16(2) + bytes([6, 0]) + be16(0) + A2)                 # second record missing
    # Mobile IPv6 (144-147)
    i6(144, 0, be16(42) + be16(0))
    i6(145, 0, be16(42) + be16(1) + A1 + A3 + b"12345")
    i6(146, 0, be16(43) + be16(2))
    # option 15 (name type, size_t pad length): valid, pad past the option
    i6(147, 0, be16(44) + be16(0xC005) +
       opt(15, 2, bytes([2]) + (2).to_bytes(8, "little") + b"a\x07b" + b"\x01\x02"))
    i6(147, 0, be16(44) + be16(0x4000) + opt(15, 2, bytes([7]) + (99).to_bytes(8, "little") + bytes(5)))
    # SEND (148-149): options 16, 17 (20-byte form and the wrong-length branch)
    i6(148, 0, be16(1) + be16(2) + opt(16, 1, bytes([1, 0x33]) + b"\xde\xad\xbe\xef"))
    i6(149, 0, be16(1) + be16(3) + be16(2) + be16(0) +
       opt(17, 3, bytes([2, 64]) + b"\x01\x00\x00\x00" + A3) + opt(17, 2, bytes([9, 48]) + bytes(range(12))))
    # 150-154 and option 19
    i6(150, 0, bytes([0x11, 0x22, 0x33, 0x44]) + b"opts")
    i6(151, 0, be16(20) + be16(2))
    i6(152, 0, b"")
    i6(153, 0, b"\x09")
    i6(154, 0, bytes([1, 2]) + be16(300) + opt(19, 1, bytes([4]) + bytes.fromhex("0011223344")) +
       opt(19, 1, bytes([9]) + bytes(5)))
    i6(154, 3, bytes([1, 2]))                                                    # body pull fails


# cases whose text is rendered by host leaves (ARP, LLDP, IGMP,
# DCCP, ICMPv6 130-154) or outside the parity domain; records still compared
HOST_ONLY_TEXT = {"arp", "lldp", "igmp", "dccp", "icmpv6-ndp"}
