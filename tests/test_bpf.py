"""Classic BPF (the capture loop's filter step, read_pcap netsniff-ng.c:707-725).

CPU (-m "not gpu"): the oracle restatement (oracle/nsd_bpf_oracle.c) and the
product validator (nsd_bpf_validate, host code) against known answers: the
programs the reference itself holds (astraceroute.c:131-152, bpfc.8:241-275,
the accept-all default of bpf.c:711) and hand-assembled ones covering every
opcode and bounds edge, with verdicts derived by hand.  bpf.c cannot be built
here (config.h), so these known answers are what pin the restatement.

GPU (-m gpu): the device filter (nsd_bpf_filter_device / _batch) against the
oracle on the same programs, on random valid programs x edge / synthetic
packets, the order-preserving compaction of accepted descriptors, and
filter -> dissect on the device.
"""
import ctypes
import random

import numpy as np
import pytest

import edge_cases as E
import nsd
import nsd_testlib as T

ACCEPT = 0xFFFFFFFF


def prog(*ins):
    a = np.zeros(len(ins), dtype=nsd.BPF_INSN)
    for i, (c, jt, jf, k) in enumerate(ins):
        a[i] = (c, jt, jf, k & 0xFFFFFFFF)
    return a


def ret(k):
    return (0x06, 0, 0, k)


# ---- programs the reference holds -------------------------------------------------
# astraceroute.c:131-141: IPv4, ICMP, not a fragment, type 11 (time exceeded)
P_AST4 = prog((0x28, 0, 0, 0x0c), (0x15, 0, 8, 0x800), (0x30, 0, 0, 0x17), (0x15, 0, 6, 1),
              (0x28, 0, 0, 0x14), (0x45, 4, 0, 0x1fff), (0xb1, 0, 0, 0x0e), (0x50, 0, 0, 0x0e),
              (0x15, 0, 1, 0x0b), ret(ACCEPT), ret(0))
# astraceroute.c:145-152: IPv6, next header ICMPv6, type 3
P_AST6 = prog((0x28, 0, 0, 0x0c), (0x15, 0, 5, 0x86dd), (0x30, 0, 0, 0x14), (0x15, 0, 3, 0x3a),
              (0x30, 0, 0, 0x36), (0x15, 0, 1, 3), ret(ACCEPT), ret(0))
# bpf.c:711: no rule file -> accept everything
P_ALL = prog(ret(ACCEPT))
# bpfc.8:245-250 "Only allow ARP packets" (ldh [12]; jne #0x806, drop; ret #-1; drop: ret #0)
P_ARP = prog((0x28, 0, 0, 12), (0x15, 0, 1, 0x806), ret(ACCEPT), ret(0))
# bpfc.8:252-259 "Only allow IPv4 TCP packets"
P_TCP = prog((0x28, 0, 0, 12), (0x15, 0, 3, 0x800), (0x30, 0, 0, 23), (0x15, 0, 1, 6), ret(ACCEPT), ret(0))
# bpfc.8:261-275 "Only allow IPv4 TCP SSH traffic"
P_SSH = prog((0x28, 0, 0, 12), (0x15, 0, 10, 0x800), (0x30, 0, 0, 23), (0x15, 0, 8, 6),
             (0x28, 0, 0, 20), (0x45, 6, 0, 0x1fff), (0xb1, 0, 0, 14), (0x48, 0, 0, 14),
             (0x15, 2, 0, 0x16), (0x48, 0, 0, 16), (0x15, 0, 1, 0x16), ret(ACCEPT), ret(0))
# bpfc.8:241-243 "ld poff; ret a": a Linux extension load (SKF_AD_OFF + 52); the
# userland interpreter has none, the load is out of bounds -> 0
P_POFF = prog((0x20, 0, 0, 0xFFFFF000 + 52), (0x16, 0, 0, 0))
REF_PROGS = [P_ALL, P_AST4, P_AST6, P_ARP, P_TCP, P_SSH, P_POFF]


def tcp_pkt(sport, dport, frag=0x4000, ihl=5):
    opts = bytes(4 * (ihl - 5))
    return E.eth(0x0800) + E.ipv4(6, 20, ihl=ihl, opts=opts, frag=frag) + E.tcp(sport=sport, dport=dport)


def icmp4(t, frag=0x4000):
    return E.eth(0x0800) + E.ipv4(1, 8, frag=frag) + E.icmp(typ=t)


def icmp6(t):
    return E.eth(0x86DD) + E.ipv6(58, 8) + bytes([t, 0]) + E.be16(0) + bytes(4)


KNOWN = [
    # (program, packet, verdict)
    (P_AST4, icmp4(11), ACCEPT),
    (P_AST4, icmp4(3), 0),
    (P_AST4, icmp4(11, frag=0x2001), 0),                 # fragment offset set
    (P_AST4, tcp_pkt(1, 2), 0),
    (P_AST4, E.eth(0x86DD) + E.ipv6(17, 8) + E.udp(), 0),
    (P_AST4, icmp4(11)[:34], 0),                          # ldb [x + 14] = [34]: past the end
    (P_AST4, icmp4(11)[:35], ACCEPT),                     # ... just inside
    (P_AST6, icmp6(3), ACCEPT),
    (P_AST6, icmp6(1), 0),
    (P_AST6, icmp4(3), 0),
    (P_AST6, icmp6(3)[:54], 0),                           # ldb [54] out of bounds
    (P_ALL, b"", ACCEPT),
    (P_ALL, b"\x01", ACCEPT),
    (P_ARP, E.eth(0x0806) + bytes(28), ACCEPT),
    (P_ARP, E.eth(0x0800) + bytes(28), 0),
    (P_ARP, b"\x00" * 13, 0),                             # ldh [12] needs 14 bytes
    (P_ARP, E.eth(0x0806), ACCEPT),                       # 14 bytes are enough
    (P_TCP, tcp_pkt(1, 2), ACCEPT),
    (P_TCP, E.eth(0x0800) + E.ipv4(17, 8) + E.udp(), 0),
    (P_SSH, tcp_pkt(22, 40000), ACCEPT),
    (P_SSH, tcp_pkt(40000, 22), ACCEPT),
    (P_SSH, tcp_pkt(40000, 22, ihl=7), ACCEPT),           # X = 4 * ihl
    (P_SSH, tcp_pkt(80, 443), 0),
    (P_SSH, tcp_pkt(22, 1, frag=0x0010), 0),              # a fragment
    (P_SSH, E.eth(0x0800) + E.ipv4(17, 8) + E.udp(sport=22), 0),
    (P_POFF, tcp_pkt(1, 2), 0),
]


def _arith_cases():
    """Every ALU / load / store / misc / jump opcode with a hand-derived result."""
    imm = lambda k: (0x00, 0, 0, k)       # noqa: E731  ld #k
    ldx = lambda k: (0x01, 0, 0, k)       # noqa: E731  ldx #k
    ra = (0x16, 0, 0, 0)                  # ret a
    c = []
    c.append((prog(imm(5), (0x04, 0, 0, 3), ra), b"", 8))                     # add k
    c.append((prog(imm(5), (0x14, 0, 0, 7), ra), b"", 0xFFFFFFFE))            # sub k wraps
    c.append((prog(imm(0x10001), (0x24, 0, 0, 0x10001), ra), b"", 0x20001))   # mul k mod 2^32
    c.append((prog(imm(100), (0x34, 0, 0, 7), ra), b"", 14))                  # div k
    c.append((prog(imm(100), (0x94, 0, 0, 7), ra), b"", 2))                   # mod k
    c.append((prog(imm(0xF0F0), (0x54, 0, 0, 0xFF00), ra), b"", 0xF000))      # and k
    c.append((prog(imm(0xF0F0), (0x44, 0, 0, 0x0F0F), ra), b"", 0xFFFF))      # or k
    c.append((prog(imm(0xFF00), (0xa4, 0, 0, 0x0FF0), ra), b"", 0xF0F0))      # xor k
    c.append((prog(imm(1), (0x64, 0, 0, 31), ra), b"", 0x80000000))           # lsh k
    c.append((prog(imm(1), (0x64, 0, 0, 33), ra), b"", 2))                    # lsh by 33 = by 1 (x86)
    c.append((prog(imm(0x80000000), (0x74, 0, 0, 31), ra), b"", 1))           # rsh k
    c.append((prog(imm(7), (0x84, 0, 0, 0), ra), b"", 0xFFFFFFF9))            # neg
    c.append((prog(imm(9), ldx(4), (0x0c, 0, 0, 0), ra), b"", 13))            # add x
    c.append((prog(imm(9), ldx(4), (0x1c, 0, 0, 0), ra), b"", 5))             # sub x
    c.append((prog(imm(9), ldx(4), (0x2c, 0, 0, 0), ra), b"", 36))            # mul x
    c.append((prog(imm(9), ldx(4), (0x3c, 0, 0, 0), ra), b"", 2))             # div x
    c.append((prog(imm(9), ldx(0), (0x3c, 0, 0, 0), ra), b"", 0))             # div by X = 0 -> 0
    c.append((prog(imm(9), ldx(4), (0x9c, 0, 0, 0), ra), b"", 1))             # mod x
    c.append((prog(imm(9), ldx(0), (0x9c, 0, 0, 0), ra), b"", 0))             # mod by X = 0 -> 0
    c.append((prog(imm(12), ldx(10), (0x5c, 0, 0, 0), ra), b"", 8))           # and x
    c.append((prog(imm(12), ldx(10), (0x4c, 0, 0, 0), ra), b"", 14))          # or x
    c.append((prog(imm(12), ldx(10), (0xac, 0, 0, 0), ra), b"", 6))           # xor x
    c.append((prog(imm(3), ldx(4), (0x6c, 0, 0, 0), ra), b"", 48))            # lsh x
    c.append((prog(imm(48), ldx(36), (0x7c, 0, 0, 0), ra), b"", 3))           # rsh x by 36 = by 4
    c.append((prog(imm(3), (0x07, 0, 0, 0), imm(0), (0x87, 0, 0, 0), ra), b"", 3))   # tax, txa
    c.append((prog((0x80, 0, 0, 0), ra), b"abcdef", 6))                        # ld len
    c.append((prog((0x81, 0, 0, 0), (0x87, 0, 0, 0), ra), b"abc", 3))          # ldx len
    c.append((prog(imm(77), (0x02, 0, 0, 15), imm(0), (0x60, 0, 0, 15), ra), b"", 77))   # st, ld M[]
    c.append((prog(ldx(66), (0x03, 0, 0, 3), (0x61, 0, 0, 3), (0x87, 0, 0, 0), ra), b"", 66))
    c.append((prog((0x60, 0, 0, 5), ra), b"", 0))                              # M[] starts zeroed
    pkt = bytes(range(0x10, 0x30))
    c.append((prog((0x20, 0, 0, 2), ra), pkt, 0x12131415))                     # ld w abs, big-endian
    c.append((prog((0x28, 0, 0, 3), ra), pkt, 0x1314))                         # ld h abs
    c.append((prog((0x30, 0, 0, 31), ra), pkt, 0x2f))                          # ld b abs, last byte
    c.append((prog((0x20, 0, 0, 28), ra), pkt, 0x2c2d2e2f))                    # ld w at plen - 4
    c.append((prog((0x20, 0, 0, 29), ra), pkt, 0))                             # ... at plen - 3: out
    c.append((prog((0x28, 0, 0, 31), ra), pkt, 0))                             # ld h at plen - 1: out
    c.append((prog((0x30, 0, 0, 32), ra), pkt, 0))                             # ld b at plen: out
    c.append((prog(ldx(5), (0x40, 0, 0, 1), ra), pkt, 0x16171819))            # ld w ind
    c.append((prog(ldx(5), (0x48, 0, 0, 1), ra), pkt, 0x1617))                # ld h ind
    c.append((prog(ldx(5), (0x50, 0, 0, 1), ra), pkt, 0x16))                  # ld b ind
    c.append((prog(ldx(0xFFFFFFFF), (0x50, 0, 0, 2), ra), pkt, 0x11))         # X + k wraps to 1
    c.append((prog(ldx(0xFFFFFFFF), (0x40, 0, 0, 0), ra), pkt, 0))            # X + k = 2^32 - 1: out
    c.append((prog((0xb1, 0, 0, 0), (0x87, 0, 0, 0), ra), b"\x4f", 60))       # ldxb 4*([0]&0xf)
    c.append((prog((0xb1, 0, 0, 1), ra), b"\x4f", 0))                         # msh out of bounds
    c.append((prog((0x20, 0, 0, 0xFFFFFFFF), ra), pkt, 0))                    # k + 4 does not wrap
    c.append((prog((0x05, 0, 0, 1), ret(1), ret(2)), b"", 2))                 # ja
    for code, a, b, taken in [(0x25, 5, 4, True), (0x25, 4, 4, False), (0x35, 4, 4, True),
                              (0x35, 3, 4, False), (0x15, 4, 4, True), (0x15, 5, 4, False),
                              (0x45, 6, 4, True), (0x45, 3, 4, False)]:
        c.append((prog(imm(a), (code, 1, 0, b), ret(10), ret(20)), b"", 20 if taken else 10))
        c.append((prog(imm(a), ldx(b), (code | 0x08, 1, 0, 0), ret(10), ret(20)), b"", 20 if taken else 10))
    # codes the validator accepts but the interpreter's switch does not -> 0
    c.append((prog((0x21, 0, 0, 0), ret(1)), pkt, 0))                         # ldx w abs
    c.append((prog((0x08, 0, 0, 0), ret(1)), pkt, 0))                         # ld h imm
    c.append((prog((0x0d, 0, 0, 0), ret(1), ret(2)), b"", 0))                  # ja x
    c.append((prog((0x0e, 0, 0, 0)), b"", 0))                                  # ret x
    c.append((prog((0x8c, 0, 0, 0), ret(1)), b"", 0))                          # neg x
    c.append((prog((0x27, 0, 0, 0), ret(1)), b"", 0))                          # misc 0x20
    c.append((prog((0x106, 0, 0, 5)), b"", 0))                                 # high code bits
    return c


ARITH = _arith_cases()

VALIDATE = [
    # (program, valid) following __bpf_validate (bpf.c:388-506)
    (prog(), 0),
    (P_ALL, 1), (P_AST4, 1), (P_AST6, 1), (P_SSH, 1), (P_POFF, 1),
    (prog((0x00, 0, 0, 0)), 0),                         # last insn is not RET
    (prog((0x60, 0, 0, 16), ret(0)), 0),                # LD MEM k >= 16
    (prog((0x61, 0, 0, 15), ret(0)), 1),
    (prog((0x02, 0, 0, 16), ret(0)), 0),                # ST k >= 16
    (prog((0x03, 0, 0, 99), ret(0)), 0),                # STX
    (prog((0xc0, 0, 0, 0), ret(0)), 0),                 # LD mode 0xc0
    # DIV / MOD by constant 0 pass: the check reads BPF_RVAL (code & 0x18),
    # which is 0x10 for every DIV / MOD code (bpf.c:447), so it never fires
    (prog((0x34, 0, 0, 0), ret(0)), 1),
    (prog((0x94, 0, 0, 0), ret(0)), 1),
    (prog((0x3c, 0, 0, 0), ret(0)), 1),                 # DIV X: checked at run time
    (prog((0xb4, 0, 0, 0), ret(0)), 0),                 # ALU op 0xb0
    (prog((0x05, 0, 0, 1), ret(0)), 0),                 # JA past the end
    (prog((0x05, 0, 0, 0), ret(0)), 1),
    (prog((0x05, 0, 0, 0xFFFFFFFF), ret(0)), 1),        # JA k overflows 32 bits: accepted (bpf.c:483)
    (prog((0x15, 1, 0, 0), ret(0)), 0),                 # jt past the end
    (prog((0x15, 0, 1, 0), ret(0)), 0),                 # jf past the end
    (prog((0x55, 0, 0, 0), ret(0)), 0),                 # JMP op 0x50
    (prog((0x0e, 0, 0, 0)), 1),                         # RET X: any RET class passes
    (prog((0xf7, 0, 0, 0), ret(0)), 1),                 # any MISC passes
]


def oracle():
    L = T.oracle()
    if not getattr(L, "_bpf_set", False):
        L.nsor_bpf_validate.restype = ctypes.c_int
        L.nsor_bpf_validate.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.nsor_bpf_run.restype = ctypes.c_uint32
        L.nsor_bpf_run.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
        L.nsor_bpf_batch.restype = None
        L.nsor_bpf_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint32, ctypes.c_void_p]
        L._bpf_set = True
    return L


def oracle_run(p, pkt):
    buf = np.frombuffer(bytes(pkt) + bytes(8), dtype=np.uint8)
    return oracle().nsor_bpf_run(p.ctypes.data if len(p) else None, len(p), buf.ctypes.data, len(pkt))


def oracle_batch(p, frames, desc):
    v = np.zeros(len(desc), np.uint32)
    oracle().nsor_bpf_batch(p.ctypes.data, len(p), frames.ctypes.data, desc.ctypes.data, len(desc),
                            v.ctypes.data)
    return v


@pytest.mark.parametrize("i", range(len(KNOWN)))
def test_oracle_reference_programs(i):
    p, pkt, want = KNOWN[i]
    assert oracle().nsor_bpf_validate(p.ctypes.data, len(p)) == 1
    assert oracle_run(p, pkt) == want


@pytest.mark.parametrize("i", range(len(ARITH)))
def test_oracle_every_opcode(i):
    p, pkt, want = ARITH[i]
    assert oracle().nsor_bpf_validate(p.ctypes.data, len(p)) == 1
    assert oracle_run(p, pkt) == want


def test_oracle_no_program_accepts():
    # bpf_run_filter with no filter returns 0xFFFFFFFF (bpf.c:517-518)
    assert oracle_run(prog(), b"x") == ACCEPT


@pytest.mark.parametrize("i", range(len(VALIDATE)))
def test_validator(i):
    p, want = VALIDATE[i]
    ptr = p.ctypes.data if len(p) else None
    assert oracle().nsor_bpf_validate(ptr, len(p)) == want
    assert nsd.bpf_validate(p) == want     # the product's validator (host code, no GPU needed)


def test_loader_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(nsd.NsdError):
        nsd.BpfProgram(P_AST4)


# ---- random programs (GPU parity) -----------------------------------------------------
OPS_K = [0x04, 0x14, 0x24, 0x34, 0x94, 0x54, 0x44, 0xa4, 0x64, 0x74]
OPS_X = [o | 0x08 for o in OPS_K]
JMPS = [0x25, 0x35, 0x15, 0x45, 0x2d, 0x3d, 0x1d, 0x4d]


def random_program(rnd, n=24):
    """A valid program of n instructions: forward jumps only, every opcode
    class, packet offsets mostly inside the first 64 bytes and some past the
    end, a few codes the interpreter rejects."""
    ins = []
    for i in range(n - 1):
        left = n - 1 - i          # instructions after this one
        r = rnd.random()
        if r < 0.25:
            code = rnd.choice([0x20, 0x28, 0x30, 0x40, 0x48, 0x50])
            k = rnd.choice([rnd.randrange(64), rnd.randrange(64), rnd.randrange(2000),
                            0xFFFFFFF0 + rnd.randrange(16)])
            ins.append((code, 0, 0, k))
        elif r < 0.3:
            ins.append((0xb1, 0, 0, rnd.choice([14, rnd.randrange(80)])))
        elif r < 0.45:
            code = rnd.choice(OPS_K + OPS_X + [0x84])
            ins.append((code, 0, 0, rnd.choice([rnd.randrange(1, 40), rnd.getrandbits(32) | 1])))
        elif r < 0.6:
            code = rnd.choice(JMPS)
            jt, jf = rnd.randrange(min(left, 6)), rnd.randrange(min(left, 6))
            ins.append((code, jt, jf, rnd.choice([rnd.randrange(256), 0x800, 0x86dd, rnd.getrandbits(32)])))
        elif r < 0.65:
            ins.append((0x05, 0, 0, rnd.randrange(min(left, 4))))
        elif r < 0.75:
            ins.append((rnd.choice([0x00, 0x01, 0x80, 0x81, 0x07, 0x87]), 0, 0, rnd.getrandbits(12)))
        elif r < 0.85:
            ins.append((rnd.choice([0x02, 0x03, 0x60, 0x61]), 0, 0, rnd.randrange(16)))
        elif r < 0.92:
            ins.append((rnd.choice([0x06, 0x16]), 0, 0, rnd.getrandbits(32)))
        else:
            ins.append((rnd.choice([0x21, 0x08, 0x0e, 0x27, 0x8c]), 0, 0, 0))
    ins.append((0x16, 0, 0, 0))
    return prog(*ins)


def test_random_programs_are_valid():
    rnd = random.Random(5)
    for _ in range(200):
        p = random_program(rnd, rnd.randrange(2, 40))
        assert oracle().nsor_bpf_validate(p.ctypes.data, len(p)) == 1
        assert nsd.bpf_validate(p) == 1


def _packets():
    return [x[1] for x in KNOWN] + [x[1] for x in ARITH] + list(E.cases())


@pytest.mark.gpu
@pytest.mark.parametrize("align", [1, 16])
def test_device_known_answers(align):
    frames, desc = T.batch_from_packets(_packets(), align=align)
    for p in REF_PROGS + [a[0] for a in ARITH]:
        got = nsd.BpfProgram(p).filter_batch(frames, desc)
        assert np.array_equal(got, oracle_batch(p, frames, desc))
    for p, pkt, want in KNOWN + ARITH:
        f, d = T.batch_from_packets([pkt])
        assert nsd.BpfProgram(p).filter_batch(f, d)[0] == want


@pytest.mark.gpu
def test_device_refuses_overflowing_jump():
    with pytest.raises(nsd.NsdError):
        nsd.BpfProgram(prog((0x05, 0, 0, 0xFFFFFFFF), ret(0)))   # valid per __bpf_validate
    with pytest.raises(nsd.NsdError):
        nsd.BpfProgram(prog((0x34, 0, 0, 0), ret(0)))            # valid, divides by 0 (SIGFPE in the ref)
    with pytest.raises(nsd.NsdError):
        nsd.BpfProgram(prog((0x15, 1, 0, 0), ret(0)))            # invalid


@pytest.mark.gpu
def test_device_random_programs():
    rnd = random.Random(11)
    frames, desc = T.batch_from_packets(_packets() * 3, align=2)
    sf, sd = T.make_batch(T.SYN_IMIX, 20000)
    for t in range(60):
        p = random_program(rnd, rnd.randrange(2, 48))
        bp = nsd.BpfProgram(p)
        assert np.array_equal(bp.filter_batch(frames, desc), oracle_batch(p, frames, desc)), t
        if t % 6 == 0:
            assert np.array_equal(bp.filter_batch(sf, sd), oracle_batch(p, sf, sd)), t


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,n", [(T.SYN_IMIX, 100000), (T.SYN_UDP64, 3000), (T.SYN_IPV6X, 1),
                                   (T.SYN_IMIX, 1024), (T.SYN_IMIX, 1025), (T.SYN_IMIX, 3 << 20),
                                   (T.SYN_IMIX, (4 << 20) + 4097)])
def test_device_compaction(cfg, n):
    """Device-resident filter with compaction: verdicts identical to the
    oracle's, the accepted descriptors packed in batch order (the last size:
    16,401 per-block counts, so the count scan takes a second, ragged pass)."""
    import torch
    frames, desc = T.make_batch(cfg, n)
    p = P_TCP if cfg != T.SYN_IPV6X else P_ALL
    bp = nsd.BpfProgram(p)
    f = torch.from_numpy(frames).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    verdict, out, count = bp.filter_device(f, d, compact=True)
    torch.cuda.synchronize()
    want = oracle_batch(p, frames, desc)
    assert np.array_equal(verdict.cpu().numpy().view(np.uint32), want)
    k = int(count.item())
    assert k == int((want != 0).sum())
    assert np.array_equal(out.cpu().numpy().view(np.uint64)[:k], desc[want != 0])


@pytest.mark.gpu
def test_device_filter_then_dissect():
    """Capture-loop order (read_pcap: filter, then dissect the survivors): the
    compacted descriptors feed the dissect kernels; records and counters
    equal the oracle's for the accepted packets."""
    import torch
    frames, desc = T.make_batch(T.SYN_IMIX, 50000)
    bp = nsd.BpfProgram(P_TCP)
    f = torch.from_numpy(frames).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    _, out, count = bp.filter_device(f, d, compact=True)
    torch.cuda.synchronize()
    k = int(count.item())
    rec, _, _, counters = nsd.dissect_device(f, out[:k])
    torch.cuda.synchronize()
    kept = desc[oracle_batch(P_TCP, frames, desc) != 0]
    assert len(kept) == k > 0
    orec, _, ocnt, _ = T.oracle_records(frames, kept)
    drec = rec.cpu().numpy().view(nsd.REC_DTYPE)
    for fld in ("chain", "data_off", "tail_off", "ip_csum", "nflags"):
        assert np.array_equal(drec[fld], orec[fld]), fld
    assert np.array_equal(counters.cpu().numpy().view(np.uint64), ocnt)


@pytest.mark.gpu
@pytest.mark.parametrize("usesmem", [False, True])
def test_device_largest_program(usesmem):
    """A program of BPF_MAXINSNS (4096) instructions, with and without the
    scratch words (the largest LDS the filter block takes): packet loads at
    every offset around the staged 64-byte window's end (and past it), so
    the staged and the HBM loads meet in one program; verdicts equal the
    oracle's at alignments 1 and 16."""
    rnd = random.Random(13)
    ins = []
    while len(ins) < 4095:
        k = rnd.choice([rnd.randrange(56, 72), rnd.randrange(0, 64), rnd.randrange(64, 300)])
        ins.append((rnd.choice([0x20, 0x28, 0x30]), 0, 0, k))        # ld [k]
        if usesmem:
            j = rnd.randrange(16)
            ins.append((0x02, 0, 0, j))                              # st M[j]
            ins.append((0x61, 0, 0, j))                              # ldx M[j]
        else:
            ins.append((0x07, 0, 0, 0))                              # tax
        ins.append((0x0c, 0, 0, 0))                                  # add x
    ins = ins[:4095]
    ins.append((0x16, 0, 0, 0))                                      # ret a
    p = prog(*ins)
    assert len(p) == 4096 and nsd.bpf_validate(p) == 1
    pkts = [bytes(rnd.randrange(256) for _ in range(rnd.choice([60, 64, 65, 70, 300, 1500]))) for _ in range(700)]
    for align in (1, 16):
        frames, desc = T.batch_from_packets(pkts, align=align)
        assert np.array_equal(nsd.BpfProgram(p).filter_batch(frames, desc), oracle_batch(p, frames, desc))
