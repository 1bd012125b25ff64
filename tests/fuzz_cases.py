"""Seeded mutation fuzz frames for parity tests: the hand-built edge frames
and samples of the C3 / C4 synthetic configs, with header bytes, next-protocol
keys, length fields and capture lengths perturbed so chains take the branches
the synthetic configs never reach (bad lengths, truncations at every layer,
unexpected key chains, deep stacks).  Data only; the tests compare the device
with the oracle and the formatter with the reference's objects on them."""
import random

import numpy as np

import edge_cases
import nsd_testlib as T

ETHERTYPES = [0x0800, 0x86DD, 0x8100, 0x88A8, 0x8847, 0x0806, 0x88CC]
IPPROTOS = [0, 1, 2, 6, 17, 33, 41, 43, 44, 50, 51, 58, 59, 60, 135]


def _samples(cfg, n):
    frames, desc = T.make_batch(cfg, n)
    out = []
    for d in desc:
        d = int(d)
        off, cl = d & 0xFFFFFFFFFF, d >> 40
        out.append(bytes(frames[off:off + cl]))
    return out


def mutants(n, seed=0xF022):
    rnd = random.Random(seed)
    base = [p for p in edge_cases.cases() if len(p) < 4096]
    base += _samples(T.SYN_IMIX, 512) + _samples(T.SYN_IPV6X, 512)
    out = []
    for _ in range(n):
        p = bytearray(rnd.choice(base))
        for _ in range(rnd.randint(1, 4)):
            op = rnd.random()
            if not p:
                break
            if op < 0.30:                                   # header byte
                k = rnd.randrange(min(len(p), 160))
                p[k] = rnd.randrange(256)
            elif op < 0.45 and len(p) >= 14:                # ethertype / tag key
                at = rnd.choice([12, 16, 20]) if len(p) >= 22 else 12
                v = rnd.choice(ETHERTYPES + [rnd.randrange(65536)])
                p[at:at + 2] = v.to_bytes(2, "big")
            elif op < 0.65 and len(p) > 24:                 # IP proto / next header
                at = rnd.choice([23, 27, 20, 24, 54, 62, 70])
                if at < len(p):
                    p[at] = rnd.choice(IPPROTOS + [rnd.randrange(256)])
            elif op < 0.78 and len(p) > 20:                 # length-ish fields
                at = rnd.choice([14, 15, 16, 17, 18, 19, 55, 56, 57, 63, 71])
                if at < len(p):
                    p[at] = rnd.choice([0, 1, 2, 3, 4, 5, 15, 0x45, 0x4F, 255, rnd.randrange(256)])
            elif op < 0.92:                                 # capture length
                del p[rnd.randrange(len(p) + 1):]
            else:                                           # longer capture
                p += bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 200)))
        out.append(bytes(p))
    return out


def fuzz_batch(n, seed=0xF022, align=16):
    return T.batch_from_packets(mutants(n, seed), align=align)
