"""LINKTYPE_LINUX_SLL heads (dissector_sll.c:39-82): the "cooked" head prints
the packet's struct sockaddr_ll and, in print_full, continues in eth_lay2
with sll_protocol for Ethernet-class hatypes (pcap_devtype_to_linktype,
pcap_io.h:205-267).

dissector_sll.c itself is unbuildable here (dissector.h -> ring.h -> the
configure-generated config.h), so its text is pinned by the CPU restatement;
the tables it prints through — device_type2str / device_addr2str, dev.c —
compile from the reference and pin the formatter's tables
(oracle/_ref/nsref -T)."""
import os
import re
import subprocess

import numpy as np
import pytest

import edge_cases as E
import nsd
import nsd_testlib as T

ADDR = bytes.fromhex("deadbeef01020304")


def ref_tables():
    out = subprocess.run([T.REF_BIN, "-T"], check=True, capture_output=True, timeout=60).stdout.decode()
    types, addrs = {}, {}
    for line in out.splitlines():
        f = line.split(" ", 3)
        if f[0] == "T":
            types[int(f[1])] = f[2]
        elif f[0] == "A":
            addrs[(int(f[1]), int(f[2]))] = f[3] if len(f) > 3 else ""
    return types, addrs


def sll_cases():
    """(payload, sll) pairs over every named hatype, the EN10MB / netlink /
    other dispatch classes, packet types, address lengths (incl. > 8)."""
    types = [0, 1, 2, 5, 19, 32, 256, 512, 768, 769, 772, 776, 777, 778, 787, 799, 800, 803, 820,
             823, 824, 0xFFFE, 0xFFFF, 5000]
    protos = [0x0800, 0x86DD, 0x0806, 0x8100, 0x1234, 0x88CC]
    pay = {
        0x0800: E.ipv4(17, 8 + 6) + E.udp(payload=b"cooked"),
        0x86DD: E.ipv6(17, 8 + 2) + E.udp(payload=b"v6"),
        0x0806: bytes(28),
        0x8100: E.be16(5) + E.be16(0x0800) + E.ipv4(6, 20) + bytes(20),
        0x1234: b"opaque",
        0x88CC: bytes(16),
    }
    out = []
    k = 0
    for t in types:
        for pr in protos:
            s = np.zeros(1, dtype=nsd.SLL_DTYPE)[0]
            s["family"] = 17
            s["protocol"] = pr
            s["ifindex"] = 2 + k
            s["hatype"] = t
            s["pkttype"] = k % 9
            s["halen"] = [6, 0, 4, 8, 16, 10, 1][k % 7]
            s["addr"] = np.frombuffer(ADDR, dtype=np.uint8)
            out.append((pay[pr], s))
            k += 1
    return out


def batch():
    cases = sll_cases()
    frames, desc = T.batch_from_packets([p for p, _ in cases])
    sll = np.array([s for _, s in cases], dtype=nsd.SLL_DTYPE)
    return frames, desc, sll


@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_formatter_matches_restatement(mode):
    frames, desc, sll = batch()
    rec, ext, _, _ = T.oracle_records(frames, desc, linktype=nsd.LINKTYPE_LINUX_SLL, mode=mode, sll=sll)
    texts, rc = nsd.format_batch(frames, desc, rec, ext, mode=mode, linktype=nsd.LINKTYPE_LINUX_SLL, sll=sll)
    ora = T.oracle_text_packets(frames, desc, linktype=nsd.LINKTYPE_LINUX_SLL, mode=mode, sll=sll)
    chained = 0
    for i in range(len(desc)):
        last = (int(rec[i]["chain"]) >> (5 * ((int(rec[i]["nflags"]) & 7) - 1))) & 31
        if last == 27:   # netlink continuation: nlmsg is outside the path
            assert sll[i]["hatype"] == 824 and rc[i] != 0
            continue
        assert rc[i] == 0, f"packet {i}: status {rc[i]}"
        if not ora[i][1]:
            assert texts[i] == ora[i][0], f"packet {i}"
        chained += (int(rec[i]["nflags"]) & 7) > 1
    if mode == T.PRINT_NORM:
        assert chained >= 40       # 8 Ethernet-class hatypes x 5 eth_lay2 keys continue
    else:
        assert chained == 0        # sll_print_less dispatches nothing


@pytest.mark.skipif(not os.path.exists(T.REF_BIN), reason="needs oracle/_ref/nsref (built with /root/reference)")
def test_tables_match_reference_dev_c():
    types, addrs = ref_tables()
    assert len(types) > 60
    # every named hatype, rendered through the product formatter
    pk = E.ipv4(17, 8) + E.udp()
    for t, name in list(types.items()) + [(5000, "Unknown"), (0, "Unknown")]:
        s = np.zeros(1, dtype=nsd.SLL_DTYPE)
        s["hatype"] = t
        s["protocol"] = 0x0800
        frames, desc = T.batch_from_packets([pk])
        rec, ext, _, _ = T.oracle_records(frames, desc, linktype=nsd.LINKTYPE_LINUX_SLL, sll=s)
        texts, _ = nsd.format_batch(frames, desc, rec, ext, linktype=nsd.LINKTYPE_LINUX_SLL, sll=s)
        m = re.search(rb"If Type (\d+) \(([^)]*)\)", texts[0])
        assert m and int(m.group(1)) == t and m.group(2).decode() == name, (t, name, texts[0][:120])
    # device_addr2str at every (type, alen) the harness dumped
    for (t, alen), want in addrs.items():
        s = np.zeros(1, dtype=nsd.SLL_DTYPE)
        s["hatype"] = t & 0xFFFF
        s["halen"] = alen
        s["addr"] = np.frombuffer(ADDR, dtype=np.uint8)
        frames, desc = T.batch_from_packets([b"x"])
        rec, ext, _, _ = T.oracle_records(frames, desc, linktype=nsd.LINKTYPE_LINUX_SLL, sll=s)
        texts, _ = nsd.format_batch(frames, desc, rec, ext, linktype=nsd.LINKTYPE_LINUX_SLL, sll=s)
        m = re.search(rb"Src \((.*?)\), Proto", texts[0])
        assert m and m.group(1).decode() == want, (t, alen, want, texts[0][:160])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_sll_device_vs_oracle(mode):
    from test_device_parity import assert_same_records
    frames, desc, sll = batch()
    rec, ext, cnt = nsd.entry_batch(frames, desc, mode=mode, linktype=nsd.LINKTYPE_LINUX_SLL, sll=sll)
    orec, oext, ocnt, _ = T.oracle_records(frames, desc, linktype=nsd.LINKTYPE_LINUX_SLL, mode=mode, sll=sll)
    assert_same_records(rec, orec, ext, oext)
    assert np.array_equal(cnt, ocnt)
    # without per-packet sockaddr_ll the head reads zeros (hatype 0: no dispatch)
    rec0, _, _ = nsd.entry_batch(frames, desc, mode=mode, linktype=nsd.LINKTYPE_LINUX_SLL)
    orec0, _, _, _ = T.oracle_records(frames, desc, linktype=nsd.LINKTYPE_LINUX_SLL, mode=mode)
    assert np.array_equal(rec0["chain"], orec0["chain"]) and np.array_equal(rec0["nflags"], orec0["nflags"])
