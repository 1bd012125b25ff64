"""TPACKET_V3 RX ring front end (nsd_t3_block_desc; walk_t3_block
netsniff-ng.c:990-1039, struct block_desc :1061-1066, linux/if_packet.h
tpacket3_hdr / tpacket_hdr_v1 layouts): synthetic retired blocks built here,
frames at hdr + tp_mac, skip_packet rules; on the GPU the block itself is the
batch's frame buffer and the records equal the oracle's."""
import struct

import numpy as np
import pytest

import edge_cases
import nsd
import nsd_testlib as T

PACKET_HOST, PACKET_OUTGOING = 0, 4


def make_block(pkts, pkttypes=None, ifindex=None, block_len=1 << 20, mac_pad=2, slls=None, hv1=None):
    """tpacket_block_desc (48 B) + per frame tpacket3_hdr (48 B) + sockaddr_ll
    (20 B) + pad so the MAC header sits at 2 mod 16 (as the kernel places it),
    frames TPACKET_ALIGN'ed (16).  hv1: per frame (tp_status, tp_vlan_tci,
    tp_vlan_tpid) (default status 1, no VLAN)."""
    blk = bytearray(block_len)
    first = 48
    h = first
    offs = []
    for i, p in enumerate(pkts):
        mac = ((48 + 20 + 15) & ~15) + mac_pad      # TPACKET_ALIGN(hdr + sll) + NET_IP_ALIGN-ish
        nxt = (mac + len(p) + 15) & ~15
        last = i == len(pkts) - 1
        st, tci, tpid = hv1[i] if hv1 else (1, 0, 0)
        hdr = struct.pack("<IIIIIIHHIIH", 0 if last else nxt, 1000 + i, 7 * i, len(p), len(p) + 4, st, mac,
                          mac + 14, 0x5A5A5A5A, tci, tpid)
        blk[h:h + len(hdr)] = hdr
        pt = pkttypes[i] if pkttypes else PACKET_HOST
        ix = ifindex[i] if ifindex else 2
        sll = struct.pack("<HHiHBB8s", 17, 0x0008, ix, 1, pt, 6, bytes(8)) if slls is None else slls[i].tobytes()
        blk[h + 48:h + 48 + 20] = sll
        blk[h + mac:h + mac + len(p)] = p
        offs.append(h + mac)
        h += nxt
    struct.pack_into("<IIIIIIQ", blk, 0, 3, 0, 1, len(pkts), first, h, 9)
    return np.frombuffer(bytes(blk[:h + 64]), dtype=np.uint8).copy(), offs


def test_block_desc_frames():
    pkts = [p for p in edge_cases.cases() if p][:90]
    blk, offs = make_block(pkts)
    desc = nsd.t3_block_desc(blk)
    assert [int(d) & 0xFFFFFFFFFF for d in desc] == offs
    assert [bytes(blk[int(d) & 0xFFFFFFFFFF:][:int(d) >> 40]) for d in desc] == pkts
    assert all(o % 16 == 2 for o in offs)


def test_block_skip_packet_rules():
    pkts = [p for p in edge_cases.cases() if p][:20]
    types = [PACKET_OUTGOING if i % 3 == 0 else PACKET_HOST for i in range(20)]
    ifx = [1 if i % 2 == 0 else 2 for i in range(20)]
    blk, offs = make_block(pkts, types, ifx)
    # default: loopback (ifindex 1) outgoing frames are skipped
    d = nsd.t3_block_desc(blk, packet_type=-1, lo_ifindex=1)
    assert [int(x) & 0xFFFFFFFFFF for x in d] == [o for i, o in enumerate(offs) if not (ifx[i] == 1 and types[i] == 4)]
    # -t outgoing: only PACKET_OUTGOING frames
    d = nsd.t3_block_desc(blk, packet_type=PACKET_OUTGOING, lo_ifindex=1)
    assert [int(x) & 0xFFFFFFFFFF for x in d] == [o for i, o in enumerate(offs) if types[i] == 4]


def test_block_inconsistent():
    pkts = [p for p in edge_cases.cases() if p][:5]
    blk, _ = make_block(pkts)
    bad = blk.copy()
    struct.pack_into("<I", bad, 12, 50)            # more frames than the chain holds
    with pytest.raises(nsd.NsdError):
        nsd.t3_block_desc(bad)
    with pytest.raises(nsd.NsdError):
        nsd.t3_block_desc(blk[:200])               # headers past the block


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_block_dissect_on_device(mode):
    from test_device_parity import assert_same_records
    pkts = [p for p in edge_cases.cases() if p]
    blk, _ = make_block(pkts)
    desc = nsd.t3_block_desc(blk)
    rec, ext, cnt = nsd.entry_batch(blk, desc, mode=mode)
    orec, oext, ocnt, _ = T.oracle_records(blk, desc, mode=mode)
    assert_same_records(rec, orec, ext, oext)
    assert np.array_equal(cnt, ocnt)


def test_block_sll_copied():
    """nsd_t3_block_desc_sll hands each kept frame's sockaddr_ll (hdr + 48,
    walk_t3_block's `sll`) out beside its descriptor, skip rules applied."""
    pkts = [p for p in edge_cases.cases() if p][:30]
    types = [PACKET_OUTGOING if i % 3 == 0 else PACKET_HOST for i in range(30)]
    ifx = [1 if i % 2 == 0 else 2 + i for i in range(30)]
    blk, offs = make_block(pkts, types, ifx)
    desc, sll = nsd.t3_block_desc(blk, packet_type=-1, lo_ifindex=1, sll=True)
    keep = [i for i in range(30) if not (ifx[i] == 1 and types[i] == 4)]
    assert [int(x) & 0xFFFFFFFFFF for x in desc] == [offs[i] for i in keep]
    assert list(sll["ifindex"]) == [ifx[i] for i in keep]
    assert list(sll["pkttype"]) == [types[i] for i in keep]
    assert set(sll["protocol"]) == {0x0800} and set(sll["hatype"]) == {1} and set(sll["family"]) == {17}


def _live_ring():
    import ring_live as RL
    r = RL.open_ring()
    if r is None:
        pytest.skip("AF_PACKET sockets need CAP_NET_RAW here")
    return r


def _live_frames():
    """Edge and leaf frames for the loopback ring, minus 802.1Q / 802.1ad ones
    (the receive path moves their tag into tp_vlan_tci) and jumbo ones."""
    import leaf_cases
    import ring_live as RL
    pkts = [p for p in edge_cases.cases() + leaf_cases.cases(300, seed=5) if 14 <= len(p) <= 9000]
    return RL.marked([p for p in pkts if p[12:14] not in (b"\x81\x00", b"\x88\xa8")])


def test_live_ring_block_desc():
    """A real PACKET_RX_RING on lo (ring_rx.c:28-229 setup): the frames the
    retired blocks hold, through nsd_t3_block_desc with netsniff-ng's skip
    rule for loopback's outgoing copies (skip_packet, netsniff-ng.c), are
    the frames sent, in order."""
    import ring_live as RL
    r = _live_ring()
    try:
        pkts = _live_frames()
        r.send(pkts)

        def frames_of(k):
            blk = r.block(k)
            desc = nsd.t3_block_desc(blk, packet_type=-1, lo_ifindex=r.ifindex)
            return [bytes(blk[int(d) & 0xFFFFFFFFFF:][:int(d) >> 40]) for d in desc]
        got = RL.collect(r, len(pkts), frames_of)
        assert got == pkts
    finally:
        r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_live_ring_registered_through_pipe(mode):
    """The same ring on the GPU: each retired block is registered with
    nsd_host_register (hipHostRegister of the mmap'd ring memory), walked
    through nsd_pipe_submit straight from the block, and its records and
    counters equal the oracle's."""
    import ring_live as RL
    from test_device_parity import assert_same_records
    r = _live_ring()
    pipe = nsd.Pipe(1 << 16, r.block_size, ext_words=nsd.ext_pool_words(1 << 16), depth=2, mode=mode)
    L = nsd.lib()
    try:
        pkts = _live_frames()
        r.send(pkts)

        def walk(k):
            blk = r.block(k)
            assert L.nsd_host_register(blk.ctypes.data, blk.nbytes) == 0
            try:
                desc = nsd.t3_block_desc(blk, packet_type=-1, lo_ifindex=r.ifindex)
                n = len(desc)
                rec = np.zeros(n, dtype=nsd.REC_DTYPE)
                ext = np.zeros(pipe.ext_words, dtype=np.uint32)
                used = np.zeros(1, dtype=np.uint32)
                cnt = np.zeros(nsd.NCOUNTERS, dtype=np.uint64)
                st = np.full(1, -99, dtype=np.int32)
                pipe.submit(blk, desc, rec, ext, used, cnt, st)
                assert pipe.drain() == 0 and st[0] == 0
                orec, oext, ocnt, _ = T.oracle_records(blk, desc, mode=mode)
                assert_same_records(rec, orec, ext[:int(used[0])], oext)
                assert np.array_equal(cnt, ocnt)
                return [bytes(blk[int(d) & 0xFFFFFFFFFF:][:int(d) >> 40]) for d in desc]
            finally:
                assert L.nsd_host_unregister(blk.ctypes.data) == 0
        got = RL.collect(r, len(pkts), walk)
        assert got == pkts
    finally:
        pipe.close()
        r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_cooked_ring_through_pipe(mode):
    """A cooked (LINKTYPE_LINUX_SLL) ring: the block is the frame buffer, the
    per-frame sockaddr_ll goes with it through nsd_pipe_submit_sll, records
    and counters equal the oracle's."""
    from test_device_parity import assert_same_records
    import test_sll as TS
    cases = TS.sll_cases()
    slls = np.array([s for _, s in cases], dtype=nsd.SLL_DTYPE)
    blk, _ = make_block([p for p, _ in cases], slls=slls)
    desc, sll = nsd.t3_block_desc(blk, sll=True)
    assert sll.tobytes() == slls.tobytes()
    n = len(desc)
    words = nsd.ext_pool_words(n)
    pipe = nsd.Pipe(n, blk.nbytes, ext_words=words, depth=2, mode=mode, linktype=nsd.LINKTYPE_LINUX_SLL)
    rec = np.zeros(n, dtype=nsd.REC_DTYPE)
    ext = np.zeros(words, dtype=np.uint32)
    used = np.zeros(1, dtype=np.uint32)
    cnt = np.zeros(nsd.NCOUNTERS, dtype=np.uint64)
    st = np.full(1, -99, dtype=np.int32)
    pipe.submit(blk, desc, rec, ext, used, cnt, st, sll=sll)
    assert pipe.drain() == 0 and st[0] == 0
    pipe.close()
    orec, oext, ocnt, _ = T.oracle_records(blk, desc, linktype=nsd.LINKTYPE_LINUX_SLL, mode=mode, sll=sll)
    assert_same_records(rec, orec, ext[:int(used[0])], oext)
    assert np.array_equal(cnt, ocnt)
