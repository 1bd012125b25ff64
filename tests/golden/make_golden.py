"""Regenerate the committed golden fixtures (run in the build container, where
/root/reference exists and oracle/_ref/nsref is built):

  tiny.pcap            C1: 1000 x 64 B Eth/IPv4/UDP
  edge.pcap            tests/edge_cases.py (every §8a quirk)
  big.pcap             records longer than a batch carries (NSD_MAX_CAPLEN <
                       caplen <= read_pcap's 1 MiB buffer) between short ones
  leaves.pcap          tests/leaf_cases.py: ARP / DCCP / IGMP / LLDP / ICMPv6
                       130-154 frames (NORM and LESS text; --leaves-only)
  <pcap>.m<M>.w<C>.txt.gz / .ends.json
                       text printed by the REFERENCE parser objects
                       (oracle/_ref/nsref) for print mode M, terminal width C
                       (65535 = unwrapped, 80 = tprintf's default wrap),
                       names off (no conf files);  .names. = conf files of
                       /root/reference loaded
  prefix.json          SHA-256 of the nsref text of the first 65536 packets of
                       C2/C3/C4 (NORM, LESS) and of the oracle records / counters
  wsum.json            sum of W(pkt) (algorithmic read bytes) over
                       the 16M-packet shards used by bench.py (rank r of
                       --gpus N walks shard r; 8 IMIX shards = C5)
  shard_counters.json  the oracle's PRINT_NORM counter vector per bench shard
                       (bench.py checks the all-reduced device counters
                       against their sum; --shards-only: these two only)
  lines.json           the line floor per bench shard (distinct 128-byte lines
                       of the bytes the chains inspect; --lines-only)
  ip_vectors.npz       tests/ip_vectors.py: IPv4 / IPv6 / ICMPv4 frames and
                       the values the reference's csum.h / ipv4.h / ipv6.h
                       give for them (oracle/_ref/libnsdrefip.so; --ip-only)
  (--edge-only: the two pcaps and their texts only)
  <pcap>.fh.m<M>.w<C>  `netsniff-ng --in <pcap>` (nsref -f: read_pcap's loop
                       over the reference's own pcap reader and
                       pcap_pkthdr_to_tpacket_hdr, show_frame_hdr's line
                       before each packet's dissector text) for tiny, big,
                       leaves and the record-format fixtures below
  fh_*.pcap            edge.pcap's non-empty frames in each record format
                       (tests/pcap_formats.py: usec / nsec / Kuznetzov /
                       Borkmann, both byte orders, the *_LL form of SLL
                       files) with varied timestamps, lengths and link-layer
                       metadata (--fh-only: these and the .fh. texts only)

IPv4/IPv6 layers inside nsref come from the restatement (their reference
sources need the configure-generated config.h); see oracle/ref_harness.c.
"""
import gzip
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import edge_cases  # noqa: E402
import leaf_cases  # noqa: E402
import nsd_testlib as T  # noqa: E402

MODES = [T.PRINT_NORM, T.PRINT_LESS, T.PRINT_HEX, T.PRINT_ASCII, T.PRINT_HEX_ASCII]


def save_text(base, texts):
    ends, off = [], 0
    for t in texts:
        off += len(t)
        ends.append(off)
    with gzip.open(base + ".txt.gz", "wb", compresslevel=9) as f:
        f.write(b"".join(texts))
    with open(base + ".ends.json", "w") as f:
        json.dump(ends, f)


def rec_digest(rec, ext):
    """Records with ext slots replaced by the slot's content (slot order is
    arbitrary on the device)."""
    h = hashlib.sha256()
    for i in range(len(rec)):
        r = rec[i]
        if (int(r["nflags"]) & 7) == 7:
            slot = int.from_bytes(bytes(r["off2"][:4]), "little")
            h.update(r.tobytes()[:11])
            if slot != 0xFFFFFFFF:
                # pool entry: {pkt, nlayers, 0, 0, id | off << 16 ...}; hashed
                # as u8 ids then LE u16 offsets
                m = int(ext[slot + 1]) & 0xFFFF
                w = np.asarray(ext[slot + 4:slot + 4 + m], dtype=np.uint32)
                h.update((w & 0xFF).astype(np.uint8).tobytes() + (w >> 16).astype("<u2").tobytes())
        else:
            h.update(r.tobytes())
    return h.hexdigest()


def big_cases():
    """Frames above 65535 bytes (tcpdump's default snaplen is 262144; GRO
    frames), with payload patterns that compress: Eth/IPv4/UDP (tot_len at
    its u16 maximum: the IPv4 trim cuts the tail), Eth/IPv4/ICMP echo (the
    checksum reads the whole post-trim message), Eth/IPv6/HBH/UDP, between
    short frames of tiny.pcap and edge.pcap."""
    import struct
    lt, tiny = T.read_pcap(os.path.join(HERE, "tiny.pcap"))
    _, edge = T.read_pcap(os.path.join(HERE, "edge.pcap"))

    def pay(n, k):
        return bytes((i * k) % 251 for i in range(n))

    eth4 = bytes.fromhex("0a0b0c0d0e0f" "020304050607" "0800")
    eth6 = bytes.fromhex("0a0b0c0d0e0f" "020304050607" "86dd")

    def ipv4(proto, tot_len):
        h = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, tot_len, 7, 0x4000, 64, proto, 0,
                                  bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])))
        s = sum(struct.unpack(">10H", bytes(h)))
        s = (s & 0xFFFF) + (s >> 16)
        s = (s & 0xFFFF) + (s >> 16)
        h[10:12] = struct.pack(">H", ~s & 0xFFFF)
        return bytes(h)

    udp_big = eth4 + ipv4(17, 65535) + struct.pack(">HHHH", 5353, 53, 65515, 0) + pay(70000 - 42, 7)
    icmp_big = eth4 + ipv4(1, 65535) + bytes([8, 0, 0x12, 0x34, 0, 1, 0, 2]) + pay(66002 - 42, 13)
    v6 = (eth6 + bytes([0x60, 0, 0, 0]) + struct.pack(">HBB", 0, 0, 64) + bytes(range(32))
          + bytes([17, 0, 1, 4, 0, 0, 0, 0]) + struct.pack(">HHHH", 1000, 2000, 8, 0) + pay(100000 - 70, 3))
    return [tiny[0], udp_big, edge[5], icmp_big, v6, tiny[1]]


def frame_goldens():
    """The `--in` texts with frame headers (nsref -f)."""
    import pcap_formats as PF
    _, edge = T.read_pcap(os.path.join(HERE, "edge.pcap"))
    frames = [p for p in edge if p]
    for name, kw in PF.VARIANTS.items():
        path = os.path.join(HERE, name + ".pcap")
        PF.write(path, frames, **kw)
        modes = MODES if name == "fh_usec" else (T.PRINT_NORM, T.PRINT_LESS)
        for m in modes:
            save_text(os.path.join(HERE, f"{name}.fh.m{m}.w65535"), T.run_ref(path, mode=m, cols=65535, frames="f"))
        if name in ("fh_usec", "fh_kuz"):
            for m in (T.PRINT_NORM, T.PRINT_LESS):
                save_text(os.path.join(HERE, f"{name}.fh.m{m}.w80"), T.run_ref(path, mode=m, cols=0, frames="f"))
    for stem, modes in (("tiny", MODES), ("big", MODES), ("leaves", (T.PRINT_NORM, T.PRINT_LESS))):
        path = os.path.join(HERE, stem + ".pcap")
        for m in modes:
            save_text(os.path.join(HERE, f"{stem}.fh.m{m}.w65535"), T.run_ref(path, mode=m, cols=65535, frames="f"))
    for m in (T.PRINT_NORM, T.PRINT_LESS):
        save_text(os.path.join(HERE, f"tiny.fh.m{m}.w80"), T.run_ref(os.path.join(HERE, "tiny.pcap"), mode=m,
                                                                     cols=0, frames="f"))


def main():
    T.build_native()
    if "--lines-only" in sys.argv:
        line_floor_shards()
        return
    if "--shards-only" in sys.argv:
        wsum_shards()
        return
    if "--fh-only" in sys.argv:
        frame_goldens()
        return
    if "--prefix-only" in sys.argv:
        prefix_digests()
        return
    import ip_vectors
    ip_vectors.save()
    if "--ip-only" in sys.argv:
        return
    leaves = os.path.join(HERE, "leaves.pcap")
    T.write_pcap(leaves, leaf_cases.cases())
    for m in (T.PRINT_NORM, T.PRINT_LESS):
        save_text(os.path.join(HERE, f"leaves.m{m}.w65535"), T.run_ref(leaves, mode=m, cols=65535))
    if "--leaves-only" in sys.argv:
        return
    big = os.path.join(HERE, "big.pcap")
    T.write_pcap(big, big_cases())
    for m in MODES:
        save_text(os.path.join(HERE, f"big.m{m}.w65535"), T.run_ref(big, mode=m, cols=65535))
    if "--big-only" in sys.argv:
        return
    tiny = os.path.join(HERE, "tiny.pcap")
    edge = os.path.join(HERE, "edge.pcap")
    T.synth().nsd_synth_pcap(T.SYN_UDP64, T.SEED, 0, 1000, tiny.encode())
    T.write_pcap(edge, edge_cases.cases())
    for pcap in (tiny, edge):
        stem = os.path.splitext(pcap)[0]
        for m in MODES:
            save_text(f"{stem}.m{m}.w65535", T.run_ref(pcap, mode=m, cols=65535))
        for m in (T.PRINT_NORM, T.PRINT_LESS):
            save_text(f"{stem}.m{m}.w80", T.run_ref(pcap, mode=m, cols=0))
            save_text(f"{stem}.names.m{m}.w65535", T.run_ref(pcap, mode=m, cols=65535, names=True))
    frame_goldens()
    if "--edge-only" in sys.argv:
        return
    prefix_digests()
    if "--prefix-only" in sys.argv:
        return
    wsum_shards()


def prefix_digests():
    prefix = {}
    for key, cfg in (("udp64", T.SYN_UDP64), ("imix", T.SYN_IMIX), ("ipv6x", T.SYN_IPV6X)):
        path = f"/tmp/golden_{key}.pcap"
        T.synth().nsd_synth_pcap(cfg, T.SEED, 0, 65536, path.encode())
        frames, desc = T.make_batch(cfg, 65536)
        for m in (T.PRINT_NORM, T.PRINT_LESS):
            txt = b"".join(T.run_ref(path, mode=m, cols=65535, timeout=600))
            txt_fh = b"".join(T.run_ref(path, mode=m, cols=65535, timeout=600, frames="f"))
            rec, ext, cnt, sw = T.oracle_records(frames, desc, mode=m)
            prefix[f"{key}:m{m}"] = {"text_sha256": hashlib.sha256(txt).hexdigest(),
                                     "replay_text_sha256": hashlib.sha256(txt_fh).hexdigest(),
                                     "records_sha256": rec_digest(rec, ext),
                                     "counters": [int(x) for x in cnt], "wsum": sw}
        os.unlink(path)
    with open(os.path.join(HERE, "prefix.json"), "w") as f:
        json.dump(prefix, f, indent=1)


def wsum_shards():
    """wsum.json (ΣW per bench shard) and shard_counters.json (the oracle's
    PRINT_NORM counter vector per bench shard): the 16M-packet shards
    [r * 16M, (r + 1) * 16M) that rank r of `bench.py --gpus N` walks, r < 8,
    for every bench config (8 IMIX shards = C5)."""
    wsum, cnts = {}, {}
    n = 1 << 24
    for key, cfg, shards in (("imix", T.SYN_IMIX, 8), ("ipv6x", T.SYN_IPV6X, 8), ("udp64", T.SYN_UDP64, 8)):
        for r in range(shards):
            frames, desc = T.make_batch(cfg, n, lo=r * n)
            counters = np.zeros(64, dtype=np.uint64)
            sw = T.oracle().nsor_dissect_batch_mt(frames.ctypes.data, desc.ctypes.data, n, 1,
                                                  T.PRINT_NORM, None, counters.ctypes.data, 8)
            if key != "udp64":   # C2's W is caplen (bench.wsum_for)
                wsum[f"{key}:{r * n}:{n}"] = int(sw)
            cnts[f"{key}:{r * n}:{n}"] = [int(x) for x in counters]
            del frames, desc
            print(key, r, sw, flush=True)
    with open(os.path.join(HERE, "wsum.json"), "w") as f:
        json.dump(wsum, f, indent=1)
    with open(os.path.join(HERE, "shard_counters.json"), "w") as f:
        json.dump(cnts, f)



def line_floor_shards():
    """lines.json: the line floor of each bench shard - the distinct 128-byte
    lines holding the bytes its chains must inspect ([off, off + W) per
    packet, nsor_line_floor_mt), the least whole-line HBM reads any schedule
    can fetch (bench.py reports the measured traffic against it)."""
    import ctypes
    L = T.oracle()
    L.nsor_line_floor_mt.restype = ctypes.c_uint64
    L.nsor_line_floor_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int]
    lines = {}
    n = 1 << 24
    for key, cfg, shards in (("imix", T.SYN_IMIX, 8), ("ipv6x", T.SYN_IPV6X, 8), ("udp64", T.SYN_UDP64, 8)):
        for r in range(shards):
            frames, desc = T.make_batch(cfg, n, lo=r * n)
            lines[f"{key}:{r * n}:{n}"] = int(L.nsor_line_floor_mt(frames.ctypes.data, desc.ctypes.data, n, 1,
                                                                   T.PRINT_NORM, 8))
            del frames, desc
            print(key, r, lines[f"{key}:{r * n}:{n}"], flush=True)
    with open(os.path.join(HERE, "lines.json"), "w") as f:
        json.dump(lines, f, indent=1)


if __name__ == "__main__":
    main()
