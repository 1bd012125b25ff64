"""Shared helpers for the test suite: ctypes bindings to the synthetic
generators (tools/), the CPU oracle (oracle/, TEST INFRASTRUCTURE) and the
oracle/_ref reference harness, plus pcap I/O.  Only tests/, bench.py's
cpu_baseline leg and __graft_entry__.smoke() use the oracle parts."""
import ctypes
import os
import struct
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
REF_BIN = os.path.join(ORACLE_DIR, "_ref", "nsref")
SYNTH_SO = os.path.join(ROOT, "tools", "libnsdsynth.so")
ORACLE_SO = os.path.join(ORACLE_DIR, "libnsdoracle.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

PRINT_NORM, PRINT_LESS, PRINT_HEX, PRINT_ASCII, PRINT_HEX_ASCII, PRINT_NONE = range(6)
SYN_UDP64, SYN_IMIX, SYN_IPV6X = 1, 3, 4
SEED = 0x5EED

REC_DTYPE = np.dtype([("chain", "<u4"), ("data_off", "<u2"), ("tail_off", "<u2"),
                      ("ip_csum", "<u2"), ("nflags", "u1"), ("off2", "u1", (5,))])
assert REC_DTYPE.itemsize == 16
NCOUNTERS = 64


def build_native(quiet=True):
    """Build tools/ and oracle/ C libraries (and oracle/_ref when the
    reference tree is present).  Idempotent."""
    out = subprocess.DEVNULL if quiet else None
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools")], check=True, stdout=out)
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True, stdout=out)
    if os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "ref"], check=True, stdout=out)


_synth = None
_oracle = None


def synth():
    global _synth
    if _synth is None:
        lib = ctypes.CDLL(SYNTH_SO)
        lib.nsd_synth_layout.restype = ctypes.c_uint64
        lib.nsd_synth_layout.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                         ctypes.c_void_p]
        lib.nsd_synth_fill.restype = None
        lib.nsd_synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int]
        lib.nsd_synth_pcap.restype = ctypes.c_uint64
        lib.nsd_synth_pcap.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_uint64, ctypes.c_char_p]
        _synth = lib
    return _synth


def make_batch(cfg, n, lo=0, seed=SEED, align=16, threads=8, pad=64):
    """Generate packets [lo, lo+n) of a config: returns (frames u8 array,
    desc u64 array)."""
    s = synth()
    desc = np.zeros(n, dtype=np.uint64)
    end = s.nsd_synth_layout(cfg, seed, lo, n, align, 0, desc.ctypes.data)
    frames = np.zeros(end + pad, dtype=np.uint8)
    s.nsd_synth_fill(cfg, seed, lo, n, frames.ctypes.data, desc.ctypes.data, threads)
    return frames, desc


def make_device_batch(cfg, n, lo=0, seed=SEED, device="cuda", chunk=1 << 24, threads=16, on_chunk=None,
                      pad=64):
    """Packets [lo, lo+n) of a config generated chunk by chunk on the host
    and copied into one device buffer (the host never holds more than one
    chunk of frames: C5's 128M IMIX frames are 47.6 GB).  Frames are packed
    at 16-byte boundaries from byte 0 exactly as make_batch() packs them.
    on_chunk(a, frames_chunk, desc_chunk_rebased) is called per chunk with
    the host copy (descriptors rebased to the chunk's first byte), e.g. for
    oracle checks.  Returns (frames u8 cuda tensor, desc i64 cuda tensor,
    desc numpy u64)."""
    import torch
    s = synth()
    desc = np.zeros(n, dtype=np.uint64)
    end = s.nsd_synth_layout(cfg, seed, lo, n, 16, 0, desc.ctypes.data)
    frames = torch.empty(end + pad, dtype=torch.uint8, device=device)
    frames[end:].zero_()
    offs, caps = desc_off(desc), desc_caplen(desc)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        lo_b = int(offs[a])
        hi_b = int(offs[b - 1] + caps[b - 1])
        host = np.zeros(hi_b - lo_b + pad, dtype=np.uint8)
        d = desc[a:b] - np.uint64(lo_b)
        s.nsd_synth_fill(cfg, seed, lo + a, b - a, host.ctypes.data, d.ctypes.data, threads)
        frames[lo_b:hi_b].copy_(torch.from_numpy(host[:hi_b - lo_b]))
        if on_chunk is not None:
            on_chunk(a, host, d)
        del host
    dd = torch.from_numpy(desc.view(np.int64)).to(device)
    return frames, dd, desc


def desc_pack(off, caplen):
    return (np.uint64(caplen) << np.uint64(40)) | np.uint64(off)


def desc_off(desc):
    return (desc & np.uint64(0xFFFFFFFFFF)).astype(np.int64)


def desc_caplen(desc):
    return (desc >> np.uint64(40)).astype(np.int64)


def batch_from_packets(pkts, align=16, pad=64):
    """List of bytes -> (frames, desc)."""
    offs, off = [], 0
    for p in pkts:
        off = (off + align - 1) & ~(align - 1)
        offs.append(off)
        off += len(p)
    frames = np.zeros(off + pad, dtype=np.uint8)
    desc = np.zeros(len(pkts), dtype=np.uint64)
    for i, (o, p) in enumerate(zip(offs, pkts)):
        frames[o:o + len(p)] = np.frombuffer(bytes(p), dtype=np.uint8)
        desc[i] = desc_pack(o, len(p))
    return frames, desc


def write_pcap(path, pkts, linktype=1):
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, linktype))
        for i, p in enumerate(pkts):
            f.write(struct.pack("<IIII", i, 0, len(p), len(p)))
            f.write(bytes(p))


def read_pcap(path):
    with open(path, "rb") as f:
        data = f.read()
    magic = struct.unpack_from("<I", data, 0)[0]
    e = "<" if magic in (0xA1B2C3D4, 0xA1B23C4D) else ">"
    linktype = struct.unpack_from(e + "I", data, 20)[0]
    pkts, o = [], 24
    while o + 16 <= len(data):
        _, _, caplen, _ = struct.unpack_from(e + "IIII", data, o)
        o += 16
        pkts.append(data[o:o + caplen])
        o += caplen
    return linktype, pkts


# ---- oracle (TEST INFRASTRUCTURE) ------------------------------------------
class _Text(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_void_p), ("len", ctypes.c_size_t), ("cap", ctypes.c_size_t),
                ("unsupported", ctypes.c_int)]


def oracle():
    global _oracle
    if _oracle is None:
        lib = ctypes.CDLL(ORACLE_SO)
        lib.nsor_dissect_batch.restype = ctypes.c_uint64
        lib.nsor_dissect_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_void_p]
        lib.nsor_dissect_batch_sll.restype = ctypes.c_uint64
        lib.nsor_dissect_batch_sll.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                               ctypes.c_void_p, ctypes.c_void_p]
        lib.nsor_set_sll.restype = None
        lib.nsor_set_sll.argtypes = [ctypes.c_void_p]
        lib.nsor_dissect_batch_mt.restype = ctypes.c_uint64
        lib.nsor_dissect_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_int]
        lib.nsor_dissect_batch_text_mt.restype = ctypes.c_uint64
        lib.nsor_dissect_batch_text_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                   ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_void_p]
        lib.nsor_dissect_batch_text.restype = ctypes.c_uint64
        lib.nsor_dissect_batch_text.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                ctypes.c_int, ctypes.c_int, ctypes.POINTER(_Text)]
        lib.nsor_dissect.restype = None
        lib.nsor_dissect.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(_Text), ctypes.c_void_p, ctypes.c_void_p]
        lib.nsor_text_free.argtypes = [ctypes.POINTER(_Text)]
        lib.nsor_lookup_init.restype = ctypes.c_int
        lib.nsor_lookup_init.argtypes = [ctypes.c_char_p]
        lib.nsor_dissect_batch_text_fh_mt.restype = ctypes.c_uint64
        lib.nsor_dissect_batch_text_fh_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        lib.nsor_frame_hdr.restype = None
        lib.nsor_frame_hdr.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(_Text)]
        lib.nsor_pcap_meta.restype = ctypes.c_long
        lib.nsor_pcap_meta.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint32]
        _oracle = lib
    return _oracle


def oracle_records(frames, desc, linktype=1, mode=PRINT_NORM, ext_words=None, sll=None):
    """Returns (rec, ext pool words[:used], counters, sum_w)."""
    lib = oracle()
    n = len(desc)
    if ext_words is None:
        ext_words = 48 * n + 4096          # NSD_EXT_POOL_WORDS(n)
    rec = np.zeros(n, dtype=REC_DTYPE)
    ext = np.zeros(max(ext_words, 1), dtype=np.uint32)
    used = np.zeros(1, dtype=np.uint32)
    counters = np.zeros(NCOUNTERS, dtype=np.uint64)
    sw = lib.nsor_dissect_batch_sll(frames.ctypes.data, desc.ctypes.data,
                                    None if sll is None else sll.ctypes.data, n, linktype, mode,
                                    rec.ctypes.data, ext.ctypes.data, ext_words, used.ctypes.data,
                                    counters.ctypes.data)
    return rec, ext[:min(int(used[0]), ext_words)], counters, int(sw)


def oracle_text_packets(frames, desc, linktype=1, mode=PRINT_NORM, sll=None):
    """Per-packet oracle text (list of (bytes, unsupported))."""
    lib = oracle()
    out = []
    offs, caps = desc_off(desc), desc_caplen(desc)
    for i in range(len(desc)):
        t = _Text()
        p = frames[offs[i]:offs[i] + caps[i]]
        lib.nsor_set_sll(None if sll is None else sll[i:i + 1].ctypes.data)
        lib.nsor_dissect(p.ctypes.data, int(caps[i]), linktype, mode, ctypes.byref(t), None, None)
        s = ctypes.string_at(t.buf, t.len) if t.len else b""
        out.append((s, bool(t.unsupported)))
        lib.nsor_text_free(ctypes.byref(t))
    lib.nsor_set_sll(None)
    return out


# nsd_frame_hdr_t / struct sockaddr_ll (as netsniff-ng_amd/nsd.py declares them)
FH_DTYPE = np.dtype([("len", "<u4"), ("sec", "<u4"), ("nsec", "<u4"), ("status", "<u4"), ("vlan_tci", "<u4"),
                     ("vlan_tpid", "<u2"), ("v3", "u1"), ("reserved", "u1")])
SLL_DTYPE = np.dtype([("family", "<u2"), ("protocol", ">u2"), ("ifindex", "<i4"), ("hatype", "<u2"),
                      ("pkttype", "u1"), ("halen", "u1"), ("addr", "u1", (8,))])


def oracle_pcap_meta(path, max_n=1 << 20):
    """read_pcap's per-record frame header fields, sockaddr_ll and caplen,
    restated (nsor_pcap_meta): (fh, sll, caplen) arrays, or None for a file
    read_pcap refuses."""
    fh = np.zeros(max_n, dtype=FH_DTYPE)
    sll = np.zeros(max_n, dtype=SLL_DTYPE)
    cl = np.zeros(max_n, dtype=np.uint32)
    n = oracle().nsor_pcap_meta(os.fsencode(path), fh.ctypes.data, sll.ctypes.data, cl.ctypes.data, max_n)
    if n < 0:
        return None
    return fh[:n], sll[:n], cl[:n]


def oracle_frame_hdr(fh, sll=None, pkt=b"", linktype=1, mode=PRINT_NORM, count=1):
    """show_frame_hdr's line restated (nsor_frame_hdr)."""
    lib = oracle()
    f = np.asarray(fh, dtype=FH_DTYPE).reshape(1)
    s = None if sll is None else np.asarray(sll, dtype=SLL_DTYPE).reshape(1)
    p = np.frombuffer(bytes(pkt) + b"\0", dtype=np.uint8)
    t = _Text()
    lib.nsor_frame_hdr(f.ctypes.data, None if s is None else s.ctypes.data, p.ctypes.data, len(pkt), linktype,
                       mode, count, ctypes.byref(t))
    out = ctypes.string_at(t.buf, t.len) if t.len else b""
    lib.nsor_text_free(ctypes.byref(t))
    return out


def run_ref(pcap_path, mode=PRINT_NORM, cols=65535, names=False, timeout=120, frames=None):
    """Run oracle/_ref/nsref; returns list of per-packet text (bytes).
    frames="f": `netsniff-ng --in` (frame header line + dissector, read_pcap's
    loop over the reference's pcap reader); "F": frame header lines only."""
    idx = pcap_path + f".m{mode}.idx"
    args = [REF_BIN, "-m", str(mode), "-w", str(cols), "-i", idx]
    if names:
        args.append("-n")
    if frames:
        args.append("-" + frames)
    args.append(pcap_path)
    txt = pcap_path + f".m{mode}.txt"
    with open(txt, "wb") as fo:
        r = subprocess.run(args, stdout=fo, stderr=subprocess.PIPE, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"nsref failed rc={r.returncode}: {r.stderr[:500]!r}")
    ends = np.fromfile(idx, dtype=np.uint64)
    with open(txt, "rb") as fi:
        data = fi.read()
    os.unlink(idx)
    os.unlink(txt)
    out, prev = [], 0
    for e in ends:
        out.append(data[prev:int(e)])
        prev = int(e)
    return out
