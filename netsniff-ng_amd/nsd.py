"""nsd.py - Python binding of libnsdissect.so (the C ABI in
include/netsniff_dissect.h).  Plumbing only: every dissection runs in the HIP
kernels of the library; there is no Python or CPU fallback.  If the library or
a GPU is missing the calls raise.

Device-resident use (bench / multi-GPU) passes torch tensors; the kernel is
launched on torch's current HIP stream so torch events time it correctly.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libnsdissect.so")

PRINT_NORM, PRINT_LESS, PRINT_HEX, PRINT_ASCII, PRINT_HEX_ASCII, PRINT_NONE = range(6)
LINKTYPE_EN10MB = 1
NCOUNTERS = 64
NSD_OPS_COUNT = 28
CNT_PKTS, CNT_BYTES, CNT_IP_BAD, CNT_ICMP_BAD, CNT_HOST, CNT_EXT, CNT_OVERFLOW, CNT_TRIM = range(32, 40)
CNT_LISTOVF = 40   # pending-list overruns (a broken kernel invariant; never expected)
FRAME_PAD = 64
F_ICMP_BAD, F_HOST, F_OVERFLOW, F_LEAF_END = 0x08, 0x10, 0x20, 0x40

REC_DTYPE = np.dtype([("chain", "<u4"), ("data_off", "<u2"), ("tail_off", "<u2"),
                      ("ip_csum", "<u2"), ("nflags", "u1"), ("off2", "u1", (5,))])
REC_BYTES = 16
# nsd_crec: the compact 8-byte record (chain ids or ext slot, ip_csum, nflags)
CREC_DTYPE = np.dtype([("chain", "<u4"), ("ip_csum", "<u2"), ("nflags", "u1"), ("nlayers", "u1")])
CREC_BYTES = 8

# ext pool (include/netsniff_dissect.h "ext pool"): u32 words; an entry is a
# 4-word header {packet, nlayers, 0, 0} + one word per layer (id | off << 16)
EXT_HDR_WORDS = 4
EXT_MAX_LAYERS = 64

# struct sock_filter (linux/filter.h) = nsd_bpf_insn
BPF_INSN = np.dtype([("code", "<u2"), ("jt", "u1"), ("jf", "u1"), ("k", "<u4")])


def source_hash():
    """First 16 hex digits of the SHA-256 of the library's sources as they lie
    in this tree: the sorted csrc/* files, the Makefile and the ABI header,
    concatenated (the Makefile's SRCHASH, which it compiles into
    nsd_build_info)."""
    import glob
    import hashlib
    csrc = sorted(glob.glob(os.path.join(HERE, "csrc", "*")), key=lambda p: os.path.basename(p).encode())
    files = [p for p in csrc if os.path.isfile(p)] + [os.path.join(HERE, "Makefile"),
                                                      os.path.join(HERE, "..", "include", "netsniff_dissect.h")]
    h = hashlib.sha256()
    for p in files:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def built_source_hash(path=None):
    """The source hash compiled into a built library (read from the file, not
    loaded), or None when it has none or is missing."""
    import re
    try:
        with open(path or LIB_PATH, "rb") as f:
            m = re.search(rb"; sources ([0-9a-f]{16})", f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def ensure_built(jobs=8):
    """Build the library in-tree when it is missing or its embedded source
    hash is not the tree's (make by timestamps first; a full rebuild if the
    hash still differs, e.g. a copied tree with older mtimes)."""
    import subprocess
    want = source_hash()
    if built_source_hash() != want:
        subprocess.run(["make", "-s", f"-j{jobs}", "-C", HERE], check=True)
    if built_source_hash() != want:
        subprocess.run(["make", "-s", "-B", f"-j{jobs}", "-C", HERE], check=True)
    got = built_source_hash()
    if got != want:
        raise RuntimeError(f"libnsdissect.so carries sources {got}, the tree is {want}")
    return got


def ext_words(nlayers):
    """Words one pool entry of a chain of `nlayers` layers occupies (NSD_EXT_WORDS)."""
    return EXT_HDR_WORDS + (16 if nlayers <= 16 else EXT_MAX_LAYERS)


def ext_pool_words(n):
    """NSD_EXT_POOL_WORDS(n): a pool that never overflows for n packets whose
    chains are at most 16 layers, plus room for a few deeper ones."""
    return 48 * n + 4096


def ext_entry(pool, slot):
    """(packet, ids tuple, offsets tuple) of the pool entry at word `slot`."""
    p = np.asarray(pool).view(np.uint32)
    nl = int(p[slot + 1]) & 0xFFFF
    words = p[slot + EXT_HDR_WORDS: slot + EXT_HDR_WORDS + nl]
    return int(p[slot]), tuple(int(x) & 0xFF for x in words), tuple(int(x) >> 16 for x in words)


OPS_NAMES = ["invalid", "ethernet", "vlan", "QinQ", "mpls_uc", "arp", "lldp", "ipv4", "ipv6",
             "ipv6_in_ipv4", "icmpv4", "icmpv6", "igmp", "ip_auth", "ip_esp", "ipv6_dest_opts",
             "ipv6_fragm", "ipv6_hop_by_hop", "ipv6_mobility", "ipv6_no_next_header",
             "ipv6_routing", "tcp", "udp", "dccp", "none", "sll", "ieee80211", "nlmsg"]

# every entry point declared in include/netsniff_dissect.h
ABI_SYMBOLS = ["dissector_init_all", "dissector_entry_point", "dissector_cleanup_all",
               "dissector_set_print_type", "nsd_dissect_device", "dissector_entry_batch",
               "nsd_workspace_bytes", "nsd_dissect_device_ws", "nsd_format_packet", "nsd_lookup_init",
               "nsd_lookup_cleanup", "nsd_tprintf_wrap", "nsd_version", "nsd_device_count",
               "nsd_pipe_create", "nsd_pipe_submit", "nsd_pipe_wait", "nsd_pipe_drain",
               "nsd_pipe_destroy", "nsd_host_alloc", "nsd_host_free", "nsd_host_register",
               "nsd_host_unregister", "nsd_bpf_validate", "nsd_bpf_load", "nsd_bpf_free",
               "nsd_bpf_workspace_bytes", "nsd_bpf_filter_device", "nsd_bpf_filter_batch",
               "nsd_pcap_open", "nsd_pcap_linktype", "nsd_pcap_read_batch", "nsd_pcap_close",
               "nsd_replay_pcap", "nsd_t3_block_desc", "nsd_dissect_device_sll",
               "dissector_entry_batch_sll", "nsd_format_packet_sll", "nsd_format_batch_sll",
               "nsd_pipe_submit_sll", "nsd_pcap_read_batch_sll", "nsd_t3_block_desc_sll",
               "nsd_replay_pcap_out", "nsd_build_info", "nsd_walk_packet_cpu", "nsd_set_etcdir",
               "nsd_dissect_device_compact", "nsd_format_batch_compact", "nsd_pipe_create_compact",
               "nsd_pipe_submit_compact", "nsd_format_range_compact", "nsd_set_schedule",
               "nsd_last_schedule", "nsd_format_frame_hdr", "nsd_format_range_compact_fh",
               "nsd_pcap_read_batch_fh", "nsd_t3_block_desc_fh", "nsd_pcap_index", "nsd_set_grid_cap",
               "nsd_set_record_ring"]

# struct sockaddr_ll (nsd_sll_t), one per packet for LINKTYPE_LINUX_SLL batches
SLL_DTYPE = np.dtype([("family", "<u2"), ("protocol", ">u2"), ("ifindex", "<i4"), ("hatype", "<u2"),
                      ("pkttype", "u1"), ("halen", "u1"), ("addr", "u1", (8,))])
LINKTYPE_LINUX_SLL = 113
LINKTYPE_NETLINK = 253

# nsd_frame_hdr_t: the tpacket header fields show_frame_hdr prints
FH_DTYPE = np.dtype([("len", "<u4"), ("sec", "<u4"), ("nsec", "<u4"), ("status", "<u4"), ("vlan_tci", "<u4"),
                     ("vlan_tpid", "<u2"), ("v3", "u1"), ("reserved", "u1")])

_lib = None
_vp, _u32, _u64, _int, _sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t


def lib():
    """Load libnsdissect.so (raises OSError if it is not built)."""
    global _lib
    if _lib is None:
        # torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's):
        # whichever is loaded first serves the whole process, so let torch's
        # runtime load first when torch is installed
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built (run make -C netsniff-ng_amd)")
        L = ctypes.CDLL(LIB_PATH)
        L.nsd_dissect_device.restype = _int
        L.nsd_dissect_device.argtypes = [_vp, _vp, _u32, _int, _int, _vp, _vp, _u32, _vp, _vp, _vp]
        L.nsd_dissect_device_grid.restype = _int
        L.nsd_dissect_device_grid.argtypes = [_vp, _vp, _u32, _int, _int, _vp, _vp, _u32, _vp, _vp,
                                              _vp, _int, _vp]
        L.nsd_dissect_device_ws.restype = _int
        L.nsd_dissect_device_ws.argtypes = [_vp, _vp, _u32, _int, _int, _vp, _vp, _u32, _vp, _vp,
                                            _vp, _vp]
        L.nsd_workspace_bytes.restype = _sz
        L.nsd_workspace_bytes.argtypes = [_u32]
        L.dissector_entry_batch.restype = _int
        L.dissector_entry_batch.argtypes = [_vp, _sz, _vp, _u32, _int, _int, _vp, _vp, _u32, _vp, _vp]
        L.nsd_format_packet.restype = ctypes.c_long
        L.nsd_format_packet.argtypes = [_vp, _u32, _int, _int, _vp, _vp, ctypes.c_char_p, _sz]
        L.nsd_format_batch.restype = ctypes.c_long
        L.nsd_format_batch.argtypes = [_vp, _vp, _u32, _int, _int, _vp, _vp, _vp, _sz, _vp, _vp]
        L.nsd_lookup_init.restype = _int
        L.nsd_lookup_init.argtypes = [ctypes.c_char_p]
        L.nsd_lookup_cleanup.restype = None
        L.nsd_tprintf_wrap.restype = ctypes.c_long
        L.nsd_tprintf_wrap.argtypes = [ctypes.c_char_p, _sz, _int, ctypes.POINTER(ctypes.c_long),
                                       ctypes.c_char_p, _sz]
        L.nsd_version.restype = ctypes.c_char_p
        L.nsd_build_info.restype = ctypes.c_char_p
        L.nsd_device_count.restype = _int
        L.nsd_pipe_create.restype = _vp
        L.nsd_pipe_create.argtypes = [_u32, _sz, _u32, _int, _int, _int]
        L.nsd_pipe_submit.restype = _int
        L.nsd_pipe_submit.argtypes = [_vp, _vp, _sz, _vp, _u32, _vp, _vp, _vp, _vp, _vp]
        L.nsd_pipe_wait.restype = _int
        L.nsd_pipe_wait.argtypes = [_vp]
        L.nsd_pipe_drain.restype = _int
        L.nsd_pipe_drain.argtypes = [_vp]
        L.nsd_pipe_destroy.restype = None
        L.nsd_pipe_destroy.argtypes = [_vp]
        L.nsd_host_alloc.restype = _vp
        L.nsd_host_alloc.argtypes = [_sz]
        L.nsd_host_free.restype = None
        L.nsd_host_free.argtypes = [_vp]
        L.nsd_host_register.restype = _int
        L.nsd_host_register.argtypes = [_vp, _sz]
        L.nsd_host_unregister.restype = _int
        L.nsd_host_unregister.argtypes = [_vp]
        L.dissector_init_all.argtypes = [_int]
        L.dissector_entry_point.argtypes = [_vp, _sz, _int, _int, _vp]
        L.nsd_bpf_validate.restype = _int
        L.nsd_bpf_validate.argtypes = [_vp, _u32]
        L.nsd_bpf_load.restype = _vp
        L.nsd_bpf_load.argtypes = [_vp, _u32]
        L.nsd_bpf_free.restype = None
        L.nsd_bpf_free.argtypes = [_vp]
        L.nsd_bpf_workspace_bytes.restype = _sz
        L.nsd_bpf_workspace_bytes.argtypes = [_u32]
        L.nsd_bpf_filter_device.restype = _int
        L.nsd_bpf_filter_device.argtypes = [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp]
        L.nsd_bpf_filter_batch.restype = _int
        L.nsd_bpf_filter_batch.argtypes = [_vp, _vp, _sz, _vp, _u32, _vp]
        L.nsd_pcap_open.restype = _vp
        L.nsd_pcap_open.argtypes = [ctypes.c_char_p]
        L.nsd_pcap_linktype.restype = _int
        L.nsd_pcap_linktype.argtypes = [_vp]
        L.nsd_pcap_read_batch.restype = ctypes.c_long
        L.nsd_pcap_read_batch.argtypes = [_vp, _vp, _sz, _vp, _u32, _vp, _vp]
        L.nsd_pcap_close.restype = None
        L.nsd_pcap_close.argtypes = [_vp]
        L.dissector_entry_batch_sll.restype = _int
        L.dissector_entry_batch_sll.argtypes = [_vp, _sz, _vp, _vp, _u32, _int, _int, _vp, _vp, _u32, _vp, _vp]
        L.nsd_dissect_device_sll.restype = _int
        L.nsd_dissect_device_sll.argtypes = [_vp, _vp, _vp, _u32, _int, _int, _vp, _vp, _u32, _vp, _vp,
                                             _vp, _vp]
        L.nsd_format_packet_sll.restype = ctypes.c_long
        L.nsd_format_packet_sll.argtypes = [_vp, _u32, _int, _int, _vp, _vp, _vp, ctypes.c_char_p, _sz]
        L.nsd_format_batch_sll.restype = ctypes.c_long
        L.nsd_format_batch_sll.argtypes = [_vp, _vp, _vp, _u32, _int, _int, _vp, _vp, _vp, _sz, _vp, _vp]
        L.nsd_t3_block_desc.restype = ctypes.c_long
        L.nsd_t3_block_desc.argtypes = [_vp, _sz, _int, _int, _vp, _u32]
        L.nsd_replay_pcap_out.restype = ctypes.c_long
        L.nsd_replay_pcap_out.argtypes = [ctypes.c_char_p, _int, _vp, _int, _int, _vp, _int, _int]
        L.nsd_t3_block_desc_sll.restype = ctypes.c_long
        L.nsd_t3_block_desc_sll.argtypes = [_vp, _sz, _int, _int, _vp, _vp, _u32]
        L.nsd_pcap_read_batch_sll.restype = ctypes.c_long
        L.nsd_pcap_read_batch_sll.argtypes = [_vp, _vp, _sz, _vp, _vp, _u32, _vp, _vp]
        L.nsd_pipe_submit_sll.restype = _int
        L.nsd_pipe_submit_sll.argtypes = [_vp, _vp, _sz, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp]
        L.nsd_walk_packet_cpu.restype = _int
        L.nsd_walk_packet_cpu.argtypes = [_vp, _u32, _int, _int, _vp, _vp, _vp, _u32, _vp]
        L.nsd_set_etcdir.restype = None
        L.nsd_set_etcdir.argtypes = [ctypes.c_char_p]
        L.nsd_dissect_device_compact.restype = _int
        L.nsd_dissect_device_compact.argtypes = [_vp, _vp, _vp, _u32, _int, _int, _vp, _vp, _u32, _vp, _vp,
                                                 _vp, _vp]
        L.nsd_format_batch_compact.restype = ctypes.c_long
        L.nsd_format_batch_compact.argtypes = [_vp, _vp, _vp, _u32, _int, _int, _vp, _vp, _vp, _sz, _vp, _vp]
        # (entries newer than a dev tool's variant library may lack: bound when
        # present, tests/test_abi.py checks the product library has them all)
        for name, res, args in (
                ("nsd_pipe_create_compact", _vp, [_u32, _sz, _u32, _int, _int, _int]),
                ("nsd_pipe_submit_compact", _int, [_vp, _vp, _sz, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp]),
                ("nsd_format_range_compact", ctypes.c_long,
                 [_vp, _vp, _vp, _u32, _u32, _int, _int, _vp, _vp, _vp, _sz, _vp, _vp]),
                ("nsd_set_schedule", _int, [_int]),
                ("nsd_format_frame_hdr", ctypes.c_long, [_vp, _vp, _vp, _u32, _int, _int, _u64, ctypes.c_char_p, _sz]),
                ("nsd_format_range_compact_fh", ctypes.c_long,
                 [_vp, _vp, _vp, _vp, _u64, _u32, _u32, _int, _int, _vp, _vp, _vp, _sz, _vp, _vp]),
                ("nsd_pcap_read_batch_fh", ctypes.c_long, [_vp, _vp, _sz, _vp, _vp, _vp, _u32]),
                ("nsd_t3_block_desc_fh", ctypes.c_long, [_vp, _sz, _int, _int, _vp, _vp, _vp, _u32]),
                ("nsd_pcap_index", ctypes.c_long, [ctypes.c_char_p, _u64, _int, _vp, _vp, _sz]),
                ("nsd_last_schedule", _int, [])):
            if hasattr(L, name):
                getattr(L, name).restype = res
                getattr(L, name).argtypes = args
        L.nsd_replay_pcap.restype = ctypes.c_long
        L.nsd_replay_pcap.argtypes = [ctypes.c_char_p, _int, _vp, _int, _int, _vp, _int]
        _lib = L
    return _lib


SCHED_ADAPTIVE, SCHED_SPLIT, SCHED_FUSED = 0, 1, 2
SCHED_NAMES = {0: None, 1: "split", 2: "fused"}


def set_schedule(sched):
    """Force the batch walks' kernel schedule (SCHED_SPLIT / SCHED_FUSED) or
    let the library pick it (SCHED_ADAPTIVE, the default); returns the
    previous setting."""
    if not hasattr(lib(), "nsd_set_schedule"):
        return 0   # (a dev tool's variant library from before schedules)
    rc = lib().nsd_set_schedule(sched)
    if rc < 0:
        raise ValueError(f"bad schedule {sched}")
    return rc


RING_ADAPTIVE, RING_ON, RING_OFF = 0, 1, 2


def set_record_ring(mode):
    """The fused kernel's record ring: RING_ADAPTIVE (default), RING_ON or
    RING_OFF; returns the previous setting (nsd_set_record_ring, tests)."""
    rc = lib().nsd_set_record_ring(mode)
    if rc < 0:
        raise ValueError(f"bad record ring mode {mode}")
    return rc


def set_grid_cap(blocks):
    """Cap every batch walk's grid at `blocks` blocks (0: none); returns the
    previous cap (nsd_set_grid_cap, tests)."""
    rc = lib().nsd_set_grid_cap(blocks)
    if rc < 0:
        raise ValueError(f"bad grid cap {blocks}")
    return rc


def last_schedule():
    """"split" / "fused": the schedule of the last launch (None before any,
    or from a library without schedules)."""
    return SCHED_NAMES.get(lib().nsd_last_schedule()) if hasattr(lib(), "nsd_last_schedule") else None


class NsdError(RuntimeError):
    pass


def _check(rc, what):
    if rc != 0:
        raise NsdError(f"{what} failed with status {rc}")


def dissect_device(frames, desc, mode=PRINT_NORM, linktype=LINKTYPE_EN10MB, rec=None, ext=None,
                   ext_used=None, counters=None, grid=0, stream=None, workspace=None):
    """Walk a device-resident batch.  frames: uint8 cuda tensor (padded by
    FRAME_PAD bytes), desc: int64/uint64 cuda tensor (packed descriptors).
    Returns (rec u8[n*16], ext i32[words] (the pool), ext_used i32[1] (pool
    words handed out), counters i64[64]) as cuda tensors; counters and
    ext_used accumulate if passed in."""
    import torch
    n = desc.numel()
    dev = desc.device
    if rec is None:
        rec = torch.empty(n * REC_BYTES, dtype=torch.uint8, device=dev)
    if ext is None:
        ext = torch.empty(ext_pool_words(n), dtype=torch.int32, device=dev)
    if ext_used is None:
        ext_used = torch.zeros(1, dtype=torch.int32, device=dev)
    if counters is None:
        counters = torch.zeros(NCOUNTERS, dtype=torch.int64, device=dev)
    assert ext.element_size() == 4, "the ext pool is u32 words"
    words = ext.numel()
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    L = lib()
    if workspace is None:
        workspace = torch.empty(L.nsd_workspace_bytes(n), dtype=torch.uint8, device=dev)
    if grid:
        rc = L.nsd_dissect_device_grid(frames.data_ptr(), desc.data_ptr(), n, linktype, mode,
                                       rec.data_ptr(), ext.data_ptr(), words, ext_used.data_ptr(),
                                       counters.data_ptr(), workspace.data_ptr(), grid, stream)
    else:
        rc = L.nsd_dissect_device_ws(frames.data_ptr(), desc.data_ptr(), n, linktype, mode,
                                     rec.data_ptr(), ext.data_ptr(), words, ext_used.data_ptr(),
                                     counters.data_ptr(), workspace.data_ptr(), stream)
    _check(rc, "nsd_dissect_device")
    return rec, ext, ext_used, counters


def dissect_device_compact(frames, desc, mode=PRINT_NORM, linktype=LINKTYPE_EN10MB, crec=None, ext=None,
                           ext_used=None, counters=None, stream=None, workspace=None, sll=None):
    """dissect_device writing compact 8-byte records (nsd_crec).  Returns
    (crec u8[n*8], ext, ext_used, counters) as cuda tensors."""
    import torch
    n = desc.numel()
    dev = desc.device
    if crec is None:
        crec = torch.empty(n * CREC_BYTES, dtype=torch.uint8, device=dev)
    if ext is None:
        ext = torch.empty(ext_pool_words(n), dtype=torch.int32, device=dev)
    if ext_used is None:
        ext_used = torch.zeros(1, dtype=torch.int32, device=dev)
    if counters is None:
        counters = torch.zeros(NCOUNTERS, dtype=torch.int64, device=dev)
    assert ext.element_size() == 4, "the ext pool is u32 words"
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    L = lib()
    if workspace is None:
        workspace = torch.empty(L.nsd_workspace_bytes(n), dtype=torch.uint8, device=dev)
    rc = L.nsd_dissect_device_compact(frames.data_ptr(), desc.data_ptr(),
                                      None if sll is None else sll.data_ptr(), n, linktype, mode,
                                      crec.data_ptr(), ext.data_ptr(), ext.numel(), ext_used.data_ptr(),
                                      counters.data_ptr(), workspace.data_ptr(), stream)
    _check(rc, "nsd_dissect_device_compact")
    return crec, ext, ext_used, counters


def compact_of(rec, ext=None):
    """(crec, pool): the compact records (CREC_DTYPE) and their ext pool that
    carry what 16-byte records `rec` with pool `ext` do, minus the cursors
    (include/netsniff_dissect.h "compact records"): ids inline up to 6
    layers, 7..12 layers with ids 6.. in the packet's side word (pool word
    i), longer chains as entries (their slots moved past the n side words)."""
    n = len(rec)
    out = np.zeros(n, dtype=CREC_DTYPE)
    side = np.zeros(n, dtype=np.uint32)
    src = np.zeros(0, dtype=np.uint32) if ext is None else np.asarray(ext).view(np.uint32)
    src = src.copy()
    out["chain"] = rec["chain"]
    out["ip_csum"] = rec["ip_csum"]
    out["nflags"] = rec["nflags"]
    # a host-rendered leaf (NSD_F_HOST) keeps its end (data_off) in the side
    # word of an inline chain, or in word 2 of an entry (NSD_F_LEAF_END)
    host = ((rec["nflags"] & F_HOST) != 0) & ((rec["nflags"] & F_OVERFLOW) == 0)
    inline = host & ((rec["nflags"] & 7) != 7)
    side[inline] = rec["data_off"][inline]
    out["nflags"][inline] |= F_LEAF_END
    slots = rec["off2"][:, :4].copy().view("<u4").reshape(-1)
    for i in np.nonzero((rec["nflags"] & 7) == 7)[0]:
        s, flags = int(slots[i]), int(rec[i]["nflags"]) & 0xF8
        if s == 0xFFFFFFFF:                  # no entry: pool full
            out[i]["chain"] = s
            continue
        _, ids, _ = ext_entry(src, s)
        if len(ids) > 12:
            out[i]["chain"] = s + n
            if host[i]:
                src[s + 2] = rec[i]["data_off"]
                out[i]["nflags"] |= F_LEAF_END
            continue
        out[i]["chain"] = sum(ids[k] << (5 * k) for k in range(min(len(ids), 6)))
        if len(ids) <= 6:                    # ext form only for an offset past 510
            out[i]["nflags"] = len(ids) | flags | (F_LEAF_END if host[i] else 0)
            if host[i]:
                side[i] = rec[i]["data_off"]
        else:
            out[i]["nlayers"] = len(ids)
            side[i] = sum(ids[k] << (5 * (k - 6)) for k in range(6, len(ids)))
    return out, np.concatenate([side, src])


def entry_batch(frames, desc, mode=PRINT_NORM, linktype=LINKTYPE_EN10MB, ext_words=None, sll=None):
    """Host-memory batch through the device (H2D, kernel, D2H).
    Returns (rec, ext pool words[:used], counters) as numpy arrays."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    desc = np.ascontiguousarray(desc, dtype=np.uint64)
    n = len(desc)
    if ext_words is None:
        ext_words = ext_pool_words(n)
    rec = np.zeros(n, dtype=REC_DTYPE)
    ext = np.zeros(max(ext_words, 1), dtype=np.uint32)
    used = np.zeros(1, dtype=np.uint32)
    counters = np.zeros(NCOUNTERS, dtype=np.uint64)
    sll = None if sll is None else np.ascontiguousarray(sll, dtype=SLL_DTYPE)
    rc = lib().dissector_entry_batch_sll(frames.ctypes.data, frames.nbytes, desc.ctypes.data,
                                         None if sll is None else sll.ctypes.data, n,
                                         linktype, mode, rec.ctypes.data, ext.ctypes.data, ext_words,
                                         used.ctypes.data, counters.ctypes.data)
    _check(rc, "dissector_entry_batch")
    return rec, ext[:min(int(used[0]), ext_words)], counters


def walk_cpu(frames, desc, mode=PRINT_NORM, linktype=LINKTYPE_EN10MB, sll=None):
    """The per-packet entry point's walk (host CPU, nsd_walk_packet_cpu) over
    every packet of a host batch: (records, {packet: (ids, offs)} of the ext
    chains, counters).  The batch path is nsd_dissect_device / entry_batch."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    desc = np.ascontiguousarray(desc, dtype=np.uint64)
    sll = None if sll is None else np.ascontiguousarray(sll, dtype=SLL_DTYPE)
    n = len(desc)
    rec = np.zeros(n, dtype=REC_DTYPE)
    cnt = np.zeros(NCOUNTERS, dtype=np.uint64)
    ext = np.zeros(ext_words(EXT_MAX_LAYERS), dtype=np.uint32)
    chains = {}
    L = lib()
    base = frames.ctypes.data
    for i in range(n):
        d = int(desc[i])
        off, cl = d & 0xFFFFFFFFFF, d >> 40
        r = rec[i:i + 1]
        rc = L.nsd_walk_packet_cpu(base + off, cl, linktype, mode,
                                   None if sll is None else sll[i:i + 1].ctypes.data,
                                   r.ctypes.data, ext.ctypes.data, len(ext), cnt.ctypes.data)
        _check(rc, "nsd_walk_packet_cpu")
        if (int(r[0]["nflags"]) & 7) == 7 and not (int(r[0]["nflags"]) & 0x20):
            _, ids, offs = ext_entry(ext, 0)
            chains[i] = (ids, offs)
    return rec, chains, cnt


class Pipe:
    """Pipelined host-batch path (nsd_pipe_*): submit numpy batches, records
    land in the caller's arrays when the batch completes.  Arrays passed to
    submit() are kept alive until then."""

    def __init__(self, max_pkts, max_frame_bytes, ext_words=0, depth=3, mode=PRINT_NORM,
                 linktype=LINKTYPE_EN10MB, compact=False):
        """compact: records are nsd_crec (CREC_DTYPE) and the pool holds the
        side words first (nsd_pipe_create_compact: ext_words >= max_pkts)."""
        self.L = lib()
        create = self.L.nsd_pipe_create_compact if compact else self.L.nsd_pipe_create
        self.p = create(max_pkts, max_frame_bytes, ext_words, depth, linktype, mode)
        if not self.p:
            raise NsdError("nsd_pipe_create failed")
        self.compact = compact
        self.ext_words = ext_words
        self.depth = depth
        self.inflight = []

    def submit(self, frames, desc, rec, ext=None, ext_used=None, counters=None, status=None, sll=None):
        """ext: u32[ext_words] receiving the pool, ext_used: u32[1]; sll: one
        SLL_DTYPE sockaddr_ll per packet (SLL link types) or None."""
        n = len(desc)
        ptr = lambda a: None if a is None else a.ctypes.data  # noqa: E731
        if ext is not None:
            assert ext.dtype == np.uint32 and len(ext) >= self.ext_words
        if sll is not None:
            sll = np.ascontiguousarray(sll, dtype=SLL_DTYPE)
            assert len(sll) == n
        submit = self.L.nsd_pipe_submit_compact if self.compact else self.L.nsd_pipe_submit_sll
        assert rec.dtype == (CREC_DTYPE if self.compact else REC_DTYPE)
        rc = submit(self.p, frames.ctypes.data, frames.nbytes, desc.ctypes.data, ptr(sll), n, rec.ctypes.data,
                    ptr(ext), ptr(ext_used), ptr(counters), ptr(status))
        _check(rc, "nsd_pipe_submit")
        self.inflight.append((frames, desc, rec, ext, ext_used, counters, status, sll))
        if len(self.inflight) > self.depth:   # the library completed the oldest first
            self.inflight.pop(0)

    def wait(self):
        rc = self.L.nsd_pipe_wait(self.p)
        if self.inflight:
            self.inflight.pop(0)
        return rc

    def drain(self):
        rc = self.L.nsd_pipe_drain(self.p)
        self.inflight.clear()
        return rc

    def close(self):
        if self.p:
            self.L.nsd_pipe_destroy(self.p)
            self.p = None

    def __del__(self):
        self.close()


def format_batch(frames, desc, rec, ext=None, mode=PRINT_NORM, linktype=LINKTYPE_EN10MB, sll=None):
    """Render records to the reference text (ext: the u32 pool the records'
    slots index).  Returns (list of bytes per packet, status array)."""
    n = len(desc)
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    desc = np.ascontiguousarray(desc, dtype=np.uint64)
    rec = np.ascontiguousarray(rec)
    ext_keep = None if ext is None or len(ext) == 0 else np.ascontiguousarray(ext).view(np.uint32)
    ext_ptr = None if ext_keep is None else ext_keep.ctypes.data
    ends = np.zeros(n, dtype=np.uint64)
    rc = np.zeros(n, dtype=np.int8)
    cap = int(frames.nbytes) * 7 + 1024 * n + 4096
    out = ctypes.create_string_buffer(cap)
    sll = None if sll is None else np.ascontiguousarray(sll, dtype=SLL_DTYPE)
    total = lib().nsd_format_batch_sll(frames.ctypes.data, desc.ctypes.data,
                                       None if sll is None else sll.ctypes.data, n, linktype, mode,
                                       rec.ctypes.data, ext_ptr, ctypes.addressof(out), cap,
                                       ends.ctypes.data, rc.ctypes.data)
    if total < 0:
        raise NsdError("format buffer too small")
    raw = out.raw[:total]
    texts, prev = [], 0
    for e in ends:
        texts.append(raw[prev:int(e)])
        prev = int(e)
    return texts, rc


def format_batch_compact(frames, desc, crec, ext=None, mode=PRINT_NORM, linktype=LINKTYPE_EN10MB, sll=None):
    """format_batch over compact records (CREC_DTYPE)."""
    n = len(desc)
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    desc = np.ascontiguousarray(desc, dtype=np.uint64)
    crec = np.ascontiguousarray(crec, dtype=CREC_DTYPE)
    ext_keep = None if ext is None or len(ext) == 0 else np.ascontiguousarray(ext).view(np.uint32)
    ends = np.zeros(n, dtype=np.uint64)
    rc = np.zeros(n, dtype=np.int8)
    cap = int(frames.nbytes) * 7 + 1024 * n + 4096
    out = ctypes.create_string_buffer(cap)
    sll = None if sll is None else np.ascontiguousarray(sll, dtype=SLL_DTYPE)
    total = lib().nsd_format_batch_compact(frames.ctypes.data, desc.ctypes.data,
                                           None if sll is None else sll.ctypes.data, n, linktype, mode,
                                           crec.ctypes.data, None if ext_keep is None else ext_keep.ctypes.data,
                                           ctypes.addressof(out), cap, ends.ctypes.data, rc.ctypes.data)
    if total < 0:
        raise NsdError("format buffer too small")
    raw = out.raw[:total]
    texts, prev = [], 0
    for e in ends:
        texts.append(raw[prev:int(e)])
        prev = int(e)
    return texts, rc


def tprintf_wrap(text, cols=80, state=0):
    """Apply the reference tprintf wrap (tprintf.c:65-103) to one flushed
    buffer; returns (bytes, new_state)."""
    st = ctypes.c_long(state)
    cap = 2 * len(text) + 16
    out = ctypes.create_string_buffer(cap)
    k = lib().nsd_tprintf_wrap(text, len(text), cols, ctypes.byref(st), out, cap)
    if k < 0:
        raise NsdError("wrap failed")
    return out.raw[:k], st.value


def lookup_init(directory):
    return lib().nsd_lookup_init(directory.encode() if directory else None)


def lookup_cleanup():
    lib().nsd_lookup_cleanup()


def unpack_counters(counters):
    c = np.asarray(counters, dtype=np.uint64)
    out = {OPS_NAMES[i]: int(c[i]) for i in range(1, NSD_OPS_COUNT) if c[i]}
    for name, k in [("pkts", CNT_PKTS), ("bytes", CNT_BYTES), ("ip_bad", CNT_IP_BAD),
                    ("icmp_bad", CNT_ICMP_BAD), ("host", CNT_HOST), ("ext", CNT_EXT),
                    ("overflow", CNT_OVERFLOW), ("trim", CNT_TRIM)]:
        out[name] = int(c[k])
    if c[CNT_LISTOVF]:
        out["list_overrun"] = int(c[CNT_LISTOVF])
    return out


# ---- classic BPF (nsd_bpf_*: the capture loop's filter step) -------------------------
def bpf_validate(prog):
    """__bpf_validate (bpf.c:388-506) through the product library: 1 / 0."""
    p = np.ascontiguousarray(prog, dtype=BPF_INSN)
    return lib().nsd_bpf_validate(p.ctypes.data if len(p) else None, len(p))


class BpfProgram:
    """A classic-BPF program validated, decoded and loaded on the device
    (nsd_bpf_load); raises NsdError for an invalid program or without a GPU."""

    def __init__(self, prog):
        self.L = lib()
        p = np.ascontiguousarray(prog, dtype=BPF_INSN)
        self.h = self.L.nsd_bpf_load(p.ctypes.data if len(p) else None, len(p))
        if not self.h:
            raise NsdError("nsd_bpf_load refused the program (invalid program or no GPU)")
        self.len = len(p)

    def filter_batch(self, frames, desc):
        """Host-memory batch -> u32 verdict per packet (0 = drop)."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=np.uint64)
        v = np.zeros(len(desc), dtype=np.uint32)
        rc = self.L.nsd_bpf_filter_batch(self.h, frames.ctypes.data, frames.nbytes, desc.ctypes.data,
                                         len(desc), v.ctypes.data)
        _check(rc, "nsd_bpf_filter_batch")
        return v

    def filter_device(self, frames, desc, compact=False, verdict=None, out=None, count=None,
                      workspace=None, stream=None):
        """Device-resident batch on torch's current stream.  Returns
        (verdict i32[n], accepted descriptors i64[n] or None, count i32[1] or
        None); with compact=True the accepted packets' descriptors are packed
        in batch order into out[:count]."""
        import torch
        n = desc.numel()
        dev = desc.device
        if verdict is None:
            verdict = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        if compact:
            if out is None:
                out = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
            if count is None:
                count = torch.zeros(1, dtype=torch.int32, device=dev)
            if workspace is None:
                workspace = torch.empty(self.L.nsd_bpf_workspace_bytes(n), dtype=torch.uint8, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        rc = self.L.nsd_bpf_filter_device(self.h, frames.data_ptr(), desc.data_ptr(), n, verdict.data_ptr(),
                                          out.data_ptr() if compact else None,
                                          count.data_ptr() if compact else None,
                                          workspace.data_ptr() if compact else None, stream)
        _check(rc, "nsd_bpf_filter_device")
        return verdict[:n], out, count

    def close(self):
        if getattr(self, "h", None):
            self.L.nsd_bpf_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


# ---- pcap replay front end (nsd_pcap.cpp) ---------------------------------------
def pcap_read(path, cap=64 << 20, max_n=1 << 16, sll=False):
    """Read a whole pcap through nsd_pcap_read_batch_sll: (linktype, [batches]),
    each batch = (frames uint8, desc uint64, wire_len uint32, ts_ns uint64)
    [+ one SLL_DTYPE sockaddr_ll per record when sll=True]."""
    L = lib()
    h = L.nsd_pcap_open(os.fsencode(path))
    if not h:
        raise NsdError(f"nsd_pcap_open({path}) failed")
    try:
        lt = L.nsd_pcap_linktype(h)
        out = []
        while True:
            frames = np.zeros(cap, dtype=np.uint8)
            desc = np.zeros(max_n, dtype=np.uint64)
            wl = np.zeros(max_n, dtype=np.uint32)
            ts = np.zeros(max_n, dtype=np.uint64)
            ll = np.zeros(max_n, dtype=SLL_DTYPE)
            n = L.nsd_pcap_read_batch_sll(h, frames.ctypes.data, cap, desc.ctypes.data,
                                          ll.ctypes.data if sll else None, max_n,
                                          wl.ctypes.data, ts.ctypes.data)
            if n < 0:
                raise NsdError(f"nsd_pcap_read_batch failed with status {n}")
            if n == 0:
                return lt, out
            out.append((frames, desc[:n], wl[:n], ts[:n]) + ((ll[:n],) if sll else ()))
    finally:
        L.nsd_pcap_close(h)


def pcap_frame_hdrs(path, cap=64 << 20, max_n=1 << 16):
    """Every record's frame header fields and sockaddr_ll as read_pcap holds
    them (nsd_pcap_read_batch_fh): (linktype, packets [bytes], fh FH_DTYPE,
    sll SLL_DTYPE)."""
    L = lib()
    h = L.nsd_pcap_open(os.fsencode(path))
    if not h:
        raise NsdError(f"nsd_pcap_open({path}) failed")
    try:
        lt = L.nsd_pcap_linktype(h)
        pkts, fhs, slls = [], [], []
        while True:
            frames = np.zeros(cap, dtype=np.uint8)
            desc = np.zeros(max_n, dtype=np.uint64)
            fh = np.zeros(max_n, dtype=FH_DTYPE)
            ll = np.zeros(max_n, dtype=SLL_DTYPE)
            n = L.nsd_pcap_read_batch_fh(h, frames.ctypes.data, cap, desc.ctypes.data, ll.ctypes.data,
                                         fh.ctypes.data, max_n)
            if n < 0:
                raise NsdError(f"nsd_pcap_read_batch_fh failed with status {n}")
            if n == 0:
                break
            for d in desc[:n]:
                d = int(d)
                pkts.append(bytes(frames[d & 0xFFFFFFFFFF:(d & 0xFFFFFFFFFF) + (d >> 40)]))
            fhs.append(fh[:n].copy())
            slls.append(ll[:n].copy())
        fh = np.concatenate(fhs) if fhs else np.zeros(0, dtype=FH_DTYPE)
        ll = np.concatenate(slls).astype(SLL_DTYPE) if slls else np.zeros(0, dtype=SLL_DTYPE)
        return lt, pkts, fh, ll
    finally:
        L.nsd_pcap_close(h)


def pcap_index(path, window=0, chunks=1):
    """The replay reader's record index of a mapped pcap file
    (nsd_pcap_index): (header offsets uint64, caplens uint32), windows of
    `window` bytes (0: the replay's) cut into `chunks` walked from guesses."""
    L = lib()
    n = L.nsd_pcap_index(os.fsencode(path), window, chunks, None, None, 0)
    if n < 0:
        raise NsdError(f"nsd_pcap_index({path}) failed with status {n}")
    off = np.zeros(max(n, 1), dtype=np.uint64)
    cap = np.zeros(max(n, 1), dtype=np.uint32)
    m = L.nsd_pcap_index(os.fsencode(path), window, chunks, off.ctypes.data, cap.ctypes.data, n)
    if m != n:
        raise NsdError(f"nsd_pcap_index({path}): {m} records, then {n}")
    return off[:n], cap[:n]


def format_frame_hdr(fh, pkt=b"", sll=None, linktype=LINKTYPE_EN10MB, mode=PRINT_NORM, count=1):
    """show_frame_hdr's line for one packet (nsd_format_frame_hdr)."""
    L = lib()
    f = np.asarray(fh, dtype=FH_DTYPE).reshape(1)
    s = None if sll is None else np.asarray(sll, dtype=SLL_DTYPE).reshape(1)
    p = np.frombuffer(bytes(pkt) + b"\0", dtype=np.uint8)
    buf = ctypes.create_string_buffer(512)
    n = L.nsd_format_frame_hdr(f.ctypes.data, None if s is None else s.ctypes.data, p.ctypes.data, len(pkt),
                               linktype, mode, count, buf, 512)
    _check(0 if n >= 0 else n, "nsd_format_frame_hdr")
    return buf.raw[:n]


def replay_pcap(path, mode=PRINT_NORM, prog=None, cols=0, counters=None, threads=0, out_fd=None,
                pcap_out=None):
    """`netsniff-ng --in path` through the device: returns (records printed,
    text bytes), or (records printed, None) when writing to out_fd.  Each
    packet's text is its frame header line (show_frame_hdr) followed by the
    dissector's.
    prog: a BpfProgram (or None).  pcap_out: path of the `--out f.pcap`
    write-out (nsd_replay_pcap_out), or None."""
    import tempfile
    L = lib()
    cnt = counters if counters is not None else np.zeros(NCOUNTERS, dtype=np.uint64)
    h = prog.h if prog is not None else None
    pfd = os.open(pcap_out, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644) if pcap_out else -1
    try:
        if out_fd is not None:
            n = L.nsd_replay_pcap_out(os.fsencode(path), mode, h, out_fd, cols, cnt.ctypes.data, threads, pfd)
            _check(0 if n >= 0 else n, "nsd_replay_pcap_out")
            return n, None
        with tempfile.TemporaryFile() as f:
            n = L.nsd_replay_pcap_out(os.fsencode(path), mode, h, f.fileno(), cols, cnt.ctypes.data, threads,
                                      pfd)
            if n < 0:
                raise NsdError(f"nsd_replay_pcap_out failed with status {n}")
            f.seek(0)
            return n, f.read()
    finally:
        if pfd >= 0:
            os.close(pfd)


def t3_block_desc(block, packet_type=-1, lo_ifindex=-1, max_n=1 << 16, sll=False, fh=False):
    """Descriptors of a TPACKET_V3 block's frames (nsd_t3_block_desc_fh);
    with sll=True also each kept frame's sockaddr_ll, with fh=True its frame
    header fields: desc, or a tuple (desc[, sll][, fh])."""
    block = np.ascontiguousarray(block, dtype=np.uint8)
    desc = np.zeros(max_n, dtype=np.uint64)
    ll = np.zeros(max_n, dtype=SLL_DTYPE)
    f = np.zeros(max_n, dtype=FH_DTYPE)
    n = lib().nsd_t3_block_desc_fh(block.ctypes.data, block.nbytes, packet_type, lo_ifindex,
                                   desc.ctypes.data, ll.ctypes.data if sll else None,
                                   f.ctypes.data if fh else None, max_n)
    _check(0 if n >= 0 else n, "nsd_t3_block_desc_fh")
    out = (desc[:n],) + ((ll[:n],) if sll else ()) + ((f[:n],) if fh else ())
    return out if len(out) > 1 else out[0]
