"""bw_msgs.py - the ICMPv4 checksum pass's access shape alone over the C3
(IMIX) bench batch (tools/bw/nsd_bw.hip k_msgs): the batch's pending
messages (ICMPv4 messages running past the 64-byte window, as the fused
kernel lists them), read and summed with nothing else, by variant (lanes
per message, loads in flight per lane, line-aligned groups, two groups in
flight) and list order ("kernel": the fused kernel's per-wave lists of its
grid-stride tiles; "sorted": each wave a contiguous slice of the batch).
Development tool (GPU box).

  python tools/bw_msgs.py [--packets N]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def pending(frames, desc):
    """(packet index, message byte offset, message length) of every ICMPv4
    message past its packet's 64-byte window (PRINT_NORM, 16-byte aligned
    frames; proto_icmpv4.c:42 after the IPv4 trim)."""
    import torch
    off = desc & ((1 << 40) - 1)
    cap = desc >> 40
    f = frames
    b = lambda k: f[off + k].to(torch.int64)   # noqa: E731
    vlan = (b(12) == 0x81) & (b(13) == 0)
    v = vlan.to(torch.int64) * 4
    proto = f[off + 23 + v].to(torch.int64)
    tot = f[off + 16 + v].to(torch.int64) * 256 + f[off + 17 + v].to(torch.int64)
    d2 = 34 + v
    x = tot - 20
    tail = torch.where((x >= 0) & (x < cap - d2), d2 + x, cap)
    ln = tail - d2
    m = off & 15
    pend = (proto == 1) & (ln >= 8) & (m + d2 + (ln & ~1) > 64)
    idx = torch.nonzero(pend).flatten()
    return idx, (off + d2)[idx], (ln & ~1)[idx]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    import bench
    L = ctypes.CDLL(bench.BW_SO)
    L.nsd_bw_msgs.restype = ctypes.c_int
    L.nsd_bw_msgs.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                      ctypes.c_void_p]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    b = bench.Batch("imix", args.packets, 0, 1, dev, compact=True)
    idx, moff, mlen = pending(b.frames, b.desc)
    npend = int(idx.numel())
    lines = int((((moff + mlen + 127) // 128) - (moff // 128)).sum().item())
    print(f"imix {b.n} packets: {npend} pending messages ({npend / b.n:.4f}), {int(mlen.sum())} message bytes "
          f"({int(mlen.sum()) / b.n:.1f} B/pkt), {lines * 128 / b.n:.1f} line B/pkt", flush=True)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    nl = cus * 4 * 4   # the fused kernel's waves: CUs x 4 blocks x 4 waves
    ent = moff | (mlen << 48)
    orders = {}
    # kernel order: wave w lists the tiles t = w, w + nl, ... (grid-stride), packets ascending
    w = (idx // 64) % nl
    key = w * (1 << 40) + idx
    srt = torch.argsort(key)
    cnt = torch.bincount(w, minlength=nl)
    orders["kernel"] = (ent[srt], cnt)
    # sorted: contiguous slices of the batch's pending list
    ws = torch.arange(npend, device=dev) * nl // npend
    orders["sorted"] = (ent, torch.bincount(ws, minlength=nl))
    variants = []
    for lanes, u in ((8, 12), (8, 8), (8, 6), (16, 6), (16, 8), (4, 12)):
        for al in (0, 1):
            for pi in (0, 1):
                for o4 in (1, 0):
                    variants.append((lanes, u, al, pi, o4))
    for oname, (e, c) in orders.items():
        e = e.contiguous()
        c32 = c.to(torch.int32)
        loff = (torch.cumsum(c, 0) - c).to(torch.int32)
        for (lanes, u, al, pi, o4) in variants:
            var = al | pi << 1 | o4 << 2 | lanes << 8 | u << 16
            for nt in (0,):
                def go():
                    rc = L.nsd_bw_msgs(b.frames.data_ptr(), e.data_ptr(), loff.data_ptr(), c32.data_ptr(), nl, var,
                                       nt, stream, sink.data_ptr())
                    assert rc == 0, rc
                go()
                go()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                for _ in range(args.reps):
                    go()
                ev[1].record()
                torch.cuda.synchronize()
                ms = ev[0].elapsed_time(ev[1]) / args.reps
                print(f"{oname:6s} lanes={lanes:2d} U={u:2d} align={al} pipe={pi} occ4={o4} ms={ms:.4f} "
                      f"line_TBps={lines * 128 / ms / 1e9:.2f}", flush=True)


if __name__ == "__main__":
    main()
