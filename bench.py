"""bench.py - device-resident dissection throughput on MI355X.

Workload (BASELINE.json configs[1], "C2"): 16,777,216 synthetic 64 B
Eth/IPv4/UDP frames per GPU, resident in HBM; one step = one pass of the
dissector chain kernel over the batch (records + ext + per-protocol counters)
plus, for N > 1 GPUs, the RCCL all-reduce of the counter vector.
--config imix / ipv6x select C3 / C4 instead.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU, weak scaling: every rank walks its
own 16M-packet shard).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import nsd  # noqa: E402
import nsd_testlib as T  # noqa: E402  (input generators; oracle only in cpu_baseline)

CONFIGS = {
    "udp64": dict(cfg=T.SYN_UDP64, name="C2: 16M x 64 B Eth/IPv4/UDP"),
    "imix": dict(cfg=T.SYN_IMIX, name="C3: 16M IMIX 64/576/1500 Eth/[VLAN]/IPv4/{TCP,UDP,ICMP}"),
    "ipv6x": dict(cfg=T.SYN_IPV6X, name="C4: 16M IPv6 + 0..6 extension headers"),
}
HBM_PEAK_GBS = 8000.0      # MI355X spec (MI355X_MICROARCH.md)
REC_B, DESC_B = 16, 8


def wsum_for(cfg_key, n, lo):
    """Sum of algorithmic read bytes W over the shard (DESIGN.md "Roofline").
    C2: every frame is 64 B, W = caplen.  C3/C4: committed per-config sums
    (tests/golden/wsum.json, made by tests/golden/make_golden.py from the CPU
    restatement) for the standard 16M shard at lo = 0, else None."""
    if cfg_key == "udp64":
        return 64 * n
    path = os.path.join(ROOT, "tests", "golden", "wsum.json")
    if os.path.exists(path):
        with open(path) as f:
            table = json.load(f)
        key = f"{cfg_key}:{lo}:{n}"
        if key in table:
            return int(table[key])
    return None


def cpu_baseline(cfg, n_sample, threads, seconds):
    """CPU restatement (oracle, "port") timed on this host: the fields-only
    walk (records + counters, no text) with `threads` threads, repeated over
    one resident sample of `n_sample` packets until `seconds` have passed.
    Returns (Mpkt/s, packets walked, seconds)."""
    frames, desc = T.make_batch(cfg, n_sample, lo=0, threads=threads)
    lib = T.oracle()
    counters = np.zeros(64, dtype=np.uint64)
    rec = np.zeros(n_sample, dtype=T.REC_DTYPE)
    done, t0 = 0, time.perf_counter()
    while True:
        lib.nsor_dissect_batch_mt(frames.ctypes.data, desc.ctypes.data, n_sample, 1, T.PRINT_NORM,
                                  rec.ctypes.data, counters.ctypes.data, threads)
        done += n_sample
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return done / dt / 1e6, done, dt


def bpf_bench(frames, desc, n, line_bytes, steps, warmup):
    """Device BPF filter (nsd_bpf.hip) over the same resident batch:
    bpfc.8's "Only allow IPv4 TCP packets" program (ldh [12]; jne #0x800;
    ldb [23]; jneq #6; ret #-1; ret #0), verdicts only and with the compaction
    of accepted descriptors.  Algorithmic bytes per packet: 8 (descriptor) +
    the frame's first 64-B line (capped at caplen; the program reads bytes
    12..23) + 4 (verdict); compaction adds 12 B read + 8 B per accepted packet.
    Kernel time by HIP events on torch's current stream (the launch stream)."""
    prog = np.array([(0x28, 0, 0, 12), (0x15, 0, 3, 0x800), (0x30, 0, 0, 23), (0x15, 0, 1, 6),
                     (0x06, 0, 0, 0xFFFFFFFF), (0x06, 0, 0, 0)], dtype=nsd.BPF_INSN)
    bp = nsd.BpfProgram(prog)
    dev = desc.device
    verdict = torch.empty(n, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.empty(nsd.lib().nsd_bpf_workspace_bytes(n), dtype=torch.uint8, device=dev)
    res = {}
    for compact in (False, True):
        for _ in range(max(warmup, 1)):
            bp.filter_device(frames, desc, compact, verdict, out, count, ws)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(steps):
            bp.filter_device(frames, desc, compact, verdict, out, count, ws)
        ev[1].record()
        torch.cuda.synchronize()
        res[compact] = ev[0].elapsed_time(ev[1]) / steps
    kept = int(count.item())
    algo = 8 * n + line_bytes + 4 * n
    gbs = algo / (res[False] * 1e-3) / 1e9
    bp.close()
    return {"program": "bpfc.8 'Only allow IPv4 TCP packets' (6 insns)", "accepted": kept,
            "value": round(n / (res[False] * 1e-3) / 1e6, 1), "unit": "Mpkt/s",
            "kernel_ms": round(res[False], 4), "compact_ms": round(res[True], 4),
            "compact_mpps": round(n / (res[True] * 1e-3) / 1e6, 1),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_pkt": round(algo / n, 2)}}


def end_to_end(cfg, batch, nbatch, depth, mode, reps=3):
    """Host memory in, records in host memory out: `nbatch`
    batches of `batch` packets from one pinned host buffer go through the
    pipelined path (nsd_pipe_*: H2D, dissect kernels, D2H of records, ext and
    counters, `depth` batches in flight).  Returns a dict for the JSON line."""
    L = nsd.lib()
    n = batch * nbatch
    frames, desc = T.make_batch(cfg, n, lo=0, threads=16)
    off = (desc & np.uint64((1 << 40) - 1)).astype(np.int64)
    cap = (desc >> np.uint64(40)).astype(np.int64)
    rec = np.zeros(n, dtype=nsd.REC_DTYPE)
    pinned = [a for a in (frames, rec) if L.nsd_host_register(a.ctypes.data, a.nbytes) == 0]
    slices = []
    for k in range(nbatch):
        a, b = k * batch, (k + 1) * batch
        lo, hi = int(off[a]), int(off[b - 1] + cap[b - 1])
        d = (desc[a:b] - np.uint64(lo)).astype(np.uint64)
        slices.append((frames[lo:hi + nsd.FRAME_PAD], d, rec[a:b]))
    descs_pinned = [L.nsd_host_register(d.ctypes.data, d.nbytes) == 0 for _, d, _ in slices]
    max_bytes = max(f.nbytes for f, _, _ in slices)
    ext_w = nsd.ext_pool_words(batch) if cfg == T.SYN_IPV6X else nsd.ext_pool_words(batch // 64)
    pipe = nsd.Pipe(batch, max_bytes, ext_words=ext_w, depth=depth, mode=mode)
    exts = [np.zeros(ext_w, dtype=np.uint32) for _ in range(depth + 1)]
    cnts = np.zeros((nbatch, nsd.NCOUNTERS), np.uint64)
    ecs = np.zeros(nbatch, np.uint32)
    sts = np.zeros(nbatch, np.int32)
    times = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        for k, (f, d, rr) in enumerate(slices):
            pipe.submit(f, d, rr, exts[k % (depth + 1)], ecs[k:k + 1], cnts[k], sts[k:k + 1])
        assert pipe.drain() == 0
        dt = time.perf_counter() - t0
        if r:
            times.append(dt)
    pipe.close()
    assert int(cnts[:, nsd.CNT_PKTS].sum()) == n and not sts.any()
    h2d = sum(f.nbytes - nsd.FRAME_PAD + d.nbytes for f, d, _ in slices)
    d2h = n * REC_B
    dt = min(times)
    for a in pinned:
        L.nsd_host_unregister(a.ctypes.data)
    for ok, (_, d, _) in zip(descs_pinned, slices):
        if ok:
            L.nsd_host_unregister(d.ctypes.data)
    return {"value": round(n / dt / 1e6, 2), "unit": "Mpkt/s",
            "pcie_gbs": round((h2d + d2h) / dt / 1e9, 2),
            "h2d_bytes_per_pkt": round(h2d / n, 2), "d2h_bytes_per_pkt": REC_B,
            "batches": nbatch, "batch_packets": batch, "depth": depth,
            "pinned": len(pinned) == 2 and all(descs_pinned),
            "note": "host frames -> H2D -> dissect kernels -> D2H records/ext/counters "
                    "(nsd_pipe_*), best of %d passes" % reps}


def replay_leg(cfg, n, mode, threads, reps=2):
    """`netsniff-ng --in file.pcap` through the device (nsd_replay_pcap): a
    synthetic pcap of n records in a temp file -> reader -> pipelined device
    walk -> host formatter on `threads` threads -> /dev/null.  Reported
    beside the device-resident number; never `value`."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "replay.pcap")
        T.synth().nsd_synth_pcap(cfg, T.SEED, 0, n, path.encode())
        size = os.path.getsize(path)
        fd = os.open(os.devnull, os.O_WRONLY)
        try:
            best = None
            for _ in range(reps):
                t0 = time.perf_counter()
                got, _ = nsd.replay_pcap(path, mode=mode, threads=threads, out_fd=fd)
                dt = time.perf_counter() - t0
                assert got == n
                best = dt if best is None else min(best, dt)
        finally:
            os.close(fd)
    return {"value": round(n / best / 1e6, 3), "unit": "Mpkt/s", "packets": n,
            "file_gbs": round(size / best / 1e9, 2), "format_threads": threads,
            "note": "pcap file -> nsd_pcap reader -> H2D -> dissect kernels -> D2H -> host text "
                    "formatter -> /dev/null (nsd_replay_pcap), best of %d" % reps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="udp64", choices=sorted(CONFIGS))
    ap.add_argument("--packets", type=int, default=1 << 24, help="packets per GPU")
    ap.add_argument("--mode", type=int, default=nsd.PRINT_NORM)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1 << 22, help="packets in the CPU sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline duration")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory end-to-end pass")
    ap.add_argument("--no-bpf", action="store_true", help="skip the device BPF filter pass")
    ap.add_argument("--no-replay", action="store_true", help="skip the pcap replay (--in) pass")
    ap.add_argument("--replay-packets", type=int, default=1 << 20)
    ap.add_argument("--e2e-batch", type=int, default=1 << 20)
    ap.add_argument("--e2e-batches", type=int, default=16)
    ap.add_argument("--e2e-depth", type=int, default=3)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    c = CONFIGS[args.config]
    n = args.packets
    lo = rank * n
    frames_np, desc_np = T.make_batch(c["cfg"], n, lo=lo, threads=16)
    frames = torch.from_numpy(frames_np).to(dev)
    desc = torch.from_numpy(desc_np.view(np.int64)).to(dev)
    frame_bytes = int(T.desc_caplen(desc_np).sum())
    line_bytes = int(np.minimum(T.desc_caplen(desc_np), 64).sum())   # first 64-B line per frame
    del frames_np
    ext_w = nsd.ext_pool_words(n) if args.config == "ipv6x" else nsd.ext_pool_words(n // 64)
    rec = torch.empty(n * REC_B, dtype=torch.uint8, device=dev)
    ext = torch.empty(ext_w, dtype=torch.int32, device=dev)
    ext_count = torch.zeros(1, dtype=torch.int32, device=dev)
    counters = torch.zeros(nsd.NCOUNTERS, dtype=torch.int64, device=dev)
    workspace = torch.empty(nsd.lib().nsd_workspace_bytes(n), dtype=torch.uint8, device=dev)

    def step(ev=None):
        ext_count.zero_()
        counters.zero_()
        if ev is not None:
            ev[0].record()
        nsd.dissect_device(frames, desc, mode=args.mode, rec=rec, ext=ext, ext_used=ext_count,
                           counters=counters, grid=args.grid, workspace=workspace)
        if ev is not None:
            ev[1].record()
        if dist is not None:
            dist.all_reduce(counters)   # RCCL over xGMI: per-protocol counters

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    if dist is not None:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    # achievable streaming rate on this device: a 1 GiB
    # device-to-device copy, read + write bytes / time
    cbuf = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    cdst = torch.empty_like(cbuf)
    for _ in range(2):
        cdst.copy_(cbuf)
    ce = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ce[0].record()
    for _ in range(5):
        cdst.copy_(cbuf)
    ce[1].record()
    torch.cuda.synchronize()
    copy_gbs = 2 * cbuf.numel() * 5 / (ce[0].elapsed_time(ce[1]) * 1e-3) / 1e9
    del cbuf, cdst

    bpf = None if args.no_bpf else bpf_bench(frames, desc, n, line_bytes, args.steps, args.warmup)

    cnt = counters.cpu().numpy().view(np.uint64)
    total_pkts = n * world
    # (experiment builds that skip a phase on purpose set NSD_BENCH_NOCHECK)
    assert int(cnt[nsd.CNT_PKTS]) == total_pkts or os.environ.get("NSD_BENCH_NOCHECK"), \
        "counter check failed"
    ms_per_step = elapsed / args.steps * 1e3
    mpps = total_pkts * args.steps / elapsed / 1e6

    wsum = wsum_for(args.config, n, lo)
    roofline = None
    if wsum is not None:
        read_b = DESC_B * n + wsum
        total_b = read_b + REC_B * n
        achieved = total_b / (kern_ms * 1e-3) / 1e9
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": None,
                    "read_frac": round(read_b / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "bytes_per_pkt": {"read": round(read_b / n, 2), "write": REC_B},
                    "kernel_ms": round(kern_ms, 4),
                    "copy_gbs": round(copy_gbs, 1),
                    "frac_of_copy": round(achieved / copy_gbs, 4)}
        prof = os.path.join(ROOT, "profiles", f"pmc_{args.config}.json")
        if os.path.exists(prof):
            with open(prof) as f:
                roofline["traffic"] = json.load(f).get("hbm_bytes_per_launch")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = min(os.cpu_count() or 1, 16)
        v1, p1, d1 = cpu_baseline(c["cfg"], args.cpu_sample // 4, 1, args.cpu_seconds / 2)
        vN, pN, dN = cpu_baseline(c["cfg"], args.cpu_sample, threads, args.cpu_seconds)
        cpu = {"value": round(vN, 3), "unit": "Mpkt/s", "cores": threads, "kind": "port",
               "sample": f"{args.config}: {pN} packets ({pN // args.cpu_sample} passes over a resident"
                         f" {args.cpu_sample}-packet sample) in {dN:.1f} s, fields-only restatement"
                         f" walk (oracle/nsd_oracle.c), {threads} threads; 1 thread:"
                         f" {v1:.3f} Mpkt/s ({p1} packets, {d1:.1f} s)"}

    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        e2e = end_to_end(c["cfg"], args.e2e_batch, args.e2e_batches, args.e2e_depth, args.mode)

    replay = None
    if rank == 0 and world == 1 and not args.no_replay:
        replay = replay_leg(c["cfg"], args.replay_packets, args.mode, min(os.cpu_count() or 1, 16))

    if rank == 0:
        out = {
            "metric": "Mpkt/s + GB/s device-resident dissect, 64B & IMIX; bit-exact fields vs ref",
            "value": round(mpps, 2), "unit": "Mpkt/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded splitmix64 generators, tools/nsd_synth.c)",
            "config": {"workload": c["name"], "packets_per_gpu": n, "frame_bytes_per_gpu": frame_bytes,
                       "mode": ["PRINT_NORM", "PRINT_LESS", "PRINT_HEX", "PRINT_ASCII",
                                "PRINT_HEX_ASCII", "PRINT_NONE"][args.mode],
                       "parallelism": f"dp{world}"},
            "gbps_frames": round(frame_bytes * world * args.steps / elapsed / 1e9, 1),
            "roofline": roofline,
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "replay": replay,
            "bpf_filter": bpf,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
