"""kbench.py - development timing of the dissect kernel alone: K launches over
one resident synthetic batch per config, kernel ms from HIP events (no
result checks: experiment variants that skip a phase run through it too).
Not the benchmark (bench.py is).

  python tools/kbench.py --configs udp64,imix,ipv6x --steps 10 [--lib path]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="udp64,imix,ipv6x")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--records", default="both", choices=["compact", "full", "both"])
    ap.add_argument("--sched", default="adaptive", choices=["adaptive", "split", "fused"],
                    help="kernel schedule (nsd_set_schedule)")
    ap.add_argument("--bpf", action="store_true", help="also time the device BPF filter (bench.bpf_bench: "
                    "verdicts, and with the compaction, whose accepted count it checks)")
    ap.add_argument("--lib", default=None, help="a variant libnsdissect.so (tools/build_variant.sh) "
                    "loaded instead of the in-tree one (dev tools only; the product loads its own)")
    args = ap.parse_args()
    import nsd
    if args.lib:
        nsd.LIB_PATH = os.path.abspath(args.lib)
    print(f"library {os.path.relpath(nsd.LIB_PATH, ROOT)} schedule {args.sched}", flush=True)
    nsd.set_schedule({"adaptive": nsd.SCHED_ADAPTIVE, "split": nsd.SCHED_SPLIT, "fused": nsd.SCHED_FUSED}[args.sched])
    import bench
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    forms = {"compact": [True], "full": [False], "both": [False, True]}[args.records]
    for key in args.configs.split(","):
        for compact in forms:
            b = bench.Batch(key, args.packets, 0, 1, dev, compact=compact)
            if args.bpf:
                r = bench.bpf_bench(b, args.steps, args.warmup)
                print(f"{key:6s} bpf kernel_ms={r['kernel_ms']:.4f} compact_ms={r['compact_ms']:.4f} "
                      f"frac={r['roofline']['frac']} accepted={r['accepted']}", flush=True)
            ms = bench.time_steps(b, args.mode, args.steps, args.warmup, 0 if compact else args.grid)
            cnt = b.counters.cpu().numpy().view(np.uint64)
            r = b.roofline(ms)
            print(f"{key:6s} rec{b.rec_b:<2d} {nsd.last_schedule()} kernel_ms={ms:.4f} frac={r['frac'] if r else None} "
                  f"read_frac={r['read_frac'] if r else None} pkts_counted={int(cnt[32])}", flush=True)
            if os.environ.get("KB_ENDS"):
                # counters 56..61 of an instrumented variant (a timeline patch):
                # ~min / max of block start, wave tile-phase end, block end
                # (s_memrealtime, 100 MHz), one more launch with zeroed counters
                b.counters.zero_()
                b.step(args.mode, 0 if compact else args.grid, zero=False)
                b.sync()
                c = b.counters.cpu().numpy().view(np.uint64)
                inv = lambda x: int(~np.uint64(x))   # noqa: E731
                t0 = inv(c[56])
                us = lambda t: round((t - t0) / 100.0, 1)   # noqa: E731
                print(f"{key:6s} timeline_us start {us(t0)}..{us(int(c[57]))} tiles_end {us(inv(c[58]))}.."
                      f"{us(int(c[59]))} block_end {us(inv(c[60]))}..{us(int(c[61]))}", flush=True)
                if os.environ.get("KB_ENDS") == "xcd":
                    print(f"{key:6s} per-group (block * 4 / grid: dispatch round) last tile-phase end {[us(int(x)) for x in c[40:48]]} "
                          f"last block end {[us(int(x)) for x in c[48:56]]}", flush=True)
            if os.environ.get("KB_DBG"):
                # a variant with per-wave start / tile-phase end times (g_dbg,
                # nsd_dbg_read): one more launch, then the spread within and
                # across blocks
                import ctypes
                b.step(args.mode, 0 if compact else args.grid, zero=False)
                b.sync()
                buf = np.zeros(3 * 16384, dtype=np.uint64)
                assert nsd.lib().nsd_dbg_read(ctypes.c_void_p(buf.ctypes.data)) == 0
                st, en = buf[:16384].astype(np.int64), buf[16384:32768].astype(np.int64)
                nw = int(np.count_nonzero(st))
                st, en = st[:nw], en[:nw]
                t = (en - st.min()) / 100.0
                blk = t.reshape(-1, 4)
                print(f"{key:6s} waves {nw}: tile-phase end us p0 {t.min():.1f} p10 {np.percentile(t, 10):.1f} "
                      f"p50 {np.median(t):.1f} p90 {np.percentile(t, 90):.1f} p100 {t.max():.1f}; within-block "
                      f"spread mean {np.mean(blk.max(1) - blk.min(1)):.1f}, block means' spread "
                      f"{blk.mean(1).max() - blk.mean(1).min():.1f}; wave-in-block means "
                      f"{[round(float(x), 1) for x in blk.mean(0)]}", flush=True)
                np.save(os.path.join(ROOT, "gpurun_out", "var", f"dbg_{key}.npy"), buf)
            if os.environ.get("KB_PHASES"):
                # counters 48..55 of an instrumented variant (tools/variants/phases.patch),
                # summed over waves, last launch: fast-walk part, walker engine, window
                # staging, layer steps, emit (cycles), sessions, step iterations, take (cycles)
                print(f"{key:6s} phases {[int(x) for x in cnt[48:56]]}", flush=True)
            b.free()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
