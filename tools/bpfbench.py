"""bpfbench.py - development timing of the device BPF filter alone (bench.py's
bpf_bench over one resident batch per config, verdicts and the compacted
form), optionally from a variant library.  Not the benchmark.

  python tools/bpfbench.py --configs udp64,imix [--lib variants/x/libnsdissect.so]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="udp64,imix")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--lib", default=None)
    args = ap.parse_args()
    import torch
    import nsd
    if args.lib:
        nsd.LIB_PATH = os.path.abspath(args.lib)
    import bench
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    print(f"library {os.path.relpath(nsd.LIB_PATH, ROOT)}", flush=True)
    for key in args.configs.split(","):
        b = bench.Batch(key, args.packets, 0, 1, dev, compact=True)
        r = bench.bpf_bench(b, args.steps, args.warmup)
        print(f"{key:6s} bpf kernel_ms={r['kernel_ms']:.4f} compact_ms={r['compact_ms']:.4f} "
              f"accepted={r['accepted']} frac={r['roofline']['frac']}", flush=True)
        b.free()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
