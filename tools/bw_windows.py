"""bw_windows.py - the fast walk's access shape alone over a bench batch
(tools/bw/nsd_bw.hip k_windows: every packet's first 64 bytes, descriptors;
nothing computed), by blocks per CU and load form: the ceiling of a tile
phase on that layout.  Development tool (GPU box).

  python tools/bw_windows.py --configs udp64,imix,ipv6x
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="udp64,imix,ipv6x")
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    import bench
    L = ctypes.CDLL(bench.BW_SO)
    L.nsd_bw_windows.restype = ctypes.c_int
    L.nsd_bw_windows.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    for key in args.configs.split(","):
        b = bench.Batch(key, args.packets, 0, 1, dev, compact=True)
        n = b.n
        for bpc in (2, 3, 4, 6, 8):
            for nt in (1, 0):
                def go():
                    assert L.nsd_bw_windows(b.frames.data_ptr(), b.desc.data_ptr(), n, bpc, nt, stream,
                                            sink.data_ptr()) == 0
                go()
                go()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                for _ in range(args.reps):
                    go()
                ev[1].record()
                torch.cuda.synchronize()
                ms = ev[0].elapsed_time(ev[1]) / args.reps
                print(f"{key:6s} windows bpc={bpc} nt={nt} ms={ms:.4f}", flush=True)
        b.free()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
