"""replay_scale.py - `netsniff-ng --in` replay rate (nsd_replay_pcap, frame
headers + dissector text to /dev/null) by formatter threads and file size,
with the replay's stage times (NSD_REPLAY_STATS) on stderr.  Development
tool (GPU box), not the benchmark.

  python tools/replay_scale.py --packets 1048576,4194304 --threads 1,2,4,8,16
"""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", default="1048576")
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--cfg", type=int, default=1)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--lib", default="", help="a variant libnsdissect.so")
    args = ap.parse_args()
    os.environ["NSD_REPLAY_STATS"] = "1"
    import nsd
    if args.lib:
        nsd.LIB_PATH = os.path.abspath(args.lib)
    import nsd_testlib as T
    fd = os.open(os.devnull, os.O_WRONLY)
    with tempfile.TemporaryDirectory() as d:
        for n in [int(x) for x in args.packets.split(",")]:
            path = os.path.join(d, f"r{n}.pcap")
            T.synth().nsd_synth_pcap(args.cfg, T.SEED, 0, n, path.encode())
            for th in [int(x) for x in args.threads.split(",")]:
                best = None
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    got, _ = nsd.replay_pcap(path, mode=0, threads=th, out_fd=fd)
                    dt = time.perf_counter() - t0
                    assert got == n
                    best = dt if best is None else min(best, dt)
                print(f"packets {n} threads {th} {n / best / 1e6:.3f} Mpkt/s", flush=True)
    os.close(fd)


if __name__ == "__main__":
    main()
