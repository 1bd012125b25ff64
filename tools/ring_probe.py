"""ring_probe.py - how often the fused kernel's record ring hands a slot to a
new tile while walkers still hold packets of its old tile (the eviction path
of ring_turn), on C4, long extension chains and the edge set, at the default
grid and at grids of 3 and 8 blocks.  Needs a variant library counting them
into counters 41 (evictions) and 42 (packets still held), e.g.
tools/build_variant.sh with a patch adding those counts; parity of the path
itself is the GPU suite's (schedule fixture "fused": ring on).  Dev tool.

  python tools/ring_probe.py --lib variants/evict/libnsdissect.so"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    args = ap.parse_args()
    import nsd
    nsd.LIB_PATH = os.path.abspath(args.lib)
    import nsd_testlib as T
    import test_device_parity as P
    nsd.set_schedule(nsd.SCHED_FUSED)
    nsd.set_record_ring(nsd.RING_ON)
    torch.cuda.set_device(0)
    cases = [("ipv6x 1M", *T.make_batch(T.SYN_IPV6X, 1 << 20)),
             ("long chains", *T.batch_from_packets(P._long_chains(30000), align=2))]
    for name, frames, desc in cases:
        want = T.oracle_records(frames, desc)
        wc, wpool = nsd.compact_of(want[0], want[1])
        for grid in (0, 3, 8):
            nsd.set_grid_cap(grid)
            f = torch.from_numpy(frames).cuda()
            d = torch.from_numpy(desc.view(np.int64)).cuda()
            crec, ext, used, cnt = nsd.dissect_device_compact(f, d)
            torch.cuda.synchronize()
            c = cnt.cpu().numpy().view(np.uint64)
            got = crec.cpu().numpy().view(nsd.CREC_DTYPE)
            # (chains past 12 layers carry pool slots, which differ in order)
            m = ((wc["nflags"] & 7) != 7) | (wc["nlayers"] != 0)
            same = bool(np.array_equal(got[m], wc[m]))
            print(f"{name:12s} grid {grid}: evictions {int(c[41])} packets held {int(c[42])} "
                  f"records equal the oracle's {same}", flush=True)
    nsd.set_grid_cap(0)


if __name__ == "__main__":
    main()
