"""Development check (GPU box): the fused kernel's group tile counters
across plain launches and HIP graph replays."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import nsd  # noqa: E402
import nsd_testlib as T  # noqa: E402

nsd.set_schedule(nsd.SCHED_FUSED)
n = 8192
f, d = T.make_batch(T.SYN_IMIX, n)
dev = torch.device("cuda", 0)
frames = torch.from_numpy(f).to(dev)
desc = torch.from_numpy(d.view(np.int64)).to(dev)
rec = torch.empty(n * nsd.CREC_BYTES, dtype=torch.uint8, device=dev)
ext = torch.empty(nsd.ext_pool_words(n), dtype=torch.int32, device=dev)
used = torch.zeros(1, dtype=torch.int32, device=dev)
cnt = torch.zeros(nsd.NCOUNTERS, dtype=torch.int64, device=dev)
wsb = nsd.lib().nsd_workspace_bytes(n)
ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
# gtiles at sched_pair_at(n) - NSD_MAX_GRID * 128 = wsb - 256 - 4096 * 128
gt_off = wsb - 256 - 4096 * 128


def walk():
    used.zero_()
    cnt.zero_()
    nsd.dissect_device_compact(frames, desc, mode=T.PRINT_NORM, crec=rec, ext=ext, ext_used=used, counters=cnt,
                               workspace=ws)


def show(tag):
    torch.cuda.synchronize()
    g = ws[gt_off:gt_off + 8 * 128].view(torch.int32).cpu().numpy().reshape(8, 32)[:, :2]
    print(tag, "pkts", int(cnt[32].item()), "counters", g.tolist(), flush=True)


for k in range(2):
    walk()
    show(f"plain {k}")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    walk()
torch.cuda.current_stream().wait_stream(s)
show("side")
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    walk()
show("captured")
for k in range(3):
    gr.replay()
    show(f"replay {k}")
