"""step_cost.py - what one general-walk layer step costs (the walker pool's
gen_step iteration), measured: two synthetic batches of
Ethernet / IPv6 / K Hop-by-Hop headers (8 bytes each) / UDP, K = K1 and K2,
walked by the fused kernel.  The fast walk takes Ethernet, IPv6 and the
first Hop-by-Hop header (its 64-byte window), the walkers the other K - 1
and UDP, so the two batches differ by exactly K2 - K1 walker steps per
packet, in the same session structure.  The difference of their per-launch
instruction counts (rocprofv3 --pmc SQ_INSTS_*: wave instructions) and
kernel times, per 64-packet tile and step, is the cost of one step with
every lane of the wave stepping the same kind of header.
Development tool (GPU box):
  python tools/step_cost.py [--packets N] [--k1 4 --k2 9]  (7 and 12 layers: both past 6, side words either way)
"""
import argparse
import csv
import glob
import json
import os
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
CTRS = "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"


def frame(k):
    eth = bytes.fromhex("0a0b0c0d0e0f020304050607") + b"\x86\xdd"
    udp = struct.pack(">HHHH", 1000, 2000, 12, 0) + b"abcd"
    hbh = b"".join(bytes([0 if j + 1 < k else 17, 0, 1, 4, 0, 0, 0, 0]) for j in range(k))
    pl = hbh + udp
    ip6 = bytes([0x60, 0, 0, 0]) + struct.pack(">HBB", len(pl), 0, 64) + bytes(range(32))
    return eth + ip6 + pl


def batch(k, n):
    import numpy as np
    import nsd_testlib as T
    f = frame(k)
    return T.batch_from_packets([f] * n)


def child(args):
    import numpy as np
    import torch
    import nsd
    if args.lib:
        nsd.LIB_PATH = os.path.abspath(args.lib)
    torch.cuda.set_device(0)
    nsd.set_schedule(nsd.SCHED_FUSED)
    for k in (args.k1, args.k2):
        frames, desc = batch(k, args.packets)
        f = torch.from_numpy(frames).cuda()
        d = torch.from_numpy(desc.view(np.int64)).cuda()
        crec = torch.empty(args.packets * nsd.CREC_BYTES, dtype=torch.uint8, device="cuda")
        ext = torch.empty(nsd.ext_pool_words(args.packets) + args.packets, dtype=torch.int32, device="cuda")
        used = torch.zeros(1, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(nsd.NCOUNTERS, dtype=torch.int64, device="cuda")
        ws = torch.empty(nsd.lib().nsd_workspace_bytes(args.packets), dtype=torch.uint8, device="cuda")
        times = []
        for r in range(args.reps + 2):
            used.zero_()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            nsd.dissect_device_compact(f, d, crec=crec, ext=ext, ext_used=used, counters=cnt, workspace=ws)
            ev[1].record()
            torch.cuda.synchronize()
            if r >= 2:
                times.append(ev[0].elapsed_time(ev[1]))
        c = cnt.cpu().numpy().view(np.uint64)
        layers = int(sum(int(c[j]) for j in range(1, nsd.NSD_OPS_COUNT)))
        print(json.dumps({"k": k, "ms": sorted(times)[len(times) // 2], "layers_per_pkt": layers / args.packets /
                          (args.reps + 2)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 22)
    ap.add_argument("--k1", type=int, default=4)
    ap.add_argument("--k2", type=int, default=9)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--lib", default=None, help="a variant libnsdissect.so (tools/build_variant.sh)")
    args = ap.parse_args()
    if args.child:
        child(args)
        return
    base = [sys.executable, os.path.abspath(__file__), "--child", "--packets", str(args.packets), "--k1",
            str(args.k1), "--k2", str(args.k2), "--reps", str(args.reps)] + \
        (["--lib", os.path.abspath(args.lib)] if args.lib else [])
    r = subprocess.run(base, stdout=subprocess.PIPE, text=True, check=True)
    timing = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc"] + CTRS.split() + \
              ["--kernel-trace", "-d", d, "-o", "run", "--output-format", "csv", "--"] + base
        subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL, check=True)
        rows = []
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for j, row in enumerate(csv.DictReader(open(fn))):
                if "dissect_all" in row["Kernel_Name"]:
                    rows.append((int(row.get("Dispatch_Id") or j), row["Counter_Name"], float(row["Counter_Value"])))
    per = {}
    for disp, name, v in rows:
        per.setdefault(disp, {})[name] = per.get(disp, {}).get(name, 0.0) + v
    disps = sorted(per)
    n = args.reps + 2
    assert len(disps) == 2 * n, (len(disps), n)
    out = {"packets": args.packets, "timing": timing}
    avg = []
    for i in range(2):
        ds = disps[i * n + 2:(i + 1) * n]
        avg.append({c: sum(per[x].get(c, 0.0) for x in ds) / len(ds) for c in CTRS.split()})
    tiles = args.packets / 64
    steps = args.k2 - args.k1
    out["per_tile_step"] = {c: round((avg[1][c] - avg[0][c]) / tiles / steps, 2) for c in CTRS.split()
                            if c != "SQ_WAVES"}
    out["counts"] = avg
    out["ms_per_tile_step_ns"] = round((timing[1]["ms"] - timing[0]["ms"]) * 1e6 / tiles / steps, 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
