"""bench.py - device-resident dissection throughput on MI355X.

Workload (BASELINE.json configs[1], "C2"): 16,777,216 synthetic 64 B
Eth/IPv4/UDP frames per GPU, resident in HBM; one step = one pass of the
dissector chain kernel over the batch (records + ext + per-protocol counters)
plus, for N > 1 GPUs, the RCCL all-reduce of the counter vector.  Records
are the compact 8-byte form by default (nsd_crec: ops ids, IPv4 checksum,
flags; the renderer re-derives the cursors), --records full
times the 16-byte nsd_rec; the other form is measured beside it
("other_records").
--config imix / ipv6x select C3 / C4 as the headline instead; --shards S
walks S contiguous 16M shards of the same stream as one batch on one GPU
(--config imix --shards 8 = C5's 128M packets on a single MI355X).

At every N (rank r walks its own 16M-packet shard [r * 16M, (r + 1) * 16M)
of each config; the counter vector is all-reduced over the ranks inside the
timed region and checked against the oracle's per-shard counters,
tests/golden/shard_counters.json):
  headline    C2 (or --config), `value` = whole-job Mpkt/s, per-GPU roofline;
  legs        C3 IMIX (the metric is "64B & IMIX"; at N = 8 its shards are
              C5's 128M IMIX packets across 8 GPUs) and C4, each with its
              whole-job rate, per-GPU kernel time and roofline.
Beside them, at N = 1 only:
  traffic     HBM bytes per launch from rocprofv3 PMC counters, collected
              in-run by two child processes (FETCH_SIZE and WRITE_SIZE in
              separate passes, MI355X_MICROARCH.md "HBM") before this
              process touches the GPU;
  other_records the other record form over the headline workload;
  cpu_baseline the CPU restatement (oracle, "port") on this host's cores:
              fields + text (what the reference does: it prints as it
              parses) and fields only, 1 thread and all threads; and the
              reference's own objects (oracle/_ref/nsref) on one core and
              as one process per core of the 16-CPU share, C2 and C3;
  end_to_end / replay / bpf_filter (reported, never `value`).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU, weak scaling: every rank walks its
own 16M-packet shard).  Rank 0 prints one JSON line.
"""
import argparse
import ctypes
import csv
import glob
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import nsd  # noqa: E402
import nsd_dist  # noqa: E402
import nsd_testlib as T  # noqa: E402  (input generators; oracle only in cpu_baseline)

CONFIGS = {
    "udp64": dict(cfg=T.SYN_UDP64, name="C2: 16M x 64 B Eth/IPv4/UDP"),
    "imix": dict(cfg=T.SYN_IMIX, name="C3: 16M IMIX 64/576/1500 Eth/[VLAN]/IPv4/{TCP,UDP,ICMP}"),
    "ipv6x": dict(cfg=T.SYN_IPV6X, name="C4: 16M IPv6 + 0..6 extension headers"),
}
LEGS = ("imix", "ipv6x")
HBM_PEAK_GBS = 8000.0      # MI355X spec (MI355X_MICROARCH.md)
REC_B, DESC_B = 16, 8          # record bytes of the 16-byte form, descriptor bytes
CREC_B = 8                     # compact record (nsd_crec)
MODES = ["PRINT_NORM", "PRINT_LESS", "PRINT_HEX", "PRINT_ASCII", "PRINT_HEX_ASCII", "PRINT_NONE"]


def workload_name(key, n, shards):
    if shards > 1:
        return (f"C5 on one GPU: {shards} x {n // (1 << 20)}M-packet IMIX shards ({shards * n} packets)"
                if key == "imix" else f"{CONFIGS[key]['name']} x {shards} shards")
    return CONFIGS[key]["name"]


def wsum_for(key, n, lo, shards=1):
    """Sum of algorithmic read bytes W over [lo, lo + shards*n) (DESIGN.md
    "Roofline").  C2: every frame is 64 B, W = caplen.  C3/C4: committed
    per-shard sums (tests/golden/wsum.json, made by make_golden.py from the
    CPU restatement; shard keys lo:n), else None."""
    if key == "udp64":
        return 64 * n * shards
    path = os.path.join(ROOT, "tests", "golden", "wsum.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        table = json.load(f)
    total = 0
    for r in range(shards):
        k = f"{key}:{lo + r * n}:{n}"
        if k not in table:
            return None
        total += int(table[k])
    return total


def lines_for(key, n, lo, shards=1):
    """The line floor of [lo, lo + shards*n): distinct 128-byte lines holding
    the bytes the chains must inspect (tests/golden/lines.json, made by
    make_golden.py --lines-only from the CPU restatement), else None."""
    path = os.path.join(ROOT, "tests", "golden", "lines.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        table = json.load(f)
    total = 0
    for r in range(shards):
        k = f"{key}:{lo + r * n}:{n}"
        if k not in table:
            return None
        total += int(table[k])
    return total


def library_info():
    """The benched library: its file hash, the source hash compiled into it
    (the Makefile's SRCHASH over csrc/*, the Makefile and the ABI header) and
    the same hash over this tree's sources, so the line names the code that
    produced the binary it timed."""
    L = nsd.lib()
    with open(nsd.LIB_PATH, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    built, tree = nsd.built_source_hash(), nsd.source_hash()
    return {"path": os.path.relpath(nsd.LIB_PATH, ROOT), "sha256_16": sha,
            "source_sha256_16": built, "tree_source_sha256_16": tree, "source_matches_tree": built == tree,
            "version": L.nsd_version().decode(), "build": L.nsd_build_info().decode()}


# ---- device batches --------------------------------------------------------------
class Batch:
    """A config's packets resident in HBM plus the output buffers of one walk."""

    def __init__(self, key, n, lo, shards, dev, compact=True):
        self.key, self.n_shard, self.shards = key, n, shards
        self.compact = compact
        self.rec_b = CREC_B if compact else REC_B
        self.n = n * shards
        cfg = CONFIGS[key]["cfg"]
        # (4M-packet host chunks: at 8 ranks a 16M C4 chunk each would hold
        # 8 x 13 GB of host memory at once)
        self.frames, self.desc, desc_np = T.make_device_batch(cfg, self.n, lo=lo, device=dev, chunk=1 << 22)
        caps = T.desc_caplen(desc_np)
        self.frame_bytes = int(caps.sum())
        self.line_bytes = int(np.minimum(caps, 64).sum())   # first 64-B line per frame (BPF leg)
        del desc_np
        ext_w = nsd.ext_pool_words(self.n) if key == "ipv6x" else nsd.ext_pool_words(self.n // 64)
        if compact:
            ext_w += self.n   # the side words (compact records of 7..12 layers)
        self.rec = torch.empty(self.n * self.rec_b, dtype=torch.uint8, device=dev)
        self.ext = torch.empty(ext_w, dtype=torch.int32, device=dev)
        self.ext_used = torch.zeros(1, dtype=torch.int32, device=dev)
        self.counters = torch.zeros(nsd.NCOUNTERS, dtype=torch.int64, device=dev)
        self.ws = torch.empty(nsd.lib().nsd_workspace_bytes(self.n), dtype=torch.uint8, device=dev)
        self.wsum = wsum_for(key, n, lo, shards)
        self.lines = lines_for(key, n, lo, shards)

    def step(self, mode, grid=0, ev=None, zero=True):
        if zero:
            self.ext_used.zero_()
            self.counters.zero_()
        if ev is not None:
            ev[0].record()
        if self.compact:
            assert not grid, "--grid applies to the 16-byte record kernels"
            nsd.dissect_device_compact(self.frames, self.desc, mode=mode, crec=self.rec, ext=self.ext,
                                       ext_used=self.ext_used, counters=self.counters, workspace=self.ws)
        else:
            nsd.dissect_device(self.frames, self.desc, mode=mode, rec=self.rec, ext=self.ext,
                               ext_used=self.ext_used, counters=self.counters, grid=grid, workspace=self.ws)
        if ev is not None:
            ev[1].record()

    def roofline(self, kern_ms, traffic=None, copy_gbs=None, ceiling=None):
        if self.wsum is None:
            return None
        read_b = DESC_B * self.n + self.wsum
        total_b = read_b + self.rec_b * self.n
        achieved = total_b / (kern_ms * 1e-3) / 1e9
        r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(achieved / HBM_PEAK_GBS, 4),
             "traffic": None if traffic is None else round(traffic["bytes_per_launch"]),
             "read_frac": round(read_b / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
             "bytes_per_pkt": {"read": round(read_b / self.n, 2), "write": self.rec_b},
             "kernel_ms": round(kern_ms, 4)}
        if traffic is not None:
            r["traffic_bytes_per_pkt"] = {"read": round(traffic["read_bytes"] / self.n, 1),
                                          "write": round(traffic["write_bytes"] / self.n, 1)}
        if self.lines is not None:
            # the least any schedule reading whole 128-byte lines can fetch:
            # each needed line once, plus the descriptors
            floor = 128 * self.lines + DESC_B * self.n
            r["line_floor_bytes_per_pkt"] = {"read": round(floor / self.n, 2),
                                             "source": "tests/golden/lines.json (nsor_line_floor_mt)"}
            if traffic is not None:
                r["traffic_vs_line_floor"] = {"read": round(traffic["read_bytes"] / floor, 3),
                                              "write": round(traffic["write_bytes"] / (self.rec_b * self.n), 3)}
        if copy_gbs:
            r["copy_gbs"] = round(copy_gbs, 1)
            r["frac_of_copy"] = round(achieved / copy_gbs, 4)
        if ceiling:
            # the achievable read rate measured in this run (read_ceiling)
            r["read_ceiling_gbs"] = ceiling["gbs"]
            r["read_frac_of_ceiling"] = round(read_b / (kern_ms * 1e-3) / 1e9 / ceiling["gbs"], 4)
            r["frac_of_ceiling"] = round(achieved / ceiling["gbs"], 4)
        return r

    def free(self):
        for a in ("frames", "desc", "rec", "ext", "ext_used", "counters", "ws"):
            setattr(self, a, None)

    @staticmethod
    def event():
        return torch.cuda.Event(enable_timing=True)

    @staticmethod
    def sync():
        torch.cuda.synchronize()


class HostEvent:
    """torch.cuda.Event's timing interface on the host clock."""

    def __init__(self):
        self.t = None

    def record(self):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class HostBatch:
    """The rank body's batch for the CPU tests (tests/test_multi.py, gloo):
    the same packets a GPU rank would hold, walked by the product's host
    walk (nsd.walk_cpu -> nsd_walk_packet_cpu, the layer step the per-packet
    dissector_entry_point runs) instead of the kernel, so measure_rank()'s
    sharding, timing and counter reduce run unchanged without a GPU.  Never
    used by a bench run."""

    def __init__(self, key, n, lo, shards, compact=True):
        self.key, self.n_shard, self.shards, self.compact = key, n, shards, compact
        self.rec_b = CREC_B if compact else REC_B
        self.n = n * shards
        self.frames, self.desc = T.make_batch(CONFIGS[key]["cfg"], self.n, lo=lo)
        self.frame_bytes = int(T.desc_caplen(self.desc).sum())
        self.counters = torch.zeros(nsd.NCOUNTERS, dtype=torch.int64)
        self.ext_used = torch.zeros(1, dtype=torch.int32)
        self.wsum = None

    def step(self, mode, grid=0, ev=None, zero=True):
        if zero:
            self.counters.zero_()
        if ev is not None:
            ev[0].record()
        _, _, cnt = nsd.walk_cpu(self.frames, self.desc, mode=mode)
        self.counters += torch.from_numpy(cnt.view(np.int64))
        if ev is not None:
            ev[1].record()

    def roofline(self, *a, **k):
        return None

    def free(self):
        self.frames = self.desc = None

    @staticmethod
    def event():
        return HostEvent()

    @staticmethod
    def sync():
        pass


WARM_SECONDS = 0.25


def warm(b, mode, warmup, grid=0, seconds=WARM_SECONDS, reduce=None):
    """The untimed warmup: launches for `seconds`, then `warmup` launches,
    so the timed region starts at the GPU's steady clocks (3 launches of
    0.25 ms leave it ramping: C2 measured 0.262 ms after them, 0.249 after
    0.25 s of launches, on one box).  `reduce` (the multi-GPU counter
    all-reduce) follows each of the `warmup` launches only: the timed part
    of the warmup runs a different number of launches on each rank, so it
    holds no collective."""
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        b.step(mode, grid)
        k += 1
        if k % 16 == 0:
            b.sync()
    for _ in range(warmup):
        b.step(mode, grid)
        if reduce is not None:
            reduce()
    b.sync()


def time_steps(b, mode, steps, warmup, grid=0):
    """Kernel time per launch: HIP events on the launch stream (torch's
    current one) around `steps` back-to-back launches over the resident
    batch (a capture loop's steady state).  The per-protocol counters
    accumulate across the launches and must sum to steps x packets.  A
    workload whose launches take ext-pool words is timed launch by launch
    instead (each launch needs its pool reset, as the caller does between
    batches), with one event pair per launch."""
    warm(b, mode, warmup, grid)
    if int(b.ext_used.item()) != 0:
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for k in range(steps):
            b.step(mode, grid, evs[k])
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(c) for a, c in evs]))
    b.counters.zero_()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(steps):
        b.step(mode, grid, zero=False)
    ev[1].record()
    torch.cuda.synchronize()
    cnt = b.counters.cpu().numpy().view(np.uint64)
    assert int(cnt[nsd.CNT_PKTS]) == steps * b.n and int(b.ext_used.item()) == 0, "counter check failed"
    b.counters.zero_()
    b.step(mode, grid)   # leaves one launch's counters for the caller's checks
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / steps


# ---- in-run PMC traffic ----------------------------------------------------------
PMC_WARM = 80   # launches per config before the counted ones: the adaptive schedule settles


def pmc_child(args):
    """Runs under rocprofv3 --pmc: PMC_WARM + `steps` dissect launches per
    config, in the order of --pmc-configs (the parent splits the dispatches
    by order and counts the last `steps` of each config: by then the adaptive
    schedule is the one the timed run uses)."""
    torch.cuda.set_device(0)
    for key in args.pmc_configs.split(","):
        shards = args.shards if key == args.config else 1
        b = Batch(key, args.packets, 0, shards, torch.device("cuda", 0), compact=args.records == "compact")
        for k in range(PMC_WARM + args.steps):
            b.step(args.mode, args.grid)
            if k % 16 == 15:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        print(f"pmc-child {key} schedule {nsd.last_schedule()}", flush=True)
        b.free()
        torch.cuda.empty_cache()


def pmc_traffic(args, keys, steps=3):
    """HBM bytes per dissect launch for each config in `keys`, from two
    rocprofv3 --pmc child runs (FETCH_SIZE, WRITE_SIZE: separate passes).
    FETCH_SIZE counts half the bytes of a wide coalesced read on gfx950 and is
    doubled; both are KiB (MI355X_MICROARCH.md "HBM").  Returns
    {key: {...}} or {"error": ...}."""
    got = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory(dir="/tmp") as d:
            cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", ctr, "--kernel-trace", "-d", d, "-o",
                   "run", "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__),
                   "--pmc-child", "--pmc-configs", ",".join(keys), "--config", args.config,
                   "--packets", str(args.packets), "--shards", str(args.shards), "--steps", str(steps),
                   "--mode", str(args.mode), "--grid", str(args.grid), "--records", args.records]
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                return {"error": f"rocprofv3 --pmc {ctr} rc={r.returncode}: "
                                 + r.stdout.decode(errors="replace")[-300:]}
            rows = []
            for fn in files:
                with open(fn) as f:
                    for j, row in enumerate(csv.DictReader(f)):
                        if "nsd::dissect_" in row["Kernel_Name"] and row["Counter_Name"] == ctr:
                            order = row.get("Dispatch_Id") or row.get("Correlation_Id") or j
                            rows.append((int(order), row["Kernel_Name"], float(row["Counter_Value"])))
            rows.sort()
            # one launch = dissect_fast + the dissect_walk after it (the split
            # schedule), or one dissect_all (the fused kernel)
            launches = []
            for _, name, v in rows:
                if "dissect_walk" in name and launches:
                    launches[-1] += v
                else:
                    launches.append(v)
            per = PMC_WARM + steps
            if len(launches) != per * len(keys):
                return {"error": f"{ctr}: {len(launches)} dissect launches, expected {per * len(keys)}"}
            for i, key in enumerate(keys):
                v = launches[(i + 1) * per - steps:(i + 1) * per]
                got.setdefault(key, {})[ctr] = sum(v) / len(v) * 1024
    out = {}
    for key in keys:
        rd, wr = 2 * got[key]["FETCH_SIZE"], got[key]["WRITE_SIZE"]
        out[key] = {"read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr}
    return out


# ---- CPU baseline ------------------------------------------------------------------
def cpu_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return model, os.cpu_count() or 1, min(avail, cpu_quota() or avail)


def cpu_quota():
    """CPUs this process may use by its cgroup's CFS quota (v2 cpu.max or v1
    cfs_quota_us / cfs_period_us), None when unlimited: the GPU boxes show
    every core of the machine but grant each GPU's jobs a 16-CPU share."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                return max(1, int(int(q) // int(per)))
            return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return max(1, q // per) if q > 0 else None
    except (OSError, ValueError):
        return None


def cpu_rate(cfg, n_sample, threads, seconds, text):
    """CPU restatement (oracle, "port") over one resident sample of
    `n_sample` packets, repeated until `seconds` have passed: fields only
    (records + counters) or fields + PRINT_NORM text (per-packet sink,
    discarded like a write to /dev/null).  The text is what `netsniff-ng
    --in` prints for the synthetic pcap the replay leg reads (records (i, 0)
    timestamps): each packet's frame header line (show_frame_hdr), then the
    dissector's.  Returns (Mpkt/s, packets, s)."""
    frames, desc = T.make_batch(cfg, n_sample, lo=0, threads=threads)
    fh = np.zeros(n_sample, dtype=T.FH_DTYPE)
    fh["sec"] = np.arange(n_sample, dtype=np.uint32)
    fh["len"] = T.desc_caplen(desc).astype(np.uint32)
    lib = T.oracle()
    counters = np.zeros(64, dtype=np.uint64)
    rec = np.zeros(n_sample, dtype=T.REC_DTYPE)
    tb = np.zeros(1, dtype=np.uint64)
    done, t0 = 0, time.perf_counter()
    while True:
        if text:
            lib.nsor_dissect_batch_text_fh_mt(frames.ctypes.data, desc.ctypes.data, fh.ctypes.data, None, 1,
                                              n_sample, 1, T.PRINT_NORM, threads, tb.ctypes.data)
        else:
            lib.nsor_dissect_batch_mt(frames.ctypes.data, desc.ctypes.data, n_sample, 1, T.PRINT_NORM,
                                      rec.ctypes.data, counters.ctypes.data, threads)
        done += n_sample
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return done / dt / 1e6, done, dt


def ref_harness_rate(cfg, key, n=1 << 17, frames=True):
    """`netsniff-ng --in`'s loop through the reference's own objects on one
    core: oracle/_ref/nsref (built here from /root/reference's sources: its
    pcap reader and record conversion, parser objects and tprintf.c; the
    IPv4/IPv6 layers are the restatement, their sources need config.h) over a
    synthetic pcap of n records, text to /dev/null.  None when the harness
    was not built."""
    exe = os.path.join(ROOT, "oracle", "_ref", "nsref")
    if not os.path.exists(exe):
        return None
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "ref.pcap")
        T.synth().nsd_synth_pcap(cfg, T.SEED, 0, n, path.encode())
        t0 = time.perf_counter()
        r = subprocess.run([exe] + (["-f"] if frames else []) +
                           ["-m", str(T.PRINT_NORM), "-w", "0", "-i", os.path.join(d, "idx"), path],
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=300)
        dt = time.perf_counter() - t0
    if r.returncode != 0:
        return {"error": f"nsref rc={r.returncode}: {r.stderr.decode(errors='replace')[-200:]}"}
    return {"value": round(n / dt / 1e6, 4), "unit": "Mpkt/s", "cores": 1, "kind": "reference",
            "sample": f"{key}: {n} records, `nsref{' -f' if frames else ''}` "
                      f"({'frame header line (if_indextoname per packet, as the reference) + ' if frames else ''}"
                      f"dissector text, tprintf's 80-column wrap) to /dev/null in {dt:.2f} s, process start "
                      f"included"}


def ref_harness_all_cores(cfg, key, procs, rate1, seconds=8.0):
    """The reference's own objects on `procs` host cores at once, the way
    the reference scales a capture out (one netsniff-ng process per CPU in
    a PACKET_FANOUT group, ring_rx.c:197-215; the `--in` loop,
    netsniff-ng.c:707-756): `procs` oracle/_ref/nsref -f processes, each over
    its own contiguous shard of the workload as a pcap file (records
    [p * n, (p + 1) * n)), started together, text to /dev/null.  n is sized
    from the one-core rate `rate1` (Mpkt/s) for about `seconds` of work per
    process.  Rate = all records / the wall time from the first start to the
    last exit (process start included).  None when the harness was not
    built."""
    exe = os.path.join(ROOT, "oracle", "_ref", "nsref")
    if not os.path.exists(exe) or not rate1:
        return None
    from concurrent.futures import ThreadPoolExecutor
    n = int(min(max(rate1 * 1e6 * seconds, 4096), 1 << 20))
    with tempfile.TemporaryDirectory() as d:
        paths = [os.path.join(d, f"shard{p}.pcap") for p in range(procs)]
        with ThreadPoolExecutor(procs) as ex:
            list(ex.map(lambda p: T.synth().nsd_synth_pcap(cfg, T.SEED, p * n, n, paths[p].encode()),
                        range(procs)))
        t0 = time.perf_counter()
        ps = [subprocess.Popen([exe, "-f", "-m", str(T.PRINT_NORM), "-w", "0", "-i", paths[p] + ".idx", paths[p]],
                               stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
              for p in range(procs)]
        errs = []
        for pr in ps:
            _, e = pr.communicate(timeout=600)
            if pr.returncode != 0:
                errs.append(f"rc={pr.returncode}: {e.decode(errors='replace')[-120:]}")
        dt = time.perf_counter() - t0
    if errs:
        return {"error": "; ".join(errs[:2])}
    return {"value": round(procs * n / dt / 1e6, 4), "unit": "Mpkt/s", "cores": procs, "processes": procs,
            "kind": "reference",
            "sample": f"{key}: {procs} concurrent `nsref -f` processes (the reference's pcap reader, record "
                      f"conversion, frame header line, parser objects and tprintf.c at 80 columns; IPv4/IPv6 "
                      f"restated), each over its own {n}-record contiguous shard, text to /dev/null, "
                      f"{procs * n} records in {dt:.2f} s wall, process start included",
            "vs_1core": round(procs * n / dt / 1e6 / rate1, 2)}


def cpu_baseline(key, seconds):
    """The CPU baseline on this host (SURVEY 8d / BASELINE.md "CPU-baseline
    plan").  `value` is the reference itself: its own objects
    (oracle/_ref/nsref: pcap reader, record conversion, frame header line,
    parser objects, tprintf.c) as one process per core of the GPU's 16-CPU
    share over contiguous shards of the headline workload, the way the
    reference scales out (kind "reference", `cores` the processes).  Beside
    it: the same for C3 IMIX, the reference on one core, and the CPU
    restatement (oracle/nsd_oracle.c, kind "port"): fields + PRINT_NORM text
    and fields only, on 1 thread, the 16-thread share and every available
    core.  When the reference's objects are not built, `value` falls back to
    the port's text rate on every available core."""
    cfg = CONFIGS[key]["cfg"]
    model, nproc, avail = cpu_info()
    t16 = min(avail, 16)   # the GPU box's CPU share per GPU is 16 threads
    more = avail > t16   # every available core is more than the 16-thread share
    legs = 6 if more else 4
    t1, p1, d1 = cpu_rate(cfg, 1 << 16, 1, seconds / legs, True)
    tS, pS, dS = cpu_rate(cfg, 1 << 20, t16, seconds / legs, True)
    f1, q1, e1 = cpu_rate(cfg, 1 << 20, 1, seconds / legs, False)
    fS, qS, eS = cpu_rate(cfg, 1 << 22, t16, seconds / legs, False)
    if more:
        tA, pA, dA = cpu_rate(cfg, max(1 << 20, 4096 * avail), avail, seconds / legs, True)
        fA, qA, eA = cpu_rate(cfg, max(1 << 22, 65536 * avail), avail, seconds / legs, False)
    else:
        tA, pA, dA, fA = tS, pS, dS, fS
    ref1, refA = {}, {}
    for k in dict.fromkeys(("udp64", "imix", key)):
        r1 = ref_harness_rate(CONFIGS[k]["cfg"], k, n=(1 << 17) if k == "udp64" else (1 << 15))
        ref1[k] = r1
        refA[k] = ref_harness_all_cores(CONFIGS[k]["cfg"], k, t16,
                                        r1.get("value") if isinstance(r1, dict) else None)
    port = {"value": round(tA, 3), "unit": "Mpkt/s", "cores": avail, "kind": "port",
            "sample": f"{key}: fields + PRINT_NORM text with frame header lines (the reference prints as "
                      f"it parses; `netsniff-ng --in`'s text) by the CPU "
                      f"restatement (oracle/nsd_oracle.c), {avail} threads (every available core) over "
                      f"contiguous shards, {pA} packets (passes over a resident "
                      f"{max(1 << 20, 4096 * avail) if more else 1 << 20}-packet sample) in {dA:.1f} s"}
    ref = refA.get(key)
    if isinstance(ref, dict) and ref.get("value"):
        head = {"value": ref["value"], "unit": "Mpkt/s", "cores": ref["cores"], "kind": "reference",
                "sample": ref["sample"], "port": port}
    else:
        head = dict(port, reference_error=ref.get("error") if isinstance(ref, dict) else "oracle/_ref not built")
    return dict(head, **{
            "cpu_model": model, "nproc": nproc, "cpus_available": avail, "cgroup_cpu_quota": cpu_quota(),
            "text_1thread": round(t1, 3),
            "text_16threads": {"threads": t16, "value": round(tS, 3)},
            "fields_only": {"all_cores": round(fA, 3), "threads16": round(fS, 3), "1thread": round(f1, 3)},
            "reference_harness_container": "0.182 Mpkt/s PRINT_NORM 1 core (BASELINE.md, measured in the "
                                           "build container, not on this host)",
            "reference_harness_1thread": ref1.get(key, ref1["udp64"]),
            "reference_harness_1thread_by_workload": ref1,
            "reference_harness_all_cores": refA,
            "reference_dissector_1thread": ref_harness_rate(cfg, key, frames=False)})


# ---- host-memory legs (reported, never `value`) ----------------------------------------
def bpf_bench(b, steps, warmup):
    """Device BPF filter (nsd_bpf.hip) over the same resident batch:
    bpfc.8's "Only allow IPv4 TCP packets" program (ldh [12]; jne #0x800;
    ldb [23]; jneq #6; ret #-1; ret #0), verdicts only and with the compaction
    of accepted descriptors.  Algorithmic bytes per packet: 8 (descriptor) +
    the frame's first 64-B line (capped at caplen; the program reads bytes
    12..23) + 4 (verdict)."""
    prog = np.array([(0x28, 0, 0, 12), (0x15, 0, 3, 0x800), (0x30, 0, 0, 23), (0x15, 0, 1, 6),
                     (0x06, 0, 0, 0xFFFFFFFF), (0x06, 0, 0, 0)], dtype=nsd.BPF_INSN)
    bp = nsd.BpfProgram(prog)
    n, dev = b.n, b.desc.device
    verdict = torch.empty(n, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.empty(nsd.lib().nsd_bpf_workspace_bytes(n), dtype=torch.uint8, device=dev)
    res = {}
    for compact in (False, True):
        for _ in range(max(warmup, 1)):
            bp.filter_device(b.frames, b.desc, compact, verdict, out, count, ws)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(steps):
            bp.filter_device(b.frames, b.desc, compact, verdict, out, count, ws)
        ev[1].record()
        torch.cuda.synchronize()
        res[compact] = ev[0].elapsed_time(ev[1]) / steps
    kept = int(count.item())
    # the program's verdict restated over the resident bytes (ethertype
    # 0x0800 at 12, protocol 6 at 23; a load past caplen returns 0,
    # bpf.c:538-551): the accepted count the compaction wrote must match
    d = b.desc
    off = d & ((1 << 40) - 1)
    cap = d >> 40
    fr = b.frames
    ok = (cap >= 24) & (fr[off + 12] == 8) & (fr[off + 13] == 0) & (fr[off + 23] == 6)
    want = int(ok.sum().item())
    assert kept == want, f"bpf: {kept} accepted, restated program {want}"
    algo = 8 * n + b.line_bytes + 4 * n
    gbs = algo / (res[False] * 1e-3) / 1e9
    bp.close()
    return {"program": "bpfc.8 'Only allow IPv4 TCP packets' (6 insns)", "workload": CONFIGS[b.key]["name"],
            "packets": n, "accepted": kept, "accepted_check": "equal to the program restated over the bytes",
            "value": round(n / (res[False] * 1e-3) / 1e6, 1), "unit": "Mpkt/s",
            "kernel_ms": round(res[False], 4), "compact_ms": round(res[True], 4),
            "compact_mpps": round(n / (res[True] * 1e-3) / 1e6, 1),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_pkt": round(algo / n, 2)}}


def end_to_end(key, batch, nbatch, depth, mode, reps=3):
    """Host memory in, records in host memory out: `nbatch`
    batches of `batch` packets of config `key` from one pinned host buffer
    go through the pipelined path (nsd_pipe_*, compact records: H2D, dissect
    kernels, D2H of records, counters and - when a record needs them - side
    words / ext entries, `depth` batches in flight).  The batches' summed
    counters are checked against the oracle's for the same packets when the
    run covers a whole golden shard (tests/golden/shard_counters.json)."""
    cfg = CONFIGS[key]["cfg"]
    L = nsd.lib()
    n = batch * nbatch
    frames, desc = T.make_batch(cfg, n, lo=0, threads=16)
    off = (desc & np.uint64((1 << 40) - 1)).astype(np.int64)
    cap = (desc >> np.uint64(40)).astype(np.int64)
    rec = np.zeros(n, dtype=nsd.CREC_DTYPE)
    pinned = [a for a in (frames, rec) if L.nsd_host_register(a.ctypes.data, a.nbytes) == 0]
    slices = []
    for k in range(nbatch):
        a, b = k * batch, (k + 1) * batch
        lo, hi = int(off[a]), int(off[b - 1] + cap[b - 1])
        d = (desc[a:b] - np.uint64(lo)).astype(np.uint64)
        slices.append((frames[lo:hi + nsd.FRAME_PAD], d, rec[a:b]))
    descs_pinned = [L.nsd_host_register(d.ctypes.data, d.nbytes) == 0 for _, d, _ in slices]
    max_bytes = max(f.nbytes for f, _, _ in slices)
    ext_w = batch + (nsd.ext_pool_words(batch) if cfg == T.SYN_IPV6X else nsd.ext_pool_words(batch // 64))
    pipe = nsd.Pipe(batch, max_bytes, ext_words=ext_w, depth=depth, mode=mode, compact=True)
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
    # every pass wrote the same counters; the last one's are checked
    want = golden_counters(key, n, 1) if mode == nsd.PRINT_NORM else None
    if want is not None:
        assert np.array_equal(cnts.sum(axis=0, dtype=np.uint64), want), f"e2e {key}: counters differ from the oracle's"
    h2d = sum(f.nbytes - nsd.FRAME_PAD + d.nbytes for f, d, _ in slices)
    d2h = n * CREC_B
    dt = min(times)
    for a in pinned:
        L.nsd_host_unregister(a.ctypes.data)
    for ok, (_, d, _) in zip(descs_pinned, slices):
        if ok:
            L.nsd_host_unregister(d.ctypes.data)
    return {"workload": CONFIGS[key]["name"], "value": round(n / dt / 1e6, 2), "unit": "Mpkt/s",
            "pcie_gbs": round((h2d + d2h) / dt / 1e9, 2),
            "counters_check": ("summed over the batches = the oracle's counters of the shard "
                               "(tests/golden/shard_counters.json)") if want is not None else None,
            "h2d_bytes_per_pkt": round(h2d / n, 2), "d2h_bytes_per_pkt": CREC_B,
            "records": "compact 8 B (nsd_crec)",
            "batches": nbatch, "batch_packets": batch, "depth": depth,
            "pinned": len(pinned) == 2 and all(descs_pinned),
            "note": "host frames -> H2D -> dissect kernels -> D2H records/counters "
                    "(nsd_pipe_*, compact records), best of %d passes" % reps}


PREFIX = os.path.join(ROOT, "tests", "golden", "prefix.json")


def replay_digest(key, mode, threads):
    """The replay's text checked: the first 65,536 records of config `key`
    as a pcap replayed through the device (the timed leg's path, unwrapped
    text) must hash to what the reference's own read_pcap loop printed for
    the same file (nsref -f; tests/golden/prefix.json replay_text_sha256).
    Returns the check's description (None: no golden for this mode)."""
    if not os.path.exists(PREFIX):
        return None
    with open(PREFIX) as f:
        want = json.load(f).get(f"{key}:m{mode}", {}).get("replay_text_sha256")
    if want is None:
        return None
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "prefix.pcap")
        T.synth().nsd_synth_pcap(CONFIGS[key]["cfg"], T.SEED, 0, 65536, path.encode())
        got, text = nsd.replay_pcap(path, mode=mode, threads=threads)
    assert got == 65536 and hashlib.sha256(text).hexdigest() == want, f"replay {key}: text differs from the reference's"
    return ("sha256 of the replayed text of the first 65,536 records = the reference's own --in loop's "
            "(nsref -f, tests/golden/prefix.json)")


def replay_leg(key, n, mode, threads, reps=2):
    """`netsniff-ng --in file.pcap` through the device (nsd_replay_pcap): a
    synthetic pcap of n records of config `key` in a temp file -> reader ->
    pipelined device walk (compact records) -> host formatter pool of
    `threads` threads -> /dev/null; and the same with one formatter thread
    over n/8 records (the product formatter's single-thread rate, beside
    cpu_baseline.text_1thread).  The text itself is checked by
    replay_digest."""
    cfg = CONFIGS[key]["cfg"]
    check = replay_digest(key, mode, threads)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "replay.pcap")
        T.synth().nsd_synth_pcap(cfg, T.SEED, 0, n, path.encode())
        path1 = os.path.join(d, "replay1.pcap")
        n1 = max(n // 8, 1)
        T.synth().nsd_synth_pcap(cfg, T.SEED, 0, n1, path1.encode())
        size = os.path.getsize(path)
        fd = os.open(os.devnull, os.O_WRONLY)
        try:
            def best_of(pth, cnt, th):
                best = None
                for _ in range(reps):
                    t0 = time.perf_counter()
                    got, _ = nsd.replay_pcap(pth, mode=mode, threads=th, out_fd=fd)
                    dt = time.perf_counter() - t0
                    assert got == cnt
                    best = dt if best is None else min(best, dt)
                return best
            best = best_of(path, n, threads)
            best1 = best_of(path1, n1, 1)
        finally:
            os.close(fd)
    return {"workload": CONFIGS[key]["name"], "value": round(n / best / 1e6, 3), "unit": "Mpkt/s", "packets": n,
            "file_gbs": round(size / best / 1e9, 2), "format_threads": threads, "text_check": check,
            "format_1thread": round(n1 / best1 / 1e6, 3),
            "note": "pcap file -> nsd_pcap reader -> H2D -> dissect kernels -> D2H compact records -> "
                    "formatter pool -> writev /dev/null (nsd_replay_pcap), best of %d" % reps}


def copy_rate(dev):
    """Achievable streaming rate on this device: a 1 GiB
    device-to-device copy, read + write bytes / time."""
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
    gbs = 2 * cbuf.numel() * 5 / (ce[0].elapsed_time(ce[1]) * 1e-3) / 1e9
    del cbuf, cdst
    return gbs


BW_SO = os.path.join(ROOT, "tools", "bw", "libnsdbw.so")


def read_ceiling(buf, reps=5):
    """The read rate this device reaches in this run (the
    achievable rate beside the spec peak): tools/bw/nsd_bw.hip streams the
    resident frame buffer of the timed batch (four 16-B loads in flight per
    lane, grid-stride), best over 2 / 4 / 8 blocks of 256 per CU x plain /
    nontemporal loads, `reps` launches each between HIP events.  A read-only
    ceiling, unlike copy_gbs (read + write of a torch copy)."""
    L = ctypes.CDLL(BW_SO)
    L.nsd_bw_read.restype = ctypes.c_int
    L.nsd_bw_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                              ctypes.c_void_p]
    nbytes = (buf.numel() // 16) * 16
    sink = torch.zeros(4, dtype=torch.int32, device=buf.device)
    stream = torch.cuda.current_stream().cuda_stream
    best = None
    for bpc in (2, 4, 8):
        for nt in (0, 1):
            def go():
                assert L.nsd_bw_read(buf.data_ptr(), nbytes, bpc, nt, stream, sink.data_ptr()) == 0
            go()
            go()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(reps):
                go()
            ev[1].record()
            torch.cuda.synchronize()
            gbs = nbytes * reps / (ev[0].elapsed_time(ev[1]) * 1e-3) / 1e9
            if best is None or gbs > best["gbs"]:
                best = {"gbs": round(gbs, 1), "blocks_per_cu": bpc, "nontemporal": bool(nt), "bytes": nbytes}
    return best


def measure_rank(args, rank, world, dev, engine="device"):
    """One rank's measurement (the whole job at N = 1): its weak shard of
    args.packets x args.shards packets [rank * per_rank, ...) resident, the
    untimed warmup, then exactly args.steps launches between a barrier +
    sync on both sides, the per-protocol counters summed over the ranks by
    one all-reduce inside the timed region (RCCL over xGMI; gloo in the CPU
    test) and the times maxed over the ranks (nsd_dist).  Counters must come
    to world x packets x steps.  engine "host" (tests/test_multi.py only)
    walks the shard with the product's host walk instead of the kernel.
    Returns (batch, info dict)."""
    per_rank = args.packets * args.shards
    lo, _ = nsd_dist.weak_shard(per_rank, rank)
    compact = args.records == "compact"
    t_setup = time.perf_counter()   # the shard's generation and upload (the N-rank budget)
    if engine == "device":
        b = Batch(args.config, args.packets, lo, args.shards, dev, compact=compact)
        torch.cuda.synchronize()
    else:
        b = HostBatch(args.config, args.packets, lo, args.shards, compact=compact)
    t_setup = time.perf_counter() - t_setup
    multi = nsd_dist.initialized()
    warm(b, args.mode, args.warmup, args.grid,
         seconds=WARM_SECONDS if engine == "device" else 0.0,
         reduce=(lambda: nsd_dist.reduce_counters(b.counters)) if multi else None)
    # the K launches back to back, counters accumulating across them; a
    # workload whose launches take ext-pool words (none of the bench's) is
    # timed launch by launch with its pool and counters reset before each,
    # as a caller does between batches
    accumulate = nsd_dist.all_ranks_agree(int(b.ext_used.item()) == 0, dev)
    if accumulate:
        b.counters.zero_()
    nsd_dist.barrier()
    b.sync()
    evs = [(b.event(), b.event()) for _ in range(1 if accumulate else args.steps)]
    t0 = time.perf_counter()
    if accumulate:
        evs[0][0].record()
        for _ in range(args.steps):
            b.step(args.mode, args.grid, zero=False)
        evs[0][1].record()
        nsd_dist.reduce_counters(b.counters)
    else:
        for k in range(args.steps):
            b.step(args.mode, args.grid, evs[k])
            nsd_dist.reduce_counters(b.counters)
    b.sync()
    nsd_dist.barrier()
    b.sync()
    elapsed = time.perf_counter() - t0
    kern_ms = (evs[0][0].elapsed_time(evs[0][1]) / args.steps if accumulate
               else float(np.mean([a.elapsed_time(c) for a, c in evs])))
    elapsed, kern_ms, t_setup = nsd_dist.max_over_ranks([elapsed, kern_ms, t_setup], dev)
    cnt = b.counters.cpu().numpy().view(np.uint64).copy()
    total_pkts = b.n * world
    assert int(cnt[nsd.CNT_PKTS]) == total_pkts * (args.steps if accumulate else 1), "counter check failed"
    assert not accumulate or int(b.ext_used.item()) == 0, "ext pool used while accumulating"
    return b, {"elapsed": elapsed, "kern_ms": kern_ms, "counters": cnt, "total_pkts": total_pkts,
               "accumulate": accumulate, "frame_bytes": b.frame_bytes, "setup_s": t_setup}



SHARD_COUNTERS = os.path.join(ROOT, "tests", "golden", "shard_counters.json")


def golden_counters(key, n, world, shards=1):
    """The oracle's PRINT_NORM counter vector summed over the shards the
    `world` ranks walk (rank r: packets [r * n * shards, (r + 1) * n * shards)
    in n-packet shards; tests/golden/shard_counters.json, made by
    make_golden.py --shards-only), or None when the table lacks a shard."""
    if not os.path.exists(SHARD_COUNTERS):
        return None
    with open(SHARD_COUNTERS) as f:
        table = json.load(f)
    total = np.zeros(nsd.NCOUNTERS, dtype=np.uint64)
    for j in range(world * shards):
        k = f"{key}:{j * n}:{n}"
        if k not in table:
            return None
        total += np.array(table[k], dtype=np.uint64)
    return total


def workload_name_n(key, n, shards, world):
    if world > 1 and key == "imix" and shards == 1:
        tag = "C5" if world == 8 else "C5-style"
        return (f"{tag}: {world * n} IMIX packets sharded across {world} GPUs "
                f"({n // (1 << 20)}M per GPU, counters all-reduced)")
    name = workload_name(key, n, shards)
    return name if world == 1 else f"{name}, {world} GPUs x {n * shards} packets"


def workload_result(args, key, b, m, world, engine, traffic=None, copy_gbs=None, ceiling=None):
    """One workload of the line, measured by measure_rank at this N: the
    whole-job rate (wall clock, max over ranks, counter all-reduce inside),
    the per-GPU kernel time and roofline, and the all-reduced counters
    checked against the oracle's per-shard counters (a mismatch fails the
    run)."""
    elapsed, kern_ms, total = m["elapsed"], m["kern_ms"], m["total_pkts"]
    reps = args.steps if m["accumulate"] else 1
    want = golden_counters(key, b.n_shard, world, b.shards) if engine == "device" else None
    if want is not None:
        assert np.array_equal(m["counters"], want * np.uint64(reps)), \
            f"{key}: all-reduced counters differ from the oracle's shard counters"
    tr = traffic.get(key) if isinstance(traffic, dict) else None
    return {"workload": workload_name_n(key, b.n_shard, b.shards, world), "packets": total,
            "packets_per_gpu": b.n, "schedule": nsd.last_schedule() if engine == "device" else "host walk",
            "value": round(total * args.steps / elapsed / 1e6, 2), "unit": "Mpkt/s",
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "kernel_value": round(total / (kern_ms * 1e-3) / 1e6, 2),
            "setup_s": round(m["setup_s"], 2),
            "gbps_frames": round(m["frame_bytes"] * world * args.steps / elapsed / 1e9, 1),
            "roofline": b.roofline(kern_ms, tr, copy_gbs, ceiling),
            "counters": nsd.unpack_counters(m["counters"]),
            "counters_check": (f"all-reduced over {world} rank(s) = the oracle's counters of the {world * b.shards} "
                               f"shard(s) x {reps} launch(es) (tests/golden/shard_counters.json)")
            if want is not None else "packets = ranks x shard x launches (no golden for this shard size)"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)   # (a capture loop runs continuously: 100 back-to-back batches, ≈ 20 ms on C2)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="udp64", choices=sorted(CONFIGS))
    ap.add_argument("--packets", type=int, default=1 << 24, help="packets per shard")
    ap.add_argument("--shards", type=int, default=1, help="contiguous shards walked as one batch per GPU")
    ap.add_argument("--mode", type=int, default=nsd.PRINT_NORM)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--records", default="compact", choices=["compact", "full"],
                    help="record form of the timed launches: 8-byte nsd_crec or 16-byte nsd_rec")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=24.0, help="CPU baseline duration (all legs)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory end-to-end pass")
    ap.add_argument("--no-bpf", action="store_true", help="skip the device BPF filter pass")
    ap.add_argument("--no-replay", action="store_true", help="skip the pcap replay (--in) pass")
    ap.add_argument("--no-legs", action="store_true", help="skip the C3 / C4 legs")
    ap.add_argument("--no-pmc", action="store_true", help="skip the in-run rocprofv3 PMC traffic pass")
    ap.add_argument("--replay-packets", type=int, default=1 << 20)
    ap.add_argument("--e2e-batch", type=int, default=1 << 20)
    ap.add_argument("--e2e-batches", type=int, default=16)
    ap.add_argument("--e2e-depth", type=int, default=3)
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    # the CPU tests' switch: every rank walks its shards with the product's
    # host walk over gloo (tests/test_multi.py runs `bench.py --gpus 2` this
    # way, through spawn_ranks and torch.distributed.run); never a bench run
    ap.add_argument("--engine", default="device", choices=["device", "host"], help=argparse.SUPPRESS)
    ap.add_argument("--pmc-configs", default="", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def run(args, rank, world, dev, engine="device", traffic=None):
    """Every rank's measurements in launch order (the same collectives on
    every rank), and rank 0's JSON line (a dict; None on other ranks).  At
    every N: the headline workload and each leg (C3 IMIX, whose 8-rank run is
    C5, and C4) through measure_rank, the counters all-reduced and checked
    against the oracle's per-shard counters.  N = 1 only: the other record
    form, the CPU baseline, end to end, replay and BPF.  engine "host"
    (tests/test_multi.py) walks each shard with the product's host walk and
    skips the device-only legs."""
    solo = rank == 0 and world == 1
    dev_eng = engine == "device"
    legs = [k for k in LEGS if k != args.config] if not args.no_legs else []
    n = args.packets
    compact = args.records == "compact"

    b, m = measure_rank(args, rank, world, dev, engine)
    schedule = nsd.last_schedule() if dev_eng else "host walk"
    elapsed, kern_ms, total_pkts = m["elapsed"], m["kern_ms"], m["total_pkts"]
    ms_per_step = elapsed / args.steps * 1e3
    mpps = total_pkts * args.steps / elapsed / 1e6

    copy_gbs = copy_rate(dev) if dev_eng else None
    ceiling = read_ceiling(b.frames) if dev_eng else None
    head = workload_result(args, args.config, b, m, world, engine, traffic, copy_gbs, ceiling)
    roofline = head["roofline"]
    # the BPF leg filters C3's IMIX (its "IPv4 TCP" program accepts the
    # untagged TCP sixth; C2's UDP would leave the compaction nothing)
    want_bpf = solo and dev_eng and not args.no_bpf
    bpf = bpf_bench(b, args.steps, args.warmup) if want_bpf and (args.config == "imix" or "imix" not in legs) \
        else None
    frame_bytes = b.frame_bytes
    b.free()
    if dev_eng:
        torch.cuda.empty_cache()

    # the other record form over the same workload (kernel time, roofline)
    other = None
    if solo and dev_eng and not args.no_legs:
        ob = Batch(args.config, n, 0, args.shards, dev, compact=not compact)
        oms = time_steps(ob, args.mode, args.steps, args.warmup, 0)
        other = {"records": "full 16 B (nsd_rec)" if compact else "compact 8 B (nsd_crec)",
                 "value": round(ob.n / (oms * 1e-3) / 1e6, 2), "unit": "Mpkt/s (kernel time)",
                 "roofline": ob.roofline(oms, None, copy_gbs, ceiling)}
        ob.free()
        torch.cuda.empty_cache()
    if roofline is not None:
        # which of SURVEY 8(a)'s chain-walk fields the timed launches write
        if compact:
            roofline["record_form"] = ("compact 8 B nsd_crec: ops-id chain, IPv4 checksum, layer count + flags "
                                       "(side word / ext entry past 6 layers); the per-layer offsets and the "
                                       "final data/tail cursor are re-derived by the renderer, not written")
        else:
            roofline["record_form"] = ("full 16 B nsd_rec: ops-id chain, per-layer offsets, final data/tail "
                                       "cursor, IPv4 checksum, layer count + flags")
        if other is not None and other["roofline"] is not None:
            roofline["other_record_form"] = {"records": other["records"],
                                             "frac": other["roofline"]["frac"],
                                             "read_frac": other["roofline"]["read_frac"],
                                             "kernel_ms": other["roofline"]["kernel_ms"]}

    # every leg at every N: rank r walks its own 16M shard of each config
    # (8 IMIX ranks = C5's 128M packets), counters all-reduced and checked
    leg_out = {}
    for key in legs:
        la = argparse.Namespace(**vars(args))
        la.config, la.shards = key, 1
        lb, lm = measure_rank(la, rank, world, dev, engine)
        if key == "imix" and want_bpf and bpf is None:
            bpf = bpf_bench(lb, args.steps, args.warmup)
        leg_out[key] = workload_result(la, key, lb, lm, world, engine, traffic, copy_gbs, ceiling)
        lb.free()
        if dev_eng:
            torch.cuda.empty_cache()

    cpu = None
    if solo and dev_eng and not args.no_cpu:
        cpu = cpu_baseline(args.config, args.cpu_seconds)

    # the host-memory legs for the headline workload and, beside it, IMIX
    # (north_star: 64 B and IMIX), as "imix" keys of the headline's dicts
    host_keys = [args.config] + (["imix"] if args.config != "imix" and not args.no_legs else [])
    e2e = None
    if solo and dev_eng and not args.no_e2e:
        for k in host_keys:
            r = end_to_end(k, args.e2e_batch, args.e2e_batches, args.e2e_depth, args.mode)
            if e2e is None:
                e2e = r
            else:
                e2e[k] = r

    replay = None
    if solo and dev_eng and not args.no_replay:
        for k in host_keys:
            r = replay_leg(k, args.replay_packets, args.mode, min(cpu_info()[2], 16))
            if cpu is not None and k == args.config:
                # the CPU-only text rate on the same thread count
                r["cpu_text_same_threads"] = cpu["text_16threads"]["value"]
                r["vs_cpu_text_same_threads"] = round(r["value"] / cpu["text_16threads"]["value"], 3)
            ref = ((cpu or {}).get("reference_harness_all_cores") or {}).get(k)
            if isinstance(ref, dict) and ref.get("value"):
                r["reference_same_cores"] = ref["value"]
                r["vs_reference_same_cores"] = round(r["value"] / ref["value"], 2)
            if replay is None:
                replay = r
            else:
                replay[k] = r

    if rank != 0:
        return None
    out = {
        "metric": "Mpkt/s + GB/s device-resident dissect, 64B & IMIX; bit-exact fields vs ref",
        "value": round(mpps, 2), "unit": "Mpkt/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 generators, tools/nsd_synth.c)",
        "config": {"workload": workload_name_n(args.config, n, args.shards, world), "packets_per_gpu": n * args.shards,
                   "frame_bytes_per_gpu": frame_bytes, "mode": MODES[args.mode],
                   "records": "compact 8 B (nsd_crec)" if compact else "full 16 B (nsd_rec)",
                   "schedule": schedule, "parallelism": f"dp{world}"},
        "gbps_frames": round(frame_bytes * world * args.steps / elapsed / 1e9, 1),
        "roofline": roofline,
        "counters_total": int(m["counters"][nsd.CNT_PKTS]),
        "counters_check": head["counters_check"],
        "setup_s": head["setup_s"],
        "legs": leg_out or None,
        "other_records": other,
        "cpu_baseline": cpu,
        "end_to_end": e2e,
        "replay": replay,
        "bpf_filter": bpf,
        "library": library_info() if dev_eng else None,
    }
    if isinstance(traffic, dict) and "error" in traffic:
        out["pmc_error"] = traffic["error"]
    return out


def main():
    t_start = time.perf_counter()
    args = parse_args()
    if args.pmc_child:
        pmc_child(args)
        return
    host = args.engine == "host"

    rank, world, local = nsd_dist.rank_env()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks here, as fresh processes; this one
        # never touches a GPU (the devices are counted in a child process)
        have = nsd_dist.count_devices()
        if have < args.gpus and not host:
            print(f"bench.py: --gpus {args.gpus} but {have} GPU(s) visible", file=sys.stderr)
            sys.exit(2)
        sys.exit(nsd_dist.spawn_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} under a launcher of {world} ranks", file=sys.stderr)
        sys.exit(2)
    solo = rank == 0 and world == 1
    legs = [k for k in LEGS if k != args.config] if not args.no_legs else []

    # PMC traffic first, in child processes, before this process initialises the GPU
    traffic = None
    if solo and not args.no_pmc and not host:
        traffic = pmc_traffic(args, [args.config] + legs)

    if host:
        if world > 1:
            nsd_dist.init("gloo")
        dev = torch.device("cpu")
    elif world > 1:
        nsd_dist.init("nccl", local)
        dev = torch.device("cuda", local)
    else:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
    out = run(args, rank, world, dev, args.engine, traffic)
    if out is not None:
        # this process's wall time from start to the line (rank 0; the ranks
        # meet at every workload's barriers, so it is the job's)
        out["bench_wall_s"] = round(time.perf_counter() - t_start, 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
