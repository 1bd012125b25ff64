"""Turn a tools/gpu_round.sh run (gpurun_out/round/) into the committed
profile files:

  profiles/<tag>_bench_default.json    the default bench JSON line (C2 headline,
                                       C3/C4 legs, both record forms, in-run PMC
                                       traffic, CPU baseline, e2e, replay, BPF)
  profiles/<tag>_bench_c5_one_gpu.json C5's 128M IMIX packets on one GPU
  profiles/<tag>_kernel_stats.csv      rocprofv3 --kernel-trace --stats of the
                                       default bench command (--no-pmc)
  profiles/<tag>_kernel_check.json     per workload: the rocprof trace's kernels
                                       (fused dissect_all, or split dissect_fast
                                       + dissect_walk), their averages, the
                                       launch span and period, against the
                                       bench's HIP-event time
  profiles/<tag>_pytest_gpu.log, <tag>_smoke.log

The bench's `traffic` comes from its own two rocprofv3 --pmc child passes
(FETCH_SIZE doubled: the gfx950 wide-read correction; WRITE_SIZE exact;
MI355X_MICROARCH.md "HBM")."""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def last_json(path):
    if not os.path.exists(path):
        return None
    for line in reversed(open(path).read().strip().splitlines()):
        if line.startswith("{"):
            return line
    return None


def main(tag, src=os.path.join(ROOT, "gpurun_out", "round")):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    for name, out in (("bench_default.log", "bench_default.json"), ("bench_c5.log", "bench_c5_one_gpu.json")):
        line = last_json(os.path.join(src, name))
        if line:
            json.loads(line)
            with open(os.path.join(prof, f"{tag}_{out}"), "w") as f:
                f.write(line + "\n")
    for name in ("pytest_gpu.log", "smoke.log"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(prof, f"{tag}_{name}"))
    st = os.path.join(src, "stats", "run_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, os.path.join(prof, f"{tag}_kernel_stats.csv"))
        rows = {}
        with open(st) as f:
            for row in csv.DictReader(f):
                if "nsd::dissect_" in row["Name"]:
                    rows[row["Name"]] = {"calls": int(row["Calls"]),
                                         "average_us": float(row["AverageNs"]) / 1e3}
        bench = last_json(os.path.join(src, "stats.log"))
        check = {"rocprof_stats": rows}
        # per workload: the bench launches dissect_all per workload in this
        # order (headline compact, the other record form, then each leg),
        # each a run of warmup launches (a time-based part: any count) + the
        # timed steps (+ one launch after them for the legs' counter checks,
        # bench.time_steps); the workloads are apart by seconds of batch
        # generation, so a gap of > 50 ms splits them
        tr = os.path.join(src, "stats", "run_kernel_trace.csv")
        if os.path.exists(tr) and bench:
            b = json.loads(bench)
            steps = b["steps"]
            # one launch = dissect_all (fused) or dissect_fast + dissect_walk
            # (split); per record form (the template's bool), in time order
            launches = {"true": [], "false": []}
            with open(tr) as f:
                for row in csv.DictReader(f):
                    nm = row["Kernel_Name"]
                    if "nsd::dissect_" not in nm or "<0," not in nm:
                        continue
                    kern = nm.split("nsd::")[1].split("<")[0]
                    form = "true" if ("<0, true>" in nm or "<0, true," in nm) else "false"
                    launches[form].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), kern))

            def steps_of(ks):
                out = []
                for s0, e0, kern in sorted(ks):
                    if kern == "dissect_walk" and out and out[-1]["kernels"][-1][0] == "dissect_fast":
                        out[-1]["kernels"].append((kern, s0, e0))
                        out[-1]["end"] = e0
                    else:
                        out.append({"start": s0, "end": e0, "kernels": [(kern, s0, e0)]})
                return out

            def runs(st):
                out, cur = [], []
                for x in st:
                    if cur and x["start"] - cur[-1]["end"] > 50_000_000:
                        out.append(cur)
                        cur = []
                    cur.append(x)
                if cur:
                    out.append(cur)
                return out

            def summary(seg):
                if not seg:
                    return None
                per = {}
                for x in seg:
                    for kern, s0, e0 in x["kernels"]:
                        per.setdefault(kern, []).append((e0 - s0) / 1e3)
                spans = [(x["end"] - x["start"]) / 1e3 for x in seg]
                gaps = [(seg[k + 1]["start"] - seg[k]["end"]) / 1e3 for k in range(len(seg) - 1)]
                return {"schedule": "fused" if "dissect_all" in per else "split",
                        "kernel_avg_us": {k: round(sum(v) / len(v), 1) for k, v in per.items()},
                        "launch_span_avg_us": round(sum(spans) / len(spans), 1),
                        "launch_period_avg_us": round((seg[-1]["end"] - seg[0]["start"]) / 1e3 / len(seg), 1),
                        "gap_avg_us": round(sum(gaps) / len(gaps), 2) if gaps else None}

            names = ["headline"] + list((b.get("legs") or {}).keys())
            split = {}
            for k, run in enumerate(runs(steps_of(launches["true"]))):
                if k < len(names):
                    split[names[k]] = summary(run[-steps:] if k == 0 else run[-steps - 1:-1])
            full = runs(steps_of(launches["false"]))
            if full:
                split["other_records"] = summary(full[0][-steps - 1:-1])
            check["rocprof_trace"] = split
        if bench:
            b = json.loads(bench)
            check["bench_kernel_ms"] = {"headline": b["roofline"]["kernel_ms"] if b.get("roofline") else None}
            for k, leg in (b.get("legs") or {}).items():
                check["bench_kernel_ms"][k] = leg["roofline"]["kernel_ms"] if leg.get("roofline") else None
            if b.get("other_records") and b["other_records"].get("roofline"):
                check["bench_kernel_ms"]["other_records"] = b["other_records"]["roofline"]["kernel_ms"]
        with open(os.path.join(prof, f"{tag}_kernel_check.json"), "w") as f:
            json.dump(check, f, indent=1)
        print(json.dumps(check, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
