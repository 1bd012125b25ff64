"""Per-config PMC summary of the dissect launches the bench times: instruction
counts per 64-packet tile and the wave-cycle split, from rocprofv3 --pmc runs
of bench.py's PMC child (each config warmed until the adaptive schedule
settles, then the last `steps` launches counted; a launch is dissect_fast +
dissect_walk or one dissect_all).  One rocprofv3 run per counter group (the
hardware's per-block limits: 8 SQ counters a pass).  Run on the GPU box:
  python tools/pmc_groups.py out.json [udp64,imix,ipv6x]"""
import csv
import glob
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GROUPS = {
    "sq1": "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU "
           "SQ_INSTS_VMEM_RD SQ_INSTS_SALU",
    "sq2": "SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_ANY "
           "SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH",
}
PACKETS = 1 << 24
STEPS = 3


def run_group(ctrs, keys):
    import bench
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        cmd = ["timeout", "-s", "KILL", "300", "rocprofv3", "--pmc"] + ctrs.split() + [
            "--kernel-trace", "-d", d, "-o", "run", "--output-format", "csv", "--", sys.executable,
            os.path.join(ROOT, "bench.py"), "--pmc-child", "--pmc-configs", ",".join(keys), "--steps", str(STEPS)]
        r = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT)
        if r.returncode != 0:
            raise SystemExit(f"rocprofv3 rc={r.returncode}: {r.stdout.decode(errors='replace')[-500:]}")
        disp = {}
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(fn)):
                if "nsd::dissect_" not in row["Kernel_Name"]:
                    continue
                k = int(row["Dispatch_Id"])
                e = disp.setdefault(k, {"name": row["Kernel_Name"], "c": {}})
                e["c"][row["Counter_Name"]] = e["c"].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    launches = []
    for k in sorted(disp):
        e = disp[k]
        if "dissect_walk" in e["name"] and launches:
            for c, v in e["c"].items():
                launches[-1]["c"][c] = launches[-1]["c"].get(c, 0.0) + v
            launches[-1]["kernels"].append("dissect_walk")
        else:
            launches.append({"c": dict(e["c"]), "kernels": [e["name"].split("nsd::")[1].split("<")[0]]})
    per = bench.PMC_WARM + STEPS
    if len(launches) != per * len(keys):
        raise SystemExit(f"{len(launches)} launches, expected {per * len(keys)}")
    out = {}
    for i, key in enumerate(keys):
        seg = launches[(i + 1) * per - STEPS:(i + 1) * per]
        avg = {}
        for L in seg:
            for c, v in L["c"].items():
                avg[c] = avg.get(c, 0.0) + v / len(seg)
        out[key] = {"kernels": "+".join(seg[-1]["kernels"]), "c": avg}
    return out


def main(path, keys="udp64,imix,ipv6x"):
    keys = keys.split(",")
    res = {k: {} for k in keys}
    for g, ctrs in GROUPS.items():
        for k, v in run_group(ctrs, keys).items():
            res[k]["kernels"] = v["kernels"]
            res[k].setdefault("c", {}).update(v["c"])
    tiles = PACKETS / 64
    out = {}
    for k, r in res.items():
        c = r["c"]
        o = {"kernels": r["kernels"]}
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR"):
            if n in c:
                o[n.lower().replace("sq_insts_", "") + "_per_tile"] = round(c[n] / tiles, 1)
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS"):
                if n in c:
                    o[n.lower() + "_frac"] = round(c[n] / wc, 3)
        if "SQ_LDS_BANK_CONFLICT" in c:
            o["lds_bank_conflict_cycles_per_tile"] = round(c["SQ_LDS_BANK_CONFLICT"] / tiles, 1)
        o["raw"] = {n: round(v, 1) for n, v in c.items()}
        out[k] = o
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: {n: v for n, v in o.items() if n != "raw"} for k, o in out.items()}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
