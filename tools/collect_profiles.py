"""Turn a tools/gpu_round.sh run (gpurun_out/round/) into the committed
profile files:

  profiles/<tag>_bench_<cfg>.json         the bench JSON line
  profiles/<tag>_<cfg>_kernel_stats.csv   rocprofv3 --stats summary
  profiles/pmc_<cfg>.json                 HBM bytes per dissect call (read by bench.py)

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE come
from separate --pmc passes, in KiB; FETCH_SIZE counts half the bytes of a
wide (16 B/lane) coalesced read on gfx950, so it is doubled; WRITE_SIZE is
exact for 16 B/lane stores.  A dissect call is one dissect_all launch (pass 1,
pass 2 and the ICMPv4 checksums as phases of one kernel); the BPF filter
kernels are reported separately (bpf_filter)."""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PACKETS = 1 << 24


def counter_sum(path, counter, kernel="nsd::dissect_all"):
    total, calls = 0.0, 0
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if kernel not in name or row["Counter_Name"] != counter:
                continue
            total += float(row["Counter_Value"])
            calls += 1
    return total, calls


def main(tag, src=os.path.join(ROOT, "gpurun_out", "round")):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    for cfg in ("udp64", "imix", "ipv6x"):
        log = os.path.join(src, f"bench_{cfg}.log")
        if os.path.exists(log):
            line = open(log).read().strip().splitlines()[-1]
            json.loads(line)
            with open(os.path.join(prof, f"{tag}_bench_{cfg}.json"), "w") as f:
                f.write(line + "\n")
        st = os.path.join(src, f"stats_{cfg}", "run_kernel_stats.csv")
        if os.path.exists(st):
            shutil.copy(st, os.path.join(prof, f"{tag}_{cfg}_kernel_stats.csv"))
        fp = os.path.join(src, f"pmc_{cfg}_FETCH_SIZE", "run_counter_collection.csv")
        wp = os.path.join(src, f"pmc_{cfg}_WRITE_SIZE", "run_counter_collection.csv")
        if os.path.exists(fp) and os.path.exists(wp):
            fk, fc = counter_sum(fp, "FETCH_SIZE")
            wk, wc = counter_sum(wp, "WRITE_SIZE")
            read_b = 2 * fk * 1024 / fc
            write_b = wk * 1024 / wc
            res = {"tag": tag, "calls": [fc, wc], "FETCH_SIZE_KiB_per_call": fk / fc,
                   "WRITE_SIZE_KiB_per_call": wk / wc, "read_bytes_corrected": read_b,
                   "write_bytes": write_b, "hbm_bytes_per_launch": read_b + write_b,
                   "bytes_per_packet": (read_b + write_b) / PACKETS,
                   "note": "per dissect_all launch; read = 2 x FETCH_SIZE "
                           "(gfx950 wide-read correction), KiB -> bytes"}
            bk, bc = counter_sum(fp, "FETCH_SIZE", "bpf_filter<false>")
            bw, bwc = counter_sum(wp, "WRITE_SIZE", "bpf_filter<false>")
            if bc and bwc:
                res["bpf_filter"] = {"read_bytes_corrected": 2 * bk * 1024 / bc, "write_bytes": bw * 1024 / bwc,
                                     "hbm_bytes_per_launch": 2 * bk * 1024 / bc + bw * 1024 / bwc,
                                     "launches": [bc, bwc]}
            with open(os.path.join(prof, f"pmc_{cfg}.json"), "w") as f:
                json.dump(res, f, indent=1)
            print(cfg, json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
