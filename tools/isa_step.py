"""isa_step.py - the instruction count of one walker step (gen_step inside the
walkers' session loop) from the disassembly: compiles
nsd_kernels.hip for gfx950 to assembly, finds the session's step loop in
dissect_all<PRINT_NORM, compact> (the loop holding the per-layer LDS count
and the eth_lay3 byte lookup), and prints per basic block its VALU / SALU /
LDS / branch / wait instructions and the loop's totals (the rare kinds'
bodies sit behind exec-mask branches a wave skips when none of its lanes
needs them, so one step issues a subset: DESIGN.md §5 walks the
Hop-by-Hop path through this table).  Development tool (CPU).

  python tools/isa_step.py [--src netsniff-ng_amd/csrc/nsd_kernels.hip] [--out file]
"""
import argparse
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = os.environ.get("ISA_KERNEL", "_ZN3nsd11dissect_allILi0ELb1ELb1EEEv")   # (prefix of the mangled name: the ring build)


def classify(op):
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_"):
        return "vmem"
    return "other"


def blocks_of(lines):
    out, cur = [], None
    for ln in lines:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", ln)
        if m:
            cur = {"label": m.group(1), "n": {}, "to": [], "text": []}
            out.append(cur)
            continue
        t = ln.strip()
        if cur is None or not t or t.startswith(";") or t.startswith("."):
            continue
        op = t.split()[0]
        k = classify(op)
        cur["n"][k] = cur["n"].get(k, 0) + 1
        cur["text"].append(t)
        if k == "branch":
            cur["to"].append(t)
    return out


def find_loop(lines):
    labels = {}
    for i, ln in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):", ln)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, ln in enumerate(lines):
        m = re.match(r"\s*s_(?:c)?branch\w* (\.LBB\d+_\d+)", ln)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            h = labels[m.group(1)]
            body = lines[h:i + 1]
            if any("ds_add_u32" in x for x in body) and any("ds_read_u8" in x for x in body) and \
                    300 < i - h < 2000 and (best is None or i - h < best[1] - best[0]):
                best = (h, i + 1)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "netsniff-ng_amd", "csrc", "nsd_kernels.hip"))
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        s = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-Wno-unused-function", "--cuda-device-only", "-S", "-o", s, args.src],
                       check=True, stderr=subprocess.DEVNULL)
        text = open(s).read().split("\n")
    i0 = next(i for i, ln in enumerate(text) if ln.startswith(KERNEL) and ln.split(";")[0].rstrip().endswith(":"))
    i1 = next(i for i in range(i0, len(text)) if "s_endpgm" in text[i])
    fn = text[i0:i1 + 1]
    h, e = find_loop(fn)
    bl = blocks_of(fn[h:e])
    keys = ("valu", "salu", "lds", "vmem", "branch", "wait")
    rows = [f"step loop of {KERNEL} (dissect_all<PRINT_NORM, compact>), {e - h} asm lines",
            "block            " + " ".join(f"{k:>6s}" for k in keys) + "  branches"]
    tot = {k: 0 for k in keys}
    for b in bl:
        for k in keys:
            tot[k] += b["n"].get(k, 0)
        rows.append(f"{b['label']:16s} " + " ".join(f"{b['n'].get(k, 0):6d}" for k in keys) + "  " +
                    " | ".join(b["to"]))
    rows.append("loop total       " + " ".join(f"{tot[k]:6d}" for k in keys))
    out = "\n".join(rows) + "\n"
    if args.out:
        open(args.out, "w").write(out)
    print(out, end="")


if __name__ == "__main__":
    main()
