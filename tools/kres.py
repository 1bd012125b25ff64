"""Per-kernel resource usage of a HIP source for gfx950 (VGPRs, SGPRs, spills,
LDS, occupancy) from hipcc -Rpass-analysis=kernel-resource-usage.
usage: python tools/kres.py netsniff-ng_amd/csrc/nsd_kernels.hip [-DNAME=V ...]"""
import re
import subprocess
import sys

src, extra = sys.argv[1], sys.argv[2:]
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src,
                    "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"] + extra,
                   stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
cur, rows = None, []
for line in r.stdout.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": subprocess.run(["c++filt"], input=t.split(":", 1)[1].strip(), text=True,
                                      stdout=subprocess.PIPE).stdout.strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for c in rows:
    print(f"{c['name'][:70]:72s} vgpr={c.get('VGPRs')} agpr={c.get('AGPRs')} sgpr={c.get('TotalSGPRs')} "
          f"vspill={c.get('VGPRs Spill')} sspill={c.get('SGPRs Spill')} lds={c.get('LDS Size [bytes/block]')} "
          f"occ={c.get('Occupancy [waves/SIMD]')}")
sys.exit(r.returncode)
