"""Write the inputs of fmt_bench.cpp (C2 frames, descriptors, compact
records and side words from the CPU oracle, frame header fields) to a dir."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
import nsd  # noqa: E402
import nsd_testlib as T  # noqa: E402

d, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
os.makedirs(d, exist_ok=True)
f, desc = T.make_batch(T.SYN_UDP64, n)
rec, ext, _, _ = T.oracle_records(f, desc)
crec, pool = nsd.compact_of(rec, ext)
pool = np.asarray(pool, np.uint32)
if len(pool) < n:
    pool = np.concatenate([pool, np.zeros(n - len(pool), np.uint32)])
fh = np.zeros(n, dtype=nsd.FH_DTYPE)
fh["sec"] = np.arange(n)
fh["len"] = T.desc_caplen(desc)
for nm, a in (("frames", f), ("desc", desc), ("crec", np.ascontiguousarray(crec)), ("pool", pool), ("fh", fh)):
    a.tofile(os.path.join(d, nm + ".bin"))
