"""Device vs oracle on seeded mutation-fuzz batches (tests/fuzz_cases.py),
several seeds, modes and alignments, both record forms (16-byte records
through the host batch entry, compact records through the device-resident
entry); prints mismatch counts.  GPU box tool:
  python tools/fuzz_device.py [n] [seeds] [split|fused] [ring|noring]
(ring / noring: the fused kernel's record ring forced on / off)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import fuzz_cases  # noqa: E402
import nsd  # noqa: E402
import nsd_testlib as T  # noqa: E402
from test_device_parity import _check_compact, assert_same_records  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
if len(sys.argv) > 3:   # split / fused (default: the adaptive choice)
    nsd.set_schedule({"split": nsd.SCHED_SPLIT, "fused": nsd.SCHED_FUSED}[sys.argv[3]])
if len(sys.argv) > 4:
    nsd.set_record_ring({"ring": nsd.RING_ON, "noring": nsd.RING_OFF}[sys.argv[4]])
fails = 0
for seed in range(seeds):
    for mode, align in ((T.PRINT_NORM, 16), (T.PRINT_LESS, 16), (T.PRINT_NORM, 2)):
        frames, desc = fuzz_cases.fuzz_batch(n, seed=1000 + seed, align=align)
        rec, ext, cnt = nsd.entry_batch(frames, desc, mode=mode)
        orec, oext, ocnt, _ = T.oracle_records(frames, desc, mode=mode)
        try:
            assert_same_records(rec, orec, ext, oext)
            assert np.array_equal(cnt, ocnt), "counters differ"
            _check_compact(frames, desc, mode)
            print(f"seed {1000 + seed} mode {mode} align {align}: {n} records identical (16-B and compact)",
                  flush=True)
        except AssertionError as e:
            fails += 1
            print(f"seed {1000 + seed} mode {mode} align {align}: MISMATCH {e}", flush=True)
sys.exit(1 if fails else 0)
