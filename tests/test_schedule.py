"""The adaptive kernel schedule (nsd_launch_dissect_rec):
with no schedule forced, batches whose packets mostly go to the general
walk (C4's IPv6 extension chains) or leave many ICMPv4 checksums to a pass
(C3 IMIX) switch the launches to the fused kernel, batches the fast walk
finishes (C2) switch them back to the split kernels, and the records stay
those of the oracle throughout."""
import numpy as np
import pytest

import nsd
import nsd_testlib as T

pytestmark = pytest.mark.gpu


def _walk(torch, f, d):
    crec, ext, used, cnt = nsd.dissect_device_compact(f, d)
    torch.cuda.synchronize()
    return crec.cpu().numpy().view(nsd.CREC_DTYPE), cnt.cpu().numpy().view(np.uint64)


def test_adaptive_schedule_follows_the_traffic():
    import torch
    prev = nsd.set_schedule(nsd.SCHED_ADAPTIVE)
    try:
        batches = {}
        for cfg in (T.SYN_IPV6X, T.SYN_UDP64, T.SYN_IMIX):
            frames, desc = T.make_batch(cfg, 1 << 16)
            orec, oext, ocnt, _ = T.oracle_records(frames, desc)
            want, _ = nsd.compact_of(orec, oext)
            batches[cfg] = (torch.from_numpy(frames).cuda(), torch.from_numpy(desc.view(np.int64)).cuda(), want,
                            ocnt)
        for cfg, sched in ((T.SYN_IPV6X, "fused"), (T.SYN_UDP64, "split"), (T.SYN_IMIX, "fused"),
                           (T.SYN_UDP64, "split"), (T.SYN_IPV6X, "fused")):
            f, d, want, ocnt = batches[cfg]
            seen = []
            for _ in range(160):
                crec, cnt = _walk(torch, f, d)
                seen.append(nsd.last_schedule())
                assert np.array_equal(cnt, ocnt)
                for fld in ("ip_csum", "nflags", "nlayers"):
                    assert np.array_equal(crec[fld], want[fld]), fld
            assert seen[-1] == sched, f"config {cfg}: schedule {seen[-1]} after 160 launches, want {sched}"
            assert seen.count(sched) > 60
    finally:
        nsd.set_schedule(prev)
