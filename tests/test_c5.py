"""C5 (BASELINE.json configs[4]: 128M IMIX frames sharded across 8 GPUs) on
ONE MI355X: the 8 contiguous 16M-packet shards of the same seeded stream
(shard r = packets [r*16M, (r+1)*16M), exactly what rank r of `bench.py
--gpus 8 --config imix` walks) resident together in one 47.6 GB buffer.

* every shard walked as its own batch gives the records the whole 128M
  batch gives for those packets (what the 8-GPU split relies on), and the
  shards' counter vectors sum to the whole batch's (the RCCL all-reduce);
* every record of all 134,217,728 packets is bit-exact against the CPU
  oracle (multi-threaded fields walk over each shard's host copy);
* the same for the compact 8-byte records bench.py times (shards vs whole,
  every record vs nsd.compact_of(oracle), counters);
* the counters equal the oracle's, and the oracle's sum of algorithmic read
  bytes W per shard equals the committed tests/golden/wsum.json entry
  (the bench's roofline denominator for that shard)."""
import json
import os

import numpy as np
import pytest

import nsd
import nsd_testlib as T

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("schedule")]

SHARD = 1 << 24
SHARDS = 8


@pytest.mark.timeout(600)
def test_c5_shards_on_one_gpu():
    import torch
    with open(os.path.join(T.GOLDEN, "wsum.json")) as f:
        wsum = json.load(f)
    n = SHARD * SHARDS
    orecs = []
    ocnt = np.zeros(nsd.NCOUNTERS, dtype=np.uint64)
    osw = []

    def check_chunk(a, host, d):
        rec = np.zeros(len(d), dtype=T.REC_DTYPE)
        cnt = np.zeros(nsd.NCOUNTERS, dtype=np.uint64)
        sw = T.oracle().nsor_dissect_batch_mt(host.ctypes.data, d.ctypes.data, len(d), 1, T.PRINT_NORM,
                                              rec.ctypes.data, cnt.ctypes.data, 16)
        assert not ((rec["nflags"] & 7) == 7).any(), "IMIX chains fit the 16-byte record"
        orecs.append(rec)
        ocnt[:] += cnt
        osw.append(int(sw))

    frames, desc, _ = T.make_device_batch(T.SYN_IMIX, n, lo=0, chunk=SHARD, on_chunk=check_chunk)
    assert len(orecs) == SHARDS
    for r in range(SHARDS):
        assert osw[r] == wsum[f"imix:{r * SHARD}:{SHARD}"], f"shard {r}: sum W"

    ext = torch.empty(nsd.ext_pool_words(n // 64), dtype=torch.int32, device="cuda")
    ws = torch.empty(nsd.lib().nsd_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    rec_all = torch.empty(n * nsd.REC_BYTES, dtype=torch.uint8, device="cuda")
    used = torch.zeros(1, dtype=torch.int32, device="cuda")
    cnt_all = torch.zeros(nsd.NCOUNTERS, dtype=torch.int64, device="cuda")
    nsd.dissect_device(frames, desc, rec=rec_all, ext=ext, ext_used=used, counters=cnt_all, workspace=ws)
    torch.cuda.synchronize()
    cnt_all = cnt_all.cpu().numpy().view(np.uint64)
    assert int(cnt_all[nsd.CNT_PKTS]) == n and int(cnt_all[nsd.CNT_OVERFLOW]) == 0
    assert np.array_equal(cnt_all, ocnt), "whole-batch counters vs oracle"

    rec_sh = torch.empty(SHARD * nsd.REC_BYTES, dtype=torch.uint8, device="cuda")
    cnt_sum = np.zeros(nsd.NCOUNTERS, dtype=np.uint64)
    for r in range(SHARDS):
        cnt_r = torch.zeros(nsd.NCOUNTERS, dtype=torch.int64, device="cuda")
        used.zero_()
        nsd.dissect_device(frames, desc[r * SHARD:(r + 1) * SHARD], rec=rec_sh, ext=ext, ext_used=used,
                           counters=cnt_r, workspace=ws)
        torch.cuda.synchronize()
        whole = rec_all[r * SHARD * nsd.REC_BYTES:(r + 1) * SHARD * nsd.REC_BYTES]
        assert torch.equal(rec_sh, whole), f"shard {r}: shard batch != whole batch"
        cnt_sum += cnt_r.cpu().numpy().view(np.uint64)
        got = whole.cpu().numpy().view(nsd.REC_DTYPE)
        want = orecs[r]
        for fld in ("chain", "data_off", "tail_off", "ip_csum", "nflags", "off2"):
            bad = np.nonzero((got[fld] != want[fld]).reshape(SHARD, -1).any(axis=1))[0]
            assert len(bad) == 0, f"shard {r}: {fld} differs at packets {(bad[:10] + r * SHARD).tolist()}"
    assert np.array_equal(cnt_sum, cnt_all), "sum of shard counters != whole batch"
    del rec_all, rec_sh
    torch.cuda.empty_cache()

    # the compact form (the one bench.py times): 8 shards vs the whole batch,
    # every record against the oracle's (IMIX chains are inline: <= 6 layers)
    crec_all = torch.empty(n * nsd.CREC_BYTES, dtype=torch.uint8, device="cuda")
    ccnt_all = torch.zeros(nsd.NCOUNTERS, dtype=torch.int64, device="cuda")
    used.zero_()
    nsd.dissect_device_compact(frames, desc, crec=crec_all, ext=ext, ext_used=used, counters=ccnt_all,
                               workspace=ws)
    torch.cuda.synchronize()
    assert np.array_equal(ccnt_all.cpu().numpy().view(np.uint64), ocnt), "compact whole-batch counters vs oracle"
    crec_sh = torch.empty(SHARD * nsd.CREC_BYTES, dtype=torch.uint8, device="cuda")
    csum = np.zeros(nsd.NCOUNTERS, dtype=np.uint64)
    for r in range(SHARDS):
        cnt_r = torch.zeros(nsd.NCOUNTERS, dtype=torch.int64, device="cuda")
        used.zero_()
        nsd.dissect_device_compact(frames, desc[r * SHARD:(r + 1) * SHARD], crec=crec_sh, ext=ext,
                                   ext_used=used, counters=cnt_r, workspace=ws)
        torch.cuda.synchronize()
        whole = crec_all[r * SHARD * nsd.CREC_BYTES:(r + 1) * SHARD * nsd.CREC_BYTES]
        assert torch.equal(crec_sh, whole), f"shard {r}: compact shard batch != whole batch"
        csum += cnt_r.cpu().numpy().view(np.uint64)
        got = whole.cpu().numpy().view(nsd.CREC_DTYPE)
        want, _ = nsd.compact_of(orecs[r])
        for fld in ("chain", "ip_csum", "nflags", "nlayers"):
            bad = np.nonzero(got[fld] != want[fld])[0]
            assert len(bad) == 0, f"shard {r}: compact {fld} differs at packets {(bad[:10] + r * SHARD).tolist()}"
    assert np.array_equal(csum, ocnt), "sum of compact shard counters != oracle"
