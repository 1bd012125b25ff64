"""Full-size parity (BASELINE.json configs C2 / C3 / C4: 16,777,216 packets
per GPU) through size-independent properties, on an MI355X:

* sampled oracle parity: 65,536 random packets plus the first and last
  4,096 of the batch (the last grid strides, the tail tile) bit-exact vs the
  CPU oracle, ext chains resolved on both sides;
* determinism: a second launch over the same resident batch gives the same
  records, ext chains and counters (ext slots may land elsewhere in the pool);
* shard independence (what the multi-GPU split relies on): the two halves
  walked as separate batches give the full batch's records and their
  counter vectors sum to the full one's;
* counter consistency: the per-ops counters equal the layer ids tallied over
  the records (ext chains included)."""
import numpy as np
import pytest

import nsd
import nsd_testlib as T
from test_device_parity import _chain

pytestmark = pytest.mark.gpu

N = 1 << 24


def _run(torch, f, d):
    rec, ext, used, cnt = nsd.dissect_device(f, d, mode=T.PRINT_NORM)
    torch.cuda.synchronize()
    return (rec.cpu().numpy().view(nsd.REC_DTYPE), ext.cpu().numpy().view(np.uint32)[:int(used.item())].copy(),
            cnt.cpu().numpy().view(np.uint64).copy())


def _ids(rec, ext, i):
    """(ids, offs) of record i with the ext entry's packet index dropped."""
    r = rec[i]
    if (int(r["nflags"]) & 7) == 7:
        slot = int.from_bytes(bytes(r["off2"][:4]), "little")
        if slot == 0xFFFFFFFF:
            return ("overflow",)
        _, ids, offs = nsd.ext_entry(ext, slot)
        return ids, offs
    return _chain(rec, ext, i)


@pytest.mark.parametrize("cfg", [T.SYN_UDP64, T.SYN_IMIX, T.SYN_IPV6X])
def test_full_size_properties(cfg):
    import torch
    frames, desc = T.make_batch(cfg, N, threads=16)
    f = torch.from_numpy(frames).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    rec, ext, cnt = _run(torch, f, d)
    assert int(cnt.sum()) > 0

    # sampled oracle parity
    rng = np.random.default_rng(cfg)
    idx = np.unique(np.concatenate([rng.integers(0, N, 1 << 16), np.arange(4096), np.arange(N - 4096, N)]))
    orec, oext, _, _ = T.oracle_records(frames, desc[idx])
    srec = rec[idx]
    for fld in ("data_off", "tail_off", "ip_csum", "nflags", "chain"):
        bad = np.nonzero(srec[fld] != orec[fld])[0]
        assert len(bad) == 0, f"{fld} differs at packets {idx[bad[:10]]}"
    nonext = (orec["nflags"] & 7) != 7
    assert np.array_equal(srec["off2"][nonext], orec["off2"][nonext])
    for k in np.nonzero(~nonext)[0]:
        assert _ids(rec, ext, int(idx[k])) == _ids(orec, oext, int(k)), f"ext chain differs at {idx[k]}"

    # determinism
    # (an ext record's slot is where its wave's pool chunk landed, which
    # depends on launch timing: the chain behind it must be the same)
    rec2, ext2, cnt2 = _run(torch, f, d)
    for fld in ("data_off", "tail_off", "ip_csum", "nflags", "chain"):
        assert np.array_equal(rec2[fld], rec[fld]), fld
    ext_rec = np.nonzero((rec["nflags"] & 7) == 7)[0]
    nonext_all = (rec["nflags"] & 7) != 7
    assert np.array_equal(rec2["off2"][nonext_all], rec["off2"][nonext_all])
    assert np.array_equal(cnt2, cnt)
    for i in ext_rec[:: max(1, len(ext_rec) // 2000)]:
        assert _ids(rec2, ext2, int(i)) == _ids(rec, ext, int(i))

    # shard independence: halves as separate batches
    h = N // 2
    ra, exa, ca = _run(torch, f, d[:h])
    rb, exb, cb = _run(torch, f, d[h:])
    same = ["data_off", "tail_off", "ip_csum", "nflags", "chain"]
    for fld in same:
        assert np.array_equal(np.concatenate([ra[fld], rb[fld]]), rec[fld]), fld
    assert np.array_equal(ca + cb, cnt)

    # counters vs the records: per-ops counts = layer ids over every chain
    assert int(cnt[32]) == N and int(cnt[38]) == 0          # NSD_CNT_PKTS, NSD_CNT_OVERFLOW
    ops = np.zeros(32, dtype=np.uint64)
    nl = rec["nflags"] & 7
    for k in range(6):
        m = (nl != 7) & (nl > k)
        ids = ((rec["chain"][m] >> np.uint32(5 * k)) & 31).astype(np.int64)
        ops += np.bincount(ids, minlength=32).astype(np.uint64)
    if len(ext_rec):
        slots = rec["off2"][ext_rec][:, :4].copy().view(np.uint32).ravel().astype(np.int64)
        assert np.array_equal(ext[slots], ext_rec.astype(np.uint32))   # entry's packet index
        enl = (ext[slots + 1] & 0xFFFF).astype(np.int64)
        for k in range(int(enl.max())):
            m = enl > k
            ids = (ext[slots[m] + nsd.EXT_HDR_WORDS + k] & 0xFF).astype(np.int64)
            ops += np.bincount(ids, minlength=32).astype(np.uint64)
    assert np.array_equal(cnt[:32], ops)
