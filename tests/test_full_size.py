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

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("schedule")]

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


# ---- the compact record form (nsd_crec: the form bench.py times) -------------------
def _run_compact(torch, f, d, mode=T.PRINT_NORM):
    crec, ext, used, cnt = nsd.dissect_device_compact(f, d, mode=mode)
    torch.cuda.synchronize()
    n = d.numel()
    return (crec.cpu().numpy().view(nsd.CREC_DTYPE).copy(),
            ext.cpu().numpy().view(np.uint32)[:n + int(used.item())].copy(),
            cnt.cpu().numpy().view(np.uint64).copy())


def _cids(crec, pool, i):
    """Ops ids of compact record i (batch index i): inline, inline + the side
    word (pool word i), or the ext entry at the record's slot."""
    r = crec[i]
    nl, chain = int(r["nflags"]) & 7, int(r["chain"])
    if nl != 7:
        return tuple((chain >> (5 * k)) & 31 for k in range(nl))
    if int(r["nlayers"]):
        side = int(pool[i])
        return tuple((chain >> (5 * k)) & 31 for k in range(6)) + tuple(
            (side >> (5 * (k - 6))) & 31 for k in range(6, int(r["nlayers"])))
    if chain == 0xFFFFFFFF:
        return ("overflow",)
    pkt, ids, offs = nsd.ext_entry(pool, chain)
    assert pkt == i and not any(offs)
    return ids


def _compact_ops(crec, pool):
    """Per-ops layer counts tallied over every compact chain (vectorised)."""
    ops = np.zeros(32, dtype=np.uint64)
    nl = (crec["nflags"] & 7).astype(np.int64)
    chain = crec["chain"].astype(np.uint64)
    for k in range(6):
        m = (nl != 7) & (nl > k) | (nl == 7) & (crec["nlayers"] > 0)
        ops += np.bincount(((chain[m] >> np.uint64(5 * k)) & np.uint64(31)).astype(np.int64),
                           minlength=32).astype(np.uint64)
    sw = np.nonzero((nl == 7) & (crec["nlayers"] > 0))[0]
    side = pool[sw].astype(np.uint64)
    for k in range(6, 12):
        m = crec["nlayers"][sw] > k
        ops += np.bincount(((side[m] >> np.uint64(5 * (k - 6))) & np.uint64(31)).astype(np.int64),
                           minlength=32).astype(np.uint64)
    for i in np.nonzero((nl == 7) & (crec["nlayers"] == 0))[0]:
        ids = _cids(crec, pool, int(i))
        assert ids != ("overflow",)
        ops += np.bincount(np.array(ids[:nsd.EXT_MAX_LAYERS], dtype=np.int64), minlength=32).astype(np.uint64)
    return ops


@pytest.mark.parametrize("cfg", [T.SYN_UDP64, T.SYN_IMIX, T.SYN_IPV6X])
def test_full_size_compact(cfg):
    """The headline kernel (dissect_all<PRINT_NORM, compact>) at BASELINE's
    16,777,216 packets: sampled records (65,536 random + first/last 4,096)
    equal nsd.compact_of(oracle) field by field with side words and ext
    entries resolved; determinism; two half batches = the whole; counters =
    the oracle's tally over the records."""
    import torch
    frames, desc = T.make_batch(cfg, N, threads=16)
    f = torch.from_numpy(frames).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    crec, pool, cnt = _run_compact(torch, f, d)
    assert int(cnt[nsd.CNT_PKTS]) == N and int(cnt[nsd.CNT_OVERFLOW]) == 0

    rng = np.random.default_rng(cfg + 100)
    idx = np.unique(np.concatenate([rng.integers(0, N, 1 << 16), np.arange(4096), np.arange(N - 4096, N)]))
    orec, oext, _, _ = T.oracle_records(frames, desc[idx])
    want, _ = nsd.compact_of(orec, oext)
    got = crec[idx]
    for fld in ("ip_csum", "nflags", "nlayers"):
        bad = np.nonzero(got[fld] != want[fld])[0]
        assert len(bad) == 0, f"{fld} differs at packets {idx[bad[:10]]}"
    inline = (want["nflags"] & 7) != 7
    assert np.array_equal(got["chain"][inline], want["chain"][inline])
    for k in np.nonzero(~inline)[0]:
        assert _cids(crec, pool, int(idx[k])) == _chain(orec, oext, int(k))[0], f"chain differs at {idx[k]}"

    # determinism (entries may land in other pool slots)
    crec2, pool2, cnt2 = _run_compact(torch, f, d)
    assert np.array_equal(cnt2, cnt)
    for fld in ("ip_csum", "nflags", "nlayers"):
        assert np.array_equal(crec2[fld], crec[fld]), fld
    deep = ((crec["nflags"] & 7) == 7) & (crec["nlayers"] == 0)
    assert np.array_equal(crec2["chain"][~deep], crec["chain"][~deep])
    side = ((crec["nflags"] & 7) == 7) & (crec["nlayers"] > 0)
    assert np.array_equal(pool2[:N][side], pool[:N][side])
    for i in np.nonzero(deep)[0]:
        assert _cids(crec2, pool2, int(i)) == _cids(crec, pool, int(i))

    # two half batches = the whole (what the multi-GPU shards rely on)
    h = N // 2
    ca, pa, na = _run_compact(torch, f, d[:h])
    cb, pb, nb = _run_compact(torch, f, d[h:])
    assert np.array_equal(na + nb, cnt)
    for fld in ("ip_csum", "nflags", "nlayers"):
        assert np.array_equal(np.concatenate([ca[fld], cb[fld]]), crec[fld]), fld
    cat = np.concatenate([ca["chain"], cb["chain"]])
    assert np.array_equal(cat[~deep], crec["chain"][~deep])
    assert np.array_equal(np.concatenate([pa[:h], pb[:N - h]])[side], pool[:N][side])
    for i in np.nonzero(deep)[0]:
        i = int(i)
        half = _cids(ca, pa, i) if i < h else _cids(cb, pb, i - h)
        assert half == _cids(crec, pool, i)

    # counters = the tally over every chain
    assert np.array_equal(cnt[:32], _compact_ops(crec, pool))


@pytest.mark.parametrize("cfg", [T.SYN_IMIX, T.SYN_IPV6X])
def test_full_size_compact_less(cfg):
    """PRINT_LESS at 16,777,216 packets, compact records (the chain without
    the IPv4 trim and checksum, Mobility without its sub-type pulls, ICMPv6
    without its bodies: dissector.c:22-41): sampled
    records equal nsd.compact_of(oracle in PRINT_LESS), counters = the tally
    over every chain."""
    import torch
    frames, desc = T.make_batch(cfg, N, threads=16)
    f = torch.from_numpy(frames).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    crec, pool, cnt = _run_compact(torch, f, d, mode=T.PRINT_LESS)
    assert int(cnt[nsd.CNT_PKTS]) == N and int(cnt[nsd.CNT_OVERFLOW]) == 0
    rng = np.random.default_rng(cfg + 200)
    idx = np.unique(np.concatenate([rng.integers(0, N, 1 << 16), np.arange(4096), np.arange(N - 4096, N)]))
    orec, oext, _, _ = T.oracle_records(frames, desc[idx], mode=T.PRINT_LESS)
    want, _ = nsd.compact_of(orec, oext)
    got = crec[idx]
    for fld in ("ip_csum", "nflags", "nlayers"):
        bad = np.nonzero(got[fld] != want[fld])[0]
        assert len(bad) == 0, f"{fld} differs at packets {idx[bad[:10]]}"
    inline = (want["nflags"] & 7) != 7
    assert np.array_equal(got["chain"][inline], want["chain"][inline])
    for k in np.nonzero(~inline)[0]:
        assert _cids(crec, pool, int(idx[k])) == _chain(orec, oext, int(k))[0], f"chain differs at {idx[k]}"
    assert np.array_equal(cnt[:32], _compact_ops(crec, pool))
