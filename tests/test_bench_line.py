"""bench.py's line fields that need no GPU: the roofline's algorithmic bytes,
line floor and traffic ratios from the committed goldens (wsum.json,
lines.json), the CPU baseline's shape (the reference's objects as `value`),
and the library's source provenance."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import nsd  # noqa: E402


def _fake_batch(key, n=1 << 24):
    b = object.__new__(bench.Batch)
    b.key, b.n_shard, b.shards, b.n, b.compact, b.rec_b = key, n, 1, n, True, bench.CREC_B
    b.wsum = bench.wsum_for(key, n, 0)
    b.lines = bench.lines_for(key, n, 0)
    return b


def test_roofline_line_floor():
    n = 1 << 24
    for key in ("udp64", "imix", "ipv6x"):
        b = _fake_batch(key)
        assert b.wsum is not None and b.lines is not None, key
        floor = 128 * b.lines + 8 * n
        traffic = {"read_bytes": 1.1 * floor, "write_bytes": 2.0 * 8 * n, "bytes_per_launch": 1.1 * floor + 16 * n}
        r = b.roofline(1.0, traffic, None, {"gbs": 7000.0})
        assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
        alg = 8 * n + b.wsum + 8 * n
        assert abs(r["achieved"] - alg / 1e-3 / 1e9) < 0.1
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
        assert r["line_floor_bytes_per_pkt"]["read"] == round(floor / n, 2)
        assert r["traffic_vs_line_floor"] == {"read": 1.1, "write": 2.0}
        assert r["line_floor_bytes_per_pkt"]["read"] >= r["bytes_per_pkt"]["read"] - 1e-9, key
    # C2: 64-byte frames, two to a line: the floor is the algorithmic bytes
    assert _fake_batch("udp64").lines * 128 == 64 * n
    # a shard the tables do not hold gives no floor
    assert bench.lines_for("imix", 1000, 0) is None


def test_golden_counters_cover_c5():
    want = bench.golden_counters("imix", 1 << 24, 8)
    assert want is not None and int(want[nsd.CNT_PKTS]) == 8 << 24


def test_library_info_names_its_sources():
    info = bench.library_info()
    assert info["source_matches_tree"] and info["source_sha256_16"] == nsd.source_hash()
    assert info["build"].endswith(info["source_sha256_16"])
    assert len(info["sha256_16"]) == 16 and int(info["sha256_16"], 16) >= 0


def test_cpu_baseline_value_is_the_reference(monkeypatch):
    """`cpu_baseline.value` is the reference's own objects on the 16-CPU
    share (kind "reference"); the restatement sits beside it as `port`;
    without the reference's objects the port's rate is the value."""
    monkeypatch.setattr(bench, "cpu_rate", lambda cfg, n, th, sec, text: (2.0 if text else 30.0, n, sec))
    monkeypatch.setattr(bench, "ref_harness_rate",
                        lambda cfg, key, n=0, frames=True: {"value": 0.1, "cores": 1, "kind": "reference"})
    monkeypatch.setattr(bench, "ref_harness_all_cores",
                        lambda cfg, key, procs, rate1, seconds=8.0: {"value": 1.5, "cores": procs, "kind": "reference",
                                                                     "sample": f"{key} x{procs}"})
    c = bench.cpu_baseline("udp64", 0.01)
    assert c["kind"] == "reference" and c["value"] == 1.5 and c["cores"] == min(bench.cpu_info()[2], 16)
    assert c["port"]["kind"] == "port" and c["port"]["value"] == 2.0
    assert set(c["reference_harness_all_cores"]) >= {"udp64", "imix"}
    monkeypatch.setattr(bench, "ref_harness_all_cores", lambda *a, **k: None)
    c = bench.cpu_baseline("imix", 0.01)
    assert c["kind"] == "port" and c["value"] == 2.0 and "reference_error" in c
    np.testing.assert_equal(c["text_16threads"]["value"], 2.0)
