"""The reference's per-packet surface, linked the way netsniff-ng links it
(INTEGRATION.md): a C program (tests/c/entry_harness.c) built against
libnsdissect.so with its own tprintf / tprintf_flush runs
dissector_init_all(mode) -> dissector_entry_point per pcap record ->
dissector_cleanup_all, and its text must equal the golden text of the
reference's own parser objects byte for byte, in all five print modes,
names off and on (tests/golden/, oracle/_ref/nsref).

The per-packet entry runs on the host CPU (nsd_proto.cpp): its
walk is the product's layer step (nsd_walk.h gen_step) with a host byte
source, checked here against the oracle on the edge and fuzz frames.  No
GPU is involved, so these run in the CPU suite."""
import os
import subprocess

import numpy as np
import pytest

import edge_cases
import fuzz_cases
import nsd
import nsd_testlib as T
from test_golden import load_golden

LIBDIR = os.path.join(T.ROOT, "netsniff-ng_amd")
REF_CONF = "/root/reference"


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("harness") / "entry_harness")
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-Wall", "-o", exe, os.path.join(T.ROOT, "tests", "c", "entry_harness.c"),
                    "-L" + LIBDIR, "-lnsdissect", "-Wl,-rpath," + LIBDIR], check=True)
    return exe


def run_harness(exe, pcap, mode, tmp_path, etc=None, cols=65535):
    txt, ends = str(tmp_path / f"m{mode}.txt"), str(tmp_path / f"m{mode}.ends")
    args = [exe, "-m", str(mode), "-w", str(cols)] + (["-e", etc] if etc else []) + [pcap, txt, ends]
    r = subprocess.run(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert r.returncode == 0, f"harness rc={r.returncode}: {r.stderr[-2000:]!r}"
    with open(txt, "rb") as f:
        data = f.read()
    out, prev = [], 0
    for e in np.fromfile(ends, dtype=np.uint64):
        out.append(data[prev:int(e)])
        prev = int(e)
    return out, r.stderr


@pytest.mark.parametrize("name", ["tiny", "edge", "big"])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS, T.PRINT_HEX, T.PRINT_ASCII, T.PRINT_HEX_ASCII])
def test_entry_point_matches_golden(harness, tmp_path, name, mode):
    gold = load_golden(f"{name}.m{mode}.w65535")
    got, err = run_harness(harness, os.path.join(T.GOLDEN, name + ".pcap"), mode, tmp_path)
    assert len(got) == len(gold)
    bad = [i for i in range(len(gold)) if got[i] != gold[i]]
    assert not bad, f"packets {bad[:10]} differ; first: {got[bad[0]][:300]!r} vs {gold[bad[0]][:300]!r}"
    # no conf dir: lookup_init's message for each of the four tables (lookup.c:48-51)
    assert err.count(b"Port name resolution won't be available.") == 4


@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_entry_point_leaves_match_golden(harness, tmp_path, mode):
    """ARP / DCCP / IGMP / LLDP / ICMPv6 130-154 frames (tests/leaf_cases.py):
    the walk's leaf end (nsd_leaf.h) must agree with the renderer's pulls on
    every layer (run_layer aborts otherwise) and the text, exit-op dump
    included, equals the reference objects' byte for byte."""
    gold = load_golden(f"leaves.m{mode}.w65535")
    got, _ = run_harness(harness, os.path.join(T.GOLDEN, "leaves.pcap"), mode, tmp_path)
    assert len(got) == len(gold)
    bad = [i for i in range(len(gold)) if got[i] != gold[i]]
    assert not bad, f"packets {bad[:10]} differ; first: {got[bad[0]][:400]!r} vs {gold[bad[0]][:400]!r}"


@pytest.mark.parametrize("name", ["tiny", "edge"])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_entry_point_wrapped_80(harness, tmp_path, name, mode):
    """Through netsniff-ng's tprintf at 80 columns (the harness restates
    tprintf.c's buffer and wrap) == the reference objects' wrapped text."""
    gold = load_golden(f"{name}.m{mode}.w80")
    got, _ = run_harness(harness, os.path.join(T.GOLDEN, name + ".pcap"), mode, tmp_path, cols=80)
    bad = [i for i in range(len(gold)) if got[i] != gold[i]]
    assert not bad, f"packets {bad[:10]} differ; first: {got[bad[0]][:300]!r} vs {gold[bad[0]][:300]!r}"


def test_entry_point_print_none(harness, tmp_path):
    got, _ = run_harness(harness, os.path.join(T.GOLDEN, "edge.pcap"), T.PRINT_NONE, tmp_path)
    assert all(t == b"" for t in got)      # dissector.c:70-71


@pytest.mark.skipif(not os.path.isdir(REF_CONF), reason="conf files live in /root/reference")
@pytest.mark.parametrize("name", ["tiny", "edge"])
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_entry_point_names_on(harness, tmp_path, name, mode):
    """dissector_init_all loads udp/tcp/ether/oui.conf from ETCDIRE
    (dissector_eth.c:71-74, dissector_sll.c:104)."""
    gold = load_golden(f"{name}.names.m{mode}.w65535")
    got, err = run_harness(harness, os.path.join(T.GOLDEN, name + ".pcap"), mode, tmp_path, etc=REF_CONF)
    assert b"Cannot open" not in err
    bad = [i for i in range(len(gold)) if got[i] != gold[i]]
    assert not bad, f"packets {bad[:10]} differ"


@pytest.mark.skipif(not os.path.exists(T.REF_BIN), reason="needs oracle/_ref/nsref (built with /root/reference)")
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_entry_point_fuzz_vs_reference(harness, tmp_path, mode):
    """20K mutated frames: the per-packet entry's text vs the reference's
    parser objects, every packet (no layer budget on this path), except
    mobility type 7 whose reference text reads stack bytes (DESIGN.md
    "Parity domain")."""
    pkts = fuzz_cases.mutants(20000)
    path = str(tmp_path / "fuzz.pcap")
    T.write_pcap(path, pkts)
    gold = T.run_ref(path, mode=mode, cols=65535)
    got, _ = run_harness(harness, path, mode, tmp_path)
    bad = [i for i in range(len(pkts)) if got[i] != gold[i] and b"Home Addr (" not in gold[i]]
    assert not bad, f"packets {bad[:10]} differ; first: {got[bad[0]][:400]!r} vs {gold[bad[0]][:400]!r}"


def _assert_cpu_walk_matches_oracle(frames, desc, mode):
    rec, chains, cnt = nsd.walk_cpu(frames, desc, mode=mode)
    orec, oext, ocnt, _ = T.oracle_records(frames, desc, mode=mode)
    for f in ("data_off", "tail_off", "ip_csum", "nflags", "chain"):
        bad = np.nonzero(rec[f] != orec[f])[0]
        assert len(bad) == 0, f"{f} differs at {bad[:10]}"
    nonext = (orec["nflags"] & 7) != 7
    assert np.array_equal(rec["off2"][nonext], orec["off2"][nonext])
    for i in np.nonzero(~nonext)[0]:
        if orec[i]["nflags"] & 0x20:
            continue
        slot = int.from_bytes(bytes(orec[i]["off2"][:4]), "little")
        _, ids, offs = nsd.ext_entry(oext, slot)
        assert chains[int(i)] == (ids, offs), f"ext chain differs at {i}"
    assert np.array_equal(cnt, ocnt)


@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS, T.PRINT_HEX])
def test_cpu_walk_edge_vs_oracle(mode):
    frames, desc = T.batch_from_packets(edge_cases.cases())
    _assert_cpu_walk_matches_oracle(frames, desc, mode)


@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_cpu_walk_leaves_vs_oracle(mode):
    _, pkts = T.read_pcap(os.path.join(T.GOLDEN, "leaves.pcap"))
    frames, desc = T.batch_from_packets(pkts)
    _assert_cpu_walk_matches_oracle(frames, desc, mode)


@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_cpu_walk_fuzz_vs_oracle(mode):
    frames, desc = fuzz_cases.fuzz_batch(20000)
    _assert_cpu_walk_matches_oracle(frames, desc, mode)


def test_entry_point_rate(harness, tmp_path):
    """µs per packet of the per-packet entry on this host (C1's 64-B frames,
    PRINT_NORM, text into the harness's buffer); printed for DESIGN.md."""
    r = subprocess.run([harness, "-m", "0", "-r", "200", os.path.join(T.GOLDEN, "tiny.pcap")],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300, check=True)
    line = r.stdout.decode().strip()
    us = float(line.split("us_per_pkt=")[1])
    print(f"dissector_entry_point C1 PRINT_NORM: {us:.3f} us/packet ({line})")
    assert us > 0
