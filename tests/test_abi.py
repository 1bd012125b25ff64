"""C ABI checks that need no GPU: the product library loads, exports every
entry point declared in include/netsniff_dissect.h, and its pure-host parts
(formatter, wrap, lookups) behave; device calls fail loudly without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

import nsd
import nsd_testlib as T

HDR = os.path.join(T.ROOT, "include", "netsniff_dissect.h")


def declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:[a-z_][\w\s\*]*?)\b([a-z_]\w*)\s*\(", src, flags=re.M)
    return sorted({n for n in names if n not in ("if", "return", "sizeof")})


def test_header_declares_abi():
    decl = set(declared_functions())
    assert set(nsd.ABI_SYMBOLS) <= decl, set(nsd.ABI_SYMBOLS) - decl


def test_library_exports_every_declared_symbol():
    lib = nsd.lib()
    for name in declared_functions():
        assert hasattr(lib, name), f"libnsdissect.so does not export {name}"


def test_record_layout_matches_header():
    assert nsd.REC_DTYPE.itemsize == 16 and nsd.BPF_INSN.itemsize == 8
    assert nsd.ext_words(6) == 20 and nsd.ext_words(16) == 20 and nsd.ext_words(17) == 68
    assert nsd.REC_DTYPE.fields["nflags"][1] == 10 and nsd.REC_DTYPE.fields["off2"][1] == 11


def test_version_and_device_count():
    assert b"netsniff" in nsd.lib().nsd_version()
    assert nsd.lib().nsd_device_count() >= 0


def test_record_ring_knob():
    """nsd_set_record_ring: 0 adaptive / 1 on / 2 off, returns the previous
    setting, refuses anything else (NSD_ERR_ARG)."""
    prev = nsd.set_record_ring(nsd.RING_OFF)
    try:
        assert nsd.set_record_ring(nsd.RING_ON) == nsd.RING_OFF
        assert nsd.set_record_ring(nsd.RING_ADAPTIVE) == nsd.RING_ON
        for bad in (-1, 3):
            with pytest.raises(ValueError):
                nsd.set_record_ring(bad)
    finally:
        nsd.set_record_ring(prev)


def test_library_carries_the_tree_source_hash():
    """The library names the sources it was built from (nsd_build_info's
    `sources` hash, the Makefile's SRCHASH) and they are this tree's: what
    a bench line's `library` reports and the test fixture rebuilds on."""
    info = nsd.lib().nsd_build_info().decode()
    assert re.search(r"; sources [0-9a-f]{16}$", info), info
    assert info.endswith(nsd.source_hash()) and nsd.built_source_hash() == nsd.source_hash()


def test_device_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    frames, desc = T.batch_from_packets([b"\x00" * 64])
    with pytest.raises(nsd.NsdError):
        nsd.entry_batch(frames, desc)


def test_replay_fails_loudly_without_gpu(tmp_path):
    """`--in` through the library needs the device walk: without a GPU the
    replay reports an error (no CPU fallback), the pcap reader alone works."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    path = str(tmp_path / "x.pcap")
    T.write_pcap(path, [b"\x00" * 64] * 3)
    assert len(nsd.pcap_frame_hdrs(path)[1]) == 3
    with pytest.raises(nsd.NsdError):
        nsd.replay_pcap(path)


def test_format_rejects_inconsistent_record():
    frames, desc = T.make_batch(T.SYN_UDP64, 4)
    rec, ext, _, _ = T.oracle_records(frames, desc)
    bad = rec.copy()
    bad["data_off"] += 2               # claims a cursor the bytes do not give
    _, rc = nsd.format_batch(frames, desc, bad, ext)
    assert (rc != 0).all()
    bad = rec.copy()
    bad["off2"][:, 1] += 1             # wrong UDP layer start
    _, rc = nsd.format_batch(frames, desc, bad, ext)
    assert (rc != 0).all()


def test_wrap_basics():
    out, st = nsd.tprintf_wrap(b"x" * 100 + b"\n", cols=80)
    assert out == b"x" * 75 + b"\n   " + b"x" * 25 + b"\n"
    assert st == 0
    # wrap point on spaces/commas: they are dropped
    out, _ = nsd.tprintf_wrap(b"a" * 75 + b" , b\n", cols=80)
    assert out == b"a" * 75 + b"\n   b\n"
    # colour sequences suppress wrapping until closed
    s = b"\033[1m" + b"y" * 90 + b"\033[0m\n"
    out, _ = nsd.tprintf_wrap(s, cols=80)
    assert out.count(b"\n   ") == 1
