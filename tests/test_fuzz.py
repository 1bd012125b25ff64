"""Mutation-fuzz parity (tests/fuzz_cases.py): 20K perturbed frames.

CPU: the product formatter, fed the oracle's records, prints exactly what the
reference's own parser objects print (oracle/_ref/nsref, built where
/root/reference exists) for every record that holds a full chain; the
oracle's text agrees wherever it restates the parser.
GPU: device records and counters equal the oracle's, bit for bit."""
import os

import numpy as np
import pytest

import fuzz_cases
import nsd
import nsd_testlib as T

N = 20000


@pytest.mark.skipif(not os.path.exists(T.REF_BIN), reason="needs oracle/_ref/nsref (built with /root/reference)")
@pytest.mark.parametrize("mode", [T.PRINT_NORM, T.PRINT_LESS])
def test_fuzz_formatter_vs_reference(tmp_path, mode):
    pkts = fuzz_cases.mutants(N)
    path = str(tmp_path / "fuzz.pcap")
    T.write_pcap(path, pkts)
    gold = T.run_ref(path, mode=mode, cols=65535)
    frames, desc = T.batch_from_packets(pkts)
    rec, ext, _, _ = T.oracle_records(frames, desc, mode=mode)
    texts, rc = nsd.format_batch(frames, desc, rec, ext, mode=mode)
    ora = T.oracle_text_packets(frames, desc, mode=mode)
    assert len(gold) == N
    compared = 0
    for i in range(N):
        if rec[i]["nflags"] & 0x20:          # layer-budget overflow: no full chain in the record
            continue
        assert rc[i] == 0, f"packet {i}: status {rc[i]}"
        assert texts[i] == gold[i], f"packet {i}: formatter text differs"
        if not ora[i][1]:
            assert ora[i][0] == gold[i], f"packet {i}: oracle text differs"
        compared += 1
    assert compared > N * 0.99


@pytest.mark.gpu
@pytest.mark.usefixtures("schedule")
@pytest.mark.parametrize("mode,align", [(T.PRINT_NORM, 16), (T.PRINT_LESS, 16), (T.PRINT_NORM, 1)])
def test_fuzz_device_vs_oracle(mode, align):
    from test_device_parity import assert_same_records
    frames, desc = fuzz_cases.fuzz_batch(N, align=align)
    rec, ext, cnt = nsd.entry_batch(frames, desc, mode=mode)
    orec, oext, ocnt, _ = T.oracle_records(frames, desc, mode=mode)
    assert_same_records(rec, orec, ext, oext)
    assert np.array_equal(cnt, ocnt)
