import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "netsniff-ng_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP kernels)")


@pytest.fixture(scope="session", autouse=True)
def native_build():
    """Build the C test infrastructure (tools/, oracle/, oracle/_ref when the
    reference tree is present) and the product library when it is missing or
    was built from other sources than the tree's (the source hash it carries,
    nsd.ensure_built)."""
    import nsd
    import nsd_testlib
    nsd_testlib.build_native()
    nsd.ensure_built()
    yield


def _schedule(request):
    import nsd
    prev = nsd.set_schedule(nsd.SCHED_SPLIT if request.param == "split" else nsd.SCHED_FUSED)
    ring = nsd.set_record_ring(nsd.RING_OFF if request.param == "fused_noring" else nsd.RING_ON)
    if request.param.startswith("fused_grid"):
        nsd.set_grid_cap(int(request.param[len("fused_grid"):]))
    yield request.param
    nsd.set_schedule(prev)
    nsd.set_record_ring(ring)
    nsd.set_grid_cap(0)


@pytest.fixture(params=["split", "fused", "fused_noring"])
def schedule(request):
    """Runs a parity test under both kernel schedules (nsd_set_schedule): the
    split fast + walker kernels and the fused kernel - with its record ring
    (nsd_set_record_ring) on and off - must each match the oracle; the
    library's adaptive choices are restored after."""
    yield from _schedule(request)


@pytest.fixture(params=["split", "fused", "fused_noring", "fused_grid3", "fused_grid8"])
def schedule_small(request):
    """`schedule` for small batches, plus the fused kernel with its grid
    capped at 3 blocks (nsd_set_grid_cap), so each wave walks many tiles:
    walkers carried across tiles, the pending lists of many tiles, waves of
    a block with unequal tile counts; and at 8 blocks: two CU groups of four
    blocks sharing their tiles through the group counters (walk_tiles), with
    many tiles per wave."""
    yield from _schedule(request)
