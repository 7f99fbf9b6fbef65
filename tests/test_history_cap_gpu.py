"""Bounded replay history (csrc/spg_api.cpp enforce_history_cap / spill_batch): with a small HBM cap the
engine's own batch copies move to pinned host memory once folded, and every reader of the history — the
exact replay of band positions, the exact record of IUPAC positions, the counted mode's fold of the positions
that may call, a full re-materialization for the table — reads them there.  Calls, memory and the table
against the oracle."""
import numpy as np
import pytest

import spings  # noqa: F401
from oracle.c_oracle import COracle
from oracle_util import compare_variants
from test_many_batches_gpu import _many

pytestmark = pytest.mark.gpu
RTOL = 1e-9


def _engine(ref, calls_only):
    from covid_spings_variant_caller_amd.engine import PileupEngine
    return PileupEngine(len(ref), 30, 10, 5, 0.10, device=0, reference=ref, calls_only=calls_only)


@pytest.mark.parametrize("calls_only", [True, False])
def test_spilled_history_band_and_iupac_replays(calls_only):
    """300 batches (~60 KB each) under a 2 MB cap: ~270 spilled.  A band position (98 x Q31 of a non-REF
    base: exact replay over the history) and an IUPAC allele (exotic: exact replay) at positions whose batches
    are mostly on the host; per-batch accumulate calls with a finalize every 100 batches, then the table."""
    L = 1500
    ref, batches = _many(L, 300, 40, 9900, span=1100, band_pos=700, iupac_pos=710, cap=35)
    eng = _engine(ref, calls_only)
    eng.set_history_cap(2 << 20)
    orc = COracle(ref, 30, 10, 5, 0.10)
    for i, b in enumerate(batches):
        eng.accumulate(*b)
        orc.accumulate(*b)
        if (i + 1) % 100 == 0:
            eng.finalize()
            orc.finalize()
            compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    dev, n_sp, arena = eng.history_resident()
    assert n_sp >= 200, (dev, n_sp, arena)
    assert dev <= (2 << 20) + (256 << 10)
    t = eng.table()                                # every record: re-materialized from the host copies
    assert eng.counts()[1] >= 1                    # the table's exact replays ran over spilled batches
    assert t["flags"][710] & 12 == 12
    assert eng.memory_summary() == orc.memory_summary()
    eng.close()


def test_cap_set_after_accumulating_and_reset():
    """A cap set after 200 batches spills what is folded at once; a reset frees the host copies and the next
    sample runs uncapped in HBM again (0 = no cap)."""
    L = 1200
    ref, batches = _many(L, 200, 30, 5100, span=900, band_pos=450)
    eng = _engine(ref, True)
    orc = COracle(ref, 30, 10, 5, 0.10)
    eng.accumulate_batches(batches)
    for b in batches:
        orc.accumulate(*b)
    eng.finalize()
    eng.set_history_cap(1 << 20)
    assert eng.history_resident()[1] > 100
    orc.finalize()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    eng.finalize()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    eng.reset()
    eng.set_history_cap(0)
    assert eng.history_resident()[:2] == (0, 0)
    eng.accumulate_batches(batches[:50])
    o2 = COracle(ref, 30, 10, 5, 0.10)
    for b in batches[:50]:
        o2.accumulate(*b)
    eng.finalize()
    o2.finalize()
    compare_variants(eng.variants(), o2.variants(), rtol=RTOL)
    assert eng.history_resident()[1] == 0
    eng.close()
