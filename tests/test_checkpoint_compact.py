"""Checkpoint compaction (tests/ck_util.bq_compact, the host restatement of spg_history_copy_compact): a batch stored without the entries the
base-quality filter drops gives the same memory (counts, q lists, dict order, first visits) and the same
calls as the full batch, for the C oracle (CPU; the GPU round trip is tests/test_live_caller_gpu.py)."""
import numpy as np
import pytest

import spings  # noqa: F401
from oracle.c_oracle import COracle


@pytest.mark.parametrize("bq", [0, 13, 30])
def test_compacted_batches_same_memory_and_calls(bq):
    from covid_spings_variant_caller_amd import synth
    from ck_util import bq_compact as _bq_compact
    L = 3000
    ref = synth.reference(L, seed=5)
    batches = []
    for s in range(4):
        pb, off, c, q = synth.pileup(L, 25, seed=40 + s, ref=ref, snv_every=37, lo=100 * s, hi=L - 50 * s)
        q = q.copy()
        # columns whose every entry fails the filter (first visits that only a marker entry can keep)
        off64 = off.astype(np.int64)
        for col in range(0, len(off) - 1, 97):
            q[off64[col]:off64[col + 1]] = 2
        batches.append((pb, off, c, q))
    full, comp = COracle(ref, bq, 10, 5, 0.10), COracle(ref, bq, 10, 5, 0.10)
    n_full = n_comp = 0
    for pb, off, c, q in batches:
        full.accumulate(pb, off, c, q)
        o2, c2, q2 = _bq_compact(off, c, q, bq)
        comp.accumulate(pb, o2, c2, q2)
        n_full += len(c)
        n_comp += len(c2)
        assert int(o2[-1]) == len(c2) and len(o2) == len(off)
    full.finalize()
    comp.finalize()
    assert comp.memory_summary() == full.memory_summary()
    assert comp.variants() == full.variants()
    if bq >= 30:
        assert n_comp < 0.8 * n_full
    else:
        assert n_comp <= n_full
