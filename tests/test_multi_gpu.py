"""spg_multi_* (csrc/spg_multi.cpp): the one-process multi-device context of the C-ABI — coordinate cuts on the
first batch, host batches sliced at them, one RCCL ncclGather of the call tables.  On the one-GPU box it runs
with n = 1 (the cuts, the slicing, the gather and the merge order all exercised); the merged table must equal a
single context's and the oracle's.  (Multi-device runs: unmeasured on hardware until the driver's 8-GPU node.)"""
import numpy as np
import pytest

import spings  # noqa: F401
from oracle.c_oracle import COracle

pytestmark = pytest.mark.gpu


def test_multi_n1_equals_single_context_and_oracle():
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.multi import MultiEngine
    L = 20_000
    ref = synth.reference(L, seed=17)
    batches = [synth.pileup(L, 40, seed=18 + i, ref=ref, snv_every=61, lo=(i * 1500) % 6000, hi=L - (i * 700) % 5000)
               for i in range(6)]
    m = MultiEngine([0], L, reference=ref)
    s = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    orc = COracle(ref, 30, 10, 5, 0.10)
    for b in batches:
        m.accumulate(*b)
        s.accumulate(*b)
        orc.accumulate(*b)
    assert list(m.partition()) == [0, L]
    m.finalize()
    s.finalize()
    orc.finalize()
    got, one = m.candidates(), s.candidates()
    assert len(got) > 50
    assert got.tobytes() == one.tobytes()
    exp = orc.variants()
    assert [int(x) for x in got["pos"]] == [v["start"] for v in exp]
    # a second sample: reset, a batch that starts later (new cuts), and an empty-slice-free n = 1 run
    m.reset()
    s.reset()
    for b in batches[3:]:
        m.accumulate(*b)
        s.accumulate(*b)
    m.finalize()
    s.finalize()
    assert m.candidates().tobytes() == s.candidates().tobytes()
    m.close()
    s.close()
