"""GPU tests of context-lifecycle hazards in the C-ABI (csrc/spg_api.cpp), each against the oracle.

* a contig switch (spg_set_reference) right after a calls-only fused finalize: the records that finalize
  left unwritten are re-folded under the reference they were accumulated with (first-visit REF chars,
  live_variant_caller.py:77-85), not the new one;
* reset / accumulate(other runs) / finalize in a loop with no result read in between: each step's
  descriptor upload reads the pinned mirror the next step rewrites;
* the run kernel's error word is reported once and cleared: a reset context works again.
"""
import numpy as np
import pytest

import spings  # noqa: F401
from oracle.c_oracle import COracle
from oracle_util import compare_variants

pytestmark = pytest.mark.gpu
RTOL = 1e-9


def _engine(n_pos, ref, calls_only=True):
    from covid_spings_variant_caller_amd.engine import PileupEngine
    return PileupEngine(n_pos, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=calls_only)


def test_contig_switch_after_fused_finalize_keeps_first_visit_ref():
    """process_bam(contig A) -> prepare_variants() (fused: records of non-calling positions unwritten) ->
    process_bam(contig B, shorter, REF differs at covered positions) -> prepare_variants(): REF chars and
    calls as the reference's memory (keyed by position, REF stored at the first visit) gives them."""
    from covid_spings_variant_caller_amd import synth
    from oracle.reference_port import OracleCaller
    LA, LB = 3000, 1500
    refA = synth.reference(LA, seed=501)
    bA = synth.pileup(LA, 30, seed=502, ref=refA, snv_every=23)
    covered = np.diff(bA[1].astype(np.int64)) > 0
    # contig B: A's first LB chars, every 5th covered position changed (a REF that only B would give)
    rb = list(refA[:LB])
    for p in range(0, LB, 5):
        if covered[p]:
            rb[p] = {"A": "C", "C": "G", "G": "T", "T": "A"}[rb[p]]
    refB = "".join(rb)
    bB = synth.pileup(LB, 30, seed=503, ref=refB, snv_every=29)
    eng = _engine(LA, refA)
    eng.accumulate(*bA)
    eng.finalize()
    oA = OracleCaller(refA, 30, 10, 5, 0.10)
    oA.accumulate(*bA)
    compare_variants(eng.variants(), oA.prepare_variants(), RTOL)
    eng.set_reference(refB)
    eng.accumulate(*bB)
    eng.finalize()
    # oracle: positions first visited by A keep refA's char; those first visited by B get refB's
    first_ref = "".join(refA[p] if (p >= LB or covered[p]) else refB[p] for p in range(LA))
    o = OracleCaller(first_ref, 30, 10, 5, 0.10)
    o.accumulate(*bA)
    o.accumulate(*bB)
    exp = o.prepare_variants()
    assert len(exp) > 30
    compare_variants(eng.variants(), exp, RTOL)
    eng.close()


def test_reset_accumulate_finalize_loop_without_reads():
    """12 steps of reset / accumulate_batches(a different run of host batches) / finalize with nothing read
    back in between; then the last step's calls equal the oracle's for that step's run."""
    from covid_spings_variant_caller_amd import synth
    L = 4000
    ref = synth.reference(L, seed=601)
    runs = []
    for s in range(12):
        runs.append([synth.pileup(L, 25 + 5 * (s % 3), seed=700 + 10 * s + i, ref=ref, snv_every=17 + s,
                                  lo=(37 * i) % 300, hi=L - (53 * i) % 300) for i in range(6 + s % 4)])
    eng = _engine(L, ref)
    for run in runs:
        eng.reset()
        eng.accumulate_batches(run)
        eng.finalize()
    got = eng.variants()
    orc = COracle(ref, 30, 10, 5, 0.10)
    for b in runs[-1]:
        orc.accumulate(*b)
    orc.finalize()
    compare_variants(got, orc.variants(), RTOL)
    eng.close()


def test_run_error_is_reported_once_and_cleared_by_reset():
    """A run holding a batch with 2^30 entries in one tile (16 columns: the batch's mean depth puts 4 lanes on
    a column) fails its settle (the record path's shallow kernel, k_acc_tile, does not fold a tile that size;
    a full-table context, so the finalize takes that path rather than calls-only counting); after reset the
    context accumulates and finalizes normally again."""
    import torch
    from covid_spings_variant_caller_amd import synth
    dev = torch.device("cuda", 0)
    n_cols = 1 << 23
    ref = synth.reference(n_cols, seed=801)
    big = 1 << 30
    lens = torch.zeros(n_cols, dtype=torch.int64, device=dev)
    lens[:16] = big // 16
    off = torch.zeros(n_cols + 1, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(lens, 0)
    codes = torch.ones(big + 16, dtype=torch.uint8, device=dev)
    quals = torch.full((big + 16,), 35, dtype=torch.uint8, device=dev)
    small = synth.pileup(n_cols, 0.01, seed=802, ref=ref, lo=1000, hi=3000)
    so, sc, sq = synth.to_device(small[1], small[2], small[3])
    torch.cuda.synchronize()
    eng = _engine(n_cols, ref, calls_only=False)
    eng.accumulate_batches([(0, off, codes, quals, big), (1000, so, sc, sq, len(small[2]))], device=True, borrow=True)
    eng.finalize()
    with pytest.raises(RuntimeError):
        eng.counts()
    eng.reset()
    b = synth.pileup(n_cols, 0.01, seed=803, ref=ref, snv_every=7, lo=5000, hi=9000)
    eng.accumulate(*b)
    eng.finalize()
    orc = COracle(ref, 30, 10, 5, 0.10)
    orc.accumulate(*b)
    orc.finalize()
    compare_variants(eng.variants(), orc.variants(), RTOL)
    eng.close()
    del codes, quals
    torch.cuda.empty_cache()
