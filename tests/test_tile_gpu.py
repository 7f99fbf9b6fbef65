"""GPU parity of the shallow-batch kernel k_acc_tile (csrc/spg_tile.hip) against the bit-exact C oracle.

k_acc_tile folds one shallow batch (process_bam's columns, live_variant_caller.py:54-103) or a run of
them (many BAMs into one `memory`, vc_queue.py:142-144): LDS-DMA tile staging, LPC lanes per column
(1, 2, 4, 8 by the batch's mean depth), the tile bytes past the 2 KiB slot read from memory, runs split
over batch ranges.  Each case here drives one of those shapes and compares memory (counts, dict order,
first visits) and the call table with the oracle; calls-only contexts decide their calls without it (k_acc_lite for a
lone batch of <= 40 entries per column, else counted mode) and re-materialize every record through it for the table.
"""
import numpy as np
import pytest

import spings  # noqa: F401
from oracle.c_oracle import COracle
from oracle_util import compare_variants

pytestmark = pytest.mark.gpu

RTOL = 1e-9
DEF = dict(minBaseQuality=30, minTotalDepth=10, minAlleleDepth=5, minEvidenceRatio=0.10)


def _engine(ref, p, calls_only):
    from covid_spings_variant_caller_amd.engine import PileupEngine
    return PileupEngine(len(ref), p["minBaseQuality"], p["minTotalDepth"], p["minAlleleDepth"], p["minEvidenceRatio"],
                        device=0, reference=ref, calls_only=calls_only)


def _oracle(ref, p):
    return COracle(ref, p["minBaseQuality"], p["minTotalDepth"], p["minAlleleDepth"], p["minEvidenceRatio"])


def _run(ref, batches, p, calls_only, one_call=False, check_mem=True):
    eng, orc = _engine(ref, p, calls_only), _oracle(ref, p)
    if one_call:
        eng.accumulate_batches(batches)
    for b in batches:
        if not one_call:
            eng.accumulate(*b)
        orc.accumulate(*b)
    eng.finalize()
    orc.finalize()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    if check_mem:
        assert eng.memory_summary() == orc.memory_summary()
    else:
        got = eng.table()
        m = orc.memory_arrays()
        pos = m["pos"].astype(np.int64)
        np.testing.assert_array_equal(got["depth"][pos].astype(np.uint64), m["depth"])
    return eng, orc


def _splice(outer, inner):
    """CSR batch `outer` with the columns of `inner` (a sub-range of the same positions) swapped in."""
    pb, off, c, q = outer
    ib, ioff, ic, iq = inner
    c0, c1 = ib - pb, ib - pb + len(ioff) - 1
    off = np.asarray(off, np.int64)
    ioff = np.asarray(ioff, np.int64)
    e0, e1 = int(off[c0]), int(off[c1])
    codes = np.concatenate([c[:e0], ic, c[e1:]])
    quals = np.concatenate([q[:e0], iq, q[e1:]])
    lens = np.diff(off)
    lens[c0:c1] = np.diff(ioff)
    off2 = np.zeros(len(off), np.uint64)
    np.cumsum(lens, out=off2[1:])
    return pb, off2, codes, quals


@pytest.mark.parametrize("calls_only", [True, False])
@pytest.mark.parametrize("depth", [8, 30, 45, 90, 180])
def test_single_batch_lpc_by_depth(depth, calls_only):
    """One batch per depth class: LPC 1 (8x, 30x), 2 (45x), 4 (90x), 8 (180x)."""
    from covid_spings_variant_caller_amd import synth
    L = 40_000 if depth < 100 else 12_000
    ref = synth.reference(L, seed=depth)
    b = synth.pileup(L, depth, seed=depth + 1, ref=ref, snv_every=53, lo=17, hi=L - 3)
    eng, _ = _run(ref, [b], DEF, calls_only)
    assert len(eng.variants()) > 20
    eng.close()


@pytest.mark.parametrize("calls_only", [True, False])
def test_single_batch_tiles_past_the_slot(calls_only):
    """30x with a 120x region (columns < 128 entries: not listed as deep): those tiles hold ~7.7 KB per
    array, far past the 2 KiB DMA slot, and are finished from memory; planted SNVs there make the fused
    form recompute the REF sums of their columns across the slot boundary."""
    from covid_spings_variant_caller_amd import synth
    L = 60_000
    ref = synth.reference(L, seed=41)
    base = synth.pileup(L, 30, seed=42, ref=ref, snv_every=97)
    hot = synth.pileup(L, 120, seed=43, ref=ref, snv_every=7, lo=20_000, hi=23_000, max_depth=127)
    b = _splice(base, hot)
    eng, _ = _run(ref, [b], DEF, calls_only)
    assert sum(1 for v in eng.variants() if 20_000 <= v["start"] < 23_000) > 100
    eng.close()


@pytest.mark.parametrize("calls_only", [True, False])
@pytest.mark.parametrize("depth", [20, 60, 100])
def test_runs_of_batches_with_shifted_ranges(depth, calls_only):
    """Runs of 120 batches whose [lo, hi) ranges start and end inside tiles (columns before a batch's first
    column and past its last), folded in one call and split over batch ranges (few tiles, many batches)."""
    from covid_spings_variant_caller_amd import synth
    L = 5_000
    ref = synth.reference(L, seed=depth + 100)
    bs = []
    for i in range(120):
        lo = (i * 37) % 700
        hi = L - (i * 53) % 900
        bs.append(synth.pileup(L, depth, seed=5000 + i, ref=ref, snv_every=31, lo=lo, hi=hi, max_depth=depth + 20))
    eng, _ = _run(ref, bs, DEF, calls_only, one_call=True)
    assert len(eng.variants()) > 50
    eng.close()


@pytest.mark.parametrize("bq", [0, 4, 30])
def test_rare_qualities_in_shallow_tiles(bq):
    """Q0..Q3, Q127/128 and Q200/255 entries (the exact per-entry path: LUT rows past 127, q lower bounds
    under 4, eps(Q0) = 1) in a 30x batch, single batch and a run."""
    from covid_spings_variant_caller_amd import synth
    L = 20_000
    ref = synth.reference(L, seed=61)
    out = []
    for s in range(3):
        lo, off, c, q = synth.pileup(L, 30, seed=62 + s, ref=ref, snv_every=17)
        rng = np.random.default_rng(bq + s)
        q = q.copy()
        m = rng.random(len(q)) < 0.03
        q[m] = rng.choice(np.array([0, 1, 2, 3, 127, 128, 200, 255], np.uint8), size=m.sum())
        out.append((lo, off, c, q))
    p = dict(DEF, minBaseQuality=bq, minEvidenceRatio=0.05, minAlleleDepth=3)
    for calls_only in (True, False):
        eng, _ = _run(ref, out[:1], p, calls_only)
        eng.close()
        eng, _ = _run(ref, out, p, calls_only, one_call=True)
        eng.close()


def test_chr_scale_single_batch_fused_vs_oracle():
    """A 4 Mb 30x batch (chr1's shape, ~62,500 tiles): the fused calls-only finalize vs the oracle, then the
    full per-position table (records re-materialized) vs the oracle's depths."""
    from covid_spings_variant_caller_amd import synth
    L = 4_000_000
    ref = synth.reference(L, seed=71)
    b = synth.pileup(L, 30, seed=72, ref=ref, snv_every=997)
    eng, orc = _run(ref, [b], DEF, True, check_mem=False)
    assert len(eng.variants()) > 1000
    eng.close()


@pytest.mark.parametrize("calls_only", [True, False])
def test_lite_single_batch_shapes(calls_only):
    """The fused single-batch kernel k_acc_lite (csrc/spg_lite.hip; calls-only, mean column <= 40 entries):
    a 30x batch over [13, L - 29) (tiles cut by the batch range) with a 55-70x region (columns straddling the
    61-entry prefetch window: the rest of the column from memory), a 200x region (columns >= 128 entries,
    listed for k_acc_seg<1>) and a region with IUPAC / deletion / skip codes (exotic alleles: exact replay).
    Plain mode (calls_only False) takes k_acc_tile on the same batch."""
    from covid_spings_variant_caller_amd import synth
    L = 50_000
    ref = synth.reference(L, seed=91)
    b = synth.pileup(L, 30, seed=92, ref=ref, snv_every=41, lo=13, hi=L - 29)
    b = _splice(b, synth.pileup(L, 65, seed=93, ref=ref, snv_every=11, lo=10_000, hi=12_000, max_depth=70))
    b = _splice(b, synth.pileup(L, 200, seed=94, ref=ref, snv_every=13, lo=20_000, hi=20_500))
    pb, off, c, q = b
    c = c.copy()
    off = np.asarray(off, np.int64)
    e0, e1 = int(off[30_000 - pb]), int(off[31_000 - pb])
    rng = np.random.default_rng(95)
    m = np.zeros(len(c), bool)
    m[e0:e1] = rng.random(e1 - e0) < 0.01
    c[m] = rng.choice(np.array([5, 16, 17, 0], np.uint8), size=m.sum())
    eng, _ = _run(ref, [(pb, off.astype(np.uint64), c, q)], DEF, calls_only, check_mem=not calls_only)
    v = eng.variants()
    assert sum(1 for x in v if 10_000 <= x["start"] < 12_000) > 50
    assert sum(1 for x in v if 20_000 <= x["start"] < 20_500) > 10
    eng.close()


def test_lite_offsets_past_2_32():
    """k_acc_lite with every CSR offset above 2^32 (the device batch arrays open with 2^32 bytes no column
    references; offsets index them as given): the tile bases, the slot-overflow reads of a 120x stretch and the
    exact fold all address past 4 GiB.  Calls vs the oracle on the same columns."""
    import torch
    from covid_spings_variant_caller_amd import synth
    dev = torch.device("cuda", 0)
    L = 60_000
    ref = synth.reference(L, seed=121)
    b = synth.pileup(L, 30, seed=122, ref=ref, snv_every=89)
    b = _splice(b, synth.pileup(L, 120, seed=123, ref=ref, snv_every=7, lo=30_000, hi=33_000, max_depth=127))
    pb, off, c, q = b
    SH = 1 << 32
    E = len(c)
    codes = torch.zeros(SH + E + 16, dtype=torch.uint8, device=dev)
    quals = torch.zeros(SH + E + 16, dtype=torch.uint8, device=dev)
    codes[SH:SH + E] = torch.from_numpy(np.ascontiguousarray(c)).to(dev)
    quals[SH:SH + E] = torch.from_numpy(np.ascontiguousarray(q)).to(dev)
    d_off = torch.from_numpy(np.asarray(off, np.int64) + SH).to(dev)
    torch.cuda.synchronize()
    eng = _engine(ref, DEF, True)
    eng.accumulate(pb, d_off, codes, quals, borrow=True, n_entries=E)
    eng.finalize()
    orc = _oracle(ref, DEF)
    orc.accumulate(*b)
    orc.finalize()
    got = eng.variants()
    compare_variants(got, orc.variants(), rtol=RTOL)
    assert sum(1 for v in got if 30_000 <= v["start"] < 33_000) > 100
    eng.close()
    del codes, quals
    torch.cuda.empty_cache()
