"""GPU parity of the many-BAM path (BASELINE config 4: many BAMs accumulated into one `memory`,
live_variant_caller.py:54-103 once per BAM, vc_queue.py:142-144) against the bit-exact C oracle.

Shallow batches are folded per position in runs (k_acc_multi): a run of K batches reads and writes
each record once, split over batch ranges (k_merge_parts) when the positions alone cannot fill the
chip.  These tests drive >= 1,000 batches through that path, through the one-call entry point
(spg_accumulate_batches) and per-batch calls, with heterogeneous column ranges, depth caps, planted
SNVs, an IUPAC allele and a position whose P product lands in the subnormal band after the run (so
the exact wave-parallel replay walks 1,000 batches through the replay index).
"""
import numpy as np
import pytest

import spings  # noqa: F401
from oracle.c_oracle import COracle
from oracle_util import compare_variants

pytestmark = pytest.mark.gpu

RTOL = 1e-9
DEF = {"minBaseQuality": 30, "minTotalDepth": 10, "minAlleleDepth": 5, "minEvidenceRatio": 0.10}


def _engine(ref, calls_only, n_pos=None):
    from covid_spings_variant_caller_amd.engine import PileupEngine
    return PileupEngine(n_pos or len(ref), DEF["minBaseQuality"], DEF["minTotalDepth"], DEF["minAlleleDepth"],
                        DEF["minEvidenceRatio"], device=0, reference=ref, calls_only=calls_only)


def _oracle(ref):
    return COracle(ref, DEF["minBaseQuality"], DEF["minTotalDepth"], DEF["minAlleleDepth"], DEF["minEvidenceRatio"])


def _plant(batch, pos, code, q):
    """Append one entry (code, q) at the end of column `pos` of a CSR batch."""
    pb, off, c, qq = batch
    col = pos - pb
    if col < 0 or col >= len(off) - 1:
        return batch
    at = int(off[col + 1])
    c = np.insert(c, at, np.uint8(code))
    qq = np.insert(qq, at, np.uint8(q))
    off = off.copy()
    off[col + 1:] += np.uint64(1)
    return pb, off, c, qq


def _many(L, n, depth, seed0, span, band_pos=None, iupac_pos=None, cap=0):
    from covid_spings_variant_caller_amd import synth
    ref = synth.reference(L, seed=seed0)
    out = []
    for i in range(n):
        lo = (i * 131) % max(1, L - span)
        b = synth.pileup(L, depth, seed=seed0 + 1 + i, ref=ref, snv_every=41, lo=lo, hi=min(L, lo + span),
                         max_depth=cap)
        if band_pos is not None and i < 98:
            # 98 x Q31 of a non-REF base: sum(q) >= 3038, at or past the subnormal band
            b = _plant(b, band_pos, 2 if ref[band_pos] != "C" else 4, 31)
        if iupac_pos is not None and i == n // 2:
            b = _plant(b, iupac_pos, 5, 35)         # one 'R' (IUPAC): exotic position, exact replay
        out.append(b)
    return ref, out


def _check(eng, orc, check_mem=True):
    eng.finalize()
    orc.finalize()
    if check_mem:
        assert eng.memory_summary() == orc.memory_summary()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)


@pytest.mark.parametrize("calls_only", [True, False])
def test_1000_batches_one_call_vs_oracle(calls_only):
    L = 1500
    ref, batches = _many(L, 1000, 40, 7000, span=1100, band_pos=700, iupac_pos=710, cap=35)
    # the band position: REF at 700 must not be C for the planted allele to be an extra allele
    eng = _engine(ref, calls_only)
    orc = _oracle(ref)
    eng.accumulate_batches(batches)
    for b in batches:
        orc.accumulate(*b)
    _check(eng, orc)
    t = eng.table()
    assert t["flags"][710] & 12 == 12, "IUPAC position not replayed (exact walk over 1,000 batches)"
    assert eng.counts()[1] >= 1
    assert len(eng.variants()) > 10
    eng.close()


def test_1000_batches_per_call_and_live_finalize():
    """Per-batch accumulate() calls (the live path) with a finalize every 125 BAMs (write_vcf after
    BAMs, vc_queue.py:142-144): each intermediate call table equals the oracle's."""
    L = 1200
    ref, batches = _many(L, 1000, 30, 9100, span=900, band_pos=450)
    eng = _engine(ref, True)
    orc = _oracle(ref)
    for i, b in enumerate(batches):
        eng.accumulate(*b)
        orc.accumulate(*b)
        if (i + 1) % 125 == 0:
            eng.finalize()
            orc.finalize()
            compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    _check(eng, orc)
    eng.close()


def test_unsplit_run_wide_range():
    """A run over enough positions that it is not split over batch ranges (S = 1): 2 batches x 600 kb
    at 30x, plus a deep batch in between (run, k_acc_seg, run)."""
    from covid_spings_variant_caller_amd import synth
    L = 600_000
    ref = synth.reference(L, seed=77)
    b1 = synth.pileup(L, 30, seed=78, ref=ref, snv_every=997, lo=0, hi=L)
    b2 = synth.pileup(L, 25, seed=79, ref=ref, snv_every=991, lo=1000, hi=L - 5000, max_depth=20)
    b3 = synth.pileup(L, 600, seed=80, ref=ref, snv_every=97, lo=200_000, hi=203_000)
    b4 = synth.pileup(L, 30, seed=81, ref=ref, snv_every=997, lo=100, hi=L)
    eng = _engine(ref, True)
    orc = _oracle(ref)
    eng.accumulate_batches([b1, b2])
    eng.accumulate(*b3)
    eng.accumulate(*b4)
    for b in (b1, b2, b3, b4):
        orc.accumulate(*b)
    _check(eng, orc, check_mem=False)
    # counts and dict order at every position (memory_summary at this size is slow in Python)
    got = eng.table()
    m = orc.memory_arrays()
    pos = m["pos"].astype(np.int64)
    np.testing.assert_array_equal(got["depth"][pos].astype(np.uint64), m["depth"])
    eng.close()


def test_device_borrowed_many_batches():
    """Borrowed HBM batches through spg_accumulate_batches (no copy): same calls as host input."""
    import torch
    from covid_spings_variant_caller_amd import synth
    L = 1000
    ref, batches = _many(L, 300, 50, 4200, span=800)
    dev = []
    for pb, off, c, q in batches:
        o, dc, dq = synth.to_device(off, c, q)
        dev.append((pb, o, dc, dq, len(c)))
    torch.cuda.synchronize()
    eng = _engine(ref, True)
    eng.accumulate_batches(dev, device=True, borrow=True)
    orc = _oracle(ref)
    for b in batches:
        orc.accumulate(*b)
    _check(eng, orc)
    eng.close()


def test_pinned_host_batches():
    """Inputs in pinned host memory (spg_host_alloc) are copied asynchronously on the copy stream."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import pinned_empty
    L = 1000
    ref, batches = _many(L, 64, 60, 5200, span=900)
    pinned = []
    for pb, off, c, q in batches:
        po, pc, pq = pinned_empty(len(off), np.uint64), pinned_empty(len(c), np.uint8), pinned_empty(len(q), np.uint8)
        po[:], pc[:], pq[:] = off, c, q
        pinned.append((pb, po, pc, pq))
    eng = _engine(ref, True)
    eng.accumulate_batches(pinned)
    eng.wait_input()
    orc = _oracle(ref)
    for b in batches:
        orc.accumulate(*b)
    _check(eng, orc)
    eng.close()


def test_config4_device_generated_batches_vs_oracle():
    """The bench's config-4 data path: BAM-sized 100x samples generated in HBM (synth_device), fed as
    borrowed spg_batch records (one binding call), coordinate shard [lo, hi) of the genome — calls and
    memory vs the oracle on host copies of the same batches."""
    import torch
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.synth_device import many_bams
    L = 29903
    ref = synth.reference(L, seed=1)
    lo, hi = 11000, 13500
    data = many_bams(ref, 400, 100, seed=1000, lo=lo, hi=hi, max_depth=8000, device=torch.device("cuda", 0))
    torch.cuda.synchronize()
    eng = PileupEngine(hi - lo, 30, 10, 5, 0.10, device=0, reference=ref[lo:hi], calls_only=True)
    eng.accumulate_records(data.records(pos_begin=0))
    eng.finalize()
    orc = COracle(ref[lo:hi], 30, 10, 5, 0.10)
    for i in range(len(data)):
        pb, off, c, q = data.host(i)
        orc.accumulate(pb - lo, off, c, q)
    orc.finalize()
    assert eng.memory_summary() == orc.memory_summary()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    assert len(eng.variants()) >= 2
    # twice in a row on the same context (the bench's step: reset + accumulate + finalize)
    eng.reset()
    eng.accumulate_records(data.records(pos_begin=0))
    eng.finalize()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    eng.close()


def _drop_cols(batch, c0, c1):
    """A sample batch with no entries in columns [c0, c1) (the sample does not cover them)."""
    pb, off, c, q = batch
    off = np.asarray(off, np.int64)
    e0, e1 = int(off[c0]), int(off[c1])
    keep = np.r_[np.arange(0, e0), np.arange(e1, len(c))].astype(np.int64)
    off2 = off.copy()
    off2[c0 + 1:c1 + 1] = e0
    off2[c1 + 1:] -= (e1 - e0)
    return pb, off2.astype(np.uint64), c[keep], q[keep]


@pytest.mark.parametrize("calls_only", [True, False])
def test_multisample_batch_equals_sequential_samples(calls_only):
    """spg_accumulate_samples (n BAMs as one column-major batch, the multi-BAM pileup layout) equals n
    per-sample accumulates: memory (first visits by sample, dict order), calls; mixed with ordinary
    batches before and after (batch numbering)."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import samples_to_columns
    L = 3000
    ref = synth.reference(L, seed=31)
    lo, hi = 200, 2600
    samples = [synth.pileup(L, 60, seed=3100 + s, ref=ref, snv_every=29, lo=lo, hi=hi, max_depth=50)
               for s in range(24)]
    samples[0] = _drop_cols(samples[0], 100, 300)        # columns first visited by sample 1 (or later)
    samples[1] = _drop_cols(samples[1], 150, 300)
    samples[2] = _drop_cols(samples[2], 280, 300)
    samples[5] = _plant(samples[5], 900, 5, 35)          # IUPAC in sample 5: exact replay of the batch
    before = synth.pileup(L, 40, seed=3050, ref=ref, snv_every=29, lo=1500, hi=L)
    after = synth.pileup(L, 40, seed=3051, ref=ref, snv_every=29, lo=1000, hi=L)
    pb, off, first, codes, quals = samples_to_columns(samples)
    assert first[150] == 2 and first[290] == 3
    eng = _engine(ref, calls_only)
    orc = _oracle(ref)
    eng.accumulate(*before)
    eng.accumulate_samples(pb, off, first, codes, quals, len(samples))
    eng.accumulate(*after)
    for b in [before] + samples + [after]:
        orc.accumulate(*b)
    _check(eng, orc)
    t = eng.table()
    assert t["first_batch"][lo + 290] == 1 + 1 + 3       # batch 1 = `before`, samples from batch 2
    assert t["flags"][900] & 8
    from covid_spings_variant_caller_amd import _native as N
    import ctypes as C
    ns = C.c_int64()
    fs = np.zeros(hi - lo, np.uint32)
    N.check(eng._L.spg_history_samples(eng._h, 1, C.byref(ns), N.ptr(fs)))
    assert ns.value == len(samples) and np.array_equal(fs, first)
    eng.close()


def test_multisample_device_columns_vs_oracle():
    """The bench's config-4 layout generated in HBM (many_bams_columns), borrowed: calls and memory vs
    the oracle fed the same column-major stream (every column's first sample is 0 here)."""
    import torch
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.synth_device import many_bams_columns
    L = 29903
    ref = synth.reference(L, seed=1)
    lo, hi = 20000, 21500
    d = many_bams_columns(ref, 300, 100, seed=1000, lo=lo, hi=hi, max_depth=8000, device=torch.device("cuda", 0))
    torch.cuda.synchronize()
    first = d.first_sample.cpu().numpy()
    assert (first == 0).all()
    eng = PileupEngine(hi - lo, 30, 10, 5, 0.10, device=0, reference=ref[lo:hi], calls_only=True)
    eng.accumulate_samples(0, d.offsets, d.first_sample, d.codes, d.quals, d.n_samples, borrow=True,
                           n_entries=d.n_entries)
    eng.finalize()
    orc = COracle(ref[lo:hi], 30, 10, 5, 0.10)
    orc.accumulate(0, d.offsets.cpu().numpy().view(np.uint64), d.codes[:d.n_entries].cpu().numpy(),
                   d.quals[:d.n_entries].cpu().numpy())
    orc.finalize()
    assert eng.memory_summary() == orc.memory_summary()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    assert len(eng.variants()) >= 1
    eng.close()


def test_fused_fresh_run_then_more_batches_and_table():
    """A calls-only finalize of one FRESH run (chr1-like: wide range, unsplit) writes records only for
    positions that can produce a call and finalizes just those; the context re-materializes every
    record before it reads them again (another batch, the per-position table, memory)."""
    from covid_spings_variant_caller_amd import synth
    L = 400_000
    ref = synth.reference(L, seed=91)
    b1 = synth.pileup(L, 30, seed=92, ref=ref, snv_every=997, lo=0, hi=L)
    for _ in range(8):                              # IUPAC entries (an exotic allele that can be called): replayed
        b1 = _plant(b1, 123_456, 5, 35)
    b2 = synth.pileup(L, 20, seed=93, ref=ref, snv_every=501, lo=50_000, hi=350_000)
    eng = _engine(ref, True)
    orc = _oracle(ref)
    eng.accumulate(*b1)
    orc.accumulate(*b1)
    eng.finalize()
    orc.finalize()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    assert eng.counts()[1] >= 1                     # the exotic position went through the replay
    eng.accumulate(*b2)                             # records re-materialized first
    orc.accumulate(*b2)
    eng.finalize()
    orc.finalize()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    got = eng.table()                               # full table: every record present
    m = orc.memory_arrays()
    pos = m["pos"].astype(np.int64)
    np.testing.assert_array_equal(got["depth"][pos].astype(np.uint64), m["depth"])
    assert (got["flags"][pos] & 1).all()
    eng.reset()                                     # and a fused step again on a fresh sample
    eng.accumulate(*b2)
    eng.finalize()
    orc2 = _oracle(ref)
    orc2.accumulate(*b2)
    orc2.finalize()
    compare_variants(eng.variants(), orc2.variants(), rtol=RTOL)
    eng.close()


def test_chr1_30x_full_size_count_conservation():
    """BASELINE config 5 at full size (chr1, L = 248,956,422, 30x: E = 7.5e9 > 2^32 entries, generated in
    HBM): a calls-only finalize of the FRESH run (fused path) then the per-position table (records
    re-materialized): every entry with q >= minBaseQuality lands in exactly one position's totalDepth
    and one allele / D / N bucket (process_pileup_column :75-101), so depths equal direct per-column
    counts of the CSR and per-code totals equal direct counts."""
    import ctypes as C
    import torch
    from covid_spings_variant_caller_amd import _native as N, synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.synth_device import many_bams_columns
    L = 248_956_422
    ref = synth.reference(L, seed=1)
    dev = torch.device("cuda", 0)
    d = many_bams_columns(ref, 1, 30.0, seed=7, device=dev)
    E = d.n_entries
    assert E > (1 << 32)
    eng = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    eng.accumulate(0, d.offsets, d.codes, d.quals, borrow=True, n_entries=E)
    eng.finalize()
    n_calls = eng.counts()[0]
    assert n_calls > 10_000
    codes_tot = torch.zeros(32, dtype=torch.int64, device=dev)
    got_tot = np.zeros(8, np.int64)
    off_h = d.offsets.cpu().numpy()
    step = 1 << 25
    depth = np.zeros(step, np.uint32)
    counts = np.zeros((step, 8), np.uint32)
    for c0 in range(0, L, step):
        c1 = min(L, c0 + step)
        e0, e1 = int(off_h[c0]), int(off_h[c1])
        keep = d.quals[e0:e1] >= 30
        cs = torch.zeros(e1 - e0 + 1, dtype=torch.int64, device=dev)
        cs[1:] = torch.cumsum(keep, 0)
        o = d.offsets[c0:c1 + 1] - e0
        want = (cs[o[1:]] - cs[o[:-1]]).cpu().numpy()
        codes_tot += torch.bincount(d.codes[e0:e1][keep].long(), minlength=32)
        n = c1 - c0
        N.check(eng._L.spg_get_table(eng._h, c0, n, N.ptr(depth), N.ptr(counts), None, None, None, None), "table")
        np.testing.assert_array_equal(depth[:n].astype(np.int64), want)
        got_tot += counts[:n].astype(np.int64).sum(axis=0)
        del keep, cs
    want_codes = codes_tot.cpu().numpy()
    assert [int(x) for x in got_tot[:5]] == [int(want_codes[k]) for k in (1, 2, 4, 8, 15)]
    assert int(got_tot[5]) == int(want_codes[16]) and int(got_tot[6]) == int(want_codes[17])
    eng.finalize()                                  # the full finalize agrees with the fused one
    assert eng.counts()[0] == n_calls
    eng.close()
    del d
    torch.cuda.empty_cache()


def test_2500_batches_counted_fold_across_workgroups():
    """A calls-only finalize over 2,500 batches: counted mode's exact fold splits each listed position's history
    over several workgroups (merged in batch order by the last to arrive) — calls, dict order and first visits
    vs the oracle, then the table (re-materialized) vs the oracle's memory."""
    L = 900
    ref, batches = _many(L, 2500, 20, 12000, span=600, band_pos=450, iupac_pos=460, cap=18)
    eng = _engine(ref, True)
    orc = _oracle(ref)
    eng.accumulate_batches(batches)
    for b in batches:
        orc.accumulate(*b)
    eng.finalize()
    orc.finalize()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    assert len(eng.variants()) > 10
    assert eng.memory_summary() == orc.memory_summary()
    eng.close()
