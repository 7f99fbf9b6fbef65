"""GPU parity: the HIP engine (through the C-ABI) vs. the oracle.

* golden cases (outputs of the reference's own code, tests/golden/cases.json)
* seeded synthetic pileups vs. the bit-exact C restatement (oracle/spg_oracle.c), including
  1,000x and 10,000x depth windows, 100,000x columns (uncapped), shallow 30x columns,
  multi-batch accumulation and the device-input (borrowed HBM) path.

Bar: counts, depth, dict order, REF, DP/AD/PL/SCORE and exact zeros bit-exact; GL and QUAL within
1e-9 relative (north star; QUAL is a re-ordered fp64 sum).  Positions resolved by the exact replay
(subnormal band, IUPAC) are compared bit-exactly for GL.
"""
import math

import numpy as np
import pytest

import spings  # noqa: F401
from oracle.c_oracle import COracle
from oracle_util import (batches_np, compare_variants, gl_expected, load_golden, variants_expected)

pytestmark = pytest.mark.gpu

RTOL = 1e-9
GOLD = load_golden()
CASES = GOLD["cases"]


def _engine(reference, p, n_pos=None, calls_only=False):
    from covid_spings_variant_caller_amd.engine import PileupEngine
    return PileupEngine(n_pos or len(reference), p["minBaseQuality"], p["minTotalDepth"], p["minAlleleDepth"],
                        p["minEvidenceRatio"], device=0, reference=reference, calls_only=calls_only)


def _cmp_gl(got, exp, replayed=()):
    assert list(got.keys()) == list(exp.keys()) or sorted(got) == sorted(exp)
    for pos in exp:
        assert list(got[pos].keys()) == list(exp[pos].keys()), (pos, got[pos], exp[pos])
        for a, e in exp[pos].items():
            g = got[pos][a]
            if pos in replayed:
                assert float(g).hex() == float(e).hex(), (pos, a, g, e)
            elif e == 0 or g == 0:
                assert g == e, (pos, a, g, e)
            else:
                assert abs(g - e) <= RTOL * abs(e), (pos, a, g, e)


def _sorted_mem(m):
    return m


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_case(case):
    eng = _engine(case["reference"], case["params"])
    for pb, off, c, q in batches_np(case):
        eng.accumulate(pb, off, c, q)
    eng.finalize()
    assert eng.memory_summary() == case["expected"]["memory"]
    t = eng.table()
    replayed = set(np.nonzero(t["flags"] & 4)[0].tolist())
    _cmp_gl(eng.gl_table(), gl_expected(case), replayed)
    compare_variants(eng.variants(), variants_expected(case), rtol=RTOL)
    eng.close()


def test_band_case_is_replayed_exactly():
    case = next(c for c in CASES if c["name"] == "band")
    eng = _engine(case["reference"], case["params"])
    for pb, off, c, q in batches_np(case):
        eng.accumulate(pb, off, c, q)
    eng.finalize()
    t = eng.table()
    assert (t["flags"] & 4).sum() > 0     # some positions needed the exact replay
    exp = gl_expected(case)
    for pos, row in exp.items():
        for a, v in row.items():
            if 0 < v < 2.2250738585072014e-308:
                assert t["flags"][pos] & 4, pos


def _vs_oracle(reference, batches, p, check_mem=True, calls_only=False, eng=None):
    eng = eng if eng is not None else _engine(reference, p, calls_only=calls_only)
    orc = COracle(reference, p["minBaseQuality"], p["minTotalDepth"], p["minAlleleDepth"], p["minEvidenceRatio"])
    for pb, off, c, q in batches:
        eng.accumulate(pb, off, c, q)
        orc.accumulate(pb, off, c, q)
    eng.finalize()
    orc.finalize()
    # calls-only: the call table of THIS finalize (a single deep batch runs it fused into k_acc_seg);
    # table() below re-finalizes with the per-position table
    first_calls = eng.variants() if calls_only else None
    if check_mem:
        assert eng.memory_summary() == orc.memory_summary()
    t = eng.table()
    replayed = set(np.nonzero(t["flags"] & 4)[0].tolist())
    if calls_only:
        # table GLs: exact where computed; NaN only at positions flagged SPG_F_PARTIAL
        got, exp = eng.gl_table(), orc.gl_table()
        partial = set(np.nonzero(t["flags"] & 32)[0].tolist())
        for pos in exp:
            for a, e in exp[pos].items():
                g = got[pos][a]
                if math.isnan(g):
                    assert pos in partial, (pos, a)
                elif pos in replayed:
                    assert float(g).hex() == float(e).hex(), (pos, a, g, e)
                elif e == 0 or g == 0:
                    assert g == e, (pos, a, g, e)
                else:
                    assert abs(g - e) <= RTOL * abs(e), (pos, a, g, e)
    else:
        _cmp_gl(eng.gl_table(), orc.gl_table(), replayed)
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    if first_calls is not None:
        compare_variants(first_calls, orc.variants(), rtol=RTOL)
    return eng, orc


DEF = {"minBaseQuality": 30, "minTotalDepth": 10, "minAlleleDepth": 5, "minEvidenceRatio": 0.10}


def test_sars_1000x_window():
    from covid_spings_variant_caller_amd import synth
    L = 29903
    ref = synth.reference(L)
    b = synth.pileup(L, 1000, seed=2, ref=ref, snv_every=97, lo=0, hi=6000)
    eng, _ = _vs_oracle(ref, [b], DEF)
    assert len(eng.variants()) > 20


def test_sars_10000x_window():
    from covid_spings_variant_caller_amd import synth
    L = 29903
    ref = synth.reference(L)
    b = synth.pileup(L, 10000, seed=3, ref=ref, snv_every=37, lo=12000, hi=13500)
    _vs_oracle(ref, [b], dict(DEF, minEvidenceRatio=0.01))


def test_100000x_columns_uncapped():
    from covid_spings_variant_caller_amd import synth
    L = 2000
    ref = synth.reference(L, seed=5)
    b = synth.pileup(L, 100000, seed=4, ref=ref, snv_every=11, lo=900, hi=960)
    _vs_oracle(ref, [b], dict(DEF, minEvidenceRatio=0.01))


def test_shallow_30x_lane_path():
    from covid_spings_variant_caller_amd import synth
    L = 400000
    ref = synth.reference(L, seed=6)
    b = synth.pileup(L, 30, seed=7, ref=ref, snv_every=101)
    _vs_oracle(ref, [b], DEF)


@pytest.mark.parametrize("bq", [0, 4, 13, 30, 60])
def test_min_base_quality_sweep(bq):
    from covid_spings_variant_caller_amd import synth
    L = 3000
    ref = synth.reference(L, seed=8)
    lo, off, c, q = synth.pileup(L, 400, seed=9, ref=ref, snv_every=13)
    rng = np.random.default_rng(bq)
    q = q.copy()
    m = rng.random(len(q)) < 0.02
    q[m] = rng.choice(np.array([0, 1, 2, 3, 4, 127, 128, 200, 255], np.uint8), size=m.sum())
    _vs_oracle(ref, [(lo, off, c, q)], dict(DEF, minBaseQuality=bq, minEvidenceRatio=0.02, minAlleleDepth=2))


@pytest.mark.parametrize("calls_only", [False, True])
def test_multibatch_accumulation_and_order(calls_only):
    from covid_spings_variant_caller_amd import synth
    L = 5000
    ref = synth.reference(L, seed=10)
    batches = [synth.pileup(L, 300, seed=20 + i, ref=ref, snv_every=17, lo=lo, hi=hi)
               for i, (lo, hi) in enumerate([(2000, 4000), (0, 2500), (3500, 5000), (1000, 1200)])]
    _vs_oracle(ref, batches, DEF, calls_only=calls_only)


@pytest.mark.parametrize("calls_only", [False, True])
def test_shallow_then_deep_then_shallow(calls_only):
    """Lane-kernel (shallow) FRESH records written partially, then merged by the deep kernel and the
    lane kernel again: stale bytes of absent slots must never leak into the sums."""
    from covid_spings_variant_caller_amd import synth
    L = 3000
    ref = synth.reference(L, seed=40)
    batches = [synth.pileup(L, 30, seed=41, ref=ref, snv_every=13, lo=0, hi=2000, read_len=40),
               synth.pileup(L, 3000, seed=42, ref=ref, snv_every=13, lo=500, hi=2500, read_len=60),
               synth.pileup(L, 20, seed=43, ref=ref, snv_every=13, lo=1000, hi=3000, read_len=40)]
    # a first epoch leaves stale records behind (reset is an epoch bump, not a memset)
    eng = _engine(ref, DEF, calls_only=calls_only)
    eng.accumulate(*synth.pileup(L, 500, seed=44, ref=ref, snv_every=7, lo=0, hi=L))
    eng.finalize()
    eng.reset()
    _vs_oracle(ref, batches, DEF, calls_only=calls_only, eng=eng)


def test_device_borrowed_input_matches_host_input():
    import torch
    from covid_spings_variant_caller_amd import synth
    L = 29903
    ref = synth.reference(L)
    lo, off, c, q = synth.pileup(L, 2000, seed=11, ref=ref, lo=5000, hi=9000)
    host = _engine(ref, DEF)
    host.accumulate(lo, off, c, q)
    host.finalize()
    dev = _engine(ref, DEF)
    do, dc, dq = synth.to_device(off, c, q)
    dev.accumulate(lo, do, dc, dq, borrow=True, n_entries=len(c))
    dev.finalize()
    th, td = host.table(), dev.table()
    for k in th:
        np.testing.assert_array_equal(th[k], td[k])
    assert host.variants() == dev.variants()
    # reset + reuse (bench step shape)
    dev.reset()
    dev.accumulate(lo, do, dc, dq, borrow=True, n_entries=len(c))
    dev.finalize()
    t2 = dev.table()
    for k in th:
        np.testing.assert_array_equal(th[k], t2[k])
    torch.cuda.synchronize()


@pytest.mark.parametrize("calls_only", [False, True])
def test_offsets_beyond_2_31(calls_only):
    """Device CSR whose entries sit past byte 2^31 of the code/qual buffers (a 100,000x SARS-CoV-2
    batch reaches 3e9): the deep kernel's segment base must widen the CSR offsets unsigned."""
    import torch
    from covid_spings_variant_caller_amd import synth
    L = 2000
    ref = synth.reference(L, seed=8)
    lo, off, c, q = synth.pileup(L, 10000, seed=9, ref=ref, snv_every=7, lo=900, hi=1020)
    E = len(c)
    host = _engine(ref, DEF, calls_only=calls_only)
    host.accumulate(lo, off, c, q)
    host.finalize()
    base = (1 << 31) - 4 * 1024 - 5           # columns straddle 2^31; unaligned start
    n = base + E + 64
    dc = torch.empty(n, dtype=torch.uint8, device="cuda")
    dq = torch.empty(n, dtype=torch.uint8, device="cuda")
    dc[base:base + E] = torch.from_numpy(c).cuda()
    dq[base:base + E] = torch.from_numpy(q).cuda()
    dc[base + E:].fill_(0xFF)
    dq[base + E:].zero_()
    do = torch.from_numpy((off.astype(np.int64) + base)).cuda()
    dev = _engine(ref, DEF, calls_only=calls_only)
    dev.accumulate(lo, do, dc, dq, borrow=True, n_entries=E)
    dev.finalize()
    assert dev.memory_summary() == host.memory_summary()
    # another 16-B alignment of the entries regroups the fp64 sums (QUAL / GL): tolerance, not bits
    compare_variants(dev.variants(), host.variants(), rtol=RTOL)
    del dc, dq
    torch.cuda.empty_cache()


def test_empty_and_degenerate_batches():
    ref = "ACGT" * 50
    eng = _engine(ref, DEF)
    eng.accumulate(0, np.zeros(1, np.uint64), np.zeros(0, np.uint8), np.zeros(0, np.uint8))   # 0 columns
    eng.accumulate(10, np.zeros(6, np.uint64), np.zeros(0, np.uint8), np.zeros(0, np.uint8))  # empty columns
    eng.finalize()
    assert eng.memory_summary() == []
    assert eng.variants() == []
    with pytest.raises(Exception):
        eng.accumulate(199, np.array([0, 1, 2], np.uint64), np.array([1, 1], np.uint8), np.array([30, 30], np.uint8))
    with pytest.raises(Exception):
        eng.accumulate(0, np.array([0, 1], np.uint64), np.array([18], np.uint8), np.array([30], np.uint8))


def test_reference_switch_between_batches_replays_skipped_eps():
    """Positions are keyed by coordinate only (live_variant_caller.py:77-87): a later batch read
    against another contig's sequence keeps the REF char of the first visit.  The deep kernel skips
    the eps sum of a column's major allele when it equals the *current* REF char; when that allele
    is a candidate against the stored REF, the position must come out of the exact replay."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from oracle.reference_port import OracleCaller
    L = 400
    r1 = synth.reference(L, seed=31)
    r2 = "".join("G" if (i % 7 == 3) else ch for i, ch in enumerate(synth.reference(L, seed=32)))
    b1 = synth.pileup(L, 40, seed=33, ref=r1, lo=0, hi=L, read_len=50)
    b2 = synth.pileup(L, 4000, seed=34, ref=r2, lo=60, hi=340, read_len=50)     # deep: k_acc_seg<4>
    eng = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=r1)
    eng.accumulate(*b1)
    eng.set_reference(r2)
    eng.accumulate(*b2)
    eng.finalize()
    o = OracleCaller(r1, 30, 10, 5, 0.10)
    o.accumulate(*b1)
    o.accumulate(*b2)
    exp = o.prepare_variants()
    assert len(exp) > 20
    compare_variants(eng.variants(), exp, RTOL)


def test_copy_candidates_device_orders_torch_stream():
    """spg_copy_candidates_device + spg_stream: the call table lands in a torch tensor and torch's
    stream waits for it without a host sync (the path bench.py's RCCL gather uses)."""
    import torch
    from covid_spings_variant_caller_amd import _native as N
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    L = 5000
    ref = synth.reference(L, seed=8)
    pb, off, c, q = synth.pileup(L, 400, seed=9, ref=ref, snv_every=53)
    do, dc, dq = synth.to_device(off, c, q)
    eng = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref)
    buf = torch.zeros(8 + 4096 * 56, dtype=torch.uint8, device="cuda:0")
    for _ in range(3):
        eng.reset()
        eng.accumulate(pb, do, dc, dq, borrow=True, n_entries=len(c))
        eng.finalize()
        eng.copy_candidates_device(buf)
        host = buf.cpu().numpy()                     # torch's stream, ordered after the copy
        n = int(host[:8].view(np.uint64)[0])
        got = host[8:8 + n * 56].view(N.CANDIDATE_DTYPE)
        exp = eng.candidates()
        assert n == len(exp) > 10
        got = got[np.lexsort((got["rank"], got["pos"], got["first_batch"]))]
        assert got.tobytes() == exp.tobytes()


@pytest.mark.parametrize("case", ["sars1000", "sars10000", "col100000", "shallow", "bq0", "bq13", "switch"])
def test_calls_only_mode_matches_oracle(case):
    """SPG_P_CALLS_ONLY (what LiveVariantCaller and bench.py run): calls bit-exact / within 1e-9 of
    the oracle on every workload shape; table GLs exact where computed."""
    from covid_spings_variant_caller_amd import synth
    if case == "sars1000":
        ref = synth.reference(29903)
        eng, _ = _vs_oracle(ref, [synth.pileup(29903, 1000, seed=2, ref=ref, snv_every=97, lo=0, hi=6000)], DEF,
                            calls_only=True)
        assert (eng.table()["flags"] & 32).sum() > 1000      # the mode is active
    elif case == "sars10000":
        ref = synth.reference(29903)
        _vs_oracle(ref, [synth.pileup(29903, 10000, seed=3, ref=ref, snv_every=37, lo=12000, hi=13500)],
                   dict(DEF, minEvidenceRatio=0.01), calls_only=True)
    elif case == "col100000":
        ref = synth.reference(2000, seed=5)
        _vs_oracle(ref, [synth.pileup(2000, 100000, seed=4, ref=ref, snv_every=11, lo=900, hi=960)],
                   dict(DEF, minEvidenceRatio=0.01), calls_only=True)
    elif case == "shallow":
        ref = synth.reference(400000, seed=6)
        _vs_oracle(ref, [synth.pileup(400000, 30, seed=7, ref=ref, snv_every=101)], DEF, calls_only=True)
    elif case in ("bq0", "bq13"):
        bq = int(case[2:])
        ref = synth.reference(6000, seed=12)
        b = synth.pileup(6000, 3000, seed=13, ref=ref, snv_every=29, lo=1000, hi=2500)
        _vs_oracle(ref, [b], dict(DEF, minBaseQuality=bq, minEvidenceRatio=0.02), calls_only=True)
    else:
        from covid_spings_variant_caller_amd.engine import PileupEngine
        from oracle.reference_port import OracleCaller
        L = 400
        r1 = synth.reference(L, seed=31)
        r2 = "".join("G" if (i % 7 == 3) else ch for i, ch in enumerate(synth.reference(L, seed=32)))
        b1 = synth.pileup(L, 40, seed=33, ref=r1, lo=0, hi=L, read_len=50)
        b2 = synth.pileup(L, 4000, seed=34, ref=r2, lo=60, hi=340, read_len=50)
        eng = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=r1, calls_only=True)
        eng.accumulate(*b1)
        eng.set_reference(r2)
        eng.accumulate(*b2)
        eng.finalize()
        o = OracleCaller(r1, 30, 10, 5, 0.10)
        o.accumulate(*b1)
        o.accumulate(*b2)
        compare_variants(eng.variants(), o.prepare_variants(), RTOL)


def test_many_bams_accumulated():
    """BASELINE config 4 in miniature: 64 BAM-sized batches (100x, own seeds, pysam-style per-BAM
    depth cap) accumulated in one context — memory insertion order, first visits, dict order and
    calls vs the oracle."""
    from covid_spings_variant_caller_amd import synth
    L = 2500
    ref = synth.reference(L, seed=50)
    batches = []
    for i in range(64):
        lo = (i * 37) % 900
        batches.append(synth.pileup(L, 100, seed=1000 + i, ref=ref, snv_every=23, lo=lo, hi=min(L, lo + 1600),
                                    max_depth=80))
    for calls_only in (False, True):
        _vs_oracle(ref, batches, DEF, calls_only=calls_only)


@pytest.mark.parametrize("depth", [10000, 100000])
def test_full_size_count_conservation(depth):
    """BASELINE sizes (SARS-CoV-2 at 10,000x: E = 3.0e8; 100,000x: E = 3.0e9, past 2^31) through a
    size-independent property: every entry with q >= minBaseQuality lands in exactly one position's
    totalDepth and one allele / D / N bucket (process_pileup_column :75-101), so per-position depth
    and per-code totals equal direct counts of the CSR."""
    import torch
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.pileup import synth_batch
    L = 29903
    ref = synth.reference(L, seed=1)
    b = synth_batch(ref, depth, seed=2, n_threads=16)
    E = b.n_entries
    keep = b.quals >= 30
    want_depth = np.add.reduceat(keep, b.offsets[:-1].astype(np.int64)).astype(np.int64)
    want_depth[np.diff(b.offsets.astype(np.int64)) == 0] = 0
    want_codes = np.bincount(b.codes[keep], minlength=256)
    del keep
    dc = torch.from_numpy(b.codes_padded).cuda()
    dq = torch.from_numpy(b.quals_padded).cuda()
    do = torch.from_numpy(b.offsets.view(np.int64).copy()).cuda()
    eng = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    eng.accumulate(0, do, dc, dq, borrow=True, n_entries=E)
    eng.finalize()
    t = eng.table()
    np.testing.assert_array_equal(t["depth"].astype(np.int64), want_depth)
    cnt = t["counts"].astype(np.int64).sum(axis=0)
    assert [int(x) for x in cnt[:5]] == [int(want_codes[k]) for k in (1, 2, 4, 8, 15)]
    assert int(cnt[5]) == int(want_codes[16]) and int(cnt[6]) == int(want_codes[17])
    assert int(cnt[7]) == int(want_codes.sum() - want_codes[[1, 2, 4, 8, 15, 16, 17]].sum())
    assert eng.counts()[0] > 0
    eng.close()
    del dc, dq, do
    b.close()
    torch.cuda.empty_cache()


def _plant_many(batch, pos, code, q, n):
    """Append n entries (code, q) at the end of column `pos` of a CSR batch."""
    pb, off, c, qq = batch
    at = int(off[pos - pb + 1])
    c = np.insert(c, at, np.full(n, code, np.uint8))
    qq = np.insert(qq, at, np.full(n, q, np.uint8))
    off = off.copy()
    off[pos - pb + 1:] += np.uint64(n)
    return pb, off, c, qq


@pytest.mark.parametrize("depth", [1000, 10000])
def test_fused_deep_finalize_replays(depth):
    """A calls-only sample whose only batch is deep: spg_finalize runs accumulate + prepare_variants in
    ONE launch (k_acc_seg<..., FUSE>).  Planted IUPAC alleles (a call 'R' and a lone 'M': exotic, exact
    replay) and a P product in the subnormal band (exact replay) are resolved by the finishing waves;
    calls equal the oracle's, the fused launch leaves the records complete for a later table, and a
    second finalize (k_finalize) returns the same calls."""
    from covid_spings_variant_caller_amd import synth
    L = 4000
    ref = synth.reference(L, seed=71)
    b = synth.pileup(L, depth, seed=72, ref=ref, snv_every=53, lo=500, hi=1700)
    d = depth // 5
    b = _plant_many(b, 800, 5, 35, d)                        # 'R' x 20 %: an IUPAC call
    b = _plant_many(b, 801, 3, 33, 1)                        # one 'M': exotic, replayed, no call
    alt = 2 if ref[900] != "C" else 4
    b = _plant_many(b, 900, alt, 31, 100)                    # sum q = 3100: P in the subnormal band
    orc = COracle(ref, 30, 10, 5, 0.01)
    eng = _engine(ref, dict(DEF, minEvidenceRatio=0.01), calls_only=True)
    eng.accumulate(*b)
    orc.accumulate(*b)
    eng.finalize()
    orc.finalize()
    fused = eng.variants()
    compare_variants(fused, orc.variants(), rtol=RTOL)
    assert any(v["alleles"][1] == "R" for v in fused)
    eng.finalize()                                           # records complete: the unfused finalize agrees
    compare_variants(eng.variants(), fused, rtol=0)
    assert eng.memory_summary() == orc.memory_summary()
    t = eng.table()
    assert t["flags"][800] & 12 == 12 and t["flags"][801] & 12 == 12   # exotic + replayed
    eng.close()


def _cut_column(batch, pos, keep):
    """Keep only the first `keep` entries of column `pos` of a CSR batch."""
    pb, off, c, qq = batch
    a, e = int(off[pos - pb]), int(off[pos - pb + 1])
    n = (e - a) - keep
    if n <= 0:
        return batch
    c = np.delete(c, np.s_[a + keep:e])
    qq = np.delete(qq, np.s_[a + keep:e])
    off = off.copy()
    off[pos - pb + 1:] -= np.uint64(n)
    return pb, off, c, qq


@pytest.mark.parametrize("depth", [6000, 10000])
def test_fused_tail_columns_ragged(depth):
    """The fused deep launch's last columns (its tail waves: G / 2 columns each at 10,000x and above, the columns
    a split-tail experiment (profiles/r05zj_split_tail) cut four ways): an IUPAC call, a lone exotic allele, a P
    product in the subnormal band, SNVs (dual mode) and ragged lengths — empty, under one 1,024-entry chunk, one to
    five chunks.  Every position's counts, dict order and first visits (memory_summary) and the calls equal the
    oracle's; a second, unfused finalize gives the same calls."""
    from covid_spings_variant_caller_amd import synth
    L = 1400
    ref = synth.reference(L, seed=171)
    b = synth.pileup(L, depth, seed=172, ref=ref, snv_every=17, lo=0, hi=L)
    b = _plant_many(b, 1250, 5, 35, depth // 5)             # 'R' x 20 %: an IUPAC call near the batch's end
    b = _plant_many(b, 1251, 3, 33, 1)                      # one 'M': exotic, replayed, no call
    alt = 2 if ref[1300] != "C" else 4
    b = _plant_many(b, 1300, alt, 31, 100)                  # sum q = 3100: P in the subnormal band
    for pos, keep in [(1380, 0), (1381, 700), (1382, 1024), (1383, 1500), (1384, 2100), (1385, 3000),
                      (1386, 4100), (1387, 5200), (1388, 1)]:
        b = _cut_column(b, pos, keep)
    p = dict(DEF, minEvidenceRatio=0.01)
    eng, orc = _vs_oracle(ref, [b], p, calls_only=True)
    fused = eng.variants()
    assert any(v["alleles"][1] == "R" for v in fused)
    assert sum(1 for v in fused if v["start"] >= 700) > 20
    eng.finalize()                                           # unfused: from the records in memory
    compare_variants(eng.variants(), fused, rtol=0)
    t = eng.table()
    assert t["flags"][1250] & 12 == 12 and t["flags"][1251] & 12 == 12   # exotic + replayed
    eng.close()


@pytest.mark.parametrize("shift", [0, 3, 8, 13])
def test_fused_dual_second_allele_eps_only(shift):
    """FUSE dual mode: a column's frequent second allele (an SNV at AF 0.05-0.5) accumulates counts,
    sum(q) and sum(eps) but not sum ln(1-eps) (acc.misc skip + "eps complete" bits): a deep call's GL is
    exactly 0 without it.  Entries at several 16-B alignments (the CSR shifted by `shift` bytes in device
    memory).  Calls vs the oracle (QUAL within 1e-9), no replays for the deep calls, and a second,
    unfused finalize from the records in memory gives the same calls bit for bit."""
    import torch
    from covid_spings_variant_caller_amd import synth
    L = 3000
    ref = synth.reference(L, seed=81)
    p = dict(DEF, minEvidenceRatio=0.02)
    lo, off, c, q = synth.pileup(L, 3000, seed=82, ref=ref, snv_every=13, lo=700, hi=1500)
    E = len(c)
    orc = COracle(ref, p["minBaseQuality"], p["minTotalDepth"], p["minAlleleDepth"], p["minEvidenceRatio"])
    orc.accumulate(lo, off, c, q)
    orc.finalize()
    dc = torch.full((shift + E + 64,), 0xFF, dtype=torch.uint8, device="cuda")
    dq = torch.zeros(shift + E + 64, dtype=torch.uint8, device="cuda")
    dc[shift:shift + E] = torch.from_numpy(c).cuda()
    dq[shift:shift + E] = torch.from_numpy(q).cuda()
    do = torch.from_numpy(off.astype(np.int64) + shift).cuda()
    eng = _engine(ref, p, calls_only=True)
    eng.accumulate(lo, do, dc, dq, borrow=True, n_entries=E)
    eng.finalize()
    fused = eng.variants()
    exp = orc.variants()
    assert len(exp) > 40
    compare_variants(fused, exp, rtol=RTOL)
    eng.finalize()                                           # unfused: from the records in memory
    compare_variants(eng.variants(), fused, rtol=0)
    t = eng.table()
    deep = [v["start"] for v in fused if v["info"]["DP"] >= 1000]
    assert len(deep) > 40 and not (t["flags"][deep] & 4).any()   # deep calls: no exact replay
    eng.close()


def test_fused_then_more_batches_keep_eps_bits_exact():
    """A fused deep finalize (second alleles keep only sum(eps): acc.misc eps-complete bits), then more
    batches into the same memory — a deep one (k_acc_seg, non-FRESH record merge) and a shallow one
    (k_acc_multi) — each followed by a finalize: calls vs the oracle after every step."""
    from covid_spings_variant_caller_amd import synth
    L = 3000
    ref = synth.reference(L, seed=91)
    p = dict(DEF, minEvidenceRatio=0.02)
    b1 = synth.pileup(L, 3000, seed=92, ref=ref, snv_every=13, lo=600, hi=1400)
    b2 = synth.pileup(L, 2000, seed=93, ref=ref, snv_every=17, lo=900, hi=1700)
    b3 = synth.pileup(L, 40, seed=94, ref=ref, snv_every=11, lo=0, hi=L)
    orc = COracle(ref, p["minBaseQuality"], p["minTotalDepth"], p["minAlleleDepth"], p["minEvidenceRatio"])
    eng = _engine(ref, p, calls_only=True)
    for b in (b1, b2, b3):
        eng.accumulate(*b)
        orc.accumulate(*b)
        eng.finalize()
        orc.finalize()
        got, exp = eng.variants(), orc.variants()
        assert len(exp) > 20
        compare_variants(got, exp, rtol=RTOL)
    assert eng.memory_summary() == orc.memory_summary()
    eng.close()


@pytest.mark.parametrize("lpc", [0, 4, 16, 64, "list"])
def test_mid_depth_lone_batch_counted(lpc, monkeypatch):
    """A calls-only sample whose only batch is mid-depth (1,000x: BASELINE config 2): spg_finalize counts every
    column (k_count_cols, lpc lanes per column: 0 = the default choice), folds exactly only the listed columns
    (k_acc_seg<1>) and runs the sparse finalize.
    Planted: short columns that may call (< 128 entries), an IUPAC call, a lone exotic entry, a P product in the
    subnormal band, q in {0..3, >= 128}.  Calls vs the oracle; a second finalize (the records materialized through
    k_acc_seg) returns the same calls bit for bit; then a second batch folds into the same memory."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    L = 5000
    ref = synth.reference(L, seed=171)
    p = dict(DEF, minEvidenceRatio=0.02)
    lo, off, c, q = synth.pileup(L, 1000, seed=172, ref=ref, snv_every=41, lo=300, hi=2300)
    rng = np.random.default_rng(173)
    q = q.copy()
    m = rng.random(len(q)) < 0.01
    q[m] = rng.choice(np.array([0, 1, 2, 3, 4, 127, 128, 200, 255], np.uint8), size=m.sum())
    b = (lo, off, c, q)
    b = _plant_many(b, 900, 5, 35, 200)                      # 'R' x 20 %: an IUPAC call
    b = _plant_many(b, 901, 3, 33, 1)                        # one 'M': exotic, replayed, no call
    alt = 2 if ref[1000] != "C" else 4
    b = _plant_many(b, 1000, alt, 31, 100)                   # sum q = 3100: P in the subnormal band
    # the last columns of the window: short (tens of entries), some with an SNV that calls
    pb, off, c, q = b
    offs = off.astype(np.int64)
    keep = np.ones(len(c), bool)
    for col in range(2300 - 300 - 12, 2300 - 300):
        s, e = offs[col], offs[col + 1]
        keep[s + 40 + col % 7:e] = False
    starts = offs[:-1]
    newoff = np.concatenate([[0], np.cumsum(np.add.reduceat(keep.astype(np.int64), starts) * (np.diff(offs) > 0))])
    c, q = c[keep].copy(), q[keep].copy()
    for col in range(2300 - 300 - 12, 2300 - 300, 3):
        s = newoff[col]
        alt = 1 if ref[pb + col] != "A" else 8
        c[s:s + 12] = alt
        q[s:s + 12] = 37
    b = (pb, newoff.astype(np.uint64), c, q)
    if lpc == "list":                                        # the fused kernel's list mode (multi-sample batches)
        monkeypatch.setenv("SPG_COUNT_COLS", "0")
    elif lpc:
        monkeypatch.setenv("SPG_COUNT_LPC", str(lpc))
    eng = PileupEngine(L, p["minBaseQuality"], p["minTotalDepth"], p["minAlleleDepth"], p["minEvidenceRatio"],
                       device=0, reference=ref, calls_only=True)
    orc = COracle(ref, p["minBaseQuality"], p["minTotalDepth"], p["minAlleleDepth"], p["minEvidenceRatio"])
    eng.accumulate(*b)
    orc.accumulate(*b)
    eng.finalize()
    orc.finalize()
    got = eng.variants()
    exp = orc.variants()
    assert len(exp) > 40
    assert any(v["alleles"][1] == "R" for v in exp)
    assert any(v["info"]["DP"] < 128 for v in exp)
    compare_variants(got, exp, rtol=RTOL)
    pc = eng.path_counters()
    assert pc["mid_counted_finalizes"] == (0 if lpc == "list" else 1) and pc["fused_deep_finalizes"] == 1, pc
    eng.finalize()                                           # records materialized: the same calls, bit for bit
    compare_variants(eng.variants(), got, rtol=0)
    assert eng.memory_summary() == orc.memory_summary()
    b2 = synth.pileup(L, 300, seed=174, ref=ref, snv_every=17, lo=1500, hi=3500)
    eng.accumulate(*b2)
    orc.accumulate(*b2)
    eng.finalize()
    orc.finalize()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    eng.close()
