"""The live server's loop (client_server/vc_queue.py:142-144): process_bam, create_checkpoint, then write_vcf —
i.e. prepare_variants (variant_caller/live_variant_caller.py:120-231) — after EVERY BAM, against the bit-exact C
oracle after each step.

The engine's path for it (csrc/spg_api.cpp countable / finalize_impl): every finalize is counted mode — the new BAM
counted into the per-position totals, the positions that may call listed, and their records re-folded incrementally
(only the batches since the position's last fold, k_fold_hist's watermark); a replayed position resumes its exact
fold from the replay cache.  No record-path run (k_acc_tile) and no
full-range k_finalize after BAM 1: spg_path_counters checks it.
"""
import numpy as np
import pytest

import spings  # noqa: F401
from oracle.c_oracle import COracle
from oracle_util import compare_variants
from test_many_batches_gpu import _many, _plant

pytestmark = pytest.mark.gpu
RTOL = 1e-9


def _engine(ref, calls_only=True):
    from covid_spings_variant_caller_amd.engine import PileupEngine
    return PileupEngine(len(ref), 30, 10, 5, 0.10, device=0, reference=ref, calls_only=calls_only)


def test_finalize_after_every_bam_300_vs_oracle():
    """300 shallow BAMs, prepare_variants after each: calls (incl. a subnormal-band position replayed exactly and
    an IUPAC allele) equal the oracle's after every BAM; the loop never leaves counted mode."""
    L = 1500
    ref, batches = _many(L, 300, 40, 31000, span=1100, band_pos=700, iupac_pos=710, cap=35)
    eng = _engine(ref)
    orc = COracle(ref, 30, 10, 5, 0.10)
    n_band_seen = 0
    for i, b in enumerate(batches):
        eng.accumulate(*b)
        orc.accumulate(*b)
        eng.finalize()
        orc.finalize()
        got, want = eng.variants(), orc.variants()
        compare_variants(got, want, rtol=RTOL)
        n_band_seen += eng.counts()[1] > 0
    pc = eng.path_counters()
    # (BAM 1, a lone batch of <= 40 entries per column, may take k_acc_lite; every later finalize counts)
    assert pc["counted_finalizes"] + pc["fused_shallow_finalizes"] == 300 and pc["counted_finalizes"] >= 299, pc
    assert pc["record_runs"] == 0, pc                                # no k_acc_tile fold of the records
    assert pc["materializations"] == 0 and pc["full_finalizes"] == 0, pc
    assert pc["batches_counted"] == 300, pc                          # every BAM counted once
    assert n_band_seen > 0                                          # the exact replay ran inside the loop
    assert eng.memory_summary() == orc.memory_summary()             # the table (re-materialized) at the end
    eng.close()


def test_every_bam_finalize_with_planted_calls_appearing_late():
    """Calls whose positions are listed only late in the loop (a planted allele from BAM 140 on passes AD/DP >= 0.10 at ~BAM 160,
    at positions listed earlier and at positions never listed before): the incremental fold must merge into the
    records of earlier folds and fold never-listed positions from batch 0 — dict order, first visits, AD/DP
    against the oracle at every step."""
    L = 900
    ref, batches = _many(L, 200, 12, 33000, span=700, cap=12)
    late = [100, 350, 600]
    for i in range(140, 200):
        for p in late:
            code = 8 if ref[p] != "T" else 1
            for k in range(8):
                batches[i] = _plant(batches[i], p, code, 36 + (k & 1))
    eng = _engine(ref)
    orc = COracle(ref, 30, 10, 5, 0.10)
    for i, b in enumerate(batches):
        eng.accumulate(*b)
        orc.accumulate(*b)
        eng.finalize()
        orc.finalize()
        compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    assert {v["start"] for v in orc.variants()} >= set(late)
    assert eng.memory_summary() == orc.memory_summary()
    eng.close()


def test_reset_between_samples_invalidates_fold_watermarks():
    """Two samples through one engine (reset_memory between): the second sample's incremental folds must not
    merge into the first sample's records (the watermark generation changes at every counted run)."""
    L = 800
    ref, batches = _many(L, 60, 20, 35000, span=600, band_pos=300, cap=20)
    eng = _engine(ref)
    for round_ in range(2):
        eng.reset()
        orc = COracle(ref, 30, 10, 5, 0.10)
        sub = batches[round_ * 30:(round_ + 1) * 30]
        for b in sub:
            eng.accumulate(*b)
            orc.accumulate(*b)
            eng.finalize()
            orc.finalize()
            compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    eng.close()


def test_table_read_inside_the_loop_then_more_bams():
    """A full table read in the middle of the loop (LiveVariantCaller.memory) re-materializes the records; the loop
    then continues on the record path and the calls still match."""
    L = 800
    ref, batches = _many(L, 40, 25, 36000, span=600, band_pos=400, iupac_pos=410, cap=25)
    eng = _engine(ref)
    orc = COracle(ref, 30, 10, 5, 0.10)
    for i, b in enumerate(batches):
        eng.accumulate(*b)
        orc.accumulate(*b)
        eng.finalize()
        orc.finalize()
        compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
        if i == 19:
            assert eng.memory_summary() == orc.memory_summary()
    assert eng.memory_summary() == orc.memory_summary()
    eng.close()


def test_deep_batches_respect_history_cap():
    """deep batches (>= 256 entries per column, k_acc_seg) under a history cap spill their folded
    copies like shallow ones; calls after the spill (band replays read the host copies) vs the oracle."""
    from covid_spings_variant_caller_amd import synth
    L = 3000
    ref = synth.reference(L, seed=37000)
    eng = _engine(ref, calls_only=False)
    cap = 4 << 20
    eng.set_history_cap(cap)
    orc = COracle(ref, 30, 10, 5, 0.10)
    for i in range(12):
        b = synth.pileup(L, 600, seed=37001 + i, ref=ref, snv_every=97, lo=100 * i, hi=100 * i + 1500)
        eng.accumulate(*b)
        orc.accumulate(*b)
    dev, n_sp, _ = eng.history_resident()
    assert n_sp >= 6 and dev <= cap + (1 << 20), (dev, n_sp)
    eng.finalize()
    orc.finalize()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    assert eng.memory_summary() == orc.memory_summary()
    eng.close()


def test_records_input_validation():
    """spg_accumulate_records bounds its offsets (monotone, <= n_entries) and each read's record offset
    (fixed fields inside the records buffer) before anything is copied or launched."""
    import ctypes as C
    from covid_spings_variant_caller_amd import _native as N
    L = 1000
    ref = "ACGT" * (L // 4)
    eng = _engine(ref)
    data = np.zeros(4096, np.uint8)
    offs = np.array([0, 3, 1, 4], np.uint64)            # not monotone in the middle
    rec = np.array([0], np.uint64)
    i32 = np.array([0], np.int32)
    neg = np.array([-1], np.int32)
    r = N.SpgRecords()
    r.pos_begin, r.n_cols, r.n_entries = 10, 3, 4
    r.offsets = offs.ctypes.data
    r.data, r.data_bytes = data.ctypes.data, len(data)
    r.n_reads = 1
    r.rec, r.rpos, r.rend, r.tweak = rec.ctypes.data, i32.ctypes.data, i32.ctypes.data, neg.ctypes.data
    with pytest.raises(RuntimeError, match="monotone"):
        N.check(eng._L.spg_accumulate_records(eng._h, C.byref(r), 0), "spg_accumulate_records")
    offs[:] = [0, 1, 2, 4]
    rec[0] = len(data) - 20                              # fixed fields past the buffer
    with pytest.raises(RuntimeError, match="past the records buffer"):
        N.check(eng._L.spg_accumulate_records(eng._h, C.byref(r), 0), "spg_accumulate_records")
    eng.close()


def _deep_calls_only_vs_oracle(ref, b):
    eng = _engine(ref)
    orc = COracle(ref, 30, 10, 5, 0.10)
    eng.accumulate(*b)
    orc.accumulate(*b)
    eng.finalize()
    orc.finalize()
    compare_variants(eng.variants(), orc.variants(), rtol=RTOL)
    return eng, orc


def test_mid_depth_single_batch_list_mode_vs_oracle():
    """A calls-only sample whose only batch is mid-depth (1,000x over the whole SARS-CoV-2 genome: G = 16 columns
    per wave, wider than the fused kernel's finishing ring): k_acc_seg lists the positions that may call at each
    ring finish and the sparse k_finalize decides them (spg_api.cpp launch_seg list mode) — calls vs the oracle,
    with planted SNVs every 97th position, an IUPAC allele and a subnormal-band position."""
    from covid_spings_variant_caller_amd import synth
    L = 29903
    ref = synth.reference(L, seed=38000)
    b = synth.pileup(L, 1000, seed=38001, ref=ref, snv_every=97)
    b = _plant(b, 5000, 5, 35)                               # 'R': exotic, exact replay
    for k in range(98):                                      # 98 x Q31 of a non-REF base at a 0-AF position
        b = _plant(b, 7001, 2 if ref[7001] != "C" else 4, 31)
    eng, orc = _deep_calls_only_vs_oracle(ref, b)
    pc = eng.path_counters()
    assert pc["fused_deep_finalizes"] == 1 and pc["sparse_finalizes"] == 1 and pc["full_finalizes"] == 0, pc
    assert len(orc.variants()) > 200
    assert eng.memory_summary() == orc.memory_summary()
    eng.close()


def test_stacked_samples_one_context_equals_separate_engines():
    """The bench's stacked layout (bench.py build_shard): S samples of one coordinate range side by side in one
    context (sample s = positions [s C, (s+1) C)) give, per sample, exactly the calls of a context of its own."""
    from covid_spings_variant_caller_amd import synth
    L, S = 3000, 8
    ref = synth.reference(L, seed=39000)
    samples = [synth.pileup(L, 1000, seed=39001 + s, ref=ref, snv_every=31) for s in range(S)]
    offs, cs, qs, base = [np.zeros(1, np.uint64)], [], [], 0
    for _, o, c, q in samples:
        offs.append(o[1:] + np.uint64(base))
        base += int(o[-1])
        cs.append(c)
        qs.append(q)
    big = _engine(ref * S)
    big.accumulate(0, np.concatenate(offs), np.concatenate(cs), np.concatenate(qs))
    big.finalize()
    got = big.variants()
    for s, b in enumerate(samples):
        one = _engine(ref)
        one.accumulate(*b)
        one.finalize()
        mine = [dict(v, start=v["start"] - s * L, stop=v["stop"] - s * L) for v in got if s * L <= v["start"] < (s + 1) * L]
        compare_variants(mine, one.variants(), rtol=RTOL)
        one.close()
    big.close()
