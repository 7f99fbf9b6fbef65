"""spg_multi_* (csrc/spg_multi.cpp): the one-process multi-device context of the C-ABI — equal-entry coordinate cuts,
per-device contexts over their own ranges, host batches and BAM records plans sliced at the cuts, re-plans when the
load drifts, one RCCL ncclGather of the call tables.  On the one-GPU box it runs with n = 1 and with device 0 listed
several times (every slicing, empty-slice, re-plan and merge path; the gather by device copies instead of RCCL);
the merged table must equal a single context's and the oracle's.  (Distinct devices — RCCL — are unmeasured on
hardware until the driver's 8-GPU node runs.)"""
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


def _variants_equal(a, b):
    from oracle_util import compare_variants
    compare_variants(a, b, rtol=1e-9)


def test_multi_three_contexts_on_one_gpu_slices_and_merge():
    """n = 3 contexts on device 0 (listed three times: no RCCL, tables gathered by device copies): batches sliced at
    the cuts, empty slices as one-column batches (a batch inside one device's range), per-device coordinate spaces,
    and the merged table in memory order — vs one context and the oracle, after several samples."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.multi import MultiEngine
    L = 12_000
    ref = synth.reference(L, seed=41)
    batches = [synth.pileup(L, 60, seed=42 + i, ref=ref, snv_every=53, lo=(i * 900) % 4000, hi=L - (i * 500) % 3000)
               for i in range(5)]
    batches.append(synth.pileup(L, 80, seed=60, ref=ref, snv_every=53, lo=200, hi=900))      # one device only
    m = MultiEngine([0, 0, 0], L, reference=ref)
    m.set_rebalance(1e9, 0)                       # fixed cuts here (re-plans: the next test)
    s = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    for rnd in range(2):
        m.reset()
        s.reset()
        orc = COracle(ref, 30, 10, 5, 0.10)
        for b in batches[rnd:]:
            m.accumulate(*b)
            s.accumulate(*b)
            orc.accumulate(*b)
        cuts = m.partition()
        assert len(cuts) == 4 and cuts[0] == 0 and cuts[-1] == L and np.all(np.diff(cuts) > 0)
        m.finalize()
        s.finalize()
        orc.finalize()
        got = m.candidates()
        assert len(got) > 20
        assert got.tobytes() == s.candidates().tobytes()
        _variants_equal(m.variants(), orc.variants())
        # the table and the history, reassembled in reference coordinates
        t, ts = m.table(), s.table()
        np.testing.assert_array_equal(t["depth"], ts["depth"])
        np.testing.assert_array_equal(t["first_batch"], ts["first_batch"])
        hm, hs = m.history(), s.history()
        assert len(hm) == len(hs)
        for (pa, oa, ca, qa), (pb, ob, cb, qb) in zip(hm, hs):
            assert int(oa[-1]) == int(ob[-1])
            np.testing.assert_array_equal(ca, cb)
            np.testing.assert_array_equal(qa, qb)
    m.close()
    s.close()


def test_multi_amplicon_first_batch_replans():
    """An amplicon-shaped first batch (three short windows) plans every cut inside the windows; later full-coverage
    batches overload the last device, the sample is re-planned (history re-sliced at the new cuts) and the calls
    stay those of one context; the next sample is planned from this sample's histogram."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.multi import MultiEngine
    L = 12_000
    ref = synth.reference(L, seed=43)
    amp = [synth.pileup(L, 300, seed=44 + k, ref=ref, snv_every=29, lo=lo, hi=lo + 300) for k, lo in
           enumerate((500, 5000, 9000))]
    full = [synth.pileup(L, 50, seed=50 + i, ref=ref, snv_every=37) for i in range(4)]
    m = MultiEngine([0, 0, 0, 0], L, reference=ref)
    m.set_rebalance(1.25, 256)
    s = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    orc = COracle(ref, 30, 10, 5, 0.10)
    per_pos = np.zeros(L, np.int64)
    for b in amp + full:
        m.accumulate(*b)
        s.accumulate(*b)
        orc.accumulate(*b)
        per_pos[b[0]:b[0] + len(b[1]) - 1] += np.diff(b[1].astype(np.int64))
        if b is amp[0]:
            first_cuts = m.partition()
        # after every batch: no device holds more than the re-plan threshold (bucket granularity: + 5 %)
        loads = np.add.reduceat(per_pos, m.partition()[:-1])
        assert loads.max() <= 1.25 * 1.05 * loads.mean(), (m.partition(), loads)
    assert first_cuts[-2] < 800                                      # every cut inside the first window
    assert m.replans() >= 2
    cuts = m.partition()
    m.finalize()
    s.finalize()
    orc.finalize()
    # (the re-sliced history folds its fp64 sums in another grouping: QUAL / GL within the oracle tolerance)
    _variants_equal(m.variants(), s.variants())
    _variants_equal(m.variants(), orc.variants())
    m.reset()                                                        # planned from the previous histogram,
    m.accumulate(*amp[0])                                            # not from this amplicon batch
    assert m.partition()[-2] > 2000
    m.close()
    s.close()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_multi_records_path_vs_oracle(tmp_path, devices):
    """The device pileup sharded (spg_multi_accumulate_records): LiveVariantCaller(devices=...) over simulated BAMs —
    each context decodes the reads that reach its range — vs the oracle on the host pileup of the same BAMs, and vs
    the single-device caller; then the memory view and a checkpoint round trip."""
    import samgen
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.live_variant_caller import LiveVariantCaller
    from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams, simulate_bam
    L = 6000
    ref = synth.reference(L, seed=45)
    fasta = str(tmp_path / "ref.fa")
    samgen.write_fasta(fasta, [("NC_045512.2", ref)])
    bams = []
    for i in range(3):
        p = str(tmp_path / f"b{i}.bam")
        simulate_bam(p, "NC_045512.2", ref, depth=150.0 + 50 * i, seed=70 + i, n_threads=4)
        bams.append(p)
    mc = LiveVariantCaller(fasta, 30, 20, 10, 5, 0.10, 1, devices=devices)
    sc = LiveVariantCaller(fasta, 30, 20, 10, 5, 0.10, 1, device=0)
    orc = COracle(ref, 30, 10, 5, 0.10)
    for p in bams:
        mc.process_bam(p)
        sc.process_bam(p)
        with AlignmentFile(p) as f:
            b = f.pileup_batch("NC_045512.2", PileupParams(n_threads=4))
            orc.accumulate(b.pos_begin, b.offsets.copy(), b.codes.copy(), b.quals.copy())
        orc.finalize()
        _variants_equal(mc.prepare_variants(), orc.variants())       # after every BAM (vc_queue.py:142-144)
    _variants_equal(mc.prepare_variants(), sc.prepare_variants())
    mm, ms = mc.memory, sc.memory
    assert list(mm) == list(ms)
    assert all(mm[p] == ms[p] for p in list(ms)[::97])
    ck = str(tmp_path / "ck.npz")
    mc.create_checkpoint(ck)
    mc2 = LiveVariantCaller(fasta, 30, 20, 10, 5, 0.10, 1, devices=devices)
    mc2.load_checkpoint(ck)
    _variants_equal(mc2.prepare_variants(), orc.variants())


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_device_slices_vs_single_context(devices):
    """spg_multi_plan + spg_multi_accumulate_slices (bench.py's multi_device leg): a batch resident in HBM, sliced at the
    plan's cuts into per-device tensors (borrowed), stacked samples over one coordinate space — the merged table equals
    one context's on the whole batch, every step after a reset; a slice that does not match its cut is refused before
    any device takes the batch."""
    import torch
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.multi import MultiEngine
    L, S = 5000, 3
    ref = synth.reference(L, seed=81)
    smp = [synth.pileup(L, 400, seed=82 + s, ref=ref, snv_every=41) for s in range(S)]
    off = np.zeros(S * L + 1, np.uint64)
    base = 0
    for s, (_, o, _, _) in enumerate(smp):
        off[s * L + 1:(s + 1) * L + 1] = o[1:] + np.uint64(base)
        base += int(o[-1])
    codes = np.concatenate([c for _, _, c, _ in smp])
    quals = np.concatenate([q for _, _, _, q in smp])
    m = MultiEngine(devices, S * L, reference=ref * S)
    cuts = m.plan(0, off)
    assert cuts[0] == 0 and cuts[-1] == S * L and np.all(np.diff(cuts) > 0)
    dev = torch.device("cuda", 0)
    pad = np.zeros(16, np.uint8)
    slices = []
    for d in range(len(devices)):
        lo, hi = int(cuts[d]), int(cuts[d + 1])
        a, b = int(off[lo]), int(off[hi])
        so = (off[lo:hi + 1] - off[lo]).astype(np.int64)
        slices.append((lo, torch.from_numpy(so).to(dev), torch.from_numpy(np.concatenate([codes[a:b], pad + 0xFF])).to(dev),
                       torch.from_numpy(np.concatenate([quals[a:b], pad])).to(dev)))
    s = PileupEngine(S * L, 30, 10, 5, 0.10, device=0, reference=ref * S, calls_only=True)
    s.accumulate(0, off, codes, quals)
    s.finalize()
    one = s.candidates()
    assert len(one) > 30
    for _ in range(3):
        m.reset()
        m.accumulate_slices(0, off, slices, borrow=True)
        m.finalize()
        got = m.candidates()
        # integer fields exact; GL / QUAL within the parity bar (a slice starts its columns at another 16-B alignment
        # than the whole batch: the deep kernel's chunks, and so its fp64 summation order, differ)
        assert len(got) == len(one)
        for f in ("pos", "dp", "ad", "pl", "score", "ref", "alt", "rank", "first_batch", "gl_zero"):
            np.testing.assert_array_equal(got[f], one[f])
        for f in ("gl", "gl_linear", "qual"):
            np.testing.assert_allclose(got[f], one[f], rtol=1e-9, atol=0)
        assert np.array_equal(m.partition(), cuts)
    if len(devices) > 1:
        bad = list(slices)
        lo, so, c, q = bad[1]
        bad[1] = (lo + 1, so[1:] - so[1], c, q)
        m.reset()
        with pytest.raises(Exception, match="not the batch's columns"):
            m.accumulate_slices(0, off, bad, borrow=True)
    m.close()
    s.close()


@pytest.mark.parametrize("n", [1, 3])
def test_multi_async_tables_pipelined(n):
    """spg_multi_get_candidates_async / spg_multi_wait_candidates (verdict r05 item 3): sample k's table is enqueued
    (device copies + gather + one pinned copy, no host wait) and waited for after sample k + 1 has been reset, accumulated
    and finalized; every waited table equals a single context's for that sample.  A table larger than the first copies
    (1,024 records per device) comes back as TableRetry and is then taken synchronously before the reset; the copies grow
    and the next async tables of that size pass.  A third table in flight retires the oldest ticket."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.multi import MultiEngine, TableRetry
    L = 12_000
    ref = synth.reference(L, seed=71)
    samples = [[synth.pileup(L, 60, seed=72 + 7 * k + i, ref=ref, snv_every=41 + 6 * k, lo=(i * 900) % 4000,
                             hi=L - (i * 500) % 3000) for i in range(3)] for k in range(4)]
    m = MultiEngine([0] * n, L, reference=ref)
    m.set_rebalance(1e9, 0)
    s = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    expect = []
    for bs in samples:
        s.reset()
        for b in bs:
            s.accumulate(*b)
        s.finalize()
        expect.append(s.candidates())
    assert all(len(e) > 20 for e in expect)
    for rnd in range(2):
        pend = []
        for k, bs in enumerate(samples):
            m.reset()
            for b in bs:
                m.accumulate(*b)
            m.finalize()
            pend.append((k, m.candidates_async()))
            if len(pend) > 1:
                j, t = pend.pop(0)
                assert m.wait_candidates(t).tobytes() == expect[j].tobytes(), (rnd, j)
        j, t = pend.pop(0)
        assert m.wait_candidates(t).tobytes() == expect[j].tobytes()
    # a table that outgrows the first copies: TableRetry, then the synchronous table (and larger copies from then on)
    big = [synth.pileup(L, 60, seed=90 + i, ref=ref, snv_every=2, lo=0, hi=L) for i in range(2)]
    s.reset()
    for b in big:
        s.accumulate(*b)
    s.finalize()
    exp_big = s.candidates()
    assert len(exp_big) > 1024 * n
    m2 = MultiEngine([0] * n, L, reference=ref)
    m2.set_rebalance(1e9, 0)
    for b in big:
        m2.accumulate(*b)
    m2.finalize()
    t = m2.candidates_async()
    with pytest.raises(TableRetry):
        m2.wait_candidates(t)
    assert m2.candidates().tobytes() == exp_big.tobytes()
    m2.reset()
    for b in big:
        m2.accumulate(*b)
    m2.finalize()
    assert m2.wait_candidates(m2.candidates_async()).tobytes() == exp_big.tobytes()
    # three tables in flight: the oldest ticket is retired
    t1, t2, t3 = m2.candidates_async(), m2.candidates_async(), m2.candidates_async()
    with pytest.raises(Exception):
        m2.wait_candidates(t1)
    assert m2.wait_candidates(t2).tobytes() == exp_big.tobytes()
    assert m2.wait_candidates(t3).tobytes() == exp_big.tobytes()
    m.close()
    m2.close()
    s.close()


@pytest.mark.parametrize("n", [1, 3])
def test_multi_async_enqueue_does_not_wait_for_device(n):
    """The host part of a multi-device step does not grow with a device round trip per context: with every context's
    stream held busy (a spin kernel of ~0.2 s on it), candidates_async() returns at once and the wait delivers the table
    once the streams drain."""
    import ctypes as C
    import time
    import torch
    from covid_spings_variant_caller_amd import _native as N
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.multi import MultiEngine
    L = 12_000
    ref = synth.reference(L, seed=81)
    bs = [synth.pileup(L, 60, seed=82 + i, ref=ref, snv_every=47, lo=0, hi=L) for i in range(2)]
    m = MultiEngine([0] * n, L, reference=ref)
    for b in bs:
        m.accumulate(*b)
    m.finalize()
    want = m.candidates()
    dev = torch.device("cuda", 0)
    # the spin kernel's rate on this device: cycles for ~0.2 s
    t0 = time.perf_counter()
    torch.cuda._sleep(10_000_000)
    torch.cuda.synchronize(dev)
    cycles = int(10_000_000 * 0.2 / max(time.perf_counter() - t0, 1e-4))
    t0 = time.perf_counter()
    torch.cuda._sleep(cycles)
    torch.cuda.synchronize(dev)
    spin = time.perf_counter() - t0
    assert spin > 0.05
    for ctx in m._contexts():
        h = C.c_void_p()
        N.check(m._L.spg_stream(ctx, C.byref(h)), "spg_stream")
        with torch.cuda.stream(torch.cuda.ExternalStream(h.value, device=dev)):
            torch.cuda._sleep(cycles)
    t0 = time.perf_counter()
    t = m.candidates_async()
    dt = time.perf_counter() - t0
    got = m.wait_candidates(t)
    total = time.perf_counter() - t0
    assert got.tobytes() == want.tobytes()
    assert dt < 0.25 * spin and total > 0.5 * spin, (dt, total, spin)
    m.close()
