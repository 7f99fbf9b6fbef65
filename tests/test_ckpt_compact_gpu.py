"""spg_history_copy_compact (csrc/spg_ckpt.hip): the checkpoint's view of a history batch computed in HBM — the entries
the base-quality filter keeps plus a first-entry marker per column whose entries all fail it — bit-identical to the
host restatement (tests/ck_util.bq_compact) on owned, borrowed and spilled (host-mapped) batches, on columns that
straddle 16-B blocks, and on a 10,000x SARS-CoV-2 batch (3e8 entries: compacted in two column ranges)."""
import numpy as np
import pytest

import spings  # noqa: F401
from ck_util import bq_compact

pytestmark = pytest.mark.gpu


def _check(eng, bq):
    full = eng.history()
    comp = list(eng.iter_history(0, min_bq=bq))
    assert len(full) == len(comp)
    for (pa, oa, ca, qa), (pb, ob, cb, qb) in zip(full, comp):
        eo, ec, eq = bq_compact(oa, ca, qa, bq)
        assert pa == pb
        np.testing.assert_array_equal(ob, eo)
        np.testing.assert_array_equal(cb, ec)
        np.testing.assert_array_equal(qb, eq)
    # the packed form (spg_history_copy_packed: one byte per kept entry + exceptions), decoded, is the same; and with
    # too small an exception capacity it hands back the unpacked arrays instead
    for cap in (1 << 20, 3):
        for (pa, oa, ca, qa), ent in zip(full, eng.iter_history_packed(0, bq, exc_cap=cap)):
            eo, ec, eq = bq_compact(oa, ca, qa, bq)
            np.testing.assert_array_equal(ent["off"], eo)
            if "packed" in ent:
                pk = ent["packed"]
                codes, quals = np.array([1, 2, 4, 8], np.uint8)[pk >> 6], pk & 63
                codes[ent["xi"].astype(np.int64)] = ent["xc"]
                quals[ent["xi"].astype(np.int64)] = ent["xq"]
                assert cap > 3 or len(ent["xi"]) <= 3
            else:
                codes, quals = ent["codes"], ent["quals"]
            np.testing.assert_array_equal(codes, ec)
            np.testing.assert_array_equal(quals, eq)


@pytest.mark.parametrize("bq", [0, 1, 13, 30, 60])
def test_compact_matches_host(bq):
    import torch
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    L = 4000
    ref = synth.reference(L, seed=91)
    eng = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    rng = np.random.default_rng(bq)
    for s, depth in enumerate((3, 25, 400, 2500)):
        pb, off, c, q = synth.pileup(L, depth, seed=92 + s, ref=ref, snv_every=37, lo=50 * s, hi=L - 31 * s)
        q = q.copy()
        off64 = off.astype(np.int64)
        for col in rng.choice(len(off) - 1, size=min(60, len(off) - 1), replace=False):   # all-fail columns
            q[off64[col]:off64[col + 1]] = rng.integers(0, max(1, bq), off64[col + 1] - off64[col])
        q[rng.integers(0, len(q), 200)] = 255
        c = c.copy()
        c[rng.integers(0, len(c), 150)] = rng.choice(np.array([3, 15, 16, 17], np.uint8), 150)   # packed exceptions
        if s == 2:                                  # borrowed device batch
            dev = torch.device("cuda", 0)
            pad = np.zeros(16, np.uint8)
            t = (torch.from_numpy(off.astype(np.int64)).to(dev), torch.from_numpy(np.concatenate([c, pad + 0xFF])).to(dev),
                 torch.from_numpy(np.concatenate([q, pad])).to(dev))
            eng.accumulate(pb, *t, borrow=True, n_entries=len(c))
            eng._hold = t
        else:
            eng.accumulate(pb, off, c, q)
    _check(eng, bq)
    eng.finalize()
    _check(eng, bq)
    eng.close()


def test_compact_spilled_history():
    """Batches moved to host-mapped memory by the history cap are compacted in place over PCIe."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    L = 3000
    ref = synth.reference(L, seed=93)
    eng = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    eng.set_history_cap(1 << 20)
    for s in range(40):
        eng.accumulate(*synth.pileup(L, 60, seed=100 + s, ref=ref, snv_every=41))
    eng.finalize()
    _, spilled, _ = eng.history_resident()
    assert spilled > 10
    _check(eng, 30)
    eng.close()


def test_compact_10000x_two_ranges():
    import torch
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.pileup import synth_batch
    L = 29903
    ref = synth.reference(L, seed=1)
    b = synth_batch(ref, 10000.0, lo=0, hi=L, seed=2, n_threads=16)
    off, c, q = b.offsets.copy(), b.codes.copy(), b.quals.copy()
    b.close()
    assert int(off[-1]) > (256 << 20)
    eng = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    eng.accumulate(0, off, c, q)
    eng.finalize()
    (pb, o2, c2, q2), = list(eng.iter_history(0, min_bq=30))
    eo, ec, eq = bq_compact(off, c, q, 30)
    np.testing.assert_array_equal(o2, eo)
    assert np.array_equal(c2, ec) and np.array_equal(q2, eq)
    eng.close()
    torch.cuda.empty_cache()
