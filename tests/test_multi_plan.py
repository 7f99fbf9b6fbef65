"""spg_multi's cut planning (csrc/spg_multi.cpp spg_multi_plan_cuts), host only: equal entries per device over a
bucket histogram, every range non-empty.  An amplicon-shaped first BAM (all entries in a few short windows) must
not leave one device with most of a later full-coverage sample: the sample is re-planned from its cumulative
histogram (exercised on the GPU in tests/test_multi_gpu.py); here the plans themselves."""
import numpy as np
import pytest

import spings  # noqa: F401


def _plan(w, bucket, n_pos, n):
    from covid_spings_variant_caller_amd.multi import plan_cuts
    return plan_cuts(w, bucket, n_pos, n)


def _loads(w, bucket, cuts):
    pos = np.arange(len(w)) * bucket + bucket // 2
    d = np.searchsorted(cuts[1:-1], pos, side="right")
    return np.bincount(d, weights=w.astype(np.float64), minlength=len(cuts) - 1)


def test_uniform_coverage_equal_ranges():
    n_pos, bucket = 29903, 64
    w = np.full((n_pos + bucket - 1) // bucket, 6400, np.uint64)
    for n in (1, 2, 3, 8):
        cuts = _plan(w, bucket, n_pos, n)
        assert cuts[0] == 0 and cuts[-1] == n_pos and np.all(np.diff(cuts) > 0)
        ld = _loads(w, bucket, cuts)
        assert ld.max() <= ld.mean() * 1.01 + 6400


def test_amplicon_first_batch_then_full_coverage():
    """Plan from an amplicon-shaped batch (three 400-bp windows), then the cumulative histogram of a sample whose
    later BAMs cover the genome: the first plan crowds every cut into the windows (its last device holds most of
    the genome); the plan from the cumulative histogram is balanced again."""
    n_pos, bucket, n = 29903, 64, 8
    nb = (n_pos + bucket - 1) // bucket
    amp = np.zeros(nb, np.uint64)
    for lo in (1000, 15000, 27000):
        amp[lo // bucket:(lo + 400) // bucket] = 40000
    cuts = _plan(amp, bucket, n_pos, n)
    assert np.all(np.diff(cuts) > 0) and cuts[-1] == n_pos
    assert cuts[-2] <= 27400                        # every cut inside the windows
    full = np.full(nb, 6400, np.uint64)
    cum = amp + 20 * full                           # 1 amplicon BAM + 20 full-coverage BAMs
    ld_first = _loads(cum, bucket, cuts)
    assert ld_first.max() > 1.5 * ld_first.mean()   # what triggers the re-plan
    cuts2 = _plan(cum, bucket, n_pos, n)
    ld = _loads(cum, bucket, cuts2)
    assert ld.max() <= 1.05 * ld.mean()


def test_degenerate_inputs():
    n_pos = 100
    assert list(_plan(np.zeros(2, np.uint64), 64, n_pos, 4)) == [0, 25, 50, 75, 100]
    w = np.zeros(2, np.uint64)
    w[0] = 1000                                      # all entries in the first bucket: ranges stay non-empty
    cuts = _plan(w, 64, n_pos, 4)
    assert np.all(np.diff(cuts) >= 1) and cuts[-1] == n_pos
    with pytest.raises(RuntimeError):
        _plan(w, 64, 3, 4)                           # fewer positions than devices
