"""The deep kernel's SWAR entry classification (csrc/spg_kernels.hip: swar4), restated in numpy and
checked against the per-entry definition it replaces: process_svn's allele key plus pysam's base-quality
filter (live_variant_caller.py:96-103).

fast = valid & q >= max(min_bq, 4) & q < 128 & code == M   (summed in bulk)
rare = valid & (q >= min_bq | q >= 128) & !fast             (decoded exactly, filtered by min_bq there)

The rare set may over-approximate (q >= 128 below min_bq; the entry after a code byte >= 128, which valid
input never holds) because the rare path re-applies the exact filter and accumulates exactly; the test
checks that contract: nothing is fast that should not be, and every entry that passes the filter and is
not fast is rare."""
import numpy as np
import pytest

M32 = np.uint64(0xFFFFFFFF)


def swar4(cw, qw, v80, mrep, kpass, kok):
    cw, qw, v80 = (x.astype(np.uint64) for x in (cw, qw, v80))
    q7 = qw & np.uint64(0x7F7F7F7F)
    pass_ = (q7 + np.uint64(kpass)) & M32
    ok = (q7 + np.uint64(kok)) & M32
    ne = ((cw ^ np.uint64(mrep)) + np.uint64(0x7F7F7F7F)) & M32
    fast = ok & ~(ne | qw | cw) & v80 & M32
    rare = (pass_ | qw) & ~fast & v80 & M32
    return fast, rare


def params(min_bq):
    qlo = max(min_bq, 4)
    kpass = 0x80808080 if min_bq <= 0 else (0 if min_bq >= 128 else (0x80 - min_bq) * 0x01010101)
    kok = 0 if qlo >= 128 else (0x80 - qlo) * 0x01010101
    return qlo, kpass, kok


@pytest.mark.parametrize("min_bq", [0, 1, 4, 13, 30, 60, 127, 128, 200])
@pytest.mark.parametrize("M", [1, 2, 4, 8])
def test_swar_matches_per_entry_rules(min_bq, M):
    rng = np.random.default_rng(min_bq * 31 + M)
    n = 200_000
    # codes: mostly valid BAM nibbles / D / N-skip, some stray bytes >= 18 and >= 128
    codes = rng.choice(np.r_[np.arange(18), [18, 100, 127, 128, 200, 255]], size=(n, 4),
                       p=np.r_[np.full(18, 0.9 / 18), np.full(6, 0.1 / 6)]).astype(np.uint8)
    codes[rng.random((n, 4)) < 0.4] = M
    quals = rng.integers(0, 256, size=(n, 4), dtype=np.uint8)
    quals[rng.random((n, 4)) < 0.5] = rng.integers(0, 64, size=1)[0]
    valid = rng.random((n, 4)) < 0.9
    cw = codes.view("<u4").ravel()
    qw = quals.view("<u4").ravel()
    v80 = (valid.astype(np.uint8) * 0x80).view("<u4").ravel()
    qlo, kpass, kok = params(min_bq)
    fast, rare = swar4(cw, qw, v80, M * 0x01010101, kpass, kok)
    fbytes = fast.astype("<u4").view(np.uint8).reshape(n, 4)
    rbytes = rare.astype("<u4").view(np.uint8).reshape(n, 4)
    assert np.all((fbytes & 0x7F) == 0) and np.all((rbytes & 0x7F) == 0)
    is_fast = fbytes != 0
    is_rare = rbytes != 0
    q = quals.astype(int)
    want_fast = valid & (q >= qlo) & (q < 128) & (codes == M)
    passes = valid & (q >= min_bq)
    carry_in = np.zeros_like(valid)
    carry_in[:, 1:] = codes[:, :-1] >= 128                           # (code ^ M) + 0x7F carries out
    assert not np.any(is_fast & ~want_fast)
    assert np.all(carry_in[want_fast & ~is_fast])                     # fast entries demoted ...
    assert np.all(is_rare[want_fast & ~is_fast])                      # ... to the exact rare path
    assert not np.any(is_fast & is_rare)
    assert np.all(is_rare[passes & ~want_fast])                       # nothing that counts is lost
    assert not np.any(is_rare & ~valid)
    # over-approximation only where the exact path filters it out again (or a code byte >= 128)
    extra = is_rare & ~(passes & ~want_fast)
    assert np.all((q[extra] >= 128) | (codes[extra] >= 128) | carry_in[extra])
