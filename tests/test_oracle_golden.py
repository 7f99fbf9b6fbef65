"""Pin the oracle: both CPU restatements vs. golden vectors produced by the reference's own code."""
import math

import numpy as np
import pytest

from oracle import reference_port as rp
from oracle.c_oracle import COracle
from oracle_util import (batches_np, compare_variants, gl_expected, load_golden, variants_expected)

GOLD = load_golden()
CASES = GOLD["cases"]


def test_eps_lut_matches_reference():
    lut = rp.eps_lut()
    assert [float(x).hex() for x in lut] == GOLD["eps_lut"]


def test_to_phred_grid():
    for h, expect in GOLD["to_phred"]:
        assert rp.to_phred_scale(float.fromhex(h)) == expect


def test_np_prod_is_left_fold():
    rng = np.random.default_rng(7)
    for _ in range(200):
        a = 10 ** (-rng.integers(2, 42, size=int(rng.integers(1, 2000))) / 10)
        p = a[0]
        for x in a[1:]:
            p *= x
        assert a.prod() == p


def _port(case):
    p = case["params"]
    o = rp.OracleCaller(case["reference"], p["minBaseQuality"], p["minTotalDepth"], p["minAlleleDepth"],
                        p["minEvidenceRatio"])
    for pb, off, c, q in batches_np(case):
        o.accumulate(pb, off, c, q)
    return o


def _coracle(case):
    p = case["params"]
    o = COracle(case["reference"], p["minBaseQuality"], p["minTotalDepth"], p["minAlleleDepth"],
                p["minEvidenceRatio"])
    for pb, off, c, q in batches_np(case):
        o.accumulate(pb, off, c, q)
    o.finalize()
    return o


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_python_port_bit_exact(case):
    o = _port(case)
    mem = [[p, s["reference"], s["totalDepth"], [[a, len(v)] for a, v in s["snvs"].items()]]
           for p, s in o.memory.items()]
    assert mem == case["expected"]["memory"]
    gl = o.gl_table()
    exp = gl_expected(case)
    assert list(gl.keys()) == list(exp.keys())
    for pos in exp:
        assert list(gl[pos].keys()) == list(exp[pos].keys())
        for a in exp[pos]:
            assert float(gl[pos][a]).hex() == float(exp[pos][a]).hex()
    compare_variants(o.prepare_variants(), variants_expected(case), rtol=0.0)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_c_oracle_bit_exact(case):
    o = _coracle(case)
    assert o.memory_summary() == case["expected"]["memory"]
    gl = o.gl_table()
    exp = gl_expected(case)
    assert list(gl.keys()) == list(exp.keys())
    for pos in exp:
        assert list(gl[pos].keys()) == list(exp[pos].keys())
        for a in exp[pos]:
            assert float(gl[pos][a]).hex() == float(exp[pos][a]).hex(), (pos, a)
    compare_variants(o.variants(), variants_expected(case), rtol=0.0)


def test_band_case_really_exercises_subnormals():
    case = next(c for c in CASES if c["name"] == "band")
    vals = [v for row in gl_expected(case).values() for v in row.values()]
    assert any(0 < v < 2.2250738585072014e-308 for v in vals)
    assert any(v == 0 for v in vals)
    assert any(v >= 2.2250738585072014e-308 for v in vals)
