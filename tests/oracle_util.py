"""Helpers shared by the tests: golden-case loading and normalised comparisons."""
from __future__ import annotations

import json
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "cases.json")


def load_golden():
    with open(GOLDEN) as f:
        return json.load(f)


def golden_case(name):
    for c in load_golden()["cases"]:
        if c["name"] == name:
            return c
    raise KeyError(name)


def gl_expected(case):
    return {int(p): {a: float.fromhex(h) for a, h in rows} for p, rows in case["expected"]["gl"]}


def variants_expected(case):
    out = []
    for v in case["expected"]["variants"]:
        info = {k: (float.fromhex(x) if isinstance(x, str) else x) for k, x in v["info"].items()}
        out.append({"start": v["start"], "stop": v["stop"], "alleles": tuple(v["alleles"]),
                    "qual": float.fromhex(v["qual"]) if isinstance(v["qual"], str) else v["qual"], "info": info})
    return out


def norm_variants(vs):
    out = []
    for v in vs:
        out.append({"start": int(v["start"]), "stop": int(v["stop"]), "alleles": tuple(v["alleles"]),
                    "qual": float(v["qual"]),
                    "info": {k: (float(x) if isinstance(x, (float, np.floating)) else int(x))
                             for k, x in v["info"].items()}})
    return out


def rel_close(a, b, rtol):
    if a == b:
        return True
    if a == 0 or b == 0 or math.isnan(a) or math.isnan(b):
        return False
    return abs(a - b) <= rtol * max(abs(a), abs(b))


def compare_variants(got, exp, rtol=0.0):
    """Exact on everything integer; GL / QUAL within rtol (0.0 = bit-exact)."""
    got, exp = norm_variants(got), norm_variants(exp)
    assert len(got) == len(exp), f"{len(got)} variants vs {len(exp)} expected"
    for g, e in zip(got, exp):
        assert (g["start"], g["stop"], g["alleles"]) == (e["start"], e["stop"], e["alleles"]), (g, e)
        for k in ("DP", "AD", "PL", "SCORE"):
            assert g["info"][k] == e["info"][k], (k, g, e)
        assert rel_close(g["info"]["GL"], e["info"]["GL"], rtol), ("GL", g, e)
        assert rel_close(g["qual"], e["qual"], rtol), ("QUAL", g, e)


def batches_np(case):
    for b in case["batches"]:
        yield (b["pos_begin"], np.asarray(b["offsets"], np.uint64), np.asarray(b["codes"], np.uint8),
               np.asarray(b["quals"], np.uint8))
