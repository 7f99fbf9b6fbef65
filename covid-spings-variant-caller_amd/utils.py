"""Probability helpers of the reference (variant_caller/utils.py:9-24), kept for API
compatibility.  The engine does not call these per entry: eps comes from the 256-entry table that
``engine.eps_lut()`` builds with this same ``from_phred_scale`` (bit-identical on device), and GLs
are computed by the gfx950 kernels.  ``genotype_likelihood`` here serves single calls made by
user code against a dict of eps lists, with the reference's semantics (left-fold products)."""
import functools
import math
import operator
from typing import Dict, List


def from_phred_scale(score: float) -> float:
    """utils.py:9-10."""
    return math.pow(10, score / -10)


def to_phred_scale(probability: float, threshold: int = 99) -> int:
    """utils.py:12-13 (Python round: half-to-even)."""
    return min(round(-10 * math.log10(probability)), threshold) if probability > 0.0 else threshold


def _fold(xs):
    it = iter(xs)
    p = next(it, None)
    if p is None:
        return 1.0                      # np.prod([]) == 1.0
    for x in it:
        p = p * x
    return p


def genotype_likelihood(hypothesis: str, alleles: Dict[str, List[float]]) -> float:
    """utils.py:16-24: prod(1-eps_h) * prod over the other alleles (dict order) of prod(eps)."""
    hyp = _fold([1.0 - e for e in alleles[hypothesis]])
    non = functools.reduce(operator.mul, [_fold(alleles[a]) for a in alleles if a != hypothesis], 1.0)
    return hyp * non
