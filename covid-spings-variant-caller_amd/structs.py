"""State types of the reference (variant_caller/structs.py:2-14), kept for API compatibility.
``Variant['qual']`` is annotated int in the reference but holds np.float64 (np.mean)."""
from typing import Dict, List, Tuple, TypedDict


class Site(TypedDict):
    reference: str
    totalDepth: int
    snvs: Dict[str, List[int]]
    indels: Dict[str, List[int]]


class Variant(TypedDict):
    start: int
    stop: int
    alleles: Tuple[str, str]
    qual: float
    info: Dict
