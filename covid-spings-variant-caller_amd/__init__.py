"""MI355X-native pileup + genotype-likelihood engine for the COVID-SpiNGS live variant caller.

Drop-in for the hot path of variant_caller/live_variant_caller.py (process_bam / prepare_variants /
write_vcf) and variant_caller/utils.py.  Compute runs in hand-written gfx950 HIP kernels behind the
C-ABI in include/spings_gpu.h; this package is the host side (ctypes bindings, the
LiveVariantCaller-compatible shim, BAM/SAM pileup front end, multi-GPU sharding).
"""
__version__ = "0.1.0"

from .engine import PileupEngine, eps_lut, device_count  # noqa: F401
from .utils import from_phred_scale, to_phred_scale, genotype_likelihood  # noqa: F401
from .structs import Site, Variant  # noqa: F401


def __getattr__(name):
    if name == "LiveVariantCaller":
        from .live_variant_caller import LiveVariantCaller
        return LiveVariantCaller
    raise AttributeError(name)
