"""Coordinate-sharded engines on one GPU (the N>1 data path without the collective): shards
covering [0, L) merged on the host equal the single engine's call table bit-exactly."""
import numpy as np
import pytest

import spings  # noqa: F401

pytestmark = pytest.mark.gpu


def test_sharded_engines_match_single():
    from covid_spings_variant_caller_amd import shard, synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    L = 6000
    ref = synth.reference(L, seed=5)
    batches = [synth.pileup(L, 300, seed=6, ref=ref, snv_every=97, lo=0, hi=4000),
               synth.pileup(L, 200, seed=7, ref=ref, snv_every=97, lo=2500, hi=6000)]
    single = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref)
    for b in batches:
        single.accumulate(*b)
    single.finalize()
    exp = single.candidates()
    parts = shard.partition(batches[0][1], 3, batches[0][0], span=(0, L))
    engines = [shard.ShardedEngine(lo, hi, ref, device=0) for lo, hi in parts]
    for e in engines:
        for b in batches:
            e.accumulate(*b)
    got = shard.merge_candidates([e.local_candidates() for e in engines])
    assert len(exp) > 20
    for k in ("pos", "dp", "ad", "pl", "score", "ref", "alt", "gl_zero", "rank", "first_batch"):
        np.testing.assert_array_equal(got[k], exp[k], err_msg=k)
    # fp64 sums: a shard's CSR slice starts at another byte alignment, so entries meet the 16-byte
    # chunk lanes in another grouping and the sums round differently (parity bar: 1e-9 relative)
    for k in ("gl", "gl_linear", "qual"):
        np.testing.assert_allclose(got[k], exp[k], rtol=1e-12, atol=0, err_msg=k)


def test_sharded_process_bam_region_pileup_matches_single(tmp_path):
    """ShardedEngine.process_bam: each shard runs the region pileup (spp_pileup_region) of the same
    BAMs; merged call tables equal one engine over whole-contig pileups."""
    from covid_spings_variant_caller_amd import shard, synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams, simulate_bam
    L = 8000
    ref = synth.reference(L, seed=15)
    bams = []
    for i, d in enumerate((300.0, 120.0, 500.0)):
        p = str(tmp_path / f"s{i}.bam")
        simulate_bam(p, "chrQ", ref, depth=d, seed=40 + i, n_threads=4)
        bams.append(p)
    prm = PileupParams(max_depth=250, n_threads=4)
    single = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    for p in bams:
        with AlignmentFile(p) as f:
            b = f.pileup_batch("chrQ", prm)
            single.accumulate(b.pos_begin, b.offsets, b.codes, b.quals)
            b.close()
    single.finalize()
    exp = single.candidates()
    engines = [shard.ShardedEngine(lo, hi, ref, device=0) for lo, hi in ((0, 2000), (2000, 5100), (5100, L))]
    for e in engines:
        for p in bams:
            e.process_bam(p, "chrQ", prm)
    got = shard.merge_candidates([e.local_candidates() for e in engines])
    assert len(exp) > 5
    for k in ("pos", "dp", "ad", "pl", "score", "ref", "alt", "gl_zero", "rank", "first_batch"):
        np.testing.assert_array_equal(got[k], exp[k], err_msg=k)
    for k in ("gl", "gl_linear", "qual"):
        np.testing.assert_allclose(got[k], exp[k], rtol=1e-12, atol=0, err_msg=k)
