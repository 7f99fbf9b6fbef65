"""The GPU inflater's decoder (csrc/spg_inflate.hip inflate_member) compiled for the host (spg_bgzf_inflate_check):
its logic checked on CPU against Python's zlib on every DEFLATE block type and strategy, against gzip on a simulated
BAM, and on corrupt members (reported, never read out of bounds).  tests/test_inflate_gpu.py runs the kernel."""
import gzip

import numpy as np

import spings  # noqa: F401
from inflate_util import all_block_types, bgzf_members, corrupt_set, inflate, inflate_par_host, pack


def test_decoder_every_block_type_and_strategy_matches_zlib():
    payloads = all_block_types(np.random.default_rng(7))
    comp, members = pack(payloads)
    out, st, _ = inflate(comp, members, gpu=False)
    assert (st == 0).all(), [(i, int(s)) for i, s in enumerate(st) if s]
    assert out == b"".join(d for _, d in payloads)


def test_decoder_simulated_bam_matches_gzip(tmp_path):
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    ref = synth.reference(3000, seed=3)
    bam = str(tmp_path / "s.bam")
    simulate_bam(bam, "NC_045512.2", ref, depth=400.0, seed=5, n_threads=4)
    raw = open(bam, "rb").read()
    members = bgzf_members(raw)
    out, st, _ = inflate(raw, members, gpu=False)
    assert (st == 0).all()
    assert out == gzip.decompress(raw)


def test_decoder_corrupt_members_are_reported():
    good, payloads = corrupt_set(np.random.default_rng(9))
    comp, members = pack(payloads)
    out, st, _ = inflate(comp, members, gpu=False)
    assert st[0] == 0 and out[:len(good)] == good
    assert (st[1:] != 0).all(), st


def test_parallel_algorithm_every_block_type_matches_zlib():
    """k_inflate_par's segment decode + sync + resolve (the same functions, lane after lane on the host): every member it
    keeps is zlib's bytes; it leaves only stored blocks and token overflows (highly compressible data) to the lane
    decoder."""
    payloads = all_block_types(np.random.default_rng(7))
    comp, members = pack(payloads)
    out, st, stats = inflate_par_host(comp, members)
    uo = 0
    for (raw, data), s in zip(payloads, st):
        if s == 0:
            assert out[uo:uo + len(data)] == data
        uo += len(data)
    assert (st == 0).sum() == stats[0] and stats[0] > len(members) // 2
    assert stats[2] == stats[4] == stats[5] == stats[6] == 0, stats      # no sync failure, no bad header / resolve


def test_parallel_algorithm_simulated_bam_no_fallback(tmp_path):
    """On a simulator BAM (zlib members of two blocks, ~5-6-bit quality codes: the slowest self-synchronisation seen)
    every member is inflated by the parallel algorithm, identical to gzip."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    ref = synth.reference(6000, seed=3)
    bam = str(tmp_path / "s.bam")
    simulate_bam(bam, "NC_045512.2", ref, depth=1500.0, seed=5, n_threads=4)
    raw = open(bam, "rb").read()
    members = bgzf_members(raw)
    out, st, stats = inflate_par_host(raw, members)
    assert (st == 0).all(), stats
    assert out == gzip.decompress(raw)
    assert stats[8] > len(members)                  # (multi-block members were exercised)
