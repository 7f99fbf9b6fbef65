"""The GPU inflater's decoder (csrc/spg_inflate.hip inflate_member) compiled for the host (spg_bgzf_inflate_check):
its logic checked on CPU against Python's zlib on every DEFLATE block type and strategy, against gzip on a simulated
BAM, and on corrupt members (reported, never read out of bounds).  tests/test_inflate_gpu.py runs the kernel."""
import gzip

import numpy as np

import spings  # noqa: F401
from inflate_util import all_block_types, bgzf_members, corrupt_set, inflate, pack


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
