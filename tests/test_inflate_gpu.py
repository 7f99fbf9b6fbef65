"""BGZF members inflated on the GPU (spg_bgzf_inflate, csrc/spg_inflate.hip): every DEFLATE block type and zlib
strategy against Python's zlib, a simulated BAM's members against gzip, and corrupt members reported (never a fault).
The reference reads BAMs through pysam/htslib's BGZF reader (live_variant_caller.py:54-72); the bytes must be
identical.  (tests/test_inflate_check.py runs the same decoder compiled for the host.)"""
import gzip

import numpy as np
import pytest

import spings  # noqa: F401
from inflate_util import all_block_types, bgzf_members, corrupt_set, fallbacks, inflate, pack

pytestmark = pytest.mark.gpu


def test_every_block_type_and_strategy_matches_zlib():
    payloads = all_block_types(np.random.default_rng(7))
    comp, members = pack(payloads)
    out, st, _ = inflate(comp, members)
    assert (st == 0).all(), [(i, int(s)) for i, s in enumerate(st) if s]
    assert out == b"".join(d for _, d in payloads)
    assert 0 < fallbacks() < len(members) // 2     # stored blocks and token overflows went to the lane decoder


def test_simulated_bam_members_match_gzip(tmp_path):
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    ref = synth.reference(3000, seed=3)
    bam = str(tmp_path / "s.bam")
    simulate_bam(bam, "NC_045512.2", ref, depth=400.0, seed=5, n_threads=4)
    raw = open(bam, "rb").read()
    members = bgzf_members(raw)
    assert len(members) > 10
    out, st, _ = inflate(raw, members)
    assert (st == 0).all()
    assert out == gzip.decompress(raw)
    assert fallbacks() == 0                         # every member went through k_inflate_par


def test_simulated_deep_bam_parallel_kernel_only(tmp_path):
    """A 1,500x BAM (two-block members of 5-6-bit quality codes): k_inflate_par inflates every member itself."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    ref = synth.reference(6000, seed=3)
    bam = str(tmp_path / "s.bam")
    simulate_bam(bam, "NC_045512.2", ref, depth=1500.0, seed=5, n_threads=4)
    raw = open(bam, "rb").read()
    members = bgzf_members(raw)
    out, st, _ = inflate(raw, members)
    assert (st == 0).all()
    assert out == gzip.decompress(raw)
    assert fallbacks() == 0


def test_corrupt_members_are_reported():
    good, payloads = corrupt_set(np.random.default_rng(9))
    comp, members = pack(payloads)
    out, st, _ = inflate(comp, members)
    assert st[0] == 0 and out[:len(good)] == good
    assert (st[1:] != 0).all(), st


@pytest.mark.parametrize("flip", [False, True])
def test_crc_segment_edges(flip):
    """k_crc32 cuts a member into 1 KiB segments aligned to its end and combines the lanes' CRCs by a tree: member
    sizes around the segment edges (0, 1, 1,023-1,025, 2,047-2,049, 63 KiB + 1, 65,535, 65,536) at odd output offsets all
    pass, and a trailer CRC off by one bit is reported for every size (status 10) without touching the others."""
    import zlib
    from inflate_util import deflate
    rng = np.random.default_rng(17)
    sizes = [0, 1, 1023, 1024, 1025, 2047, 2048, 2049, 63 * 1024 + 1, 65535, 65536]
    datas = [rng.integers(0, 6, n, dtype=np.uint8).tobytes() for n in sizes]
    comp, members, uoff = bytearray(), [], 3                        # (odd output offsets: a 3-byte lead-in member)
    lead = b"xyz"
    for raw, data in [(deflate(lead, 6, zlib.Z_DEFAULT_STRATEGY), lead)] + \
            [(deflate(d, 6, zlib.Z_DEFAULT_STRATEGY), d) for d in datas]:
        coff = len(comp)
        comp += raw
        crc = zlib.crc32(data)
        if flip and data is not lead:
            crc ^= 1 << (len(data) % 32)
        comp += crc.to_bytes(4, "little") + len(data).to_bytes(4, "little")
        members.append((coff, len(raw), len(data), 0 if data is lead else uoff))
        uoff += 0 if data is lead else len(data)
    out, st, _ = inflate(bytes(comp), members)
    assert st[0] == 0
    if flip:
        assert (st[1:] == 10).all(), st
    else:
        assert (st == 0).all(), st
        assert out[3:] == b"".join(datas)
