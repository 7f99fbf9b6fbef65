"""Hand-derived pileup fixtures (parity of the pileup step is unpinned: pysam/htslib is absent).

Each case is a tiny SAM whose expected CSR pileup was worked out BY HAND from the published htslib /
pysam rules (oracle/README.md, "Pileup rules"), independently of both restatements — the product's
C++ emulator (csrc/spp_pileup.cpp) and oracle/pileup_port.py.  Both must reproduce every fixture.
Reference use: live_variant_caller.py:55-60 (pileup kwargs), :75 / :89 (PileupColumn.pileups).

CSR convention (include/spings_pileup.h): columns [pos_begin, ...), codes = BAM nibbles
(A=1 C=2 G=4 T=8 N=15), 16 = CIGAR D, 17 = CIGAR N; qual of a D/N entry = the quality of the next
query base, 0 when the deletion ends the read (pysam pileup_base_qual_skip reads 0 past l_qseq).
"""
import numpy as np
import pytest

import spings  # noqa: F401
from covid_spings_variant_caller_amd import build as B
from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams
from oracle import pileup_port as pp
import samgen

A, C, G, T, N, DEL, SKIP = 1, 2, 4, 8, 15, 16, 17


@pytest.fixture(scope="module", autouse=True)
def _lib():
    B.build_pileup()


def rec(qname, pos1, cigar, seq, qual, flag=0, pnext=0, tlen=0, rnext="*"):
    return dict(qname=qname, flag=flag, rname="c", pos=pos1, mapq=60, cigar=cigar, rnext=rnext, pnext=pnext,
                tlen=tlen, seq=seq, qual="".join(chr(33 + q) for q in qual))


def both(tmp_path, recs, L=60, **kw):
    sam = str(tmp_path / "h.sam")
    samgen.write_sam(sam, [("c", L)], recs)
    with AlignmentFile(sam) as f:
        b = f.pileup_batch("c", PileupParams(n_threads=2, **kw))
        got = (b.pos_begin, b.offsets.copy(), b.codes.copy(), b.quals.copy())
    port = pp.to_csr(pp.pileup_columns(sam, "c", **kw))
    return got, port


def expect(got, pos_begin, columns):
    """columns: list of [(code, qual), ...] per column from pos_begin (hand-derived)."""
    off = np.zeros(len(columns) + 1, np.uint64)
    np.cumsum([len(c) for c in columns], out=off[1:])
    codes = np.array([c for col in columns for c, _ in col], np.uint8)
    quals = np.array([q for col in columns for _, q in col], np.uint8)
    assert got[0] == pos_begin, (got[0], pos_begin)
    np.testing.assert_array_equal(got[1], off)
    np.testing.assert_array_equal(got[2], codes)
    np.testing.assert_array_equal(got[3], quals)


def test_maxcnt_boundary(tmp_path):
    """htslib bam_plp_push: a read starting at the iterator's pending position is dropped when the
    node count (buffered reads + 1) exceeds maxcnt.  max_depth = 3; five 10M reads at pos 0, then two
    10M reads at pos 2.
    * reads 1-3 at pos 0: counts 1, 2, 3 <= 3 -> kept; reads 4-5: count 4 > 3 -> dropped.
    * the first read at pos 2 arrives while the pending position is still 0 (no column was emitted:
      nothing started past 0 yet) -> kept regardless of the count; columns 0 and 1 are emitted (3
      reads), the pending position becomes 2.
    * the second read at pos 2: pending position 2, count 4 + 1 > 3 -> dropped.
    Columns 0-1: 3 x A; 2-9: 3 x A + 1 x C; 10-11: 1 x C."""
    q = [30] * 10
    recs = [rec(f"a{i}", 1, "10M", "A" * 10, q) for i in range(5)]
    recs += [rec(f"b{i}", 3, "10M", "C" * 10, q) for i in range(2)]
    got, port = both(tmp_path, recs, max_depth=3)
    cols = [[(A, 30)] * 3] * 2 + [[(A, 30)] * 3 + [(C, 30)]] * 8 + [[(C, 30)]] * 2
    expect(got, 0, cols)
    expect(port, 0, cols)


def test_maxcnt_zero_is_uncapped(tmp_path):
    q = [30] * 4
    recs = [rec(f"a{i}", 5, "4M", "G" * 4, q) for i in range(9)]
    got, port = both(tmp_path, recs, max_depth=0)
    cols = [[(G, 30)] * 9] * 4
    expect(got, 4, cols)
    expect(port, 4, cols)


def test_deletion_inside_and_at_read_end(tmp_path):
    """resolve_cigar2: a D column is is_del with qpos = the next query base.  '3M2D2M' (quals 10 11
    12 13 14): D entries at ref 3-4 carry qual[3] = 13.  '5M2D' (deletion ending the read): qpos = 5 =
    l_qseq, so the bq filter reads 0.  'N' (refskip) gives code 17 with the same rule."""
    recs = [rec("d1", 1, "3M2D2M", "ACGTA", [10, 11, 12, 13, 14]),
            rec("d2", 1, "5M2D", "TTTTT", [20, 21, 22, 23, 24]),
            rec("n1", 1, "2M3N1M", "GGC", [30, 31, 32])]
    got, port = both(tmp_path, recs)
    cols = [
        [(A, 10), (T, 20), (G, 30)],          # ref 0
        [(C, 11), (T, 21), (G, 31)],          # ref 1
        [(G, 12), (T, 22), (SKIP, 32)],       # ref 2
        [(DEL, 13), (T, 23), (SKIP, 32)],     # ref 3
        [(DEL, 13), (T, 24), (SKIP, 32)],     # ref 4
        [(T, 13), (DEL, 0), (C, 32)],         # ref 5
        [(A, 14), (DEL, 0)],                  # ref 6
    ]
    expect(got, 0, cols)
    expect(port, 0, cols)


def _pair(seq1, q1, seq2, q2, pos2=6):
    """A proper pair (flags 99 / 147): read 1 at ref 0 (10M), its mate at ref pos2 - 1 (10M)."""
    r1 = rec("p", 1, "10M", seq1, q1, flag=99, rnext="=", pnext=pos2, tlen=pos2 + 9)
    r2 = rec("p", pos2, "10M", seq2, q2, flag=147, rnext="=", pnext=1, tlen=-(pos2 + 9))
    return [r1, r2]


def test_mate_overlap_agreement(tmp_path):
    """ignore_overlaps (htslib overlap_push -> tweak_overlap_quality): where the mates overlap (ref
    5-9) and agree, read 1 (the first pushed) gets min(q1 + q2, 200) and the mate 0."""
    got, port = both(tmp_path, _pair("A" * 10, [30] * 10, "A" * 10, [25] * 10))
    cols = [[(A, 30)]] * 5 + [[(A, 55), (A, 0)]] * 5 + [[(A, 25)]] * 5
    expect(got, 0, cols)
    expect(port, 0, cols)
    # capped at 200 (qualities above 93 need BAM: SAM text cannot carry them)
    bam = str(tmp_path / "cap.bam")
    samgen.write_bam(bam, [("c", 60)], _pair("A" * 10, [150] * 10, "A" * 10, [90] * 10))
    with AlignmentFile(bam) as f:
        b = f.pileup_batch("c", PileupParams(n_threads=2))
        got = (b.pos_begin, b.offsets.copy(), b.codes.copy(), b.quals.copy())
    expect(got, 0, [[(A, 150)]] * 5 + [[(A, 200), (A, 0)]] * 5 + [[(A, 90)]] * 5)


def test_mate_overlap_disagreement(tmp_path):
    """Mates disagree: the higher quality keeps int(0.8 q) and the other gets 0 (ties favour read 1)."""
    # read 1 higher: 30 -> 24, mate -> 0
    got, port = both(tmp_path, _pair("A" * 10, [30] * 10, "C" * 10, [20] * 10))
    cols = [[(A, 30)]] * 5 + [[(A, 24), (C, 0)]] * 5 + [[(C, 20)]] * 5
    expect(got, 0, cols)
    expect(port, 0, cols)
    # mate higher: read 1 -> 0, mate 33 -> 26
    got, port = both(tmp_path, _pair("G" * 10, [21] * 10, "T" * 10, [33] * 10))
    cols = [[(G, 21)]] * 5 + [[(G, 0), (T, 26)]] * 5 + [[(T, 33)]] * 5
    expect(got, 0, cols)
    expect(port, 0, cols)
    # tie: read 1 keeps int(0.8 * 25) = 20
    got, _ = both(tmp_path, _pair("G" * 10, [25] * 10, "T" * 10, [25] * 10))
    expect(got, 0, [[(G, 25)]] * 5 + [[(G, 20), (T, 0)]] * 5 + [[(T, 25)]] * 5)


def test_overlap_off_and_improper_pairs(tmp_path):
    """No tweak with ignore_overlaps=False, nor for a pair without the proper-pair flag (0x2)."""
    pair = _pair("A" * 10, [30] * 10, "A" * 10, [25] * 10)
    got, port = both(tmp_path, pair, ignore_overlaps=False)
    cols = [[(A, 30)]] * 5 + [[(A, 30), (A, 25)]] * 5 + [[(A, 25)]] * 5
    expect(got, 0, cols)
    expect(port, 0, cols)
    pair[0]["flag"], pair[1]["flag"] = 97, 145                      # paired, not proper
    got, port = both(tmp_path, pair)
    expect(got, 0, cols)
    expect(port, 0, cols)


def test_stepper_all_filters(tmp_path):
    """pysam stepper 'all' (pileup's default): reads with UNMAP | SECONDARY | QCFAIL | DUP (0x704)
    are skipped; MAPQ is not filtered (min_mapping_quality belongs to the samtools stepper)."""
    q = [30] * 4
    recs = [rec("ok", 1, "4M", "AAAA", q),
            dict(rec("sec", 1, "4M", "CCCC", q), flag=0x100),
            dict(rec("qc", 1, "4M", "GGGG", q), flag=0x200),
            dict(rec("dup", 1, "4M", "TTTT", q), flag=0x400),
            dict(rec("mq0", 1, "4M", "CCCC", q), mapq=0)]
    got, port = both(tmp_path, recs, min_mapping_quality=20)
    cols = [[(A, 30), (C, 30)]] * 4
    expect(got, 0, cols)
    expect(port, 0, cols)
    got, port = both(tmp_path, recs, stepper="samtools", min_mapping_quality=20)
    expect(got, 0, [[(A, 30)]] * 4)
    expect(port, 0, [[(A, 30)]] * 4)
