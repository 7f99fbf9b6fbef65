"""Device-side pileup: spg_accumulate_records' kernel (csrc/spg_fill.hip)
decodes the BAM records and walks their CIGARs on the GPU.  Its batch is checked against values the product
did not compute: the hand-derived columns of tests/test_pileup_handderived.py (worked out from the htslib /
pysam rules), oracle/pileup_port.py's column-by-column restatement on the same reads (random reads with every
CIGAR op / '*' SEQ+QUAL / stacks / overlapping pairs under each stepper and depth cap), and config 1's
restatement-generated fixture — and, on every fixture, against spp_batch_fill's host CSR (regions, long
skips, the simulator's BAMs up to 10,000x).  Then process_bam through it vs the host fill.  (Parity with
pysam itself stays unpinned: pysam/htslib is absent here and on the GPU box.)"""
import ctypes as C
import os

import numpy as np
import pytest

import spings  # noqa: F401
from covid_spings_variant_caller_amd import _native as N
from covid_spings_variant_caller_amd.engine import PileupEngine
from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams
import samgen

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def host_fill(path, contig, start=None, stop=None, **kw):
    with AlignmentFile(path) as f:
        b = f.pileup_plan(contig, PileupParams(n_threads=kw.pop("n_threads", 4), **kw), start, stop)
        b.fill()
        out = (b.pos_begin, b.offsets.copy(), b.codes.copy(), b.quals.copy())
        b.close()
    return out


def device_fill(path, contig, start=None, stop=None, pinned=False, **kw):
    if pinned:
        N.use_pinned_records()
    with AlignmentFile(path) as f:
        L = f.get_reference_length(contig)
        b = f.pileup_records(contig, PileupParams(n_threads=kw.pop("n_threads", 4), **kw), start, stop)
    eng = PileupEngine(L + 1, reference="A" * (L + 1))
    try:
        if b.n_cols == 0:
            return None
        eng.accumulate_bam_records(b)
        eng.sync()
        hist = eng.history()
        assert len(hist) == 1
        eng.finalize()
        eng.counts()                      # settles: raises if the kernel flagged an inconsistent plan
        return hist[0]
    finally:
        b.close()
        eng.close()


def bam_device_fill(path, contig, gpu_plan=False, **kw):
    """The BAM kept in HBM (spg_bam_open -> spg_bam_reads_copy -> spp_pileup_plan_fields -> spg_bam_accumulate; with
    gpu_plan the depth cap / pairing on the GPU: spg_bam_plan_build -> spg_bam_accumulate(SPG_IN_DEVICE)): the batch the
    engine then holds, or None for a contig without entries."""
    params = PileupParams(n_threads=kw.pop("n_threads", 4), **kw)
    with AlignmentFile(path) as f:
        L = f.get_reference_length(contig)
        eng = PileupEngine(L + 1, reference="A" * (L + 1))
        try:
            bmap = f.bam_map(4)
            n = eng.bam_open(bmap, f.tid(contig), params)
            bmap.close()
            assert n is not None, eng.bam_fallback
            if gpu_plan:
                plan = eng.bam_plan_build(params.max_depth, params.ignore_overlaps)
                assert plan is not None, eng.bam_fallback
                if plan.n_cols == 0:
                    return None
                assert eng.bam_accumulate_planned(plan), eng.bam_fallback
                b = None
            else:
                b = f.pileup_fields(contig, eng.bam_reads(n), params)
            try:
                if b is not None:
                    if b.n_cols == 0:
                        return None
                    assert eng.bam_accumulate(b), eng.bam_fallback
                eng.sync()
                hist = eng.history()
                assert len(hist) == 1
                eng.finalize()
                eng.counts()                  # settles: raises if the fill flagged an inconsistent plan
                return hist[0]
            finally:
                if b is not None:
                    b.close()
        finally:
            eng.close()


def _host_plan_arrays(v):
    """spp_pileup_plan_fields' spg_bam_plan (host pointers) as numpy arrays."""
    def arr(p, n, t):
        if n <= 0 or not p:
            return np.zeros(0, t)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(t))), shape=(n,)).copy()
    return {"offsets": arr(v.offsets, int(v.n_cols) + 1, np.uint64), "kept": arr(v.kept, int(v.n_kept), np.uint32),
            "pair_a": arr(v.pair_a, int(v.n_pairs), np.uint32), "pair_b": arr(v.pair_b, int(v.n_pairs), np.uint32),
            "pair_col": arr(v.pair_col, int(v.n_pairs), np.int64), "pair_orig": arr(v.pair_orig, int(v.n_pairs), np.uint64)}


def plan_compare(path, contig, **kw):
    """spg_bam_plan_build (htslib's depth cap and mate pairing on the GPU) against spp_pileup_plan_fields (the host's
    replay of bam_plp_push / bam_plp_next on the same reads' fields): every array of the plan identical.  Returns the
    number of pairs and of kept reads, or None when the GPU declined (then the reads hold one without reference span)."""
    params = PileupParams(n_threads=kw.pop("n_threads", 4), **kw)
    with AlignmentFile(path) as f:
        L = f.get_reference_length(contig)
        eng = PileupEngine(L + 1, reference="A" * (L + 1))
        try:
            bmap = f.bam_map(4)
            n = eng.bam_open(bmap, f.tid(contig), params)
            bmap.close()
            assert n is not None, eng.bam_fallback
            dplan = eng.bam_plan_build(params.max_depth, params.ignore_overlaps)
            reads = eng.bam_reads(n)
            if dplan is None:
                assert "reference span" in eng.bam_fallback and (reads["end"] <= reads["pos"]).any(), eng.bam_fallback
                return None
            dev = eng.bam_plan_arrays(dplan)
            b = f.pileup_fields(contig, reads, params)
            try:
                hv = b.device_plan()
                host = _host_plan_arrays(hv)
                if int(hv.n_cols) == 0:
                    assert int(dplan.n_cols) == 0
                    return 0, 0
                for k in ("pos_begin", "n_cols", "n_entries", "n_kept", "n_pairs", "orig_bytes", "max_span"):
                    assert int(getattr(dplan, k)) == int(getattr(hv, k)), k
                for k in host:
                    np.testing.assert_array_equal(dev[k], host[k], err_msg=k)
                return int(hv.n_pairs), int(hv.n_kept)
            finally:
                b.close()
        finally:
            eng.close()


def assert_same(a, b):
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_array_equal(a[3], b[3])


def sam_to_bam(sam, bam):
    targets, recs = [], []
    for line in open(sam):
        if line.startswith("@SQ"):
            f = dict(x.split(":", 1) for x in line.rstrip("\n").split("\t")[1:])
            targets.append((f["SN"], int(f["LN"])))
        elif line.strip() and not line.startswith("@"):
            v = line.rstrip("\n").split("\t")
            recs.append(dict(qname=v[0], flag=int(v[1]), rname=v[2], pos=int(v[3]), mapq=int(v[4]), cigar=v[5],
                             rnext=v[6], pnext=int(v[7]), tlen=int(v[8]), seq=v[9], qual=v[10]))
    samgen.write_bam(bam, targets, recs, block=3000)
    return targets


def test_testfile_config1(tmp_path):
    """Config 1's input (test/testdata/testfile.sam as BAM): 4 reads, 421 columns, 1,642 entries."""
    bam = str(tmp_path / "t.bam")
    sam_to_bam(os.path.join(GOLD, "testfile.sam"), bam)
    got = device_fill(bam, "NC_045512.2")
    assert got[0] == 10 and len(got[1]) == 422 and int(got[1][-1]) == 1642
    assert_same(got, host_fill(bam, "NC_045512.2"))
    assert_same(bam_device_fill(bam, "NC_045512.2"), got)
    z = np.load(os.path.join(GOLD, "testfile_pileup.npz"))
    np.testing.assert_array_equal(got[2], z["codes"])
    np.testing.assert_array_equal(got[3], z["quals"])


def _port(recs, contig, targets, tmp_path, **kw):
    """oracle/pileup_port.py (the column-by-column restatement, a construction independent of the product's
    emulator) on the same reads written as SAM text."""
    from oracle import pileup_port as pp
    sam = str(tmp_path / "port.sam")
    samgen.write_sam(sam, targets, recs)
    return pp.to_csr(pp.pileup_columns(sam, contig, **kw))


def _hand_cases():
    """(records, pileup kwargs, hand-derived columns from pos_begin, pos_begin): the fixtures of
    tests/test_pileup_handderived.py, whose expected columns were worked out by hand from the htslib / pysam
    rules (oracle/README.md)."""
    import test_pileup_handderived as H
    A, C, G, T, DEL, SKIP = H.A, H.C, H.G, H.T, H.DEL, H.SKIP
    q = [30] * 10
    yield ([H.rec(f"a{i}", 1, "10M", "A" * 10, q) for i in range(5)] + [H.rec(f"b{i}", 3, "10M", "C" * 10, q) for i in range(2)],
           dict(max_depth=3), [[(A, 30)] * 3] * 2 + [[(A, 30)] * 3 + [(C, 30)]] * 8 + [[(C, 30)]] * 2, 0)
    yield [H.rec(f"a{i}", 5, "4M", "G" * 4, [30] * 4) for i in range(9)], dict(max_depth=0), [[(G, 30)] * 9] * 4, 4
    yield ([H.rec("d1", 1, "3M2D2M", "ACGTA", [10, 11, 12, 13, 14]), H.rec("d2", 1, "5M2D", "TTTTT", [20, 21, 22, 23, 24]),
            H.rec("n1", 1, "2M3N1M", "GGC", [30, 31, 32])], dict(),
           [[(A, 10), (T, 20), (G, 30)], [(C, 11), (T, 21), (G, 31)], [(G, 12), (T, 22), (SKIP, 32)],
            [(DEL, 13), (T, 23), (SKIP, 32)], [(DEL, 13), (T, 24), (SKIP, 32)], [(T, 13), (DEL, 0), (C, 32)],
            [(A, 14), (DEL, 0)]], 0)
    yield (H._pair("A" * 10, [30] * 10, "A" * 10, [25] * 10), dict(),
           [[(A, 30)]] * 5 + [[(A, 55), (A, 0)]] * 5 + [[(A, 25)]] * 5, 0)
    yield (H._pair("A" * 10, [150] * 10, "A" * 10, [90] * 10), dict(),
           [[(A, 150)]] * 5 + [[(A, 200), (A, 0)]] * 5 + [[(A, 90)]] * 5, 0)
    yield (H._pair("A" * 10, [30] * 10, "C" * 10, [20] * 10), dict(),
           [[(A, 30)]] * 5 + [[(A, 24), (C, 0)]] * 5 + [[(C, 20)]] * 5, 0)
    yield (H._pair("G" * 10, [21] * 10, "T" * 10, [33] * 10), dict(),
           [[(G, 21)]] * 5 + [[(G, 0), (T, 26)]] * 5 + [[(T, 33)]] * 5, 0)
    yield (H._pair("G" * 10, [25] * 10, "T" * 10, [25] * 10), dict(),
           [[(G, 25)]] * 5 + [[(G, 20), (T, 0)]] * 5 + [[(T, 25)]] * 5, 0)
    yield (H._pair("A" * 10, [30] * 10, "A" * 10, [25] * 10), dict(ignore_overlaps=False),
           [[(A, 30)]] * 5 + [[(A, 30), (A, 25)]] * 5 + [[(A, 25)]] * 5, 0)
    improper = H._pair("A" * 10, [30] * 10, "A" * 10, [25] * 10)
    improper[0]["flag"], improper[1]["flag"] = 97, 145
    yield improper, dict(), [[(A, 30)]] * 5 + [[(A, 30), (A, 25)]] * 5 + [[(A, 25)]] * 5, 0
    q4 = [30] * 4
    flt = [H.rec("ok", 1, "4M", "AAAA", q4), dict(H.rec("sec", 1, "4M", "CCCC", q4), flag=0x100),
           dict(H.rec("qc", 1, "4M", "GGGG", q4), flag=0x200), dict(H.rec("dup", 1, "4M", "TTTT", q4), flag=0x400),
           dict(H.rec("mq0", 1, "4M", "CCCC", q4), mapq=0)]
    yield flt, dict(min_mapping_quality=20), [[(A, 30), (C, 30)]] * 4, 0
    yield flt, dict(stepper="samtools", min_mapping_quality=20), [[(A, 30)]] * 4, 0


N_HAND = 12


@pytest.mark.parametrize("case", range(N_HAND))
def test_hand_derived_fixtures(tmp_path, case):
    """The GPU fill against the hand-derived columns directly (not only against the host fill), and against
    oracle/pileup_port.py where SAM text can carry the qualities (<= 93)."""
    import test_pileup_handderived as H
    recs, kw, cols, pb = list(_hand_cases())[case]
    bam = str(tmp_path / "h.bam")
    samgen.write_bam(bam, [("c", 60)], recs)
    got = device_fill(bam, "c", **kw)
    H.expect(got, pb, cols)
    H.expect(bam_device_fill(bam, "c", **kw), pb, cols)
    H.expect(bam_device_fill(bam, "c", gpu_plan=True, **kw), pb, cols)
    plan_compare(bam, "c", **kw)
    if all(ord(ch) - 33 <= 93 for r in recs for ch in r["qual"]):
        assert_same(got, _port(recs, "c", [("c", 60)], tmp_path, **kw))
    assert_same(got, host_fill(bam, "c", **kw))


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("kw", [dict(), dict(max_depth=4), dict(max_depth=0), dict(ignore_overlaps=False, max_depth=3),
                                dict(stepper="samtools", min_mapping_quality=20, max_depth=6), dict(stepper="nofilter")])
def test_random_reads(tmp_path, seed, kw):
    """Random reads with every CIGAR op, '*' SEQ/QUAL, stacks and overlapping pairs: the GPU fill against
    oracle/pileup_port.py, and against the host fill."""
    contigs = [("chrA", 700), ("chrB", 700)]
    recs = samgen.random_records(seed, contigs, n_reads=400)
    bam = str(tmp_path / "r.bam")
    samgen.write_bam(bam, contigs, recs, block=5000)
    for c, _ in contigs:
        got = device_fill(bam, c, **kw)
        port = _port(recs, c, contigs, tmp_path, **kw)
        if got is None:
            assert int(port[1][-1]) == 0
            continue
        assert_same(got, port)
        assert_same(got, host_fill(bam, c, **kw))
        assert_same(bam_device_fill(bam, c, **kw), port)
        if plan_compare(bam, c, **kw) is not None:
            assert_same(bam_device_fill(bam, c, gpu_plan=True, **kw), port)


@pytest.mark.parametrize("region", [(100, 300), (0, 50), (550, 700), (250, 251)])
def test_regions(tmp_path, region):
    contigs = [("chrA", 700)]
    bam = str(tmp_path / "r.bam")
    samgen.write_bam(bam, contigs, samgen.random_records(7, contigs, n_reads=500), block=9000)
    assert_same(device_fill(bam, "chrA", *region), host_fill(bam, "chrA", *region))


def test_long_spans_and_gaps(tmp_path):
    """Reads with 5 kb N skips (the tile look-back spans ~80 tiles) around a coverage gap."""
    recs = []
    for i in range(60):
        s = 1 + 37 * i if i < 30 else 9000 + 11 * i
        cig = "20M5000N30M" if i % 3 == 0 else "50M"
        recs.append(dict(qname=f"r{i}", flag=0, rname="c", pos=s, mapq=60, cigar=cig, rnext="*", pnext=0, tlen=0,
                         seq="ACGTN" * 10, qual="".join(chr(33 + (7 * i + j) % 42) for j in range(50))))
    recs.sort(key=lambda r: r["pos"])
    bam = str(tmp_path / "g.bam")
    samgen.write_bam(bam, [("c", 20000)], recs)
    assert_same(device_fill(bam, "c", max_depth=0), host_fill(bam, "c", max_depth=0))
    assert_same(bam_device_fill(bam, "c", max_depth=0), host_fill(bam, "c", max_depth=0))
    assert_same(bam_device_fill(bam, "c", gpu_plan=True, max_depth=0), host_fill(bam, "c", max_depth=0))
    plan_compare(bam, "c", max_depth=0)
    plan_compare(bam, "c", max_depth=7)


@pytest.mark.parametrize("depth,max_depth", [(200, 8000), (10000, 8000), (10000, 0)])
def test_simulated_bams(tmp_path, depth, max_depth):
    """The simulator's reads (150M, 1 % 2D / 2I) over 3 kb, up to 10,000x — through the pinned path."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    bam = str(tmp_path / "s.bam")
    simulate_bam(bam, "NC_045512.2", synth.reference(3000, seed=1), depth=depth, seed=5, n_threads=8)
    host = host_fill(bam, "NC_045512.2", max_depth=max_depth)
    assert_same(device_fill(bam, "NC_045512.2", pinned=True, max_depth=max_depth), host)
    assert_same(bam_device_fill(bam, "NC_045512.2", max_depth=max_depth), host)
    assert_same(bam_device_fill(bam, "NC_045512.2", gpu_plan=True, max_depth=max_depth), host)
    n_pairs, n_kept = plan_compare(bam, "NC_045512.2", max_depth=max_depth)
    assert n_kept > 0                             # (the simulator's reads are single-end: no pairs)


@pytest.mark.parametrize("read_len", [60, 300])
def test_simulated_read_lengths(tmp_path, read_len):
    """k_f2_fill stages each chunk's record bytes in LDS when they fit (20 KiB a chunk: 64 reads of ~150 bp) and keeps
    register windows over global memory otherwise: 60 bp reads take the LDS form, 300 bp reads (~30 KiB a chunk) the
    window form — both bit-identical to the host fill."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    bam = str(tmp_path / "s.bam")
    simulate_bam(bam, "NC_045512.2", synth.reference(3000, seed=1), depth=2000, seed=7, n_threads=8, read_len=read_len)
    host = host_fill(bam, "NC_045512.2", max_depth=0)
    assert_same(device_fill(bam, "NC_045512.2", pinned=True, max_depth=0), host)
    assert_same(bam_device_fill(bam, "NC_045512.2", max_depth=0), host)


def test_bam_device_declines_corrupt_member(tmp_path):
    """A member whose compressed bytes were damaged (its CRC32 no longer matches, or it fails to decode): spg_bam_open
    declines the BAM (return 1, nothing accumulated) and process_bam takes the records plan, whose host inflate
    reports the damage as the reference's pysam would (an exception), or recovers when the damage was harmless."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    bam = str(tmp_path / "s.bam")
    ref = synth.reference(3000, seed=1)
    simulate_bam(bam, "NC_045512.2", ref, depth=300, seed=5, n_threads=4)
    with AlignmentFile(bam) as f:
        bmap = f.bam_map(4)
        mem = np.ctypeslib.as_array(C.cast(bmap.info.members, C.POINTER(C.c_uint64)), (bmap.info.n_members * 3,))
        k = bmap.info.n_members // 2
        coff, clen = int(mem[3 * k]), int(mem[3 * k + 1] & 0xFFFFFFFF)
        comp = np.ctypeslib.as_array(C.cast(bmap.info.comp, C.POINTER(C.c_uint8)), (bmap.info.comp_bytes,))
        comp[coff + clen] ^= 0x5A                    # the member's stored CRC32: the data decodes, the check fails
        eng = PileupEngine(3001, reference=ref + "A")
        assert eng.bam_open(bmap, f.tid("NC_045512.2"), PileupParams()) is None
        assert "did not inflate" in eng.bam_fallback and "status 10" in eng.bam_fallback
        bmap.close()
        eng.close()


def test_process_bam_device_pileup_matches_host(tmp_path):
    """LiveVariantCaller.process_bam (live_variant_caller.py:54-72) over 3 BAMs with the BAM kept in HBM
    (pileup="device", spg_bam_*), the records plan (pileup="records", with and without the GPU inflater) and the host
    fill (pileup="host"): identical prepare_variants() and memory."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.live_variant_caller import LiveVariantCaller
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    ref = synth.reference(4000, seed=3)
    fa = str(tmp_path / "r.fa")
    samgen.write_fasta(fa, [("NC_045512.2", ref)])
    bams = []
    for k in range(3):
        p = str(tmp_path / f"b{k}.bam")
        simulate_bam(p, "NC_045512.2", ref, depth=300, seed=10 + k, n_threads=4, snv_every=97)
        bams.append(p)
    out = []
    for mode, gi in (("device", True), ("records", True), ("records", False), ("host", True)):
        vc = LiveVariantCaller(fa, 20, 0, 10, 5, 0.1, 0, pileup=mode, gpu_inflate=gi, device_min_bytes=0)
        assert vc.device_pileup == (mode != "host")
        for p in bams:
            vc.process_bam(p)
            assert vc.last_bam_path == mode
        out.append((vc.prepare_variants(), {k: (v["reference"], v["totalDepth"]) for k, v in vc.memory.items()}))
        del vc
    assert len(out[0][0]) > 0
    for o in out[1:]:
        assert o[0] == out[0][0]
        assert o[1] == out[0][1]


@pytest.mark.parametrize("max_depth", [0, 1, 2, 50, 333, 2000, 8000])
@pytest.mark.parametrize("ignore_overlaps", [True, False])
def test_gpu_plan_caps_and_pairs(tmp_path, max_depth, ignore_overlaps):
    """spg_bam_plan_build vs spp_pileup_plan_fields over depth caps from 1 (only the first read of each start position)
    to pysam's 8,000, with and without htslib's mate pairing: the simulator's 2,000x single-end reads (150M, indels) and
    short reads (the sweep's window is min(64, shortest span) positions), and samgen's random reads with overlapping
    proper pairs, stacks and every CIGAR op."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    ref = synth.reference(4000, seed=3)
    for k, kw in enumerate([dict(depth=2000.0), dict(depth=600.0, read_len=40)]):
        bam = str(tmp_path / f"p{k}.bam")
        simulate_bam(bam, "NC_045512.2", ref, seed=11 + k, n_threads=8, **kw)
        got = plan_compare(bam, "NC_045512.2", max_depth=max_depth, ignore_overlaps=ignore_overlaps)
        assert got is not None and got[1] > 0
    contigs = [("chrA", 900)]
    n_pairs = 0
    for seed in (21, 22, 23):
        bam = str(tmp_path / f"r{seed}.bam")
        samgen.write_bam(bam, contigs, samgen.random_records(seed, contigs, n_reads=600), block=7000)
        got = plan_compare(bam, "chrA", max_depth=max_depth, ignore_overlaps=ignore_overlaps)
        if got is not None:
            n_pairs += got[0]
    assert (n_pairs > 0) == ignore_overlaps


def test_gpu_plan_name_groups_and_gaps(tmp_path):
    """Reads that share a name beyond a pair (secondary-like triples, a mate that is dropped by the cap, a mate freed
    before its partner arrives) and coverage gaps longer than the sweep's ring: the name-group replay and the sweep's
    gap handling, vs the host replay and pileup_port."""
    recs = []
    rng = np.random.default_rng(5)
    names = [f"q{i}" for i in range(90)]
    for i in range(400):
        pos = 1 + int(rng.integers(0, 300)) if i < 300 else 20000 + int(rng.integers(0, 200))
        nm = names[int(rng.integers(0, len(names)))]
        fl = int(rng.choice([0x1 | 0x2 | 0x20, 0x1 | 0x2 | 0x10, 0x1 | 0x2, 0]))
        mpos = pos + int(rng.integers(-60, 120))
        recs.append(dict(qname=nm, flag=fl, rname="c", pos=pos, mapq=60, cigar="50M", rnext="=" if fl else "*",
                         pnext=max(1, mpos) if fl else 0, tlen=int(rng.integers(-300, 300)) if fl else 0,
                         seq="".join("ACGT"[int(x)] for x in rng.integers(0, 4, 50)),
                         qual="".join(chr(33 + int(x)) for x in rng.integers(10, 40, 50))))
    recs.sort(key=lambda r: r["pos"])
    bam = str(tmp_path / "g.bam")
    samgen.write_bam(bam, [("c", 30000)], recs, block=4000)
    for md in (0, 3, 12):
        got = plan_compare(bam, "c", max_depth=md)
        assert got is not None
        port = _port(recs, "c", [("c", 30000)], tmp_path, max_depth=md)
        assert_same(bam_device_fill(bam, "c", gpu_plan=True, max_depth=md), port)
