"""The host half of the BAM-in-HBM path (CPU): spp_bam_map_open (the file's BGZF members and header end, checked
against Python's gzip and a header parse) and spp_pileup_plan_fields (htslib's depth cap and mate pairing replayed on
the reads' fixed fields as spg_bam_reads_copy returns them, names as 64-bit hashes): its CSR offsets and kept reads
equal the host plan of the same BAM (spp_pileup_plan), and its overlapping mate pairs are the records plan's tweaked
reads, for every stepper, depth cap and overlap setting."""
import gzip
import struct

import numpy as np
import pytest

import spings  # noqa: F401
import samgen
from covid_spings_variant_caller_amd import _native as N
from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams


def fnv1a64(s: bytes) -> int:
    h = 0xcbf29ce484222325
    for b in s:
        h = ((h ^ b) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def _keeps(flag, mapq, kw):
    stepper = kw.get("stepper", "all")
    if flag & 0x4:
        return False
    if stepper == "nofilter":
        return True
    if stepper == "all":
        return not flag & (0x4 | 0x100 | 0x200 | 0x400)
    if flag & 0x704 or mapq < kw.get("min_mapping_quality", 0):
        return False
    return not ((flag & 1) and not (flag & 2))


def fields_of(recs, contigs, contig, kw):
    """The fields spg_bam_reads_copy returns, computed from the records (BAM order, stepper filter applied)."""
    names = [c for c, _ in contigs]
    tid = names.index(contig)
    out = {k: [] for k, _ in N.BAM_READ_FIELDS}
    for r in recs:
        if r["rname"] != contig or not _keeps(r["flag"], r["mapq"], kw):
            continue
        pos = r["pos"] - 1
        rl = sum(n for op, n in samgen.parse_cigar(r["cigar"]) if op in "MDN=X")
        rn = r["rnext"]
        mtid = tid if rn == "=" else (-1 if rn == "*" else names.index(rn))
        out["pos"].append(pos)
        out["end"].append(pos + rl)
        out["mtid"].append(mtid)
        out["mpos"].append(r["pnext"] - 1)
        out["isize"].append(r["tlen"])
        out["flag"].append(r["flag"])
        out["l_seq"].append(0 if r["seq"] == "*" else len(r["seq"]))
        out["name_hash"].append(fnv1a64(r["qname"].encode()))
    return {k: np.ascontiguousarray(out[k], dtype=dt) for k, dt in N.BAM_READ_FIELDS}


@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("kw", [dict(), dict(max_depth=4), dict(max_depth=0), dict(ignore_overlaps=False, max_depth=3),
                                dict(stepper="samtools", min_mapping_quality=20, max_depth=6), dict(stepper="nofilter")])
def test_plan_fields_equals_host_plan(tmp_path, seed, kw):
    contigs = [("chrA", 700), ("chrB", 700)]
    recs = samgen.random_records(seed, contigs, n_reads=400)
    bam = str(tmp_path / "r.bam")
    samgen.write_bam(bam, contigs, recs, block=5000)
    params = PileupParams(n_threads=2, **kw)
    for contig, _ in contigs:
        with AlignmentFile(bam) as f:
            host = f.pileup_plan(contig, params)
            rp = f.pileup_records(contig, params)
            dp = f.pileup_fields(contig, fields_of(recs, contigs, contig, kw), params)
        assert (dp.pos_begin, dp.n_cols, dp.n_entries) == (host.pos_begin, host.n_cols, host.n_entries)
        v = dp.device_plan()
        if dp.n_cols:
            off = np.ctypeslib.as_array(C_u64(v.offsets), (dp.n_cols + 1,))
            host.fill()
            np.testing.assert_array_equal(off, host.offsets)
            r = rp.records()
            assert v.n_kept == r.n_reads
            assert v.n_pairs == r.n_tweaks
            assert v.max_span == r.max_span
            if v.n_pairs:
                col = np.ctypeslib.as_array(C_i64(v.pair_col), (v.n_pairs,))
                rcol = np.ctypeslib.as_array(C_i64(r.tweak_col), (r.n_tweaks,))
                assert sorted(col.tolist()) == sorted(rcol.tolist())
        for b in (host, rp, dp):
            b.close()


def C_u64(p):
    import ctypes as C
    return C.cast(p, C.POINTER(C.c_uint64))


def C_i64(p):
    import ctypes as C
    return C.cast(p, C.POINTER(C.c_int64))


def test_bam_map_members_and_header(tmp_path):
    import ctypes as C
    contigs = [("chrA", 700), ("chrB", 900)]
    bam = str(tmp_path / "m.bam")
    samgen.write_bam(bam, contigs, samgen.random_records(5, contigs, n_reads=300), block=2000)
    raw = gzip.decompress(open(bam, "rb").read())
    l_text = struct.unpack_from("<i", raw, 4)[0]
    cur = 8 + l_text
    n_ref = struct.unpack_from("<i", raw, cur)[0]
    cur += 4
    for _ in range(n_ref):
        cur += 8 + struct.unpack_from("<i", raw, cur)[0]
    with AlignmentFile(bam) as f:
        m = f.bam_map(3)
        i = m.info
        assert i.n_ref == 2 and i.body == cur and i.inflated_bytes == len(raw)
        assert i.comp_bytes == len(open(bam, "rb").read())
        mem = np.ctypeslib.as_array(C.cast(i.members, C.POINTER(C.c_uint64)), (i.n_members * 3,)).reshape(-1, 3)
        ulen = mem[:, 1] >> 32
        uoff = mem[:, 2]
        assert int(ulen.sum()) == len(raw)
        np.testing.assert_array_equal(uoff[1:], np.cumsum(ulen)[:-1])
        comp = np.ctypeslib.as_array(C.cast(i.comp, C.POINTER(C.c_uint8)), (i.comp_bytes,))
        assert comp.tobytes() == open(bam, "rb").read()
        m.close()


def test_concurrent_plans_on_the_worker_pool(tmp_path):
    """The pileup library's parallel loops run on one pool of persistent workers shared by every host thread
    (process_bams reads the next BAM while it plans this one): four host plans of a 60,000-read BAM made at once from
    four Python threads (ctypes releases the GIL) equal the same plan made alone — CSR offsets, entries, codes, quals."""
    from concurrent.futures import ThreadPoolExecutor
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    bam = str(tmp_path / "s.bam")
    simulate_bam(bam, "NC_045512.2", synth.reference(3000, seed=3), depth=3000, seed=9, n_threads=4)

    def plan(max_depth):
        with AlignmentFile(bam) as f:
            b = f.pileup_plan("NC_045512.2", PileupParams(n_threads=4, max_depth=max_depth)).fill()
            out = (b.pos_begin, b.offsets.copy(), b.codes.copy(), b.quals.copy())
            b.close()
            return out

    for md in (0, 1500):
        want = plan(md)
        assert len(want[2]) > 1_000_000
        with ThreadPoolExecutor(4) as ex:
            got = list(ex.map(plan, [md] * 4))
        for g in got:
            assert g[0] == want[0]
            np.testing.assert_array_equal(g[1], want[1])
            np.testing.assert_array_equal(g[2], want[2])
            np.testing.assert_array_equal(g[3], want[3])
