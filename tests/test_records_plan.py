"""Records plans (spp_pileup_plan_records): the host half of the device-side pileup.

The plan keeps the inflated BAM bytes and a per-read index (record offset, reference span, overlap-tweak
entry) instead of decoded bases; spg_accumulate_records' kernel (csrc/spg_fill.hip) writes the CSR from
them.  Here (CPU) the index is checked by restating that kernel's walk in Python — per read in BAM order,
its CIGAR's reference ops over the batch's columns, D / N taking the next query base's quality (the
pre-tweak quality in columns before the tweak column) — and comparing with spp_batch_fill of an ordinary
plan of the same BAM (tests/test_pileup.py pins that against oracle/pileup_port.py).  The GPU kernel is
compared with the same host fill in tests/test_device_pileup_gpu.py."""
import ctypes as C

import numpy as np
import pytest

import spings  # noqa: F401
from covid_spings_variant_caller_amd import build as B
from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams
import samgen

REF_OPS, QUERY_OPS = (0, 2, 3, 7, 8), (0, 1, 4, 7, 8)


@pytest.fixture(scope="module", autouse=True)
def _lib():
    B.build_pileup()


def _arr(p, n, t):
    if n == 0:
        return np.zeros(0, t)
    return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(t))), (n,)).copy()


def fill_from_records(r):
    """Python restatement of k_fill over one spg_records view -> (pos_begin, offsets, codes, quals)."""
    nc, E, n = r.n_cols, r.n_entries, r.n_reads
    off = _arr(r.offsets, nc + 1, np.uint64)
    data = _arr(r.data, r.data_bytes, np.uint8).tobytes()
    rec, rpos, rend = _arr(r.rec, n, np.uint64), _arr(r.rpos, n, np.int32), _arr(r.rend, n, np.int32)
    tw = _arr(r.tweak, n, np.int32)
    tcol, tq = _arr(r.tweak_col, r.n_tweaks, np.int64), _arr(r.tweak_qual, r.n_tweaks, np.uint64)
    orig = _arr(r.orig_qual, r.orig_bytes, np.uint8)
    codes, quals = np.zeros(E, np.uint8), np.zeros(E, np.uint8)
    cur = off[:-1].astype(np.int64).copy()
    lo, hi = r.pos_begin, r.pos_begin + nc
    assert np.all(np.diff(rpos) >= 0), "reads in BAM (coordinate) order"
    for i in range(n):
        ro = int(rec[i])
        l_name = data[ro + 8]
        ncig = int.from_bytes(data[ro + 12:ro + 14], "little")
        ls = int.from_bytes(data[ro + 16:ro + 20], "little", signed=True)
        co = ro + 32 + l_name
        so = co + 4 * ncig
        qo = so + (ls + 1) // 2
        x, y = int(rpos[i]), 0
        t = int(tw[i])
        tc = int(tcol[t]) if t >= 0 else -(1 << 62)     # columns < tc: pre-tweak qualities (none if untweaked)
        for k in range(ncig):
            w = int.from_bytes(data[co + 4 * k:co + 4 * k + 4], "little")
            op, ln = w & 15, w >> 4
            if op in REF_OPS:
                for col in range(max(x, lo), min(x + ln, hi)):
                    j = cur[col - lo]
                    if op in (2, 3):
                        codes[j] = 16 if op == 2 else 17
                        quals[j] = (orig[int(tq[t]) + y] if col < tc else data[qo + y]) if y < ls else 0
                    else:
                        qp = y + col - x
                        if qp < ls:
                            b = data[so + qp // 2]
                            codes[j] = (b & 15) if qp & 1 else (b >> 4)
                            quals[j] = data[qo + qp]
                        else:
                            codes[j], quals[j] = 15, 0
                    cur[col - lo] += 1
                x += ln
            if op in QUERY_OPS:
                y += ln
        assert x == rend[i]
    np.testing.assert_array_equal(cur, off[1:].astype(np.int64))
    return r.pos_begin, off, codes, quals


def host_fill(path, contig, start=None, stop=None, **kw):
    with AlignmentFile(path) as f:
        b = f.pileup_plan(contig, PileupParams(n_threads=kw.pop("n_threads", 3), **kw), start, stop)
        b.fill()
        out = (b.pos_begin, b.offsets.copy(), b.codes.copy(), b.quals.copy())
        b.close()
    return out


def records_fill(path, contig, start=None, stop=None, **kw):
    with AlignmentFile(path) as f:
        b = f.pileup_records(contig, PileupParams(n_threads=kw.pop("n_threads", 3), **kw), start, stop)
        r = b.records()
        assert (r.pos_begin, r.n_cols, r.n_entries) == (b.pos_begin, b.n_cols, b.n_entries)
        out = fill_from_records(r)
        b.close()
    return out


def assert_same(a, b):
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_array_equal(a[3], b[3])


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("kw", [dict(), dict(max_depth=4), dict(max_depth=0), dict(ignore_overlaps=False, max_depth=3),
                                dict(stepper="samtools", min_mapping_quality=20, max_depth=6), dict(stepper="nofilter")])
def test_records_index_matches_host_fill(tmp_path, seed, kw):
    """Random reads with every CIGAR op, '*' SEQ/QUAL, stacks and overlapping proper pairs (tweaks)."""
    contigs = [("chrA", 700), ("chrB", 700)]
    recs = samgen.random_records(seed, contigs, n_reads=400)
    bam = str(tmp_path / "r.bam")
    samgen.write_bam(bam, contigs, recs, block=5000)           # records straddle BGZF members
    for c, _ in contigs:
        assert_same(records_fill(bam, c, **kw), host_fill(bam, c, **kw))


@pytest.mark.parametrize("region", [(100, 300), (0, 50), (550, 700), (250, 251)])
def test_records_region(tmp_path, region):
    contigs = [("chrA", 700)]
    recs = samgen.random_records(7, contigs, n_reads=500)
    bam = str(tmp_path / "r.bam")
    samgen.write_bam(bam, contigs, recs, block=9000)
    assert_same(records_fill(bam, "chrA", *region), host_fill(bam, "chrA", *region))


def test_records_overlap_tweak_indexed(tmp_path):
    """A proper pair overlapping by 5 bases: the first mate gets a tweak entry (its D/N entries before the
    tweak column read the original qualities) and the records hold the tweaked qualities."""
    def rec(qname, pos1, cigar, seq, qual, flag, pnext, tlen):
        return dict(qname=qname, flag=flag, rname="c", pos=pos1, mapq=60, cigar=cigar, rnext="=", pnext=pnext,
                    tlen=tlen, seq=seq, qual="".join(chr(33 + q) for q in qual))
    recs = [rec("p", 1, "4M2D6M", "A" * 10, [30] * 10, 99, 6, 15),
            rec("p", 6, "10M", "A" * 10, [25] * 10, 147, 1, -15)]
    bam = str(tmp_path / "t.bam")
    samgen.write_bam(bam, [("c", 60)], recs)
    with AlignmentFile(bam) as f:
        b = f.pileup_records("c", PileupParams(n_threads=2))
        r = b.records()
        assert r.n_reads == 2 and r.n_tweaks == 1 and r.orig_bytes == 10
        got = fill_from_records(r)
        b.close()
    assert_same(got, host_fill(bam, "c"))


def test_records_many_members_and_threads(tmp_path):
    """The simulator's BAM (many BGZF members, deletions and insertions) at several thread counts."""
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    bam = str(tmp_path / "s.bam")
    simulate_bam(bam, "NC_045512.2", synth.reference(3000, seed=1), depth=40, seed=3, n_threads=4)
    exp = host_fill(bam, "NC_045512.2", max_depth=30)
    for t in (1, 2, 5):
        assert_same(records_fill(bam, "NC_045512.2", max_depth=30, n_threads=t), exp)


def test_records_need_bam(tmp_path):
    sam = str(tmp_path / "a.sam")
    samgen.write_sam(sam, [("c", 60)], [dict(qname="a", flag=0, rname="c", pos=1, mapq=60, cigar="4M", rnext="*",
                                             pnext=0, tlen=0, seq="ACGT", qual="IIII")])
    with AlignmentFile(sam) as f:
        with pytest.raises(RuntimeError, match="needs a BAM"):
            f.pileup_records("c")


def test_records_truncated_bam_raises(tmp_path):
    contigs = [("chrA", 700)]
    bam = str(tmp_path / "r.bam")
    samgen.write_bam(bam, contigs, samgen.random_records(3, contigs, n_reads=200), block=4000)
    raw = open(bam, "rb").read()
    cut = str(tmp_path / "cut.bam")
    with open(cut, "wb") as f:
        f.write(raw[:len(raw) // 2])
    with AlignmentFile(cut) as f:
        with pytest.raises(RuntimeError, match="truncated"):
            f.pileup_records("chrA")


def test_records_fill_refused(tmp_path):
    """spp_batch_fill is not available on a records plan (its entries are written on the GPU)."""
    contigs = [("chrA", 700)]
    bam = str(tmp_path / "r.bam")
    samgen.write_bam(bam, contigs, samgen.random_records(4, contigs, n_reads=50))
    with AlignmentFile(bam) as f:
        b = f.pileup_records("chrA")
        with pytest.raises(RuntimeError, match="filled on the GPU"):
            b.fill()
        b.close()


_SCAN_CHILD = r"""
import sys, hashlib, numpy as np
sys.path.insert(0, sys.argv[1])
import spings
from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams
from test_records_plan import _arr
with AlignmentFile(sys.argv[2]) as f:
    b = f.pileup_records(sys.argv[3], PileupParams(n_threads=8, max_depth=int(sys.argv[4])))
r = b.records()
h = hashlib.sha256()
for a in (_arr(r.offsets, r.n_cols + 1, np.uint64), _arr(r.rec, r.n_reads, np.uint64), _arr(r.rpos, r.n_reads, np.int32),
          _arr(r.rend, r.n_reads, np.int32), _arr(r.tweak, r.n_reads, np.int32)):
    h.update(a.tobytes())
print(r.pos_begin, r.n_cols, r.n_entries, r.n_reads, h.hexdigest())
"""


@pytest.mark.parametrize("max_depth", [8000, 0])
def test_parallel_record_scan_equals_serial(tmp_path, max_depth):
    """The records plan's record boundaries found in parallel (validated chains per range that must meet exactly,
    csrc/spp_pileup.cpp read_bam_raw; each thread steps several ranges' chains in turn) give the plan the serial
    block_size walk gives (SPP_PAR_SCAN=0): a BAM of ~80 MB inflated (2,000x over 30 kb, 150-bp reads with D/I), 8 threads."""
    import os
    import subprocess
    import sys
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    bam = str(tmp_path / "p.bam")
    simulate_bam(bam, "NC_045512.2", synth.reference(29903, seed=1), depth=2000, seed=9, n_threads=8)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    here = os.path.dirname(os.path.abspath(__file__))
    out = {}
    # ("1:c": the parallel scan with c chains stepped in turn per thread — 8 by default, so 64 ranges here)
    for par in ("1", "1:3", "0"):
        env = dict(os.environ, SPP_PAR_SCAN=par[0], SPP_SCAN_CHAINS=par[2:] or "8", PYTHONPATH=here)
        r = subprocess.run([sys.executable, "-c", _SCAN_CHILD, root, bam, "NC_045512.2", str(max_depth)], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        out[par] = r.stdout.strip().splitlines()[-1]
    assert out["1"] == out["0"] == out["1:3"]
    assert int(out["1"].split()[3]) > 300_000


def test_host_inflater_reported():
    """spp_host_inflater names the host BGZF inflater this process uses (bench.py records it)."""
    import os
    from covid_spings_variant_caller_amd import _native as N
    name = N.pileup_lib().spp_host_inflater().decode()
    assert name in ("libdeflate", "zlib")
    if os.environ.get("SPP_NO_LIBDEFLATE"):
        assert name == "zlib"


def test_records_plans_on_zlib(tmp_path):
    """The zlib host inflater (SPP_NO_LIBDEFLATE=1; libdeflate is present in this image, so it is otherwise never run):
    this file's plan tests once more in a process where the pileup library binds zlib."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, SPP_NO_LIBDEFLATE="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        os.path.join(here, "test_records_plan.py"), "-k", "not test_records_plans_on_zlib"],
                       env=env, cwd=os.path.dirname(here), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout
