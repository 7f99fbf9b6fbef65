"""CPU restatement of the third-party pileup step — TEST INFRASTRUCTURE ONLY.

Restates pysam ``AlignmentFile.pileup(...)`` + ``PileupColumn.pileups`` as used by
``LiveVariantCaller.process_bam`` / ``process_pileup_column`` (variant_caller/live_variant_caller.py:
55-60, 75, 89-103).  pysam wraps htslib; neither is vendored in the reference nor installed in this
image (pysam is unpinned in the reference's requirements.txt:1), so this follows their published
behaviour:

* pysam stepper "all" (the default): skip reads with flag & (UNMAP|SECONDARY|QCFAIL|DUP);
  "samtools": flag_filter, MAPQ < min_mapping_quality, paired-but-not-proper; "nofilter".
* htslib ``bam_plp_push``: a read whose start equals the iterator's pending position is dropped
  when the mempool node count (buffered reads + 1 tail node) exceeds maxcnt (pysam max_depth,
  default 8000).  Reads with an empty reference span are not buffered.
* htslib ``bam_plp_next``: columns are produced while the newest read starts beyond the pending
  position (or at EOF); scanning a column frees reads whose end <= column; the pending position
  then jumps to the head read's start or advances by one.  Columns without reads are not emitted.
* ``resolve_cigar2``: M/=/X give (qpos, base); D -> is_del, N -> is_del+is_refskip, both with
  qpos = index of the next query base.
* mate overlaps (pysam ignore_overlaps=True -> htslib tweak_overlap_quality) for proper pairs.
* pysam ``pileup_base_qual_skip``: entry dropped when qual[qpos] (0 if qpos >= l_qseq) < min_bq.

This is written as a direct column-by-column simulation (a Python list as the read buffer) — a
different construction from the product's C++ emulator (post-hoc CSR fill) — so agreement is a
meaningful check.  **Parity unpinned**: no pysam/htslib output exists here to pin it against.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

NT16 = {c: i for i, c in enumerate("=ACMGRSVTWYHKDBN")}
NT16.update({c.lower(): i for c, i in list(NT16.items())})
NT16.update({"U": 8, "u": 8})
OPS = "MIDNSHP=X"
REF_OPS = set("MDN=X")
QRY_OPS = set("MIS=X")


@dataclass
class Read:
    qname: str
    flag: int
    pos: int
    mapq: int
    cigar: List[Tuple[str, int]]
    mtid_same: Optional[bool]       # True: mate on this contig, False: other contig, None: '*'
    mpos: int
    isize: int
    seq: List[int]
    qual: List[int]
    end: int = 0


def parse_sam(path: str) -> Tuple[List[Tuple[str, int]], List[Tuple[str, Read]]]:
    targets, reads = [], []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n").rstrip("\r")
            if not line:
                continue
            if line.startswith("@"):
                if line.startswith("@SQ"):
                    d = dict(x.split(":", 1) for x in line.split("\t")[1:] if ":" in x)
                    targets.append((d["SN"], int(d["LN"])))
                continue
            t = line.split("\t")
            cig = []
            if t[5] != "*":
                num = ""
                for ch in t[5]:
                    if ch.isdigit():
                        num += ch
                    else:
                        cig.append((ch, int(num)))
                        num = ""
            seq = [] if t[9] == "*" else [NT16.get(c, 15) for c in t[9]]
            qual = [255] * len(seq) if t[10] == "*" else [ord(c) - 33 for c in t[10]]
            rn = t[6]
            mts = None if rn == "*" else (True if rn == "=" or rn == t[2] else False)
            r = Read(t[0], int(t[1]), int(t[3]) - 1, int(t[4]), cig, mts, int(t[7]) - 1, int(t[8]), seq, qual)
            r.end = r.pos + sum(n for op, n in cig if op in REF_OPS)
            reads.append((t[2], r))
    return targets, reads


def _stepper_keeps(r: Read, stepper: str, min_mapq: int, flag_filter: int) -> bool:
    if r.flag & 0x4:
        return False
    if stepper == "nofilter":
        return True
    if stepper == "all":
        return not (r.flag & 0x704)
    if r.flag & flag_filter:
        return False
    if r.mapq < min_mapq:
        return False
    if (r.flag & 0x1) and not (r.flag & 0x2):
        return False
    return True


def _aligned(r: Read) -> List[Tuple[int, int]]:
    out, x, y = [], r.pos, 0
    for op, n in r.cigar:
        if op in "M=X":
            out.extend((x + k, y + k) for k in range(n))
        if op in REF_OPS:
            x += n
        if op in QRY_OPS:
            y += n
    return out


def _tweak(a: Read, b: Read) -> None:
    pb = dict(_aligned(b))
    for x, ia in _aligned(a):
        if x not in pb:
            continue
        ib = pb[x]
        if ia >= len(a.seq) or ib >= len(b.seq):
            return
        if a.seq[ia] == b.seq[ib]:
            a.qual[ia] = min(a.qual[ia] + b.qual[ib], 200)
            b.qual[ib] = 0
        elif a.qual[ia] >= b.qual[ib]:
            a.qual[ia] = int(0.8 * a.qual[ia])
            b.qual[ib] = 0
        else:
            b.qual[ib] = int(0.8 * b.qual[ib])
            a.qual[ia] = 0


def _resolve(r: Read, col: int) -> Tuple[int, int]:
    """(code, qual used by the bq filter) of read r at column col (resolve_cigar2)."""
    x, y = r.pos, 0
    for op, n in r.cigar:
        if op in REF_OPS:
            if x <= col < x + n:
                if op == "D" or op == "N":
                    return (16 if op == "D" else 17), (r.qual[y] if y < len(r.qual) else 0)
                qp = y + (col - x)
                return (r.seq[qp] if qp < len(r.seq) else 15), (r.qual[qp] if qp < len(r.qual) else 0)
            x += n
        if op in QRY_OPS:
            y += n
    raise AssertionError("column outside read")


def pileup_columns(path: str, contig: str, stepper: str = "all", min_mapping_quality: int = 0,
                   max_depth: int = 8000, ignore_overlaps: bool = True, flag_filter: int = 0x704):
    """Yield (pos, [(code, qual), ...]) per emitted column, before the base-quality filter."""
    targets, reads = parse_sam(path)
    names = [t[0] for t in targets]
    tid = names.index(contig)
    rs = [r for c, r in reads if c == contig and _stepper_keeps(r, stepper, min_mapping_quality, flag_filter)]
    maxcnt = max_depth if max_depth > 0 else float("inf")
    buf: List[Read] = []                 # the iterator's linked list (tail node not stored)
    olap: Dict[str, Read] = {}
    it_pos, started = 0, tid == 0
    max_pos = -1
    out = []

    def olap_remove(r):
        if ignore_overlaps and r.qname in olap:
            del olap[r.qname]

    def plp_next(eof):
        nonlocal it_pos
        while buf and (eof or max_pos > it_pos):
            col = []
            keep = []
            for r in buf:
                if r.end <= it_pos:
                    olap_remove(r)
                    continue
                keep.append(r)
                if r.pos <= it_pos:
                    col.append(_resolve(r, it_pos))
            buf[:] = keep
            if col:
                out.append((it_pos, col))
            if buf:
                if it_pos < buf[0].pos:
                    it_pos = buf[0].pos
                else:
                    it_pos += 1

    for r in rs:
        if started and it_pos == r.pos and len(buf) + 1 > maxcnt:
            olap_remove(r)
            continue
        max_pos = r.pos
        if r.end > it_pos or not started:
            buf.append(r)
            if ignore_overlaps and (r.flag & 0x2) and not (r.flag & 0x8) and r.mtid_same is not False \
                    and not (abs(r.isize) >= 2 * len(r.seq) and r.mpos >= r.end):
                if r.qname not in olap:
                    if r.mpos >= r.pos or ((r.flag & 0x1) and r.mpos == -1):
                        olap[r.qname] = r
                else:
                    _tweak(olap.pop(r.qname), r)
        if not started:
            started = True
            it_pos = buf[0].pos if buf else it_pos
        plp_next(False)
    plp_next(True)
    return out


def to_csr(columns):
    """Columns -> (pos_begin, offsets u64, codes u8, quals u8) over [first, last] column."""
    import numpy as np
    if not columns:
        return 0, np.zeros(1, np.uint64), np.zeros(0, np.uint8), np.zeros(0, np.uint8)
    lo, hi = columns[0][0], columns[-1][0] + 1
    cnt = np.zeros(hi - lo, np.int64)
    for p, col in columns:
        cnt[p - lo] = len(col)
    off = np.zeros(hi - lo + 1, np.uint64)
    np.cumsum(cnt, out=off[1:])
    codes = np.array([c for _, col in columns for c, _ in col], np.uint8)
    quals = np.array([q for _, col in columns for _, q in col], np.uint8)
    return lo, off, codes, quals
