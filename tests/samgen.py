"""Test helpers: synthetic SAM records and a small BAM (BGZF) writer, so the pileup front end can
be exercised on both formats with identical reads."""
from __future__ import annotations

import random
import struct
import zlib

OPS = "MIDNSHP=X"
NT16 = "=ACMGRSVTWYHKDBN"


def reg2bin(beg, end):
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


def parse_cigar(c):
    if c == "*":
        return []
    out, num = [], ""
    for ch in c:
        if ch.isdigit():
            num += ch
        else:
            out.append((ch, int(num)))
            num = ""
    return out


def write_sam(path, targets, records):
    """records: dicts with qname flag rname pos(1-based) mapq cigar rnext pnext tlen seq qual."""
    with open(path, "w") as f:
        f.write("@HD\tVN:1.6\tSO:coordinate\n")
        for n, l in targets:
            f.write(f"@SQ\tSN:{n}\tLN:{l}\n")
        for r in records:
            f.write("\t".join(str(r[k]) for k in ("qname", "flag", "rname", "pos", "mapq", "cigar", "rnext",
                                                  "pnext", "tlen", "seq", "qual")) + "\n")


def _bgzf_block(data: bytes) -> bytes:
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    comp = c.compress(data) + c.flush()
    bsize = len(comp) + 25
    hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
    return hdr + comp + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


def write_bam(path, targets, records, block=60000):
    tid = {n: i for i, (n, _) in enumerate(targets)}
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join(f"@SQ\tSN:{n}\tLN:{l}\n" for n, l in targets)
    raw = bytearray(b"BAM\1" + struct.pack("<i", len(text)) + text.encode() + struct.pack("<i", len(targets)))
    for n, l in targets:
        nb = n.encode() + b"\0"
        raw += struct.pack("<i", len(nb)) + nb + struct.pack("<i", l)
    for r in records:
        cig = parse_cigar(r["cigar"])
        seq = "" if r["seq"] == "*" else r["seq"]
        qual = bytes([255] * len(seq)) if r["qual"] == "*" else bytes(ord(c) - 33 for c in r["qual"])
        pos = int(r["pos"]) - 1
        rlen = sum(n for op, n in cig if op in "MDN=X")
        name = r["qname"].encode() + b"\0"
        rn = r["rnext"]
        mt = -1 if rn == "*" else (tid[r["rname"]] if rn == "=" else tid[rn])
        packed = bytearray((len(seq) + 1) // 2)
        for i, ch in enumerate(seq):
            code = NT16.index(ch.upper()) if ch.upper() in NT16 else 15
            packed[i >> 1] |= code << (4 if i % 2 == 0 else 0)
        body = struct.pack("<iiBBHHHiiii", tid[r["rname"]], pos, len(name), int(r["mapq"]),
                           reg2bin(max(pos, 0), max(pos, 0) + max(rlen, 1)), len(cig), int(r["flag"]), len(seq),
                           mt, int(r["pnext"]) - 1, int(r["tlen"]))
        body += name + b"".join(struct.pack("<I", n << 4 | OPS.index(op)) for op, n in cig) + bytes(packed) + qual
        raw += struct.pack("<i", len(body)) + body
    with open(path, "wb") as f:
        for i in range(0, len(raw), block):
            f.write(_bgzf_block(bytes(raw[i:i + block])))
        f.write(_bgzf_block(b""))


def random_records(seed, contigs, n_reads=300, L=600, read_len=60, pair_frac=0.3, stack_every=7):
    """Coordinate-sorted reads with every CIGAR op, assorted flags, MAPQ, '*' SEQ/QUAL, stacks of
    reads sharing a start (depth-cap stress) and overlapping proper pairs."""
    rng = random.Random(seed)
    recs = []
    for ci, (cname, clen) in enumerate(contigs):
        starts = sorted(rng.randrange(0, max(1, min(L, clen) - read_len)) for _ in range(n_reads))
        starts = [s - (s % stack_every) if rng.random() < 0.4 else s for s in starts]
        starts.sort()
        pairs = {}
        for i, s in enumerate(starts):
            ops = []
            left = read_len
            if rng.random() < 0.2:
                k = rng.randrange(1, 6)
                ops.append(("H" if rng.random() < 0.3 else "S", k))
                left -= k if ops[-1][0] == "S" else 0
            while left > 0:
                k = min(left, rng.randrange(5, 30))
                ops.append((rng.choice("MMMM=X"), k))
                left -= k
                r = rng.random()
                if left > 0 and r < 0.15:
                    ops.append(("D", rng.randrange(1, 4)))
                elif left > 0 and r < 0.2:
                    ops.append(("N", rng.randrange(2, 20)))
                elif left > 2 and r < 0.3:
                    k = rng.randrange(1, 3)
                    ops.append(("I", k))
                    left -= k
                elif left > 0 and r < 0.32:
                    ops.append(("P", 1))
            if rng.random() < 0.1:
                ops.append(("S", 3))
            cigar = "".join(f"{n}{op}" for op, n in ops)
            qlen = sum(n for op, n in ops if op in "MIS=X")
            seq = "".join(rng.choice("ACGTACGTACGTNRY") for _ in range(qlen))
            qual = "".join(chr(33 + rng.choice([0, 2, 10, 20, 25, 30, 30, 33, 37, 40, 41, 60])) for _ in range(qlen))
            flag = 0
            r = rng.random()
            if r < 0.03:
                flag |= 0x4
            elif r < 0.06:
                flag |= 0x100
            elif r < 0.08:
                flag |= 0x200
            elif r < 0.10:
                flag |= 0x400
            elif r < 0.12:
                flag |= 0x800
            if rng.random() < 0.05:
                seq, qual = "*", "*"
            elif rng.random() < 0.05:
                qual = "*"
            mapq = rng.choice([0, 5, 20, 30, 60, 60, 60])
            qname = f"r{ci}_{i}"
            rnext, pnext, tlen = "*", 0, 0
            if rng.random() < pair_frac:
                flag |= 0x1 | (0x2 if rng.random() < 0.8 else 0)
                rnext, pnext, tlen = "=", s + 1 + rng.randrange(0, 40), read_len + 20
                pairs[qname] = pnext
            recs.append(dict(qname=qname, flag=flag, rname=cname, pos=s + 1, mapq=mapq, cigar=cigar, rnext=rnext,
                             pnext=pnext, tlen=tlen, seq=seq, qual=qual))
        # mates: same qname, start at pnext, pointing back
        for qname, p in pairs.items():
            mate_of = next(r for r in recs if r["qname"] == qname)
            qlen = 50
            recs.append(dict(qname=qname, flag=(mate_of["flag"] & 0x3) | 0x80, rname=cname, pos=p, mapq=60,
                             cigar=f"{qlen}M", rnext="=", pnext=mate_of["pos"], tlen=-mate_of["tlen"],
                             seq="".join(rng.choice("ACGT") for _ in range(qlen)),
                             qual="".join(chr(33 + rng.choice([20, 30, 35, 40])) for _ in range(qlen))))
        recs_c = [r for r in recs if r["rname"] == cname]
        recs = [r for r in recs if r["rname"] != cname] + sorted(recs_c, key=lambda r: r["pos"])
    return recs


def snv_records(contig, ref, n_reads, read_len=60, snvs=None, seed=0, del_frac=0.05, qual_choices=None):
    """Single-end reads sampled from `ref` with planted SNVs {pos: (alt, af)} (0-based), random
    errors, a few 2-base deletions; coordinate-sorted SAM records."""
    rng = random.Random(seed)
    snvs = snvs or {}
    qual_choices = qual_choices or [12, 20, 28, 30, 32, 35, 37, 38, 40, 41]
    L = len(ref)
    starts = sorted(rng.randrange(0, L - read_len) for _ in range(n_reads))
    recs = []
    for i, s in enumerate(starts):
        if rng.random() < del_frac:
            k = rng.randrange(10, read_len - 12)
            cig = [("M", k), ("D", 2), ("M", read_len - k)]
        else:
            cig = [("M", read_len)]
        seq, x = [], s
        for op, n in cig:
            if op == "M":
                for j in range(n):
                    b = ref[x + j].upper()
                    if (x + j) in snvs and rng.random() < snvs[x + j][1]:
                        b = snvs[x + j][0]
                    if rng.random() < 0.01:
                        b = rng.choice("ACGTN")
                    seq.append(b)
            x += n
        qual = "".join(chr(33 + rng.choice(qual_choices)) for _ in seq)
        recs.append(dict(qname=f"q{i}", flag=0, rname=contig, pos=s + 1, mapq=60,
                         cigar="".join(f"{n}{op}" for op, n in cig), rnext="*", pnext=0, tlen=0,
                         seq="".join(seq), qual=qual))
    return recs


def write_fasta(path, seqs, width=60):
    with open(path, "w") as f:
        for name, s in seqs:
            f.write(f">{name} synthetic\n")
            for i in range(0, len(s), width):
                f.write(s[i:i + width] + "\n")


def read_bam_as_sam(bam_path, sam_path):
    """BAM -> SAM text (test helper: lets the SAM-only Python oracle read simulator output)."""
    import gzip
    data = gzip.open(bam_path, "rb").read()
    assert data[:4] == b"BAM\1"
    l_text = struct.unpack_from("<i", data, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", data, p)[0]
    p += 4
    targets = []
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", data, p)[0]
        name = data[p + 4:p + 4 + ln - 1].decode()
        targets.append((name, struct.unpack_from("<i", data, p + 4 + ln)[0]))
        p += 8 + ln
    recs = []
    while p < len(data):
        bs = struct.unpack_from("<i", data, p)[0]
        b = data[p + 4:p + 4 + bs]
        p += 4 + bs
        tid, pos, l_name, mapq, _bin, n_cig, flag, l_seq, mt, mp, tlen = struct.unpack_from("<iiBBHHHiiii", b, 0)
        name = b[32:32 + l_name - 1].decode()
        o = 32 + l_name
        cig = "".join(f"{c >> 4}{OPS[c & 15]}" for c in struct.unpack_from(f"<{n_cig}I", b, o)) or "*"
        o += 4 * n_cig
        seq = "".join(NT16[(b[o + i // 2] >> (4 if i % 2 == 0 else 0)) & 15] for i in range(l_seq))
        o += (l_seq + 1) // 2
        qual = "".join(chr(33 + min(q, 93)) for q in b[o:o + l_seq])
        recs.append(dict(qname=name, flag=flag, rname=targets[tid][0], pos=pos + 1, mapq=mapq, cigar=cig,
                         rnext="*" if mt < 0 else ("=" if mt == tid else targets[mt][0]), pnext=mp + 1, tlen=tlen,
                         seq=seq or "*", qual=qual or "*"))
    write_sam(sam_path, targets, recs)
    return targets, recs
