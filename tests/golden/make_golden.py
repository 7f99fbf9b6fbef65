"""Generate golden vectors by running the REFERENCE's own code (this container only).

Test infrastructure — not shipped, never run on the GPU box.  It imports
``variant_caller.live_variant_caller`` / ``variant_caller.utils`` from
``/root/reference`` (read-only) with an I/O-only ``pysam`` stub in
``sys.modules`` (pysam/htslib is not installed here), feeds
seeded synthetic pileup columns to the reference's own
``LiveVariantCaller.process_pileup_column`` (live_variant_caller.py:74-103) and
``prepare_variants`` (:120-231), and records:

* ``memory``   — per position in dict-insertion order: REF char, totalDepth and
                 the per-allele list lengths in dict order (structs.py:2-6);
* ``gl``       — the reference's ``genotype_likelihood`` (utils.py:16-24) for every
                 allele of every position with totalDepth >= minTotalDepth, computed
                 exactly the way prepare_variants builds it (:132-143), as float.hex;
* ``variants`` — the list ``prepare_variants()`` returns (floats as float.hex);
* ``eps_lut``  — ``from_phred_scale(q)`` for q in 0..255 (utils.py:9-10);
* ``to_phred`` — ``to_phred_scale`` on a grid including half-way ties (utils.py:12-13).

The only behaviour the stub adds is pysam's access-time base-quality filter of
``PileupColumn.pileups`` (pysam ``pileup_base_qual_skip``: drop an entry when
``qual[qpos] < min_base_quality``; D/N entries are tested with the quality of
the next aligned query base, which is what the ``quals`` array carries for them).
That filter is third-party behaviour, restated — see oracle/README.md.

Input column format (the build's CSR boundary): per batch
``pos_begin``, ``offsets[n_cols+1]``, ``codes[E]`` (BAM 4-bit nibble 0..15,
16 = CIGAR D, 17 = CIGAR N) and ``quals[E]``.

Run:  python tests/golden/make_golden.py   (writes tests/golden/cases.json)
"""
from __future__ import annotations

import io
import json
import math
import os
import sys
import types
import contextlib

import numpy as np

REF_ROOT = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
NIBBLE = "=ACMGRSVTWYHKDBN"
DEL, SKIP = 16, 17

# ----------------------------------------------------------------------------------
# I/O-only pysam stub
# ----------------------------------------------------------------------------------
_FASTAS: dict[str, tuple[str, str]] = {}


class _FastaFile:
    def __init__(self, path):
        self.contig, self.seq = _FASTAS[path]
        self.references = (self.contig,)

    def fetch(self, reference=None, start=None, end=None):
        return self.seq

    def get_reference_length(self, ref):
        return len(self.seq)

    def close(self):
        pass


def _install_stub():
    m = types.ModuleType("pysam")
    m.FastaFile = _FastaFile
    m.AlignedSegment = object
    m.AlignmentFile = None
    sys.modules["pysam"] = m
    sys.path.insert(0, REF_ROOT)
    sys.dont_write_bytecode = True
    from variant_caller import live_variant_caller as lvc_mod  # noqa: E402
    from variant_caller import utils as ref_utils  # noqa: E402
    return lvc_mod, ref_utils


class _Aln:
    __slots__ = ("query_sequence", "query_qualities")

    def __init__(self, s, q):
        self.query_sequence = s
        self.query_qualities = q


class _Read:
    __slots__ = ("alignment", "query_position", "is_del", "is_refskip")

    def __init__(self, code, q):
        ch = NIBBLE[code] if code < 16 else "N"
        self.alignment = _Aln(ch, [q])
        self.query_position = 0
        # htslib resolve_cigar2 sets is_del=1 for BOTH D and N; is_refskip only for N.
        self.is_del = code in (DEL, SKIP)
        self.is_refskip = code == SKIP


class _Column:
    def __init__(self, contig, pos, entries, min_bq):
        self.reference_name = contig
        self.reference_pos = pos
        self._entries = entries
        self._min_bq = min_bq

    @property
    def pileups(self):
        # pysam pileup_base_qual_skip: entries whose quality < min_base_quality are dropped
        return [_Read(c, q) for (c, q) in self._entries if not (self._min_bq > 0 and q < self._min_bq)]


# ----------------------------------------------------------------------------------
# case construction
# ----------------------------------------------------------------------------------
def _hex(x):
    return float(x).hex() if isinstance(x, (float, np.floating)) else x


def _batch_from_columns(pos_begin, cols):
    offs = [0]
    codes, quals = [], []
    for ent in cols:
        for c, q in ent:
            codes.append(int(c))
            quals.append(int(q))
        offs.append(len(codes))
    return {"pos_begin": int(pos_begin), "offsets": offs, "codes": codes, "quals": quals}


def _columns_of(batch):
    o = batch["offsets"]
    out = []
    for i in range(len(o) - 1):
        out.append(list(zip(batch["codes"][o[i]:o[i + 1]], batch["quals"][o[i]:o[i + 1]])))
    return out


def run_reference(lvc_mod, ref_utils, case):
    p = case["params"]
    path = f"/stub/{case['name']}.fa"
    _FASTAS[path] = (case["contig"], case["reference"])
    lvc = lvc_mod.LiveVariantCaller(path, p["minBaseQuality"], p["minMappingQuality"], p["minTotalDepth"],
                                    p["minAlleleDepth"], p["minEvidenceRatio"], p["maxVariants"])
    sink = io.StringIO()
    with contextlib.redirect_stderr(sink):
        for b in case["batches"]:
            for i, ent in enumerate(_columns_of(b)):
                if not ent:
                    continue  # htslib never emits a column with no reads
                lvc.process_pileup_column(_Column(case["contig"], b["pos_begin"] + i, ent, p["minBaseQuality"]))
        variants = lvc.prepare_variants()
    memory = []
    gl = []
    for pos, site in lvc.memory.items():
        memory.append([int(pos), site["reference"], int(site["totalDepth"]),
                       [[a, len(v)] for a, v in site["snvs"].items()]])
        if site["totalDepth"] >= p["minTotalDepth"]:
            snvs = {a: [ref_utils.from_phred_scale(q) for q in site["snvs"][a]] for a in site["snvs"]}
            gl.append([int(pos), [[a, float(ref_utils.genotype_likelihood(a, snvs)).hex()] for a in snvs]])
    var_out = []
    for v in variants:
        var_out.append({
            "start": int(v["start"]), "stop": int(v["stop"]), "alleles": list(v["alleles"]),
            "qual": _hex(v["qual"]),
            "info": {k: _hex(x) if not isinstance(x, (int, np.integer)) else int(x) for k, x in v["info"].items()},
        })
    return {"memory": memory, "gl": gl, "variants": var_out}


def _ref_seq(rng, L, lower_frac=0.0):
    s = rng.choice(list("ACGT"), size=L)
    if lower_frac:
        m = rng.random(L) < lower_frac
        s = np.where(m, np.char.lower(s), s)
    return "".join(s.tolist())


CODE = {"A": 1, "C": 2, "G": 4, "T": 8, "N": 15}


def _q_normal(rng, n, mu=33, sd=6, lo=2, hi=41):
    return np.clip(np.rint(rng.normal(mu, sd, size=n)), lo, hi).astype(int)


def case_planted(rng, name, L=240, depth=(12, 400), af_cycle=(1.0, 0.5, 0.2, 0.05), every=7, params=None,
                 lower_frac=0.0, del_frac=0.01, n_frac=1e-3):
    ref = _ref_seq(rng, L, lower_frac)
    cols = []
    for i in range(L):
        d = int(rng.integers(depth[0], depth[1] + 1))
        rb = ref[i].upper()
        af = af_cycle[(i // every) % len(af_cycle)] if i % every == every // 2 else 0.0
        alt = "ACGT"[("ACGT".index(rb) + 1 + (i % 3)) % 4]
        q = _q_normal(rng, d)
        ent = []
        for k in range(d):
            u = rng.random()
            if u < del_frac:
                ent.append((DEL if rng.random() < 0.8 else SKIP, int(q[k])))
                continue
            b = alt if rng.random() < af else rb
            eps = 10 ** (-q[k] / 10)
            if rng.random() < eps:
                b = "ACGT"[("ACGT".index(b) + 1 + int(rng.integers(0, 3))) % 4]
            if rng.random() < n_frac:
                b = "N"
            ent.append((CODE[b], int(q[k])))
        cols.append(ent)
    return {"name": name, "params": params or DEFAULT_PARAMS, "contig": "NC_045512.2", "reference": ref,
            "batches": [_batch_from_columns(0, cols)]}


DEFAULT_PARAMS = {"minBaseQuality": 30, "minMappingQuality": 20, "minTotalDepth": 10, "minAlleleDepth": 5,
                  "minEvidenceRatio": 0.10, "maxVariants": 1}


def case_band(rng):
    """Columns whose GL chains land in / around the fp64 subnormal band."""
    L = 60
    ref = _ref_seq(rng, L + 1000)[1000:]
    cols = []
    for i in range(L):
        rb = ref[i]
        alt = "ACGT"[("ACGT".index(rb) + 1) % 4]
        alt2 = "ACGT"[("ACGT".index(rb) + 2) % 4]
        n_ref = 20 + (i % 5) * 7
        # sum of alt quals sweeps 2950 .. 3300 (log10 P_alt from -295 to -330): straddles the band
        target = 2950 + i * 6
        ent = [(CODE[rb], int(q)) for q in rng.integers(30, 42, size=n_ref)]
        s = 0
        alts = []
        while s < target:
            q = int(min(41, max(30, target - s))) if target - s < 30 else int(rng.integers(30, 42))
            if target - s < 30:
                q = 30
            alts.append(q)
            s += q
        if i % 4 == 1:   # split the alt mass over two alleles -> chain product crosses the band
            half = len(alts) // 2
            ent += [(CODE[alt], q) for q in alts[:half]] + [(CODE[alt2], q) for q in alts[half:]]
        else:
            ent += [(CODE[alt], q) for q in alts]
        order = rng.permutation(len(ent))
        cols.append([ent[j] for j in order])
    return {"name": "band", "params": dict(DEFAULT_PARAMS, minEvidenceRatio=0.05), "contig": "NC_045512.2",
            "reference": _ref_seq(rng, 1000) + ref, "batches": [_batch_from_columns(1000, cols)]}


def case_deep(rng):
    """8000x columns: every GL underflows to exactly 0."""
    c = case_planted(rng, "deep8000", L=4, depth=(7990, 8000), every=1, af_cycle=(0.5, 0.2, 0.05, 1.0))
    return c


def case_iupac(rng):
    """IUPAC nibbles, '=', N, D/N entries, lowercase REF, q>=128 and q=255."""
    L = 40
    ref = _ref_seq(rng, L + 5, lower_frac=0.3)[5:]
    cols = []
    for i in range(L):
        d = int(rng.integers(10, 60))
        ent = []
        for k in range(d):
            u = rng.random()
            q = int(rng.integers(25, 45)) if rng.random() < 0.95 else int(rng.choice([0, 1, 2, 3, 127, 128, 200, 255]))
            if u < 0.15:
                code = int(rng.integers(0, 16))  # any nibble incl. '=' and IUPAC
            elif u < 0.2:
                code = int(rng.choice([DEL, SKIP]))
            else:
                code = CODE[ref[i].upper()] if rng.random() < 0.7 else int(rng.choice([1, 2, 4, 8, 15]))
            ent.append((code, q))
        cols.append(ent)
    return {"name": "iupac", "params": dict(DEFAULT_PARAMS, minEvidenceRatio=0.05, minAlleleDepth=2),
            "contig": "NC_045512.2", "reference": "GGGGG" + ref, "batches": [_batch_from_columns(5, cols)]}


def case_multibatch(rng):
    """Three batches over overlapping windows: accumulation + dict insertion order (vc_queue.py:142)."""
    L = 120
    ref = _ref_seq(rng, L)
    batches = []
    for bi, (lo, hi) in enumerate([(30, 90), (0, 60), (50, 120)]):
        sub = case_planted(np.random.default_rng(100 + bi), "tmp", L=hi - lo, depth=(0, 40), every=5)
        cols = _columns_of(sub["batches"][0])
        # re-code onto this reference so REF comparisons are meaningful
        batches.append(_batch_from_columns(lo, cols))
    return {"name": "multibatch", "params": DEFAULT_PARAMS, "contig": "NC_045512.2", "reference": ref,
            "batches": batches}


def case_lowq(rng):
    """minBaseQuality 0 and 4: Q0 entries (eps=1 -> 1-eps=0), Q<=3 (eps>=0.5, subnormal stalls)."""
    L = 16
    ref = _ref_seq(rng, L)
    cols = []
    for i in range(L):
        rb = ref[i]
        alt = "ACGT"[("ACGT".index(rb) + 1) % 4]
        if i < 4:     # many Q3/Q4 alt reads -> P_alt underflows, eps(3)=0.501 stalls at 1 ulp
            ent = [(CODE[rb], 35)] * 30 + [(CODE[alt], 3 + (i % 2))] * 1500
        elif i < 8:   # H for the hypothesis underflows: 1-eps(4)=0.60 over 1600 reads
            ent = [(CODE[rb], 4)] * 1600 + [(CODE[alt], 30)] * 20
        elif i < 12:  # Q0 entries present in some alleles
            ent = [(CODE[rb], int(q)) for q in rng.integers(0, 8, size=40)] + [(CODE[alt], 0)] * 6
        else:
            ent = [(CODE[rb], int(q)) for q in rng.integers(0, 45, size=60)] + \
                  [(CODE[alt], int(q)) for q in rng.integers(0, 45, size=20)]
        order = rng.permutation(len(ent))
        cols.append([ent[j] for j in order])
    p0 = dict(DEFAULT_PARAMS, minBaseQuality=0, minEvidenceRatio=0.01, minAlleleDepth=1)
    return {"name": "lowq_bq0", "params": p0, "contig": "NC_045512.2", "reference": ref,
            "batches": [_batch_from_columns(0, cols)]}


def case_edges(rng):
    """Depth/ratio threshold edges, empty columns, all-filtered columns, single-allele columns."""
    ref = "ACGTACGTACGTACGTACGT"
    A, C, G, T = 1, 2, 4, 8
    cols = [
        [],                                      # raw-empty column: not emitted by htslib
        [(A, 10)] * 5,                           # present but every entry fails bq -> totalDepth 0
        [(C, 35)] * 9 + [(A, 35)],               # depth 10 exactly, AD 9
        [(G, 35)] * 8,                           # depth 8 < minTotalDepth
        [(A, 35)] * 9 + [(G, 35)] * 1,           # AD 1 < minAlleleDepth
        [(A, 30)] * 45 + [(C, 30)] * 5,          # AD/DP = 0.1 exactly
        [(A, 30)] * 46 + [(C, 30)] * 5,          # AD/DP just below 0.1
        [(T, 41)] * 30,                          # single allele == REF? (REF index 7 is T)
        [(A, 41)] * 30,                          # single non-REF allele: GL=H, S=GL -> SCORE 99
        [(DEL, 35)] * 20 + [(A, 35)] * 6,        # D entries count in depth only
        [(SKIP, 35)] * 12,                       # only refskips
        [(G, 33)] * 6 + [(C, 33)] * 6 + [(T, 33)] * 6 + [(A, 33)] * 6 + [(15, 33)] * 6,
    ]
    return {"name": "edges", "params": DEFAULT_PARAMS, "contig": "NC_045512.2", "reference": ref,
            "batches": [_batch_from_columns(0, cols)]}


def main():
    lvc_mod, ref_utils = _install_stub()
    rng = np.random.default_rng(20261015)
    cases = [
        case_planted(rng, "planted_low", L=200, depth=(8, 120)),
        case_planted(rng, "planted_mid", L=60, depth=(300, 1200), every=3),
        case_planted(rng, "planted_lower_ref", L=80, depth=(20, 200), lower_frac=0.4, every=4),
        case_deep(rng),
        case_band(rng),
        case_iupac(rng),
        case_multibatch(rng),
        case_lowq(rng),
        case_edges(rng),
    ]
    out = {"eps_lut": [float(ref_utils.from_phred_scale(q)).hex() for q in range(256)]}
    grid = [0.0, 1e-300, 1e-12, 10 ** -0.05, 10 ** -0.15, 10 ** -0.25, 10 ** -9.95, 10 ** -9.85, 0.5, 0.9, 1.0,
            2.5e-10, 1e-10, 1.0000000000000002e-10]
    out["to_phred"] = [[float(p).hex(), int(ref_utils.to_phred_scale(p))] for p in grid]
    out["cases"] = []
    for c in cases:
        res = run_reference(lvc_mod, ref_utils, c)
        c = dict(c)
        c["expected"] = res
        out["cases"].append(c)
        print(f"{c['name']:>20}: positions={len(res['memory'])} gl_rows={len(res['gl'])} "
              f"variants={len(res['variants'])}", file=sys.stderr)
    path = os.path.join(HERE, "cases.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {path} ({os.path.getsize(path)/1e6:.2f} MB)", file=sys.stderr)


if __name__ == "__main__":
    main()
