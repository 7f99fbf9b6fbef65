"""Seeded synthetic pileups in the engine's CSR layout (SURVEY §8 d: "Synthetic inputs").

Column-major construction: reads of length R start uniformly on [0, L-R] (sorted); column c holds
the reads covering it in start order (htslib pileup order for single-end, flag 0, MAPQ 60 reads).
Per entry: q = clip(round(N(33, 6)), 2, 41); base = REF (or the planted SNV allele at every
`snv_every`-th position with AF cycling {1.0, 0.5, 0.2, 0.05}); a sequencing error replaces it by
a uniform other base with probability eps(q); N with probability 1e-4; CIGAR D entries with the
rate of 1% of reads carrying a 2-base deletion (code 16, quality of the next base).
Entries are drawn i.i.d. per (read, column) — the pileup byte stream has the statistics of the
survey's read model; per-read CIGAR structure is produced by the C++ read simulator
(libspings_pileup) when exact read-level pileups are needed.
"""
from __future__ import annotations

import numpy as np

ACGT = np.array([1, 2, 4, 8], dtype=np.uint8)
CODE_OF = {"A": 1, "C": 2, "G": 4, "T": 8, "N": 15}


def reference(L: int, seed: int = 1) -> str:
    rng = np.random.default_rng(seed)
    return np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=L)].tobytes().decode("ascii")


def pileup(L: int, depth: float, seed: int = 2, read_len: int = 150, ref: str | None = None,
           snv_every: int = 997, lo: int = 0, hi: int | None = None, max_depth: int = 0):
    """Return (pos_begin, offsets u64[C+1], codes u8[E], quals u8[E]) for columns [lo, hi)."""
    hi = L if hi is None else hi
    ref = reference(L) if ref is None else ref
    rng = np.random.default_rng(seed)
    n_reads = int(round(depth * L / read_len))
    starts = np.sort(rng.integers(0, max(1, L - read_len + 1), size=n_reads))
    cols = np.arange(lo, hi, dtype=np.int64)
    r_lo = np.searchsorted(starts, cols - read_len + 1, side="left")
    r_hi = np.searchsorted(starts, cols, side="right")
    lens = (r_hi - r_lo).astype(np.int64)
    if max_depth:
        lens = np.minimum(lens, max_depth)
    offsets = np.zeros(len(cols) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    E = int(offsets[-1])
    ref_codes = np.frombuffer(ref.encode(), dtype=np.uint8)
    lut = np.zeros(256, np.uint8)
    for ch, c in CODE_OF.items():
        lut[ord(ch)] = c
        lut[ord(ch.lower())] = c
    rc = lut[ref_codes[lo:hi]]
    col_of = np.repeat(np.arange(len(cols), dtype=np.int64), lens)
    base = rc[col_of]
    # planted SNVs
    pos = cols[col_of]
    planted = (pos % snv_every) == (snv_every // 2)
    if planted.any():
        afs = np.array([1.0, 0.5, 0.2, 0.05])
        af = afs[(pos[planted] // snv_every) % 4]
        alt_idx = (np.log2(base[planted]).astype(np.int64) + 1 + (pos[planted] % 3)) % 4
        take = rng.random(planted.sum()) < af
        b = base[planted]
        b[take] = ACGT[alt_idx[take]]
        base[planted] = b
    q = np.clip(np.rint(rng.normal(33.0, 6.0, size=E)), 2, 41).astype(np.uint8)
    eps = 10.0 ** (-q.astype(np.float64) / 10.0)
    err = rng.random(E) < eps
    if err.any():
        cur = np.log2(base[err]).astype(np.int64)
        base[err] = ACGT[(cur + 1 + rng.integers(0, 3, size=err.sum())) % 4]
    base[rng.random(E) < 1e-4] = 15
    dele = rng.random(E) < (0.01 * 2 / read_len)
    base[dele] = 16
    return lo, offsets, base.astype(np.uint8), q


def to_device(offsets, codes, quals, device: int = 0):
    """Copy a CSR batch to HBM as torch tensors (16-byte padded byte arrays)."""
    import torch
    dev = torch.device("cuda", device)
    E = len(codes)
    pad = (E + 16 + 15) & ~15
    c = torch.full((pad,), 0xFF, dtype=torch.uint8)
    q = torch.zeros((pad,), dtype=torch.uint8)
    c[:E] = torch.from_numpy(codes)
    q[:E] = torch.from_numpy(quals)
    o = torch.from_numpy(offsets.view(np.int64).copy())
    return o.to(dev), c.to(dev), q.to(dev)
