"""Seeded synthetic pileups generated directly in HBM (bench / test data, not the product path).

Same read model as ``synth.pileup`` (SURVEY §8 d): 150-bp single-end reads with uniform sorted starts;
column c of a sample holds the reads covering it in start order (htslib pileup order), capped at
``max_depth``; q = clip(round(N(33, 6)), 2, 41); a sequencing error replaces the base by a uniform
other base with probability eps(q); N with probability 1e-4; CIGAR-D entries at the rate of 1% of
reads carrying a 2-base deletion; a planted SNV every ``snv_every``-th position with AF cycling
{1.0, 0.5, 0.2, 0.05}.  Random numbers come from torch's seeded device generator (Philox), so one
(seed, shape) always gives the same batches; they are not the numpy streams of ``synth.pileup``.

Used for BASELINE config 4 (10,000 BAM-sized 100x batches of SARS-CoV-2 = 3.0e10 entries, 60 GB):
building that on the host would take minutes; here a chunk of samples is one batch of device ops.
Batches of one call share three arenas (offsets int64 [n][C+1], codes, quals with 16 bytes of
padding after the last entry), so each batch is a borrowed device input of the engine.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

import numpy as np

ACGT = (1, 2, 4, 8)


@dataclass
class DeviceBatches:
    pos_begin: int
    n_cols: int
    offsets: "object"              # torch int64 [n, C+1] (per-batch rows start at 0)
    codes: "object"                # torch uint8 [sum E + 16]
    quals: "object"
    base: np.ndarray               # entry offset of batch i in the code / qual arenas
    n_entries: np.ndarray          # entries of batch i
    extra: list = field(default_factory=list)

    def __len__(self):
        return len(self.base)

    def batch(self, i):
        """(pos_begin, offsets, codes, quals, n_entries) views of batch i (borrowable)."""
        b, e = int(self.base[i]), int(self.n_entries[i])
        return (self.pos_begin, self.offsets[i], self.codes[b:b + e + 16], self.quals[b:b + e + 16], e)

    def records(self, pos_begin=None):
        """spg_batch records (include/spings_gpu.h) of every batch, for PileupEngine.accumulate_records;
        ``pos_begin`` overrides the first column's position (0 for an engine over this shard only)."""
        from . import _native as N
        rec = np.zeros(len(self), N.BATCH_DTYPE)
        C = self.n_cols
        rec["pos_begin"] = self.pos_begin if pos_begin is None else pos_begin
        rec["n_cols"] = C
        rec["offsets"] = self.offsets.data_ptr() + np.arange(len(self), dtype=np.uint64) * np.uint64(8 * (C + 1))
        rec["base_code"] = np.uint64(self.codes.data_ptr()) + self.base.astype(np.uint64)
        rec["qual"] = np.uint64(self.quals.data_ptr()) + self.base.astype(np.uint64)
        rec["n_entries"] = self.n_entries.astype(np.uint64)
        return rec

    def host(self, i):
        """Host copy of batch i: (pos_begin, offsets u64, codes u8, quals u8) for the oracle."""
        pb, off, c, q, e = self.batch(i)
        return (pb, off.cpu().numpy().view(np.uint64).copy(), c[:e].cpu().numpy().copy(), q[:e].cpu().numpy().copy())


def _q_table(device):
    """clip(round(N(33, 6)), 2, 41) as a 4096-entry inverse-CDF table (uniform index -> q)."""
    import torch
    from scipy.stats import norm
    u = (np.arange(4096) + 0.5) / 4096.0
    q = np.clip(np.rint(norm.ppf(u, loc=33.0, scale=6.0)), 2, 41).astype(np.uint8)
    return torch.from_numpy(q).to(device)


def many_bams(reference: str, n_batches: int, depth: float, seed: int = 1000, lo: int = 0, hi: int | None = None,
              read_len: int = 150, max_depth: int = 0, snv_every: int = 997, device=None,
              chunk_entries: float = 2.0e8) -> DeviceBatches:
    """``n_batches`` samples ("BAMs") of ``depth`` x over ``reference``, columns [lo, hi) only (a
    coordinate shard), generated in HBM.  Sample i is seeded by seed + i."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    L = len(reference)
    hi = L if hi is None else hi
    C = hi - lo
    cols = torch.arange(lo, hi, device=dev, dtype=torch.int64)
    gen = _EntryGen(reference, lo, hi, read_len, snv_every, seed, dev)
    n_reads = int(round(depth * L / read_len))
    per_sample = max(1.0, depth * C)
    chunk = max(1, min(n_batches, int(chunk_entries // per_sample)))
    offsets = torch.zeros((n_batches, C + 1), dtype=torch.int64, device=dev)
    lens_all = []
    # pass 1: column depths of every sample (read starts are cheap to regenerate per chunk)
    for s0 in range(0, n_batches, chunk):
        s1 = min(n_batches, s0 + chunk)
        lens_all.append(_lens(s0, s1, seed, n_reads, L, read_len, cols, max_depth, dev)[1])
    lens_cat = torch.cat(lens_all)
    offsets[:, 1:] = torch.cumsum(lens_cat, dim=1)
    n_entries = offsets[:, -1].cpu().numpy().astype(np.int64)
    base = np.zeros(n_batches, np.int64)
    np.cumsum(n_entries[:-1], out=base[1:])
    E = int(n_entries.sum())
    codes = torch.empty(E + 16, dtype=torch.uint8, device=dev)
    quals = torch.empty(E + 16, dtype=torch.uint8, device=dev)
    codes[E:] = 0xFF
    quals[E:] = 0
    for s0 in range(0, n_batches, chunk):
        s1 = min(n_batches, s0 + chunk)
        lens = lens_cat[s0:s1]
        e0, e1 = int(base[s0]), int(base[s1 - 1] + n_entries[s1 - 1])
        flat = lens.reshape(-1)
        col = torch.repeat_interleave(torch.arange(C, device=dev).repeat(s1 - s0), flat)
        b, q = gen.draw(col, s0)
        codes[e0:e1] = b
        quals[e0:e1] = q
        del col, q, b
    return DeviceBatches(lo, C, offsets, codes, quals, base, n_entries)


@dataclass
class DeviceColumns:
    """n_samples BAMs as ONE column-major multi-sample batch (spg_accumulate_samples layout): column c
    holds sample 0's entries at c, then sample 1's, ...; first_sample[c] is the first sample with any."""
    pos_begin: int
    n_cols: int
    n_samples: int
    offsets: "object"              # torch int64 [C+1]
    first_sample: "object"         # torch int32 [C]
    codes: "object"                # torch uint8 [E + 16]
    quals: "object"
    n_entries: int


def many_bams_columns(reference: str, n_samples: int, depth: float, seed: int = 1000, lo: int = 0,
                      hi: int | None = None, read_len: int = 150, max_depth: int = 0, snv_every: int = 997,
                      device=None, chunk_entries: float = 2.0e8) -> DeviceColumns:
    """Same samples as ``many_bams`` (read starts and per-BAM depth caps per sample, seeded per chunk of
    samples), laid out column-major.  Entry values are i.i.d. given the column under the read model,
    so each column's concatenated stream is drawn directly in HBM."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    L = len(reference)
    hi = L if hi is None else hi
    C = hi - lo
    cols = torch.arange(lo, hi, device=dev, dtype=torch.int64)
    n_reads = int(round(depth * L / read_len))
    chunk = max(1, min(n_samples, int(chunk_entries // max(1.0, depth * C))))
    tot = torch.zeros(C, dtype=torch.int64, device=dev)
    first = torch.full((C,), -1, dtype=torch.int64, device=dev)
    for s0 in range(0, n_samples, chunk):
        s1 = min(n_samples, s0 + chunk)
        lens = _lens(s0, s1, seed, n_reads, L, read_len, cols, max_depth, dev)[1]
        tot += lens.sum(dim=0)
        has = lens > 0
        f = torch.where(has.any(dim=0), has.int().argmax(dim=0) + s0, torch.full_like(first, -1))
        first = torch.where((first < 0) & (f >= 0), f, first)
    offsets = torch.zeros(C + 1, dtype=torch.int64, device=dev)
    offsets[1:] = torch.cumsum(tot, dim=0)
    E = int(offsets[-1].item())
    codes = torch.empty(E + 16, dtype=torch.uint8, device=dev)
    quals = torch.empty(E + 16, dtype=torch.uint8, device=dev)
    codes[E:] = 0xFF
    quals[E:] = 0
    # entries in column chunks of ~chunk_entries
    gen = _EntryGen(reference, lo, hi, read_len, snv_every, seed, dev)
    c0 = 0
    off_h = offsets.cpu().numpy()
    while c0 < C:
        c1 = int(np.searchsorted(off_h, off_h[c0] + chunk_entries, side="right"))
        c1 = min(C, max(c0 + 1, c1 - 1))
        e0, e1 = int(off_h[c0]), int(off_h[c1])
        if e1 > e0:
            col = torch.repeat_interleave(torch.arange(c0, c1, device=dev), tot[c0:c1])
            b, q = gen.draw(col, c0)
            codes[e0:e1] = b
            quals[e0:e1] = q
            del col, b, q
        c0 = c1
    return DeviceColumns(lo, C, n_samples, offsets, first.clamp(min=0).to(torch.int32), codes, quals, E)


class _EntryGen:
    """Per-entry draws of the read model given each entry's column (shared by the generators)."""

    def __init__(self, reference, lo, hi, read_len, snv_every, seed, dev):
        import torch
        ref_codes = np.zeros(256, np.uint8)
        for ch, c in zip("ACGTN", (1, 2, 4, 8, 15)):
            ref_codes[ord(ch)] = c
            ref_codes[ord(ch.lower())] = c
        self.rc = torch.from_numpy(ref_codes[np.frombuffer(reference[lo:hi].encode(), np.uint8)]).to(dev)
        cols = torch.arange(lo, hi, device=dev, dtype=torch.int64)
        self.planted = (cols % snv_every) == (snv_every // 2)
        self.af = torch.tensor([1.0, 0.5, 0.2, 0.05], device=dev)[((cols // snv_every) % 4)]
        self.acgt = torch.tensor(ACGT, dtype=torch.uint8, device=dev)
        self.ref_idx = torch.zeros_like(self.rc, dtype=torch.int64)
        for k, v in {1: 0, 2: 1, 4: 2, 8: 3}.items():
            self.ref_idx[self.rc == k] = v
        self.alt_idx = (self.ref_idx + 1 + (cols % 3)) % 4
        self.qtab = _q_table(dev)
        self.eps = torch.tensor([10.0 ** (-q / 10.0) for q in range(256)], device=dev, dtype=torch.float32)
        self.read_len, self.seed, self.dev = read_len, seed, dev

    def draw(self, col, salt):
        import torch
        dev = self.dev
        g = torch.Generator(device=dev)
        g.manual_seed(int(self.seed) * 1_000_003 + int(salt))
        ne = col.numel()
        q = self.qtab[torch.randint(0, 4096, (ne,), generator=g, device=dev)]
        b = self.rc[col]
        bi = self.ref_idx[col]
        pl = self.planted[col]
        if bool(pl.any()):
            take = pl & (torch.rand(ne, generator=g, device=dev) < self.af[col])
            b = torch.where(take, self.acgt[self.alt_idx[col]], b)
            bi = torch.where(take, self.alt_idx[col], bi)
        err = torch.rand(ne, generator=g, device=dev) < self.eps[q.long()]
        shift = torch.randint(1, 4, (ne,), generator=g, device=dev)
        b = torch.where(err, self.acgt[(bi + shift) % 4], b)
        b = torch.where(torch.rand(ne, generator=g, device=dev) < 1e-4, torch.full_like(b, 15), b)
        b = torch.where(torch.rand(ne, generator=g, device=dev) < (0.01 * 2 / self.read_len), torch.full_like(b, 16), b)
        return b, q


def _lens(s0, s1, seed, n_reads, L, read_len, cols, max_depth, dev):
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed) * 7_919 + s0)
    starts = torch.randint(0, max(1, L - read_len + 1), (s1 - s0, n_reads), generator=g, device=dev)
    starts, _ = torch.sort(starts, dim=1)
    q_lo = (cols - read_len + 1).unsqueeze(0).expand(s1 - s0, -1).contiguous()
    q_hi = cols.unsqueeze(0).expand(s1 - s0, -1).contiguous()
    r_lo = torch.searchsorted(starts, q_lo, right=False)
    r_hi = torch.searchsorted(starts, q_hi, right=True)
    lens = r_hi - r_lo
    if max_depth:
        lens = torch.clamp(lens, max=max_depth)
    return r_lo, lens
