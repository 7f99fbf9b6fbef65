"""Multi-GPU: coordinate sharding of the pileup engine (SURVEY §8 e).

Positions are independent once a batch's pileup is built, so each rank (one process per GPU,
``torch.distributed`` over RCCL/xGMI) owns one contiguous coordinate range, accumulates every
batch's columns in that range into its own engine, and finalizes locally.  The only exchange is
the final call table: one gather of the compact candidate records to rank 0 (a few KB per rank),
which merges them in the reference's memory order.  No data-path collective exists — there is
nothing to reduce, and reducing per-position fp64 sums across ranks would break the ordered
subnormal-band replay.

Ranges are cut on the CSR prefix sum so every rank gets the same number of entries (depth-
balanced, which matters for amplicon data), not the same number of positions.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N


def partition(offsets: np.ndarray, world: int, pos_begin: int = 0, span: Optional[Tuple[int, int]] = None
              ) -> List[Tuple[int, int]]:
    """Split columns [pos_begin, pos_begin + n_cols) into `world` contiguous ranges of ~equal
    entry count.  Returns absolute (lo, hi) positions per rank (possibly empty ranges).  With
    `span` (e.g. (0, contig length)) the first/last ranges are widened to cover it, so later
    batches reaching outside this batch's columns still have an owner."""
    off = np.asarray(offsets, dtype=np.uint64).astype(np.int64)
    C = len(off) - 1
    E = int(off[-1]) if C > 0 else 0
    cuts = [0]
    for r in range(1, world):
        # first column whose start offset reaches r/world of the entries
        cuts.append(int(np.searchsorted(off[:-1], (E * r + world - 1) // world, side="left")) if E else C * r // world)
    cuts.append(C)
    cuts = np.maximum.accumulate(np.array(cuts))
    parts = [[pos_begin + int(cuts[r]), pos_begin + int(cuts[r + 1])] for r in range(world)]
    if span is not None:
        parts[0][0] = min(parts[0][0], span[0])
        parts[-1][1] = max(parts[-1][1], span[1])
    return [tuple(p) for p in parts]


def slice_batch(pos_begin: int, offsets, codes, quals, lo: int, hi: int):
    """The CSR sub-batch of columns [lo, hi) (absolute positions) with rebased offsets."""
    off = np.asarray(offsets, dtype=np.uint64)
    c0 = max(0, lo - pos_begin)
    c1 = min(len(off) - 1, hi - pos_begin)
    if c1 <= c0:
        return lo, np.zeros(1, np.uint64), codes[:0], quals[:0]
    e0, e1 = int(off[c0]), int(off[c1])
    return pos_begin + c0, (off[c0:c1 + 1] - np.uint64(e0)), codes[e0:e1], quals[e0:e1]


def merge_candidates(tables: Sequence[np.ndarray]) -> np.ndarray:
    """Rank tables -> one call table in prepare_variants() order: memory insertion order
    (first batch, then position) and snvs dict order."""
    allc = np.concatenate([np.asarray(t, dtype=N.CANDIDATE_DTYPE) for t in tables]) if tables else \
        np.zeros(0, N.CANDIDATE_DTYPE)
    return allc[np.lexsort((allc["rank"], allc["pos"], allc["first_batch"]))]


def gather_candidates(local: np.ndarray, group=None, dst: int = 0, device=None) -> Optional[np.ndarray]:
    """Gather every rank's candidate records to `dst` with ONE padded gather (after a scalar
    all-gather of the counts).  `device`: torch device for the backend (cuda for nccl/RCCL, cpu
    for gloo).  Returns the merged table on `dst`, None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = torch.device("cpu") if device is None else torch.device(device)
    rec = N.CANDIDATE_DTYPE.itemsize
    n = torch.tensor([len(local)], dtype=torch.int64, device=dev)
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    cap = max(1, max(counts))
    buf = torch.zeros(cap * rec, dtype=torch.uint8)
    if len(local):
        buf[:len(local) * rec] = torch.from_numpy(np.ascontiguousarray(local).view(np.uint8).copy())
    buf = buf.to(dev)
    out = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, out, dst=dst, group=group)
    if rank != dst:
        return None
    tables = [o.cpu().numpy()[:counts[r] * rec].view(N.CANDIDATE_DTYPE) for r, o in enumerate(out)]
    return merge_candidates(tables)


class ShardedEngine:
    """One rank's share of a coordinate-sharded engine: a context over positions [lo, hi) only
    (rebased to 0, so HBM holds just this rank's accumulators), fed the [lo, hi) columns of every
    batch; its candidates go to the rank-0 call table with absolute positions."""

    def __init__(self, lo: int, hi: int, reference: str, min_base_quality=30, min_total_depth=10,
                 min_allele_depth=5, min_evidence_ratio=0.10, device=0, calls_only=True):
        from .engine import PileupEngine
        self.lo, self.hi = lo, hi
        self.engine = PileupEngine(max(1, hi - lo), min_base_quality, min_total_depth, min_allele_depth,
                                   min_evidence_ratio, device=device, reference=reference[lo:max(hi, lo + 1)],
                                   calls_only=calls_only)

        self.n_batches = 0          # batches seen by the job (global sequence)
        self._global_seq = []       # local engine batch seq - 1 -> global batch seq

    def reset(self):
        self.engine.reset()
        self.n_batches = 0
        self._global_seq = []

    def accumulate(self, pos_begin, offsets, codes, quals):
        """Every rank sees every batch (so the global batch sequence — memory insertion order —
        is the same everywhere); only its own columns reach its engine."""
        self.n_batches += 1
        pb, off, c, q = slice_batch(pos_begin, offsets, codes, quals, self.lo, self.hi)
        if len(off) > 1 and int(off[-1]) > 0:
            self.engine.accumulate(pb - self.lo, off, c, q)
            self._global_seq.append(self.n_batches)

    def process_bam(self, path: str, contig: str, params=None):
        """process_bam (live_variant_caller.py:54-72) for this rank's range only: the host pileup builds
        just the [lo, hi) columns (spp_pileup_region; the depth cap still sees every read), so each
        rank inflates the BAM but decodes and flattens only its shard."""
        from .pileup import AlignmentFile
        self.n_batches += 1
        with AlignmentFile(path) as f:
            b = f.pileup_batch(contig, params, start=self.lo, stop=self.hi)
            if b.n_cols and b.n_entries:
                self.engine.accumulate(b.pos_begin - self.lo, b.offsets, b.codes, b.quals)
                self._global_seq.append(self.n_batches)
            b.close()

    def local_candidates(self) -> np.ndarray:
        self.engine.finalize()
        c = self.engine.candidates()
        c["pos"] += self.lo
        if len(c):
            c["first_batch"] = np.asarray(self._global_seq, np.uint32)[c["first_batch"].astype(np.int64) - 1]
        return c

    def gather(self, group=None, device=None):
        return gather_candidates(self.local_candidates(), group=group, device=device)
