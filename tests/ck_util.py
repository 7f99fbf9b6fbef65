"""Host restatement of the checkpoint's batch compaction (test checker for spg_history_copy_compact, which runs it on
the GPU): the entries the base-quality filter keeps (live_variant_caller.py:89, :96-103) plus a first-entry marker per
column whose entries all fail it (its first visit, :77-85)."""
import numpy as np


def bq_compact(off, codes, quals, min_bq: int):
    off = np.asarray(off, np.uint64)
    if min_bq <= 0 or len(codes) == 0:
        return off, codes, quals
    lens = np.diff(off.astype(np.int64))
    col = np.repeat(np.arange(len(lens), dtype=np.int64), lens)
    keep = quals >= min_bq
    kept = np.bincount(col[keep], minlength=len(lens))
    marker = (lens > 0) & (kept == 0)
    keep[off[:-1][marker].astype(np.int64)] = True
    new_lens = np.bincount(col[keep], minlength=len(lens))
    new_off = np.zeros(len(off), np.uint64)
    np.cumsum(new_lens, out=new_off[1:])
    return new_off, np.ascontiguousarray(codes[keep]), np.ascontiguousarray(quals[keep])
