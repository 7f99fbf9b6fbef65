"""Per-column statistics of a synthetic batch as k_acc_seg sees them (dev tool, CPU only): the
first-chunk allele vote (major M, second M2, dual mode), rare-entry counts per column and per lane
slice, chunks whose rare slices fill the queue.

python tools/colstats.py DEPTH [LO HI] [--native]
  default data: tools/kbench.py's cached batch; --native: bench.py's (libspings_pileup spp_synth_batch)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
args = [a for a in sys.argv[1:] if not a.startswith("--")]
depth = int(args[0]) if args else 100000
import spings  # noqa: E402,F401
from covid_spings_variant_caller_amd import synth  # noqa: E402

ref = synth.reference(29903, seed=1)
if "--native" in sys.argv:
    from covid_spings_variant_caller_amd.pileup import synth_batch
    bt = synth_batch(ref, depth, lo=0, hi=29903, seed=2, n_threads=16, max_depth=0)
    off, c, q = bt.offsets, bt.codes, bt.quals
else:
    from kbench import data
    _, off, c, q = data(depth, 0)
C = len(off) - 1
lo, hi = (int(args[1]), int(args[2])) if len(args) > 2 else (0, C)
VC = [1, 2, 4, 8, 15, 16, 17]
MIN_BQ = 30
duals = {}
rows = []
for col in range(lo, hi):
    b, e = int(off[col]), int(off[col + 1])
    if e <= b:
        continue
    a = b & ~15
    lanes = a + 16 * np.arange(64)
    ok = (lanes >= b) & (lanes < e)
    v = c[lanes[ok]]
    cnt = [int(np.sum(v == k)) for k in VC]
    b1 = int(np.argmax(cnt[:4]))
    b2, c2n = -1, 1
    for k in range(7):
        if k != b1 and cnt[k] > c2n:
            c2n, b2 = cnt[k], k
    M, M2 = VC[b1], (VC[b2] if b2 >= 0 else 0)
    if b2 >= 0:
        duals[M2] = duals.get(M2, 0) + 1
    cc, qq = c[b:e], q[b:e]
    rare = (qq >= MIN_BQ) & (cc != M) & ((cc != M2) if M2 else True)
    idx = np.nonzero(rare)[0] + (b - a)          # lane slices: 16-entry blocks from the aligned start
    sl = np.bincount(idx // 16) if len(idx) else np.zeros(1, int)
    per_chunk = np.bincount(np.nonzero(sl)[0] // 64) if len(idx) else np.zeros(1, int)
    refc = ref[col].upper()
    rows.append((col, e - b, M, M2, int(rare.sum()), int(sl.max()), int(per_chunk.max()),
                 "ACGT"[b1] != refc, cnt, sorted(set(np.unique(cc).tolist())), int(qq.min()), int(qq.max())))
n_rare = np.array([r[4] for r in rows])
print("columns", hi - lo, "dual by M2", duals, "rare/col: mean %.1f max %d" % (n_rare.mean(), n_rare.max()))
print("col len M M2 rare max_per_slice max_slices_per_chunk major!=REF votes codes qmin qmax")
for r in rows:
    if r[3] or r[7] or r[4] > 3 * n_rare.mean() or r[5] > 4 or r[6] > 32 or len(r[9]) > 6 or r[10] < 2 or r[11] > 41:
        print(*r)
