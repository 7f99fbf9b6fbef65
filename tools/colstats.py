"""Per-column statistics of a cached kbench batch ($TMPDIR/spg_sars_<depth>_0.npz) as k_acc_seg sees
them (dev tool): the first-chunk allele vote (major M, second M2, dual mode) and rare-entry counts."""
import os
import sys

import numpy as np

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
if "--native" in sys.argv:          # bench.py's data: libspings_pileup spp_synth_batch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import spings  # noqa: F401
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import synth_batch
    bt = synth_batch(synth.reference(29903, seed=1), depth, lo=0, hi=29903, seed=2, n_threads=16, max_depth=0)
    off, c, q = bt.offsets, bt.codes, bt.quals
else:                               # tools/kbench.py's data (cached npz, generated if missing)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import spings  # noqa: F401
    from kbench import data
    _, off, c, q = data(depth, 0)
C = len(off) - 1
VC = [1, 2, 4, 8, 15, 16, 17]
duals = {}
special = []
for col in range(C):
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
    if b2 >= 0:
        duals[VC[b2]] = duals.get(VC[b2], 0) + 1
        if VC[b2] >= 15:
            special.append((col, VC[b1], VC[b2], cnt))
print("columns", C, "dual by M2", duals)
print("dual with M2 in {N, D, skip}:", special[:20])
