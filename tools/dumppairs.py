"""Dump column pairs of tools/kbench.py's cached batch (dev tool, CPU only): codes, quals, offsets
rebased to the pair, REF chars -> gpurun_out/pairs_<depth>.npz."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spings  # noqa: E402,F401
from kbench import data  # noqa: E402

depth = int(sys.argv[1])
cols = [int(x) for x in sys.argv[2:]]
ref, off, c, q = data(depth, 0)
out = {}
for g0 in cols:
    b, e = int(off[g0]), int(off[g0 + 2])
    out[f"off_{g0}"] = off[g0:g0 + 3].astype(np.int64) - b
    out[f"c_{g0}"] = c[b:e]
    out[f"q_{g0}"] = q[b:e]
    out[f"base_{g0}"] = np.array([b], np.int64)
out["ref"] = np.frombuffer(ref.encode(), np.uint8)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/pairs_{depth}.npz", **out)
print("dumped", cols)
