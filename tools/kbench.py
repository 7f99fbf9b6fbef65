"""Kernel A/B micro-benchmark (dev tool): times accumulate / finalize kernels with HIP events on the
10,000x SARS-CoV-2 workload.  The library under test comes from $SPG_GPU_LIB (default: in-tree build).
The synthetic batch is cached in $TMPDIR so several variants can be compared in one GPU session."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def data(depth, max_depth):
    from covid_spings_variant_caller_amd import synth
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"spg_sars_{int(depth)}_{max_depth}.npz")
    ref = synth.reference(29903)
    if os.path.exists(path):
        z = np.load(path)
        return ref, z["off"], z["c"], z["q"]
    _, off, c, q = synth.pileup(29903, depth, seed=2, ref=ref, max_depth=max_depth)
    np.savez(path, off=off, c=c, q=q)
    return ref, off, c, q


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=float, default=10000)
    ap.add_argument("--max-depth", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default=os.environ.get("SPG_GPU_LIB", "default"))
    ap.add_argument("--calls-only", action="store_true")
    a = ap.parse_args()
    import torch
    import spings  # noqa: F401
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    torch.cuda.set_device(0)
    ref, off, c, q = data(a.depth, a.max_depth)
    do, dc, dq = synth.to_device(off, c, q)
    eng = PileupEngine(len(off) - 1, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=a.calls_only)
    accs, fins, steps = [], [], []
    for it in range(a.iters + 3):
        t0 = time.perf_counter()
        eng.reset()
        eng.accumulate(0, do, dc, dq, borrow=True, n_entries=len(c))
        eng.finalize()
        eng.sync()
        t1 = time.perf_counter()
        if it >= 3:
            steps.append((t1 - t0) * 1e3)
    accs, fins = eng.kernel_times()
    accs, fins = accs[3:], fins[3:]
    E = len(c)
    B = 2 * E + 8 * len(off)
    acc = float(np.median(accs))
    print(json.dumps({"tag": a.tag, "calls_only": a.calls_only, "acc_ms": acc, "acc_min_ms": float(np.min(accs)), "fin_ms": float(np.median(fins)),
                      "step_ms": float(np.median(steps)), "GBps": B / acc / 1e6, "frac": B / acc / 1e6 / 8000,
                      "n_cand": eng.counts()[0]}))


if __name__ == "__main__":
    main()
