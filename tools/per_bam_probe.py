"""Probe the per-BAM finalize loop (vc_queue.py:142-144) on device-generated 100x SARS-CoV-2 BAMs: per-BAM latency,
GPU interval times, replayed positions and the engine's path counters; prints the slowest BAMs.

    python tools/per_bam_probe.py [n_bams] [out.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    out = sys.argv[2] if len(sys.argv) > 2 else None
    import torch
    import spings  # noqa: F401
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.synth_device import many_bams
    L = 29903
    ref = synth.reference(L, seed=1)
    data = many_bams(ref, nb, 100.0, seed=1000, max_depth=8000, device=torch.device("cuda", 0))
    torch.cuda.synchronize()
    recs = data.records(pos_begin=0)
    eng = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    for rnd in range(2):
        eng.reset()
        eng.sync()
        eng.kernel_times(4096)
        eng.set_timing(2)
        lat, acc, fin, band, ncand = (np.zeros(nb) for _ in range(5))
        done = 0
        for i in range(nb):
            t = time.perf_counter()
            eng.accumulate_records(recs[i:i + 1])
            eng.finalize()
            calls = eng.candidates()
            lat[i] = time.perf_counter() - t
            ncand[i], band[i] = eng.counts()
            if (i + 1) % 128 == 0 or i == nb - 1:
                a, f = eng.kernel_times(4096)
                acc[done:done + len(a)] = a
                fin[done:done + len(f)] = f
                done += len(a)
        slow = np.argsort(-lat)[:25]
        res = {"round": rnd, "bams": nb, "total_s": float(lat.sum()), "p50_ms": float(np.median(lat) * 1e3),
               "mean_ms": float(lat.mean() * 1e3), "acc_ms_mean": float(acc.mean()), "fin_ms_mean": float(fin.mean()),
               "bams_with_replays": int((band > 0).sum()), "replays_total": int(band.sum()),
               "slow": [[int(i), round(lat[i] * 1e3, 3), round(float(acc[i]), 3), round(float(fin[i]), 3), int(band[i]),
                         int(ncand[i])] for i in slow],
               "paths": eng.path_counters()}
        print(json.dumps(res), flush=True)
        if out:
            with open(out, "a") as f:
                f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
