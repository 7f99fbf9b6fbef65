"""Per-wave timeline of the deep accumulate kernel (profiling; SPG_WAVE_TIMES instrumentation).

Runs the bench's 10,000x SARS-CoV-2 batch through the fused accumulate a few times with
SPG_WAVE_TIMES=<file> (k_acc_seg records per wave: entry, lifetime from entry and entry-to-loop prologue in
s_memrealtime ticks of 10 ns, its first column, and HW_ID / XCC_ID), then reports the launch's span, the wave generations, setup and lifetime
distributions, and how the tail ends.  Usage: python tools/wavetimes.py [depth] [out.json] [max_depth]
(max_depth 8000: the parity-mode batch the bench's nested parity_mode line runs)
"""
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(depth, path, max_depth=0):
    import torch
    import spings  # noqa: F401
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.engine import PileupEngine
    from covid_spings_variant_caller_amd.pileup import synth_batch
    L = 29903
    ref = synth.reference(L, seed=1)
    b = synth_batch(ref, depth, seed=2, n_threads=16, max_depth=max_depth)
    dc = torch.from_numpy(b.codes_padded).cuda()
    dq = torch.from_numpy(b.quals_padded).cuda()
    do = torch.from_numpy(b.offsets.view(np.int64).copy()).cuda()
    eng = PileupEngine(L, 30, 10, 5, 0.10, device=0, reference=ref, calls_only=True)
    for _ in range(4):
        eng.reset()
        eng.accumulate(0, do, dc, dq, borrow=True, n_entries=b.n_entries)
        eng.finalize()
    eng.sync()
    eng.close()


def analyse(path):
    raw = open(path, "rb").read()
    at, launches = 0, []
    while at < len(raw):
        n, g = np.frombuffer(raw[at:at + 16], np.int64)
        at += 16
        w = np.frombuffer(raw[at:at + 16 * n], np.uint32).reshape(n, 4)
        at += 16 * int(n)
        launches.append((int(g), w))
    per_launch = []                                  # per-XCC spans of every launch (is the slow XCD always the same?)
    for _, wl in launches:
        wl = wl[wl[:, 2] != 0]
        s0 = wl[:, 0].astype(np.int64)
        e0 = (s0 - s0.min()) * 10e-3 + (wl[:, 2] & 0xFFFFF) * 10e-3
        x0 = wl[:, 3] >> 24
        per_launch.append({int(x): round(float(e0[x0 == x].max()), 2) for x in np.unique(x0)})
    g, w = launches[-1]
    n_all = len(w)
    w = w[w[:, 2] != 0]                              # (dynamic-tail waves that found no unit exit unrecorded)
    t0 = w[:, 0].astype(np.int64)
    t0 = (t0 - t0.min()) * 10e-3                     # us
    col = (w[:, 1] & 0x7FFF).astype(np.int64)        # (first column mod 2^15: SARS-CoV-2 fits)
    lend = (w[:, 1] >> 15) * 10e-3                   # entry -> the chunk loop's end
    tailed = ((w[:, 3] >> 20) & 1).astype(bool)      # the wave ran the fused finalize (a possible call)
    life = (w[:, 2] & 0xFFFFF) * 10e-3              # from the wave's entry
    pro = (w[:, 2] >> 20) * 10e-3                    # entry -> first chunk loop setup (LUT, CSR offsets)
    end = t0 + life
    xcc = w[:, 3] >> 24
    span = float(end.max())
    q = lambda a: {p: round(float(np.percentile(a, p)), 2) for p in (5, 25, 50, 75, 95, 100)}
    res = {"waves": int(len(w)), "waves_launched": int(n_all), "G": g, "span_us": round(span, 2),
           "start_us": q(t0), "life_us": q(life), "prologue_us": q(pro), "end_us": q(end),
           "longest_waves": [{"first_column": int(col[i]), "life_us": round(float(life[i]), 2),
                              "loop_end_us": round(float(lend[i]), 2), "fused_finalize": bool(tailed[i]),
                              "start_us": round(float(t0[i]), 2)} for i in np.argsort(-life)[:12]],
           "fused_finalize_waves": int(tailed.sum()),
           "finalize_us_of_those": q(life[tailed] - lend[tailed]) if tailed.any() else None,
           "loop_us_of_those": q(lend[tailed] - pro[tailed]) if tailed.any() else None,
           "loop_us_all": q(lend - pro),
           "last_10_waves_to_end": [{"first_column": int(col[i]), "start_us": round(float(t0[i]), 2),
                                     "loop_end_us": round(float(lend[i]), 2), "life_us": round(float(life[i]), 2),
                                     "fused_finalize": bool(tailed[i]), "xcc": int(xcc[i])}
                                    for i in np.argsort(-end)[:10]],
           "waves_ending_after_span_minus_5us": int((end > span - 5).sum()),
           "waves_starting_after_span_minus_10us": int((t0 > span - 10).sum()),
           "busy_wave_us_over_span": round(float(life.sum()) / span, 1),
           "per_xcc_span_us": {int(x): round(float(end[xcc == x].max() - t0[xcc == x].min()), 2)
                               for x in np.unique(xcc)}}
    # a workgroup's LDS is held until its longest wave ends: wave-time its finished waves leave idle
    # (records are indexed by wave id; 4 waves per workgroup)
    nb4 = len(w) // 4 * 4
    blk_end = end[:nb4].reshape(-1, 4).max(axis=1)
    res["workgroup_slack_over_wave_time"] = round(float((blk_end[:, None] - end[:nb4].reshape(-1, 4)).sum())
                                                  / float(life.sum()), 3)
    # wave slot turnover: per hardware wave slot (XCC, HW_ID wave/SIMD/CU/SA/SE fields), the gap from
    # one wave's end to the next wave's entry in that slot (dispatch of the next workgroup)
    key = (xcc.astype(np.int64) << 20) | (w[:, 3] & 0xFFFF).astype(np.int64)
    o = np.lexsort((t0, key))
    same = key[o][1:] == key[o][:-1]
    gaps = (t0[o][1:] - end[o][:-1])[same]
    if len(gaps):
        res["slot_gap_us"] = q(gaps)
        res["slot_gap_total_over_wave_time"] = round(float(np.clip(gaps, 0, None).sum()) / float(life.sum()), 3)
    hist, edges = np.histogram(t0, bins=20, range=(0, span))
    res["start_histogram"] = hist.tolist()
    conc = [int(((t0 <= t) & (end > t)).sum()) for t in np.linspace(0, span, 23)[1:-1]]
    res["resident_waves_over_time"] = conc
    res["per_xcc_end_us_every_launch"] = per_launch
    return res


if __name__ == "__main__":
    depth = float(sys.argv[1]) if len(sys.argv) > 1 else 10000.0
    out = sys.argv[2] if len(sys.argv) > 2 else None
    max_depth = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    # (set before the library is loaded, in this process: an A/B build loaded by tools/ab_run.py is the one timed)
    path = os.environ.get("SPG_WAVE_TIMES")
    if not path:
        path = os.path.join(tempfile.mkdtemp(), "wt.bin")
        os.environ["SPG_WAVE_TIMES"] = path
    if os.path.exists(path):
        os.remove(path)
    run(depth, path, max_depth)
    res = analyse(path)
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)
