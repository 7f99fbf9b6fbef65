"""plan_bench.py [depth] [max_depth]: spg_bam_plan_build (htslib's depth cap and mate pairing on the GPU) on the end-to-end
leg's 10,000x SARS-CoV-2 BAM kept in HBM: wall ms per build (each synchronised), and the plan's counts.  Dev tool."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spings  # noqa: E402,F401
from covid_spings_variant_caller_amd import synth  # noqa: E402
from covid_spings_variant_caller_amd.engine import PileupEngine  # noqa: E402
from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams, simulate_bam  # noqa: E402

depth = float(sys.argv[1]) if len(sys.argv) > 1 else 10000.0
max_depth = int(sys.argv[2]) if len(sys.argv) > 2 else 8000
ref = synth.reference(29903, seed=1)
bam = os.path.join(tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp")), "s.bam")
simulate_bam(bam, "NC_045512.2", ref, depth=depth, seed=5, n_threads=16)
eng = PileupEngine(29904, reference=ref)
prm = PileupParams(max_depth=max_depth)
res = {"depth": depth, "max_depth": max_depth, "ms": []}
with AlignmentFile(bam) as f:
    m = f.bam_map(16)
    n = eng.bam_open(m, f.tid("NC_045512.2"), prm)
    m.close()
    for _ in range(6):
        eng.sync()
        t = time.perf_counter()
        p = eng.bam_plan_build(prm.max_depth, prm.ignore_overlaps)
        eng.sync()
        res["ms"].append(round((time.perf_counter() - t) * 1e3, 3))
        if hasattr(eng._L, "spg_ab_prof"):     # (tools/src_ab.py sweep_prof build: the sweep's phase clocks)
            import ctypes as C
            pr = (C.c_uint64 * 8)()
            eng._L.spg_ab_prof(pr)
            names = ["decide", "barrier1", "stage", "recur", "mark", "barrier2", "windows", "total"]
            res["sweep_clocks"] = {k: int(pr[i]) for i, k in enumerate(names)}
    res.update(reads=n, kept=int(p.n_kept), entries=int(p.n_entries), pairs=int(p.n_pairs))
print(json.dumps(res), flush=True)
