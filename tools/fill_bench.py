"""fill_bench.py [depth] [max_depth] [reps]: the device fill of the end-to-end leg's 10,000x SARS-CoV-2 BAM — per rep
spg_bam_open + spg_bam_plan_build + spg_bam_accumulate (tweak, gather, k_f2_* fill, accumulate), each stage
synchronised and timed on the host.  Run it under rocprofv3 for the fill kernels' own times / counters.  Dev tool."""
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
max_depth = int(sys.argv[2]) if len(sys.argv) > 2 else 0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
ref = synth.reference(29903, seed=1)
bam = os.path.join(tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp")), "s.bam")
simulate_bam(bam, "NC_045512.2", ref, depth=depth, seed=5, n_threads=16)
eng = PileupEngine(29904, reference=ref)
prm = PileupParams(max_depth=max_depth)
res = {"depth": depth, "max_depth": max_depth, "open_ms": [], "plan_ms": [], "fill_acc_ms": []}
with AlignmentFile(bam) as f:
    m = f.bam_map(16)
    tid = f.tid("NC_045512.2")
    for _ in range(reps):
        eng.reset()
        eng.sync()
        t0 = time.perf_counter()
        n = eng.bam_open(m, tid, prm)
        eng.sync()
        t1 = time.perf_counter()
        p = eng.bam_plan_build(prm.max_depth, prm.ignore_overlaps)
        eng.sync()
        t2 = time.perf_counter()
        assert p is not None and eng.bam_accumulate_planned(p)
        eng.sync()
        t3 = time.perf_counter()
        for k, a, b in (("open_ms", t0, t1), ("plan_ms", t1, t2), ("fill_acc_ms", t2, t3)):
            res[k].append(round((b - a) * 1e3, 3))
    m.close()
    res.update(reads=n, kept=int(p.n_kept), entries=int(p.n_entries), pairs=int(p.n_pairs))
eng.close()
print(json.dumps(res), flush=True)
