"""Host timing of spp_pileup_plan_fields at 10,000x (dev tool, CPU only): python tools/plan_fields_bench.py [threads] [reps]

Synthetic fixed fields of 2.0 M unpaired 150-bp reads over SARS-CoV-2 (as spg_bam_reads_copy returns them for the
simulator's BAM: no mate pairs), planned `reps` times; SPP_TIMING=1 prints the stages."""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import spings  # noqa: E402,F401
import samgen  # noqa: E402
from covid_spings_variant_caller_amd import _native as N  # noqa: E402
from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams  # noqa: E402

nt = int(sys.argv[1]) if len(sys.argv) > 1 else 16
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
L, n = 29903, 1993533
d = tempfile.mkdtemp()
bam = os.path.join(d, "h.bam")
samgen.write_bam(bam, [("NC_045512.2", L)], [])
rng = np.random.default_rng(1)
pos = np.sort(rng.integers(0, L - 150, n)).astype(np.int32)
reads = {"pos": pos, "end": (pos + 150).astype(np.int32), "mtid": np.full(n, -1, np.int32), "mpos": np.full(n, -1, np.int32),
         "isize": np.zeros(n, np.int32), "flag": np.zeros(n, np.uint16), "l_seq": np.full(n, 150, np.uint32),
         "name_hash": rng.integers(0, 2**63, n).astype(np.uint64)}
for name, dt in N.BAM_READ_FIELDS:
    reads[name] = np.ascontiguousarray(reads[name], dtype=dt)
ts = []
with AlignmentFile(bam) as f:
    for _ in range(reps):
        t0 = time.perf_counter()
        b = f.pileup_fields("NC_045512.2", reads, PileupParams(n_threads=nt, max_depth=0))
        ts.append((time.perf_counter() - t0) * 1e3)
        b.close()
print("plan_fields ms:", [round(t, 2) for t in ts], "median %.2f" % float(np.median(ts)))
