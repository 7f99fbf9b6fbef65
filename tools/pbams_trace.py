"""process_bams / lone process_bam timeline (dev tool): python tools/pbams_trace.py [bams] [threads] [out.json]

One simulated 10,000x SARS-CoV-2 BAM (hard-linked as N files), warm-up, then the marked windows: N lone process_bam
calls and one process_bams over the N files.  Run under `rocprofv3 --kernel-trace --memory-copy-trace` to see how
busy the GPU is inside each window (tools/pbams_gaps.py); the window marks (host perf_counter ns and the GPU clock via
a marker kernel are not needed: rocprofv3's timestamps and time.monotonic_ns share CLOCK_MONOTONIC) go to out.json."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import spings  # noqa: E402,F401


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    nt = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    out = sys.argv[3] if len(sys.argv) > 3 else None
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.live_variant_caller import LiveVariantCaller
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    L = 29903
    ref = synth.reference(L, seed=1)
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    fasta = os.path.join(d, "ref.fa")
    with open(fasta, "w") as f:
        f.write(">NC_045512.2\n" + "".join(ref[i:i + 60] + "\n" for i in range(0, L, 60)))
    bam = os.path.join(d, "s.bam")
    simulate_bam(bam, "NC_045512.2", ref, depth=10000, seed=5, n_threads=nt)
    paths = []
    for k in range(n):
        p = os.path.join(d, f"b{k}.bam")
        os.link(bam, p)
        paths.append(p)
    c = LiveVariantCaller(fasta, 30, 20, 10, 5, 0.10, 1, max_depth=0, n_threads=nt)
    for _ in range(3):
        c.process_bam(bam)
    c.process_bams(paths[:2])
    c.reset_memory()
    c.engine.sync()
    marks = {}
    t0 = time.monotonic_ns()
    for p in paths:
        c.process_bam(p)
    c.engine.sync()
    t1 = time.monotonic_ns()
    marks["lone"] = [t0, t1]
    c.reset_memory()
    c.engine.sync()
    t0 = time.monotonic_ns()
    c.process_bams(paths)
    c.engine.sync()
    t1 = time.monotonic_ns()
    marks["process_bams"] = [t0, t1]
    res = {k: {"ns": v, "ms_per_bam": (v[1] - v[0]) / 1e6 / n} for k, v in marks.items()}
    print(json.dumps(res), flush=True)
    if out:
        json.dump(res, open(out, "w"))
    c.close()


if __name__ == "__main__":
    main()
