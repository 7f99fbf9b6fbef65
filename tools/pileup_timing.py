"""Host pileup phase timing (dev tool, CPU only): simulates one 10,000x SARS-CoV-2 BAM (the bench's
end-to-end input) and times AlignmentFile.pileup_plan with SPP_TIMING=1 phase prints, for the
records plan and the libdeflate / zlib host-fill plans.  Usage: python tools/pileup_timing.py [threads] [reps]"""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(bam, threads, reps, records=False):
    import spings  # noqa: F401
    from covid_spings_variant_caller_amd.pileup import AlignmentFile, PileupParams
    for _ in range(reps):
        t0 = time.perf_counter()
        with AlignmentFile(bam) as f:
            plan = f.pileup_records if records else f.pileup_plan
            b = plan("NC_045512.2", PileupParams(n_threads=threads, max_depth=0))
            t1 = time.perf_counter()
            del b
        print(f"plan {t1 - t0:.3f} s", flush=True)


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    if len(sys.argv) > 3:
        return child(sys.argv[3], threads, reps, records=len(sys.argv) > 4)
    import spings  # noqa: F401
    from covid_spings_variant_caller_amd import synth
    from covid_spings_variant_caller_amd.pileup import simulate_bam
    bam = os.path.join(tempfile.mkdtemp(), "sars_e2e.bam")
    simulate_bam(bam, "NC_045512.2", synth.reference(29903, seed=1), depth=10000, seed=5, n_threads=threads)
    print(f"BAM {os.path.getsize(bam) / 1e6:.1f} MB, cpus {len(os.sched_getaffinity(0))}", flush=True)
    for name, extra, rec in (("records (device-decode plan)", {}, ["records"]), ("libdeflate", {}, []),
                             ("zlib", {"SPP_NO_LIBDEFLATE": "1"}, [])):
        print(f"== {name}", flush=True)
        env = dict(os.environ, SPP_TIMING="1", **extra)
        subprocess.run([sys.executable, __file__, str(threads), str(reps), bam] + rec, env=env, check=True)
    os.remove(bam)


if __name__ == "__main__":
    main()
