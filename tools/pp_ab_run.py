"""pp_ab_run.py <pileup lib.so> <script.py> [args...]: run a dev script against an A/B build of libspings_pileup.so (built by
hand into _lib/ab/), by pointing the binding at it before anything loads the library.  Dev tool only."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import spings  # noqa: E402,F401
from covid_spings_variant_caller_amd import _native as N  # noqa: E402

lib = sys.argv[1]
N.PILEUP_LIB = lib if os.path.isabs(lib) else os.path.join(N.LIBDIR, "ab", lib)
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
