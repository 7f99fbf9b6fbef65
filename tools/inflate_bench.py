"""GPU BGZF inflate on the end-to-end leg's 10,000x SARS-CoV-2 BAM: kernel time (HIP events) and the whole call
(H2D of the compressed file + kernel + D2H of the inflated stream), checked against gzip.  Dev tool."""
import ctypes as C
import gzip
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spings  # noqa: E402,F401
from covid_spings_variant_caller_amd import _native as N, synth  # noqa: E402
from covid_spings_variant_caller_amd.engine import pinned_empty  # noqa: E402
from covid_spings_variant_caller_amd.pileup import simulate_bam  # noqa: E402


class Member(C.Structure):
    _fields_ = [("coff", C.c_uint64), ("clen", C.c_uint32), ("ulen", C.c_uint32), ("uoff", C.c_uint64)]


depth = float(sys.argv[1]) if len(sys.argv) > 1 else 10000.0
ref = synth.reference(29903, seed=1)
bam = os.path.join(tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp")), "s.bam")
simulate_bam(bam, "NC_045512.2", ref, depth=depth, seed=5, n_threads=16)
raw = open(bam, "rb").read()
members, q, uoff = [], 0, 0
while q < len(raw):
    xlen = int.from_bytes(raw[q + 10:q + 12], "little")
    x, bsize = q + 12, None
    while x < q + 12 + xlen:
        slen = int.from_bytes(raw[x + 2:x + 4], "little")
        if raw[x] == 66 and raw[x + 1] == 67:
            bsize = int.from_bytes(raw[x + 4:x + 6], "little") + 1
        x += 4 + slen
    isize = int.from_bytes(raw[q + bsize - 4:q + bsize], "little")
    members.append(Member(q + 12 + xlen, bsize - xlen - 20, isize, uoff))
    uoff += isize
    q += bsize
n = len(members)
arr = (Member * n)(*members)
comp = pinned_empty(len(raw))
comp[:] = np.frombuffer(raw, np.uint8)
out = pinned_empty(uoff + 64)
st = np.zeros(n, np.uint32)
L = N.gpu_lib()
res = {"members": n, "compressed_mb": len(raw) / 1e6, "inflated_mb": uoff / 1e6, "runs": []}
for r in range(4):
    ms = C.c_float(0)
    t = time.perf_counter()
    rc = L.spg_bgzf_inflate(0, comp.ctypes.data, len(raw), C.addressof(arr), n, out.ctypes.data, uoff, st.ctypes.data, C.byref(ms))
    dt = time.perf_counter() - t
    assert rc == 0, L.spg_bgzf_last_error()
    fb = C.c_int64(-1)
    L.spg_bgzf_fallbacks(0, C.byref(fb))
    res["runs"].append({"kernel_ms": ms.value, "call_ms": dt * 1e3, "bad_members": int((st != 0).sum()),
                        "lane_kernel_members": fb.value})
    if hasattr(L, "spg_ab_prof"):              # (tools/src_ab.py prof build: k_inflate_par's phase clocks per member)
        pr = (C.c_uint64 * 8)()
        L.spg_ab_prof(pr)
        names = ["tables", "phase_a", "sync", "phase_b", "member", "members", "blocks"]
        res["runs"][-1]["clocks_per_member"] = {k: pr[i] / max(1, pr[5]) for i, k in enumerate(names)}
t = time.perf_counter()
ref_bytes = gzip.decompress(raw)
res["gzip_1core_ms"] = (time.perf_counter() - t) * 1e3
res["identical"] = bytes(out[:uoff]) == ref_bytes
print(json.dumps(res), flush=True)
