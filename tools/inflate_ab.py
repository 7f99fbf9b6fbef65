"""inflate_ab.py <name> <edit>...: an A/B build of libspings_gpu.so whose spg_inflate.hip is the product source with
textual edits applied (diagnostics stay out of the product sources), the other objects shared with the in-tree build
-> _lib/ab/<name>.so; run tools/inflate_bench.py against it with tools/ab_run.py.  Edits (named):
  noresolve  k_inflate_par skips phase B (the token lists are decoded and synchronised, nothing resolved): phase A +
             sync time; the output is garbage (k_crc32 then flags every member).
Dev tool only."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "covid-spings-variant-caller_amd", "csrc")
LIB = os.path.join(ROOT, "covid-spings-variant-caller_amd", "_lib")

EDITS = {
    "noresolve": [("        for (int k = 0; k <= kend && !st; k++) {",
                   "        for (int k = 0; k <= kend && !st && kend < 0; k++) {"),
                  ("    if (!st && w != ulen) st = ST_FALLBACK;", "    if (!st) w = ulen;")],
}


def main():
    name, edits = sys.argv[1], sys.argv[2:]
    src = open(os.path.join(CSRC, "spg_inflate.hip")).read()
    for e in edits:
        for a, b in EDITS[e]:
            assert src.count(a) == 1, (e, a)
            src = src.replace(a, b)
    os.makedirs(os.path.join(LIB, "ab"), exist_ok=True)
    var = os.path.join(LIB, "ab", f"{name}_spg_inflate.hip")
    open(var, "w").write(src)
    obj = os.path.join(LIB, "ab", f"{name}.var.o")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}", "-c", var, "-o", obj])
    objs = [os.path.join(LIB, "obj", f + ".o") for f in ("spg_kernels.hip", "spg_tile.hip", "spg_lite.hip", "spg_fill.hip",
                                                         "spg_ckpt.hip", "spg_bam.hip", "spg_plan.hip", "spg_api.cpp",
                                                         "spg_multi.cpp")]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-Wl,-z,defs", "-o",
                           os.path.join(LIB, "ab", f"{name}.so"), obj] + objs + ["-lrccl"])
    print(os.path.join(LIB, "ab", f"{name}.so"))


if __name__ == "__main__":
    main()
