"""inflate_ab.py <name> <edit>...: an A/B build of libspings_gpu.so whose source (spg_inflate.hip, or the edit's own) is
the product source with textual edits applied (diagnostics stay out of the product sources), the other objects shared
with the in-tree build -> _lib/ab/<name>.so; run a dev script (tools/inflate_bench.py, tools/plan_bench.py) against it
with tools/ab_run.py.  Edits (named):
  noresolve  k_inflate_par skips phase B (the token lists are decoded and synchronised, nothing resolved): phase A +
             sync time; the output is garbage (k_crc32 then flags every member).
  sweep_nok  (spg_plan.hip) the depth-cap sweep skips its k recurrence (k = n): its cost; the plan is wrong.
  sweep_noatom (spg_plan.hip) the sweep marks reads but adds no ends to the ring: the atomics' cost; the plan is wrong.
  prof       k_inflate_par's phases timed with the shader clock (spg_ab_prof; tools/inflate_bench.py reports them).
  sweep_prof (spg_plan.hip) the depth-cap sweep's phases timed with the shader clock by thread 0 (spg_ab_prof;
             tools/plan_bench.py reports them).
Dev tool only."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "covid-spings-variant-caller_amd", "csrc")
LIB = os.path.join(ROOT, "covid-spings-variant-caller_amd", "_lib")

SRC_OF = {"sweep_nok": "spg_plan.hip", "sweep_noatom": "spg_plan.hip", "sweep_prof": "spg_plan.hip"}
PROF_EXPORT = """
extern "C" int spg_ab_prof(uint64_t *out8) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(spg::g_ab_prof), 8 * sizeof(uint64_t)) != hipSuccess) return -1;
    static const uint64_t zero[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(spg::g_ab_prof), zero, sizeof zero) == hipSuccess ? 0 : -1;
}
"""
EDITS = {
    # k_inflate_par's phases timed with the shader clock (summed over members, lane 0): [0] block tables, [1] phase A,
    # [2] sync rounds, [3] phase B (resolve), [4] whole member, [5] members, [6] blocks
    "prof": [("__device__ __forceinline__ uint32_t ring_slot(uint32_t g0, uint32_t x) {",
              "__device__ unsigned long long g_ab_prof[8];\n"
              "__device__ __forceinline__ uint32_t ring_slot(uint32_t g0, uint32_t x) {"),
             ("    uint32_t w = 0, flushed = 0, p = pay0, st = 0;",
              "    uint32_t w = 0, flushed = 0, p = pay0, st = 0;\n    const uint64_t tp0 = clock64();"),
             ("        const uint32_t hs = block_tables<true>(B, slice, type, fixed_built);",
              "        const uint64_t t_a = clock64();\n        const uint32_t hs = block_tables<true>(B, slice, type, fixed_built);"),
             ("        if (hs != 0) { st = ST_FALLBACK; break; }",
              "        if (hs != 0) { st = ST_FALLBACK; break; }\n        const uint64_t t_b = clock64();\n"
              "        if (lane == 0) { atomicAdd(&g_ab_prof[0], t_b - t_a); atomicAdd(&g_ab_prof[6], 1ull); }"),
             ("        __builtin_amdgcn_wave_barrier();\n        // sync rounds",
              "        const uint64_t t_c = clock64();\n        if (lane == 0) atomicAdd(&g_ab_prof[1], t_c - t_b);\n"
              "        __builtin_amdgcn_wave_barrier();\n        // sync rounds"),
             ("        const bool bad = (uint32_t)lane < K && (so.ovf || sy.fail);",
              "        const uint64_t t_d = clock64();\n        if (lane == 0) atomicAdd(&g_ab_prof[2], t_d - t_c);\n"
              "        const bool bad = (uint32_t)lane < K && (so.ovf || sy.fail);"),
             ("        if (st) break;\n        p = pnext;",
              "        if (st) break;\n        if (lane == 0) atomicAdd(&g_ab_prof[3], clock64() - t_d);\n        p = pnext;"),
             ("    if (!st) flush(ulen);\n",
              "    if (!st) flush(ulen);\n    if (lane == 0) { atomicAdd(&g_ab_prof[4], clock64() - tp0); atomicAdd(&g_ab_prof[5], 1ull); }\n"),
             ("}  // namespace spg\n\n// ---", "}  // namespace spg\n" + "@@EXPORT@@" + "\n// ---")],
    "sweep_nok": [("            if ((int64_t)alive + wave_sum32(na + nb) > (int64_t)M) {",
                   "            if ((int64_t)alive + wave_sum32(na + nb) > (int64_t)M && M < 0) {")],
    "sweep_noatom": [("                    atomicAdd(&ring[key], nxt - lane);",
                      "                    if (nxt < 0) atomicAdd(&ring[key], nxt - lane);")],
    # the sweep's phases (thread 0's shader clock, summed over windows): [0] wave 0's decision, [1] the barrier after
    # it, [2] staging, [3] the k recurrence, [4] thread 0's marking, [5] the window's closing barrier, [6] windows,
    # [7] the whole kernel
    "sweep_prof": [("namespace spg {\n\nnamespace {", "namespace spg {\n__device__ unsigned long long g_ab_prof[8];\nnamespace {"),
                   ("    while (d < D) {\n        if (d + SWEEP_W + 1 > blk1 && blk1 < D + 1) {",
                    "    const uint64_t tq0 = clock64();\n    while (d < D) {\n        const uint64_t t_top = clock64();\n"
                    "        if (d + SWEEP_W + 1 > blk1 && blk1 < D + 1) {"),
                   ("            lds_barrier();\n        }\n        if (tid < 64) {",
                    "            lds_barrier();\n        }\n        const uint64_t t_st = clock64();\n"
                    "        if (tid == 0) atomicAdd(&g_ab_prof[2], t_st - t_top);\n        if (tid < 64) {"),
                   ("                const int32_t base = __builtin_amdgcn_readfirstlane(alive);\n                if (M <",
                    "                const uint64_t t_r0 = clock64();\n"
                    "                const int32_t base = __builtin_amdgcn_readfirstlane(alive);\n                if (M <"),
                   ("                    kb = (int32_t)scum[64 + lane] - (int32_t)scum[63 + lane];",
                    "                    kb = (int32_t)scum[64 + lane] - (int32_t)scum[63 + lane];\n"
                    "                    if (tid == 0) atomicAdd(&g_ab_prof[3], clock64() - t_r0);"),
                   ("        lds_barrier();\n        // the kept reads",
                    "        const uint64_t t_dec = clock64();\n        if (tid == 0) atomicAdd(&g_ab_prof[0], t_dec - t_st);\n"
                    "        lds_barrier();\n        const uint64_t t_b1 = clock64();\n"
                    "        if (tid == 0) atomicAdd(&g_ab_prof[1], t_b1 - t_dec);\n        // the kept reads"),
                   ("        d = s_next;\n        lds_barrier();\n    }",
                    "        const uint64_t t_mk = clock64();\n        if (tid == 0) atomicAdd(&g_ab_prof[4], t_mk - t_b1);\n"
                    "        d = s_next;\n        lds_barrier();\n"
                    "        if (tid == 0) { atomicAdd(&g_ab_prof[5], clock64() - t_mk); atomicAdd(&g_ab_prof[6], 1ull); }\n    }\n"
                    "    if (tid == 0) atomicAdd(&g_ab_prof[7], clock64() - tq0);"),
                   ("}  // namespace spg\n", "}  // namespace spg\n" + "@@EXPORT@@")],
    # phase B's batches and tokens (summed over members): [0] batches, [1] tokens, [2] output bytes, [5] members
    "prof_batches": [("__device__ __forceinline__ uint32_t ring_slot(uint32_t g0, uint32_t x) {",
                      "__device__ unsigned long long g_ab_prof[8];\n"
                      "__device__ __forceinline__ uint32_t ring_slot(uint32_t g0, uint32_t x) {"),
                     ("                const uint32_t sb = o - dist;                                            // a match's source start",
                      "                const uint32_t sb = o - dist;                                            // a match's source start\n"
                      "                if (lane == 0) { atomicAdd(&g_ab_prof[0], 1ull); atomicAdd(&g_ab_prof[1], (unsigned long long)nb);"
                      " atomicAdd(&g_ab_prof[2], (unsigned long long)total); }"),
                     ("    if (!st) flush(ulen);\n", "    if (!st) flush(ulen);\n    if (lane == 0) atomicAdd(&g_ab_prof[5], 1ull);\n"),
                     ("}  // namespace spg\n\n// ---", "}  // namespace spg\n" + "@@EXPORT@@" + "\n// ---")],
    "noresolve": [("        for (int k = 0; k <= kend && !st; k++) {",
                   "        for (int k = 0; k <= kend && !st && kend < 0; k++) {"),
                  ("    if (!st && w != ulen) st = ST_FALLBACK;", "    if (!st) w = ulen;")],
}


def main():
    name, edits = sys.argv[1], sys.argv[2:]
    srcname = SRC_OF.get(edits[0], "spg_inflate.hip") if edits else "spg_inflate.hip"
    src = open(os.path.join(CSRC, srcname)).read()
    for e in edits:
        for a, b in EDITS[e]:
            assert src.count(a) == 1, (e, a)
            src = src.replace(a, b.replace("@@EXPORT@@", PROF_EXPORT))
    os.makedirs(os.path.join(LIB, "ab"), exist_ok=True)
    var = os.path.join(LIB, "ab", f"{name}_{srcname}")
    open(var, "w").write(src)
    obj = os.path.join(LIB, "ab", f"{name}.var.o")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}", "-c", var, "-o", obj])
    objs = [os.path.join(LIB, "obj", f + ".o") for f in ("spg_kernels.hip", "spg_tile.hip", "spg_lite.hip", "spg_fill.hip",
                                                         "spg_inflate.hip", "spg_ckpt.hip", "spg_bam.hip", "spg_plan.hip",
                                                         "spg_api.cpp", "spg_multi.cpp") if f != srcname]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-Wl,-z,defs", "-o",
                           os.path.join(LIB, "ab", f"{name}.so"), obj] + objs + ["-lrccl"])
    print(os.path.join(LIB, "ab", f"{name}.so"))


if __name__ == "__main__":
    main()
