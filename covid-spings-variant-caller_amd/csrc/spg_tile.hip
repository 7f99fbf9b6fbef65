// spg_tile.hip — k_acc_tile: the shallow-batch accumulate (process_pileup_column / process_svn,
// live_variant_caller.py:74-103, over batches whose columns hold < ~256 entries: one BAM at 30x, runs
// of per-BAM 100x SARS-CoV-2 batches).
//
// Work decomposition.  A unit is (tile, batch): TC = 64 / LPC consecutive columns of one batch, LPC
// lanes per column.  An item is (tile, batch range): the units of one tile over consecutive batches,
// folded into per-lane register state and written once (a record, or a partial state k_merge_parts
// folds when the batch range was split).  A wave walks its items' units as one stream.
//
// Data movement.  A unit's entries are ONE contiguous byte range per array ([off[c0], off[c0 + TC])).
// The wave copies it into LDS with LDS-DMA (buffer_load_dwordx4 ... lds: 1 KiB per wave instruction,
// fully coalesced, no VGPRs), two units ahead of the one it processes, through a ring of R = 3 slots;
// the unit's CSR offsets and REF chars (its "head") are DMA'd two units further ahead.  Lane (c, sub)
// then reads its column's 16-B blocks sub, sub + LPC, ... from LDS and classifies 4 entries per dword
// with the SWAR tests of k_acc_seg: the REF allele and a promoted second allele by popcount / dot4,
// every other entry exactly (rare: sequencing errors, D/N, IUPAC).  Bytes past the slot's capacity (a
// tile far deeper than the batch mean) are read from global memory directly.
//
// The DMA slots are read with inline-asm ds_reads: hipcc cannot tell which LDS bytes an in-flight DMA
// writes, and would wait for every outstanding DMA (vmcnt(0)) before any read of the slot array.  The
// kernel waits itself: each iteration issues a fixed number of DMA instructions (dummy, zero-length ones
// past the end of the stream), so one counted s_waitcnt vmcnt(DN + HN) before a slot is read covers
// exactly the DMAs that filled it (loads hipcc issues in between only make that wait stronger).
#include <type_traits>

#include "spg_common.h"

namespace spg {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int TW = 2;                 // waves per workgroup (5 workgroups = 10 waves per CU by LDS)
constexpr int TCAP = 2048;            // bytes per array per slot
constexpr int TR = 3;                 // data slots per wave (ring)
constexpr int THR = 3;                // head slots per wave
constexpr int TNCH = TCAP / 1024;     // DMA instructions per array per unit
constexpr int TDN = 2 * TNCH;         // data DMA instructions per unit
constexpr int THN = 4;                // head DMA instructions per unit: offsets (64 + 64 + 2 dwords), REF chars
constexpr int THOFF_REF = 528;        // head slot: offsets [0, 520), REF chars [528, 592)
constexpr int THSZ = 608;
constexpr uint32_t TNBLK = TCAP / 16;

__device__ __forceinline__ uint32_t lds_off(const void *p) { return (uint32_t)(uintptr_t)(const lds_void *)p; }

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// a lane's code and qual blocks (16 B each, qual TCAP bytes after code) from a DMA slot
__device__ __forceinline__ void slot_blk(uint32_t a, u32x4 &c, u32x4 &q) {
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:%3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(c), "=&v"(q)
                 : "v"(a), "i"(TCAP)
                 : "memory");
}
// a column's CSR bounds (two u64 at a) and its REF char (at r) from a head slot
__device__ __forceinline__ void slot_head(uint32_t a, uint32_t r, uint64_t &ob, uint64_t &oe, uint32_t &rc) {
    u32x4 v;
    uint32_t b;
    asm volatile("ds_read2_b64 %0, %2 offset1:1\n\tds_read_u8 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(v), "=&v"(b)
                 : "v"(a), "v"(r)
                 : "memory");
    ob = ((uint64_t)v.y << 32) | v.x;
    oe = ((uint64_t)v.w << 32) | v.z;
    rc = b;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_u(const void *p, uint32_t n) {   // wave-uniform inputs
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(n), 0x00020000);
}

// wave-wide max (DPP within rows of 16, then the four row results): uniform result
template <int LPC>
__device__ __forceinline__ uint32_t grp_add(uint32_t v) {
#pragma unroll
    for (int o = 1; o < LPC; o <<= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}
template <int LPC>
__device__ __forceinline__ uint32_t grp_min(uint32_t v) {
#pragma unroll
    for (int o = 1; o < LPC; o <<= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
template <int LPC>
__device__ __forceinline__ uint32_t grp_sat(uint32_t v) {   // saturating sum q
#pragma unroll
    for (int o = 1; o < LPC; o <<= 1) v = sat_add31(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
template <int LPC>
__device__ __forceinline__ double grp_addf(double v) {
#pragma unroll
    for (int o = 1; o < LPC; o <<= 1) {
        const uint64_t b = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)b, o), hi = (uint32_t)__shfl_xor((int)(uint32_t)(b >> 32), o);
        v += __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
    }
    return v;
}

// One tile unit's wave-uniform bookkeeping (SGPRs) and a lane's view of it (VGPRs)
struct TUnit { int32_t g, s, k; };           // tile, batch split, batch (run-relative); s >= S: past the end
struct TLane { uint32_t b, e, rc; };          // column bytes [b, e) relative to the unit's base; rc: REF char |
                                              // 0x100 column in range | 0x200 deep (listed for k_acc_seg<1>)
struct TSeg { uint64_t wb; uint32_t nb; };    // unit's byte range base and length

template <int LPC, bool ONE>
#ifndef SPG_TILE_WPE
#define SPG_TILE_WPE 2       // waves per SIMD the register allocation must allow (2: 256 VGPRs, no spills)
#endif
__global__ __launch_bounds__(64 * TW) __attribute__((amdgpu_waves_per_eu(SPG_TILE_WPE, 8))) void k_acc_tile(MParams P, const Hist *__restrict__ H, const uint8_t *__restrict__ ref,
                                                      int64_t ref_len, const Tables *__restrict__ T, Acc *__restrict__ acc) {
    constexpr int TC = 64 / LPC;
    __shared__ double2 lut[256];                         // {ln(1-eps), eps} per q; row 0 = {0, 0}
    __shared__ __align__(16) uint8_t dslot[TW][TR][2][TCAP];
    __shared__ __align__(16) uint8_t hslot[TW][THR][THSZ];
    for (uint32_t q = threadIdx.x; q < 256u; q += 64u * TW) lut[q] = make_double2(T->fast[q][0], T->fast[q][1]);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int w = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int cl = lane / LPC, sub = lane % LPC;        // column of the tile, part of the column
    // items (tile g, split s) = s * n_groups + g, dealt round-robin to the waves: a wave's cursor steps by the
    // grid's wave count, kept as (g, s) so no 64-bit division runs per unit
    const int32_t NG = P.n_groups;
    const int32_t istride = (int32_t)gridDim.x * TW;
    const int32_t gstep = istride % NG, sstep = istride / NG;
    const int32_t item0 = (int32_t)blockIdx.x * TW + w;
    const uint32_t dslot0 = lds_off(&dslot[w][0][0][0]), hslot0 = lds_off(&hslot[w][0][0]);
    // ONE (a single-batch run): the batch descriptor is read once, not per unit
    Hist hone{};
    if constexpr (ONE) hone = H[P.h0];
    auto hist = [&](int32_t k) -> Hist {
        if constexpr (ONE) { (void)k; return hone; }
        else return H[P.h0 + k];
    };

    auto next_unit = [&](TUnit u) -> TUnit {
        if (u.s >= P.S) return u;
        if (u.k + 1 < min(P.K, u.s * P.kper + P.kper)) return TUnit{u.g, u.s, u.k + 1};
        int32_t g = u.g + gstep, s = u.s + sstep;
        if (g >= NG) { g -= NG; s++; }
        return TUnit{g, s, s * P.kper};
    };

    // ---- head DMA: the unit's CSR offsets (TC + 1 of them, from the first in-range column) and REF chars
    auto issue_head = [&](const TUnit &u, int hs) {
        uint32_t n_off = 0, n_ref = 0;
        const uint64_t *offp = nullptr;
        int64_t p0 = 0;
        if (u.s < P.S) {
            const Hist hb = hist(u.k);
            p0 = P.u0 + (int64_t)u.g * TC;
            const int64_t col0 = p0 - hb.pos_begin;
            const int64_t colA = col0 < 0 ? 0 : col0;
            if (colA < hb.n_cols) {
                offp = hb.off + colA;
                n_off = (uint32_t)min((int64_t)(TC + 1), hb.n_cols + 1 - colA) * 8u;
            }
            // (dword accesses: a 4-B DMA is either wholly in range or wholly out; the reference allocation is
            // padded by 16 bytes, so the REF range may round up to whole dwords)
            n_ref = (uint32_t)max((int64_t)0, min((int64_t)64, (ref_len - p0 + 3) & ~(int64_t)3));
        }
        const __amdgpu_buffer_rsrc_t ro = rsrc_u(offp ? (const void *)offp : (const void *)H, n_off);
        const __amdgpu_buffer_rsrc_t rr = rsrc_u(ref + (n_ref ? p0 : 0), n_ref);
        lds_void *dst = (lds_void *)&hslot[w][hs][0];
        lds_void *dstr = (lds_void *)&hslot[w][hs][THOFF_REF];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ro, dst, 4, (uint32_t)lane * 4u, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ro, dst, 4, (uint32_t)lane * 4u, 0, 256, 0);
        if (lane < 2) __builtin_amdgcn_raw_ptr_buffer_load_lds(ro, dst, 4, (uint32_t)lane * 4u, 0, 512, 0);
        if (lane < 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, dstr, 4, (uint32_t)lane * 4u, 0, 0, 0);
    };
    // ---- read a unit's head (after its DMA landed): per-lane column bounds and REF char, the byte range
    auto read_head = [&](const TUnit &u, int hs, TLane &L, TSeg &G) {
        L = TLane{0, 0, (uint32_t)'A'};
        G = TSeg{0, 0};
        uint64_t ob = 0, oe = 0;
        bool inr = false, deep = false;
        if (u.s < P.S) {
            const Hist hb = hist(u.k);
            const int64_t p0 = P.u0 + (int64_t)u.g * TC;
            const int64_t col0 = p0 - hb.pos_begin;
            const int64_t shift = col0 < 0 ? -col0 : 0;    // columns before the batch
            const int64_t col = col0 + cl;
            const int64_t p = p0 + cl;
            inr = p < P.u1;
            const bool cov = inr && col >= 0 && col < hb.n_cols;
            const uint32_t ha = hslot0 + (uint32_t)hs * THSZ + (cov ? (uint32_t)(cl - shift) * 8u : 0u);
            uint32_t rc;
            slot_head(ha, hslot0 + (uint32_t)hs * THSZ + THOFF_REF + (uint32_t)cl, ob, oe, rc);
            if (!cov) { ob = oe = 0; }
            if (inr) L.rc = rc | 0x100u;
            if (cov && P.t_deep && oe - ob >= P.t_deep) { deep = true; oe = ob; }
        }
        const uint64_t covm = __ballot(oe > ob);
        if (covm) {
            const int lf = (int)__builtin_ctzll(covm), ll = 63 - (int)__builtin_clzll(covm);
            const uint64_t a0 = ob & ~(uint64_t)15;
            const uint64_t wb = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)a0, lf) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(a0 >> 32), lf) << 32);
            const uint64_t we = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)oe, ll) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(oe >> 32), ll) << 32);
            if (we - wb >= (1ull << 30)) {             // > 2^30 entries in one tile: not a shallow batch
                if (lane == 0) atomicOr(P.err, 1u);
            } else {
                G.wb = wb;
                G.nb = (uint32_t)(we - wb);
                if (oe > ob) { L.b = (uint32_t)(ob - wb); L.e = (uint32_t)(oe - wb); }
            }
        }
        if (deep) L.rc |= 0x200u;
    };
    // ---- data DMA: the unit's byte range (up to TCAP per array) into data slot ds
    auto issue_data = [&](const TUnit &u, const TSeg &G, int ds) {
        const uint8_t *cp = nullptr, *qp = nullptr;
        uint32_t n = 0;
        if (u.s < P.S && G.nb) {
            const Hist hb = hist(u.k);
            cp = hb.code + G.wb;
            qp = hb.qual + G.wb;
            // whole 16-B blocks (the batch arrays are padded by 16 bytes past their last entry)
            n = min((G.nb + 15u) & ~15u, (uint32_t)TCAP);
        }
        const __amdgpu_buffer_rsrc_t rc = rsrc_u(cp ? (const void *)cp : (const void *)H, n);
        const __amdgpu_buffer_rsrc_t rq = rsrc_u(qp ? (const void *)qp : (const void *)H, n);
        lds_void *dc = (lds_void *)&dslot[w][ds][0][0];
        lds_void *dq = (lds_void *)&dslot[w][ds][1][0];
        static_assert(TNCH == 2, "data DMA: two 1-KiB wave instructions per array");
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, dc, 16, (uint32_t)lane * 16u, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, dc, 16, (uint32_t)lane * 16u, 0, 1024, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rq, dq, 16, (uint32_t)lane * 16u, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rq, dq, 16, (uint32_t)lane * 16u, 0, 1024, 0);
    };

    // ---- per-lane state of the current item (registers)
    uint32_t drare = 0, n_del = 0, n_skip = 0, n_other = 0, fb = INF32, sidx = 0;
    uint32_t mcf = 0, msq = 0, mfirst = INF32;          // REF allele, fast entries
    double msl = 0.0, mse = 0.0;
    int s2 = -1;                                         // second allele (first non-REF base of the column)
    bool gon = false;                                    // ... counted by SWAR once frequent
    uint32_t gcf = 0, grc = 0, gsq = 0, gfirst = INF32, gqf = 255;
    double gsl = 0.0, gse = 0.0;
    uint32_t cc[NSLOT], csq[NSLOT], cfirst[NSLOT];      // every other entry, by slot
    uint32_t cq03 = ~0u, cq4 = 255;                      // q lower bounds of slots 0-3 (bytes) and 4
    double csl[NSLOT], cse[NSLOT];
    auto qf_get = [&](int k) -> uint32_t { return k < 4 ? (cq03 >> (8 * k)) & 0xFFu : cq4; };
    auto qf_min = [&](int k, uint32_t q) {
        if (k < 4) {
            const uint32_t v = min((cq03 >> (8 * k)) & 0xFFu, q);
            cq03 = (cq03 & ~(0xFFu << (8 * k))) | (v << (8 * k));
        } else {
            cq4 = min(cq4, q);
        }
    };
    auto reset_state = [&]() {
        drare = n_del = n_skip = n_other = 0; fb = INF32; sidx = 0;
        mcf = msq = 0; mfirst = INF32; msl = mse = 0.0;
        s2 = -1; gon = false; gcf = grc = gsq = 0; gfirst = INF32; gqf = 255; gsl = gse = 0.0;
#pragma unroll
        for (int k = 0; k < NSLOT; k++) { cc[k] = csq[k] = 0; cfirst[k] = INF32; csl[k] = cse[k] = 0.0; }
        cq03 = ~0u; cq4 = 255;
    };
    reset_state();

    // ---- the pipeline (see the header): U0 is processed, U1 / U2 in flight, heads of U3 / U4 in flight
    TUnit U0{item0 % NG, item0 / NG, (item0 / NG) * P.kper};
    TUnit U1 = next_unit(U0), U2 = next_unit(U1), U3 = next_unit(U2), U4 = next_unit(U3);
    TLane L0, L1, L2;
    TSeg G0, G1, G2;
    issue_head(U0, 0);
    issue_head(U1, 1);
    issue_head(U2, 2);
    vm_wait<2 * THN>();
    read_head(U0, 0, L0, G0);
    issue_data(U0, G0, 0);
    vm_wait<THN + TDN>();
    read_head(U1, 1, L1, G1);
    issue_data(U1, G1, 1);
    issue_head(U3, 0);
    int sp = 0;                                          // data slot of U0; head slot of U2 = (sp + 2) % 3
    for (;;) {
        vm_wait<TDN + THN>();                            // U2's head and U0's data have landed
        const int s_2 = sp == 0 ? 2 : sp - 1;            // (sp + 2) % 3
        read_head(U2, s_2, L2, G2);
        issue_data(U2, G2, s_2);
        issue_head(U4, sp == 2 ? 0 : sp + 1);            // head slot (sp + 4) % 3 = (sp + 1) % 3
        if (U0.s >= P.S) break;

        // ================= process U0 =================
        const int64_t g = U0.g;
        const int32_t k0 = U0.s * P.kper, k1 = min(P.K, k0 + P.kper);
        if (U0.k == k0) {
            reset_state();
        }
        const int64_t p = P.u0 + g * TC + cl;
        const bool inr = (L0.rc & 0x100u) != 0;
        const uint8_t refc = (uint8_t)(L0.rc & 0xFFu);
        // code_of_ref / slot_of without branches: the letter's nibble code from two packed tables (A C G T N;
        // anything else reads as A, like code_of_ref), its slot from the code's lowest bit (N: 4)
        const uint32_t lx = ((uint32_t)refc & 0xDFu) - 65u;
        const uint32_t lc = lx < 16u ? (uint32_t)(0x00F0000004000201ull >> (4u * lx)) & 0xFu
                                     : (lx < 26u ? (0x8000u >> (4u * (lx - 16u))) & 0xFu : 0u);
        const uint32_t M = lc ? lc : 1u, mrep = M * 0x01010101u;
        const int Ms = M == 15u ? 4 : (int)__builtin_ctz(M);
        const bool msum = !P.calls_only || nibble_char(M) != refc;
        const bool any_msum = __ballot(msum && inr) != 0;
        const bool rsl = !msum && P.ref_sl;
        // REF sums in a shallow calls-only run: accumulated in the loop
        const bool any_rsl = __ballot(rsl && inr) != 0;
        const bool deep = (L0.rc & 0x200u) != 0;
        const uint32_t len = L0.e - L0.b;
        if (P.deep_list) {                               // long columns of a single batch: k_acc_seg<1>
            const uint64_t dm = __ballot(deep && sub == 0);
            if (dm) {
                uint32_t at = 0;
                if (lane == 0) at = atomicAdd(P.deep_n, (uint32_t)__popcll(dm));
                at = (uint32_t)__builtin_amdgcn_readfirstlane(at);
                if (deep && sub == 0)
                    P.deep_list[at + __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u))] =
                        (uint32_t)(p - hist(U0.k).pos_begin);
            }
        }
        if (len && fb == INF32) fb = (uint32_t)U0.k;      // run-relative batch index (seq0 + fb)
        // second allele: SWAR once it holds >= 4 entries
        if (!gon && s2 >= 0 && gcf + grc >= 4u) gon = true;
        const uint32_t mrep2 = gon ? slot_code(s2) * 0x01010101u : 0x7F7F7F7Fu;
        const bool any_gon = __ballot(gon) != 0;
        uint32_t lsq = 0, lgsq = 0;
        const uint32_t cbase = dslot0 + (uint32_t)sp * (2 * TCAP);
        // the REF allele's LUT sums: non-REF major (msum) or a shallow calls-only run's REF (rsl)
        const bool msl_on = msum || rsl;
        // One 16-B block of the lane's column: SWAR classes of its four dwords (REF allele; the second allele
        // when DUAL), counts / sum(q) / LUT sums; the first-entry and exact paths run only for lanes that need
        // them (divergent branches taken once per block, not per dword).  SUMS / DUAL: wave-uniform, hoisted.
        auto classify = [&](auto sums_tag, auto dual_tag, const u32x4 &cw, const u32x4 &qw, int32_t x0, int32_t vlen) {
            constexpr bool SUMS = decltype(sums_tag)::value, DUAL = decltype(dual_tag)::value;
            uint32_t vm[4];
            valid_masks<4>(x0, 0, vlen, vm);
            uint32_t fany = 0, gany = 0;
            auto classes = [&](int d, uint32_t &f80, uint32_t &g80, uint32_t &r80, bool again) {
                uint32_t c_ = dw<4>(cw, d), q_ = dw<4>(qw, d);
                if (again) asm volatile("" : "+v"(c_), "+v"(q_));   // a recomputation, not a value kept live
                swar4(c_, q_, vm[d], mrep, P.kpass, P.kok, f80, r80);
                g80 = 0;
                if constexpr (DUAL) {
                    uint32_t r2;
                    swar4(c_, q_, vm[d], mrep2, P.kpass, P.kok, g80, r2);
                    r80 &= ~g80;
                }
            };
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const uint32_t c_ = dw<4>(cw, d), q_ = dw<4>(qw, d);
                uint32_t f80, g80, r80;
                classes(d, f80, g80, r80, false);
                mcf += __popc(f80);
                lsq = __builtin_amdgcn_udot4(q_, f80 >> 7, lsq, false);
                // (each dword's four LUT rows are read and summed before the next dword's: hipcc would otherwise
                // hoist every lookup of the block, 16 B each, and spill)
                if constexpr (SUMS) {
                    lut_sums(q_, msl_on ? f80 : 0u, lut, msl, mse);
                    asm volatile("" : "+v"(msl), "+v"(mse)::"memory");
                }
                if constexpr (DUAL) {
                    gcf += __popc(g80);
                    lgsq = __builtin_amdgcn_udot4(q_, g80 >> 7, lgsq, false);
                    lut_sums(q_, g80, lut, gsl, gse);
                    asm volatile("" : "+v"(gsl), "+v"(gse)::"memory");
                }
                fany |= f80; gany |= g80;
                while (r80) {                            // every other entry, exactly
                    const int sh = __builtin_ctz(r80) - 7;
                    r80 &= r80 - 1;
                    const uint32_t c = (c_ >> sh) & 0xFFu, q = (q_ >> sh) & 0xFFu;
                    if ((int)q < P.min_bq) continue;
                    const uint32_t idx = sidx + (uint32_t)(x0 + 4 * d + (sh >> 3));
                    drare++;
                    if (c == SPG_CODE_DEL) { n_del++; continue; }
                    if (c == SPG_CODE_SKIP) { n_skip++; continue; }
                    const int s = slot_of(c);
                    if (s < 0) { n_other++; continue; }
                    const double2 t = lut[q];
                    const double e = q == 0 ? 1.0 : t.y;
                    if (s != Ms && (s == s2 || s2 < 0)) {
                        s2 = s;
                        grc++; gsq += q; gqf = min(gqf, q); gfirst = min(gfirst, idx); gsl += t.x; gse += e;
                    } else {
#pragma unroll
                        for (int kk = 0; kk < NSLOT; kk++)
                            if (kk == s) {
                                cc[kk]++; csq[kk] += q; qf_min(kk, q); cfirst[kk] = min(cfirst[kk], idx);
                                csl[kk] += t.x; cse[kk] += e;
                            }
                    }
                }
            }
            // first fast entries (dict order): recomputed for the lanes that have none yet (a column's first blocks)
            if ((mfirst == INF32 && fany) || (DUAL && gfirst == INF32 && gany)) {
#pragma unroll
                for (int d = 3; d >= 0; d--) {
                    uint32_t f80, g80, r80;
                    classes(d, f80, g80, r80, true);
                    if (f80 && mfirst == INF32 && fany) fany = 0x100u | ((uint32_t)(4 * d) + ((uint32_t)__builtin_ctz(f80) >> 3));
                    if (DUAL && g80 && gfirst == INF32 && gany) gany = 0x100u | ((uint32_t)(4 * d) + ((uint32_t)__builtin_ctz(g80) >> 3));
                }
                if (mfirst == INF32 && fany) mfirst = sidx + (uint32_t)x0 + (fany & 0xFFu);
                if (DUAL && gfirst == INF32 && gany) gfirst = sidx + (uint32_t)x0 + (gany & 0xFFu);
            }
        };
        // blocks sub, sub + LPC, ... of the column: from the slot, then (a tile deeper than the slot) from memory
        const uint32_t j0 = L0.b >> 4, j1 = len ? (L0.e + 15u) >> 4 : j0;
        const uint32_t jl = min(j1, TNBLK);
        const uint32_t nl = jl > j0 + (uint32_t)sub ? (jl - j0 - (uint32_t)sub + LPC - 1) / LPC : 0u;
        const uint32_t mx = wave_max_u32(nl);
        const int32_t vlen_l = (int32_t)min(len, TCAP - min(L0.b, (uint32_t)TCAP));   // entries of the column in the slot
        const bool ovf = j1 > TNBLK;
        const bool any_ovf = __ballot(ovf) != 0;
        auto run = [&](auto sums_tag, auto dual_tag) {
            for (uint32_t t = 0; t < mx; t++) {
                const uint32_t blk = j0 + (uint32_t)sub + LPC * t;
                u32x4 cw, qw;
                slot_blk(cbase + 16u * min(blk, TNBLK - 1u), cw, qw);
                classify(sums_tag, dual_tag, cw, qw, (int32_t)(16u * blk) - (int32_t)L0.b, vlen_l);
            }
            if (any_ovf) {                               // the part past the slot: direct loads (rare)
                const Hist hb = hist(U0.k);
                const __amdgpu_buffer_rsrc_t oc = rsrc_u(hb.code + G0.wb, (G0.nb + 15u) & ~15u);
                const __amdgpu_buffer_rsrc_t oq = rsrc_u(hb.qual + G0.wb, (G0.nb + 15u) & ~15u);
                const uint32_t b0 = max(j0 + (uint32_t)sub, TNBLK);
                // first block of this lane's stride at or past TNBLK
                const uint32_t f0 = j0 + (uint32_t)sub + ((b0 - (j0 + (uint32_t)sub) + LPC - 1) / LPC) * LPC;
                const uint32_t no = ovf && j1 > f0 ? (j1 - f0 + LPC - 1) / LPC : 0u;
                const uint32_t mo = wave_max_u32(no);
                for (uint32_t t = 0; t < mo; t++) {
                    const uint32_t blk = f0 + LPC * t;
                    const uint32_t o = t < no ? 16u * blk : 0x80000000u;
                    const u32x4 cw = __builtin_amdgcn_raw_buffer_load_b128(oc, (int)o, 0, 0);
                    const u32x4 qw = __builtin_amdgcn_raw_buffer_load_b128(oq, (int)o, 0, 0);
                    classify(sums_tag, dual_tag, cw, qw, (int32_t)(16u * blk) - (int32_t)L0.b, (int32_t)len);
                }
            }
        };
        using T_ = std::true_type;
        using F_ = std::false_type;
        {
            const bool any_sums = any_msum || any_rsl;
            if (any_gon) { if (any_sums) run(T_{}, T_{}); else run(F_{}, T_{}); }
            else { if (any_sums) run(T_{}, F_{}); else run(F_{}, F_{}); }
        }
        msq = sat_add31(msq, lsq);                       // (dot4 against 0x01 bytes: plain sums of q)
        gsq = sat_add31(gsq, lgsq);
        sidx += len;

        const bool item_end = U0.k + 1 == k1;
        const uint32_t depth = grp_add<LPC>(mcf + gcf + drare);
        const uint32_t mcf_c = grp_add<LPC>(mcf);
        const uint32_t no_ = grp_add<LPC>(n_other);
        if (item_end) {
            // ================= item end: fold the allele states into per-slot arrays =================
            const uint32_t nd = grp_add<LPC>(n_del), ns = grp_add<LPC>(n_skip);
#pragma unroll
            for (int kk = 0; kk < NSLOT; kk++) {
                if (kk == Ms) {
                    cc[kk] += mcf; csq[kk] = sat_add31(csq[kk], msq); cfirst[kk] = min(cfirst[kk], mfirst);
                    if (mcf) qf_min(kk, (uint32_t)P.qlo);
                    csl[kk] += msl; cse[kk] += mse;
                }
                if (kk == s2) {
                    cc[kk] += gcf + grc; csq[kk] = sat_add31(csq[kk], gsq); cfirst[kk] = min(cfirst[kk], gfirst);
                    qf_min(kk, gcf ? min(gqf, (uint32_t)P.qlo) : gqf);
                    csl[kk] += gsl; cse[kk] += gse;
                }
            }
            if constexpr (LPC > 1) {
#pragma unroll
                for (int o = 1; o < LPC; o <<= 1) {      // per-byte min of the packed q bounds
                    const uint32_t x = (uint32_t)__shfl_xor((int)cq03, o);
                    uint32_t r = 0;
#pragma unroll
                    for (int kk = 0; kk < 4; kk++) r |= min((cq03 >> (8 * kk)) & 0xFFu, (x >> (8 * kk)) & 0xFFu) << (8 * kk);
                    cq03 = r;
                    cq4 = min(cq4, (uint32_t)__shfl_xor((int)cq4, o));
                }
#pragma unroll
                for (int kk = 0; kk < NSLOT; kk++) {
                    cc[kk] = grp_add<LPC>(cc[kk]); csq[kk] = grp_sat<LPC>(csq[kk]); cfirst[kk] = grp_min<LPC>(cfirst[kk]);
                    csl[kk] = grp_addf<LPC>(csl[kk]); cse[kk] = grp_addf<LPC>(cse[kk]);
                }
            }
            // calls-only: a REF-char major's sums were not accumulated (never a call), except in shallow runs
            // (P.ref_sl: both sums, so a reference switch cannot leave a candidate without its QUAL)
            const uint32_t skip = (!msum && !P.ref_sl && mcf_c > 0) ? (1u << Ms) : 0u;
            const uint32_t fbi = fb;                     // (the next item's first unit resets the state)
            auto d2 = [](double x) { return __builtin_bit_cast(uint2, x); };
            if (P.S > 1 || !P.fresh) {
                // partial state of this batch range (the 176-B MState image) -> k_merge_parts, which folds the
                // splits in order and merges them into the records (reading the old record when not fresh)
                if (inr && sub == 0) {
                    const int32_t s = U0.s;
                    uint4 *dst = reinterpret_cast<uint4 *>(P.part + (int64_t)s * P.pstride + (p - P.u0));
                    dst[0] = make_uint4(depth, nd, ns, no_);
                    dst[1] = make_uint4(cc[0], cc[1], cc[2], cc[3]);
                    dst[2] = make_uint4(cc[4], csq[0], csq[1], csq[2]);
                    dst[3] = make_uint4(csq[3], csq[4], cfirst[0], cfirst[1]);
                    dst[4] = make_uint4(cfirst[2], cfirst[3], cfirst[4], fbi);
                    dst[5] = make_uint4(cq03, cq4 | (skip << 8), 0u, 0u);
                    dst[6] = make_uint4(d2(csl[0]).x, d2(csl[0]).y, d2(csl[1]).x, d2(csl[1]).y);
                    dst[7] = make_uint4(d2(csl[2]).x, d2(csl[2]).y, d2(csl[3]).x, d2(csl[3]).y);
                    dst[8] = make_uint4(d2(csl[4]).x, d2(csl[4]).y, d2(cse[0]).x, d2(cse[0]).y);
                    dst[9] = make_uint4(d2(cse[1]).x, d2(cse[1]).y, d2(cse[2]).x, d2(cse[2]).y);
                    dst[10] = make_uint4(d2(cse[3]).x, d2(cse[3]).y, d2(cse[4]).x, d2(cse[4]).y);
                }
            } else {
                // a FRESH unsplit run: the record is this item's state (merge_state into an empty record),
                // composed straight from the per-slot arrays.  (every lane of a column holds the column's totals:
                // they agree on want / write)
                bool write = inr && !deep && fbi != INF32;
                if (write && sub == 0) {
                    // merge_state into an empty record of this epoch: first visit (:77-85), totalDepth (:87), the
                    // slots present with their sums, dict order by first entry (:100-101); absent slots stay 0
                    uint32_t newmask = 0, ocnt[NSLOT], osq[NSLOT], oqf[NSLOT];
                    double osl[NSLOT], ose[NSLOT];
                    bool sums = false;
#pragma unroll
                    for (int kk = 0; kk < NSLOT; kk++) {
                        const bool h = cc[kk] != 0;
                        newmask |= h ? (1u << kk) : 0u;
                        ocnt[kk] = cc[kk];
                        osq[kk] = h ? min(csq[kk], 0x80000000u) : 0u;
                        oqf[kk] = h ? qf_get(kk) : 0u;
                        osl[kk] = h ? csl[kk] : 0.0;
                        ose[kk] = h ? cse[kk] : 0.0;
                        sums |= h && !((skip >> kk) & 1u);
                    }
                    const uint32_t order = merge_order(0u, newmask, cfirst);
                    const uint32_t misc = (uint32_t)refc | (no_ ? MISC_EXOTIC : 0u) | (skip << MISC_SKIP_SHIFT);
                    uint4 *dst = reinterpret_cast<uint4 *>(acc + p);
                    dst[0] = make_uint4(depth, P.seq0 + fbi, order, misc);
                    dst[1] = make_uint4(nd, ns, no_, P.epoch);
                    dst[2] = make_uint4(ocnt[0], ocnt[1], ocnt[2], ocnt[3]);
                    dst[3] = make_uint4(ocnt[4], osq[0], osq[1], osq[2]);
                    dst[4] = make_uint4(osq[3], osq[4], oqf[0] | (oqf[1] << 8) | (oqf[2] << 16) | (oqf[3] << 24), oqf[4]);
                    if (sums) {
                        dst[5] = make_uint4(d2(osl[0]).x, d2(osl[0]).y, d2(osl[1]).x, d2(osl[1]).y);
                        dst[6] = make_uint4(d2(osl[2]).x, d2(osl[2]).y, d2(osl[3]).x, d2(osl[3]).y);
                        dst[7] = make_uint4(d2(osl[4]).x, d2(osl[4]).y, d2(ose[0]).x, d2(ose[0]).y);
                        dst[8] = make_uint4(d2(ose[1]).x, d2(ose[1]).y, d2(ose[2]).x, d2(ose[2]).y);
                        dst[9] = make_uint4(d2(ose[3]).x, d2(ose[3]).y, d2(ose[4]).x, d2(ose[4]).y);
                    }
                }
            }
        }
        // ---- advance the pipeline
        U0 = U1; U1 = U2; U2 = U3; U3 = U4; U4 = next_unit(U4);
        L0 = L1; L1 = L2; G0 = G1; G1 = G2;
        sp = sp == 2 ? 0 : sp + 1;
    }
    vm_wait<0>();                                        // no DMA may land in LDS after the wave ends
}

// Resident workgroups per CU of a k_acc_tile instantiation (the occupancy API; the grid never exceeds what is
// resident, or the waves of a second generation would start after the first has streamed its units)
static const void *tile_fn(int lpc, bool one) {
#define SPG_TF(L) (one ? (const void *)k_acc_tile<L, true> : (const void *)k_acc_tile<L, false>)
    switch (lpc) {
        case 1: return SPG_TF(1);
        case 2: return SPG_TF(2);
        case 4: return SPG_TF(4);
        case 8: return SPG_TF(8);
        default: return nullptr;
    }
#undef SPG_TF
}

int tile_blocks_per_cu(int lpc, bool one) {
    static int cache[2][9] = {};
    int &c = cache[one ? 1 : 0][lpc];
    if (c) return c;
    int n = 0;
    const void *f = tile_fn(lpc, one);
    if (!f || hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 64 * TW, 0) != hipSuccess || n <= 0) n = 4;
    return c = n;
}

hipError_t launch_tile(const MParams &P, const Hist *H, const uint8_t *ref, int64_t ref_len, const Tables *T, Acc *acc,
                       int lpc, int64_t max_blocks, hipStream_t st) {
    const int64_t items = (int64_t)P.n_groups * P.S;
    if (items == 0) return hipSuccess;
    if (items >= (1ll << 31)) return hipErrorInvalidValue;     // the kernel's item cursor is 32-bit
    const int64_t blocks = std::min<int64_t>((items + TW - 1) / TW, max_blocks);
#define SPG_TILE(L)                                                                                                  \
    do {                                                                                                             \
        const dim3 g_((unsigned)blocks), b_(64 * TW);                                                                \
        if (one) hipLaunchKernelGGL((k_acc_tile<L, true>), g_, b_, 0, st, P, H, ref, ref_len, T, acc);               \
        else hipLaunchKernelGGL((k_acc_tile<L, false>), g_, b_, 0, st, P, H, ref, ref_len, T, acc);                  \
    } while (0)
    const bool one = P.K == 1;
    switch (lpc) {
        case 1: SPG_TILE(1); break;
        case 2: SPG_TILE(2); break;
        case 4: SPG_TILE(4); break;
        case 8: SPG_TILE(8); break;
        default: return hipErrorInvalidValue;
    }
#undef SPG_TILE
    return hipGetLastError();
}

}  // namespace spg
