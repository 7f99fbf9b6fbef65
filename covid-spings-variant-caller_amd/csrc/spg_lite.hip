// spg_lite.hip — k_acc_lite: the fused calls-only accumulate + pre-check of ONE shallow batch into a fresh
// memory (process_bam once, live_variant_caller.py:54-103, then prepare_variants :120-185 at spg_finalize):
// BASELINE config 5, chr1 at 30x.
//
// prepare_variants only emits calls, and a position can produce one only if it passes the filters of
// :131 / :151-157 (totalDepth, an allele other than the REF char with AD >= minAlleleDepth and
// AD / DP >= minEvidenceRatio) — a test on counts.  So the streaming pass counts and nothing else: per
// 64-column tile one lane per column, the REF allele by SWAR popcount, every other entry into its slot's
// count.  The few columns that pass (about 0.06 % at 30x) are folded again exactly — every statistic of
// process_svn's lists, in BAM order — from the column's bytes (just read, L2-resident), their records
// written and listed for the sparse finalize.  Records of the other positions are never written (the
// context re-materializes them if anything reads them later, spg_api.cpp materialize()).
//
// Memory: each lane loads its column's bytes directly, four 16-B loads from its dword-aligned first entry
// (covers columns of <= 61 entries; longer ones finish with further loads), and the loads of the next tile
// are in flight while a tile is counted: the tile loop is unrolled twice over two register sets, so no
// register copy of a pending load forces a wait (hipcc waits for a load before copying its destination).
// Each tile's CSR bounds and REF chars are loaded two tiles ahead.
#include "spg_common.h"

namespace spg {

constexpr int LW = 4;      // waves per workgroup
constexpr int LB = 4;      // 16-B blocks per lane per tile, prefetched

struct LHead {             // loaded unconditionally (a load under a branch makes hipcc wait for every load
    uint64_t ob, oe;       // before the next use of any); `ok` selects at the first use
    uint32_t rc;           // REF char
    bool ok;               // column in range
};

__global__ __launch_bounds__(64 * LW) __attribute__((amdgpu_waves_per_eu(3, 8))) void k_acc_lite(
    MParams P, Hist hb, const uint8_t *__restrict__ ref, const Tables *__restrict__ T, Acc *__restrict__ acc) {
    __shared__ double2 lut[256];                       // {ln(1-eps), eps} per q (the exact fold only)
    for (uint32_t q = threadIdx.x; q < 256u; q += 64u * LW) lut[q] = make_double2(T->fast[q][0], T->fast[q][1]);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t n_tiles = P.n_groups;
    const int64_t stride = (int64_t)gridDim.x * LW;
    int64_t tile = (int64_t)__builtin_amdgcn_readfirstlane(blockIdx.x * LW + (threadIdx.x >> 6));   // wave-uniform

    auto head = [&](int64_t t) -> LHead {
        const int64_t p = P.u0 + t * 64 + lane;
        const int64_t col = p - hb.pos_begin;
        const bool ok = t < n_tiles && p < P.u1 && col >= 0 && col < hb.n_cols;
        const int64_t cc = min(max(col, (int64_t)0), hb.n_cols - 1);
        const int64_t pc = min(max(p, P.u0), P.u1 - 1);
        return LHead{__builtin_nontemporal_load(hb.off + cc), __builtin_nontemporal_load(hb.off + cc + 1), (uint32_t)ref[pc], ok};
    };
    // a tile's blocks: LB 16-B loads per array from the column's dword-aligned first entry.  Blocks past the
    // column (and every block of an empty or out-of-range column) reload the first one (in the batch arrays:
    // they carry 16 bytes of padding), and valid_masks drops them
    auto issue = [&](const LHead &h, u32x4 (&c)[LB], u32x4 (&q)[LB]) {
        const uint64_t ob = h.ok ? h.ob : 0, oe = h.ok ? h.oe : 0;
        const uint64_t a0 = ob & ~(uint64_t)3;
#pragma unroll
        for (int u = 0; u < LB; u++) {
            const uint64_t a = a0 + 16u * u < oe ? a0 + 16u * u : a0;
            c[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(hb.code + a));
            q[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(hb.qual + a));
        }
    };

    // one tile: counts of its columns, then the exact fold of the columns that may call
    auto process = [&](int64_t t, const LHead &h, const u32x4 (&c)[LB], const u32x4 (&q)[LB]) {
        const int64_t p = P.u0 + t * 64 + lane;
        const bool inr = h.ok;
        const uint64_t hob = inr ? h.ob : 0, hoe = inr ? h.oe : 0;
        const uint8_t refc = (uint8_t)h.rc;
        const uint32_t lx = ((uint32_t)refc & 0xDFu) - 65u;
        const uint32_t lc = lx < 16u ? (uint32_t)(0x00F0000004000201ull >> (4u * lx)) & 0xFu
                                     : (lx < 26u ? (0x8000u >> (4u * (lx - 16u))) & 0xFu : 0u);
        const uint32_t M = lc ? lc : 1u, mrep = M * 0x01010101u;   // code_of_ref, branch-free
        const int Ms = M == 15u ? 4 : (int)__builtin_ctz(M);
        uint32_t len = (uint32_t)(hoe - hob);
        bool deep = false;
        if (inr && P.t_deep && len >= P.t_deep) { deep = true; len = 0; }   // k_acc_seg<1> takes it
        const uint64_t dm = __ballot(deep);
        if (dm) {
            uint32_t at = 0;
            if (lane == 0) at = atomicAdd(P.deep_n, (uint32_t)__popcll(dm));
            at = (uint32_t)__builtin_amdgcn_readfirstlane(at);
            if (deep)
                P.deep_list[at + __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u))] =
                    (uint32_t)(p - hb.pos_begin);
        }
        const int32_t lead = (int32_t)(hob & 3u);
        uint32_t mcf = 0, drare = 0, n_other = 0, cnt[NSLOT] = {0, 0, 0, 0, 0};
        auto count = [&](const u32x4 &cw, const u32x4 &qw, int32_t x0) {
            uint32_t vm[4];
            valid_masks<4>(x0, 0, (int32_t)len, vm);
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const uint32_t c_ = dw<4>(cw, d), q_ = dw<4>(qw, d);
                uint32_t f80, r80;
                swar4(c_, q_, vm[d], mrep, P.kpass, P.kok, f80, r80);
                mcf += __popc(f80);
                while (r80) {                          // every other entry: its slot's count
                    const int sh = __builtin_ctz(r80) - 7;
                    r80 &= r80 - 1;
                    const uint32_t cc = (c_ >> sh) & 0xFFu, qq = (q_ >> sh) & 0xFFu;
                    if ((int)qq < P.min_bq) continue;
                    drare++;
                    const int s = slot_of(cc);
                    n_other += (s < 0 && cc < 16u) ? 1u : 0u;
#pragma unroll
                    for (int k = 0; k < NSLOT; k++) cnt[k] += k == s ? 1u : 0u;
                }
            }
        };
#pragma unroll
        for (int u = 0; u < LB; u++) count(c[u], q[u], 16 * u - lead);
        // columns longer than the prefetched window (rare at 30x: > 61 entries)
        const uint32_t nblk = len ? (uint32_t)(((uint32_t)lead + len + 15u) >> 4) : 0u;
        if (__ballot(nblk > LB)) {
            const uint64_t a0 = hob & ~(uint64_t)3;
            for (uint32_t u = LB;; u++) {
                const bool more = u < nblk;
                if (!__ballot(more)) break;
                u32x4 cw{0, 0, 0, 0}, qw{0, 0, 0, 0};
                if (more) {
                    cw = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(hb.code + a0) + u);
                    qw = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(hb.qual + a0) + u);
                }
                count(cw, qw, (int32_t)(16u * u) - lead);
            }
        }
        // prepare_variants' filters on the counts (:131, :151-157); an exotic allele goes to the exact replay
        const uint32_t depth = mcf + drare;
        bool mc = n_other != 0;
        if (!mc && (int64_t)depth >= (int64_t)P.min_td) {
            const double dlo = (double)depth * P.ratio_lo;
#pragma unroll
            for (int k = 0; k < NSLOT; k++) {
                const uint32_t n = cnt[k] + (k == Ms ? mcf : 0u);
                mc |= n != 0 && refc != nibble_char(slot_code(k)) && (int64_t)n >= P.min_ad && (double)n >= dlo;
            }
        }
        const bool want = inr && (deep || (len != 0 && mc));
        const uint64_t wm = __ballot(want);
        if (!wm) return;
        {
            uint32_t at = 0;                           // one list reservation per wave
            if (lane == 0) at = atomicAdd(P.n_list, (uint32_t)__popcll(wm));
            at = (uint32_t)__builtin_amdgcn_readfirstlane(at);
            if (want) P.list[at + __builtin_amdgcn_mbcnt_hi((uint32_t)(wm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wm, 0u))] = p;
        }
        if (!__ballot(want && !deep)) return;
        // ---- the exact fold of the columns that may call: process_pileup_column / process_svn (:74-103) in
        // BAM order — totalDepth, D/N/other, per allele count, sum q, q lower bound, first entry (dict order),
        // sum ln(1 - eps), sum eps — merged into an empty record (first visit :77-85)
        const bool fold = want && !deep;
        uint32_t fd = 0, fdel = 0, fskip = 0, foth = 0;
        uint32_t fc[NSLOT], fsq[NSLOT], ffirst[NSLOT], fqf[NSLOT];
        double fsl[NSLOT], fse[NSLOT];
#pragma unroll
        for (int k = 0; k < NSLOT; k++) { fc[k] = fsq[k] = 0; ffirst[k] = INF32; fqf[k] = 255; fsl[k] = fse[k] = 0.0; }
        const uint64_t a0 = hob & ~(uint64_t)3;
        const uint32_t nb = fold ? nblk : 0u;
        for (uint32_t u = 0;; u++) {
            const bool more = u < nb;
            if (!__ballot(more)) break;
            u32x4 cw{0, 0, 0, 0}, qw{0, 0, 0, 0};
            if (more) {
                cw = *(reinterpret_cast<const u32x4 *>(hb.code + a0) + u);
                qw = *(reinterpret_cast<const u32x4 *>(hb.qual + a0) + u);
            }
#pragma unroll
            for (int b = 0; b < 16; b++) {
                const int32_t x = (int32_t)(16u * u) + b - lead;          // index in the column
                const uint32_t cc = (dw<4>(cw, b >> 2) >> (8 * (b & 3))) & 0xFFu;
                const uint32_t qq = (dw<4>(qw, b >> 2) >> (8 * (b & 3))) & 0xFFu;
                if (!more || x < 0 || x >= (int32_t)len || (int)qq < P.min_bq) continue;
                fd++;
                if (cc == SPG_CODE_DEL) { fdel++; continue; }
                if (cc == SPG_CODE_SKIP) { fskip++; continue; }
                const int s = slot_of(cc);
                if (s < 0) { foth++; continue; }
                const double2 tt = lut[qq];
                const double e = qq == 0 ? 1.0 : tt.y;
#pragma unroll
                for (int k = 0; k < NSLOT; k++)
                    if (k == s) {
                        fc[k]++; fsq[k] = sat_add31(fsq[k], qq); fqf[k] = min(fqf[k], qq); ffirst[k] = min(ffirst[k], (uint32_t)x);
                        fsl[k] += tt.x; fse[k] += e;
                    }
            }
        }
        if (!fold) return;
        uint32_t newmask = 0;
        bool sums = false;
#pragma unroll
        for (int k = 0; k < NSLOT; k++) {
            newmask |= fc[k] ? (1u << k) : 0u;
            sums |= fc[k] != 0;
        }
        const uint32_t order = merge_order(0u, newmask, ffirst);
        const uint32_t misc = (uint32_t)refc | (foth ? MISC_EXOTIC : 0u);
        auto d2 = [](double x) { return __builtin_bit_cast(uint2, x); };
        uint32_t oq[NSLOT], osq[NSLOT];
        double osl[NSLOT], ose[NSLOT];
#pragma unroll
        for (int k = 0; k < NSLOT; k++) {
            oq[k] = fc[k] ? fqf[k] : 0u;
            osq[k] = fc[k] ? fsq[k] : 0u;
            osl[k] = fc[k] ? fsl[k] : 0.0;
            ose[k] = fc[k] ? fse[k] : 0.0;
        }
        uint4 *dst = reinterpret_cast<uint4 *>(acc + p);
        dst[0] = make_uint4(fd, P.seq0, order, misc);
        dst[1] = make_uint4(fdel, fskip, foth, P.epoch);
        dst[2] = make_uint4(fc[0], fc[1], fc[2], fc[3]);
        dst[3] = make_uint4(fc[4], osq[0], osq[1], osq[2]);
        dst[4] = make_uint4(osq[3], osq[4], oq[0] | (oq[1] << 8) | (oq[2] << 16) | (oq[3] << 24), oq[4]);
        if (sums) {
            dst[5] = make_uint4(d2(osl[0]).x, d2(osl[0]).y, d2(osl[1]).x, d2(osl[1]).y);
            dst[6] = make_uint4(d2(osl[2]).x, d2(osl[2]).y, d2(osl[3]).x, d2(osl[3]).y);
            dst[7] = make_uint4(d2(osl[4]).x, d2(osl[4]).y, d2(ose[0]).x, d2(ose[0]).y);
            dst[8] = make_uint4(d2(ose[1]).x, d2(ose[1]).y, d2(ose[2]).x, d2(ose[2]).y);
            dst[9] = make_uint4(d2(ose[3]).x, d2(ose[3]).y, d2(ose[4]).x, d2(ose[4]).y);
        }
    };

    // the pipeline: tile t's blocks are in set A or B (issued one tile ahead), heads two tiles ahead
    LHead h0 = head(tile), h1 = head(tile + stride);
    u32x4 cA[LB], qA[LB], cB[LB], qB[LB];
    issue(h0, cA, qA);
    while (tile < n_tiles) {
        LHead h2 = head(tile + 2 * stride);
        issue(h1, cB, qB);
        process(tile, h0, cA, qA);
        tile += stride;
        h0 = h1;
        h1 = h2;
        if (tile >= n_tiles) break;
        h2 = head(tile + 2 * stride);
        issue(h1, cA, qA);
        process(tile, h0, cB, qB);
        tile += stride;
        h0 = h1;
        h1 = h2;
    }
}

int lite_blocks_per_cu() {
    static int n = -1;
    if (n < 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_acc_lite, 64 * LW, 0) != hipSuccess || b < 1) b = 2;
        n = b;
    }
    return n;
}

// one wave per 64-column tile in grid-stride order; `blocks` workgroups (the resident grid: later
// generations of a grid-stride kernel only add a tail)
hipError_t launch_lite(const MParams &P, const Hist &hb, const uint8_t *ref, const Tables *T, Acc *acc, int64_t blocks,
                       hipStream_t st) {
    if (P.n_groups == 0) return hipSuccess;
    blocks = std::max<int64_t>(1, std::min<int64_t>(((int64_t)P.n_groups + LW - 1) / LW, blocks));
    hipLaunchKernelGGL(k_acc_lite, dim3((unsigned)blocks), dim3(64 * LW), 0, st, P, hb, ref, T, acc);
    return hipGetLastError();
}

}  // namespace spg
