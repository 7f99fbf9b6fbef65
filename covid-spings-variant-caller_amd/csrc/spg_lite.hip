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
// Memory: a tile's bytes [off[c0], off[c0 + 64]) are contiguous in base_code / qual; the wave loads them coalesced
// (16 B per lane, three 1 KiB chunks per array from the 16-B aligned start) into registers one tile ahead, stores
// them into its LDS slot when the tile comes up, and each lane reads its column's aligned blocks from there
// (bytes past the 3 KiB slot — a tile with a column >= 128 entries, or a rare 100x+ stretch — from global
// memory).  The tile loop is unrolled twice over two register sets, so no register copy of a pending load
// forces a wait (hipcc waits for a load before copying its destination).  CSR bounds and REF chars are loaded
// two tiles ahead.
#include "spg_common.h"

namespace spg {

constexpr int LW = 4;      // waves per workgroup
constexpr int LCH = 3;     // 1 KiB chunks per array staged per tile
constexpr int LSLOT = 1024 * LCH;   // bytes per array in a wave's LDS slot
constexpr int LNBLK = LSLOT / 16;

// One tile in flight, loaded unconditionally (a load under a branch makes hipcc wait for every load before the
// next use of any): its staged chunks (lane l: bytes 1024 k + 16 l from the tile's 16-B aligned start, per
// array) and the lane's column bounds and REF char.  Two of them alternate (no register copies: hipcc waits
// for a pending load before copying its destination).
struct LData {
    u32x4 c[LCH], q[LCH];
    uint64_t base;         // the tile's 16-B aligned start (resolved at issue)
};
struct LHead {             // the lane's column bounds and REF char (its own ping-pong pair, one tile ahead); the
    uint32_t ob, oe;       // bounds' low halves only (a loaded dword nothing reads lets hipcc reuse its register,
    uint32_t rc;           // which costs a full wait; tile-relative offsets need no more)
};
struct LBounds {           // a tile's byte range [off[c0], off[c0 + 64]) (wave-uniform)
    uint64_t b, e;
};

__global__ __launch_bounds__(64 * LW) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_acc_lite(
    MParams P, Hist hb, const uint8_t *__restrict__ ref, const Tables *__restrict__ T, Acc *__restrict__ acc) {
    __shared__ double2 lut[256];                       // {ln(1-eps), eps} per q (the exact fold only)
    __shared__ __attribute__((aligned(16))) uint8_t slots[LW][2][LSLOT];   // per wave: a tile's code, qual
    for (uint32_t q = threadIdx.x; q < 256u; q += 64u * LW) lut[q] = make_double2(T->fast[q][0], T->fast[q][1]);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t n_tiles = P.n_groups;
    const int64_t stride = (int64_t)gridDim.x * LW;
    int64_t tile = (int64_t)__builtin_amdgcn_readfirstlane(blockIdx.x * LW + (threadIdx.x >> 6));   // wave-uniform

    auto bounds = [&](int64_t t) -> LBounds {
        const int64_t c0 = min(max(P.u0 + t * 64 - hb.pos_begin, (int64_t)0), hb.n_cols);
        const int64_t c1 = min(c0 + 64, hb.n_cols);
        return LBounds{hb.off[c0], hb.off[c1]};
    };
    auto in_range = [&](int64_t t) {
        const int64_t p = P.u0 + t * 64 + lane, col = p - hb.pos_begin;
        return t < n_tiles && p < P.u1 && col >= 0 && col < hb.n_cols;
    };
    // LCH coalesced 16-B loads per lane and array; lanes past the tile's bytes (and a tile past the end) reload
    // the first chunk's line (in the batch arrays: they carry 16 bytes of padding)
    auto issue = [&](int64_t t, const LBounds &B, LData &D) {
        const uint64_t base = B.b & ~(uint64_t)15;
        const uint64_t span = t < n_tiles ? B.e - base : 0;
#pragma unroll
        for (int k = 0; k < LCH; k++) {
            const uint32_t o = 1024u * k + 16u * lane;
            const uint64_t a = o < span ? base + o : base;
            D.c[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(hb.code + a));
            D.q[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(hb.qual + a));
        }
        D.base = base;
    };
    auto head = [&](int64_t t) -> LHead {
        const int64_t p = P.u0 + t * 64 + lane;
        const int64_t cc = min(max(p - hb.pos_begin, (int64_t)0), hb.n_cols - 1);
        return LHead{reinterpret_cast<const uint32_t *>(hb.off + cc)[0], reinterpret_cast<const uint32_t *>(hb.off + cc + 1)[0],
                     (uint32_t)ref[min(max(p, P.u0), P.u1 - 1)]};
    };

    // one tile: counts of its columns, then the exact fold of the columns that may call
    uint8_t *const sc = slots[threadIdx.x >> 6][0];
    uint8_t *const sq = slots[threadIdx.x >> 6][1];
    // stage a tile into this wave's slot (LDS operations of a wave complete in order)
    auto stage = [&](const LData &D) {
#pragma unroll
        for (int k = 0; k < LCH; k++) {
            *reinterpret_cast<u32x4 *>(sc + 1024 * k + 16 * lane) = D.c[k];
            *reinterpret_cast<u32x4 *>(sq + 1024 * k + 16 * lane) = D.q[k];
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
    };
    auto process = [&](int64_t t, uint64_t base, const LHead &D) {
        const int64_t p = P.u0 + t * 64 + lane;
        const bool inr = in_range(t);
        const uint8_t refc = (uint8_t)D.rc;
        const uint32_t lx = ((uint32_t)refc & 0xDFu) - 65u;
        const uint32_t lc = lx < 16u ? (uint32_t)(0x00F0000004000201ull >> (4u * lx)) & 0xFu
                                     : (lx < 26u ? (0x8000u >> (4u * (lx - 16u))) & 0xFu : 0u);
        const uint32_t M = lc ? lc : 1u, mrep = M * 0x01010101u;   // code_of_ref, branch-free
        uint32_t len = inr ? D.oe - D.ob : 0u;
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
        const uint32_t brel = inr ? D.ob - (uint32_t)base : 0u;       // the column's first byte in the tile
        // counts: the entries that pass the bq filter (totalDepth, :87) and those that are the REF code at a
        // q of 4..127 (SWAR; every other passing entry — another allele, D/N, a REF entry at q < 4 or >= 128 —
        // counts as non-REF)
        uint32_t mcf = 0, dep = 0;
        auto count = [&](const u32x4 &cw, const u32x4 &qw, int32_t x0, int32_t vlen) {
            uint32_t vm[4];
            valid_masks<4>(x0, 0, vlen, vm);
#pragma unroll
            for (int d = 0; d < 4; d++) {
                uint32_t f80, r80;
                swar4(dw<4>(cw, d), dw<4>(qw, d), vm[d], mrep, P.kpass, P.kok, f80, r80);
                mcf += __popc(f80);
                dep += __popc(f80 | r80);
            }
        };
        // the column's aligned blocks j0 .. j1 - 1 of the tile: from the slot, then (past it) from memory
        const uint32_t j0 = brel >> 4, j1 = len ? (brel + len + 15u) >> 4 : j0;
        const uint32_t jl = min(j1, (uint32_t)LNBLK);
        const uint32_t nl = jl > j0 ? jl - j0 : 0u;
        const uint32_t mx = wave_max_u32(nl);
        const int32_t vlen = (int32_t)min(len, (uint32_t)LSLOT - min(brel, (uint32_t)LSLOT));   // entries in the slot
        for (uint32_t u = 0; u < mx; u++) {
            const uint32_t j = min(j0 + u, (uint32_t)LNBLK - 1u);
            const u32x4 cw = *reinterpret_cast<const u32x4 *>(sc + 16u * j);
            const u32x4 qw = *reinterpret_cast<const u32x4 *>(sq + 16u * j);
            count(cw, qw, (int32_t)(16u * (j0 + u)) - (int32_t)brel, vlen);
        }
        if (__ballot(j1 > (uint32_t)LNBLK)) {
            const uint32_t f0 = max(j0, (uint32_t)LNBLK);
            for (uint32_t j = f0;; j++) {
                const bool more = j < j1;
                if (!__ballot(more)) break;
                u32x4 cw{0, 0, 0, 0}, qw{0, 0, 0, 0};
                if (more) {
                    cw = *(reinterpret_cast<const u32x4 *>(hb.code + base) + j);
                    qw = *(reinterpret_cast<const u32x4 *>(hb.qual + base) + j);
                }
                count(cw, qw, (int32_t)(16u * j) - (int32_t)brel, (int32_t)len);
            }
        }
        // prepare_variants' filters (:131, :151-157) on what the counts bound: an allele other than the REF char
        // has at most dep - mcf entries; the REF code's own entries (mcf) are a candidate allele when the stored REF
        // char is not its upper-case letter (soft-masked 'a' != 'A', :151; a REF outside ACGTN maps to A).  A
        // position that passes is folded exactly by k_lite_fold and decided by the sparse finalize.
        bool mc = false;
        if ((int64_t)dep >= (int64_t)P.min_td) {
            const double dlo = (double)dep * P.ratio_lo;
            const uint32_t nonref = dep - mcf;
            mc = ((int64_t)nonref >= P.min_ad && (double)nonref >= dlo) ||
                 (refc != nibble_char(M) && (int64_t)mcf >= P.min_ad && (double)mcf >= dlo);
        }
        const bool want = inr && (deep || (len != 0 && mc));
        const uint64_t wm = __ballot(want);
        if (wm) {
            uint32_t at = 0;                           // one list reservation per wave
            if (lane == 0) at = atomicAdd(P.n_list, (uint32_t)__popcll(wm));
            at = (uint32_t)__builtin_amdgcn_readfirstlane(at);
            if (want) P.list[at + __builtin_amdgcn_mbcnt_hi((uint32_t)(wm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wm, 0u))] = p;
        }
    };

    // the pipeline: tiles t and t + stride in flight in sets A and B while t is counted, their byte ranges two
    // tiles further ahead, the lanes' column bounds one tile ahead (sets HA, HB).  A tile's set is staged into
    // the slot and reloaded with the tile two ahead before the counting starts.  Every pair alternates: no
    // register copy of a pending load (hipcc would wait for it).
    // (compiler barriers keep each set's loads together and in this order: hipcc's wait counts follow issue order)
#define SPG_ORDER asm volatile("" ::: "memory")
    LBounds B0 = bounds(tile), B1 = bounds(tile + stride);
    LData A, B;
    issue(tile, B0, A);
    SPG_ORDER;
    issue(tile + stride, B1, B);
    SPG_ORDER;
    B0 = bounds(tile + 2 * stride);
    B1 = bounds(tile + 3 * stride);
    LHead HA = head(tile), HB;
    SPG_ORDER;
    while (tile < n_tiles) {
        stage(A);
        uint64_t base = A.base;
        issue(tile + 2 * stride, B0, A);
        SPG_ORDER;
        B0 = bounds(tile + 4 * stride);
        HB = head(tile + stride);
        SPG_ORDER;
        process(tile, base, HA);
        tile += stride;
        if (tile >= n_tiles) break;
        stage(B);
        base = B.base;
        issue(tile + 2 * stride, B1, B);
        SPG_ORDER;
        B1 = bounds(tile + 4 * stride);
        HA = head(tile + stride);
        SPG_ORDER;
        process(tile, base, HB);
        tile += stride;
    }
}

// The exact fold of the positions k_acc_lite listed (the ones whose counts pass the pre-check; columns of
// >= t_deep entries are left to k_acc_seg<1>): one lane per position, its column read in BAM order from the
// batch (L2-resident after k_acc_lite) — process_pileup_column / process_svn (:74-103): totalDepth, D/N/other,
// per allele count, sum q, q lower bound, first entry (dict order), sum ln(1 - eps), sum eps — merged into an
// empty record (first visit :77-85).
__global__ __launch_bounds__(256) void k_lite_fold(MParams P, Hist hb, const uint8_t *__restrict__ ref,
                                                   const Tables *__restrict__ T, Acc *__restrict__ acc) {
    __shared__ double2 lut[256];
    for (uint32_t q = threadIdx.x; q < 256u; q += 256u) lut[q] = make_double2(T->fast[q][0], T->fast[q][1]);
    __syncthreads();
    const uint32_t n_list = *P.n_list;
    for (uint32_t i0 = blockIdx.x * 256u + (threadIdx.x & ~63u); i0 < n_list; i0 += gridDim.x * 256u) {
        const uint32_t i = i0 + (threadIdx.x & 63u);
        const int64_t p = i < n_list ? P.list[i] : P.u0;
        const int64_t col = p - hb.pos_begin;
        const uint64_t hob = hb.off[col];
        const uint32_t len = (uint32_t)(hb.off[col + 1] - hob);
        const bool fold = i < n_list && len != 0 && !(P.t_deep && len >= P.t_deep);
        const uint8_t refc = ref[p];
        uint32_t fd = 0, fdel = 0, fskip = 0, foth = 0;
        uint32_t fc[NSLOT], fsq[NSLOT], ffirst[NSLOT], fqf[NSLOT];
        double fsl[NSLOT], fse[NSLOT];
#pragma unroll
        for (int k = 0; k < NSLOT; k++) { fc[k] = fsq[k] = 0; ffirst[k] = INF32; fqf[k] = 255; fsl[k] = fse[k] = 0.0; }
        const uint64_t a0 = hob & ~(uint64_t)3;       // (dword-aligned column window, L2-resident)
        const int32_t lead = (int32_t)(hob & 3u);
        const uint32_t nb = fold && len ? (uint32_t)(((uint32_t)lead + len + 15u) >> 4) : 0u;
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
        if (!fold) continue;
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
    }
}

// ---------------------------------------------------------------------------------------------------------
// k_count_cols: the counting pass of a calls-only sample whose only batch is mid-depth (mean column >= 256
// entries, e.g. 1,000x SARS-CoV-2, BASELINE config 2), finalized once (process_bam then prepare_variants,
// live_variant_caller.py:54-185).  As k_acc_lite, but for long columns: a wave owns a tile of 64 / LPC consecutive
// columns and LPC lanes share each column, taking its 16-B blocks round-robin — a column's LPC lanes read LPC x 16
// contiguous bytes per round and the tile's columns are adjacent, so a wave's loads are a coalesced stream of the
// tile's bytes with no LDS staging.  U rounds are loaded at once (2U 16-B loads per lane in flight); the kernel
// needs few registers, so many waves per SIMD keep HBM busy while others count.  Per column the bq-passing
// entries and the REF-code entries at q 4..127 (SWAR), reduced over its lanes; the positions whose totals pass
// prepare_variants' filters (:131, :151-157) are listed — the absolute position for the sparse finalize and the
// batch column for k_acc_seg<1>'s exact fold (the same list index).  No record is written here.
// ---------------------------------------------------------------------------------------------------------
template <int LPC, int U>
__global__ __launch_bounds__(256) void k_count_cols(MParams P, Hist hb, const uint8_t *__restrict__ ref,
                                                    uint32_t *__restrict__ dlist) {
    constexpr int TC = 64 / LPC;
    const int lane = threadIdx.x & 63, sub = lane % LPC, cl = lane / LPC;
    const int64_t n_tiles = (hb.n_cols + TC - 1) / TC;
    const int64_t wstride = (int64_t)gridDim.x * 4;
    const u32x4 *const gc = reinterpret_cast<const u32x4 *>(hb.code);
    const u32x4 *const gq = reinterpret_cast<const u32x4 *>(hb.qual);
    // a tile's column header (CSR bounds, REF char), loaded one tile ahead: the data loads of a tile then wait for
    // one round trip, not two
    struct Hdr {
        uint64_t ob, oe;
        uint32_t rc;
    };
    auto header = [&](int64_t t) -> Hdr {
        const int64_t cc = min(t * TC + cl, hb.n_cols - 1);
        return Hdr{hb.off[cc], hb.off[cc + 1], (uint32_t)ref[hb.pos_begin + cc]};
    };
    int64_t tile = (int64_t)__builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    Hdr nx = header(min(tile, n_tiles - 1));
    for (; tile < n_tiles; tile += wstride) {
        const Hdr h = nx;
        nx = header(min(tile + wstride, n_tiles - 1));
        asm volatile("" ::: "memory");                  // (issued before this tile's data loads)
        const int64_t col = tile * TC + cl;
        const bool inr = col < hb.n_cols;
        const uint64_t ob = h.ob, oe = h.oe;
        const uint8_t refc = (uint8_t)h.rc;
        const uint32_t mrep = code_of_ref(refc) * 0x01010101u;
        const uint32_t len = inr ? (uint32_t)(oe - ob) : 0u;
        const uint64_t j0 = ob >> 4;                        // the column's first 16-B block (the arrays are padded)
        const uint32_t nblk = len ? (uint32_t)(((oe + 15) >> 4) - j0) : 0u;
        const uint32_t mine = nblk > (uint32_t)sub ? (nblk - (uint32_t)sub + LPC - 1) / LPC : 0u;   // this lane's blocks
        const uint32_t rounds = wave_max_u32(mine);
        const int32_t lead = (int32_t)(ob & 15u);
        uint32_t dep = 0, mcf = 0;
        for (uint32_t t0 = 0; t0 < rounds; t0 += U) {
            u32x4 cw[U], qw[U];
#pragma unroll
            for (int u = 0; u < U; u++) {                   // (blocks past the lane's share reload its first one)
                const uint32_t t = t0 + (uint32_t)u;
                const uint64_t j = j0 + (t < mine ? (uint64_t)sub + (uint64_t)LPC * t : 0u);
                cw[u] = __builtin_nontemporal_load(gc + j);
                qw[u] = __builtin_nontemporal_load(gq + j);
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t t = t0 + (uint32_t)u;
                if (t >= mine) break;
                const int32_t x0 = (int32_t)(16u * ((uint32_t)sub + (uint32_t)LPC * t)) - lead;   // entry of the block's byte 0
                uint32_t vm[4];
                valid_masks<4>(x0, 0, (int32_t)len, vm);
#pragma unroll
                for (int d = 0; d < 4; d++) {
                    uint32_t f80, r80;
                    swar4(dw<4>(cw[u], d), dw<4>(qw[u], d), vm[d], mrep, P.kpass, P.kok, f80, r80);
                    mcf += __popc(f80);
                    dep += __popc(f80 | r80);
                }
            }
        }
#pragma unroll
        for (int o = 1; o < LPC; o <<= 1) {
            dep += (uint32_t)__shfl_xor((int)dep, o);
            mcf += (uint32_t)__shfl_xor((int)mcf, o);
        }
        // prepare_variants' filters on what the counts bound (as k_acc_lite: non-REF alleles <= dep - mcf; the REF
        // code's own entries are a candidate when the stored REF char is not its upper-case letter, :151)
        bool mc = false;
        if (len && (int64_t)dep >= (int64_t)P.min_td) {
            const double dlo = (double)dep * P.ratio_lo;
            const uint32_t nonref = dep - mcf;
            mc = ((int64_t)nonref >= P.min_ad && (double)nonref >= dlo) ||
                 (refc != nibble_char(mrep & 0xFFu) && (int64_t)mcf >= P.min_ad && (double)mcf >= dlo);
        }
        const bool want = inr && sub == 0 && mc;
        const uint64_t wm = __ballot(want);
        if (wm) {
            uint32_t at = 0;
            if (lane == 0) at = atomicAdd(P.n_list, (uint32_t)__popcll(wm));
            at = (uint32_t)__builtin_amdgcn_readfirstlane(at);
            if (want) {
                const uint32_t k = at + __builtin_amdgcn_mbcnt_hi((uint32_t)(wm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wm, 0u));
                P.list[k] = hb.pos_begin + col;
                dlist[k] = (uint32_t)col;
            }
        }
    }
}

#define SPG_COUNT_COLS(L) (L == 4 ? (const void *)k_count_cols<4, 4> : L == 8 ? (const void *)k_count_cols<8, 4> \
                           : L == 16 ? (const void *)k_count_cols<16, 4> : L == 32 ? (const void *)k_count_cols<32, 4> \
                           : (const void *)k_count_cols<64, 4>)
int count_cols_blocks_per_cu(int lpc) {
    static int n[5] = {-1, -1, -1, -1, -1};
    const int i = lpc == 4 ? 0 : lpc == 8 ? 1 : lpc == 16 ? 2 : lpc == 32 ? 3 : 4;
    if (n[i] < 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, SPG_COUNT_COLS(lpc), 256, 0) != hipSuccess || b < 1) b = 2;
        n[i] = b;
    }
    return n[i];
}
hipError_t launch_count_cols(const MParams &P, const Hist &hb, const uint8_t *ref, uint32_t *dlist, int lpc, int64_t blocks,
                             hipStream_t st) {
    if (hb.n_cols == 0) return hipSuccess;
    const dim3 grid((unsigned)std::max<int64_t>(1, blocks)), blk(256);
    switch (lpc) {
        case 4: hipLaunchKernelGGL((k_count_cols<4, 4>), grid, blk, 0, st, P, hb, ref, dlist); break;
        case 8: hipLaunchKernelGGL((k_count_cols<8, 4>), grid, blk, 0, st, P, hb, ref, dlist); break;
        case 16: hipLaunchKernelGGL((k_count_cols<16, 4>), grid, blk, 0, st, P, hb, ref, dlist); break;
        case 32: hipLaunchKernelGGL((k_count_cols<32, 4>), grid, blk, 0, st, P, hb, ref, dlist); break;
        case 64: hipLaunchKernelGGL((k_count_cols<64, 4>), grid, blk, 0, st, P, hb, ref, dlist); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_lite_fold(const MParams &P, const Hist &hb, const uint8_t *ref, const Tables *T, Acc *acc, int64_t blocks,
                            hipStream_t st) {
    hipLaunchKernelGGL(k_lite_fold, dim3((unsigned)std::max<int64_t>(1, blocks)), dim3(256), 0, st, P, hb, ref, T, acc);
    return hipGetLastError();
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


// ---------------------------------------------------------------------------------------------------------
// Counted mode: a calls-only sample accumulated as many shallow batches (process_bam once per BAM,
// vc_queue.py:142-144; BASELINE config 4 in its live form).  prepare_variants' filters need, per position,
// totalDepth and the counts of its alleles; k_acc_lite_run adds each batch's bq-passing entries and its
// REF-code entries (q 4..127) into two u32 arrays — additive, so batches fold in any order and across
// finalizes — and k_count_list lists the positions whose counts can pass the filters.  k_fold_hist then
// builds those positions' records exactly from the batch history (every batch since reset, in order); the
// sparse finalize decides them.  Records of the other positions are re-materialized if anything reads them.
// ---------------------------------------------------------------------------------------------------------

struct RUnit {             // one (tile, batch) unit in flight: the batch's arrays and the tile's byte range
    const uint64_t *off;
    const uint8_t *code, *qual;
    int64_t pos_begin, n_cols;
    uint64_t b, e;
};
struct RMeta {             // a unit's values the counting needs (resolved at issue: no pending loads)
    uint64_t base;
    const uint8_t *code, *qual;
    int64_t pos_begin, n_cols;
    bool nonempty;
};
template <int NCH>
struct RData {             // its staged chunks
    u32x4 c[NCH], q[NCH];
    RMeta m;
};
struct RHead {             // the lane's column bounds in the unit's batch (ping-pong, one unit ahead); low
    uint32_t ob, oe;       // halves only (a loaded dword nothing reads lets hipcc reuse its register: a full wait)
};

// items = (tile of 64 / LPC columns, batch split); a wave streams its item's batches through the LDS slot,
// LPC lanes per column taking the column's 16-B blocks round-robin
template <int LPC, int NCH>
__global__ __launch_bounds__(64 * LW) __attribute__((amdgpu_waves_per_eu(3, 8))) void k_acc_lite_run(
    MParams P, const Hist *__restrict__ H, const uint8_t *__restrict__ ref, uint32_t *__restrict__ cdep,
    uint32_t *__restrict__ cmcf) {
    constexpr int TC = 64 / LPC;
    constexpr int RSLOT = 1024 * NCH, RNBLK = RSLOT / 16;   // NCH 1 KiB chunks per array per unit
    __shared__ __attribute__((aligned(16))) uint8_t slots[LW][2][RSLOT];
    const int lane = threadIdx.x & 63, sub = lane % LPC, cl = lane / LPC;
    uint8_t *const sc = slots[threadIdx.x >> 6][0];
    uint8_t *const sq = slots[threadIdx.x >> 6][1];
    const int64_t n_tiles = P.n_groups, n_items = n_tiles * P.S;
    const int64_t wstride = (int64_t)gridDim.x * LW;
    for (int64_t item = (int64_t)__builtin_amdgcn_readfirstlane(blockIdx.x * LW + (threadIdx.x >> 6)); item < n_items;
         item += wstride) {
        const int64_t g = item % n_tiles, sp = item / n_tiles;
        const int32_t k0 = (int32_t)sp * P.kper, k1 = min(P.K, k0 + P.kper);
        const int64_t t0 = P.u0 + g * TC, t1 = min(t0 + TC, P.u1);
        const int64_t p = t0 + cl;
        const bool inr = p < P.u1;
        const uint8_t refc = ref[min(p, P.u1 - 1)];
        const uint32_t lx = ((uint32_t)refc & 0xDFu) - 65u;
        const uint32_t lc = lx < 16u ? (uint32_t)(0x00F0000004000201ull >> (4u * lx)) & 0xFu
                                     : (lx < 26u ? (0x8000u >> (4u * (lx - 16u))) & 0xFu : 0u);
        const uint32_t mrep = (lc ? lc : 1u) * 0x01010101u;
        uint32_t dep = 0, mcf = 0;

        auto unit = [&](int32_t k) -> RUnit {         // batch k's descriptor and the tile's byte range in it
            const Hist h = H[P.h0 + min(k, P.K - 1)];
            const int64_t cA = min(max(t0 - h.pos_begin, (int64_t)0), h.n_cols);
            const int64_t cB = min(max(t1 - h.pos_begin, (int64_t)0), h.n_cols);
            return RUnit{h.off, h.code, h.qual, h.pos_begin, h.n_cols, gbl(h.off)[cA], gbl(h.off)[cB]};
        };
        auto issue = [&](int32_t k, const RUnit &U, RData<NCH> &D) {
            const uint64_t base = U.b & ~(uint64_t)15;
            const uint64_t span = k < k1 ? U.e - base : 0;
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                const uint32_t o = 1024u * c + 16u * lane;
                const uint64_t a = o < span ? base + o : base;
                D.c[c] = __builtin_nontemporal_load(gbl(reinterpret_cast<const u32x4 *>(U.code + a)));
                D.q[c] = __builtin_nontemporal_load(gbl(reinterpret_cast<const u32x4 *>(U.qual + a)));
            }
            D.m = RMeta{base, U.code, U.qual, U.pos_begin, U.n_cols, U.e > U.b};
        };
        auto head = [&](int32_t k) -> RHead {
            const Hist h = H[P.h0 + min(k, P.K - 1)];
            const int64_t cc = min(max(p - h.pos_begin, (int64_t)0), max(h.n_cols - 1, (int64_t)0));
            return RHead{gbl(reinterpret_cast<const uint32_t *>(h.off + cc))[0],
                         gbl(reinterpret_cast<const uint32_t *>(h.off + cc + 1))[0]};
        };
        auto stage = [&](const RData<NCH> &D) {
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                *reinterpret_cast<u32x4 *>(sc + 1024 * c + 16 * lane) = D.c[c];
                *reinterpret_cast<u32x4 *>(sq + 1024 * c + 16 * lane) = D.q[c];
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        };
        auto process = [&](const RMeta &U, const RHead &D) {
            const uint64_t base = U.base;
            const int64_t col = p - U.pos_begin;
            const bool inb = inr && col >= 0 && col < U.n_cols && U.nonempty;
            const uint32_t len = inb ? D.oe - D.ob : 0u;
            const uint32_t brel = inb ? D.ob - (uint32_t)base : 0u;
            auto count = [&](const u32x4 &cw, const u32x4 &qw, int32_t x0, int32_t vlen) {
                uint32_t vm[4];
                valid_masks<4>(x0, 0, vlen, vm);
#pragma unroll
                for (int d = 0; d < 4; d++) {
                    uint32_t f80, r80;
                    swar4(dw<4>(cw, d), dw<4>(qw, d), vm[d], mrep, P.kpass, P.kok, f80, r80);
                    mcf += __popc(f80);
                    dep += __popc(f80 | r80);
                }
            };
            // this lane's blocks of the column: j0 + sub, j0 + sub + LPC, ... (slot, then memory past it)
            const uint32_t j0 = brel >> 4, j1 = len ? (brel + len + 15u) >> 4 : j0;
            const uint32_t jl = min(j1, (uint32_t)RNBLK);
            const uint32_t nl = jl > j0 + (uint32_t)sub ? (jl - j0 - (uint32_t)sub + LPC - 1) / LPC : 0u;
            const uint32_t mx = wave_max_u32(nl);
            const int32_t vlen = (int32_t)min(len, (uint32_t)RSLOT - min(brel, (uint32_t)RSLOT));
            for (uint32_t t = 0; t < mx; t++) {
                const uint32_t jj = j0 + (uint32_t)sub + LPC * t;
                const uint32_t j = min(jj, (uint32_t)RNBLK - 1u);
                const u32x4 cw = *reinterpret_cast<const u32x4 *>(sc + 16u * j);
                const u32x4 qw = *reinterpret_cast<const u32x4 *>(sq + 16u * j);
                count(cw, qw, (int32_t)(16u * jj) - (int32_t)brel, vlen);
            }
            if (__ballot(j1 > (uint32_t)RNBLK)) {
                const uint32_t b0 = max(j0 + (uint32_t)sub, (uint32_t)RNBLK);
                const uint32_t f0 = j0 + (uint32_t)sub + ((b0 - (j0 + (uint32_t)sub) + LPC - 1) / LPC) * LPC;
                for (uint32_t j = f0;; j += LPC) {
                    const bool more = j < j1;
                    if (!__ballot(more)) break;
                    u32x4 cw{0, 0, 0, 0}, qw{0, 0, 0, 0};
                    if (more) {
                        cw = gbl(reinterpret_cast<const u32x4 *>(U.code + base))[j];
                        qw = gbl(reinterpret_cast<const u32x4 *>(U.qual + base))[j];
                    }
                    count(cw, qw, (int32_t)(16u * j) - (int32_t)brel, (int32_t)len);
                }
            }
        };
        // the pipeline over the item's batches (as k_acc_lite's over tiles: two units in flight, their ranges two
        // further ahead, the lanes' column bounds one ahead; every pair alternates)
        RUnit B0 = unit(k0), B1 = unit(k0 + 1);
        RData<NCH> A, B;
        issue(k0, B0, A);
        SPG_ORDER;
        issue(k0 + 1, B1, B);
        SPG_ORDER;
        B0 = unit(k0 + 2);
        B1 = unit(k0 + 3);
        RHead HA = head(k0), HB;
        SPG_ORDER;
        for (int32_t k = k0; k < k1;) {
            stage(A);
            const RMeta MA = A.m;
            issue(k + 2, B0, A);
            SPG_ORDER;
            B0 = unit(k + 4);
            HB = head(k + 1);
            SPG_ORDER;
            process(MA, HA);
            if (++k >= k1) break;
            stage(B);
            const RMeta MB = B.m;
            issue(k + 2, B1, B);
            SPG_ORDER;
            B1 = unit(k + 4);
            HA = head(k + 1);
            SPG_ORDER;
            process(MB, HB);
            ++k;
        }
        // the column's totals (its LPC lanes), added to the position's counts
#pragma unroll
        for (int o = 1; o < LPC; o <<= 1) {
            dep += (uint32_t)__shfl_xor((int)dep, o);
            mcf += (uint32_t)__shfl_xor((int)mcf, o);
        }
        if (inr && sub == 0 && dep) {
            atomicAdd(cdep + p, dep);
            atomicAdd(cmcf + p, mcf);
        }
    }
}

// prepare_variants' filters on the counted totals (as k_acc_lite's pre-check): positions listed for the exact
// fold and the sparse finalize
__global__ __launch_bounds__(256) void k_count_list(MParams P, const uint8_t *__restrict__ ref,
                                                    const uint32_t *__restrict__ cdep, const uint32_t *__restrict__ cmcf) {
    const int64_t p = P.u0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool want = false;
    if (p < P.u1) {
        const uint32_t dep = cdep[p], mcf = cmcf[p];
        if (dep && (int64_t)dep >= (int64_t)P.min_td) {
            const uint8_t refc = ref[p];
            const uint32_t lx = ((uint32_t)refc & 0xDFu) - 65u;
            const uint32_t lc = lx < 16u ? (uint32_t)(0x00F0000004000201ull >> (4u * lx)) & 0xFu
                                         : (lx < 26u ? (0x8000u >> (4u * (lx - 16u))) & 0xFu : 0u);
            const double dlo = (double)dep * P.ratio_lo;
            const uint32_t nonref = dep - mcf;
            want = ((int64_t)nonref >= P.min_ad && (double)nonref >= dlo) ||
                   (refc != nibble_char(lc ? lc : 1u) && (int64_t)mcf >= P.min_ad && (double)mcf >= dlo);
        }
    }
    const uint64_t wm = __ballot(want);
    if (!wm) return;
    uint32_t at = 0;
    if ((threadIdx.x & 63) == 0) at = atomicAdd(P.n_list, (uint32_t)__popcll(wm));
    at = (uint32_t)__builtin_amdgcn_readfirstlane(at);
    if (want) P.list[at + __builtin_amdgcn_mbcnt_hi((uint32_t)(wm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wm, 0u))] = p;
}

// wave reductions for the fold's partial states (fixed DPP pattern: deterministic)
__device__ __forceinline__ uint32_t wmin_u32(uint32_t v) {
#pragma unroll
    for (int c = 0; c < 4; c++) v = min(v, dpp_u32(v, c));
    return min(min((uint32_t)__builtin_amdgcn_readlane(v, 0), (uint32_t)__builtin_amdgcn_readlane(v, 16)),
               min((uint32_t)__builtin_amdgcn_readlane(v, 32), (uint32_t)__builtin_amdgcn_readlane(v, 48)));
}
__device__ __forceinline__ uint64_t wmin_u64(uint64_t v) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const uint64_t o = ((uint64_t)dpp_u32((uint32_t)(v >> 32), c) << 32) | dpp_u32((uint32_t)v, c);
        v = min(v, o);
    }
    uint64_t m = ~0ull;
#pragma unroll
    for (int l = 0; l < 64; l += 16) {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
        m = min(m, ((uint64_t)hi << 32) | lo);
    }
    return m;
}

struct FoldPart {          // one wave's reduced partial state of a position (k_fold_hist)
    uint32_t depth, n_del, n_skip, n_other, fb;
    uint32_t cnt[NSLOT], sq[NSLOT], qf[NSLOT];
    uint64_t key[NSLOT];
    double sl[NSLOT], se[NSLOT];
};

// The exact record of each listed position over history batches [h0, h0 + K) (every batch since reset): TPP
// threads per position (64 .. 1024, about one batch each), thread r folding a contiguous batch range in BAM
// order (the per-entry rules of process_pileup_column / process_svn, :74-103).  The partial states reduce
// with sums and with minima of the first-entry keys (thread r, stream index) — the batch order, as
// k_merge_parts' (split, index) keys — first per wave, then over the position's waves in order, into a FRESH
// record (first visit :77-85).  (The fp64 sums are added in that fixed tree order: within 1e-16 relative of
// the sequential fold; positions where the order matters are replayed exactly from the history by the
// finalize.)
struct FoldAux {            // several workgroups per position (long histories): their partials and arrival counts
    FoldPart *part;        // [cap][bpp]
    uint32_t *arrived;     // [cap], zero between launches (the last arrival resets it)
    int32_t bpp, cap;      // parts per position (1 = one workgroup), positions that may take them
};

__global__ __launch_bounds__(1024) void k_fold_hist(MParams P, const Hist *__restrict__ H, const uint8_t *__restrict__ ref,
                                                    const Tables *__restrict__ T, Acc *__restrict__ acc, FoldAux X) {
    __shared__ double2 lut[256];
    __shared__ FoldPart wp[16];
    if (threadIdx.x < 256) lut[threadIdx.x] = make_double2(T->fast[threadIdx.x][0], T->fast[threadIdx.x][1]);
    __syncthreads();
    const uint32_t n_list = *P.n_list;
    // X.bpp > 1 (a history of thousands of batches): each of the first X.cap listed positions is folded by
    // X.bpp workgroups over consecutive batch ranges (the work of one position otherwise occupies one CU); the
    // last to arrive merges their partials in range order.  Items: (position, part) for those, then one item
    // per remaining position.
    const int32_t bpp = X.bpp;
    const uint32_t n_multi = bpp > 1 ? min(n_list, (uint32_t)X.cap) : 0u;
    const uint32_t n_items_blk = n_multi * (uint32_t)bpp + (n_list - n_multi);
    uint32_t tpp = 64;
    while (tpp < 1024u && tpp < (uint32_t)P.K) tpp <<= 1;
    if (bpp > 1) tpp = 1024;
    const uint32_t G = 1024u / tpp, grp = threadIdx.x / tpp, r = threadIdx.x % tpp;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t n_iter = bpp > 1 ? n_items_blk : n_list;
    for (uint32_t lb = blockIdx.x * G; lb < n_iter; lb += gridDim.x * G) {
        uint32_t li, part = 0, nparts = 1;
        if (bpp > 1) {
            if (lb < n_multi * (uint32_t)bpp) { li = lb / (uint32_t)bpp; part = lb % (uint32_t)bpp; nparts = (uint32_t)bpp; }
            else li = n_multi + (lb - n_multi * (uint32_t)bpp);
        } else {
            li = lb + grp;
        }
        const bool act = li < n_list;
        const int64_t p = act ? P.list[li] : P.u0;
        // incremental (vc_queue.py:142-144 finalizes after every BAM): a record an earlier counted finalize of this
        // sample folded holds batches [0, kbase) already; only the batches since are folded and merged into it
        int32_t kbase = 0;
        if (act && P.wm) {
            const uint64_t w = P.wm[p];
            if ((uint32_t)(w >> 32) == P.wm_gen && acc[p].epoch == P.epoch) kbase = min((int32_t)(uint32_t)w, P.K);
        }
        kbase = __builtin_amdgcn_readfirstlane(kbase);     // (one item per wave: tpp >= 64)
        // this item's batch range, then this thread's share of it
        const int32_t kp = (P.K - kbase + (int32_t)nparts - 1) / (int32_t)nparts;
        const int32_t kb0 = min(P.K, kbase + (int32_t)part * kp), kb1 = min(P.K, kb0 + kp);
        const int32_t per = (kb1 - kb0 + (int32_t)tpp - 1) / (int32_t)tpp;
        const int32_t k0 = min(kb1, kb0 + (int32_t)r * per), k1 = min(kb1, k0 + per);
        uint32_t depth = 0, n_del = 0, n_skip = 0, n_other = 0, fb = INF32, sidx = 0;
        uint32_t cnt[NSLOT], sq[NSLOT], qf[NSLOT], first[NSLOT];
        double sl[NSLOT], se[NSLOT];
#pragma unroll
        for (int j = 0; j < NSLOT; j++) { cnt[j] = sq[j] = 0; qf[j] = 255; first[j] = INF32; sl[j] = se[j] = 0.0; }
        // batch k's column for this position (descriptor, then bounds: two dependent loads), fetched one batch
        // ahead so that those loads are in flight while the current batch folds
        struct FCol {
            const uint8_t *code, *qual;
            uint64_t ob;
            uint32_t len;
        };
        auto fetch = [&](int32_t k) -> FCol {
            const Hist h = H[P.h0 + min(k, P.K - 1)];
            const int64_t col = p - h.pos_begin;
            const bool in = act && k < k1 && col >= 0 && col < h.n_cols;
            const int64_t cc = in ? col : 0;
            const uint64_t ob = gbl(h.off)[cc], oe = gbl(h.off)[cc + 1];
            return FCol{h.code, h.qual, ob, in ? (uint32_t)(oe - ob) : 0u};
        };
        FCol cur = fetch(k0);
        for (int32_t k = k0; act && k < k1; k++) {
            const FCol nxt = fetch(k + 1);
            const uint32_t len = cur.len;
            if (len) {
                if (fb == INF32) fb = (uint32_t)k;
                const uint64_t a0 = cur.ob & ~(uint64_t)3;
                const int32_t lead = (int32_t)(cur.ob & 3u);
                const uint32_t nb = ((uint32_t)lead + len + 15u) >> 4;
                for (uint32_t u0 = 0; u0 < nb; u0 += 2) {
                    u32x4 cw[2], qw[2];
#pragma unroll
                    for (int i = 0; i < 2; i++) {         // two blocks in flight together (clamped: no branch)
                        const uint32_t u = min(u0 + (uint32_t)i, nb - 1u);
                        cw[i] = gbl(reinterpret_cast<const u32x4 *>(cur.code + a0))[u];
                        qw[i] = gbl(reinterpret_cast<const u32x4 *>(cur.qual + a0))[u];
                    }
#pragma unroll
                    for (int i = 0; i < 2; i++) {
                        const uint32_t u = u0 + (uint32_t)i;
                        if (u >= nb) break;
#pragma unroll
                        for (int b = 0; b < 16; b++) {
                            const int32_t x = (int32_t)(16u * u) + b - lead;
                            const uint32_t cc = (dw<4>(cw[i], b >> 2) >> (8 * (b & 3))) & 0xFFu;
                            const uint32_t qq = (dw<4>(qw[i], b >> 2) >> (8 * (b & 3))) & 0xFFu;
                            if (x < 0 || x >= (int32_t)len || (int)qq < P.min_bq) continue;
                            depth++;
                            if (cc == SPG_CODE_DEL) { n_del++; continue; }
                            if (cc == SPG_CODE_SKIP) { n_skip++; continue; }
                            const int s = slot_of(cc);
                            if (s < 0) { n_other++; continue; }
                            const double2 tt = lut[qq];
#pragma unroll
                            for (int j = 0; j < NSLOT; j++)
                                if (j == s) {
                                    cnt[j]++; sq[j] += qq; qf[j] = min(qf[j], qq); first[j] = min(first[j], sidx + (uint32_t)x);
                                    sl[j] += tt.x; se[j] += qq == 0 ? 1.0 : tt.y;
                                }
                        }
                    }
                }
                sidx += len;
            }
            cur = nxt;
        }
        // this wave's partial (its threads are consecutive in batch order)
        FoldPart w;
        w.depth = dsum_u32(depth); w.n_del = dsum_u32(n_del); w.n_skip = dsum_u32(n_skip); w.n_other = dsum_u32(n_other);
        w.fb = wmin_u32(fb);
#pragma unroll
        for (int j = 0; j < NSLOT; j++) {
            w.cnt[j] = dsum_u32(cnt[j]);
            w.sq[j] = dsum_u32(sq[j]);
            w.qf[j] = wmin_u32(qf[j]);
            w.key[j] = wmin_u64(cnt[j] ? ((uint64_t)(part * tpp + r) << 32) | first[j] : ~0ull);
            w.sl[j] = dsum_f64(sl[j]);
            w.se[j] = dsum_f64(se[j]);
        }
        if (tpp > 64) {
            if (lane == 0) wp[wave] = w;
            __syncthreads();
        }
        if (act && r == 0) {                           // the position's waves, in order
            const uint32_t nw = tpp / 64;
            for (uint32_t v = 1; v < nw; v++) {
                const FoldPart &o = wp[wave + v];
                w.depth += o.depth; w.n_del += o.n_del; w.n_skip += o.n_skip; w.n_other += o.n_other;
                w.fb = min(w.fb, o.fb);
#pragma unroll
                for (int j = 0; j < NSLOT; j++) {
                    w.cnt[j] += o.cnt[j]; w.sq[j] += o.sq[j]; w.qf[j] = min(w.qf[j], o.qf[j]);
                    w.key[j] = min(w.key[j], o.key[j]); w.sl[j] += o.sl[j]; w.se[j] += o.se[j];
                }
            }
            bool write = true;
            if (nparts > 1) {
                // publish this part; the last part to arrive merges them all, in range order
                X.part[(size_t)li * (size_t)bpp + part] = w;
                __threadfence();
                const uint32_t old = atomicAdd(X.arrived + li, 1u);
                write = old == (uint32_t)bpp - 1u;
                if (write) {
                    __threadfence();
                    const volatile FoldPart *pp = X.part + (size_t)li * (size_t)bpp;
                    FoldPart m;
                    m.depth = m.n_del = m.n_skip = m.n_other = 0;
                    m.fb = INF32;
#pragma unroll
                    for (int j = 0; j < NSLOT; j++) { m.cnt[j] = m.sq[j] = 0; m.qf[j] = 255; m.key[j] = ~0ull; m.sl[j] = m.se[j] = 0.0; }
                    for (int32_t v = 0; v < bpp; v++) {
                        const volatile FoldPart &o = pp[v];
                        m.depth += o.depth; m.n_del += o.n_del; m.n_skip += o.n_skip; m.n_other += o.n_other;
                        m.fb = min(m.fb, (uint32_t)o.fb);
#pragma unroll
                        for (int j = 0; j < NSLOT; j++) {
                            m.cnt[j] += o.cnt[j]; m.sq[j] += o.sq[j]; m.qf[j] = min(m.qf[j], (uint32_t)o.qf[j]);
                            m.key[j] = min(m.key[j], (uint64_t)o.key[j]); m.sl[j] += o.sl[j]; m.se[j] += o.se[j];
                        }
                    }
                    w = m;
                    X.arrived[li] = 0;                 // ready for the next launch
                }
            }
            if (write && P.wm && (kbase > 0 || w.fb != INF32)) P.wm[p] = ((uint64_t)P.wm_gen << 32) | (uint32_t)P.K;
            if (write && w.fb != INF32) {
                MState c;
                ms_init(c);
                c.depth = w.depth; c.n_del = w.n_del; c.n_skip = w.n_skip; c.n_other = w.n_other; c.fb = w.fb;
#pragma unroll
                for (int j = 0; j < NSLOT; j++) {
                    c.cnt[j] = w.cnt[j];
                    c.sq[j] = min(w.sq[j], 0x80000000u);           // (sum q saturating at 2^31)
                    c.qf[j] = (uint8_t)w.qf[j];
                    c.sl[j] = w.sl[j];
                    c.se[j] = w.se[j];
                }
                Acc a{};
                if (kbase > 0) a = acc[p];          // (the slots it holds come first in dict order, :100-101)
                else a.epoch = P.epoch;
                merge_state(a, c, w.key, P.seq0 + c.fb, ref[p]);
                const uint4 *src = reinterpret_cast<const uint4 *>(&a);
                uint4 *dst = reinterpret_cast<uint4 *>(acc + p);
#pragma unroll
                for (int t = 0; t < 10; t++) dst[t] = src[t];
            }
        }
        if (tpp > 64) __syncthreads();
    }
}

// units of about `fill` bytes per array: LPC lanes per column (64 / LPC columns per tile); 4 KiB slots for
// LPC 2 (32 columns of a 100x run), 3 KiB otherwise
#define SPG_RUN_KERNEL(L) (L == 1 ? (const void *)k_acc_lite_run<1, 3> : L == 2 ? (const void *)k_acc_lite_run<2, 4> \
                         : L == 4 ? (const void *)k_acc_lite_run<4, 3> : L == 8 ? (const void *)k_acc_lite_run<8, 3> \
                         : (const void *)k_acc_lite_run<1, 7>)
hipError_t launch_count_run(const MParams &P, const Hist *H, const uint8_t *ref, uint32_t *cdep, uint32_t *cmcf, int lpc,
                            int64_t blocks, hipStream_t st) {
    if (P.n_groups == 0 || P.K == 0) return hipSuccess;
    const dim3 grid((unsigned)std::max<int64_t>(1, blocks)), blk(64 * LW);
    switch (lpc) {
        case 1: hipLaunchKernelGGL((k_acc_lite_run<1, 3>), grid, blk, 0, st, P, H, ref, cdep, cmcf); break;
        case 2: hipLaunchKernelGGL((k_acc_lite_run<2, 4>), grid, blk, 0, st, P, H, ref, cdep, cmcf); break;
        case 4: hipLaunchKernelGGL((k_acc_lite_run<4, 3>), grid, blk, 0, st, P, H, ref, cdep, cmcf); break;
        case 8: hipLaunchKernelGGL((k_acc_lite_run<8, 3>), grid, blk, 0, st, P, H, ref, cdep, cmcf); break;
        default: hipLaunchKernelGGL((k_acc_lite_run<1, 7>), grid, blk, 0, st, P, H, ref, cdep, cmcf); break;   // "lpc" 0
    }
    return hipGetLastError();
}
int count_run_blocks_per_cu(int lpc) {
    static int n[5] = {-1, -1, -1, -1, -1};
    const int i = lpc == 1 ? 0 : lpc == 2 ? 1 : lpc == 4 ? 2 : lpc == 8 ? 3 : 4;
    if (n[i] < 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, SPG_RUN_KERNEL(lpc), 64 * LW, 0) != hipSuccess || b < 1) b = 2;
        n[i] = b;
    }
    return n[i];
}
hipError_t launch_count_list(const MParams &P, const uint8_t *ref, const uint32_t *cdep, const uint32_t *cmcf, hipStream_t st) {
    const int64_t n = P.u1 - P.u0;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_count_list, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, P, ref, cdep, cmcf);
    return hipGetLastError();
}
hipError_t launch_fold_hist(const MParams &P, const Hist *H, const uint8_t *ref, const Tables *T, Acc *acc, int64_t blocks,
                            void *part, uint32_t *arrived, int bpp, int cap, hipStream_t st) {
    const FoldAux X{(FoldPart *)part, arrived, part ? bpp : 1, cap};
    hipLaunchKernelGGL(k_fold_hist, dim3((unsigned)std::max<int64_t>(1, blocks)), dim3(1024), 0, st, P, H, ref, T, acc, X);
    return hipGetLastError();
}
size_t fold_part_bytes() { return sizeof(FoldPart); }

}  // namespace spg
