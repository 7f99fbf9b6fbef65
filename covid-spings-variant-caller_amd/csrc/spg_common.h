// spg_common.h — device helpers shared by the engine kernels (spg_kernels.hip, spg_tile.hip): wave
// reductions, dict-order bookkeeping, record merges, SWAR entry classification, buffer descriptors.
#pragma once
#include "spg_device.h"

namespace spg {

// ------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// DPP wave reductions: quad_perm / row_half_mirror / row_mirror give every lane its 16-lane row
// total with VALU-latency steps (no LDS round trips); the four row totals are combined through
// readlane.  Fixed pattern -> deterministic fp64 summation order.
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v, int ctrl) {
    switch (ctrl) {
        case 0: return __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
        case 1: return __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
        case 2: return __builtin_amdgcn_update_dpp(0u, v, 0x141, 0xF, 0xF, false);   // row_half_mirror
        default: return __builtin_amdgcn_update_dpp(0u, v, 0x140, 0xF, 0xF, false);  // row_mirror
    }
}
__device__ __forceinline__ uint32_t dsum_u32(uint32_t v) {
#pragma unroll
    for (int c = 0; c < 4; c++) v += dpp_u32(v, c);
    return (uint32_t)__builtin_amdgcn_readlane(v, 0) + (uint32_t)__builtin_amdgcn_readlane(v, 16) +
           (uint32_t)__builtin_amdgcn_readlane(v, 32) + (uint32_t)__builtin_amdgcn_readlane(v, 48);
}
__device__ __forceinline__ double rl_f64(double v, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double dsum_f64(double v) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const uint64_t b = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = dpp_u32((uint32_t)b, c), hi = dpp_u32((uint32_t)(b >> 32), c);
        v += __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
    }
    return (rl_f64(v, 0) + rl_f64(v, 16)) + (rl_f64(v, 32) + rl_f64(v, 48));
}

// New alleles join the dict in order of first appearance in this batch (:100-101).  `first` holds each
// slot's first-entry key in the accumulated stream (u32 within one run, u64 across batch splits).
template <typename KeyT>
__device__ __forceinline__ uint32_t merge_order(uint32_t order, uint32_t newmask, const KeyT *first) {
    uint32_t n = order & 7u;
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        if ((newmask >> k) & 1u) {
            uint32_t rank = 0;
#pragma unroll
            for (int j = 0; j < NSLOT; j++)
                if (j != k && ((newmask >> j) & 1u) && (first[j] < first[k] || (first[j] == first[k] && j < k)))
                    rank++;
            order |= (uint32_t)k << (3 + 3 * (n + rank));
        }
    }
    return (order & ~7u) | (n + __popc(newmask));
}

__device__ __forceinline__ uint32_t order_mask(uint32_t order) {
    uint32_t have = 0;
    const uint32_t n = order & 7u;
#pragma unroll
    for (uint32_t i = 0; i < NSLOT; i++)
        if (i < n) have |= 1u << ((order >> (3 + 3 * i)) & 7u);
    return have;
}

__device__ __forceinline__ uint32_t sat_add31(uint32_t a, uint32_t b) {   // sum q, saturating at 2^31
    const uint64_t s = (uint64_t)a + b;
    return s > 0x80000000ull ? 0x80000000u : (uint32_t)s;
}

__device__ __forceinline__ void ms_init(MState &S) {
    S.depth = S.n_del = S.n_skip = S.n_other = 0;
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        S.cnt[k] = 0; S.sq[k] = 0; S.first[k] = INF32; S.qf[k] = 255; S.sl[k] = 0.0; S.se[k] = 0.0;
    }
    S.fb = INF32; S.skip = 0; S.flags = 0;
}

// Merge one run of batches (state c, first-entry keys per slot) into the position's record `a` (already
// reset when it belongs to an older epoch): process_pileup_column's first visit (:77-85), totalDepth
// (:87) and process_svn's dict appends (:100-101) for a whole run at once.
template <typename KeyT>
__device__ __forceinline__ void merge_state(Acc &a, const MState &c, const KeyT *key, uint32_t first_seq, uint8_t refc) {
    if (a.first_batch == 0) {                       // first visit (:77-85)
        a.first_batch = first_seq;
        a.misc = refc;
    }
    a.depth += c.depth;                             // :87
    a.n_del += c.n_del;
    a.n_skip += c.n_skip;
    a.n_other += c.n_other;
    if (c.n_other) a.misc |= MISC_EXOTIC;
    a.misc |= (uint32_t)c.skip << MISC_SKIP_SHIFT;
    a.misc &= ~((uint32_t)c.skip << MISC_SEONLY_SHIFT);
    const uint32_t have = order_mask(a.order);
    uint32_t newmask = 0;
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        if (c.cnt[k]) {
            const bool had = a.cnt[k] != 0;         // absent slots' sums may hold stale bytes
            a.qf[k] = had ? (uint8_t)min((uint32_t)a.qf[k], (uint32_t)c.qf[k]) : c.qf[k];
            a.cnt[k] += c.cnt[k];
            a.sq[k] = sat_add31(a.sq[k], c.sq[k]);
            a.sl[k] = had ? a.sl[k] + c.sl[k] : c.sl[k];
            a.se[k] = had ? a.se[k] + c.se[k] : c.se[k];
            if (!((have >> k) & 1u)) newmask |= 1u << k;
        }
    }
    a.order = merge_order(a.order, newmask, key);
}

// A FRESH record needs its sl/se half (bytes 80..159) only when some present slot holds sums
__device__ __forceinline__ bool record_has_sums(const Acc &a) {
    const uint32_t skip = (a.misc >> MISC_SKIP_SHIFT) & ~(a.misc >> MISC_SEONLY_SHIFT) & 0x1Fu;
    bool sums = false;
#pragma unroll
    for (int k = 0; k < NSLOT; k++) sums |= a.cnt[k] != 0 && !((skip >> k) & 1u);
    return sums;
}
// ------------------------------------------------------------------------------------------
// SWAR classification of 4 entries (one dword of base_code, one of qual)
//   fast  = valid & q >= max(min_bq,4) & q < 128 & code == M      (the column's major allele)
//   rare  = valid & (q >= min_bq | q >= 128) & !fast                (exact per-entry path)
// Eight VALU ops: the q adds cannot carry across bytes (q & 127 plus at most 0x80); the code
// compare (code ^ M) + 0x7F can only carry out of a byte whose code is >= 128, which is never
// fast, and a carry can only turn the next byte's "equal" into "not equal" (rare, exact path).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void swar4(uint32_t cw, uint32_t qw, uint32_t v80, uint32_t mrep, uint32_t kpass,
                                      uint32_t kok, uint32_t &fast80, uint32_t &rare80) {
    const uint32_t q7 = qw & 0x7F7F7F7Fu;
    const uint32_t pass = q7 + kpass;                  // bit 7: (q & 127) >= min_bq
    const uint32_t ok = q7 + kok;                      // bit 7: (q & 127) >= max(min_bq, 4)
    const uint32_t ne = (cw ^ mrep) + 0x7F7F7F7Fu;     // bit 7: code != M (codes < 128)
    fast80 = ok & ~(ne | qw | cw) & v80;
    rare80 = (pass | qw) & ~fast80 & v80;
}

__device__ __forceinline__ uint32_t valid80(int32_t x, int32_t b, int32_t e) {   // bytes x..x+3 in [b,e)
    int32_t lead = b - x, end = e - x;
    lead = lead < 0 ? 0 : (lead > 4 ? 4 : lead);
    end = end < 0 ? 0 : (end > 4 ? 4 : end);
    return (uint32_t)((0x80808080ull << (8 * lead)) & (0x80808080ull >> (8 * (4 - end))));
}

// Validity of a lane's 4W entries o .. o + 4W - 1 against the column [b, e), one 0x80-per-byte mask
// per dword: the byte at slice position p is valid iff lead <= p < end.  With K_d holding
// 0x80 + p in each byte, K_d - lead (broadcast) has bit 7 iff p >= lead (no borrow: p, lead <= 16).
template <int W>
__device__ __forceinline__ void valid_masks(int32_t o, int32_t b, int32_t e, uint32_t (&v)[W]) {
    const uint32_t lead = (uint32_t)min(max(b - o, 0), 4 * W), end = (uint32_t)min(max(e - o, 0), 4 * W);
    const uint32_t lb = __builtin_amdgcn_perm(0u, lead, 0u), eb = __builtin_amdgcn_perm(0u, end, 0u);
#pragma unroll
    for (int d = 0; d < W; d++) {
        const uint32_t K = 0x80808080u + (uint32_t)(4 * d) * 0x01010101u + 0x03020100u;
        v[d] = (K - lb) & ~(K - eb) & 0x80808080u;
    }
}

template <int W>   // W dwords per lane per step: 4 (16 entries, dwordx4) or 1 (4 entries)
struct Vec;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <> struct Vec<4> { using T = u32x4; };
template <> struct Vec<1> { using T = uint32_t; };

template <int W>
__device__ __forceinline__ uint32_t dw(const typename Vec<W>::T &v, int d) {
    if constexpr (W == 1) { (void)d; return v; }
    else return d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
}

// Per-wave LDS record of the column the wave is processing.  Rare entries are few, so LDS atomics
// from the lanes that hold one are cheap, and the wave needs no register state for them.
struct __align__(8) WaveRare {
    double sl[NSLOT], se[NSLOT];
    uint32_t depth, n_del, n_skip, n_other;
    uint32_t cnt[NSLOT], sq[NSLOT], qf[NSLOT], first[NSLOT];
    uint32_t skip, pad;
};
static_assert(sizeof(WaveRare) == 184, "WaveRare");

__device__ __forceinline__ void rare_init(WaveRare *R, int lane) {
    uint32_t *w = reinterpret_cast<uint32_t *>(R);
    // words 0..19 doubles, 20..23 counters, 24..33 cnt/sq: 0; 34..38 qf: 255; 39..43 first: INF; 44 skip
    if (lane < 45) w[lane] = lane < 34 ? 0u : (lane < 39 ? 255u : (lane < 44 ? INF32 : 0u));
}

__device__ __forceinline__ void rare_entry(WaveRare *R, uint32_t code, uint32_t q, uint32_t idx,
                                           const double2 *__restrict__ lut, const Tables *__restrict__ T) {
    atomicAdd(&R->depth, 1u);
    if (code == SPG_CODE_DEL) { atomicAdd(&R->n_del, 1u); return; }
    if (code == SPG_CODE_SKIP) { atomicAdd(&R->n_skip, 1u); return; }
    const int sl = slot_of(code);
    if (sl < 0) { atomicAdd(&R->n_other, 1u); return; }
    atomicAdd(&R->cnt[sl], 1u);
    atomicAdd(&R->sq[sl], q);
    atomicMin(&R->qf[sl], q);
    atomicMin(&R->first[sl], idx);
    // {ln(1-eps), eps}; row 0 holds {0, 0}; q >= 128 (never a fast entry) from rows 256..383, so the
    // drain touches no global memory (a global load here would also wait for the chunk prefetch)
    (void)T;
    const double2 t = lut[q < 128u ? q : q + 128u];
    atomicAdd(&R->sl[sl], t.x);
    atomicAdd(&R->se[sl], q == 0 ? 1.0 : t.y);         // eps(Q0) = 1
}

// Wave-uniform buffer descriptor over bytes [0, n) of a column (T8/T20: the inputs go through
// readfirstlane so hipcc can prove uniformity; out-of-range lanes read zeros, no per-lane branch).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t column_rsrc(const uint8_t *p, uint32_t n) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void *base = (void *)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)__builtin_amdgcn_readfirstlane(n), 0x00020000);
}

// NT: non-temporal loads (aux = 2) for batches far larger than the 256 MiB Infinity Cache, which a
// default-policy stream only thrashes (10,000x: 6 % faster; batches that fit lose ~2 %)
template <int W, bool NT>
__device__ __forceinline__ typename Vec<W>::T bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    if constexpr (W == 4) return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, NT ? 2 : 0);
    else return __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, NT ? 2 : 0);
}

// The same with the wave-uniform part of the offset in soffset (an SGPR; the range check covers voffset + soffset,
// tools/bufcheck.hip): a streaming loop's loads then take a loop-invariant VGPR offset, so no address register is
// written while loads are in flight (hipcc otherwise drains every load at the loop header: an address VGPR it
// allocated over a pending load's destination)
template <int W, bool NT>
__device__ __forceinline__ typename Vec<W>::T bload_s(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    const int so = (int)__builtin_amdgcn_readfirstlane(soff);
    if constexpr (W == 4) return __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, so, NT ? 2 : 0);
    else return __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, so, NT ? 2 : 0);
}

__device__ __forceinline__ void write_hist(const KParams &P) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *P.hslot = P.hdesc;
}

__device__ __forceinline__ uint32_t code_of_ref(uint8_t c) {
    c = (uint8_t)(c & 0xDFu);                     // upper case
    return c == 'A' ? 1u : c == 'C' ? 2u : c == 'G' ? 4u : c == 'T' ? 8u : c == 'N' ? 15u : 1u;
}

// One entry outside the SWAR paths (lane-private LDS state; q >= 128 rows from global: rare)
__device__ __forceinline__ void ms_rare(MState &S, uint32_t code, uint32_t q, uint32_t idx,
                                        const double2 *__restrict__ lut, const Tables *__restrict__ T) {
    S.depth++;
    if (code == SPG_CODE_DEL) { S.n_del++; return; }
    if (code == SPG_CODE_SKIP) { S.n_skip++; return; }
    const int sl = slot_of(code);
    if (sl < 0) { S.n_other++; return; }
    S.cnt[sl]++;
    S.sq[sl] = sat_add31(S.sq[sl], q);
    S.qf[sl] = (uint8_t)min((uint32_t)S.qf[sl], q);
    S.first[sl] = min(S.first[sl], idx);
    const double2 t = q < 128u ? lut[q] : make_double2(T->fast[q][0], T->fast[q][1]);
    S.sl[sl] += t.x;
    S.se[sl] += q == 0 ? 1.0 : t.y;                // eps(Q0) = 1
}

// sum over a fast allele's entries of a dword: {ln(1-eps), eps} rows of the LDS LUT (row q for the
// selected bytes, whose q is in 4..127; row 0, which is zero, for every other byte: one address, so
// the lanes' reads of it broadcast instead of spreading over 128 zero rows and their banks)
__device__ __forceinline__ void lut_sums(uint32_t qw, uint32_t sel80, const double2 *__restrict__ lut, double &sl,
                                         double &se) {
    const uint32_t idx = qw & ((sel80 >> 7) * 0xFFu);
    const double2 t0 = lut[idx & 0xFFu], t1 = lut[(idx >> 8) & 0xFFu];
    const double2 t2 = lut[(idx >> 16) & 0xFFu], t3 = lut[idx >> 24];
    sl += (t0.x + t1.x) + (t2.x + t3.x);
    se += (t0.y + t1.y) + (t2.y + t3.y);
}

// sum of ln(1-eps) only (calls-only REF major of a shallow run: its sum(eps) is never used, the REF
// allele is never a call): 8-B rows, half the LDS traffic of lut_sums
__device__ __forceinline__ void lut_sl(uint32_t qw, uint32_t sel80, const double *__restrict__ l1m, double &sl) {
    const uint32_t idx = qw & ((sel80 >> 7) * 0xFFu);
    sl += (l1m[idx & 0xFFu] + l1m[(idx >> 8) & 0xFFu]) + (l1m[(idx >> 16) & 0xFFu] + l1m[idx >> 24]);
}

// A pointer read from a descriptor table is address-space generic to hipcc (flat loads: counted in both vmcnt
// and lgkmcnt, so every wait on them drains both); these assert global memory (global_load).
template <typename T>
using gptr = const T __attribute__((address_space(1))) *;
template <typename T>
__device__ __forceinline__ gptr<T> gbl(const T *p) {
    return (gptr<T>)p;
}

// wave-wide max of a per-lane count (DPP within rows, then the four row maxima)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int c = 0; c < 4; c++) v = max(v, dpp_u32(v, c));
    const uint32_t a = max((uint32_t)__builtin_amdgcn_readlane(v, 0), (uint32_t)__builtin_amdgcn_readlane(v, 16));
    const uint32_t b = max((uint32_t)__builtin_amdgcn_readlane(v, 32), (uint32_t)__builtin_amdgcn_readlane(v, 48));
    return max(a, b);
}

// MBLK: 16-B blocks per lane per load round (MBLK x 16 entries)
// prepare_variants' filters on a position's totals (:131, :151-157), a superset of the early exit
// k_finalize takes in calls-only mode: false = the position can produce no call and needs no replay
__device__ __forceinline__ bool may_call(const MState &c, uint8_t refc, const MParams &P) {
    if (c.n_other) return true;                                  // exotic: exact replay
    const uint32_t depth = c.depth;
    if ((int64_t)depth < (int64_t)P.min_td) return false;
    // AD / DP >= ratio, conservatively without a division: fl(n / d) >= r implies n >= d * r (1 - 2^-52),
    // and P.ratio_lo = r (1 - 1e-9) keeps fl(d * ratio_lo) below that; the sparse finalize then applies
    // the exact test to the listed positions
    const double dlo = (double)depth * P.ratio_lo;
    bool any = false;
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        const uint32_t n = c.cnt[k];
        any |= n != 0 && refc != nibble_char(slot_code(k)) && (int64_t)n >= P.min_ad && (double)n >= dlo;
    }
    return any;
}

}  // namespace spg
