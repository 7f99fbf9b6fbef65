// spg_kernels.hip — CDNA4 (gfx950) kernels of the pileup + genotype-likelihood engine.
//
//   k_acc_seg<W,FRESH>  process_pileup_column / process_svn (live_variant_caller.py:74-103) + pysam's
//                  base-quality filter for one deep CSR batch: a wave64 owns G consecutive columns and
//                  streams them as one sequence of 64 x 4W-entry chunks (buffer loads two chunks ahead,
//                  column descriptors in LDS behind scalar cursors).  SWAR byte tests classify 4
//                  entries per dword; the column's major (and, when frequent, second) allele takes the
//                  fast path (v_bcnt counts, v_dot4_u32_u8 quality sums, LDS {ln(1-eps), eps} table);
//                  the rare entries (other alleles, D/N, q < 4, q >= 128, IUPAC) are queued as lane
//                  slices and decoded exactly into a per-wave LDS record at column end.
//   k_merge_parts  folds the partial states of a split run of shallow batches (k_acc_tile, spg_tile.hip)
//                  into the records in batch order.
//   k_finalize     prepare_variants (:120-185) + genotype_likelihood / to_phred_scale
//                  (utils.py:12-24): per-position GL in fp64 with the reference's underflow decisions,
//                  candidate filters, GL/PL/SCORE/QUAL.  A position whose result depends on the order
//                  of fp64 roundings in the subnormal range (or that holds IUPAC alleles, or whose calls
//                  need terms calls-only mode did not accumulate) is recomputed exactly by its wave,
//                  walking the batch history (np.prod left folds in BAM order).
#include <algorithm>
#include <type_traits>

#include "spg_common.h"
#include <stdlib.h>

namespace spg {


// ------------------------------------------------------------------------------------------
// finalize: GL with the reference's underflow decisions
// ------------------------------------------------------------------------------------------
constexpr double LOG2_10_OVER_10 = 0.33219280948873623;   // log2(10)/10
constexpr double INV_LN2 = 1.4426950408889634;
constexpr double MARGIN = 1e-5;               // log2 margin around the band edges (>> rounding error)

// A value of the reference's fp64 computation, known either exactly as 0 (state 1), or accurately
// (state 0: normal, within ~1e-12 relative, l2 = its log2), or only by an upper bound (state 2,
// "band": l2 bounds log2 of the reference's value, which depends on the order of roundings in the
// subnormal range).  lv_mul follows one reference multiplication fl(a*b).
struct LV { int s; double v, l2; };
__device__ __forceinline__ LV lv_normal(double v, double l2) { return LV{0, v, l2}; }
__device__ __forceinline__ LV lv_zero() { return LV{1, 0.0, -1e300}; }
__device__ __forceinline__ LV lv_band(double ub) { return LV{2, 0.0, ub}; }
__device__ __forceinline__ LV lv_unknown() { return LV{3, 0.0, 0.0}; }   // not accumulated (calls-only)
__device__ __forceinline__ LV lv_mul(const LV &a, const LV &b) {
    if (a.s == 1 || b.s == 1) return lv_zero();                   // 0 * finite == 0
    if (a.s == 3 || b.s == 3) return lv_unknown();
    const double l2 = a.l2 + b.l2;
    if (a.s == 0 && b.s == 0) {
        if (l2 > -1022.0 + MARGIN) return lv_normal(a.v * b.v, l2);  // stays normal: one rounding
        if (l2 < -1075.0 - MARGIN) return lv_zero();                // exact product < 2^-1075 -> 0
        return lv_band(fmax(l2 + MARGIN, -1075.0) + 1.0);
    }
    const double ub = l2 + MARGIN;                                 // bound on the exact product
    if (ub < -1075.0 - MARGIN) return lv_zero();
    return lv_band(fmax(ub, -1075.0) + 1.0);                       // + half a subnormal unit
}

__device__ __forceinline__ int to_phred(double p) {      // utils.py:12-13
    if (!(p > 0.0)) return 99;
    const double r = rint(-10.0 * log10(p));
    return r < 99.0 ? (int)r : 99;
}

__device__ __forceinline__ void write_candidate(const FParams &F, const Out &O, int64_t pos, const Acc &a, int k,
                                                uint32_t code, uint32_t ad, double g, double S, double qual) {
    spg_candidate c;
    c.pos = pos; c.dp = (int32_t)a.depth; c.ad = (int32_t)ad;
    c.ref = (uint8_t)(a.misc & 0xFFu); c.alt = nibble_char(code); c.rank = (uint8_t)k;
    c.first_batch = a.first_batch;
    c.gl_linear = g;
    if (g != 0) { c.gl = log10(g); c.pl = (int32_t)rint(-10.0 * c.gl); c.gl_zero = 0; }
    else { c.gl = 0.0; c.pl = 0; c.gl_zero = 1; }
    c.score = to_phred(1.0 - (g / S));
    c.qual = qual;
    const uint32_t at = atomicAdd(&O.ctr[F.cslot].n_cand, 1u);
    if (at < (uint32_t)F.cand_cap) O.cand[at] = c;
}

__device__ __forceinline__ bool is_candidate(const FParams &F, const Acc &a, uint32_t code, uint32_t ad) {
    return (uint8_t)(a.misc & 0xFFu) != nibble_char(code) && (int64_t)ad >= F.min_ad &&
           (double)ad / (double)a.depth >= F.ratio;                            // :151-157
}

// Exact sequential recomputation of one position over the batch history (rare: subnormal band, IUPAC
// alleles, calls-only terms that were not accumulated).  np.prod is a strict left fold (utils.py:17,19)
// and N a dict-order fold (:18-22): sequential per allele, but the 16 allele codes' folds are
// independent.  The wave walks the position's entries 64 at a time (coalesced byte loads, one entry per
// lane) over the batches the replay index lists for the position; lane c owns code c's fold and takes
// the chunk's code-c factors in order through readlane, so no fold step waits on a memory load.
// Pass 1: counts, first appearance (dict order), sum(eps) and the P folds (stopped at 0: P only
// shrinks).  Pass 2: the H folds, only for alleles whose GL is not already exactly 0 through N == 0
// (H is finite, so H * 0 == 0), each stopped at 0.
struct ReplayWs {
    uint32_t cnt[16], ord[16];
    uint64_t first[16];
    double P[16], Hh[16], se[16], G[16], non[16];
    uint32_t needH, n;
};

// Walk the position's entries in history batches [from, n_hist) in accumulate order; `ord` = raw entries of the
// position in the batches before (advanced past the ones walked).  64 batches at a time: lane j resolves batch j's
// descriptor and the position's column bounds in it (two round trips for 64 batches, not per batch), a wave prefix
// sum lays their entries end to end, and the wave streams that sequence 64 entries per step — lane e finds its
// entry's batch by a binary search over the lanes' prefix (ds_bpermute, no LDS) — one step's loads in flight while
// the previous step folds.  (A live memory's position spans thousands of per-BAM batches: the per-batch walk was
// three dependent round trips each, ~15 ms for a cold replay after 2,700 BAMs.)
// (GROUPED false: batch by batch — the fused deep kernel's replays, whose history is the sample's one batch, and
// whose registers the grouped form would raise into scratch)
template <bool GROUPED, typename Fn>
__device__ __forceinline__ void replay_walk(const FParams &F, const Hist *__restrict__ H, int64_t pos, int lane,
                                            uint32_t from, uint64_t &ord, Fn &&fn) {
    const bool indexed = F.ridx.n_buckets > 0;
    uint32_t i0 = from, i1 = (uint32_t)F.n_hist;
    if (indexed) {
        const int64_t bk = pos >> RIDX_SHIFT;
        uint32_t lo = F.ridx.off[bk], hi = F.ridx.off[bk + 1];
        i1 = hi;
        while (lo < hi) {                              // a bucket's items ascend: the first batch >= from
            const uint32_t m = (lo + hi) >> 1;
            if ((uint32_t)F.ridx.items[m] < from) lo = m + 1;
            else hi = m;
        }
        i0 = lo;
    }
    if constexpr (!GROUPED) {
        for (uint32_t i = i0; i < i1; i++) {
            const int32_t b = indexed ? F.ridx.items[i] : (int32_t)i;
            const Hist h = H[b];
            const int64_t col = pos - h.pos_begin;
            if (col < 0 || col >= h.n_cols) continue;
            const uint64_t lo = h.off[col], hi = h.off[col + 1];
            // 64 entries a step, the next two steps' loads in flight (a step waited for its own load: a column of
            // 8,000 entries is 125 dependent round trips)
            auto ld = [&](uint64_t e0, uint32_t &c, uint32_t &q) {
                const uint64_t e = e0 + (uint64_t)lane;
                c = e < hi ? h.code[e] : 0xFFu;
                q = e < hi ? h.qual[e] : 0u;
            };
            uint32_t cA, qA, cB, qB, cC, qC;
            ld(lo, cA, qA);
            ld(lo + 64, cB, qB);
            for (uint64_t e0 = lo; e0 < hi; e0 += 192) {
                ld(e0 + 128, cC, qC);
                fn(cA, qA, e0 + (uint64_t)lane < hi, ord + (e0 - lo));
                if (e0 + 64 >= hi) break;
                ld(e0 + 192, cA, qA);
                fn(cB, qB, e0 + 64 + (uint64_t)lane < hi, ord + (e0 + 64 - lo));
                if (e0 + 128 >= hi) break;
                ld(e0 + 256, cB, qB);
                fn(cC, qC, e0 + 128 + (uint64_t)lane < hi, ord + (e0 + 128 - lo));
            }
            ord += hi - lo;
        }
        return;
    }
    for (uint32_t g0 = i0; g0 < i1; g0 += 64) {
        // lane j: batch g0 + j's column of this position (empty when the batch does not cover it)
        uint32_t len = 0;
        uint64_t cp = 0, qp = 0;
        if (g0 + (uint32_t)lane < i1) {
            const int32_t b = indexed ? F.ridx.items[g0 + lane] : (int32_t)(g0 + lane);
            const Hist h = H[b];
            const int64_t col = pos - h.pos_begin;
            if (col >= 0 && col < h.n_cols) {
                const uint64_t lo = h.off[col], hi = h.off[col + 1];
                len = (uint32_t)(hi - lo);
                cp = (uint64_t)(h.code + lo);
                qp = (uint64_t)(h.qual + lo);
            }
        }
        uint32_t pre = len;                            // inclusive prefix of the lengths, then exclusive
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)pre, o);
            if (lane >= o) pre += t;
        }
        const uint32_t T = (uint32_t)__builtin_amdgcn_readlane(pre, 63);
        pre -= len;
        if (T == 0) continue;
        // entry t0 + lane of the group's sequence: its batch = the last lane whose prefix is <= it
        auto fetch = [&](uint32_t t0, uint32_t &c, uint32_t &q) {
            const uint32_t gi = t0 + (uint32_t)lane;
            int k = 0;
#pragma unroll
            for (int st = 32; st >= 1; st >>= 1)
                if ((uint32_t)__shfl((int)pre, k + st) <= gi) k += st;
            const uint32_t e = gi - (uint32_t)__shfl((int)pre, k);
            const uint64_t ck = (uint64_t)(uint32_t)__shfl((int)(uint32_t)cp, k) | ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(cp >> 32), k) << 32);
            const uint64_t qk = (uint64_t)(uint32_t)__shfl((int)(uint32_t)qp, k) | ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(qp >> 32), k) << 32);
            c = 0xFFu; q = 0u;
            if (gi < T) { c = reinterpret_cast<const uint8_t *>(ck)[e]; q = reinterpret_cast<const uint8_t *>(qk)[e]; }
        };
        uint32_t cA, qA, cB, qB;
        fetch(0u, cA, qA);
        for (uint32_t t0 = 0; t0 < T; t0 += 128) {
            fetch(t0 + 64u, cB, qB);
            fn(cA, qA, t0 + (uint32_t)lane < T, ord + t0);
            if (t0 + 64u >= T) break;
            fetch(t0 + 128u, cA, qA);
            fn(cB, qB, t0 + 64u + (uint32_t)lane < T, ord + t0 + 64u);
        }
        ord += T;
    }
}

// The position's replay-cache slot (lane 0; -1: none free).  `upto` = batches its stored state covers (0: none).
__device__ __forceinline__ int32_t rcache_claim(const RCache &R, int64_t pos, uint32_t epoch, uint32_t &upto) {
    const uint64_t key = ((uint64_t)epoch << 32) | (uint64_t)(uint32_t)(pos + 1);
    const uint32_t h = (uint32_t)(((uint64_t)pos * 0x9E3779B97F4A7C15ull) >> 40) & R.mask;
    for (int i = 0; i < RCACHE_PROBE; i++) {
        const uint32_t si = (h + (uint32_t)i) & R.mask;
        unsigned long long *kp = reinterpret_cast<unsigned long long *>(&R.slot[si].key);
        const unsigned long long k = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) { upto = R.slot[si].upto; return (int32_t)si; }
        if (k == 0 || (uint32_t)(k >> 32) != epoch) {            // empty, or a slot of an older sample
            const unsigned long long old = atomicCAS(kp, k, (unsigned long long)key);
            if (old == k) { R.slot[si].upto = 0; upto = 0; return (int32_t)si; }
            if (old == key) { upto = R.slot[si].upto; return (int32_t)si; }
        }
    }
    return -1;
}

// Exact sequential recomputation of one position over the batch history (rare: subnormal band, IUPAC
// alleles, calls-only terms that were not accumulated).  np.prod is a strict left fold (utils.py:17,19)
// and N a dict-order fold (:18-22): sequential per allele, but the 16 allele codes' folds are
// independent.  The wave walks the position's entries 64 at a time (coalesced byte loads, one entry per
// lane) over the batches the replay index lists for the position; lane c owns code c's fold and takes
// the chunk's code-c factors in order through readlane, so no fold step waits on a memory load.
// Cold (no cached state): pass 1 folds counts, first appearance (dict order), sum(eps) and the P folds
// (stopped at 0: P only shrinks); pass 2 the H folds, only for alleles whose GL is not already exactly 0
// through N == 0 (H is finite, so H * 0 == 0), each stopped at 0.  Warm (F.rc holds the position's state after
// batches [0, upto)): one pass over batches [upto, n_hist) continues every fold from that state — P for every
// code, H for the codes still alive (N != 0 last time) and for codes first seen since; the state is stored back.
// rec: the position's record (HBM, or the fused accumulate's LDS image); eps(q): from_phred_scale(q)
template <bool GROUPED, typename EpsFn>
__device__ __forceinline__ void replay_wave(const FParams &F, const Hist *__restrict__ H, const Acc *rec,
                                         const Out &O, int64_t pos, ReplayWs *w, EpsFn &&eps_s) {
    const int lane = threadIdx.x & 63;
    const Acc a = *rec;
    uint32_t cnt = 0, depth = 0;
    uint64_t first = ~0ull, ord = 0;
    double P = 1.0, Hh = 1.0, se = 0.0;
    RSlot *rs = nullptr;
    uint32_t from = 0, track = 0;
    if (F.rc.slot) {
        int32_t si = -1;
        uint32_t up = 0;
        if (lane == 0) si = rcache_claim(F.rc, pos, F.epoch, up);
        si = __builtin_amdgcn_readfirstlane(si);
        up = __builtin_amdgcn_readfirstlane(up);
        if (si >= 0) {
            rs = F.rc.slot + si;
            if (up > 0 && up <= (uint32_t)F.n_hist) {
                from = up;
                depth = rs->depth;
                ord = rs->ord;
                const uint32_t alive = rs->alive;
                if (lane < 16) { cnt = rs->cnt[lane]; first = rs->first[lane]; P = rs->P[lane]; se = rs->se[lane]; }
                // H folds continue for the alive codes and start for codes not seen yet
                const bool tr = lane < 16 && (cnt == 0 || ((alive >> lane) & 1u));
                if (tr && cnt) Hh = rs->H[lane];
                track = (uint32_t)__ballot(tr) & 0xFFFFu;
            }
        }
    }
    for (int attempt = 0; attempt < 2; attempt++) {
        const bool warm = from > 0;
        replay_walk<GROUPED>(F, H, pos, lane, from, ord, [&](uint32_t c, uint32_t q, bool valid, uint64_t base) {
            const bool pass = valid && (int)q >= F.min_bq;
            depth += (uint32_t)__popcll(__ballot(pass));
            const bool isc = pass && c < 16u;
            const double e = isc ? eps_s(q) : 0.0;
            const double om = (warm && isc) ? 1.0 - e : 0.0;
            uint64_t todo = __ballot(isc);
            while (todo) {
                const int j0 = (int)__builtin_ctzll(todo);
                const uint32_t cc = __builtin_amdgcn_readlane(c, j0);
                const bool mine = isc && c == cc;
                const uint64_t bm = __ballot(mine);
                todo &= ~bm;
                const double es = dsum_f64(mine ? e : 0.0);
                double pc = rl_f64(P, (int)cc);
                for (uint64_t m = bm; m && pc != 0.0; m &= m - 1) pc = pc * rl_f64(e, (int)__builtin_ctzll(m));
                double hc = 1.0;
                if (warm && ((track >> cc) & 1u)) {
                    hc = rl_f64(Hh, (int)cc);
                    for (uint64_t m = bm; m && hc != 0.0; m &= m - 1) hc = hc * rl_f64(om, (int)__builtin_ctzll(m));
                }
                if (lane == (int)cc) {
                    if (cnt == 0) first = base + (uint64_t)j0;
                    cnt += (uint32_t)__popcll(bm);
                    se += es;
                    P = pc;
                    if (warm && ((track >> cc) & 1u)) Hh = hc;
                }
            }
        });
        if (lane < 16) { w->cnt[lane] = cnt; w->first[lane] = first; w->P[lane] = P; w->se[lane] = se; }
        wave_sync();
        if (lane == 0) {
            int n = 0;                                     // dict order: codes by first appearance
            for (int c = 0; c < 16; c++) {
                if (!w->cnt[c]) continue;
                int at = n++;
                while (at > 0 && w->first[w->ord[at - 1]] > w->first[c]) { w->ord[at] = w->ord[at - 1]; at--; }
                w->ord[at] = (uint32_t)c;
            }
            uint32_t need = 0;
            for (int h = 0; h < n; h++) {                  // N_h = ((1.0 * P_a1) * P_a2) ... over a != h
                double non = 1.0;
                for (int j = 0; j < n; j++)
                    if (j != h) non = non * w->P[w->ord[j]];
                w->non[h] = non;
                if (non != 0.0) need |= 1u << w->ord[h];
            }
            w->n = (uint32_t)n;
            w->needH = need;
        }
        wave_sync();
        // a code needing H whose fold was not tracked cannot occur (N only shrinks); if it did, fold from scratch
        if (!warm || (w->needH & ~track) == 0) break;
        from = 0; ord = 0; depth = 0; cnt = 0; first = ~0ull; P = 1.0; Hh = 1.0; se = 0.0; track = 0;
        wave_sync();
    }
    const uint32_t needH = w->needH;
    if (from == 0 && needH) {
        uint64_t ord2 = 0;
        replay_walk<GROUPED>(F, H, pos, lane, 0u, ord2, [&](uint32_t c, uint32_t q, bool valid, uint64_t) {
            const bool isc = valid && (int)q >= F.min_bq && c < 16u && ((needH >> c) & 1u);
            const double om = isc ? 1.0 - eps_s(q) : 0.0;
            uint64_t todo = __ballot(isc);
            while (todo) {
                const uint32_t cc = __builtin_amdgcn_readlane(c, (int)__builtin_ctzll(todo));
                const uint64_t bm = __ballot(isc && c == cc);
                todo &= ~bm;
                double hc = rl_f64(Hh, (int)cc);
                for (uint64_t m = bm; m && hc != 0.0; m &= m - 1) hc = hc * rl_f64(om, (int)__builtin_ctzll(m));
                if (lane == (int)cc) Hh = hc;
            }
        });
    }
    if (lane < 16) w->Hh[lane] = Hh;
    if (rs) {                                          // the state after every batch, for the next replay
        if (lane < 16) {
            rs->cnt[lane] = cnt; rs->first[lane] = first; rs->P[lane] = P; rs->se[lane] = se; rs->H[lane] = Hh;
        }
        if (lane == 0) { rs->depth = depth; rs->ord = ord; rs->alive = needH; rs->upto = (uint32_t)F.n_hist; }
    }
    wave_sync();
    if (lane == 0) {
        const int n = (int)w->n;
        const bool evaluated = (int64_t)depth >= (int64_t)F.min_td;
        double S = 0.0;
        for (int h = 0; h < n; h++) {
            w->G[h] = w->Hh[w->ord[h]] * w->non[h];
            S = S + w->G[h];
        }
        if (S == 0) S = 1.0;
        uint8_t flags = F.table ? O.flags[pos] : 0;
        if (evaluated) {
            double *gl = O.gl + pos * NSLOT;
            for (int h = 0; h < n; h++) {
                const uint32_t c = w->ord[h];
                const int s = slot_of(c);
                if (s >= 0 && F.table) gl[s] = w->G[h];
                if (is_candidate(F, a, c, w->cnt[c])) {
                    write_candidate(F, O, pos, a, h, c, w->cnt[c], w->G[h], S, w->se[c] / (double)w->cnt[c]);
                    flags |= SPG_F_CANDIDATE;
                }
            }
        }
        if (F.table) O.flags[pos] = flags;
        if (depth != a.depth) atomicOr(&O.ctr[F.cslot].err, 1u);   // history / accumulator mismatch
        const uint32_t at = atomicAdd(&O.ctr[F.cslot].n_detail, 1u);
        if (at < (uint32_t)F.detail_cap) {
            spg_detail *d = O.detail + at;
            d->pos = pos; d->depth = depth; d->n_alleles = (uint8_t)n;
            d->pad[0] = d->pad[1] = d->pad[2] = 0;
            for (int k = 0; k < 16; k++) {
                d->code[k] = k < n ? (uint8_t)w->ord[k] : 0xFF;
                d->count[k] = k < n ? w->cnt[w->ord[k]] : 0;
                d->gl[k] = (k < n && evaluated) ? w->G[k] : __builtin_nan("");
            }
        }
    }
    wave_sync();
}

// prepare_variants for one position (one lane).  Returns true when the position needs the exact replay.
// rec: the position's record (HBM, or the fused accumulate's LDS image).  CO: calls only at compile
// time (no per-position table; the fused accumulate's instantiation).
template <bool CO>
__device__ __forceinline__ bool finalize_position(const FParams &F, const Acc *rec,
                                                  const Tables *__restrict__ T, const Out &O, int64_t pos,
                                                  double *sink) {
    const double NaN = __builtin_nan("");
    const bool table = !CO && F.table;
    if (!table) {
        // calls only: the header and the counts (first 52 bytes, one round trip) decide whether this
        // position can produce a call at all; only then is the rest of the record read
        const uint4 h0 = reinterpret_cast<const uint4 *>(rec)[0];
        const uint4 h1 = reinterpret_cast<const uint4 *>(rec)[1];
        const uint4 c4 = reinterpret_cast<const uint4 *>(rec)[2];
        const uint32_t c5 = reinterpret_cast<const uint32_t *>(rec)[12];
        // not in memory (CO: the fused accumulate's own LDS image, of this epoch by construction)
        if ((!CO && h1.w != F.epoch) || h0.y == 0) return false;
        if ((int64_t)h0.x < (int64_t)F.min_td) return false;             // not evaluated (:131)
        if (!(h0.w & MISC_EXOTIC)) {
            const uint32_t cnt[NSLOT] = {c4.x, c4.y, c4.z, c4.w, c5};
            const uint8_t refc = (uint8_t)(h0.w & 0xFFu);
            bool any = false;
#pragma unroll
            for (int k = 0; k < NSLOT; k++)
                any |= cnt[k] != 0 && refc != nibble_char(slot_code(k)) && (int64_t)cnt[k] >= F.min_ad &&
                       (double)cnt[k] / (double)h0.x >= F.ratio;                         // :151-157
            if (!any) return false;
        }
    }
    const Acc a = *rec;
    const bool live = (CO || a.epoch == F.epoch) && a.first_batch != 0;
    uint32_t *cnt8 = O.counts + pos * SPG_NCOUNT;
    double *gl = table ? O.gl + pos * NSLOT : sink;     // scratch-free sink (CO: none)
    if (table) {
        O.depth[pos] = live ? a.depth : 0u;
        O.order[pos] = live ? a.order : 0u;
        O.first[pos] = live ? a.first_batch : 0u;
#pragma unroll
        for (int k = 0; k < NSLOT; k++) { cnt8[k] = live ? a.cnt[k] : 0u; gl[k] = NaN; }
        cnt8[5] = live ? a.n_del : 0u; cnt8[6] = live ? a.n_skip : 0u; cnt8[7] = live ? a.n_other : 0u;
    }
    if (!live) { if (table) O.flags[pos] = 0; return false; }
    uint8_t flags = SPG_F_PRESENT;
    const bool evaluated = (int64_t)a.depth >= (int64_t)F.min_td;   // :131
    if (evaluated) flags |= SPG_F_EVALUATED;
    if (a.misc & MISC_EXOTIC) {       // IUPAC / '=' alleles: the exact replay tabulates every allele
        if (table) O.flags[pos] = flags | SPG_F_EXOTIC | SPG_F_REPLAYED;
        return true;
    }
    if (!evaluated) { if (table) O.flags[pos] = flags; return false; }
    const int n = (int)(a.order & 7u);
    const uint32_t skip = (a.misc >> MISC_SKIP_SHIFT) & 0x1Fu;
    const uint32_t skip_se = skip & ~(a.misc >> MISC_SEONLY_SHIFT);   // slots whose Σ eps is incomplete too
    uint32_t slot[NSLOT], cnts[NSLOT];
    LV Pv[NSLOT], Hv[NSLOT];
    double Sv[NSLOT];
    // per-allele P (= prod eps, utils.py:19) and H (= prod 1-eps, utils.py:17) in dict order
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        slot[k] = (a.order >> (3 + 3 * k)) & 7u;
        cnts[k] = 0; Sv[k] = 0.0; Pv[k] = lv_normal(1.0, 0.0); Hv[k] = lv_normal(1.0, 0.0);
        if (k >= n) continue;              // only the alleles present (no exp for empty slots)
        uint32_t c_ = 0, sq = 0, qf = 0; double sl = 0.0, se = 0.0;
#pragma unroll
        for (int j = 0; j < NSLOT; j++)
            if (slot[k] == (uint32_t)j) { c_ = a.cnt[j]; sq = a.sq[j]; qf = a.qf[j]; sl = a.sl[j]; se = a.se[j]; }
        cnts[k] = c_;
        Sv[k] = se;
        // P: log10 P = -sum(q)/10 up to (n+2) ulp; exact zero proven when every factor < 1/2
        if (sq <= 3076u) Pv[k] = lv_normal(T->p10k[sq / 10u] * T->eps[sq % 10u], -(double)sq * LOG2_10_OVER_10);
        else if (sq >= 3245u && qf >= 4u) Pv[k] = lv_zero();
        else Pv[k] = lv_band(-1022.0 + 2 * MARGIN);
        // H: exp(sum ln(1-eps)); exactly 0 when a Q0 entry is present (1 - 1.0 == 0)
        if (qf == 0u) Hv[k] = lv_zero();
        else if ((skip >> slot[k]) & 1u) Hv[k] = lv_unknown();
        else {
            const double l2 = sl * INV_LN2;
            Hv[k] = l2 > -1022.0 + MARGIN ? lv_normal(exp(sl), l2) : lv_band(-1022.0 + 2 * MARGIN);
        }
    }
    double G[NSLOT];
    bool band = false, unknown = false, cand_needs_s = false;
#pragma unroll
    for (int h = 0; h < NSLOT; h++) {
        // N = ((1.0 * P_a1) * P_a2) ... over a != h in dict order (utils.py:18-22), GL = H * N
        LV c = lv_normal(1.0, 0.0);
#pragma unroll
        for (int j = 0; j < NSLOT; j++)
            if (j != h && j < n) c = lv_mul(c, Pv[j]);
        const LV g = lv_mul(Hv[h], c);
        if (h < n && g.s == 2) band = true;
        G[h] = g.s == 0 ? g.v : (g.s == 3 ? NaN : 0.0);
        if (h < n && g.s == 3) unknown = true;
        // a candidate needs S = sum(GL) unless its own GL is exactly 0 (SCORE = 0 for any S)
        // a candidate whose slot skipped Σ eps as well lacks its QUAL: exact replay (a REF-major skip on a
        // slot that is not the record's REF: a reference switch between batches)
        if (h < n && ((skip_se >> slot[h]) & 1u) && is_candidate(F, a, slot_code((int)slot[h]), cnts[h])) band = true;
        if (h < n && g.s != 1 && is_candidate(F, a, slot_code((int)slot[h]), cnts[h])) {
            cand_needs_s = true;
            if (g.s == 3) band = true;        // its own GL depends on terms not accumulated
        }
    }
    // unknown (not accumulated) GL terms only matter if a call needs S: then replay exactly
    if (band || (unknown && cand_needs_s)) {
        if (table) O.flags[pos] = flags | SPG_F_REPLAYED;
        return true;
    }
    if (unknown) flags |= SPG_F_PARTIAL;
    double S = 0.0;
#pragma unroll
    for (int k = 0; k < NSLOT; k++)
        if (k < n && !unknown) S = S + G[k];                 // :145
    if (S == 0) S = 1.0;                                     // :146 (every call has GL 0 if unknown)
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        if (k < n) {
#pragma unroll
            for (int j = 0; j < NSLOT; j++)
                if (!CO && slot[k] == (uint32_t)j) gl[j] = G[k];
            const uint32_t code = slot_code((int)slot[k]);
            if (is_candidate(F, a, code, cnts[k])) {
                write_candidate(F, O, pos, a, k, code, cnts[k], G[k], S, Sv[k] / (double)cnts[k]);
                flags |= SPG_F_CANDIDATE;
            }
        }
    }
    if (table) O.flags[pos] = flags;
    return false;
}

// Column finishing is batched: at a column's end the wave only reduces its fast-path sums into a
// ColSum (lane 0) next to the column's rare record (both in a per-wave LDS ring of NB slots).  When
// the ring is full (and at the wave's end) lane j < NB assembles column j's 160-B Acc record — the
// merge of rare record, fast sums and (not FRESH) the record already in HBM — in LDS, and the wave
// writes the records with 16-B stores, ten lanes per record.  The serial per-column work of
// process_pileup_column / process_svn's dict bookkeeping (:77-101) thus runs lane-parallel.
#ifndef SPG_NT_MIB
#define SPG_NT_MIB 192       // batches whose entries exceed this stream with non-temporal loads
#endif
#ifndef SPG_SEG_WPE
#define SPG_SEG_WPE 4
#endif
constexpr int NB = SPG_NB;   // columns a wave finishes together
constexpr int KW = 4;        // waves per k_acc_seg workgroup

struct ColSum {              // one finished column's fast-path statistics (written by lane 0)
    uint32_t M, M2, fc, fs, fc2, fs2, ffirst, ffirst2;
    uint32_t skipped, cj, crefc, fsamp;   // skipped: bit 0 the major's, bit 1 the second allele's likelihood
                                          // sums were not accumulated; fsamp: first sample of a
                                          // multi-sample column (0 otherwise)
    double fl, fe, fl2, fe2;
};
static_assert(sizeof(ColSum) == 80, "ColSum");

// prepare_variants' filters (:131, :151-157) on a finished record's LDS image, division-free and conservative
// (P.ratio_lo = ratio (1 - 1e-9)): false = the position cannot produce a call and needs no replay
__device__ __forceinline__ bool may_call_img(const KParams &P, const Acc *r) {
    const uint32_t depth = r->depth, misc = r->misc;
    if (misc & MISC_EXOTIC) return true;               // exotic allele: exact replay
    if ((int64_t)depth < (int64_t)P.min_td) return false;
    const double dlo = (double)depth * P.ratio_lo;
    const uint8_t refc = (uint8_t)(misc & 0xFFu);
    bool maybe = false;
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        const uint32_t n = r->cnt[k];
        maybe |= n != 0 && refc != nibble_char(slot_code(k)) && (int64_t)n >= P.min_ad && (double)n >= dlo;
    }
    return maybe;
}

// Lane-per-column record assembly (lane j of the finisher; R / S in LDS, out = the LDS image).
template <bool FRESH>
__device__ __forceinline__ void assemble_record(const KParams &P, const Acc *__restrict__ A, const WaveRare *R,
                                                const ColSum *S, Acc *out) {
    uint4 h0 = make_uint4(0, 0, 0, 0), h1 = make_uint4(0, 0, 0, 0);
    bool fresh = FRESH;
    if constexpr (!FRESH) {
        h0 = reinterpret_cast<const uint4 *>(A)[0];
        h1 = reinterpret_cast<const uint4 *>(A)[1];
        fresh = h1.w != P.epoch;                    // record of an older sample: start afresh
        if (fresh) { h0 = make_uint4(0, 0, 0, 0); h1 = make_uint4(0, 0, 0, 0); }
    }
    const uint32_t M = S->M, M2 = S->M2, fc = S->fc, fc2 = S->fc2;
    const int Ms = fc ? slot_of(M) : -1;
    const int s2 = (fc2 && M2 != SPG_CODE_DEL && M2 != SPG_CODE_SKIP) ? slot_of(M2) : -1;
    const uint32_t have = order_mask(h0.z);
    uint32_t newmask = 0, first[NSLOT];
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        uint32_t c = R->cnt[k], sq = R->sq[k], qf = R->qf[k];
        double sl = R->sl[k], se = R->se[k];
        first[k] = R->first[k];
        if (k == Ms) {
            c += fc; sq += S->fs; sl += S->fl; se += S->fe;
            qf = min(qf, (uint32_t)P.qlo); first[k] = min(first[k], S->ffirst);
        }
        if (k == s2) {
            c += fc2; sq += S->fs2; sl += S->fl2; se += S->fe2;
            qf = min(qf, (uint32_t)P.qlo); first[k] = min(first[k], S->ffirst2);
        }
        uint32_t oc = 0, osq = 0, oqf = 0;
        double osl = 0.0, ose = 0.0;
        if (!fresh) { oc = A->cnt[k]; osq = A->sq[k]; oqf = A->qf[k]; osl = A->sl[k]; ose = A->se[k]; }
        if (c) {
            if (!((have >> k) & 1u)) newmask |= 1u << k;
            if (oc) {                                // absent slots' sums may hold stale bytes
                qf = min(oqf, qf);
                const uint64_t t = (uint64_t)osq + sq;
                sq = t > 0x80000000ull ? 0x80000000u : (uint32_t)t;
                sl = osl + sl; se = ose + se;
            } else {
                sq = sq > 0x80000000u ? 0x80000000u : sq;
            }
            out->cnt[k] = oc + c; out->sq[k] = sq; out->qf[k] = (uint8_t)qf; out->sl[k] = sl; out->se[k] = se;
        } else {
            out->cnt[k] = oc; out->sq[k] = osq; out->qf[k] = (uint8_t)oqf; out->sl[k] = osl; out->se[k] = ose;
        }
    }
    out->qf[5] = out->qf[6] = out->qf[7] = 0;
    if (h0.y == 0) { h0.y = P.batch_seq + S->fsamp; h0.w = S->crefc; }   // first visit (:77-85)
    h0.x += R->depth + fc + fc2;                                      // :87
    h0.z = merge_order(h0.z, newmask, first);
    if (R->n_other) h0.w |= MISC_EXOTIC;
    if ((S->skipped & 1u) && Ms >= 0) {
        h0.w |= (1u << Ms) << MISC_SKIP_SHIFT;
        h0.w &= ~((1u << Ms) << MISC_SEONLY_SHIFT);           // its Σ eps is incomplete as well
    }
    if ((S->skipped & 2u) && s2 >= 0) {                       // Σ ln(1-eps) incomplete, Σ eps complete
        const uint32_t b = 1u << s2;
        const bool se_ok = !(h0.w & (b << MISC_SKIP_SHIFT)) || (h0.w & (b << MISC_SEONLY_SHIFT));
        h0.w |= b << MISC_SKIP_SHIFT;
        if (se_ok) h0.w |= b << MISC_SEONLY_SHIFT;
    }
    h1.x += R->n_del + (M2 == SPG_CODE_DEL ? fc2 : 0u);
    h1.y += R->n_skip + (M2 == SPG_CODE_SKIP ? fc2 : 0u);
    h1.z += R->n_other;
    h1.w = P.epoch;
    reinterpret_cast<uint4 *>(out)[0] = h0;
    reinterpret_cast<uint4 *>(out)[1] = h1;
}


struct RareItem {            // one lane's chunk slice (up to 16 entries) holding rare entries
    uint32_t c[4], q[4];    // (its column-relative offset is kept beside, in rqo)
};

struct Dual2 {              // per-lane partial sums of a wave's second fast allele
    double sl[64], se[64];
    uint32_t cnt[64], sq[64];
};

struct ColDesc {             // one column of a wave's segment (LDS, 16 B; the non-fused instantiations)
    uint32_t a, pre, e;     // 4W-aligned first chunk, first chunk index, end rel. to a (chunks = ceil(e / STEP))
    uint32_t bic;           // start rel. to a (bits 0-3) | column within the group (4-9) | REF char (10-17)
};

// Segment streaming: wave w owns G consecutive columns and walks them as ONE stream of 64 x 4W-entry
// chunks (each column's chunks start at its 4W-aligned first entry), loaded two chunks ahead into
// three register sets across column boundaries, so a column start costs no memory latency.
// Loads go through one wave-uniform buffer descriptor per array over the segment (range-checked:
// chunks past the end read zeros).  Per column: allele vote on its first chunk, SWAR/LUT fast path
// for the major allele, exact rare path into the wave's LDS record, then a cooperative merge.
// WPE: minimum waves per SIMD the register allocation must allow.  4 (128 VGPRs) for mid-depth
// batches, whose waves stream few chunks per column and need occupancy to hide the column starts;
// 3 (up to 168 VGPRs, no spills) for deep batches, where the chunk loop dominates.
// The fused accumulate's finalize (k_acc_seg<..., FUSE>, after the wave's loop, for the lanes whose
// column passed the pre-check): prepare_variants (:120-185) on the ring's records, whose images finish()
// left in LDS; lane j evaluates column j,
// candidates go straight to the call table, and the wave replays the few positions that need the
// exact fold over this batch's column (the sample's only batch).
__device__ __forceinline__ void fused_tail(const FParams &F, const Out &O, const Tables *__restrict__ T, int64_t pos0,
                                         uint32_t nfin, const ColSum *CS, const Acc *img, ReplayWs *ws,
                                         const Hist *hdl, const double2 *lut) {
    const int lane = threadIdx.x & 63;
    const uint32_t cjl = (uint32_t)lane < nfin ? CS[lane].cj : 0u;
    const int64_t pos = pos0 + (int64_t)cjl;
    const bool need = (uint32_t)lane < nfin && finalize_position<true>(F, img + lane, T, O, pos, nullptr);
    uint64_t rb = __ballot(need);
    if (!rb) return;
    if (need) atomicAdd(&O.ctr[F.cslot].n_band, 1u);
    while (rb) {
        const int j = (int)__builtin_ctzll(rb);
        rb &= rb - 1;
        const int64_t pj = pos0 + (int64_t)(uint32_t)__builtin_amdgcn_readlane(cjl, j);
        replay_wave<false>(F, hdl, img + j, O, pj, ws, [&](uint32_t q) {
            return q == 0u ? 1.0 : lut[q < 128u ? q : q + 128u].y;     // from_phred_scale (eps(Q0) = 1)
        });
    }
}

// FUSE (a FRESH deep batch that is the sample's only batch, finalized calls-only: spg_finalize launches
// it in place of accumulate + k_finalize): each wave owns G <= NB columns, so its one ring holds every
// record it writes; after the loop lane j runs prepare_variants' per-position logic on record j's LDS
// image and the wave replays the few positions that need the exact fold — one launch per sample.
template <int W, bool FRESH, int WPE, bool NT, bool FUSE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_acc_seg(KParams P, const uint64_t *__restrict__ off,
                                                 const uint8_t *__restrict__ code, const uint8_t *__restrict__ qual,
                                                 const uint8_t *__restrict__ ref, const Tables *__restrict__ T,
                                                 Acc *__restrict__ acc) {
    using V = typename Vec<W>::T;
    constexpr uint32_t ALIGN = 4 * W;
    constexpr uint32_t STEP = 64 * ALIGN;               // entries per chunk
    constexpr uint32_t QCAP = 64;                      // per-wave queue of lane slices holding rare entries (>= 64:
                                                       // a drain must leave room for every lane's slice)
    // LUT rows 0..127: {ln(1-eps), eps} for q < 128; rows 128..255: {0, 0} (the fast path's index
    // for entries that are not fast); rows 256..383: q = 128..255 for the rare path
    __shared__ double2 lut[384];
    __shared__ WaveRare rare[KW][NB];
    __shared__ ColSum csum[KW][NB];
    __shared__ __align__(16) RareItem rqueue[KW][QCAP];   // FUSE: the replay workspace after the loop
    static_assert(sizeof(ReplayWs) <= sizeof(RareItem) * QCAP, "ReplayWs aliases a wave's queue");
    __shared__ int32_t rqo[KW][QCAP];
    __shared__ uint32_t rqr[KW][QCAP];
    __shared__ Dual2 dual2[KW];
    __shared__ Acc accimg[KW][NB];
    __shared__ ColDesc coldesc[KW][FUSE ? 1 : (W == 4 ? SPG_GMAX_DEEP : SPG_GMAX)];
    __shared__ Hist hdl;                                // FUSE: this batch's descriptor for the replay
    const uint64_t we = P.wtime ? __builtin_amdgcn_s_memrealtime() : 0;   // SPG_WAVE_TIMES: wave entry
    // the batch's history descriptor, first (consumed at once: kept live, hipcc would park it in scratch)
    write_hist(P);
    if (FUSE && threadIdx.x == 0) hdl = P.hdesc;
    const int lane = threadIdx.x & 63;
    const uint32_t bid = P.rot ? (blockIdx.x + P.rot) % gridDim.x : blockIdx.x;
    const int64_t wave = (int64_t)bid * KW + (threadIdx.x >> 6);
    // deep_list (the long columns of a shallow batch): the waves stride over the listed columns, one
    // column each; otherwise one group of G consecutive columns per wave
    const bool listed = W == 1 && P.deep_n != nullptr;  // (W = 4: compile-time off; the loop runs once)
    // A wave's own group: its CSR offsets and REF chars are loaded before the LUT, so the two round
    // trips of a starting wave overlap (the LUT's wait covers both)
    const bool tail0 = !listed && wave >= (int64_t)P.w1;
    const int64_t g00 = tail0 ? (int64_t)P.w1 * P.G + (wave - P.w1) * P.G2 : wave * P.G;
    const int ng0 = (int)max((int64_t)0, min((int64_t)(tail0 ? P.G2 : P.G), P.n_cols - g00));
    uint64_t ob0 = 0, oe0 = 0;
    uint32_t refc0 = 0, fsv0 = 0;
    if (!listed && lane < ng0) {
        ob0 = off[g00 + lane]; oe0 = off[g00 + lane + 1]; refc0 = ref[P.pos_begin + g00 + lane];
        if (P.fsamp) fsv0 = P.fsamp[g00 + lane];
    }
    if constexpr (FUSE) {
        if (blockIdx.x == 0 && threadIdx.x == 0) P.fused->O.ctr[P.fused->F.cslot ^ 1u] = Counters{0, 0, 0, 0};   // next call's slot
    }
    for (uint32_t q = threadIdx.x; q < 256u; q += 64u * KW) {
        lut[q] = q < 128u ? make_double2(T->fast[q][0], T->fast[q][1]) : make_double2(0.0, 0.0);
        if (q >= 128u) lut[q + 128u] = make_double2(T->fast[q][0], T->fast[q][1]);
    }
    __syncthreads();
    const int64_t n_items = listed ? (int64_t)*P.deep_n : wave + 1;
    const int64_t istride = listed ? (int64_t)gridDim.x * KW : 1;
    for (int64_t item = wave; item < n_items; item += istride) {
    const int64_t g0 = listed ? (int64_t)P.deep_list[item] : g00;
    if (g0 >= P.n_cols) continue;
    const int ng = listed ? 1 : ng0;
    // SPG_TRACE: lane 0 posts (stage, a, b, c) to host-mapped memory, so a fault leaves each wave's
    // last step readable by the host
    auto prog = [&](uint32_t stage, uint32_t a, uint32_t b, uint32_t c) {
        if (P.prog && lane == 0) {
            uint32_t *pp = reinterpret_cast<uint32_t *>(P.prog + wave);
            __hip_atomic_store(pp + 1, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(pp + 2, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(pp + 3, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(pp, stage, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    };
    prog(1, (uint32_t)g0, (uint32_t)ng, 0);
    // SPG_WAVE_TIMES (profiling): wave timeline in s_memrealtime ticks
    const uint64_t wt0 = P.wtime ? __builtin_amdgcn_s_memrealtime() : 0;
    WaveRare *RR = rare[threadIdx.x >> 6];             // rare records of the ring's columns
    ColSum *CS = csum[threadIdx.x >> 6];
    Dual2 *D2 = dual2 + (threadIdx.x >> 6);
    Acc *img = accimg[threadIdx.x >> 6];
    uint32_t nb = 0;                                   // columns in the finishing ring (uniform)
    ColDesc *CD = coldesc[threadIdx.x >> 6];
    RareItem *Q = rqueue[threadIdx.x >> 6];
    int32_t *QO = rqo[threadIdx.x >> 6];
    uint32_t *QR = rqr[threadIdx.x >> 6];
    uint32_t qn = 0;                                   // queued lane slices (wave-uniform)
    // Drain: lane k decodes queued slice k (its rare entries are few) into its column's LDS rare
    // record with LDS atomics.  A queued slice carries its column-relative offset (QO) and its ring
    // slot (QR bits 0-2), so the drain runs only when the queue is full or the ring is finished.
    int32_t bl = 0, el = 0;                    // column bounds relative to its first chunk
    uint32_t mrep = 0, M = 1;
    bool dual = false;
    uint32_t mrep2 = 0, M2 = 0;
    bool sem = true;                           // the major is not the REF char (calls-only mode skips REF sums)
    bool skipped = false;                      // this column's major skipped its likelihood sums
    bool skipped2 = false;                     // ... and its second allele (FUSE dual mode)
    auto drain = [&]() __attribute__((always_inline)) {
        prog(3, qn, nb, 0);
        wave_sync();
        for (uint32_t b0 = 0; b0 < qn; b0 += 64) {
            if (b0 + lane < qn) {
                const RareItem *it = Q + b0 + lane;
                const int32_t o = QO[b0 + lane];
                uint32_t rb = QR[b0 + lane];           // bit 8 b + 7 - d: byte b of dword d is rare
                WaveRare *R = RR + (rb & 7u);
                rb &= ~15u;
                while (rb) {
                    const uint32_t p = (uint32_t)__builtin_ctz(rb);
                    rb &= rb - 1;
                    const uint32_t b = p >> 3, d = 7u - (p & 7u);
                    const uint32_t c = (it->c[d] >> (8u * b)) & 0xFFu, q = (it->q[d] >> (8u * b)) & 0xFFu;
                    if ((int)q >= P.min_bq)
                        rare_entry(R, c, q, (uint32_t)(o + 4 * (int32_t)d) + b, lut, T);
                }
            }
        }
        qn = 0;
        wave_sync();
    };

    // The ring's n records from their LDS images (16 B per lane, ten lanes per record).
    auto store_ring = [&](uint32_t n) __attribute__((always_inline)) {
        Acc *base = acc + P.pos_begin + g0;
        for (uint32_t t = (uint32_t)lane; t < 10u * n; t += 64u) {
            const uint32_t r = t / 10u, piece = t - 10u * r;
            if (P.dbg && CS[r].cj >= (uint32_t)ng) {                   // SPG_TRACE: record outside the group
                atomicAdd(P.dbg + 2, 1u);
                P.dbg[3] = CS[r].cj | ((uint32_t)ng << 8) | (r << 16) | (n << 24);
                continue;
            }
            reinterpret_cast<uint4 *>(base + CS[r].cj)[piece] = reinterpret_cast<const uint4 *>(img + r)[piece];
        }
    };
    // Finish the ring: drain the queue, lane j assembles column j's record in LDS, the wave stores the
    // records.
    auto finish = [&]() __attribute__((always_inline)) {
        if (qn) drain();
        else wave_sync();
        if ((uint32_t)lane < nb) {
            const ColSum *S = CS + lane;
            assemble_record<FRESH>(P, acc + P.pos_begin + g0 + S->cj, RR + lane, S, img + lane);
        }
        wave_sync();
        prog(4, nb, CS[0].cj, CS[nb - 1].cj);
        store_ring(nb);
        if (!FUSE && P.list) {                  // calls-only listing: the ring's records that may call
            const bool maybe = (uint32_t)lane < nb && may_call_img(P, img + lane);
            const uint64_t bm = __ballot(maybe);
            if (bm) {
                uint32_t at = 0;
                if (lane == 0) at = atomicAdd(P.n_list, (uint32_t)__popcll(bm));
                at = (uint32_t)__builtin_amdgcn_readfirstlane(at);
                if (maybe)
                    P.list[at + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u))] =
                        P.pos_begin + g0 + (int64_t)CS[lane].cj;
            }
        }
        nb = 0;
        wave_sync();
    };

    // lane j < ng describes column g0 + j
    uint64_t ob = 0, oe = 0;
    uint32_t refc = 0;
    uint32_t fsv = 0;                    // multi-sample batches: first sample holding entries of the column
    if (!listed) {
        ob = ob0; oe = oe0; refc = refc0; fsv = fsv0;
    } else if (lane < ng) {
        ob = off[g0 + lane]; oe = off[g0 + lane + 1]; refc = ref[P.pos_begin + g0 + lane];
        if (P.fsamp) fsv = P.fsamp[g0 + lane];
    }
    if (P.dbg && lane < ng && (oe < ob || oe > P.n_entries)) {       // SPG_TRACE: bad CSR offsets
        atomicAdd(P.dbg, 1u);
        P.dbg[1] = (uint32_t)(g0 + lane);
        ob = oe = 0;
    }
    // (the lane builtins return int: widen through uint32_t, or offsets >= 2^31 sign-extend into a
    // wild segment base)
    const uint64_t sb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)ob) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(ob >> 32)) << 32);
    const uint64_t base = sb & ~(uint64_t)(ALIGN - 1);
    const uint64_t send = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)oe, ng - 1) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(oe >> 32), ng - 1) << 32);
    const uint32_t nbytes = (uint32_t)(((send - base) + ALIGN - 1) & ~(uint64_t)(ALIGN - 1));
    const __amdgpu_buffer_rsrc_t rc = column_rsrc(code + base, nbytes), rq = column_rsrc(qual + base, nbytes);
    const uint32_t b_rel = (uint32_t)(ob - base), e_rel = (uint32_t)(oe - base);
    const uint32_t a_rel = b_rel & ~(ALIGN - 1);
    const uint32_t len = (uint32_t)(oe - ob);
    const uint32_t nch = (lane < ng && len > 0 && len >= P.t_deep) ? (e_rel - a_rel + STEP - 1) / STEP : 0u;
    // exclusive prefix of the chunk counts
    uint32_t pre = nch;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(pre, o);
        if (lane >= o) pre += t;
    }
    const uint32_t total = __builtin_amdgcn_readlane(pre, 63);   // SGPR: loop bounds stay scalar
    pre -= nch;
    if (total == 0) continue;
    // Column descriptors of the columns with chunks stay in their lanes (lane j: the group's column j); the loop walks
    // them with two scalar cursors (consumption and prefetch) over the ballot of lanes with chunks, reading a column's
    // fields with v_readlane into SGPRs: no VGPR is written when a cursor moves.  (They were compacted into LDS, and
    // the LDS read's address register — allocated over a pending chunk load's destination — made hipcc drain every
    // load in flight each time the prefetch cursor entered a column.)
    // (The non-fused instantiations keep the descriptors compacted in LDS as before: three more VGPRs put their
    // 127-VGPR allocation into scratch.)
    constexpr bool REGDESC = FUSE;
    const uint64_t nz = __ballot(nch > 0);
    if constexpr (!REGDESC) {
        if (nch > 0) {
            const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(nz >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nz, 0u));
            CD[k] = ColDesc{a_rel, pre, e_rel - a_rel, (b_rel - a_rel) | ((uint32_t)lane << 4) | (refc << 10)};
        }
        wave_sync();
    }
    // (three VGPRs: the start, the end, and the first chunk's index packed with the start's offset in its 16-B block and
    // the REF char — a group's chunks stay below 2^20, i.e. 10^9 entries per wave)
    const uint32_t d_a = a_rel, d_e = e_rel - a_rel, d_x = pre | ((b_rel - a_rel) << 20) | (refc << 24);
    const uint32_t lo = (uint32_t)lane * ALIGN;
    auto nxt = [&](int l) -> int {                      // the next lane with chunks after l (-1: the first); exists
        if constexpr (!REGDESC) return l + 1;           // whenever a caller asks (LDS: the compacted index)
        return (int)__builtin_ctzll(l >= 63 ? 0ull : (nz & (~0ull << (l + 1))));
    };
    auto cd = [&](int l, int f) -> uint32_t {           // field f of lane l's descriptor (uniform): start, first chunk,
        if constexpr (!REGDESC) return __builtin_amdgcn_readfirstlane(reinterpret_cast<const uint32_t *>(CD + l)[f]);
        if (f == 0) return __builtin_amdgcn_readlane(d_a, l);                       // end, start in block | column | REF
        if (f == 2) return __builtin_amdgcn_readlane(d_e, l);
        const uint32_t x = __builtin_amdgcn_readlane(d_x, l);
        return f == 1 ? (x & 0xFFFFFu) : (((x >> 20) & 15u) | ((uint32_t)l << 4) | ((x >> 24) << 10));
    };
    // prefetch cursor: column of the chunk being loaded (chunk indices only grow, by one per call)
    int pk = nxt(-1);
    uint32_t p_a = cd(pk, 0), p_pre = cd(pk, 1), p_end = p_pre + (cd(pk, 2) + STEP - 1) / STEP;
    auto chunk_off = [&](uint32_t i) -> uint32_t {   // chunks past the end reload the last one (ignored)
        if (i >= p_end && i < total) {
            pk = nxt(pk);
            p_a = cd(pk, 0);
            p_pre = cd(pk, 1);
            p_end = p_pre + (cd(pk, 2) + STEP - 1) / STEP;
        }
        const uint32_t ii = i < p_end ? i : p_end - 1;
        return p_a + (ii - p_pre) * STEP;               // (wave-uniform: the lane's part, lo, is the voffset)
    };

    // register ring of three chunks: two loads stay in flight while one chunk is processed
    V c0, q0, c1, q1, c2, q2;
#define SPG_LD(C, Q, I) do { const uint32_t o_ = chunk_off(I); C = bload_s<W, NT>(rc, lo, o_); Q = bload_s<W, NT>(rq, lo, o_); } while (0)
    SPG_LD(c0, q0, 0u);
    SPG_LD(c1, q1, 1u);

    // per-column state (consumption cursor)
    int ck = -1;
    uint32_t cj = 0, crefc = 0;
    uint32_t cs = 0, cpre = 0, cn = 0;
    uint32_t fcnt = 0, fsq = 0, ffirst = INF32;
    double fsl = 0.0, fse = 0.0;
    bool found = false;
    // second fast allele (dual mode, state above): a frequent minor allele (an SNV, an indel's D
    // entries) would otherwise push thousands of entries through the rare path and stall its wave
    uint32_t ffirst2 = INF32;
    bool found2 = false;

    // rare entries of a chunk (bit 8 b + 7 - d of rany: byte b of dword d): queue the lane slices
    // that hold any for the drain
    auto enqueue = [&](const V &cc, const V &qq, uint32_t rany, int32_t rel) {
        const uint64_t bal = __ballot(rany != 0);
        if (bal) {
            const uint32_t n = (uint32_t)__popcll(bal);
            if (qn + n > QCAP) drain();
            if (rany) {
                const uint32_t slot = qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                RareItem &it = Q[slot];
#pragma unroll
                for (int d = 0; d < W; d++) {
                    it.c[d] = dw<W>(cc, d);
                    it.q[d] = dw<W>(qq, d);
                }
                QO[slot] = rel;
                QR[slot] = rany | nb;           // rany bits 0-3 are free: ring slot
            }
            qn += n;
        }
    };

    // One chunk.  Every chunk takes the same generic SWAR path (validity masks, exact q >= 128
    // handling): specialised bodies for full / all-q<128 chunks measured slower, their extra code
    // and registers costing more occupancy than the instructions they save.
    auto process = [&](const V &cc, const V &qq, uint32_t i) {
        if (i >= total) return;                // (the last round's chunks past the end)
        if (i == cpre + cn) {                  // next column with chunks
            ck = nxt(ck);
            cpre = cd(ck, 1);
            const uint32_t e = cd(ck, 2), bic = cd(ck, 3);
            cn = (e + STEP - 1) / STEP;
            bl = (int32_t)(bic & 15u);
            el = (int32_t)e;
            cj = (bic >> 4) & 63u;
            crefc = bic >> 10;
        }
        cs = i - cpre;
        if (cs == 0) {                         // ---- column begin ----
            prog(2, (uint32_t)ck, i, cn);
            rare_init(RR + nb, lane);
            const uint32_t v0 = dw<W>(cc, 0) & 0xFFu;
            const int vote = ((int32_t)lo >= bl && (int32_t)lo < el) ? (int)v0 : -1;
            int cnt7[7];
            constexpr uint32_t VC[7] = {1u, 2u, 4u, 8u, 15u, SPG_CODE_DEL, SPG_CODE_SKIP};
#pragma unroll
            for (int k = 0; k < 7; k++) cnt7[k] = __popcll(__ballot(vote == (int)VC[k]));
            int b1 = 0;                         // major: a base (its products need the LUT path)
#pragma unroll
            for (int k = 1; k < 4; k++) if (cnt7[k] > cnt7[b1]) b1 = k;
            int b2 = -1, c2n = 1;               // second: any frequent code, >= 2 of 64 votes
#pragma unroll
            for (int k = 0; k < 7; k++) if (k != b1 && cnt7[k] > c2n) { c2n = cnt7[k]; b2 = k; }
            M = VC[b1];
            mrep = M * 0x01010101u;
            sem = nibble_char(M) != (uint8_t)crefc;
            skipped = false;
            skipped2 = false;
            dual = b2 >= 0;
            M2 = dual ? VC[b2] : 0u;
            mrep2 = dual ? M2 * 0x01010101u : 0xFFFFFFFFu;
            fcnt = 0; fsq = 0; ffirst = INF32; fsl = 0.0; fse = 0.0; found = false;
            ffirst2 = INF32; found2 = false;
            if (dual) { D2->cnt[lane] = 0; D2->sq[lane] = 0; D2->sl[lane] = 0.0; D2->se[lane] = 0.0; }
            wave_sync();
        }
        const int32_t o = (int32_t)(cs * STEP + lo);
        uint32_t vm[W];                         // entries of the lane slice inside the column
        if ((int32_t)(cs * STEP) >= bl && (int32_t)(cs * STEP + STEP) <= el) {   // full chunk (uniform)
#pragma unroll
            for (int d = 0; d < W; d++) vm[d] = 0x80808080u;
        } else {
            valid_masks<W>(o, bl, el, vm);
        }
        // SWAR classes of dword d: fast (major), second (dual mode) and rare.  Recomputed where
        // needed instead of kept in registers across the chunk.
        auto classify = [&](auto dual_tag, int d, uint32_t &f80, uint32_t &g80, uint32_t &r80, bool again = false) {
            constexpr bool DUAL = decltype(dual_tag)::value;
            uint32_t cw = dw<W>(cc, d), qw = dw<W>(qq, d);
            if (again) asm volatile("" : "+v"(cw), "+v"(qw));   // a recomputation, not a value kept live
            g80 = 0;
            swar4(cw, qw, vm[d], mrep, P.kpass, P.kok, f80, r80);
            if constexpr (DUAL) {
                uint32_t r2;
                swar4(cw, qw, vm[d], mrep2, P.kpass, P.kok, g80, r2);
                r80 &= ~g80;
            }
        };
        auto body = [&](auto dual_tag, auto sl_tag, auto sl2_tag) {
            constexpr bool DUAL = decltype(dual_tag)::value;
            constexpr bool SL = decltype(sl_tag)::value;     // false: counts / sum(q) only (calls-only REF major)
            constexpr bool SL2 = DUAL && decltype(sl2_tag)::value;   // false: Σ eps only for the second allele
            uint32_t rany = 0;                  // the chunk slice's rare entries: bit 8 b + 7 - d
            uint32_t fcnt2 = 0, fsq2 = 0, lsq = 0;
            double fsl2 = 0.0, fse2 = 0.0;
#pragma unroll
            for (int d = 0; d < W; d++) {
                const uint32_t qw = dw<W>(qq, d);
                uint32_t f80, g80, r80;
                classify(dual_tag, d, f80, g80, r80);
                if constexpr (DUAL) {           // the second allele's entries leave the rare set
                    fcnt2 += __popc(g80);
                    fsq2 = __builtin_amdgcn_udot4(qw, g80 >> 7, fsq2, false);
                }
                if constexpr (DUAL && !SL2) {   // Σ eps only: the rows' second halves (8-B reads)
                    const uint32_t idx2 = qw & ((g80 >> 7) * 0xFFu);
                    fse2 += (lut[idx2 & 0xFFu].y + lut[(idx2 >> 8) & 0xFFu].y) +
                            (lut[(idx2 >> 16) & 0xFFu].y + lut[idx2 >> 24].y);
                    asm volatile("" : "+v"(fse2) :: "memory");
                }
                if constexpr (SL2) {
                    const uint32_t idx2 = qw & ((g80 >> 7) * 0xFFu);
                    const double2 u0 = lut[idx2 & 0xFFu], u1 = lut[(idx2 >> 8) & 0xFFu];
                    fsl2 += u0.x + u1.x;
                    fse2 += u0.y + u1.y;
                    asm volatile("" : "+v"(fsl2), "+v"(fse2) :: "memory");   // two lookups in flight: registers
                    const double2 u2 = lut[(idx2 >> 16) & 0xFFu], u3 = lut[idx2 >> 24];
                    fsl2 += u2.x + u3.x;
                    fse2 += u2.y + u3.y;
                    asm volatile("" : "+v"(fsl2), "+v"(fse2) :: "memory");
                }
                fcnt += __popc(f80);
                // fast entries have q < 128: q * 0x80 sums of one chunk fit, shifted once below
                lsq = __builtin_amdgcn_udot4(qw, f80, lsq, false);
                if constexpr (SL) {
                    // fast entries have q < 128: their row is q; every other byte gets bit 7 -> a zero row
                    const uint32_t idx = qw & ((f80 >> 7) * 0xFFu);
                    const double2 t0 = lut[idx & 0xFFu], t1 = lut[(idx >> 8) & 0xFFu];
                    const double2 t2 = lut[(idx >> 16) & 0xFFu], t3 = lut[idx >> 24];
                    fsl += (t0.x + t1.x) + (t2.x + t3.x);
                    fse += (t0.y + t1.y) + (t2.y + t3.y);
                    asm volatile("" : "+v"(fsl), "+v"(fse) :: "memory");   // keep each dword's lookups together
                }
                rany |= d == 0 ? r80 : r80 >> d;
            }
            fsq += lsq >> 7;
            if constexpr (DUAL) {
                // second allele: lane-private LDS accumulators (no registers held across chunks)
                __hip_atomic_fetch_add(&D2->cnt[lane], fcnt2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&D2->sq[lane], fsq2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if constexpr (SL2) __hip_atomic_fetch_add(&D2->sl[lane], fsl2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if constexpr (DUAL) __hip_atomic_fetch_add(&D2->se[lane], fse2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (!found || (DUAL && !found2)) {   // first fast entry of each fast allele (dict order)
                uint32_t mine = INF32, mine2 = INF32;
#pragma unroll
                for (int d = W - 1; d >= 0; d--) {
                    uint32_t f80, g80, r80;
                    classify(dual_tag, d, f80, g80, r80, true);
                    if (f80) mine = (uint32_t)(o + 4 * d - bl) + ((uint32_t)__builtin_ctz(f80) >> 3);
                    if (DUAL && g80) mine2 = (uint32_t)(o + 4 * d - bl) + ((uint32_t)__builtin_ctz(g80) >> 3);
                }
                // lanes cover increasing offsets: the first fast entry is the lowest one of the
                // lowest lane that has any
                if (!found) {
                    const uint64_t b = __ballot(mine != INF32);
                    if (b) { ffirst = __builtin_amdgcn_readlane(mine, (int)__builtin_ctzll(b)); found = true; }
                }
                if (DUAL && !found2) {
                    const uint64_t b = __ballot(mine2 != INF32);
                    if (b) { ffirst2 = __builtin_amdgcn_readlane(mine2, (int)__builtin_ctzll(b)); found2 = true; }
                }
            }
            enqueue(cc, qq, rany, o - bl);
        };
        using T_ = std::true_type;
        using F_ = std::false_type;
        if (dual) {
            // FUSE (calls-only): the second allele skips Σ ln(1-eps) but keeps Σ eps (QUAL).  Its H is
            // needed only when its own GL is not exactly 0 — in a deep column the other allele's P
            // underflows to 0 — and then finalize replays the position exactly.
            if constexpr (FUSE) {
                if (sem || !P.calls_only) body(T_{}, T_{}, F_{});
                else { body(T_{}, F_{}, F_{}); skipped = true; }
                skipped2 = true;
            } else {
                if (sem || !P.calls_only) body(T_{}, T_{}, T_{});
                else {                         // calls-only, REF major: only the second allele's sums
                    body(T_{}, F_{}, T_{});
                    skipped = true;
                }
            }
        } else if (sem || !P.calls_only) body(F_{}, T_{}, F_{});
        else {                                 // calls-only, REF major: counts and sum(q) only
            body(F_{}, F_{}, F_{});
            skipped = true;
        }
        if (cs + 1 == cn) {                    // ---- column end ----
            const uint32_t fc = dsum_u32(fcnt), fs = dsum_u32(fsq);
            double fl = 0.0, fe = 0.0;
            if (!skipped) { fl = dsum_f64(fsl); fe = dsum_f64(fse); }   // skipped: no chunk summed them
            uint32_t fc2 = 0, fs2 = 0;
            double fl2 = 0.0, fe2 = 0.0;
            if (dual) {
                wave_sync();
                fc2 = dsum_u32(D2->cnt[lane]); fs2 = dsum_u32(D2->sq[lane]);
                if (!skipped2) fl2 = dsum_f64(D2->sl[lane]);
                fe2 = dsum_f64(D2->se[lane]);
            }
            const uint32_t fsc = (uint32_t)__builtin_amdgcn_readlane(fsv, (int)cj);
            if (lane == 0) {
                ColSum *S = CS + nb;
                S->M = M; S->M2 = dual ? M2 : 0u; S->fc = fc; S->fs = fs; S->fc2 = fc2; S->fs2 = fs2;
                S->ffirst = ffirst; S->ffirst2 = ffirst2; S->skipped = (skipped ? 1u : 0u) | (skipped2 ? 2u : 0u); S->cj = cj;
                S->crefc = crefc; S->fl = fl; S->fe = fe; S->fl2 = fl2; S->fe2 = fe2;
                S->fsamp = fsc;
            }
            if (++nb == NB) {
                if constexpr (!FUSE) finish();         // FUSE: G <= NB, the ring is finished after the loop
            }
        }
    };

    // rounds of three chunks with no exit in between (hipcc's wait counts stay exact across the back edge: with an
    // exit after each chunk the first of the three waited for one chunk more than it needs); a chunk index past the
    // end is a no-op (process), its load a clamped reload
    for (uint32_t i = 0; i < total; i += 3) {
        SPG_LD(c2, q2, i + 2); process(c0, q0, i);
        SPG_LD(c0, q0, i + 3); process(c1, q1, i + 1);
        SPG_LD(c1, q1, i + 4); process(c2, q2, i + 2);
    }
#undef SPG_LD
    prog(5, total, nb, qn);
    const uint64_t wt1 = P.wtime ? __builtin_amdgcn_s_memrealtime() : 0;   // SPG_WAVE_TIMES: the chunk loop's end
    const uint32_t nfin = nb;                          // FUSE: every column of the wave (G <= NB)
    if (nb) finish();
    uint32_t tailed = 0;                               // SPG_WAVE_TIMES: the wave ran the fused finalize
    if constexpr (FUSE) {
        // Division-free pre-check from the images (LDS) and the kernel's scalar parameters: most positions
        // cannot produce a call.  Only a wave holding a possible call reads the finalize parameters (vector
        // loads from memory, whose wait would also wait for the record stores just issued).
        const bool maybe = (uint32_t)lane < nfin && may_call_img(P, img + lane);
        if (__ballot(maybe)) {
            tailed = 1;
            fused_tail(P.fused->F, P.fused->O, T, P.pos_begin + g0, maybe ? nfin : 0u, CS, img,
                       reinterpret_cast<ReplayWs *>(Q), &hdl, lut);
        }
    }
    if (P.wtime && lane == 0) {
        const uint64_t wt2 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID
        // {entry, first column (bits 0-14) | entry-to-loop-end ticks (bits 15-31), lifetime from entry (bits 0-19) |
        //  entry-to-loop ticks (bits 20-31), hw id (bits 0-19) | fused finalize ran (bit 20) | XCC (bits 24-31)}
        const uint64_t pro = min(wt0 - we, (uint64_t)0xFFF), life = min(wt2 - we, (uint64_t)0xFFFFF);
        const uint64_t lend = min(wt1 - we, (uint64_t)0x1FFFF);
        P.wtime[wave] = make_uint4((uint32_t)we, ((uint32_t)g0 & 0x7FFFu) | (uint32_t)(lend << 15),
                                   (uint32_t)(life | (pro << 20)), (hw & 0xFFFFFu) | (tailed << 20) | (xcc << 24));
    }
    prog(6, 0, 0, 0);
    }   // items
}

// Fold the S partial states of a split run in batch order (first-entry keys (split, stream index)) and
// merge them into the records.  One thread per position.
__global__ __launch_bounds__(256) void k_merge_parts(MParams P, const uint8_t *__restrict__ ref,
                                                     Acc *__restrict__ acc) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t p = P.u0 + i;
    if (p >= P.u1) return;
    MState c;
    ms_init(c);
    uint64_t key[NSLOT];
#pragma unroll
    for (int k = 0; k < NSLOT; k++) key[k] = ~0ull;
    const int64_t stride = P.pstride;
    for (int32_t s = 0; s < P.S; s++) {
        const MState &q = P.part[(int64_t)s * stride + i];
        const uint32_t fb = q.fb;
        if (fb == INF32) continue;
        if (c.fb == INF32) c.fb = fb;
        c.depth += q.depth; c.n_del += q.n_del; c.n_skip += q.n_skip; c.n_other += q.n_other;
        c.skip |= q.skip;
#pragma unroll
        for (int k = 0; k < NSLOT; k++) {
            const uint32_t n = q.cnt[k];
            if (!n) continue;
            if (!c.cnt[k]) { key[k] = ((uint64_t)(uint32_t)s << 32) | q.first[k]; c.qf[k] = q.qf[k]; }
            else c.qf[k] = (uint8_t)min((uint32_t)c.qf[k], (uint32_t)q.qf[k]);
            c.cnt[k] += n;
            c.sq[k] = sat_add31(c.sq[k], q.sq[k]);
            c.sl[k] += q.sl[k];
            c.se[k] += q.se[k];
        }
    }
    if (c.fb == INF32) return;
    Acc a;
    if (!P.fresh) a = acc[p];
    if (P.fresh || a.epoch != P.epoch) { a = Acc{}; a.epoch = P.epoch; }
    merge_state(a, c, key, P.seq0 + c.fb, ref[p]);
    const uint4 *src = reinterpret_cast<const uint4 *>(&a);
    uint4 *dst = reinterpret_cast<uint4 *>(acc + p);
    const bool sums = !P.fresh || record_has_sums(a);
#pragma unroll
    for (int t = 0; t < 10; t++)
        if (t < 5 || sums) dst[t] = src[t];
}

// One wave per 64 positions: each lane runs prepare_variants' per-position logic; positions that need
// the exact replay are then replayed one after another by the whole wave.
template <bool SPARSE>
__global__ __launch_bounds__(64) void k_finalize(FParams F, const Acc *__restrict__ acc,
                                                  const Tables *__restrict__ T, const Hist *__restrict__ H, Out O) {
    __shared__ double sink[64][NSLOT];
    __shared__ double eps_s[256];
    __shared__ ReplayWs ws;
    const int lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x == 0) O.ctr[F.cslot ^ 1u] = Counters{0, 0, 0, 0};   // next call's slot
    if constexpr (SPARSE) {
        // sparse finalize: the positions the fused accumulate listed, 64 per wave iteration
        const int64_t n = (int64_t)*F.n_list;
        bool eps_loaded = false;
        for (int64_t i0 = (int64_t)blockIdx.x * 64; i0 < n; i0 += (int64_t)gridDim.x * 64) {
            const int64_t i = i0 + lane;
            const int64_t pos = i < n ? F.list[i] : 0;
            const bool need = i < n && finalize_position<false>(F, acc + pos, T, O, pos, sink[lane]);
            uint64_t rb = __ballot(need);
            if (rb == 0) continue;
            if (need) atomicAdd(&O.ctr[F.cslot].n_band, 1u);
            if (!eps_loaded) {
                for (int q = lane; q < 256; q += 64) eps_s[q] = T->eps[q];
                wave_sync();
                eps_loaded = true;
            }
            while (rb) {
                const int j = (int)__builtin_ctzll(rb);
                rb &= rb - 1;
                const int64_t pj = (int64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)pos, j) |
                                   ((int64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)((uint64_t)pos >> 32), j) << 32);
                replay_wave<true>(F, H, acc + pj, O, pj, &ws, [&](uint32_t q) { return eps_s[q]; });
            }
        }
        return;
    }
    const int64_t pos = (int64_t)blockIdx.x * 64 + lane;
    const bool need = pos < F.n_pos && finalize_position<false>(F, acc + pos, T, O, pos, sink[lane]);
    uint64_t rb = __ballot(need);
    if (rb == 0) return;
    if (need) atomicAdd(&O.ctr[F.cslot].n_band, 1u);
    for (int q = lane; q < 256; q += 64) eps_s[q] = T->eps[q];
    wave_sync();
    while (rb) {
        const int j = (int)__builtin_ctzll(rb);
        rb &= rb - 1;
        const int64_t pj = (int64_t)blockIdx.x * 64 + j;
        replay_wave<true>(F, H, acc + pj, O, pj, &ws, [&](uint32_t q) { return eps_s[q]; });
    }
}

// ------------------------------------------------------------------------------------------
// launchers (called from spg_api.cpp)
// ------------------------------------------------------------------------------------------
// k_acc_seg over one batch: every column of a deep batch (W = 4), or the long columns (>= t_deep) of a
// shallow one (W = 1; k_acc_tile / k_acc_lite take the rest)
hipError_t launch_accumulate(const KParams &P, const uint64_t *off, const uint8_t *code, const uint8_t *qual,
                             const uint8_t *ref, const Tables *T, Acc *acc, hipStream_t st) {
    if (P.n_cols == 0) return hipSuccess;
    const int64_t waves = P.w1 >= (P.n_cols + P.G - 1) / P.G ? (P.n_cols + P.G - 1) / P.G
                                                             : P.w1 + (P.n_cols - (int64_t)P.w1 * P.G + P.G2 - 1) / P.G2;
    // listed long columns: a fixed grid strides over the list (its length is on the device)
    const int64_t blocks = P.deep_n ? std::min<int64_t>((P.n_cols + KW - 1) / KW, 2048)
                                    : (waves + KW - 1) / KW;
    const bool fresh = P.batch_seq == 1;
    const bool w4 = P.t_deep <= 1 && !P.deep_n;      // (listed columns: W = 1, whatever t_deep)
    if (P.G > (uint32_t)(w4 ? SPG_GMAX_DEEP : SPG_GMAX) || (!P.deep_n && P.G2 > P.G)) return hipErrorInvalidValue;   // coldesc
    // batches far beyond the 256 MiB Infinity Cache stream with non-temporal loads
    const bool nt = 2 * P.n_entries > ((uint64_t)SPG_NT_MIB << 20);
    // (W = 1, and a deep batch into a memory that already holds records (the old record is read and
    // merged): 3 waves per SIMD, so the register allocation needs no scratch)
#define SPG_SEG(WW, FF, NN) hipLaunchKernelGGL((k_acc_seg<WW, FF, (WW == 1 || !FF) ? 3 : SPG_SEG_WPE, NN, false>), dim3((unsigned)blocks), dim3(64 * KW), 0, st, P, off, code, qual, ref, T, acc)
#define SPG_SEGF(NN) hipLaunchKernelGGL((k_acc_seg<4, true, SPG_SEG_WPE, NN, true>), dim3((unsigned)blocks), dim3(64 * KW), 0, st, P, off, code, qual, ref, T, acc)
    if (P.fused) {            // fused accumulate + calls-only finalize (FRESH deep batch, G <= NB)
        if (!w4 || !fresh || P.G > (uint32_t)NB) return hipErrorInvalidValue;
        if (nt) SPG_SEGF(true); else SPG_SEGF(false);
    } else if (w4) {
        if (nt) { if (fresh) SPG_SEG(4, true, true); else SPG_SEG(4, false, true); }
        else { if (fresh) SPG_SEG(4, true, false); else SPG_SEG(4, false, false); }
    } else {
        if (fresh) SPG_SEG(1, true, false); else SPG_SEG(1, false, false);
    }
#undef SPG_SEG
#undef SPG_SEGF
    return hipGetLastError();
}

hipError_t launch_merge(const MParams &P, const uint8_t *ref, Acc *acc, hipStream_t st) {
    const int64_t mb = (P.u1 - P.u0 + 255) / 256;
    hipLaunchKernelGGL(k_merge_parts, dim3((unsigned)mb), dim3(256), 0, st, P, ref, acc);
    return hipGetLastError();
}

hipError_t launch_finalize(const FParams &F, const Acc *acc, const Tables *T, const Out &O, const Hist *H,
                           hipStream_t st) {
    // 64-thread blocks (one wave), one position per lane; the sparse form strides over the list (its
    // length is on the device)
    const int64_t blocks = F.list ? std::min<int64_t>((F.n_pos + 63) / 64, 8192) : (F.n_pos + 63) / 64;
    if (F.list) hipLaunchKernelGGL(k_finalize<true>, dim3((unsigned)blocks), dim3(64), 0, st, F, acc, T, H, O);
    else hipLaunchKernelGGL(k_finalize<false>, dim3((unsigned)blocks), dim3(64), 0, st, F, acc, T, H, O);
    return hipGetLastError();
}

}  // namespace spg
