// spg_kernels.hip — CDNA4 (gfx950) kernels of the pileup + genotype-likelihood engine.
//
//   k_accumulate  process_pileup_column / process_svn (live_variant_caller.py:74-103) + pysam's
//                 base-quality filter, for one CSR batch; merges into the per-position Acc records.
//                 Deep columns: one wave64 per column, 16 entries per lane per step (dwordx4 loads
//                 of base_code and qual), SWAR byte tests, v_dot4_u32_u8 quality sums, v_bcnt
//                 counts and an LDS-resident {ln(1-eps), eps} table; the rare entries (minor
//                 alleles, D/N, q < 4, q >= 128, IUPAC) take an exact per-entry path.
//                 Shallow columns: one lane per column, sequential.
//   k_finalize    prepare_variants (:120-185) + genotype_likelihood / to_phred_scale
//                 (utils.py:12-24): per-position GL in fp64 with the reference's underflow
//                 decisions, candidate filters, GL/PL/SCORE/QUAL; positions whose result depends
//                 on the order of fp64 roundings in the subnormal range go to k_replay.
//   k_replay      exact sequential recomputation (np.prod left folds in BAM order, dict-order
//                 GL chains) over the batch history for the listed positions.
#include "spg_device.h"

namespace spg {

// ------------------------------------------------------------------------------------------
// per-lane column state (rare/exact path and shallow columns)
// ------------------------------------------------------------------------------------------
struct ColState {
    uint32_t depth, n_del, n_skip, n_other;
    uint32_t cnt[NSLOT], sq[NSLOT], qf[NSLOT], first[NSLOT];
    double sl[NSLOT], se[NSLOT];
};

__device__ __forceinline__ void cs_init(ColState &s) {
    s.depth = s.n_del = s.n_skip = s.n_other = 0;
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        s.cnt[k] = 0; s.sq[k] = 0; s.qf[k] = 255u; s.first[k] = INF32; s.sl[k] = 0.0; s.se[k] = 0.0;
    }
}

// One pileup entry that passed the base-quality filter (:89-103).
__device__ __forceinline__ void entry_update(ColState &s, uint32_t code, uint32_t q, uint32_t idx,
                                             const Tables *__restrict__ T) {
    s.depth++;
    if (code == SPG_CODE_DEL) { s.n_del++; return; }
    if (code == SPG_CODE_SKIP) { s.n_skip++; return; }
    const int sl = slot_of(code);
    if (sl < 0) { s.n_other++; return; }
    const double l = T->l1m[q], e = T->eps[q];
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        if (sl == k) {
            s.cnt[k] += 1u; s.sq[k] += q; s.qf[k] = min(s.qf[k], q); s.first[k] = min(s.first[k], idx);
            s.sl[k] += l; s.se[k] += e;
        }
    }
}

// ------------------------------------------------------------------------------------------
// wave64 reductions (butterfly; every lane ends with the result)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wsum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint32_t wmin(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wsumd(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ------------------------------------------------------------------------------------------
// merge one column's batch statistics into its Acc record (single lane)
// ------------------------------------------------------------------------------------------
__device__ void merge_acc(Acc *__restrict__ A, const ColState &c, uint32_t batch_seq, uint8_t refc) {
    Acc a = *A;
    if (a.first_batch == 0) {                       // first visit (:77-85)
        a.first_batch = batch_seq;
        a.misc = refc;
    }
    a.depth += c.depth;                             // :87
    a.n_del += c.n_del;
    a.n_skip += c.n_skip;
    a.n_other += c.n_other;
    if (c.n_other) a.misc |= MISC_EXOTIC;
    uint32_t n = a.order & 7u;
    uint32_t have = 0;
    for (uint32_t i = 0; i < n; i++) have |= 1u << ((a.order >> (3 + 3 * i)) & 7u);
    uint32_t newmask = 0;
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        if (c.cnt[k]) {
            if (a.cnt[k] == 0) a.qf[k] = (uint8_t)c.qf[k];
            else a.qf[k] = (uint8_t)min((uint32_t)a.qf[k], c.qf[k]);
            a.cnt[k] += c.cnt[k];
            const uint64_t s = (uint64_t)a.sq[k] + c.sq[k];
            a.sq[k] = s > 0x80000000ull ? 0x80000000u : (uint32_t)s;
            a.sl[k] += c.sl[k];
            a.se[k] += c.se[k];
            if (!((have >> k) & 1u)) newmask |= 1u << k;
        }
    }
    // new alleles join the dict in order of first appearance in this batch (:100-101)
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        if ((newmask >> k) & 1u) {
            uint32_t rank = 0;
#pragma unroll
            for (int j = 0; j < NSLOT; j++)
                if (j != k && ((newmask >> j) & 1u) && (c.first[j] < c.first[k] || (c.first[j] == c.first[k] && j < k)))
                    rank++;
            a.order |= (uint32_t)k << (3 + 3 * (n + rank));
        }
    }
    n += __popc(newmask);
    a.order = (a.order & ~7u) | n;
    *A = a;
}

// ------------------------------------------------------------------------------------------
// SWAR classification of 4 entries (one dword of base_code, one of qual)
//   fast  = valid & q >= max(min_bq,4) & q < 128 & code == M      (the column's major allele)
//   rare  = valid & (q >= min_bq | q >= 128) & !fast                (exact per-entry path)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void swar4(uint32_t cw, uint32_t qw, uint32_t v80, uint32_t mrep, uint32_t kpass,
                                      uint32_t kok, uint32_t &fast80, uint32_t &rare80) {
    const uint32_t q7 = qw & 0x7F7F7F7Fu;
    const uint32_t hi80 = qw & 0x80808080u;
    const uint32_t pass80 = (q7 + kpass) & 0x80808080u;
    const uint32_t ok80 = (q7 + kok) & 0x80808080u;
    const uint32_t x = cw ^ mrep;
    const uint32_t ne80 = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
    fast80 = ok80 & ~(ne80 | hi80) & v80;
    rare80 = (pass80 | hi80) & ~fast80 & v80;
}

__device__ __forceinline__ uint32_t valid80(int64_t base, int64_t b, int64_t e) {
    int64_t lead = b - base, end = e - base;
    lead = lead < 0 ? 0 : (lead > 4 ? 4 : lead);
    end = end < 0 ? 0 : (end > 4 ? 4 : end);
    return (uint32_t)((0x80808080ull << (8 * lead)) & (0x80808080ull >> (8 * (4 - end))));
}

__device__ __forceinline__ uint32_t pack_rare(uint32_t r80) {   // bits 7,15,23,31 -> 0..3
    const uint32_t t = r80 >> 7;
    return (t | (t >> 7) | (t >> 14) | (t >> 21)) & 0xFu;
}

template <int W>   // W dwords per lane per step: 4 (16 entries, dwordx4) or 1 (4 entries)
struct Vec;
template <> struct Vec<4> { using T = uint4; };
template <> struct Vec<1> { using T = uint32_t; };

template <int W>
__device__ __forceinline__ uint32_t dw(const typename Vec<W>::T &v, int d) {
    if constexpr (W == 1) { (void)d; return v; }
    else return d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
}

// Wave-wide processing of one deep column [b, e) of the batch arrays.  Every lane returns the
// column's complete statistics in `out`.
template <int W>
__device__ void deep_column(const uint8_t *__restrict__ code, const uint8_t *__restrict__ qual, int64_t b, int64_t e,
                            const KParams &P, const Tables *__restrict__ T, const double2 *__restrict__ lut,
                            ColState &out) {
    using V = typename Vec<W>::T;
    constexpr int STEP = 64 * 4 * W;              // entries per wave step
    const int lane = threadIdx.x & 63;
    const int64_t a0 = b & ~(int64_t)(4 * W - 1);
    const int nstep = (int)((e - a0 + STEP - 1) / STEP);

    // major allele: vote over the first entry of each lane's first chunk
    uint32_t M;
    {
        const int64_t o = a0 + (int64_t)lane * 4 * W;
        int vote = -1;
        if (o >= b && o < e) vote = (int)code[o];
        const uint64_t mA = __ballot(vote == 1), mC = __ballot(vote == 2), mG = __ballot(vote == 4),
                       mT = __ballot(vote == 8);
        const int cA = __popcll(mA), cC = __popcll(mC), cG = __popcll(mG), cT = __popcll(mT);
        M = 1; int best = cA;
        if (cC > best) { best = cC; M = 2; }
        if (cG > best) { best = cG; M = 4; }
        if (cT > best) { best = cT; M = 8; }
    }
    const uint32_t mrep = M * 0x01010101u;
    const int Ms = slot_of(M);

    uint32_t fcnt = 0, fsq = 0, ffirst = INF32;
    double fsl0 = 0.0, fsl1 = 0.0, fse0 = 0.0, fse1 = 0.0;
    bool found = false;
    ColState rs;
    cs_init(rs);

    V cc, qq, cn, qn;
    {
        const int64_t o = a0 + (int64_t)lane * 4 * W;
        if (o < e) { cc = *(const V *)(code + o); qq = *(const V *)(qual + o); }
        else { cc = V{}; qq = V{}; }
    }
    for (int s = 0; s < nstep; s++) {
        const int64_t base = a0 + (int64_t)s * STEP;
        const int64_t o = base + (int64_t)lane * 4 * W;
        if (s + 1 < nstep) {                       // prefetch the next step
            const int64_t on = o + STEP;
            if (on < e) { cn = *(const V *)(code + on); qn = *(const V *)(qual + on); }
            else { cn = V{}; qn = V{}; }
        }
        const bool full = base >= b && base + STEP <= e;   // wave-uniform
        uint32_t f80[W], r80[W];
#pragma unroll
        for (int d = 0; d < W; d++) {
            const uint32_t v = full ? 0x80808080u : valid80(o + 4 * d, b, e);
            swar4(dw<W>(cc, d), dw<W>(qq, d), v, mrep, P.kpass, P.kok, f80[d], r80[d]);
        }
        // fast path: major allele, 4 <= q < 128
#pragma unroll
        for (int d = 0; d < W; d++) {
            const uint32_t qw = dw<W>(qq, d);
            const uint32_t f01 = f80[d] >> 7;
            fcnt += __popc(f80[d]);
            fsq = __builtin_amdgcn_udot4(qw, f01, fsq, false);
            const uint32_t idx = qw & (f01 * 0xFFu);
            const double2 t0 = lut[idx & 0xFFu], t1 = lut[(idx >> 8) & 0xFFu];
            const double2 t2 = lut[(idx >> 16) & 0xFFu], t3 = lut[idx >> 24];
            fsl0 += t0.x; fse0 += t0.y; fsl1 += t1.x; fse1 += t1.y;
            fsl0 += t2.x; fse0 += t2.y; fsl1 += t3.x; fse1 += t3.y;
        }
        if (!found) {                              // first fast entry of the column (dict order)
            uint32_t mine = INF32;
#pragma unroll
            for (int d = W - 1; d >= 0; d--)
                if (f80[d]) mine = (uint32_t)(o + 4 * d - b) + ((uint32_t)__builtin_ctz(f80[d]) >> 3);
            const uint32_t w = wmin(mine);
            if (w != INF32) { ffirst = w; found = true; }
        }
        // rare path: exact per entry
        uint32_t m = 0;
#pragma unroll
        for (int d = 0; d < W; d++) m |= pack_rare(r80[d]) << (4 * d);
        if (__ballot(m != 0)) {
            while (m) {
                const int j = __builtin_ctz(m);
                m &= m - 1;
                const int d = j >> 2, sh = (j & 3) * 8;
                uint32_t cwd = dw<W>(cc, 0), qwd = dw<W>(qq, 0);
#pragma unroll
                for (int dd = 1; dd < W; dd++)
                    if (d == dd) { cwd = dw<W>(cc, dd); qwd = dw<W>(qq, dd); }
                const uint32_t c = (cwd >> sh) & 0xFFu, q = (qwd >> sh) & 0xFFu;
                if ((int)q >= P.min_bq) entry_update(rs, c, q, (uint32_t)(o + j - b), T);
            }
        }
        cc = cn; qq = qn;
    }

    // ---- wave reduction ----
    out.depth = wsum(rs.depth) + wsum(fcnt);
    out.n_del = wsum(rs.n_del);
    out.n_skip = wsum(rs.n_skip);
    out.n_other = wsum(rs.n_other);
#pragma unroll
    for (int k = 0; k < NSLOT; k++) {
        if (__ballot(rs.cnt[k] != 0)) {
            out.cnt[k] = wsum(rs.cnt[k]);
            out.sq[k] = wsum(rs.sq[k]);
            out.qf[k] = wmin(rs.qf[k]);
            out.first[k] = wmin(rs.first[k]);
            out.sl[k] = wsumd(rs.sl[k]);
            out.se[k] = wsumd(rs.se[k]);
        } else {
            out.cnt[k] = 0; out.sq[k] = 0; out.qf[k] = 255u; out.first[k] = INF32; out.sl[k] = 0.0; out.se[k] = 0.0;
        }
    }
    const uint32_t fc = wsum(fcnt);
    if (fc) {
        const uint32_t fs = wsum(fsq);
        const double fl = wsumd(fsl0 + fsl1), fe = wsumd(fse0 + fse1);
#pragma unroll
        for (int k = 0; k < NSLOT; k++) {
            if (k == Ms) {
                out.cnt[k] += fc; out.sq[k] += fs; out.sl[k] += fl; out.se[k] += fe;
                out.qf[k] = min(out.qf[k], (uint32_t)P.qlo);
                out.first[k] = min(out.first[k], ffirst);
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_accumulate(KParams P, const uint64_t *__restrict__ off,
                                                    const uint8_t *__restrict__ code,
                                                    const uint8_t *__restrict__ qual,
                                                    const uint8_t *__restrict__ ref,
                                                    const Tables *__restrict__ T, Acc *__restrict__ acc) {
    __shared__ double2 lut[128];
    if (threadIdx.x < 128) lut[threadIdx.x] = make_double2(T->fast[threadIdx.x][0], T->fast[threadIdx.x][1]);
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t g0 = wave * P.G;
    if (g0 >= P.n_cols) return;
    const int64_t ng = min((int64_t)P.G, P.n_cols - g0);

    uint64_t ob = 0, oe = 0;
    if (lane < ng) { ob = off[g0 + lane]; oe = off[g0 + lane + 1]; }
    const uint64_t len = oe - ob;

    // shallow columns: one lane each, sequential
    if (lane < ng && len > 0 && len < P.t_deep) {
        ColState st;
        cs_init(st);
        for (uint64_t i = ob; i < oe; i++) {
            const uint32_t c = code[i], q = qual[i];
            if ((int)q >= P.min_bq) entry_update(st, c, q, (uint32_t)(i - ob), T);
        }
        const int64_t pos = P.pos_begin + g0 + lane;
        merge_acc(acc + pos, st, P.batch_seq, ref[pos]);
    }
    // deep columns: the whole wave, one after another
    uint64_t deep = __ballot(lane < ng && len >= P.t_deep);
    while (deep) {
        const int i = __builtin_ctzll(deep);
        deep &= deep - 1;
        const int64_t b = (int64_t)__shfl(ob, i), e = (int64_t)__shfl(oe, i);
        ColState st;
        if (e - b >= 2048) deep_column<4>(code, qual, b, e, P, T, lut, st);
        else deep_column<1>(code, qual, b, e, P, T, lut, st);
        if (lane == 0) {
            const int64_t pos = P.pos_begin + g0 + i;
            merge_acc(acc + pos, st, P.batch_seq, ref[pos]);
        }
    }
}

// ------------------------------------------------------------------------------------------
// finalize: GL with the reference's underflow decisions
// ------------------------------------------------------------------------------------------
constexpr double DMIN = 0x1p-1022;            // smallest normal
constexpr double LOG2_10_OVER_10 = 0.33219280948873623;   // log2(10)/10
constexpr double INV_LN2 = 1.4426950408889634;
constexpr double MARGIN = 1e-5;               // log2 margin around the band edges (>> rounding)

// A value of the reference's fp64 computation, known either exactly as 0, or accurately (state 0:
// value within ~1e-12 relative, normal, l2 = log2 of it), or only by an upper bound (state 2,
// "band": l2 bounds log2 of the reference's value, which depends on the order of roundings in
// the subnormal range).  lv_mul follows one reference multiplication fl(a*b).
struct LV { int s; double v, l2; };
__device__ __forceinline__ LV lv_normal(double v, double l2) { return LV{0, v, l2}; }
__device__ __forceinline__ LV lv_zero() { return LV{1, 0.0, -1e300}; }
__device__ __forceinline__ LV lv_band(double ub) { return LV{2, 0.0, ub}; }
__device__ __forceinline__ LV lv_mul(const LV &a, const LV &b) {
    if (a.s == 1 || b.s == 1) return lv_zero();                   // 0 * finite == 0
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

// Emit the candidates of one position given final GL values in dict order (:145-185).
__device__ void emit_candidates(const FParams &F, const Out &O, int64_t pos, const Acc &a, int n,
                                const uint32_t *codes, const uint32_t *cnts, const double *G, const double *qual,
                                uint8_t &flags) {
    double S = 0.0;
    for (int k = 0; k < n; k++) S = S + G[k];              // :145
    if (S == 0) S = 1.0;                                   // :146
    const uint8_t refc = (uint8_t)(a.misc & 0xFFu);
    for (int k = 0; k < n; k++) {
        const uint8_t allele = nibble_char(codes[k]);
        const uint32_t ad = cnts[k];
        if (refc != allele && (int64_t)ad >= F.min_ad && (double)ad / (double)a.depth >= F.ratio) {
            spg_candidate c;
            c.pos = pos; c.dp = (int32_t)a.depth; c.ad = (int32_t)ad;
            c.ref = refc; c.alt = allele; c.rank = (uint8_t)k; c.first_batch = a.first_batch;
            c.gl_linear = G[k];
            if (G[k] != 0) { c.gl = log10(G[k]); c.pl = (int32_t)rint(-10.0 * c.gl); c.gl_zero = 0; }
            else { c.gl = 0.0; c.pl = 0; c.gl_zero = 1; }
            c.score = to_phred(1.0 - (G[k] / S));
            c.qual = qual[k];
            const uint32_t at = atomicAdd(&O.ctr->n_cand, 1u);
            if (at < (uint32_t)F.cand_cap) O.cand[at] = c;
            flags |= SPG_F_CANDIDATE;
        }
    }
}

__global__ __launch_bounds__(256) void k_finalize(FParams F, const Acc *__restrict__ acc,
                                                  const Tables *__restrict__ T, Out O) {
    const int64_t pos = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pos >= F.n_pos) return;
    const Acc a = acc[pos];
    const double NaN = __builtin_nan("");
    uint8_t flags = 0;
    O.depth[pos] = a.depth;
    O.order[pos] = a.order;
    O.first[pos] = a.first_batch;
    uint32_t *cnt8 = O.counts + pos * SPG_NCOUNT;
#pragma unroll
    for (int k = 0; k < NSLOT; k++) cnt8[k] = a.cnt[k];
    cnt8[5] = a.n_del; cnt8[6] = a.n_skip; cnt8[7] = a.n_other;
    double *gl = O.gl + pos * NSLOT;
#pragma unroll
    for (int k = 0; k < NSLOT; k++) gl[k] = NaN;
    if (a.first_batch == 0) { O.flags[pos] = 0; return; }
    flags |= SPG_F_PRESENT;
    const bool evaluated = (int64_t)a.depth >= (int64_t)F.min_td;   // :131
    if (evaluated) flags |= SPG_F_EVALUATED;
    if (a.misc & MISC_EXOTIC) {      // IUPAC / '=' alleles: exact replay tabulates every allele
        const uint32_t at = atomicAdd(&O.ctr->n_band, 1u);
        if (at < (uint32_t)F.band_cap) O.band[at] = pos;
        O.flags[pos] = flags | SPG_F_EXOTIC | SPG_F_REPLAYED;
        return;
    }
    if (!evaluated) { O.flags[pos] = flags; return; }

    const int n = (int)(a.order & 7u);
    uint32_t sl_[NSLOT], codes[NSLOT], cnts[NSLOT];
    for (int k = 0; k < n; k++) {
        sl_[k] = (a.order >> (3 + 3 * k)) & 7u;
        codes[k] = slot_code((int)sl_[k]);
    }
    bool band = false;
    // per-allele P (= prod eps, utils.py:19) and H (= prod 1-eps, utils.py:17) in dict order
    LV Pv[NSLOT], Hv[NSLOT];
    double Qv[NSLOT];
    for (int k = 0; k < n && !band; k++) {
        const int s = (int)sl_[k];
        uint32_t c_ = 0, sq = 0, qf = 0; double sl = 0.0, se = 0.0;
#pragma unroll
        for (int j = 0; j < NSLOT; j++)
            if (s == j) { c_ = a.cnt[j]; sq = a.sq[j]; qf = a.qf[j]; sl = a.sl[j]; se = a.se[j]; }
        cnts[k] = c_;
        Qv[k] = se / (double)c_;
        // P: log10 P = -sum(q)/10 up to (n+2) ulp; exact zero proven when every factor < 1/2
        if (sq <= 3076u) Pv[k] = lv_normal(T->p10k[sq / 10u] * T->eps[sq % 10u], -(double)sq * LOG2_10_OVER_10);
        else if (sq >= 3245u && qf >= 4u) Pv[k] = lv_zero();
        else Pv[k] = lv_band(-1022.0 + 2 * MARGIN);
        // H: exp(sum ln(1-eps)); exactly 0 when a Q0 entry is present (1 - 1.0 == 0)
        if (qf == 0u) Hv[k] = lv_zero();
        else {
            const double l2 = sl * INV_LN2;
            Hv[k] = l2 > -1022.0 + MARGIN ? lv_normal(exp(sl), l2) : lv_band(-1022.0 + 2 * MARGIN);
        }
    }
    double G[NSLOT];
    for (int h = 0; h < n && !band; h++) {
        // N = ((1.0 * P_a1) * P_a2) ... over a != h in dict order (utils.py:18-22), then GL = H * N
        LV c = lv_normal(1.0, 0.0);
        for (int j = 0; j < n; j++)
            if (j != h) c = lv_mul(c, Pv[j]);
        const LV g = lv_mul(Hv[h], c);
        if (g.s == 2) { band = true; break; }
        G[h] = g.s == 1 ? 0.0 : g.v;
    }
    if (band) {
        const uint32_t at = atomicAdd(&O.ctr->n_band, 1u);
        if (at < (uint32_t)F.band_cap) O.band[at] = pos;
        O.flags[pos] = flags | SPG_F_REPLAYED;
        return;
    }
    for (int k = 0; k < n; k++) {
        const int s = (int)sl_[k];
#pragma unroll
        for (int j = 0; j < NSLOT; j++)
            if (s == j) gl[j] = G[k];
    }
    emit_candidates(F, O, pos, a, n, codes, cnts, G, Qv, flags);
    O.flags[pos] = flags;
}

// ------------------------------------------------------------------------------------------
// replay: exact sequential recomputation over the batch history
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_replay(FParams F, const Hist *__restrict__ H, const Acc *__restrict__ acc,
                                               const Tables *__restrict__ T, Out O) {
    const uint32_t nb = min(O.ctr->n_band, (uint32_t)F.band_cap);
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nb; t += gridDim.x * blockDim.x) {
        const int64_t pos = O.band[t];
        const Acc a = acc[pos];
        uint32_t cnt[16], ord[16];
        double P[16], Hh[16], se[16];
        int n = 0;
        uint32_t depth = 0;
        for (int c = 0; c < 16; c++) { cnt[c] = 0; P[c] = 1.0; Hh[c] = 1.0; se[c] = 0.0; }
        for (int b = 0; b < F.n_hist; b++) {
            const Hist h = H[b];
            const int64_t col = pos - h.pos_begin;
            if (col < 0 || col >= h.n_cols) continue;
            const uint64_t lo = h.off[col], hi = h.off[col + 1];
            for (uint64_t i = lo; i < hi; i++) {
                const uint32_t q = h.qual[i], c = h.code[i];
                if ((int)q < F.min_bq) continue;
                depth++;
                if (c >= 16) continue;                         // D / N: depth only
                const double e = T->eps[q];
                if (cnt[c] == 0) { ord[n++] = c; P[c] = e; Hh[c] = 1.0 - e; }   // np.prod: x0, then *=
                else { P[c] = P[c] * e; Hh[c] = Hh[c] * (1.0 - e); }
                cnt[c]++;
                se[c] += e;
            }
        }
        double G[16], Q[16];
        uint32_t codes[16], cnts[16];
        const bool evaluated = (int64_t)depth >= (int64_t)F.min_td;
        for (int h = 0; h < n; h++) {
            double non = 1.0;
            for (int j = 0; j < n; j++)
                if (j != h) non = non * P[ord[j]];
            G[h] = evaluated ? Hh[ord[h]] * non : __builtin_nan("");
            codes[h] = ord[h];
            cnts[h] = cnt[ord[h]];
            Q[h] = se[ord[h]] / (double)cnt[ord[h]];
        }
        if (evaluated) {
            double *gl = O.gl + pos * NSLOT;
            for (int h = 0; h < n; h++) {
                const int s = slot_of(codes[h]);
                if (s >= 0) gl[s] = G[h];
            }
            uint8_t flags = O.flags[pos];
            emit_candidates(F, O, pos, a, n, codes, cnts, G, Q, flags);
            O.flags[pos] = flags;
        }
        if (depth != a.depth) atomicOr(&O.ctr->err, 1u);       // history / accumulator mismatch
        const uint32_t at = atomicAdd(&O.ctr->n_detail, 1u);
        if (at < (uint32_t)F.detail_cap) {
            spg_detail d;
            d.pos = pos; d.depth = depth; d.n_alleles = (uint8_t)n;
            d.pad[0] = d.pad[1] = d.pad[2] = 0;
            for (int k = 0; k < 16; k++) {
                d.code[k] = k < n ? (uint8_t)codes[k] : 0xFF;
                d.count[k] = k < n ? cnts[k] : 0;
                d.gl[k] = k < n ? G[k] : __builtin_nan("");
            }
            O.detail[at] = d;
        }
    }
}

// ------------------------------------------------------------------------------------------
// launchers (called from spg_api.cpp)
// ------------------------------------------------------------------------------------------
hipError_t launch_accumulate(const KParams &P, const uint64_t *off, const uint8_t *code, const uint8_t *qual,
                             const uint8_t *ref, const Tables *T, Acc *acc, hipStream_t st) {
    const int64_t waves = (P.n_cols + P.G - 1) / P.G;
    const int64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_accumulate, dim3((unsigned)blocks), dim3(256), 0, st, P, off, code, qual, ref, T, acc);
    return hipGetLastError();
}

__global__ void k_set_hist(Hist *dst, Hist h) { *dst = h; }

hipError_t launch_set_hist(Hist *dst, const Hist &h, hipStream_t st) {
    hipLaunchKernelGGL(k_set_hist, dim3(1), dim3(1), 0, st, dst, h);
    return hipGetLastError();
}

hipError_t launch_finalize(const FParams &F, const Acc *acc, const Tables *T, const Out &O, const Hist *H,
                           hipStream_t st) {
    const int64_t blocks = (F.n_pos + 255) / 256;
    if (blocks) hipLaunchKernelGGL(k_finalize, dim3((unsigned)blocks), dim3(256), 0, st, F, acc, T, O);
    hipLaunchKernelGGL(k_replay, dim3(64), dim3(64), 0, st, F, H, acc, T, O);
    return hipGetLastError();
}

}  // namespace spg
