// spg_plan.hip — htslib's depth cap and mate pairing decided on the GPU for a BAM kept in HBM (include/spings_gpu.h
// spg_bam_plan_build; SURVEY §8 f1 / a3: pysam's pileup() in process_bam, variant_caller/live_variant_caller.py:55-60).
//
// The host's device plan (spp_pileup_plan_fields, csrc/spp_pileup.cpp simulate()) replays bam_plp_push / bam_plp_next
// read by read over the kept reads' fixed fields.  Two facts make it data-parallel here:
//  * Which reads the iterator keeps does not depend on the mate pairing: with coordinate-sorted reads that each span
//    >= 1 column, the first read at a start position p is always pushed, and the i-th (i >= 1) is dropped iff
//    B_p + i + 1 > maxcnt, B_p = the kept reads with pos < p and end >= p (spp_pileup.cpp capped_no_pairs).  So
//    k_p = min(n_p, max(1, maxcnt - B_p)) reads are kept at p, the first ones in BAM order.  k_plan_sweep carries B_p
//    over the distinct start positions in windows of at most min(128, shortest span) positions: no read kept inside a
//    window ends inside it, so a window's frees come from a ring of earlier kept reads' end counts (LDS), two positions
//    per lane, and only a window that can reach maxcnt runs the k recurrence position by position.
//  * The overlap hash (read name -> the first mate waiting) only ever holds one entry per name, and an entry changes
//    only at events of reads with that name: a push (pair with the entry, or insert), a drop (htslib's olap removal of
//    the dropped read's name), and a free (the read's end passed: removal of its name).  A free of read y happens
//    right after the push of the first read q with pos[q] > end[y], i.e. before the push of x iff end[y] < pos[x - 1],
//    and after the entry e's insert iff pos[e - 1] <= end[y].  So k_plan_groups sorts the reads by name hash and
//    replays each name's reads on one lane.  A pair's tweak column is htslib's iterator position at the second mate's
//    push: the position of the last kept read before it.
// Then the kept list, the kept reads' coverage -> CSR offsets, and the pairs in push order with their saved-quality
// offsets — exactly spg_bam_plan's arrays, in HBM; spg_bam_accumulate takes them from there (SPG_IN_DEVICE).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "spg_device.h"

namespace spg {

namespace {

constexpr uint32_t F_PAIRED = 0x1u, F_PROPER = 0x2u, F_MUNMAP = 0x8u;
constexpr int SWEEP_T = 1024;                  // the sweep's one workgroup
constexpr int RING = 8192;                     // kept-read end counts (LDS ring of end positions)
constexpr int GROUP_MAX = 16;                  // reads sharing one name hash replayed by one lane (more: the host plans)

__device__ __forceinline__ bool cand_of(const PlanArgs &A, uint32_t r) {        // htslib overlap_push's candidate test
    const uint32_t fl = A.flag[r];
    const int64_t is = A.isize[r];
    return !(fl & F_MUNMAP) && (fl & F_PROPER) && !(A.mtid[r] >= 0 && A.mtid[r] != A.tid) &&
           !((is < 0 ? -is : is) >= 2 * (int64_t)A.l_seq[r] && A.mpos[r] >= A.end[r]);
}
__device__ __forceinline__ bool insert_of(const PlanArgs &A, uint32_t r) {      // the first mate waits for its mate
    return A.mpos[r] >= A.pos[r] || ((A.flag[r] & F_PAIRED) && A.mpos[r] == -1);
}

__device__ __forceinline__ int32_t wave_min(int32_t v) {
    for (int o = 32; o; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int32_t wave_max(int32_t v) {
    for (int o = 32; o; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int64_t wave_max64(int64_t v) {
    for (int o = 32; o; o >>= 1) v = max(v, (int64_t)__shfl_xor((long long)v, o, 64));
    return v;
}
__device__ __forceinline__ int64_t wave_min64(int64_t v) {
    for (int o = 32; o; o >>= 1) v = min(v, (int64_t)__shfl_xor((long long)v, o, 64));
    return v;
}
__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
    for (int o = 32; o; o >>= 1) v += (int64_t)__shfl_xor((long long)v, o, 64);
    return v;
}

__global__ void k_plan_init(PlanHead *h) {
    h->min_span = INT32_MAX;
    h->max_span = INT32_MIN;
    h->max_span_kept = 0;
    h->err = 0;
    h->n_distinct = h->n_kept = h->n_pairs = 0;
    h->min_pos = INT64_MAX;                      // (both updated with unsigned 64-bit atomics: positions are >= 0)
    h->max_end = 0;
    h->lo = 0;
    h->hi = 0;
    h->n_entries = h->orig_bytes = 0;
    h->max_cov = 0;
    h->n_cand = 0;
}

// The reductions into the head: per workgroup (LDS), then one atomic per field per workgroup — the head's fields share a
// cache line, so per-wave atomics from the whole grid serialised there (r06j: 0.75 ms for 2.0 M reads).
constexpr int RED_U = 8;                       // reads per thread of the reduction kernels (grid: n / (256 RED_U))
unsigned grid_red(uint64_t n) {
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 256 * RED_U - 1) / (256 * RED_U), 1024));
}

// every read: its span (>= 1 column, else the host plans), sort order, new-position flag, pair candidates
__global__ __launch_bounds__(256) void k_plan_reads(PlanArgs A) {
    __shared__ int32_t s_mn[4], s_mx[4];
    __shared__ int64_t s_pmin[4], s_emax[4];
    __shared__ uint32_t s_bad[4], s_nc[4];
    int32_t mn = INT32_MAX, mx = INT32_MIN;
    int64_t pmin = INT64_MAX, emax = INT64_MIN;
    uint32_t bad = 0, nc = 0;
    // RED_U reads per thread per round, every load of the round issued before the first store (the arrays may alias
    // for the compiler)
    for (uint32_t r0 = blockIdx.x * 256u * RED_U + threadIdx.x; r0 < A.n; r0 += gridDim.x * 256u * RED_U) {
        int32_t p[RED_U], e[RED_U], pv[RED_U];
        bool cd[RED_U];
#pragma unroll
        for (int u = 0; u < RED_U; u++) {
            const uint32_t r = r0 + 256u * u;
            const bool in = r < A.n;
            p[u] = in ? A.pos[r] : 0;
            e[u] = in ? A.end[r] : 1;
            pv[u] = in && r ? A.pos[r - 1] : INT32_MIN;
            cd[u] = in && A.olap && cand_of(A, r);
        }
#pragma unroll
        for (int u = 0; u < RED_U; u++) {
            const uint32_t r = r0 + 256u * u;
            if (r >= A.n) continue;
            mn = min(mn, e[u] - p[u]);
            mx = max(mx, e[u] - p[u]);
            pmin = min(pmin, (int64_t)p[u]);
            emax = max(emax, (int64_t)e[u]);
            bad |= (e[u] <= p[u] || pv[u] > p[u] || p[u] < 0) ? 1u : 0u;
            A.first[r] = (r == 0 || pv[u] != p[u]) ? 1u : 0u;
            nc += cd[u] ? 1u : 0u;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) A.first[A.n] = 0;
    const int w = threadIdx.x >> 6;
    mn = wave_min(mn);
    mx = wave_max(mx);
    pmin = wave_min64(pmin);
    emax = wave_max64(emax);
    const uint32_t badw = __ballot(bad != 0) ? 1u : 0u;
    const uint32_t ncw = (uint32_t)wave_sum64((int64_t)nc);
    if ((threadIdx.x & 63) == 0) {
        s_mn[w] = mn; s_mx[w] = mx; s_pmin[w] = pmin; s_emax[w] = emax; s_bad[w] = badw; s_nc[w] = ncw;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 4; i++) {
            mn = min(mn, s_mn[i]); mx = max(mx, s_mx[i]);
            pmin = min(pmin, s_pmin[i]); emax = max(emax, s_emax[i]);
        }
        const uint32_t bd = s_bad[0] | s_bad[1] | s_bad[2] | s_bad[3], ns = s_nc[0] + s_nc[1] + s_nc[2] + s_nc[3];
        if (mn != INT32_MAX) atomicMin(&A.head->min_span, mn);
        if (mx != INT32_MIN) atomicMax(&A.head->max_span, mx);
        if (pmin != INT64_MAX) atomicMin((unsigned long long *)&A.head->min_pos, (unsigned long long)pmin);
        if (emax != INT64_MIN) atomicMax((unsigned long long *)&A.head->max_end, (unsigned long long)emax);
        if (bd) atomicOr(&A.head->err, 1u);
        if (ns) atomicAdd((uint32_t *)&A.head->n_cand, ns);
    }
}

// the distinct start positions and their first reads (didx: exclusive scan of first)
__global__ __launch_bounds__(256) void k_plan_distinct(PlanArgs A) {
    for (uint32_t r = blockIdx.x * 256u + threadIdx.x; r < A.n; r += gridDim.x * 256u)
        if (A.first[r]) {
            A.dpos[A.didx[r]] = A.pos[r];
            A.dfirst[A.didx[r]] = r;
        }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        A.dfirst[A.didx[A.n]] = A.n;
        A.head->n_distinct = A.didx[A.n];
    }
}

__device__ __forceinline__ int32_t wave_incl_scan_i32(int32_t v) {
    const int lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

__device__ __forceinline__ int32_t wave_sum32(int32_t v) {
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// htslib's depth cap over the distinct start positions in order (one workgroup; see the file comment).  Wave 0 decides
// a window's k values — up to SWEEP_W positions, two per lane — from LDS (the distinct positions and their first reads
// staged SWEEP_BLK at a time, the ring of kept-read end counts); when the cap can bite, the k recurrence runs on one
// lane (below).  Then every wave marks the window's reads and adds the kept ones' ends to the ring (below).  The
// barriers fence LDS only (the keep flags are for later kernels).  r06n shader clocks per 10,000x window before the
// med3 chain and the position-major marking: decide 13.6k (the recurrence 9.8k), mark 23.4k; r06o (med3, read-major
// marking with run-aggregated atomics): decide 9.3k (5.8k), mark 11.5k — 167k at 100,000x.
constexpr int SWEEP_BLK = 2048, SWEEP_W = 128, MARK_B = SWEEP_W / (SWEEP_T / 64);
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
__global__ __launch_bounds__(SWEEP_T) void k_plan_sweep(PlanArgs A) {
    __shared__ int32_t ring[RING];
    __shared__ int32_t sdpos[SWEEP_BLK];
    __shared__ uint32_t sdfirst[SWEEP_BLK + 1];
    __shared__ __align__(16) int32_t kk[SWEEP_W];
    __shared__ __align__(16) float sg[SWEEP_W], sn[SWEEP_W], scum[SWEEP_W];
    __shared__ uint32_t ff[SWEEP_W];
    __shared__ uint32_t s_next;
    __shared__ int32_t s_w;
    const int tid = threadIdx.x, lane = tid & 63;
    const uint32_t D = A.head->n_distinct;
    const int32_t W0 = min(SWEEP_W, A.head->min_span);
    const int32_t M = (int32_t)min(A.maxcnt, (int64_t)INT32_MAX);
    for (int i = tid; i < RING; i += SWEEP_T) ring[i] = 0;
    // the next window's positions' first 64 reads' ends (kept or not), loaded while wave 0 decides it: wave wv's
    // positions wv + 16 b, when their first reads are staged in sdfirst
    const int wv = tid >> 6;
    int32_t pe0[MARK_B];
    bool pok[MARK_B];
    uint32_t pf_d = UINT32_MAX, blk0 = 0, blk1 = 0;   // (sdpos / sdfirst hold distinct positions [blk0, blk1))
    auto prefetch = [&](uint32_t dn) __attribute__((always_inline)) {
        pf_d = dn;
#pragma unroll
        for (int b = 0; b < MARK_B; b++) {
            const uint32_t i = dn + (uint32_t)(wv + (SWEEP_T / 64) * b);
            pok[b] = i >= blk0 && i + 1 < blk1;
            const uint32_t f = pok[b] ? sdfirst[i - blk0] : 0u, n = pok[b] ? sdfirst[i + 1 - blk0] - f : 0u;
            pe0[b] = (uint32_t)lane < n ? A.end[f + (uint32_t)lane] : 0;
        }
    };
    int32_t alive = 0;                                 // (wave 0) kept reads not freed yet
    int32_t at = D ? A.dpos[0] : 0;                    // (wave 0) frees applied for every end < at
    uint32_t d = 0;
    while (d < D) {
        if (d + SWEEP_W + 1 > blk1 && blk1 < D + 1) {  // (uniform) stage the next block of distinct positions
            lds_barrier();
            blk0 = d;
            blk1 = min(D + 1, d + (uint32_t)SWEEP_BLK);
            for (uint32_t i = blk0 + (uint32_t)tid; i < blk1; i += SWEEP_T) {
                sdpos[i - blk0] = i < D ? A.dpos[i] : INT32_MAX;
                sdfirst[i - blk0] = A.dfirst[i];
            }
            lds_barrier();
        }
        if (tid < 64) {
            const int32_t P = sdpos[d - blk0];
            // window positions j = lane (half 0) and j = 64 + lane (half 1)
            const uint32_t ia = d + (uint32_t)lane, ib = ia + 64;
            const int32_t pa = ia < D ? sdpos[ia - blk0] : INT32_MAX, pb = ib < D ? sdpos[ib - blk0] : INT32_MAX;
            const bool va = ia < D && pa < P + W0, vb = ib < D && pb < P + W0;
            const int w = __popcll(__ballot(va)) + __popcll(__ballot(vb));          // (valid positions are a prefix)
            const int32_t plast = w > 64 ? __builtin_amdgcn_readlane(pb, w - 65) : __builtin_amdgcn_readlane(pa, w - 1);
            // frees of the ends in [at, P): all of them when the gap exceeds the ring
            int32_t gap = 0;
            if (P - at >= RING) {
                for (int i = lane; i < RING; i += 64) ring[i] = 0;
                gap = alive;
            } else {
                for (int32_t x = at; x < P; x += 64) {
                    const int32_t s = x + lane;
                    int32_t v = 0;
                    if (s < P) { v = ring[s & (RING - 1)]; ring[s & (RING - 1)] = 0; }
                    gap += wave_sum32(v);
                }
            }
            // frees inside the window: ends in [P, plast), two slots per lane, scanned
            int32_t c0 = 0, c1 = 0;
            if (P + lane < plast) { c0 = ring[(P + lane) & (RING - 1)]; ring[(P + lane) & (RING - 1)] = 0; }
            if (P + 64 + lane < plast) { c1 = ring[(P + 64 + lane) & (RING - 1)]; ring[(P + 64 + lane) & (RING - 1)] = 0; }
            const int32_t S0 = wave_incl_scan_i32(c0);
            const int32_t S1 = wave_incl_scan_i32(c1) + __builtin_amdgcn_readlane(S0, 63);
            // frees before position p: the scan at slot p - P - 1 (none when p == P)
            auto freed = [&](int32_t p) -> int32_t {
                const int32_t o = p - P - 1;
                const int32_t a = __shfl(S0, o & 63, 64), b = __shfl(S1, o & 63, 64);
                return o < 0 ? 0 : (o < 64 ? a : b);
            };
            const int32_t Fa = gap + freed(va ? pa : P), Fb = gap + freed(vb ? pb : P);
            const int32_t o_last = plast - P - 1;
            const int32_t Ftot = gap + (o_last < 0 ? 0 : o_last < 64 ? __builtin_amdgcn_readlane(S0, o_last)
                                                                      : __builtin_amdgcn_readlane(S1, o_last - 64));
            const uint32_t fa0 = va ? sdfirst[ia - blk0] : 0u, fa1 = va ? sdfirst[ia + 1 - blk0] : 0u;
            const uint32_t fb0 = vb ? sdfirst[ib - blk0] : 0u, fb1 = vb ? sdfirst[ib + 1 - blk0] : 0u;
            const int32_t na = (int32_t)(fa1 - fa0), nb = (int32_t)(fb1 - fb0);
            int32_t ka = na, kb = nb;
            const int32_t sum_n = wave_sum32(na + nb);
            if ((int64_t)alive + sum_n > (int64_t)M) {
                // the cap may bite: k_j = min(n_j, max(1, G_j - cum_j)), G_j = M - alive + F_j (the room at j before the
                // window's pushes), cum_j = the window's kept reads before j — in order, on one lane.  The chain is
                // cum_{j+1} = med3(cum_j + 1, G_j, cum_j + n_j) (n_j >= 1): two VALU steps per position, in fp32, exact
                // while every operand stays below 2^24; the k_j are the differences, taken by every lane afterwards
                const int32_t base = __builtin_amdgcn_readfirstlane(alive);
                if (M < (1 << 22) && base < (1 << 22) && sum_n < (1 << 22)) {
                    sg[lane] = (float)(M - base + Fa);
                    sn[lane] = (float)(va ? na : 0);       // (n = 0 past the window: its values are never read)
                    sg[64 + lane] = (float)(M - base + Fb);
                    sn[64 + lane] = (float)(vb ? nb : 0);
                    wave_lds_sync();
                    if (lane == 0) {
                        // 8 positions per round, the next round's operands read while this one's chain runs
                        float u = 0.f;
                        float4 g0 = *reinterpret_cast<const float4 *>(&sg[0]), g1 = *reinterpret_cast<const float4 *>(&sg[4]);
                        float4 n0 = *reinterpret_cast<const float4 *>(&sn[0]), n1 = *reinterpret_cast<const float4 *>(&sn[4]);
                        for (int j0 = 0; j0 < w; j0 += 8) {
                            const int jn = min(j0 + 8, SWEEP_W - 8);
                            const float4 h0 = *reinterpret_cast<const float4 *>(&sg[jn]);
                            const float4 h1 = *reinterpret_cast<const float4 *>(&sg[jn + 4]);
                            const float4 m0 = *reinterpret_cast<const float4 *>(&sn[jn]);
                            const float4 m1 = *reinterpret_cast<const float4 *>(&sn[jn + 4]);
                            const float G[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
                            const float Nn[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
                            float Cu[8];
#pragma unroll
                            for (int t = 0; t < 8; t++) {
                                u = __builtin_amdgcn_fmed3f(u + 1.f, G[t], u + Nn[t]);
                                Cu[t] = u;
                            }
                            *reinterpret_cast<float4 *>(&scum[j0]) = make_float4(Cu[0], Cu[1], Cu[2], Cu[3]);
                            *reinterpret_cast<float4 *>(&scum[j0 + 4]) = make_float4(Cu[4], Cu[5], Cu[6], Cu[7]);
                            g0 = h0; g1 = h1; n0 = m0; n1 = m1;
                        }
                    }
                    wave_lds_sync();
                    ka = (int32_t)scum[lane] - (lane ? (int32_t)scum[lane - 1] : 0);
                    kb = (int32_t)scum[64 + lane] - (int32_t)scum[63 + lane];
                } else {
                    int32_t cum = 0;                       // (large operands: the integer form, lane by lane)
                    const int wa = min(w, 64);
                    for (int j = 0; j < wa; j++) {
                        const int32_t fj = __builtin_amdgcn_readlane(Fa, j), n_ = __builtin_amdgcn_readlane(na, j);
                        const int32_t kj = min(n_, max(1, M - (base - fj + cum)));
                        ka = lane == j ? kj : ka;
                        cum += kj;
                    }
                    for (int j = 64; j < w; j++) {
                        const int32_t fj = __builtin_amdgcn_readlane(Fb, j - 64), n_ = __builtin_amdgcn_readlane(nb, j - 64);
                        const int32_t kj = min(n_, max(1, M - (base - fj + cum)));
                        kb = lane == j - 64 ? kj : kb;
                        cum += kj;
                    }
                }
            }
            alive = alive - Ftot + wave_sum32((va ? ka : 0) + (vb ? kb : 0));
            at = plast;
            if (va) { kk[lane] = ka; ff[lane] = fa0; A.first[ia] = (uint32_t)ka; }
            if (vb) { kk[64 + lane] = kb; ff[64 + lane] = fb0; A.first[ib] = (uint32_t)kb; }
            if (lane == 0) {
                s_w = w;
                s_next = d + (uint32_t)w;
            }
        }
        lds_barrier();
        // the kept reads' ends into the ring, by position: wave wv takes positions wv, wv + 16, ... of the window
        // (MARK_B of them).  A position's reads are [ff, ff + n) and the first kk are kept, so only the kept reads' ends
        // are read (every read's start and end before: 670 reads per position at 100,000x for ~53 kept); lanes = the
        // position's reads.  Its kept reads mostly end together: consecutive lanes sharing a ring slot add to it with
        // one atomic (the run's head adds the run's length).  The per-read keep flags are written afterwards by
        // k_plan_keep from the k of every position (A.first), off this one workgroup.
        const int wsz = s_w;
        auto ring_add = [&](int32_t key) __attribute__((always_inline)) {
            const int32_t prev = __shfl_up(key, 1, 64);
            const bool head = key >= 0 && (lane == 0 || prev != key);
            const uint64_t brk = __ballot(head || key < 0);
            if (head) {
                const uint64_t above = lane == 63 ? 0ull : (brk >> (lane + 1)) << (lane + 1);
                const int nxt = above ? __builtin_ctzll(above) : 64;
                atomicAdd(&ring[key], nxt - lane);
            }
        };
        {
            uint32_t fj[MARK_B], kj[MARK_B];
            int32_t e0[MARK_B];
            const bool pf = pf_d == d;                                 // (uniform) the prefetch is this window's
#pragma unroll
            for (int b = 0; b < MARK_B; b++) {
                const int j = wv + (SWEEP_T / 64) * b;
                const bool ok = j < wsz;
                fj[b] = ok ? ff[j] : 0u;
                kj[b] = ok ? (uint32_t)kk[j] : 0u;
                e0[b] = pf && pok[b] ? pe0[b] : ((uint32_t)lane < kj[b] ? A.end[fj[b] + (uint32_t)lane] : 0);
            }
#pragma unroll
            for (int b = 0; b < MARK_B; b++) {
                if (kj[b] == 0) continue;                              // (wave-uniform)
                ring_add((uint32_t)lane < kj[b] ? (e0[b] & (RING - 1)) : -1);
                for (uint32_t i0 = 64; i0 < kj[b]; i0 += 64) {          // (more than 64 kept at one position)
                    const uint32_t i = i0 + (uint32_t)lane;
                    ring_add(i < kj[b] ? (A.end[fj[b] + i] & (RING - 1)) : -1);
                }
            }
        }
        prefetch(s_next);
        d = s_next;
        lds_barrier();
    }
}

// the keep flags from the sweep's per-position k (A.first[j], j = the read's distinct position: didx[r + 1] - 1)
__global__ __launch_bounds__(256) void k_plan_keep(PlanArgs A) {
    for (uint32_t r = blockIdx.x * 256u + threadIdx.x; r < A.n; r += gridDim.x * 256u) {
        const uint32_t j = A.didx[r + 1] - 1u;
        A.keep[r] = r - A.dfirst[j] < A.first[j] ? 1 : 0;
    }
}

// one lane per name hash group: the overlap hash's events for that name, in time order (see the file comment)
__global__ __launch_bounds__(256) void k_plan_groups(PlanArgs A) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < A.n; i += gridDim.x * 256u) {
        const uint64_t key = A.skey[i];
        if (i && A.skey[i - 1] == key) continue;                         // not the group's first
        uint32_t s = 1;
        while (i + s < A.n && A.skey[i + s] == key && s <= GROUP_MAX) s++;
        if (s == 1) continue;
        if (s > GROUP_MAX) { atomicOr(&A.head->err, 2u); continue; }
        int64_t e = -1;                                                 // the entry (read index) or none
        for (uint32_t t = 0; t < s; t++) {
            const uint32_t x = A.sval[i + t];
            if (e >= 0) {
                const int64_t px = A.pos[x - 1];                         // (x > e >= 0)
                const int64_t pe = e ? A.pos[e - 1] : INT64_MIN;
                bool gone = false;
                for (uint32_t u = 0; u < t && !gone; u++) {
                    const uint32_t y = A.sval[i + u];
                    if (A.keep[y]) gone = pe <= (int64_t)A.end[y] && (int64_t)A.end[y] < px;   // y freed in between
                    else gone = (int64_t)y > e;                                                 // y dropped in between
                }
                if (gone) e = -1;
            }
            if (!A.keep[x] || !cand_of(A, x)) continue;
            if (e >= 0) {
                A.pairb[x] = (uint32_t)e + 1u;
                e = -1;
            } else if (insert_of(A, x)) {
                e = x;
            }
        }
    }
}

// the pairs in push order (second mates ascending): first mate, tweak column, the first mate's l_seq
__global__ __launch_bounds__(256) void k_plan_pairs(PlanArgs A) {
    const uint32_t np = A.head->n_pairs;
    for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < np; j += gridDim.x * 256u) {
        const uint32_t b = A.pb_list[j], a = A.pairb[b] - 1u;
        uint32_t c = b - 1u;                                             // the last kept read before b (a is one)
        while (!A.keep[c]) c--;
        A.pa[j] = a;
        A.pbv[j] = b;
        A.pcol[j] = A.pos[c];
        A.lsa[j] = A.l_seq[a];
    }
}

// the kept reads' coverage difference array over [span_lo, span_lo + span_n); all reads when `all`.  A workgroup takes
// 256 RED_U consecutive reads (coordinate order): their starts and ends fall in a window [first start, max end] that is
// usually short, so the +1 / -1 go to an LDS histogram of the window first and only its non-zero bins to the global
// array (one global atomic per read end before: ~67 reads per start position hit one address, r06j 0.46 ms).
constexpr int DIFF_BINS = 8192;
__global__ __launch_bounds__(256) void k_plan_diff(PlanArgs A, int all) {
    __shared__ int32_t bins[DIFF_BINS];
    __shared__ int32_t s_mx[4];
    __shared__ int64_t s_hi[4];
    const uint32_t n = all ? A.n : A.head->n_kept;
    const uint32_t i0 = blockIdx.x * (256u * RED_U);
    if (i0 >= n) return;                                            // (workgroup-uniform)
    const int w = threadIdx.x >> 6;
    int32_t p[RED_U], e[RED_U];
#pragma unroll
    for (int u = 0; u < RED_U; u++) {
        const uint32_t i = i0 + threadIdx.x + 256u * u;
        const uint32_t r = i < n ? (all ? i : A.kept[i]) : 0u;
        p[u] = i < n ? A.pos[r] : INT32_MAX;
        e[u] = i < n ? A.end[r] : INT32_MIN;
    }
    int32_t mx = 0;
    int64_t hi = INT64_MIN;
#pragma unroll
    for (int u = 0; u < RED_U; u++) {
        if (e[u] != INT32_MIN) {
            mx = max(mx, e[u] - p[u]);
            hi = max(hi, (int64_t)e[u]);
        }
    }
    mx = wave_max(mx);
    hi = wave_max64(hi);
    if ((threadIdx.x & 63) == 0) { s_mx[w] = mx; s_hi[w] = hi; }
    __syncthreads();
    for (int i = 0; i < 4; i++) { mx = max(mx, s_mx[i]); hi = max(hi, s_hi[i]); }
    const int32_t lo = A.pos[all ? i0 : A.kept[i0]];                // (the block's first read starts first)
    const bool lds = hi - (int64_t)lo < DIFF_BINS;                  // (uniform)
    if (lds) {
        for (int i = threadIdx.x; i < DIFF_BINS; i += 256) bins[i] = 0;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < RED_U; u++) {
            if (e[u] == INT32_MIN) continue;
            atomicAdd(&bins[p[u] - lo], 1);
            atomicAdd(&bins[e[u] - lo], -1);
        }
        __syncthreads();
        const int nb = (int)(hi - (int64_t)lo) + 1;
        for (int i = threadIdx.x; i < nb; i += 256)
            if (bins[i]) atomicAdd(&A.diff[(int64_t)lo + i - A.span_lo], bins[i]);
    } else {
#pragma unroll
        for (int u = 0; u < RED_U; u++) {
            if (e[u] == INT32_MIN) continue;
            atomicAdd(&A.diff[p[u] - A.span_lo], 1);
            atomicAdd(&A.diff[e[u] - A.span_lo], -1);
        }
    }
    if (!all && threadIdx.x == 0) {
        atomicMax(&A.head->max_span_kept, mx);
        if (hi != INT64_MIN) atomicMax((unsigned long long *)&A.head->hi, (unsigned long long)hi);
    }
}

// the coverage maximum (the global cold check of a long contig)
__global__ __launch_bounds__(256) void k_plan_covmax(PlanArgs A, const int32_t *cov) {
    int32_t mx = 0;
    for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < A.span_n; c += (int64_t)gridDim.x * 256)
        mx = max(mx, cov[c]);
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) atomicMax(&A.head->max_cov, mx);
}

__global__ void k_plan_tail(PlanArgs A) {
    PlanHead *h = A.head;
    if (h->n_kept) {
        h->lo = A.pos[A.kept[0]];
        h->n_entries = A.offsets[h->hi - A.span_lo];
    } else {
        h->lo = h->hi = 0;
    }
    h->orig_bytes = h->n_pairs ? A.porig[h->n_pairs - 1] + A.lsa[h->n_pairs - 1] : 0;
}

__global__ __launch_bounds__(256) void k_plan_fill_u8(uint8_t *p, uint32_t n, uint8_t v) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) p[i] = v;
}
__global__ __launch_bounds__(256) void k_plan_iota(uint32_t *p, uint32_t n) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) p[i] = i;
}

struct NonZero {
    __host__ __device__ __forceinline__ bool operator()(const uint32_t &v) const { return v != 0; }
};
struct ToU64 {
    __host__ __device__ __forceinline__ uint64_t operator()(const int32_t &v) const { return (uint64_t)(int64_t)v; }
};
using CovU64 = hipcub::TransformInputIterator<uint64_t, ToU64, const int32_t *>;

unsigned grid_for(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 4096)); }

}  // namespace

// hipcub scratch the plan's scans / compactions / sort need for n reads and a column span of span_n
size_t plan_temp_bytes(uint32_t n, int64_t span_n) {
    size_t need = 0, b = 0;
    const int ni = (int)n;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint32_t *)nullptr, (uint32_t *)nullptr, ni + 1);
    need = std::max(need, b);
    hipcub::CountingInputIterator<uint32_t> it(0);
    (void)hipcub::DeviceSelect::Flagged(nullptr, b, it, (uint8_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr, ni);
    need = std::max(need, b);
    hipcub::TransformInputIterator<bool, NonZero, const uint32_t *> nz((const uint32_t *)nullptr, NonZero());
    (void)hipcub::DeviceSelect::Flagged(nullptr, b, it, nz, (uint32_t *)nullptr, (uint32_t *)nullptr, ni);
    need = std::max(need, b);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                             (const uint32_t *)nullptr, (uint32_t *)nullptr, ni);
    need = std::max(need, b);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr, ni);
    need = std::max(need, b);
    if (span_n > 0) {
        (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, (int32_t *)nullptr, (int32_t *)nullptr, (int)(span_n + 1));
        need = std::max(need, b);
        (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, CovU64((const int32_t *)nullptr, ToU64()), (uint64_t *)nullptr,
                                               (int)(span_n + 1));
        need = std::max(need, b);
    }
    return need + 256;
}

// stage 0: every read's fields checked, the distinct start positions listed (then the host reads the head)
hipError_t launch_plan_reads(const PlanArgs &A, void *tmp, size_t tmp_bytes, hipStream_t st) {
    k_plan_init<<<1, 1, 0, st>>>(A.head);
    k_plan_reads<<<grid_red(A.n), 256, 0, st>>>(A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, A.first, A.didx, (int)A.n + 1, st);
    if (e != hipSuccess) return e;
    k_plan_distinct<<<grid_for(A.n), 256, 0, st>>>(A);
    return hipGetLastError();
}

// the coverage of every read (all = 1: the global cold check, max_cov) or of the kept ones (CSR offsets)
hipError_t launch_plan_cov(const PlanArgs &A, int all, int32_t *cov, void *tmp, size_t tmp_bytes, hipStream_t st) {
    hipError_t e = hipMemsetAsync(A.diff, 0, sizeof(int32_t) * (size_t)(A.span_n + 1), st);
    if (e != hipSuccess) return e;
    k_plan_diff<<<(unsigned)((A.n + 256u * RED_U - 1) / (256u * RED_U)), 256, 0, st>>>(A, all);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    e = hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, A.diff, cov, (int)(A.span_n + 1), st);
    if (e != hipSuccess) return e;
    if (all) {
        k_plan_covmax<<<grid_for((uint64_t)A.span_n), 256, 0, st>>>(A, cov);
        return hipGetLastError();
    }
    // offsets[c] = the entries of columns before c (cov[span_n] is 0: the difference array sums to 0)
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, CovU64(cov, ToU64()), A.offsets, (int)(A.span_n + 1), st);
}

// keep: every read (uncapped, or the cap never reached), or the sweep
hipError_t launch_plan_keep(const PlanArgs &A, bool sweep, hipStream_t st) {
    if (!sweep) {
        k_plan_fill_u8<<<grid_for(A.n), 256, 0, st>>>(A.keep, A.n, 1);
        return hipGetLastError();
    }
    k_plan_sweep<<<1, SWEEP_T, 0, st>>>(A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    k_plan_keep<<<grid_for(A.n), 256, 0, st>>>(A);
    return hipGetLastError();
}

// the kept list, the kept reads' CSR offsets, the pairs (when pairing), the head's totals
hipError_t launch_plan_rest(const PlanArgs &A, int32_t *cov, bool pairing, void *tmp, size_t tmp_bytes, hipStream_t st) {
    hipcub::CountingInputIterator<uint32_t> it(0);
    hipError_t e = hipcub::DeviceSelect::Flagged(tmp, tmp_bytes, it, A.keep, A.kept, &A.head->n_kept, (int)A.n, st);
    if (e != hipSuccess) return e;
    if ((e = launch_plan_cov(A, 0, cov, tmp, tmp_bytes, st)) != hipSuccess) return e;
    if (pairing) {
        if ((e = hipMemsetAsync(A.pairb, 0, sizeof(uint32_t) * A.n, st)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(A.lsa, 0, sizeof(uint64_t) * A.n, st)) != hipSuccess) return e;
        k_plan_iota<<<grid_for(A.n), 256, 0, st>>>(A.pb_list, A.n);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, (const uint64_t *)A.nhash, A.skey, (const uint32_t *)A.pb_list,
                                               A.sval, (int)A.n, 0, 64, st);
        if (e != hipSuccess) return e;
        k_plan_groups<<<grid_for(A.n), 256, 0, st>>>(A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipcub::TransformInputIterator<bool, NonZero, const uint32_t *> nz(A.pairb, NonZero());
        e = hipcub::DeviceSelect::Flagged(tmp, tmp_bytes, it, nz, A.pb_list, &A.head->n_pairs, (int)A.n, st);
        if (e != hipSuccess) return e;
        k_plan_pairs<<<grid_for(A.n), 256, 0, st>>>(A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        e = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, A.lsa, A.porig, (int)A.n, st);
        if (e != hipSuccess) return e;
    }
    k_plan_tail<<<1, 1, 0, st>>>(A);
    return hipGetLastError();
}

}  // namespace spg
