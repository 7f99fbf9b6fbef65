// spg_bam.hip — a BAM kept in HBM from its compressed bytes to the CSR batch (include/spings_gpu.h
// spg_bam_*): the lone process_bam (variant_caller/live_variant_caller.py:54-72, pysam's AlignmentFile + pileup) with
// only the compressed file going up and the reads' fixed fields coming down.
//
// After k_inflate has written the inflated stream into HBM:
//   k_bam_starts  one wave per BGZF member: the first record that starts inside the member's inflated range — the
//                 offset where a block_size hop lands on a plausible record eight times in a row (or on the stream's
//                 end); the member holding the header's end starts there.
//   k_bam_walk    16 lanes per member with a start: the block_size chain from its start to the next member's start,
//                 counting the records of the contig the stepper keeps and listing them per member (pass 1; k_bam_copy
//                 moves the lists to the exclusive prefix of the counts — or, for a chain of more than BAM_RTMP, a
//                 second walk lists them there, pass 2); every chain must land exactly on the next start (else the
//                 host plans this BAM); the first / last position of the contig's records per member (sort order, on
//                 the host).
//   k_bam_fields  one lane per listed read: pos, reference end (CIGAR walk), flag, mate fields, l_seq and a 64-bit
//                 FNV-1a hash of the name — what htslib's depth cap and the mate pairing decide on (the host replays
//                 them on these fields: spp_pileup_plan_fields).
// Then, with the host's plan:
//   k_bam_pair_names  the pairs the host matched by name hash have equal names (else the host plans this BAM);
//   k_bam_tweak   htslib's mate-overlap quality tweak applied to the pair's qualities in place (the first mate's
//                 original qualities saved first: D / N entries before the tweak column read them);
//   k_bam_gather  the kept reads' record offsets / spans / tweak indices in BAM order -> k_pileup_fill (spg_fill.hip).
// Record fields are read with aligned dword loads (records start at any byte offset).
#include <hip/hip_runtime.h>

#include "spg_device.h"

namespace spg {

namespace {

template <typename T>
using gptr = const __attribute__((address_space(1))) T *;

__device__ __forceinline__ uint32_t ldu32(const uint8_t *base, uint64_t off) {
    gptr<uint32_t> w = (gptr<uint32_t>)(const void *)(base + (off & ~3ull));
    const uint32_t lo = w[0], hi = w[1];
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(off & 3));
}
__device__ __forceinline__ int32_t ldi32(const uint8_t *b, uint64_t o) { return (int32_t)ldu32(b, o); }
__device__ __forceinline__ uint32_t ldu8(const uint8_t *b, uint64_t o) { return ((gptr<uint8_t>)(const void *)b)[o]; }

__device__ __forceinline__ bool eats_ref(uint32_t op) { return op == 0 || op == 2 || op == 3 || op == 7 || op == 8; }
__device__ __forceinline__ bool eats_query(uint32_t op) { return op == 0 || op == 1 || op == 4 || op == 7 || op == 8; }

// pysam's stepper read filter + htslib's unmapped skip (spp_pileup.cpp stepper_keeps)
__device__ __forceinline__ bool keeps(const BamArgs &A, uint32_t flag, uint32_t mapq) {
    if (flag & 0x4u) return false;
    if (A.stepper == 1) return true;                                        // nofilter
    if (A.stepper == 0) return !(flag & (0x4u | 0x100u | 0x200u | 0x400u));   // all
    if (flag & A.flag_filter) return false;                                 // samtools
    if ((int32_t)mapq < A.min_mapq) return false;
    if ((flag & 0x1u) && !(flag & 0x2u)) return false;
    return true;
}

// 4 + block_size when a plausible record starts at x (the host's parallel-scan validator), else 0
__device__ __forceinline__ uint64_t rec_len(const BamArgs &A, uint64_t x) {
    if (x + 40 > A.total) return 0;
    const uint32_t bs = ldu32(A.data, x);
    if (bs < 32 || bs > (1u << 26) || x + 4 + (uint64_t)bs > A.total) return 0;
    const uint64_t b = x + 4;
    const int32_t ref = ldi32(A.data, b), pos = ldi32(A.data, b + 4), mref = ldi32(A.data, b + 20);
    if (ref < -1 || ref >= A.n_ref || mref < -1 || mref >= A.n_ref || pos < -1) return 0;
    const uint32_t w8 = ldu32(A.data, b + 8), w12 = ldu32(A.data, b + 12);
    const uint32_t l_name = w8 & 0xFFu, n_cig = w12 & 0xFFFFu;
    const int32_t l_seq = ldi32(A.data, b + 16);
    if (l_name < 1 || l_seq < 0 ||
        32ull + l_name + 4ull * n_cig + ((uint64_t)l_seq + 1) / 2 + (uint64_t)l_seq > (uint64_t)bs)
        return 0;
    if (ldu8(A.data, b + 32 + l_name - 1) != 0) return 0;
    return 4 + (uint64_t)bs;
}

}  // namespace

// one wave per member: 64 candidate offsets tested at a time, the first (lowest) that validates wins — the same answer as
// testing them one after another (r05: one lane per member scanning serially took 0.56 ms per 10,000x BAM)
__global__ __launch_bounds__(256) void k_bam_starts(BamArgs A) {
    const int lane = threadIdx.x & 63;
    const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= A.n_members) return;
    const uint64_t lo = A.uoff[m], hi = A.uoff[m + 1];
    uint64_t s = BAM_NONE;
    if (hi > A.body && lo < A.total) {
        if (lo <= A.body) {
            s = A.body;
        } else {
            const uint64_t lim = min(hi, lo + 65536ull);
            for (uint64_t x0 = lo; x0 < lim; x0 += 64) {
                const uint64_t x = x0 + (uint64_t)lane;
                bool ok = false;
                if (x < lim) {
                    uint64_t y = x;
                    int k = 0;
                    for (; k < 8 && y < A.total; k++) {
                        const uint64_t len = rec_len(A, y);
                        if (!len) break;
                        y += len;
                    }
                    ok = k == 8 || y == A.total;
                }
                const uint64_t okm = __ballot(ok);
                if (okm) {
                    s = x0 + (uint64_t)__builtin_ctzll(okm);
                    break;
                }
            }
        }
    }
    if (lane == 0) A.start[m] = s;
}

// One wave per member: the block_size chain is a dependent load per record (~240 per 64 KiB member), so the wave
// copies a WALK_W-byte window of the stream into LDS with one round of 16-B loads and walks the records' headers there
// (every lane the same walk, broadcast LDS reads; lane 0 stores), reloading the window at the record that leaves it.
// (r05-r06: one lane per member walked the chain through L2 — 8,357 lanes in 131 waves, one HBM / MALL round trip per
// record: 0.41 ms per 10,000x BAM; one member per wave 0.30 ms — the same with the next window prefetched in
// registers, r06ai: the walk's instructions, not the window loads, were left — and 4 members per wave 0.19 ms
// (8: 0.33, 16: 0.51, r06ao).)
constexpr int WALK_W = 4096, WALK_G = 4;
template <bool WRITE>
__global__ __launch_bounds__(64) void k_bam_walk(BamArgs A) {
    // WALK_G members per wave, 64 / WALK_G lanes each (a lane group walks its member; the groups run side by side, so
    // one instruction stream serves WALK_G chains)
    constexpr int GL = 64 / WALK_G;
    __shared__ __align__(16) uint32_t win[WALK_G][WALK_W / 4 + 4];
    const int lane = threadIdx.x, grp = lane / GL, gl = lane % GL;
    const int64_t m = (int64_t)blockIdx.x * WALK_G + grp;
    if (m >= A.n_members) return;                                           // (the group's lanes alike)
    uint64_t x = A.start[m];
    if (x == BAM_NONE) {
        if (!WRITE && gl == 0) { A.cnt[m] = 0; A.pos_lo[m] = INT64_MAX; A.pos_hi[m] = -1; }
        return;
    }
    uint64_t nx = A.total;                                                  // the next member with a start
    for (int64_t k = m + 1; k < A.n_members; k++) {
        const uint64_t sk = A.start[k];
        if (sk != BAM_NONE) { nx = sk; break; }
    }
    uint32_t *const wl = win[grp];
    uint64_t wa = ~0ull;                                                    // the window's first byte (none yet)
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const u32x4 gu128;
    constexpr int NV = WALK_W / 16 / GL, NR = NV;                           // 16-B chunks per lane per window
    auto refill = [&](uint64_t xx) __attribute__((always_inline)) {         // the window from xx's 16-B block on
        const uint64_t a0 = xx & ~15ull;
        wa = a0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int k0 = 0; k0 < NV; k0 += NR) {                               // NR chunks in flight per round
            u32x4 v[NR];
#pragma unroll
            for (int k = 0; k < NR; k++) {
                const uint64_t g = a0 + 16ull * (uint64_t)(gl + GL * (k0 + k));
                v[k] = g + 16 <= A.total + 64 ? *(gu128 *)(const void *)(A.data + g) : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int k = 0; k < NR; k++) *reinterpret_cast<u32x4 *>(&wl[4 * (gl + GL * (k0 + k))]) = v[k];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    uint32_t kept = 0, bad = 0;
    int64_t first = INT64_MAX, last = -1;
    const uint32_t at = WRITE ? A.base[m] : 0u;
    while (x < nx) {
        if (x + 36 > A.total) { bad = 1; break; }
        if (wa == ~0ull || x < wa || x + 36 > wa + WALK_W) refill(x);
        // the header's first 20 bytes (block_size, refID, pos, bin_mq_nl, flag_nc) from six dwords of the window
        const uint32_t o = (uint32_t)(x - wa), i0 = o >> 2, sh = o & 3u;
        uint32_t d[6];
#pragma unroll
        for (int k = 0; k < 6; k++) d[k] = wl[i0 + k];
        const uint32_t bs = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
        if (bs < 32 || x + 4 + (uint64_t)bs > A.total) { bad = 1; break; }
        const uint64_t b = x + 4;
        if ((int32_t)__builtin_amdgcn_alignbyte(d[2], d[1], sh) == A.tid) {
            const int64_t pos = (int32_t)__builtin_amdgcn_alignbyte(d[3], d[2], sh);
            if (first == INT64_MAX) first = pos;
            if (pos < last) bad |= 2;
            last = pos;
            const uint32_t w8 = __builtin_amdgcn_alignbyte(d[4], d[3], sh), w12 = __builtin_amdgcn_alignbyte(d[5], d[4], sh);
            if (keeps(A, w12 >> 16, (w8 >> 8) & 0xFFu)) {
                if (gl == 0) {
                    if (WRITE) A.rec[at + kept] = b;
                    else if (kept < BAM_RTMP) A.rtmp[(uint64_t)m * BAM_RTMP + kept] = b;
                }
                kept++;
            }
        }
        x = b + bs;
    }
    if (x != nx) bad |= 1;
    if (!WRITE && gl == 0) {
        A.cnt[m] = kept;
        A.pos_lo[m] = first;
        A.pos_hi[m] = last;
        if (bad) atomicOr(A.err, bad);
    }
}

// the counting walk's lists to their place in rec (every member's count <= BAM_RTMP; else pass 2 walks again)
__global__ __launch_bounds__(256) void k_bam_copy(BamArgs A) {
    const int lane = threadIdx.x & 63;
    const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= A.n_members) return;
    const uint32_t n = A.cnt[m], at = A.base[m];
    for (uint32_t k = (uint32_t)lane; k < n; k += 64) A.rec[at + k] = A.rtmp[(uint64_t)m * BAM_RTMP + k];
}

__global__ __launch_bounds__(256) void k_bam_fields(BamArgs A) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= A.n_reads) return;
    const uint64_t b = A.rec[i];
    // the 36-byte header [b - 4, b + 32) from four 16-B loads of its aligned window: hd[j] = the header's dword j
    // (block_size, refID, pos, bin_mq_nl, flag_nc, l_seq, next_refID, next_pos, tlen) — eight unaligned-dword reads of
    // two loads each before
    uint32_t hd[9];
    {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) const u32x4 gu128;
        const uint64_t h0 = b - 4, a0 = h0 & ~15ull;
        const uint32_t q = (uint32_t)(h0 - a0) >> 2, r = (uint32_t)(h0 - a0) & 3u;
        uint32_t W[16];
#pragma unroll
        for (int k = 0; k < 4; k++) {                                      // (inside the record + pad)
            const u32x4 v = *(gu128 *)(const void *)(A.data + a0 + 16 * k);
            W[4 * k] = v.x; W[4 * k + 1] = v.y; W[4 * k + 2] = v.z; W[4 * k + 3] = v.w;
        }
        uint32_t S[10];
#pragma unroll
        for (int t = 0; t < 10; t++) S[t] = q == 0 ? W[t] : q == 1 ? W[t + 1] : q == 2 ? W[t + 2] : W[t + 3];
#pragma unroll
        for (int j = 0; j < 9; j++) hd[j] = __builtin_amdgcn_alignbyte(S[j + 1], S[j], r);
    }
    const uint32_t bs = hd[0];
    const uint32_t w8 = hd[3], w12 = hd[4];
    const uint32_t l_name = w8 & 0xFFu, n_cig = w12 & 0xFFFFu;
    const int32_t pos = (int32_t)hd[2], l_seq = (int32_t)hd[5];
    if (l_name < 1 || l_seq < 0 ||
        32ull + l_name + 4ull * n_cig + ((uint64_t)l_seq + 1) / 2 + (uint64_t)l_seq > (uint64_t)bs) {
        atomicOr(A.err, 4u);
        return;
    }
    int64_t rl = 0;
    const uint64_t co = b + 32 + l_name;
    for (uint32_t j = 0; j < n_cig; j++) {
        const uint32_t c = ldu32(A.data, co + 4ull * j);
        if (eats_ref(c & 15u)) rl += c >> 4;
    }
    // FNV-1a 64 over the name (its NUL excluded): the 64 bytes from the name's 16-B aligned start taken with four 16-B
    // loads, each byte folded in when it lies in the name (one byte load per name byte before: ~30 scattered loads per
    // read, 0.32 ms per 10,000x BAM); a longer name's rest byte by byte
    uint64_t h = 0xcbf29ce484222325ull;
    {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) const u32x4 gu128;
        const uint64_t n0 = b + 32, n1 = n0 + l_name - 1, a0 = n0 & ~15ull;
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = *(gu128 *)(const void *)(A.data + a0 + 16 * k);   // (inside the record + pad)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t wd[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint64_t at = a0 + 16 * k + i;
                const uint64_t hx = (h ^ ((wd[i >> 2] >> (8 * (i & 3))) & 0xFFu)) * 0x100000001b3ull;
                h = at >= n0 && at < n1 ? hx : h;
            }
        }
        for (uint64_t at = a0 + 64; at < n1; at++) h = (h ^ ldu8(A.data, at)) * 0x100000001b3ull;
    }
    A.pos[i] = pos;
    A.end[i] = (int32_t)(pos + rl);
    A.flag[i] = (uint16_t)(w12 >> 16);
    A.mtid[i] = (int32_t)hd[6];
    A.mpos[i] = (int32_t)hd[7];
    A.isize[i] = (int32_t)hd[8];
    A.l_seq[i] = (uint32_t)l_seq;
    A.nhash[i] = h;
}

// the pairs the host matched by name hash: equal names, or the plan is refused (err |= 8)
__global__ __launch_bounds__(256) void k_bam_pair_names(BamPairArgs P) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= P.n_pairs) return;
    const uint32_t ia = P.pa[j], ib = P.pb[j];
    if (ia >= P.n_reads || ib >= P.n_reads) { atomicOr(P.err, 8u); return; }
    const uint64_t a = P.rec[ia], b = P.rec[ib];
    const uint32_t la = ldu32(P.data, a + 8) & 0xFFu, lb = ldu32(P.data, b + 8) & 0xFFu;
    bool same = la == lb;
    for (uint32_t k = 0; same && k < la; k++) same = ldu8(P.data, a + 32 + k) == ldu8(P.data, b + 32 + k);
    if (!same) atomicOr(P.err, 8u);
}

// htslib tweak_overlap_quality (spp_pileup.cpp tweak_overlap) on pair j: read a's qualities saved to orig + oq[j], then
// at every reference position where both mates have an aligned M/=/X base: equal bases -> a.q = min(a.q + b.q, 200),
// b.q = 0; different -> the higher (a on ties) keeps (uint8)(0.8 q), the other 0; the walk stops at a query index past
// either read's sequence
__global__ __launch_bounds__(64) void k_bam_tweak(BamPairArgs P) {
    const uint32_t j = blockIdx.x * 64 + threadIdx.x;
    if (j >= P.n_pairs) return;
    uint8_t *const D = P.wdata;
    const uint64_t ra = P.rec[P.pa[j]], rb = P.rec[P.pb[j]];
    struct Rd {
        uint64_t co, so, qo;
        uint32_t ncig, ls, ci, op, len, k;     // current op, its length, bases of it consumed
        int64_t x;                             // the op's first reference position
        uint32_t y;                            // the op's first query index
    } r[2];
    const uint64_t rr[2] = {ra, rb};
    for (int t = 0; t < 2; t++) {
        const uint64_t b = rr[t];
        const uint32_t l_name = ldu32(D, b + 8) & 0xFFu;
        r[t].ncig = ldu32(D, b + 12) & 0xFFFFu;
        r[t].ls = (uint32_t)ldi32(D, b + 16);
        r[t].co = b + 32 + l_name;
        r[t].so = r[t].co + 4ull * r[t].ncig;
        r[t].qo = r[t].so + (r[t].ls + 1) / 2;
        r[t].x = ldi32(D, b + 4);
        r[t].y = 0;
        r[t].ci = 0;
        r[t].k = 0;
        r[t].op = 15;
        r[t].len = 0;
    }
    // save a's qualities before any change
    for (uint32_t k = 0; k < r[0].ls; k++) P.orig[P.oq[j] + k] = (uint8_t)ldu8(D, r[0].qo + k);
    // advance read t to its next aligned (M / = / X) base; false when its CIGAR is exhausted
    auto next_aligned = [&](Rd &q) -> bool {
        for (;;) {
            if (q.op != 15 && (q.op == 0 || q.op == 7 || q.op == 8) && q.k < q.len) return true;
            if (q.op != 15) {                   // leave the current op
                if (eats_ref(q.op)) q.x += q.len;
                if (eats_query(q.op)) q.y += q.len;
            }
            if (q.ci >= q.ncig) return false;
            const uint32_t c = ldu32(D, q.co + 4ull * q.ci++);
            q.op = c & 15u;
            q.len = c >> 4;
            q.k = 0;
        }
    };
    bool ha = next_aligned(r[0]), hb = next_aligned(r[1]);
    while (ha && hb) {
        const int64_t pa = r[0].x + r[0].k, pb = r[1].x + r[1].k;
        if (pa < pb) {                          // skip a's aligned bases before b's position (within this op)
            r[0].k += (uint32_t)min((int64_t)(r[0].len - r[0].k), pb - pa);
            ha = next_aligned(r[0]);
            continue;
        }
        if (pb < pa) {
            r[1].k += (uint32_t)min((int64_t)(r[1].len - r[1].k), pa - pb);
            hb = next_aligned(r[1]);
            continue;
        }
        const uint32_t ia = r[0].y + r[0].k, ib = r[1].y + r[1].k;
        if (ia >= r[0].ls || ib >= r[1].ls) return;
        const uint32_t sa = ldu8(D, r[0].so + ia / 2), sb = ldu8(D, r[1].so + ib / 2);
        const uint32_t ba = (ia & 1) ? (sa & 15u) : (sa >> 4), bb = (ib & 1) ? (sb & 15u) : (sb >> 4);
        const uint32_t qa = ldu8(D, r[0].qo + ia), qb = ldu8(D, r[1].qo + ib);
        uint32_t na, nb;
        if (ba == bb) {
            na = min(qa + qb, 200u);
            nb = 0;
        } else if (qa >= qb) {
            na = (uint32_t)(uint8_t)(0.8 * (double)qa);
            nb = 0;
        } else {
            nb = (uint32_t)(uint8_t)(0.8 * (double)qb);
            na = 0;
        }
        D[r[0].qo + ia] = (uint8_t)na;
        D[r[1].qo + ib] = (uint8_t)nb;
        r[0].k++;
        r[1].k++;
        ha = next_aligned(r[0]);
        hb = next_aligned(r[1]);
    }
}

// kept read i (BAM order) -> the fill's per-read arrays; tweak index from the pairs' first mates
__global__ __launch_bounds__(256) void k_bam_gather(BamGatherArgs G) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < G.n_pairs) G.twof[G.pa[i]] = (int32_t)i;      // (twof cleared to -1 before; pairs before kept: 2 launches)
    (void)i;
}
__global__ __launch_bounds__(256) void k_bam_gather2(BamGatherArgs G) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= G.n_kept) return;
    const uint32_t r = G.kept[i];
    if (r >= G.n_reads) { atomicOr(G.err, 2u); return; }
    G.rec_k[i] = G.rec[r];
    G.rpos_k[i] = G.pos[r];
    G.rend_k[i] = G.end[r];
    G.tw_k[i] = G.twof[r];
}

// pass 0 starts, 1 counting walk (+ lists), 2 listing walk, 3 fields, 4 the lists copied (instead of pass 2)
hipError_t launch_bam_scan(const BamArgs &A, int pass, hipStream_t st) {
    const unsigned mb = (unsigned)((A.n_members + 63) / 64), mw = (unsigned)((A.n_members + 3) / 4);
    if (pass == 0) k_bam_starts<<<mw, 256, 0, st>>>(A);
    else if (pass == 1) k_bam_walk<false><<<(unsigned)((A.n_members + WALK_G - 1) / WALK_G), 64, 0, st>>>(A);
    else if (pass == 2) k_bam_walk<true><<<(unsigned)((A.n_members + WALK_G - 1) / WALK_G), 64, 0, st>>>(A);
    else if (pass == 4) k_bam_copy<<<mw, 256, 0, st>>>(A);
    else if (A.n_reads) k_bam_fields<<<(A.n_reads + 255) / 256, 256, 0, st>>>(A);
    return hipGetLastError();
}

hipError_t launch_bam_pairs(const BamPairArgs &P, bool tweak, hipStream_t st) {
    if (!P.n_pairs) return hipSuccess;
    if (!tweak) k_bam_pair_names<<<(P.n_pairs + 255) / 256, 256, 0, st>>>(P);
    else k_bam_tweak<<<(P.n_pairs + 63) / 64, 64, 0, st>>>(P);
    return hipGetLastError();
}

hipError_t launch_bam_gather(const BamGatherArgs &G, hipStream_t st) {
    if (G.n_pairs) k_bam_gather<<<(G.n_pairs + 255) / 256, 256, 0, st>>>(G);
    if (G.n_kept) k_bam_gather2<<<(G.n_kept + 255) / 256, 256, 0, st>>>(G);
    return hipGetLastError();
}

}  // namespace spg
