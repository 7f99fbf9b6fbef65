// spg_fill.hip — device-side pileup of BAM records into the CSR batch (include/spings_gpu.h
// spg_accumulate_records).
//
// Replaces the host CIGAR walk behind LiveVariantCaller.process_bam (variant_caller/live_variant_caller.py:
// 54-72, pysam's pileup columns :74-90): the host keeps what decides WHICH reads enter a column (stepper
// filter, htslib's depth cap, mate-overlap tweak, CSR offsets — spp_pileup_plan_records) and this kernel
// writes WHAT they contribute: per covered column the read's BAM nibble and quality, or 16 / 17 for a
// CIGAR D / N with the quality of the next query base (0 past the read end), in htslib's per-column order
// (the column's reads in BAM order).  Bit-identical to spp_batch_fill of the same plan (tests/
// test_device_pileup_gpu.py).
//
// Layout: one wave per tile of 64 consecutive columns; lane j holds column c0 + j's write cursor (CSR
// offset + entries written).  The tile's reads — those starting at most max_span before it, up to its end
// (tile_first) — are taken 64 at a time in BAM order, one per lane; the wave steps the columns the chunk
// covers, each lane walking its own CIGAR, and the covering lanes of a column write consecutive entries
// at (cursor + rank among them): one coalesced byte store per array per column.  Consecutive tiles go to
// one XCD (its L2 holds the records they share).  HBM-bound: the records are read once per tile they
// overlap and each entry is written once.
#include "spg_device.h"

namespace spg {


namespace {

template <typename T>
using gptr = const __attribute__((address_space(1))) T *;
template <typename T>
__device__ __forceinline__ gptr<T> g(const T *p) { return (gptr<T>)p; }

// u32 at any byte offset (two aligned dword loads + v_alignbyte; the buffers are padded)
__device__ __forceinline__ uint32_t ld32u(const uint8_t *base, uint64_t off) {
    gptr<uint32_t> w = g(reinterpret_cast<const uint32_t *>(base + (off & ~3ull)));
    const uint32_t lo = w[0], hi = w[1];
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(off & 3));
}

__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
    for (int o = 32; o; o >>= 1) v = min(v, __shfl_xor(v, o));
    return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {
    for (int o = 32; o; o >>= 1) v = max(v, __shfl_xor(v, o));
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ bool eats_ref(uint32_t op) { return op == 0 || op == 2 || op == 3 || op == 7 || op == 8; }
__device__ __forceinline__ bool eats_query(uint32_t op) { return op == 0 || op == 1 || op == 4 || op == 7 || op == 8; }

}  // namespace

// tile_first[k] = first read with rpos >= pos_begin + 64k (k >= 1), tile_first[0] = 0: thread r writes the
// boundaries between read r - 1's tile and its own (thread n_reads: those after the last read).
__global__ void k_tile_first(FillArgs A) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > A.n_reads) return;
    auto tile_of = [&](uint64_t i) -> int64_t {
        if (i >= A.n_reads) return A.n_tiles;
        const int64_t d = (int64_t)A.rpos[i] - A.pos_begin;
        return d < 0 ? -1 : min(d >> 6, (int64_t)A.n_tiles);
    };
    const int64_t hi = tile_of(r), lo = r ? tile_of(r - 1) : -1;
    if (r == 0) A.tile_first[0] = 0;
    for (int64_t k = max(lo + 1, (int64_t)1); k <= hi; k++) A.tile_first[k] = (uint32_t)r;
}

__global__ __launch_bounds__(256) void k_pileup_fill(FillArgs A) {
    const int lane = threadIdx.x & 63;
    // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs; consecutive tiles land on one
    const uint32_t nb = gridDim.x, per = nb >> 3, b = blockIdx.x;
    const uint32_t blk = (b & 7) * per + (b >> 3);
    const int32_t tile = (int32_t)(blk * 4 + (threadIdx.x >> 6));
    if (tile >= A.n_tiles) return;   // wave-uniform
    const int32_t c0 = tile * 64, W = min(64, A.n_cols - c0);
    uint64_t cur = 0, cend = 0;
    if (lane < W) {
        cur = A.off[c0 + lane];
        cend = A.off[c0 + lane + 1];
    }
    const int32_t kb = max(tile - A.back, 0);
    const uint32_t r0 = A.tile_first[kb], r1 = A.tile_first[tile + 1];
    const int64_t P0 = A.pos_begin + c0;
    uint32_t bad = 0;
    for (uint32_t rb = r0; rb < r1; rb += 64) {
        const uint32_t r = rb + (uint32_t)lane;
        int32_t s = 0, e = 0, x = 0;             // tile-relative: covered columns [s, e); CIGAR op start x
        if (r < r1) {
            x = (int32_t)((int64_t)A.rpos[r] - P0);
            s = max(x, 0);
            e = (int32_t)min((int64_t)A.rend[r] - P0, (int64_t)W);
        }
        bool act = s < e;
        if (__ballot(act) == 0) continue;
        const int32_t smin = wave_min_i32(act ? s : INT32_MAX), emax = wave_max_i32(act ? e : 0);
        uint64_t co = 0, so = 0, qo = 0, oq = 0;
        uint32_t ncig = 0, ls = 0, y = 0, ci = 0, op = 0, len = 0;
        int32_t tcol = INT32_MIN;                // D/N entries in columns < tcol read orig (none: no tweak)
        if (act) {
            const uint64_t ro = min(A.rec[r], A.data_bytes);    // (the host checked rec + 36 <= data_bytes)
            const uint32_t l_name = ld32u(A.data, ro + 8) & 0xFF;
            ncig = ld32u(A.data, ro + 12) & 0xFFFF;
            ls = ld32u(A.data, ro + 16);
            co = ro + 32 + l_name;
            so = co + 4ull * ncig;
            qo = so + (ls + 1) / 2;
            if (ncig == 0 || ls > (1u << 30) || qo + ls > A.data_bytes) { act = false; bad = 1; }
            const int32_t tw = A.tweak[r];
            if (act && tw >= 0) {
                const int64_t tc = A.tw_col[tw] - P0;
                tcol = (int32_t)max(min(tc, (int64_t)INT32_MAX), (int64_t)INT32_MIN);
                oq = A.tw_q[tw];
                if (oq + ls > A.orig_bytes) { act = false; bad = 1; }
            }
            if (act) {
                const uint32_t cg = ld32u(A.data, co);
                op = cg & 15;
                len = cg >> 4;
            }
        }
        for (int32_t c = smin; c < emax; c++) {
            const bool cov = act && c >= s && c < e;
            uint32_t cd = 0, q = 0;
            if (cov) {
                for (;;) {                        // the op covering column c (skipping I / S / H / P)
                    if (eats_ref(op)) {
                        if (c < x + (int32_t)len) break;
                        x += (int32_t)len;
                    }
                    if (eats_query(op)) y += len;
                    if (++ci >= ncig) { bad = 1; break; }
                    const uint32_t cg = ld32u(A.data, co + 4ull * ci);
                    op = cg & 15;
                    len = cg >> 4;
                }
                if (op == 2 || op == 3) {         // D / N: the next query base's quality
                    cd = op == 2 ? 16u : 17u;
                    q = y < ls ? (c < tcol ? g(A.orig)[oq + y] : g(A.data)[qo + y]) : 0u;
                } else {
                    const uint32_t qp = y + (uint32_t)(c - x);
                    if (qp < ls) {
                        const uint32_t bb = g(A.data)[so + (qp >> 1)];
                        cd = (qp & 1) ? (bb & 15u) : (bb >> 4);
                        q = g(A.data)[qo + qp];
                    } else {
                        cd = 15u;
                    }
                }
            }
            const uint64_t m = __ballot(cov);
            if (m == 0) continue;
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint64_t base = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(cur >> 32), c) << 32) |
                                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cur, c);
            const uint64_t lim = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(cend >> 32), c) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cend, c);
            if (cov) {
                const uint64_t i = base + rank;
                if (i < lim) {
                    A.code[i] = (uint8_t)cd;
                    A.qual[i] = (uint8_t)q;
                } else {
                    bad = 1;
                }
            }
            if (lane == c) cur += (uint64_t)__popcll(m);
        }
    }
    if (lane < W && cur != cend) bad = 1;         // every column's entries written exactly
    if (__ballot(bad) && lane == 0) atomicOr(A.err, 2u);
}

// One position's entries across the history (LiveVariantCaller.memory, per position): the batches that may cover it
// (the host's bucket list), their column bounds, then the entries packed in accumulate order.
__global__ __launch_bounds__(256) void k_pos_bounds(const Hist *__restrict__ H, const int32_t *__restrict__ items, int32_t n,
                                                    int64_t pos, uint64_t *__restrict__ rng) {
    const int32_t i = (int32_t)(blockIdx.x * 256 + threadIdx.x);
    if (i >= n) return;
    const Hist h = H[items[i]];
    const int64_t col = pos - h.pos_begin;
    uint64_t lo = 0, hi = 0;
    if (col >= 0 && col < h.n_cols) { lo = g(h.off)[col]; hi = g(h.off)[col + 1]; }
    rng[2 * i] = lo;
    rng[2 * i + 1] = hi;
}
__global__ __launch_bounds__(256) void k_pos_copy(const Hist *__restrict__ H, const int32_t *__restrict__ items, int32_t n,
                                                  const uint64_t *__restrict__ rng, const uint64_t *__restrict__ dst,
                                                  uint8_t *__restrict__ oc, uint8_t *__restrict__ oq) {
    const int32_t i = (int32_t)(blockIdx.x * 4 + (threadIdx.x >> 6));      // one wave per batch
    if (i >= n) return;
    const Hist h = H[items[i]];
    const uint64_t lo = rng[2 * i], hi = rng[2 * i + 1], d = dst[i];
    for (uint64_t e = lo + (threadIdx.x & 63u); e < hi; e += 64) {
        oc[d + (e - lo)] = g(h.code)[e];
        oq[d + (e - lo)] = g(h.qual)[e];
    }
}
hipError_t launch_pos_bounds(const Hist *H, const int32_t *items, int32_t n, int64_t pos, uint64_t *rng, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    k_pos_bounds<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(H, items, n, pos, rng);
    return hipGetLastError();
}
hipError_t launch_pos_copy(const Hist *H, const int32_t *items, int32_t n, const uint64_t *rng, const uint64_t *dst,
                           uint8_t *oc, uint8_t *oq, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    k_pos_copy<<<(unsigned)((n + 3) / 4), 256, 0, st>>>(H, items, n, rng, dst, oc, oq);
    return hipGetLastError();
}

hipError_t launch_pileup_fill(const FillArgs &A, hipStream_t st) {
    if (A.n_tiles <= 0) return hipSuccess;
    k_tile_first<<<(unsigned)((A.n_reads + 1 + 255) / 256), 256, 0, st>>>(A);
    const uint32_t blocks = (((uint32_t)A.n_tiles + 3) / 4 + 7) & ~7u;
    k_pileup_fill<<<blocks, 256, 0, st>>>(A);
    return hipGetLastError();
}

}  // namespace spg
