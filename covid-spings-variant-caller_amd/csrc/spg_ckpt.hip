// spg_ckpt.hip — the checkpoint's view of one history batch, computed in HBM (include/spings_gpu.h
// spg_history_copy_compact; LiveVariantCaller.create_checkpoint, variant_caller/live_variant_caller.py:40-45).
//
// The reference pickles `memory`, whose quality lists hold only the entries that passed the base-quality filter
// (:89, :96-103), plus every position's first visit (:77-85).  The checkpoint keeps the same information per
// batch: the entries with q >= min_bq, and for a column whose every entry fails the filter its first entry (a
// marker: the engine filters it again on resume, but it records the visit).  Two passes over the batch, one wave
// per column (grid-stride): count what each column keeps, scan the counts into the compact CSR's offsets, then
// write the kept bytes there in column order — only they cross PCIe.  Not on a measured path: one pass over a
// BAM's entries per checkpoint (HBM-bound, ~2 B read + <= 2 B written per entry).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "spg_device.h"

namespace spg {

namespace {

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

// 16 bytes at a 16-B aligned address below the batch end (the batch buffers carry >= 16 B of padding past it)
__device__ __forceinline__ u32x4v ld16(const uint8_t *p) {
    return *(const __attribute__((address_space(1))) u32x4v *)(const void *)p;
}

// bit j (0..15) of the result: byte j of the 16-B block at a (a + j in [b, e)) has q >= min_bq
__device__ __forceinline__ uint32_t keep_mask(const u32x4v &q, uint64_t a, uint64_t b, uint64_t e, uint32_t min_bq) {
    uint32_t m = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const uint32_t w = d == 0 ? q.x : d == 1 ? q.y : d == 2 ? q.z : q.w;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t i = a + (uint64_t)(4 * d + k);
            const uint32_t v = (w >> (8 * k)) & 0xFFu;
            m |= (uint32_t)(i >= b && i < e && v >= min_bq) << (4 * d + k);
        }
    }
    return m;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// exclusive prefix over the wave's lanes
__device__ __forceinline__ uint32_t wave_excl(uint32_t v, int lane) {
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x - v;
}

}  // namespace

// kept[c] = entries of column c with q >= min_bq, or 1 (the marker) when the column has entries and none passes
__global__ __launch_bounds__(256) void k_ck_count(Hist h, uint32_t min_bq, uint64_t *__restrict__ kept) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < h.n_cols; c += nw) {
        const uint64_t b = h.off[c], e = h.off[c + 1];
        uint32_t n = 0;
        for (uint64_t a = (b & ~15ull) + 16ull * (uint64_t)lane; a < e; a += 1024)
            n += __popc(keep_mask(ld16(h.qual + a), a, b, e, min_bq));
        n = wave_sum(n);
        if (lane == 0) kept[c] = n ? (uint64_t)n : (uint64_t)(e > b);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) kept[h.n_cols] = 0;
}

// the kept entries of every column at its compact offset, in the column's order
__global__ __launch_bounds__(256) void k_ck_scatter(Hist h, uint32_t min_bq, const uint64_t *__restrict__ noff,
                                                    uint8_t *__restrict__ oc, uint8_t *__restrict__ oq) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < h.n_cols; c += nw) {
        const uint64_t b = h.off[c], e = h.off[c + 1];
        uint64_t d = noff[c];
        uint32_t run = 0;
        for (uint64_t a0 = b & ~15ull; a0 < e; a0 += 1024) {
            const uint64_t a = a0 + 16ull * (uint64_t)lane;
            uint32_t m = 0;
            u32x4v q = {0, 0, 0, 0}, cd = {0, 0, 0, 0};
            if (a < e) {
                q = ld16(h.qual + a);
                cd = ld16(h.code + a);
                m = keep_mask(q, a, b, e, min_bq);
            }
            const uint32_t n = __popc(m);
            uint64_t o = d + run + wave_excl(n, lane);
#pragma unroll
            for (int j = 0; j < 16; j++) {
                if ((m >> j) & 1u) {
                    const uint32_t wq = j < 4 ? q.x : j < 8 ? q.y : j < 12 ? q.z : q.w;
                    const uint32_t wc = j < 4 ? cd.x : j < 8 ? cd.y : j < 12 ? cd.z : cd.w;
                    oq[o] = (uint8_t)(wq >> (8 * (j & 3)));
                    oc[o] = (uint8_t)(wc >> (8 * (j & 3)));
                    o++;
                }
            }
            run += wave_sum(n);
        }
        if (run == 0 && e > b && lane == 0) {      // every entry fails the filter: the first one marks the visit
            oc[d] = h.code[b];
            oq[d] = h.qual[b];
        }
    }
}

// One byte per compacted entry for the packed checkpoint: base A/C/G/T (BAM nibbles 1/2/4/8) as 2 bits over a 6-bit
// quality 0..62; any other code or a quality >= 63 is an exception — its byte is 63 and (index, code, quality) goes to
// the exception list (slot from an atomic counter: the index makes the order irrelevant).  In place over the codes.
__global__ __launch_bounds__(256) void k_ck_pack(uint8_t *__restrict__ oc, const uint8_t *__restrict__ oq, uint64_t m,
                                                 uint64_t base, uint64_t *__restrict__ xi, uint8_t *__restrict__ xc,
                                                 uint8_t *__restrict__ xq, uint32_t *__restrict__ xn, uint32_t xcap) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
        const uint32_t c = oc[i], q = oq[i];
        const uint32_t b2 = c == 1 ? 0u : c == 2 ? 1u : c == 4 ? 2u : c == 8 ? 3u : 4u;
        const bool esc = b2 == 4u || q >= 63u;
        if (esc) {
            const uint32_t k = atomicAdd(xn, 1u);
            if (k < xcap) {
                xi[k] = base + i;
                xc[k] = (uint8_t)c;
                xq[k] = (uint8_t)q;
            }
        }
        oc[i] = esc ? (uint8_t)63 : (uint8_t)(b2 << 6 | q);
    }
}

hipError_t launch_ck_pack(uint8_t *oc, const uint8_t *oq, uint64_t m, uint64_t base, uint64_t *xi, uint8_t *xc, uint8_t *xq,
                          uint32_t *xn, uint32_t xcap, hipStream_t st) {
    if (m == 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<uint64_t>((m + 255) / 256, 16384);
    k_ck_pack<<<blocks, 256, 0, st>>>(oc, oq, m, base, xi, xc, xq, xn, xcap);
    return hipGetLastError();
}

hipError_t launch_ck_compact(const Hist &h, uint32_t min_bq, uint64_t *kept, uint64_t *noff, void *scan_tmp,
                             size_t *scan_bytes, uint8_t *oc, uint8_t *oq, hipStream_t st) {
    // scan_tmp null: only the scan's scratch size
    if (!scan_tmp) return hipcub::DeviceScan::ExclusiveSum(nullptr, *scan_bytes, kept, noff, h.n_cols + 1, st);
    if (h.n_cols <= 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<int64_t>((h.n_cols + 3) / 4, 8192);
    k_ck_count<<<blocks, 256, 0, st>>>(h, min_bq, kept);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, *scan_bytes, kept, noff, h.n_cols + 1, st);
    if (e != hipSuccess) return e;
    k_ck_scatter<<<blocks, 256, 0, st>>>(h, min_bq, noff, oc, oq);
    return hipGetLastError();
}

}  // namespace spg
