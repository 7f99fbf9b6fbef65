// spg_fill.hip — device-side pileup of BAM records into the CSR batch (include/spings_gpu.h
// spg_accumulate_records, spg_bam_accumulate).
//
// Replaces the host CIGAR walk behind LiveVariantCaller.process_bam (variant_caller/live_variant_caller.py:
// 54-72, pysam's pileup columns :74-90): the host keeps what decides WHICH reads enter a column (stepper
// filter, htslib's depth cap, mate-overlap tweak, CSR offsets) and these kernels write WHAT they contribute: per
// covered column the read's BAM nibble and quality, or 16 / 17 for a CIGAR D / N with the quality of the next query
// base (0 past the read end), in htslib's per-column order (the column's reads in BAM order).  Bit-identical to
// spp_batch_fill of the same plan (tests/test_device_pileup_gpu.py).
//
// r05: the transposed fill (k_f2_*, below: one wave per 64-read chunk, lane = read) is the path; the tile kernels that
// follow remain for batches whose reads span too many columns for its per-chunk rows (F2_SPAN_LIMIT).
// Work items (tile kernels): a tile of 64 consecutive columns x a group of `fg` consecutive reads of the tile's read range (the
// reads starting at most max_span before the tile, up to its end: tile_first), so a 10,000x batch spreads over ~30k
// waves instead of one wave per tile.  A column's entries of a group are its covering reads of that group in BAM
// order, starting at the count of covering reads of the tile's earlier groups (k_fill_starts: one wave per tile,
// lanes = columns, a running count over the tile's reads, recorded at every group boundary).  k_fill: lanes =
// columns; per read (wave-uniform, its header and first CIGAR ops staged in LDS for 64 reads at a time) every lane
// finds the CIGAR op covering its column and loads its quality / packed base — consecutive lanes read consecutive
// bytes of the read, one coalesced load per array — four reads' loads in flight before their entries are used.
// Entries are staged per column in LDS and written out every 32 reads, one contiguous store per column (a column's
// entries of a group are contiguous in the CSR).  HBM-bound: records read once per tile they overlap, 2 B written
// per entry.
#include <hipcub/hipcub.hpp>

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

__device__ __forceinline__ bool eats_ref(uint32_t op) { return op == 0 || op == 2 || op == 3 || op == 7 || op == 8; }
__device__ __forceinline__ bool eats_query(uint32_t op) { return op == 0 || op == 1 || op == 4 || op == 7 || op == 8; }

constexpr int FILL_SB = 32;              // staged entries per column between write-outs (one per read: every 32 reads)
constexpr int FILL_ST = FILL_SB + 4;     // LDS row stride (9 dwords: the lanes' rows spread over the banks)
constexpr int FILL_OPS = 4;              // CIGAR ops staged per read (longer CIGARs read the rest from memory)

struct FillLay {                         // fill_scratch_bytes' layout
    uint32_t *tile_first, *item_off, *gstart;
    void *scan_tmp;
    size_t scan_bytes;
    int64_t items_cap;
};
__host__ __device__ __forceinline__ size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

// tile_first[k] = first read with rpos >= pos_begin + 64k (k >= 1), tile_first[0] = 0: thread r writes the
// boundaries between read r - 1's tile and its own (thread n_reads: those after the last read).
__global__ void k_tile_first(FillArgs A, uint32_t *tile_first) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > A.n_reads) return;
    auto tile_of = [&](uint64_t i) -> int64_t {
        if (i >= A.n_reads) return A.n_tiles;
        const int64_t d = (int64_t)A.rpos[i] - A.pos_begin;
        return d < 0 ? -1 : min(d >> 6, (int64_t)A.n_tiles);
    };
    const int64_t hi = tile_of(r), lo = r ? tile_of(r - 1) : -1;
    if (r == 0) tile_first[0] = 0;
    for (int64_t k = max(lo + 1, (int64_t)1); k <= hi; k++) tile_first[k] = (uint32_t)r;
}

// groups per tile (items), for the scan into item offsets; ng[n_tiles] = 0
__global__ void k_fill_ngroups(FillArgs A, const uint32_t *tile_first, uint32_t *ng, int32_t fg) {
    const int32_t t = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t > A.n_tiles) return;
    if (t == A.n_tiles) { ng[t] = 0; return; }
    const uint32_t r0 = tile_first[max(t - A.back, 0)], r1 = tile_first[t + 1];
    ng[t] = r1 > r0 ? (r1 - r0 + (uint32_t)fg - 1) / (uint32_t)fg : 0u;
}

// one wave per tile: covering reads counted in BAM order, 64 reads per step, as a difference array over the tile's
// columns in LDS (+1 at a read's first covered column, -1 after its last); at each group boundary the prefix sum over
// the columns is every column's count so far — that group's start (relative to the column's CSR offset); the total must
// be the column's entry count.  (r05: two readlanes per read per column made this pass 0.85 ms per 10,000x BAM.)
__global__ __launch_bounds__(256) void k_fill_starts(FillArgs A, const uint32_t *tile_first, const uint32_t *item_off,
                                                     uint32_t *gstart, int32_t fg) {
    __shared__ int32_t diff[4][65];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int32_t t = (int32_t)(blockIdx.x * 4 + w);
    if (t >= A.n_tiles) return;                                        // (wave-uniform; no barrier below)
    const int32_t c0 = t * 64, W = min(64, A.n_cols - c0);
    const int64_t P0 = A.pos_begin + c0;
    const uint32_t r0 = tile_first[max(t - A.back, 0)], r1 = tile_first[t + 1];
    uint32_t *gs = gstart + (size_t)item_off[t] * 64;
    int32_t *const d = diff[w];
    d[lane] = 0;
    if (lane == 0) d[64] = 0;
    // fg is a multiple of 64 (fill_group): group boundaries fall on chunk starts
    int64_t nps = 0, npe = 0;
    if (r0 + lane < r1) { nps = A.rpos[r0 + lane]; npe = A.rend[r0 + lane]; }
    uint32_t cnt = 0;
    for (uint32_t rb = r0, gi = 0, gl = 0; rb < r1; rb += 64) {
        const bool have = rb + lane < r1;
        const int64_t s = nps - P0, e = npe - P0;
        if (rb + 64 + lane < r1) { nps = A.rpos[rb + 64 + lane]; npe = A.rend[rb + 64 + lane]; }
        if (gl == 0) {                                                 // a group starts here: counts so far
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t v = (uint32_t)d[lane];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)v, o);
                if (lane >= o) v += y;
            }
            cnt = v;
            gs[(size_t)gi * 64 + lane] = cnt;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        gl += 64;
        if (gl == (uint32_t)fg) { gl = 0; gi++; }
        const int64_t cs = s < 0 ? 0 : s, ce = e > 64 ? 64 : e;
        if (have && cs < ce) {
            atomicAdd(&d[cs], 1);
            atomicAdd(&d[ce], -1);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t v = (uint32_t)d[lane];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)v, o);
        if (lane >= o) v += y;
    }
    cnt = v;
    if (lane < W && (uint64_t)cnt != A.off[c0 + lane + 1] - A.off[c0 + lane]) atomicOr(A.err, 2u);
}

// (tile, group) items: lanes = the tile's columns, the group's reads one at a time (wave-uniform)
__global__ __launch_bounds__(256) void k_fill(FillArgs A, const uint32_t *tile_first, const uint32_t *item_off,
                                              const uint32_t *gstart, int32_t fg) {
    __shared__ uint8_t stq[4][64 * FILL_ST], stc[4][64 * FILL_ST];
    __shared__ uint64_t s_co[4][64], s_qo[4][64], s_oq[4][64];
    __shared__ int32_t s_x[4][64], s_e[4][64], s_tc[4][64];
    __shared__ uint32_t s_ncig[4][64], s_ls[4][64], s_ops[4][64][FILL_OPS];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs; consecutive items (the same tile's groups and
    // the next tile's, which share reads) land on one XCD
    const uint32_t nb = gridDim.x, per = nb >> 3, b = blockIdx.x;
    const uint32_t blk = (b < (per << 3)) ? (b & 7) * per + (b >> 3) : b;
    const uint32_t item = blk * 4 + (uint32_t)w;
    const uint32_t total = item_off[A.n_tiles];
    if (item >= total) return;                                    // (wave-uniform; no barrier below)
    int32_t lo = 0, hi = A.n_tiles;                               // the tile: last t with item_off[t] <= item
    while (hi - lo > 1) {
        const int32_t mid = (lo + hi) >> 1;
        if (item_off[mid] <= item) lo = mid; else hi = mid;
    }
    const int32_t t = lo;
    const uint32_t grp = item - item_off[t];
    const int32_t c0 = t * 64, W = min(64, A.n_cols - c0);
    const int64_t P0 = A.pos_begin + c0;
    const uint32_t rt0 = tile_first[max(t - A.back, 0)], rt1 = tile_first[t + 1];
    const uint32_t ra = rt0 + grp * (uint32_t)fg, rz = min(rt1, ra + (uint32_t)fg);
    uint64_t cur = 0;
    if (lane < W) cur = A.off[c0 + lane] + gstart[(size_t)item * 64 + lane];
    uint8_t *Sq = stq[w], *Sc = stc[w];
    uint32_t k = 0, bad = 0;                                       // entries staged for this lane's column
    auto flush = [&]() {
        // column by column: lanes j < n write the column's staged bytes j (one contiguous store per array)
        for (int cc = 0; cc < 64; cc++) {
            const uint32_t n = __builtin_amdgcn_readlane(k, cc);
            if (n == 0) continue;
            const uint64_t at = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(cur >> 32), cc) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cur, cc);
            if ((uint32_t)lane < n) {
                A.code[at + lane] = Sc[cc * FILL_ST + lane];
                A.qual[at + lane] = Sq[cc * FILL_ST + lane];
            }
        }
        cur += k;
        k = 0;
    };
    for (uint32_t rb = ra; rb < rz; rb += 64) {
        const uint32_t n = min(64u, rz - rb);
        // the chunk's read headers, one read per lane, into LDS
        {
            const uint32_t r = rb + (uint32_t)lane;
            int32_t x = INT32_MAX, e = INT32_MIN, tc = INT32_MIN;
            uint32_t ncig = 0, ls = 0;
            uint64_t co = 0, qo = 0, oq = 0;
            if ((uint32_t)lane < n) {
                x = (int32_t)max(min((int64_t)A.rpos[r] - P0, (int64_t)INT32_MAX), (int64_t)INT32_MIN + 1);
                e = (int32_t)max(min((int64_t)A.rend[r] - P0, (int64_t)W), (int64_t)INT32_MIN + 1);
                if (max(x, 0) < e) {                                 // covers a column of the tile
                    const uint64_t ro = min(A.rec[r], A.data_bytes);  // (the host checked rec + 36 <= data_bytes)
                    const uint32_t l_name = ld32u(A.data, ro + 8) & 0xFF;
                    ncig = ld32u(A.data, ro + 12) & 0xFFFF;
                    ls = ld32u(A.data, ro + 16);
                    co = ro + 32 + l_name;
                    qo = co + 4ull * ncig + (ls + 1) / 2;
                    if (ncig == 0 || ls > (1u << 30) || qo + ls > A.data_bytes) { bad = 1; e = INT32_MIN; }
                    const int32_t tw = A.tweak[r];
                    if (e != INT32_MIN && tw >= 0) {
                        const int64_t tcl = A.tw_col[tw] - P0;
                        tc = (int32_t)max(min(tcl, (int64_t)INT32_MAX), (int64_t)INT32_MIN);
                        oq = A.tw_q[tw];
                        if (oq + ls > A.orig_bytes) { bad = 1; e = INT32_MIN; }
                    }
                    for (int o = 0; o < FILL_OPS; o++) s_ops[w][lane][o] = (uint32_t)o < ncig ? ld32u(A.data, co + 4ull * o) : 0u;
                } else {
                    e = INT32_MIN;
                }
            }
            s_x[w][lane] = x; s_e[w][lane] = e; s_tc[w][lane] = tc;
            s_ncig[w][lane] = ncig; s_ls[w][lane] = ls;
            s_co[w][lane] = co; s_qo[w][lane] = qo; s_oq[w][lane] = oq;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // four reads at a time: addresses and loads for all four, then their entries
        for (uint32_t i0 = 0; i0 < n; i0 += 4) {
            uint32_t cd[4], qv[4], sv[4];
            bool cov[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t i = i0 + (uint32_t)u;
                cov[u] = false;
                cd[u] = 0; qv[u] = 0; sv[u] = 0;
                if (i >= n) continue;
                const int32_t x0 = s_x[w][i], e = s_e[w][i];
                if (e == INT32_MIN) continue;                        // (wave-uniform)
                const int32_t col = lane;
                cov[u] = col >= max(x0, 0) && col < e;
                const uint32_t ncig = s_ncig[w][i], ls = s_ls[w][i];
                const uint64_t co = s_co[w][i], qo = s_qo[w][i];
                const uint64_t so = co + 4ull * ncig;
                // the op covering this lane's column: a wave-uniform walk over the ops until past the tile
                int32_t x = x0;
                uint32_t y = 0, op = 15, ox = 0, oy = 0;
                for (uint32_t o = 0; o < ncig && x < W; o++) {
                    const uint32_t c = o < (uint32_t)FILL_OPS ? s_ops[w][i][o] : ld32u(A.data, co + 4ull * o);
                    const uint32_t cop = c & 15u, len = c >> 4;
                    if (eats_ref(cop)) {
                        if (col >= x && col < x + (int32_t)len && op == 15) { op = cop; ox = (uint32_t)(col - x); oy = y; }
                        x += (int32_t)len;
                    }
                    if (eats_query(cop)) y += len;
                }
                if (cov[u] && op == 15) { bad = 1; cov[u] = false; }    // the CIGAR ends before the column
                if (!cov[u]) continue;
                if (op == 2 || op == 3) {                            // D / N: the next query base's quality
                    cd[u] = op == 2 ? 16u : 17u;
                    if (oy < ls) {
                        const int32_t tc = s_tc[w][i];
                        qv[u] = col < tc ? g(A.orig)[s_oq[w][i] + oy] : g(A.data)[qo + oy];
                    }
                    sv[u] = 0x100u;                                  // (code already final)
                } else {
                    const uint32_t qp = oy + ox;
                    if (qp < ls) {
                        qv[u] = g(A.data)[qo + qp];
                        sv[u] = g(A.data)[so + (qp >> 1)] | ((qp & 1) << 9);
                    } else {
                        cd[u] = 15u;
                        sv[u] = 0x100u;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (!cov[u]) continue;
                const uint32_t code = (sv[u] & 0x100u) ? cd[u] : ((sv[u] & 0x200u) ? (sv[u] & 15u) : ((sv[u] >> 4) & 15u));
                Sc[lane * FILL_ST + k] = (uint8_t)code;
                Sq[lane * FILL_ST + k] = (uint8_t)qv[u];
                k++;
            }
            if (__builtin_amdgcn_readfirstlane(__ballot(k > FILL_SB - 4) != 0)) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                flush();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        // (the next chunk's headers overwrite the LDS arrays: every lane is done with them)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    flush();
    // the group's entries end where the next group's start (the tile's last group: the column's end)
    if (lane < W) {
        const uint64_t want = grp + 1 < item_off[t + 1] - item_off[t] ? A.off[c0 + lane] + gstart[(size_t)(item + 1) * 64 + lane]
                                                                    : A.off[c0 + lane + 1];
        if (cur != want) bad = 1;
    }
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

// spg_copy_table_device: the finalize's call table and its status in one device-side copy, so a consumer (the
// multi-device gather) needs no host round trip per context: a 16-B header {n_cand, status, n_detail, records copied}
// and min(n_cand, cap) 56-B records (7 u64 each).  status: 1 replay depth mismatch, 2 run error word, 4 fill error word,
// 8 more candidates than the copy holds, 16 more details than the context's buffer (its finalize must run again).
__global__ __launch_bounds__(256) void k_table_copy(const Counters *__restrict__ ctr, const uint32_t *__restrict__ kerr,
                                                    const uint32_t *__restrict__ ferr, const uint64_t *__restrict__ cand,
                                                    int64_t cap, int64_t detail_cap, uint32_t *__restrict__ dst) {
    const Counters h = *ctr;
    const uint64_t n = std::min<uint64_t>(h.n_cand, (uint64_t)cap);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const uint32_t st = (h.err ? 1u : 0u) | (*kerr ? 2u : 0u) | (*ferr ? 4u : 0u) | ((int64_t)h.n_cand > cap ? 8u : 0u) |
                            ((int64_t)h.n_detail > detail_cap ? 16u : 0u);
        dst[0] = h.n_cand;
        dst[1] = st;
        dst[2] = h.n_detail;
        dst[3] = (uint32_t)n;
    }
    uint64_t *out = reinterpret_cast<uint64_t *>(dst + 4);
    const uint64_t words = n * (sizeof(spg_candidate) / 8);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 256) out[i] = cand[i];
}
hipError_t launch_table_copy(const Counters *ctr, const uint32_t *kerr, const uint32_t *ferr, const void *cand, int64_t cap,
                             int64_t detail_cap, void *dst, hipStream_t st) {
    const int64_t words = cap * (int64_t)(sizeof(spg_candidate) / 8);
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((words + 255) / 256, 64));
    k_table_copy<<<blocks, 256, 0, st>>>(ctr, kerr, ferr, static_cast<const uint64_t *>(cand), cap, detail_cap,
                                         static_cast<uint32_t *>(dst));
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------------------------
// The transposed fill (r05): one wave per chunk of 64 consecutive reads (BAM order), lane = read.  Each lane walks its
// own CIGAR once, column by column over the chunk's column span, with its quality and packed-base bytes in 8-byte
// windows (the next window loaded one ahead); at every column the covering lanes' entries are ranked by a ballot and
// written as one contiguous run at off[c] + base(chunk, c) + rank, base(chunk, c) being the covering reads of column c
// in earlier chunks.  That base comes from three small passes: each chunk's column span (k_f2_span), its per-column
// counts (k_f2_count, into rows of a scanned span layout), and per column a running sum along the chunks that cover it
// (k_f2_base, which also checks the total against the CSR offsets).  The tile kernels above made one wave-iteration of
// all 64 lanes per (read, tile) pair with a wave-uniform CIGAR walk each (1.98 ms per 10,000x BAM, r05q).
// ------------------------------------------------------------------------------------------------------------------
struct F2Lay {                           // fill_scratch_bytes' layout of the transposed fill
    int32_t *cbeg, *cend;                // per chunk: first / past-last column of its span (clamped to the batch)
    uint32_t *span, *row;                // per chunk: span length; its row's offset (exclusive scan of span)
    uint8_t *cnt;                        // [sum of spans]: covering reads per (chunk, column) (<= 64)
    uint32_t *base;                      // [sum of spans]: covering reads of the column in earlier chunks
    void *scan_tmp;
    size_t scan_bytes;
    uint64_t span_cap;
    int64_t n_chunks;
};
constexpr uint64_t F2_SPAN_LIMIT = (uint64_t)1 << 28;    // beyond this bound on the spans' sum the tile kernels run

__host__ __device__ __forceinline__ uint64_t f2_span_cap(int64_t n_cols, int64_t n_reads, int32_t back) {
    // a chunk's span <= its reads' start spread + max_span; the spreads of consecutive chunks do not overlap
    const int64_t n_chunks = (n_reads + 63) / 64;
    return (uint64_t)n_cols + (uint64_t)n_chunks * ((uint64_t)back * 64 + 2) + 64;
}

F2Lay f2_layout(void *base, int64_t n_cols, int64_t n_reads, int32_t back) {
    F2Lay L{};
    L.n_chunks = (n_reads + 63) / 64;
    L.span_cap = f2_span_cap(n_cols, n_reads, back);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, L.scan_bytes, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                           (int)(L.n_chunks + 1));
    uint8_t *p = static_cast<uint8_t *>(base);
    size_t o = 0;
    const size_t nc = (size_t)L.n_chunks + 1;
    L.cbeg = reinterpret_cast<int32_t *>(p + o); o += al256(4 * nc);
    L.cend = reinterpret_cast<int32_t *>(p + o); o += al256(4 * nc);
    L.span = reinterpret_cast<uint32_t *>(p + o); o += al256(4 * nc);
    L.row = reinterpret_cast<uint32_t *>(p + o); o += al256(4 * nc);
    L.scan_tmp = p + o; o += al256(L.scan_bytes);
    L.base = reinterpret_cast<uint32_t *>(p + o); o += al256(4 * L.span_cap);
    L.cnt = p + o; o += al256(L.span_cap);
    return L;
}
size_t f2_bytes(int64_t n_cols, int64_t n_reads, int32_t back) {
    F2Lay L = f2_layout(nullptr, n_cols, n_reads, back);
    return reinterpret_cast<size_t>(L.cnt) + al256(L.span_cap) + 256;
}

__device__ __forceinline__ int32_t f2_rel(int64_t x, int64_t P0) {
    const int64_t d = x - P0;
    return (int32_t)max(min(d, (int64_t)INT32_MAX - 1), (int64_t)INT32_MIN + 1);
}

// per chunk: the span [cbeg, cend) of the columns its reads cover, clamped to the batch
__global__ __launch_bounds__(256) void k_f2_span(FillArgs A, F2Lay L) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q > L.n_chunks) return;
    if (q == L.n_chunks) {                                        // (the scan's last element)
        if (lane == 0) L.span[q] = 0;
        return;
    }
    const uint64_t r = (uint64_t)q * 64 + (uint64_t)lane;
    const bool valid = r < A.n_reads;
    const int32_t rp = valid ? f2_rel(A.rpos[r], A.pos_begin) : INT32_MAX;
    const int32_t re = valid ? f2_rel(A.rend[r], A.pos_begin) : INT32_MIN;
    const int32_t cb = min(max(__builtin_amdgcn_readfirstlane(rp), 0), A.n_cols);
    int32_t ce = min(re, A.n_cols);
    for (int o = 32; o; o >>= 1) ce = max(ce, __shfl_xor(ce, o));
    ce = max(ce, cb);
    if (lane == 0) {
        L.cbeg[q] = cb;
        L.cend[q] = ce;
        L.span[q] = (uint32_t)(ce - cb);
    }
}

// the number of the wave's 64 ascending values s that are <= v (lane-parallel binary search over the lanes)
__device__ __forceinline__ int32_t f2_count_le(int32_t s, int32_t v) {
    int32_t k = 0;
#pragma unroll
    for (int st = 32; st; st >>= 1) {
        const int32_t t = __shfl(s, k + st - 1, 64);
        k += t <= v ? st : 0;
    }
    const int32_t t = __shfl(s, k, 64);                           // (k <= 63 here: the last element)
    return k + (k == 63 && t <= v ? 1 : 0);
}

// per chunk: covering reads per column of its span, into its row.  Column c is covered by the chunk's reads with
// start <= c minus those with end <= c; the starts are ascending (coordinate order), the ends are sorted across the
// lanes (bitonic network), and both counts are binary searches over the lanes (one readlane pass over all 64 reads per
// column before: 93 us per 10,000x BAM, r06k)
__global__ __launch_bounds__(256) void k_f2_count(FillArgs A, F2Lay L) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= L.n_chunks) return;
    const uint64_t r = (uint64_t)q * 64 + (uint64_t)lane;
    const bool valid = r < A.n_reads;
    const int32_t rp = valid ? f2_rel(A.rpos[r], A.pos_begin) : INT32_MAX;
    int32_t re = valid ? f2_rel(A.rend[r], A.pos_begin) : INT32_MAX;   // (INT32_MAX: never "ended")
    const int32_t cb = L.cbeg[q], ce = L.cend[q];
    if ((uint64_t)L.row[q] + (uint64_t)(ce - cb) > L.span_cap) return;   // (k_f2_base reports it)
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j; j >>= 1) {
            const int32_t o = __shfl_xor(re, j, 64);
            const bool up = (lane & k) == 0, lo = (lane & j) == 0;
            re = (up == lo) ? min(re, o) : max(re, o);
        }
    }
    uint8_t *const row = L.cnt + L.row[q];
    for (int32_t c0 = cb; c0 < ce; c0 += 64) {
        const int32_t c = c0 + lane;
        const int32_t n = f2_count_le(rp, c) - f2_count_le(re, c);
        if (c < ce) row[c - cb] = (uint8_t)n;
    }
}

// per 64-column tile (lane = column): running sums along the chunks that cover each column; the total must be the
// column's entry count
__global__ __launch_bounds__(64) void k_f2_base(FillArgs A, F2Lay L) {      // (one wave per tile: ~470 per BAM)
    const int lane = threadIdx.x;
    const int64_t t = blockIdx.x;
    const int32_t c_lo = (int32_t)(t * 64);
    if (c_lo >= A.n_cols) return;
    const int32_t c_hi = min(c_lo + 63, A.n_cols - 1), c = c_lo + lane;
    uint32_t run = 0;
    if (L.n_chunks == 0) {
        if (c < A.n_cols && A.off[c + 1] != A.off[c]) atomicOr(A.err, 2u);
        return;
    }
    // chunks that may cover the tile: from the one before the first whose span starts past c_lo - max_span, to the last
    // whose span starts at or before c_hi (cbeg is non-decreasing: the reads are in coordinate order)
    auto first_gt = [&](int64_t v) {                              // first chunk with cbeg > v: a 64-ary search, one
        int64_t lo = 0, hi = L.n_chunks;                          // probe per lane (~3 round trips, not ~15)
        while (lo < hi) {
            const int64_t st = (hi - lo + 63) / 64, at = lo + (int64_t)(lane + 1) * st - 1;
            const bool le = at < hi && (int64_t)L.cbeg[at] <= v;  // (a prefix of the lanes)
            const int64_t k = __popcll(__ballot(le));
            const int64_t nlo = lo + k * st;
            hi = min(hi, nlo + st - 1);                            // (cbeg[nlo + st - 1] > v when that probe ran)
            lo = nlo;
        }
        return lo;
    };
    const int64_t qa = max(first_gt((int64_t)c_lo - (int64_t)A.back * 64 - 1) - 1, (int64_t)0);
    const int64_t qb = first_gt(c_hi);                            // (exclusive)
    if ((uint64_t)L.row[L.n_chunks] > L.span_cap) {              // (a plan whose max_span understates a read's span)
        if (lane == 0) atomicOr(A.err, 2u);
        return;
    }
    // F2_BB chunks per round: their descriptors (scalar loads), then their count bytes, all in flight together
    constexpr int F2_BB = 16;
    for (int64_t q0 = qa; q0 < qb; q0 += F2_BB) {
        int32_t cbs[F2_BB], ces[F2_BB];
        uint32_t ros[F2_BB], v[F2_BB];
#pragma unroll
        for (int u = 0; u < F2_BB; u++) {
            const bool in = q0 + u < qb;
            cbs[u] = in ? L.cbeg[q0 + u] : INT32_MAX;
            ces[u] = in ? L.cend[q0 + u] : INT32_MIN;
            ros[u] = in ? L.row[q0 + u] : 0u;
        }
#pragma unroll
        for (int u = 0; u < F2_BB; u++)
            v[u] = (c >= cbs[u] && c < ces[u]) ? (uint32_t)L.cnt[ros[u] + (uint32_t)(c - cbs[u])] : 0u;
#pragma unroll
        for (int u = 0; u < F2_BB; u++) {
            if (c >= cbs[u] && c < ces[u]) L.base[ros[u] + (uint32_t)(c - cbs[u])] = run;
            run += v[u];
        }
    }
    if (c < A.n_cols && (uint64_t)run != A.off[c + 1] - A.off[c]) atomicOr(A.err, 2u);
}

// the chunk's entries: lanes = reads, columns of the span in order.  One wave per workgroup: each lane first copies
// its record's CIGAR, packed bases and qualities (one contiguous range of the record) — and, for a read the mate-overlap
// tweak touches, its original qualities — into the wave's LDS as 16-B blocks, so the column loop reads bytes from LDS and
// issues no vector-memory load: its only vector-memory instructions are the entry stores, which nothing waits for.  (The
// r05 form kept 8-byte windows in registers with the next one in flight; a refill in any lane waited for every memory
// operation the wave had issued, its entry stores included — about one L2 round trip per column, 1.12 ms per
// 10,000x BAM.)  A chunk whose ranges exceed F2_LDS takes those windows.
//
// F2_NW waves share a chunk (one workgroup): they copy its bytes into the one LDS image together (a quarter of the 16-B
// blocks each, all of a wave's loads in flight at once) and then each fills a contiguous quarter of the chunk's column
// span, every lane catching its CIGAR cursor up to the wave's first column on the way.  With one wave per chunk the
// 20 KiB image allowed 2 waves per SIMD, and a wave's ~46 us (the copy's round trips, then ~150 dependent column steps)
// was mostly waiting: r06j PMC, 31,152 waves, VALU 6.8k per wave — 0.77 ms per 10,000x BAM.
constexpr uint32_t F2_LDS = 20480;
constexpr int F2_NW = 4;

__global__ __launch_bounds__(64 * F2_NW) void k_f2_fill(FillArgs A, F2Lay L) {
    __shared__ __align__(16) uint8_t sb[F2_LDS];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs; consecutive chunks (which write adjacent runs of
    // the same columns) land on one XCD
    const uint32_t nb = gridDim.x, per = nb >> 3, b = blockIdx.x;
    const int64_t q = (b < (per << 3)) ? (b & 7) * per + (b >> 3) : b;
    if (q >= L.n_chunks) return;                                  // (workgroup-uniform)
    const uint64_t r = (uint64_t)q * 64 + (uint64_t)lane;
    bool valid = r < A.n_reads;
    const int32_t cb = L.cbeg[q], ce = L.cend[q];
    const uint32_t ro = L.row[q];
    if ((uint64_t)L.row[L.n_chunks] > L.span_cap) return;        // (k_f2_base reports it)
    int32_t rp = INT32_MAX, re = INT32_MIN, tc = INT32_MIN;
    uint32_t ncig = 0, ls = 0, bad = 0;
    uint64_t co = 0, qo = 0, so = 0, oq = 0;
    if (valid) {
        rp = f2_rel(A.rpos[r], A.pos_begin);
        re = f2_rel(A.rend[r], A.pos_begin);
        const uint64_t rr = min(A.rec[r], A.data_bytes);          // (the host checked rec + 36 <= data_bytes)
        const uint32_t l_name = ld32u(A.data, rr + 8) & 0xFF;
        ncig = ld32u(A.data, rr + 12) & 0xFFFF;
        ls = ld32u(A.data, rr + 16);
        co = rr + 32 + l_name;
        so = co + 4ull * ncig;
        qo = so + (ls + 1) / 2;
        if (ncig == 0 || ls > (1u << 30) || qo + ls > A.data_bytes) { bad = 1; valid = false; }
        const int32_t tw = A.tweak[r];
        if (valid && tw >= 0) {
            tc = f2_rel(A.tw_col[tw], A.pos_begin);
            oq = A.tw_q[tw];
            if (oq + ls > A.orig_bytes) { bad = 1; valid = false; }
        }
    }
    if (!valid) { rp = INT32_MAX; re = INT32_MIN; tc = INT32_MIN; }
    // the lane's LDS ranges: [ga, ga + gn) of the record (CIGAR .. qualities), [oa, oa + on) of the original qualities
    const uint64_t ga = co & ~15ull, oa = oq & ~15ull;
    const uint32_t gn = valid ? (uint32_t)(((qo + ls + 15) & ~15ull) - ga) : 0u;
    const uint32_t on = (valid && tc != INT32_MIN) ? (uint32_t)(((oq + ls + 15) & ~15ull) - oa) : 0u;
    uint32_t lb = gn + on;                                        // exclusive prefix over the lanes: the lane's base
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(lb, o);
        if (lane >= o) lb += t;
    }
    // lane l's region starts 4 l bytes past the prefix: lanes reading the same query offset of equal-length reads then hit
    // different banks (unskewed, regions of 16 k bytes put every lane's byte on one bank: 3.3 conflict cycles per LDS
    // cycle, r05zg)
    const uint32_t need = __builtin_amdgcn_readlane(lb, 63) + 256u;
    lb += 4u * (uint32_t)lane - (gn + on);
    const bool lds = need <= F2_LDS;                              // (uniform)
    if (lds) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) const u32x4 gu128;
        // 16-B blocks, four loads in flight; the wave takes every F2_NW-th group of four blocks; a block past the array's
        // readable end is copied byte by byte
        auto copy = [&](uint32_t dst, const uint8_t *src, uint64_t a, uint32_t n, uint64_t lim) {
            for (uint32_t i = 64u * (uint32_t)wv; i < n; i += 64u * F2_NW) {
                uint4 v[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint64_t x = a + i + 16u * k;
                    if (i + 16u * k < n && x + 16 <= lim) {
                        const u32x4 t = *(gu128 *)(const void *)(src + x);
                        v[k] = make_uint4(t.x, t.y, t.z, t.w);
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint64_t x = a + i + 16u * k;
                    if (i + 16u * k >= n) continue;
                    if (x + 16 > lim) {
                        uint32_t w[4] = {0, 0, 0, 0};
                        for (uint32_t j = 0; j < 16 && x + j < lim; j++) w[j >> 2] |= (uint32_t)src[x + j] << (8 * (j & 3));
                        v[k] = make_uint4(w[0], w[1], w[2], w[3]);
                    }
                    uint32_t *d = reinterpret_cast<uint32_t *>(sb + dst + i + 16u * k);   // (4-B aligned)
                    d[0] = v[k].x; d[1] = v[k].y; d[2] = v[k].z; d[3] = v[k].w;
                }
            }
        };
        if (gn) copy(lb, A.data, ga, gn, A.data_bytes + 64);
        if (on) copy(lb + gn, A.orig, oa, on, A.orig_bytes);
    }
    __syncthreads();
    // LDS offsets of the lane's CIGAR, packed bases, qualities and original qualities
    const uint32_t lc = lb + (uint32_t)(co - ga), lsq = lb + (uint32_t)(so - ga), lq = lb + (uint32_t)(qo - ga);
    const uint32_t lo_ = lb + gn + (uint32_t)(oq - oa);
    // The column loop, instantiated twice so that the LDS form holds no vector-memory load the waits would count
    auto body = [&](auto lds_tag) __attribute__((always_inline)) {
    constexpr bool LDS = decltype(lds_tag)::value;
    // 8-byte windows of the qualities and the packed bases, the next one in flight (chunks beyond F2_LDS)
    typedef __attribute__((address_space(1))) const uint64_t gu64;
    auto ld8 = [&](uint64_t a) -> uint64_t { return *(gu64 *)(const void *)(A.data + a); };
    uint64_t qwa = qo & ~7ull, swa = so & ~7ull, qwin = 0, qnx = 0, swin = 0, snx = 0;
    if (valid && !LDS) {
        qwin = ld8(qwa); qnx = ld8(qwa + 8);
        swin = ld8(swa); snx = ld8(swa + 8);
    }
    const uint32_t qo32 = (uint32_t)qo, so32 = (uint32_t)so;
    // the quality byte at query offset p (windows only move forward)
    auto qual_at = [&](uint32_t p) -> uint32_t {
        if constexpr (LDS) return sb[lq + p];
        uint32_t d = qo32 + p - (uint32_t)qwa;
        if (d >= 8) {
            if (d < 16) { qwin = qnx; qwa += 8; } else { qwa = (qo + p) & ~7ull; qwin = ld8(qwa); }
            qnx = ld8(qwa + 8);
            d = qo32 + p - (uint32_t)qwa;
        }
        return (uint32_t)(qwin >> (8 * d)) & 0xFFu;
    };
    // the packed-base byte holding query offset p
    auto seq_at = [&](uint32_t p) -> uint32_t {
        if constexpr (LDS) return sb[lsq + (p >> 1)];
        uint32_t d = so32 + (p >> 1) - (uint32_t)swa;
        if (d >= 8) {
            if (d < 16) { swin = snx; swa += 8; } else { swa = (so + (p >> 1)) & ~7ull; swin = ld8(swa); }
            snx = ld8(swa + 8);
            d = so32 + (p >> 1) - (uint32_t)swa;
        }
        return (uint32_t)(swin >> (8 * d)) & 0xFFu;
    };
    auto orig_at = [&](uint32_t y) -> uint32_t {
        if constexpr (LDS) return sb[lo_ + y];
        return ((const __attribute__((address_space(1))) uint8_t *)(const void *)A.orig)[oq + y];
    };
    auto cig = [&](uint32_t o) -> uint32_t {                      // CIGAR op o (o < ncig)
        if constexpr (!LDS) return ld32u(A.data, co + 4ull * o);
        const uint32_t a = lc + 4 * o;
        return (uint32_t)sb[a] | ((uint32_t)sb[a + 1] << 8) | ((uint32_t)sb[a + 2] << 16) | ((uint32_t)sb[a + 3] << 24);
    };
    // the CIGAR cursor, kept on a reference-consuming op (M / D / N / = / X; 15: past the CIGAR's end): op k of length
    // len covering ref columns [x, xe), query offset y at its start; the next op preloaded
    uint32_t o = 0, k = 15, len = 0, nxt = 0;
    int32_t x = rp, xe = rp;
    uint32_t y = 0;
    auto step = [&]() {                                           // to the next op
        if (eats_ref(k)) x += (int32_t)len;
        if (eats_query(k)) y += len;
        o++;
        if (o < ncig) {
            k = nxt & 15u;
            len = nxt >> 4;
            nxt = o + 1 < ncig ? cig(o + 1) : 0u;
        } else {
            k = 15;
            len = 0;
        }
    };
    if (valid) {
        nxt = cig(0);
        k = nxt & 15u;
        len = nxt >> 4;
        nxt = ncig > 1 ? cig(1) : 0u;
        while (k != 15 && !eats_ref(k)) step();
        xe = x + (int32_t)len;
    }
    // the wave's part of the span (the cursor catches up at its first covered column)
    const int32_t part = (ce - cb + F2_NW - 1) / F2_NW, pb = cb + wv * part, pe = min(ce, pb + part);
    for (int32_t c0 = pb; c0 < pe; c0 += 64) {
        // the next 64 columns' first entry of this chunk (CSR offset + the earlier chunks' entries), one per lane
        uint64_t at0 = 0;
        if (c0 + lane < pe) at0 = A.off[c0 + lane] + L.base[ro + (uint32_t)(c0 + lane - cb)];
        const uint32_t at_lo = (uint32_t)at0, at_hi = (uint32_t)(at0 >> 32);
        const int32_t nc = min(64, pe - c0);
        for (int32_t j = 0; j < nc; j++) {
            const int32_t c = c0 + j;
            bool cov = c >= rp && c < re;
            uint32_t cd = 0, qv = 0;
            if constexpr (LDS) {
                // branch-free but for the (rare, wave-uniform) CIGAR step: both bytes read from LDS in every lane
                const bool adv = cov && c >= xe;
                if (__ballot(adv)) {
                    if (adv) {
                        do step(); while (k != 15 && (!eats_ref(k) || c >= x + (int32_t)len));
                        xe = x + (int32_t)len;
                    }
                }
                bad |= (uint32_t)(cov && k == 15);                // the CIGAR ends before the column
                cov = cov && k != 15;
                const bool dn = (k | 1u) == 3u;                   // D / N: the next query base's quality
                const uint32_t qp = y + (dn ? 0u : (uint32_t)(c - x));
                const bool rd = cov && qp < ls;
                const uint32_t qa = rd ? ((dn && c < tc) ? lo_ + y : lq + qp) : 0u;
                const uint32_t q0 = sb[qa];
                const uint32_t sbyte = sb[rd ? lsq + (qp >> 1) : 0u];
                const uint32_t nib = (qp & 1) ? (sbyte & 15u) : (sbyte >> 4);
                cd = dn ? 14u + k : (rd ? nib : 15u);          // (15: a CIGAR longer than the sequence)
                qv = rd ? q0 : 0u;
            } else if (cov) {
                if (c >= xe) {                                    // (rare) the next reference-consuming op
                    do step(); while (k != 15 && (!eats_ref(k) || c >= x + (int32_t)len));
                    xe = x + (int32_t)len;
                }
                if (k == 15) {                                    // the CIGAR ends before the column
                    bad = 1;
                    cov = false;
                } else if (k == 2 || k == 3) {                    // D / N: the next query base's quality
                    cd = 14u + k;
                    if (y < ls) qv = c < tc ? orig_at(y) : qual_at(y);
                } else {
                    const uint32_t qp = y + (uint32_t)(c - x);
                    if (qp < ls) {
                        qv = qual_at(qp);
                        const uint32_t sbyte = seq_at(qp);
                        cd = (qp & 1) ? (sbyte & 15u) : (sbyte >> 4);
                    } else {
                        cd = 15u;                                 // (a CIGAR longer than the sequence)
                    }
                }
            }
            const uint64_t m = __ballot(cov);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint64_t at = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)at_hi, j) << 32 |
                                 (uint32_t)__builtin_amdgcn_readlane((int)at_lo, j)) + (uint64_t)rank;
            if (cov) {
                A.code[at] = (uint8_t)cd;
                A.qual[at] = (uint8_t)qv;
            }
        }
    }
    };
    if (lds) body(std::true_type{});
    else body(std::false_type{});
    if (__ballot(bad) && lane == 0) atomicOr(A.err, 2u);
}

namespace {
int32_t fill_group(int64_t n_tiles, int64_t n_reads, int32_t back, int64_t *items_cap) {
    // items <= n_tiles + n_reads (back + 1) / fg (a read is in back + 1 tiles' read ranges); group starts take 256 B per
    // item: fg grows so that they stay within ~1 GiB
    int32_t fg = 256;
    for (;;) {
        const int64_t cap = n_tiles + 1 + (n_reads * (int64_t)(back + 1) + fg - 1) / fg;
        if (cap <= ((int64_t)4 << 20) || fg >= (1 << 20)) { *items_cap = cap; return fg; }
        fg *= 2;
    }
}
FillLay fill_layout(void *base, int64_t n_tiles, int64_t n_reads, int32_t back, int32_t *fg) {
    FillLay L{};
    *fg = fill_group(n_tiles, n_reads, back, &L.items_cap);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, L.scan_bytes, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                           (int)(n_tiles + 1));
    uint8_t *p = static_cast<uint8_t *>(base);
    size_t o = 0;
    L.tile_first = reinterpret_cast<uint32_t *>(p + o);
    o += al256(4 * (size_t)(n_tiles + 1));
    L.item_off = reinterpret_cast<uint32_t *>(p + o);
    o += al256(4 * (size_t)(n_tiles + 1));
    L.scan_tmp = p + o;
    o += al256(L.scan_bytes);
    L.gstart = reinterpret_cast<uint32_t *>(p + o);
    o += al256(256 * (size_t)L.items_cap);
    return L;
}
}  // namespace

size_t fill_scratch_bytes(int64_t n_cols, int64_t n_reads, int64_t max_span) {
    const int64_t n_tiles = (n_cols + 63) / 64;
    const int32_t back = (int32_t)((max_span + 63) / 64);
    if (f2_span_cap(n_cols, n_reads, back) <= F2_SPAN_LIMIT) return f2_bytes(n_cols, n_reads, back);
    int32_t fg = 0;
    FillLay L = fill_layout(nullptr, n_tiles, n_reads, back, &fg);
    return al256(4 * (size_t)(n_tiles + 1)) * 2 + al256(L.scan_bytes) + al256(256 * (size_t)L.items_cap) + 256;
}

hipError_t launch_pileup_fill(const FillArgs &A, hipStream_t st) {
    if (A.n_tiles <= 0) return hipSuccess;
    if (f2_span_cap(A.n_cols, A.n_reads, A.back) <= F2_SPAN_LIMIT) {
        // the transposed fill: spans, scan into row offsets, counts, bases, entries
        F2Lay L = f2_layout(A.scratch, A.n_cols, A.n_reads, A.back);
        if (L.n_chunks == 0) {                   // no reads: every column must be empty (k_f2_base checks)
            k_f2_base<<<(unsigned)A.n_tiles, 64, 0, st>>>(A, L);
            return hipGetLastError();
        }
        k_f2_span<<<(unsigned)((L.n_chunks + 1 + 3) / 4), 256, 0, st>>>(A, L);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        e = hipcub::DeviceScan::ExclusiveSum(L.scan_tmp, L.scan_bytes, L.span, L.row, (int)(L.n_chunks + 1), st);
        if (e != hipSuccess) return e;
        const unsigned cb = (unsigned)((L.n_chunks + 3) / 4);
        k_f2_count<<<cb, 256, 0, st>>>(A, L);
        k_f2_base<<<(unsigned)A.n_tiles, 64, 0, st>>>(A, L);
        k_f2_fill<<<(unsigned)((L.n_chunks + 7) & ~7ll), 64 * F2_NW, 0, st>>>(A, L);
        return hipGetLastError();
    }
    int32_t fg = 0;
    FillLay L = fill_layout(A.scratch, A.n_tiles, A.n_reads, A.back, &fg);
    k_tile_first<<<(unsigned)((A.n_reads + 1 + 255) / 256), 256, 0, st>>>(A, L.tile_first);
    k_fill_ngroups<<<(unsigned)((A.n_tiles + 1 + 255) / 256), 256, 0, st>>>(A, L.tile_first, L.gstart, fg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // (group counts written into the start of gstart, scanned into item_off, before gstart is filled)
    e = hipcub::DeviceScan::ExclusiveSum(L.scan_tmp, L.scan_bytes, L.gstart, L.item_off, (int)(A.n_tiles + 1), st);
    if (e != hipSuccess) return e;
    k_fill_starts<<<(unsigned)((A.n_tiles + 3) / 4), 256, 0, st>>>(A, L.tile_first, L.item_off, L.gstart, fg);
    const unsigned blocks = (unsigned)(((L.items_cap + 3) / 4 + 7) & ~7ll);
    k_fill<<<blocks, 256, 0, st>>>(A, L.tile_first, L.item_off, L.gstart, fg);
    return hipGetLastError();
}

}  // namespace spg
