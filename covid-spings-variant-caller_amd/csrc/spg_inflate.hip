// spg_inflate.hip — BGZF members inflated on the GPU (process_bam's BAM read,
// live_variant_caller.py:54-72, whose host BGZF inflate bounds the end-to-end stream at the GPU box's 16-CPU share).
//
// A BGZF file is a sequence of independent raw-DEFLATE members (RFC 1951) of at most 64 KiB of output each: one
// lane per member decodes its blocks (stored, fixed Huffman, dynamic Huffman) into the member's output range.  All
// per-member state lives in registers and the lane's LDS slice: the Huffman tables (10-bit primary table for the
// literal/length code, 8-bit for distances, a canonical walk for the rare longer codes), the code lengths; length and
// distance bases are computed, not looked up.  The compressed stream is read as aligned 16-byte chunks one ahead of
// use.  A member's status word is 0 when it inflated to exactly its ISIZE bytes; anything else (a corrupt stream) is
// reported and the caller inflates that member on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spings_gpu.h"

#ifndef SPG_INFLATE_MATCH_HOOK
#define SPG_INFLATE_MATCH_HOOK(dist, len)     // (tools/inflate_stats.cpp: match statistics of a host run)
#endif
#ifndef SPG_INFLATE_SLOW_HOOK
#define SPG_INFLATE_SLOW_HOOK(pb)             // (tools/inflate_stats.cpp: codes longer than the primary table)
#endif

namespace spg {

// Per-member decode tables: one slice of SLICE bytes (LDS on the device: mpw slices per block; a host array in the
// check).  u16 entries of a primary table are symbol | code length << 9 (0: a longer code or no code); the counts and
// length-sorted symbols serve the canonical walk for codes longer than the primary table.  The code-length code's
// tables borrow the literal table's primary area and the distance code's count / symbol areas (it is done with
// before those codes are built); its 19 code lengths are read into the lengths area.
constexpr int IB_LIT = 10, IB_DIST = 8, IB_CL = 7;      // primary table bits
constexpr int SL_LITP = 0, SL_DISTP = 2048, SL_LCNT = 2560, SL_DCNT = 2592, SL_LSYM = 2624, SL_DSYM = 3200,
              SL_LENS = 3264, SLICE = 3584;
static_assert(SL_LENS + 320 == SLICE && SL_DSYM + 64 == SL_LENS && SL_LSYM + 576 == SL_DSYM, "slice layout");

// The bit stream: a 64-bit buffer refilled 32 bits at a time from a 128-bit reservoir r, which is refilled from the
// next 16-byte aligned chunk q, loaded one chunk ahead (its address never depends on the bits consumed, so its
// latency can hide behind the symbols of the chunk before).  Past the member's trailer the last chunk is read again
// (the overrun check then fails the member); the buffers are padded so an aligned chunk never leaves them.
struct IBits {
    const uint8_t *qa;          // the chunk held in q (r's chunk ends here)
    const uint8_t *end;         // member payload + its 8-byte trailer
    uint64_t buf, r0, r1, q0, q1;
    int n, rn;                  // bits in buf; bits in r (a multiple of 8)
    __host__ __device__ __forceinline__ void chunk(const uint8_t *a, uint64_t &x0, uint64_t &x1) const {
        // past the trailer the last chunk is read again (garbage the overrun check fails; never outside the buffer):
        // an unconditional load, so no branch merge forces a wait for it before its use one chunk later
        const uint8_t *lastc = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(end - 1) & ~(uintptr_t)15);
        a = a < end ? a : lastc;
#if defined(__HIP_DEVICE_COMPILE__)
        // a global (not flat) load: a flat load also counts on the LDS wait counter
        typedef __attribute__((address_space(1))) const uint64_t gu64;
        gu64 *c = (gu64 *)a;
#else
        const uint64_t *c = reinterpret_cast<const uint64_t *>(a);
#endif
        x0 = c[0];
        x1 = c[1];
    }
    // start at byte address s (any alignment)
    __host__ __device__ __forceinline__ void start(const uint8_t *s) {
        const uint8_t *a = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(s) & ~(uintptr_t)15);
        const int skip = (int)(s - a) * 8;
        chunk(a, r0, r1);
        if (skip >= 64) {
            r0 = r1 >> (skip - 64);
            r1 = 0;
        } else if (skip) {
            r0 = (r0 >> skip) | (r1 << (64 - skip));
            r1 >>= skip;
        }
        rn = 128 - skip;
        qa = a + 16;
        chunk(qa, q0, q1);
        buf = 0;
        n = 0;
    }
    __host__ __device__ __forceinline__ void fill() {
        if (n > 32) return;
        uint32_t v;
        if (rn >= 32) {
            v = (uint32_t)r0;
            r0 = (r0 >> 32) | (r1 << 32);
            r1 >>= 32;
            rn -= 32;
        } else {                                 // rn in {0, 8, 16, 24}: r's last bits, then q's first
            const int k = 32 - rn;               // 8..32 bits from q
            v = (uint32_t)((rn ? (r0 & ((1ull << rn) - 1)) : 0) | (q0 << rn));
            r0 = (q0 >> k) | (q1 << (64 - k));
            r1 = q1 >> k;
            rn = 128 - k;
            qa += 16;
            chunk(qa, q0, q1);
        }
        buf |= (uint64_t)v << n;
        n += 32;
    }
    __host__ __device__ __forceinline__ uint32_t peek(int k) const { return (uint32_t)(buf & ((1ull << k) - 1)); }
    __host__ __device__ __forceinline__ void drop(int k) { buf >>= k; n -= k; }
    __host__ __device__ __forceinline__ uint32_t get(int k) {   // k <= 24
        fill();
        const uint32_t v = peek(k);
        drop(k);
        return v;
    }
    // the byte address of the next unread whole byte (after a drop to a byte boundary)
    __host__ __device__ __forceinline__ const uint8_t *byte_pos() const { return qa - (rn >> 3) - (n >> 3); }
};

// canonical Huffman tables from code lengths (RFC 1951 3.2.2); false: over-subscribed, or an incomplete code with
// more than one symbol (a single-code distance alphabet may be incomplete)
__host__ __device__ __forceinline__ bool build(uint16_t *prim, uint16_t *count, uint16_t *sym, const uint8_t *len, int n,
                                               int pb) {
    for (int i = 0; i < 16; i++) count[i] = 0;
    for (int s = 0; s < n; s++) count[len[s]]++;
    uint64_t *p8 = reinterpret_cast<uint64_t *>(prim);
    for (int i = 0; i < (1 << pb) / 4; i++) p8[i] = 0;
    if (count[0] == n) return true;                      // no codes: every lookup fails (only a distance code may)
    int left = 1;
    for (int l = 1; l < 16; l++) {
        left = (left << 1) - count[l];
        if (left < 0) return false;
    }
    if (left > 0 && n - count[0] > 1) return false;
    uint16_t offs[16];
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = (uint16_t)(offs[l] + count[l]);
    for (int s = 0; s < n; s++)
        if (len[s]) sym[offs[len[s]]++] = (uint16_t)s;
    // each code of length <= pb fills 2^(pb - len) entries at its bit-reversed code
    uint32_t code = 0;
    int k = 0;
    for (int l = 1; l <= pb; l++) {
        for (int c = 0; c < count[l]; c++, k++, code++) {
            const uint32_t rev = __builtin_bitreverse32(code) >> (32 - l);
            const uint16_t e = (uint16_t)(sym[k] | (l << 9));
            for (uint32_t x = rev; x < (1u << pb); x += 1u << l) prim[x] = e;
        }
        code <<= 1;
    }
    return true;
}

// one symbol; -1 on an invalid code.  Needs >= 15 bits in the buffer (the caller's fill()).
__host__ __device__ __forceinline__ int decode(IBits &B, const uint16_t *prim, const uint16_t *count, const uint16_t *sym,
                                               int pb) {
    const uint16_t e = prim[B.peek(pb)];
    if (e >> 9) {
        B.drop(e >> 9);
        return e & 0x1FF;
    }
    // longer than the primary table (or invalid): the canonical walk, one bit at a time (first bit read = MSB)
    SPG_INFLATE_SLOW_HOOK(pb);
    int code = 0, first = 0, index = 0;
    for (int l = 1; l <= 15; l++) {
        code |= (int)B.peek(1);
        B.drop(1);
        const int c = count[l];
        if (code - first < c) return sym[index + (code - first)];
        index += c;
        first = (first + c) << 1;
        code <<= 1;
    }
    return -1;
}

// length / distance bases and extra bits (RFC 1951 3.2.5), computed: c = length code - 257, d = distance code
__host__ __device__ __forceinline__ uint32_t len_ext(int c) { return c < 8 || c == 28 ? 0u : (uint32_t)(c >> 2) - 1u; }
__host__ __device__ __forceinline__ uint32_t len_base(int c) {
    return c < 8 ? (uint32_t)c + 3u : c == 28 ? 258u : ((4u | (uint32_t)(c & 3)) << len_ext(c)) + 3u;
}
__host__ __device__ __forceinline__ uint32_t dist_ext(int d) { return d < 4 ? 0u : (uint32_t)(d >> 1) - 1u; }
__host__ __device__ __forceinline__ uint32_t dist_base(int d) {
    return d < 4 ? (uint32_t)d + 1u : ((2u | (uint32_t)(d & 1)) << dist_ext(d)) + 1u;
}

// one member into out + M.uoff; status (see k_inflate).  slice: SLICE bytes, 8-byte aligned.
__host__ __device__ __forceinline__ uint32_t inflate_member(const uint8_t *comp, const spg_bgzf_member &M, uint8_t *out,
                                                            uint8_t *slice) {
    uint16_t *const litp = reinterpret_cast<uint16_t *>(slice + SL_LITP);
    uint16_t *const distp = reinterpret_cast<uint16_t *>(slice + SL_DISTP);
    uint16_t *const lcnt = reinterpret_cast<uint16_t *>(slice + SL_LCNT);
    uint16_t *const dcnt = reinterpret_cast<uint16_t *>(slice + SL_DCNT);
    uint16_t *const lsym = reinterpret_cast<uint16_t *>(slice + SL_LSYM);
    uint16_t *const dsym = reinterpret_cast<uint16_t *>(slice + SL_DSYM);
    uint8_t *const lens = slice + SL_LENS;
    uint8_t *o = out + M.uoff;
    const uint32_t ulen = M.ulen;
    const uint8_t *const cend = comp + M.coff + M.clen;
    IBits B;
    B.end = cend + 8;
    B.start(comp + M.coff);
    uint32_t w = 0;                                      // bytes written
#if defined(SPG_INFLATE_TOKEN_STORES)
    uint32_t ntk = 0;
#endif
    uint32_t st = 0;
    int bfinal = 0;
    bool fixed_built = false;
    do {
        bfinal = (int)B.get(1);
        const uint32_t type = B.get(2);
        if (type == 0) {                                 // stored: to a byte boundary, LEN, NLEN, LEN bytes
            B.drop(B.n & 7);
            const uint32_t ln = B.get(16), nl = B.get(16);
            if ((ln ^ 0xFFFFu) != nl) { st = 2; break; }
            const uint8_t *src = B.byte_pos();
            if (w + ln > ulen) { st = 7; break; }
            if (src + ln > cend) { st = 8; break; }
#if defined(__HIP_DEVICE_COMPILE__)
            typedef __attribute__((address_space(1))) const uint8_t gu8;
            for (uint32_t i = 0; i < ln; i++) o[w + i] = ((gu8 *)src)[i];
#else
            for (uint32_t i = 0; i < ln; i++) o[w + i] = src[i];
#endif
            w += ln;
            B.start(src + ln);
            continue;
        }
        if (type == 1) {                                 // the fixed codes (RFC 1951 3.2.6), built once per member
            if (!fixed_built) {
                for (int s = 0; s < 288; s++) lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
                build(litp, lcnt, lsym, lens, 288, IB_LIT);
                for (int s = 0; s < 32; s++) lens[s] = 5;   // (30 and 31 complete the code; decoding them fails)
                build(distp, dcnt, dsym, lens, 32, IB_DIST);
                fixed_built = true;
            }
        } else if (type == 2) {
            fixed_built = false;
            const int hlit = (int)B.get(5) + 257, hdist = (int)B.get(5) + 1, hclen = (int)B.get(4) + 4;
            uint8_t *const cl = lens;                    // 19 code-length code lengths, in RFC order
            for (int i = 0; i < 19; i++) cl[i] = 0;
            for (int i = 0; i < hclen; i++) {
                const int ord = i < 3 ? 16 + i : i == 3 ? 0 : (i & 1) ? 7 - (i - 5) / 2 : 8 + (i - 4) / 2;   // RFC 1951 3.2.7
                cl[ord] = (uint8_t)B.get(3);
            }
            if (!build(litp, dcnt, dsym, cl, 19, IB_CL)) { st = 3; break; }
            int k = 0;
            while (k < hlit + hdist) {
                B.fill();
                const int s = decode(B, litp, dcnt, dsym, IB_CL);
                if (s < 0) { st = 3; break; }
                if (s < 16) { lens[k++] = (uint8_t)s; continue; }
                int rep;
                uint8_t v = 0;
                if (s == 16) {
                    if (k == 0) { st = 3; break; }
                    v = lens[k - 1];
                    rep = 3 + (int)B.get(2);
                } else if (s == 17) {
                    rep = 3 + (int)B.get(3);
                } else {
                    rep = 11 + (int)B.get(7);
                }
                if (k + rep > hlit + hdist) { st = 3; break; }
                while (rep--) lens[k++] = v;
            }
            if (st) break;
            if (lens[256] == 0) { st = 3; break; }       // no end-of-block code
            if (!build(distp, dcnt, dsym, lens + hlit, hdist, IB_DIST) || !build(litp, lcnt, lsym, lens, hlit, IB_LIT)) {
                st = 4;
                break;
            }
        } else {
            st = 1;
            break;
        }
        while (true) {                                   // the block's codes
            B.fill();
            const int s = decode(B, litp, lcnt, lsym, IB_LIT);
            if (s < 256) {
                if (s < 0) { st = 5; break; }
                if (w >= ulen) { st = 7; break; }
#if defined(SPG_INFLATE_DECODE_ONLY)                     // (A/B: decode cost alone — no output written)
                w++;
#elif defined(SPG_INFLATE_TOKEN_STORES)                  // (A/B: one byte store per symbol, no match reads)
                o[ntk++] = (uint8_t)s;
                w++;
#else
                o[w++] = (uint8_t)s;
#endif
                continue;
            }
            if (s == 256) break;
            if (s > 285) { st = 5; break; }
            B.fill();                                    // <= 5 extra bits, then <= 15 of the distance code
            const uint32_t len = len_base(s - 257) + B.peek((int)len_ext(s - 257));
            B.drop((int)len_ext(s - 257));
            const int ds = decode(B, distp, dcnt, dsym, IB_DIST);
            if (ds < 0 || ds > 29) { st = 5; break; }
            const uint32_t dist = dist_base(ds) + B.get((int)dist_ext(ds));
            SPG_INFLATE_MATCH_HOOK(dist, len);
            if (dist > w) { st = 6; break; }
            if (w + len > ulen) { st = 7; break; }
#if defined(SPG_INFLATE_DECODE_ONLY)
            w += len;
            continue;
#elif defined(SPG_INFLATE_TOKEN_STORES)
            o[ntk++] = (uint8_t)(len ^ dist);
            w += len;
            continue;
#endif
            uint8_t *dst = o + w;
            const uint8_t *from = dst - dist;
            if (dist >= 16 && w + len + 15 <= ulen) {
                // 16-byte chunks, up to four loads in flight before their stores (a round's sources all precede its
                // first store: round = min(64, dist rounded down to 16)); the last chunk may write up to 15 bytes past
                // the match, inside the member, which later symbols overwrite
                const uint32_t R = dist >= 64 ? 64u : dist & ~15u;
                for (uint32_t i = 0; i < len; i += R) {
                    uint64_t v[8];
#pragma unroll
                    for (uint32_t k = 0; k < 4; k++)
                        if (16 * k < R && i + 16 * k < len) {
                            __builtin_memcpy(&v[2 * k], from + i + 16 * k, 8);
                            __builtin_memcpy(&v[2 * k + 1], from + i + 16 * k + 8, 8);
                        }
#pragma unroll
                    for (uint32_t k = 0; k < 4; k++)
                        if (16 * k < R && i + 16 * k < len) {
                            __builtin_memcpy(dst + i + 16 * k, &v[2 * k], 8);
                            __builtin_memcpy(dst + i + 16 * k + 8, &v[2 * k + 1], 8);
                        }
                }
            } else if (dist >= 4) {                             // four bytes at a time: each source dword was written before
                uint32_t i = 0;
                for (; i + 4 <= len; i += 4) {
                    uint32_t v;
                    __builtin_memcpy(&v, from + i, 4);
                    __builtin_memcpy(dst + i, &v, 4);
                }
                for (; i < len; i++) dst[i] = from[i];
            } else {                                     // a 1-3 byte pattern repeated (runs of one quality value)
                const uint32_t b0 = from[0], b1 = dist == 1 ? b0 : from[1], b2 = dist == 3 ? from[2] : b0,
                               b3 = dist == 2 ? b1 : b0;
                const uint32_t pat = b0 | b1 << 8 | b2 << 16 | b3 << 24;
                if (dist == 3) {
                    for (uint32_t i = 0; i < len; i++) dst[i] = from[i % 3];
                } else {
                    uint32_t i = 0;
                    for (; i + 4 <= len; i += 4) __builtin_memcpy(dst + i, &pat, 4);
                    for (; i < len; i++) dst[i] = (uint8_t)(pat >> (8 * (i & 3)));
                }
            }
            w += len;
        }
        if (st) break;
        if (B.byte_pos() > cend) { st = 8; break; }
    } while (!bfinal);
    if (!st && w != ulen) st = 9;
    return st;
}

// status: 0 ok; 1 bad block type; 2 bad stored length; 3 bad code lengths; 4 bad table; 5 bad symbol;
// 6 distance too far back; 7 output overrun; 8 input overrun; 9 wrong size; 10 CRC32 mismatch (k_crc32).
// mpw members per block, one per lane (lanes >= mpw idle), each with its SLICE of the block's LDS.  Latency-bound
// (a member's symbols are a dependent chain): 96 VGPRs for 5 waves per SIMD, 3 members per block (r04ze: 19.3 ms on
// the 10,000x BAM vs 20.0 at 4 waves, 23.4 at 4 members per block)
#if defined(SPG_INFLATE_MPW_AB)
constexpr int INFLATE_MPW = SPG_INFLATE_MPW_AB;          // (A/B builds only)
#else
constexpr int INFLATE_MPW = 3;
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void k_inflate(const uint8_t *__restrict__ comp, const spg_bgzf_member *__restrict__ mem,
                                                int64_t n, uint8_t *__restrict__ out, uint32_t *__restrict__ status, int mpw) {
    extern __shared__ __align__(16) uint8_t inf_lds[];
    if ((int)threadIdx.x >= mpw) return;
    const int64_t m = (int64_t)blockIdx.x * mpw + threadIdx.x;
    if (m >= n) return;
    status[m] = inflate_member(comp, mem[m], out, inf_lds + (size_t)threadIdx.x * SLICE);
}

// ------------------------------------------------------------------------------------------------------------------
// k_inflate_w: one member per wave, its DEFLATE window in LDS.  The lane-per-member kernel above reads every match
// source back from global memory — the member's own output of up to 32 KiB before, which ~8k concurrent members do not
// keep in L2 — and a match's load waits for every store the lane issued before it (one in-order counter for loads and
// stores): ~1 us per symbol.  Here the decoder state is wave-uniform (all 64 lanes decode the same symbol stream, no
// divergence) and everything the symbol loop touches is in LDS: the 32 KiB window ring (match sources; a match's bytes
// copied by up to 64 lanes at once), the Huffman tables, and a 2 KiB ring of the compressed stream that the wave
// refills 1 KiB at a time from a global load issued 1 KiB of input earlier.  The window is written out to global memory
// 1 KiB at a time by the whole wave.  ~38.5 KiB of LDS per wave: 4 members per CU.
// ------------------------------------------------------------------------------------------------------------------
constexpr int W_WIN = 32768, W_IN = 2048, W_HALF = 1024;

struct WaveIn {                   // the compressed stream in LDS: bytes [lo, lo + W_IN) of the member (relative to base)
    const uint8_t *g;             // comp + base (global)
    uint64_t gmax;                // readable bytes from g
    uint8_t *ring;                // LDS [W_IN]
    uint32_t lo;
    uint32_t nxt[4];              // the next half [lo + W_IN, lo + W_IN + W_HALF), 16 B per lane, loaded ahead
    int lane;
    __device__ __forceinline__ void load_next() {
        const uint64_t at = (uint64_t)lo + W_IN + 16u * (uint32_t)lane;
        typedef __attribute__((address_space(1))) const uint32_t gu32;
        for (int k = 0; k < 4; k++)
            nxt[k] = at + 4u * k + 4 <= gmax ? ((gu32 *)(const void *)(g + at))[k] : 0u;
    }
    // bytes [lo, lo + W_IN) into the ring (synchronous), the half after them in flight
    __device__ __forceinline__ void reset(uint32_t at) {
        lo = at & ~(uint32_t)(W_HALF - 1);
        typedef __attribute__((address_space(1))) const uint32_t gu32;
        for (int h = 0; h < W_IN; h += W_HALF) {
            const uint64_t a = (uint64_t)lo + h + 16u * (uint32_t)lane;
            uint32_t v[4];
            for (int k = 0; k < 4; k++) v[k] = a + 4u * k + 4 <= gmax ? ((gu32 *)(const void *)(g + a))[k] : 0u;
            uint32_t *d = reinterpret_cast<uint32_t *>(ring + ((lo + h + 16u * (uint32_t)lane) & (W_IN - 1)));
            d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3];
        }
        load_next();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    // the chunk at a (16-B aligned, relative) is about to be read: slide the ring when a enters its second half
    __device__ __forceinline__ void need(uint32_t a) {
        while (a >= lo + W_HALF) {
            uint32_t *d = reinterpret_cast<uint32_t *>(ring + ((lo + 16u * (uint32_t)lane) & (W_IN - 1)));
            d[0] = nxt[0]; d[1] = nxt[1]; d[2] = nxt[2]; d[3] = nxt[3];
            lo += W_HALF;
            load_next();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __syncthreads();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
    }
};

struct WBits {                    // IBits over the LDS ring (offsets relative to the member's aligned base)
    WaveIn *in;
    uint32_t qa, end;
    uint64_t buf, r0, r1, q0, q1;
    int n, rn;
    __device__ __forceinline__ void chunk(uint32_t a, uint64_t &x0, uint64_t &x1) {
        const uint32_t lastc = (end - 1) & ~15u;
        a = a < end ? a : lastc;
        in->need(a);
        const uint64_t *c = reinterpret_cast<const uint64_t *>(in->ring + (a & (W_IN - 1)));
        x0 = c[0];
        x1 = c[1];
    }
    __device__ __forceinline__ void start(uint32_t s) {
        const uint32_t a = s & ~15u;
        const int skip = (int)(s - a) * 8;
        chunk(a, r0, r1);
        if (skip >= 64) { r0 = r1 >> (skip - 64); r1 = 0; }
        else if (skip) { r0 = (r0 >> skip) | (r1 << (64 - skip)); r1 >>= skip; }
        rn = 128 - skip;
        qa = a + 16;
        chunk(qa, q0, q1);
        buf = 0;
        n = 0;
    }
    __device__ __forceinline__ void fill() {
        if (n > 32) return;
        uint32_t v;
        if (rn >= 32) {
            v = (uint32_t)r0;
            r0 = (r0 >> 32) | (r1 << 32);
            r1 >>= 32;
            rn -= 32;
        } else {
            const int k = 32 - rn;
            v = (uint32_t)((rn ? (r0 & ((1ull << rn) - 1)) : 0) | (q0 << rn));
            r0 = (q0 >> k) | (q1 << (64 - k));
            r1 = q1 >> k;
            rn = 128 - k;
            qa += 16;
            chunk(qa, q0, q1);
        }
        buf |= (uint64_t)v << n;
        n += 32;
    }
    __device__ __forceinline__ uint32_t peek(int k) const { return (uint32_t)(buf & ((1ull << k) - 1)); }
    __device__ __forceinline__ void drop(int k) { buf >>= k; n -= k; }
    __device__ __forceinline__ uint32_t get(int k) { fill(); const uint32_t v = peek(k); drop(k); return v; }
    __device__ __forceinline__ uint32_t byte_pos() const { return qa - (uint32_t)(rn >> 3) - (uint32_t)(n >> 3); }
};

__device__ __forceinline__ int decode_w(WBits &B, const uint16_t *prim, const uint16_t *count, const uint16_t *sym, int pb) {
    const uint16_t e = prim[B.peek(pb)];
    if (e >> 9) {
        B.drop(e >> 9);
        return e & 0x1FF;
    }
    int code = 0, first = 0, index = 0;
    for (int l = 1; l <= 15; l++) {
        code |= (int)B.peek(1);
        B.drop(1);
        const int c = count[l];
        if (code - first < c) return sym[index + (code - first)];
        index += c;
        first = (first + c) << 1;
        code <<= 1;
    }
    return -1;
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__global__ __launch_bounds__(64) void k_inflate_w(const uint8_t *__restrict__ comp, uint64_t comp_bytes,
                                                  const spg_bgzf_member *__restrict__ mem, int64_t n,
                                                  uint8_t *__restrict__ out, uint32_t *__restrict__ status) {
    __shared__ __align__(16) uint8_t win[W_WIN];
    __shared__ __align__(16) uint8_t inr[W_IN];
    __shared__ __align__(16) uint8_t slice[SLICE];
    const int64_t m = blockIdx.x;
    if (m >= n) return;
    const int lane = threadIdx.x;
    uint16_t *const litp = reinterpret_cast<uint16_t *>(slice + SL_LITP);
    uint16_t *const distp = reinterpret_cast<uint16_t *>(slice + SL_DISTP);
    uint16_t *const lcnt = reinterpret_cast<uint16_t *>(slice + SL_LCNT);
    uint16_t *const dcnt = reinterpret_cast<uint16_t *>(slice + SL_DCNT);
    uint16_t *const lsym = reinterpret_cast<uint16_t *>(slice + SL_LSYM);
    uint16_t *const dsym = reinterpret_cast<uint16_t *>(slice + SL_DSYM);
    uint8_t *const lens = slice + SL_LENS;
    const spg_bgzf_member M = mem[m];
    const uint64_t base = M.coff & ~15ull;
    WaveIn in;
    in.g = comp + base;
    in.gmax = comp_bytes + 64 > base ? comp_bytes + 64 - base : 0;   // (the buffer is padded by 64 bytes)
    in.ring = inr;
    in.lane = lane;
    in.reset(0);
    WBits B;
    B.in = &in;
    const uint32_t cend = (uint32_t)(M.coff + M.clen - base);
    B.end = cend + 8;
    B.start((uint32_t)(M.coff - base));
    uint8_t *const o = out + M.uoff;
    const uint32_t ulen = M.ulen;
    uint32_t w = 0, flushed = 0, st = 0;
    int bfinal = 0;
    bool fixed_built = false;
    // the window's completed 1 KiB blocks to global memory (coalesced bytes: lane j writes bytes j, j + 64, ...)
    auto flush_to = [&](uint32_t upto) {
        while (flushed + W_HALF <= upto || (upto == ulen && flushed < upto)) {
            const uint32_t e = min(flushed + (uint32_t)W_HALF, upto);
            for (uint32_t p = flushed + (uint32_t)lane; p < e; p += 64) o[p] = win[p & (W_WIN - 1)];
            flushed = e;
        }
    };
    do {
        bfinal = (int)B.get(1);
        const uint32_t type = B.get(2);
        if (type == 0) {                                 // stored: LEN bytes straight from the compressed stream
            B.drop(B.n & 7);
            const uint32_t ln = B.get(16), nl = B.get(16);
            if ((ln ^ 0xFFFFu) != nl) { st = 2; break; }
            const uint32_t src = B.byte_pos();
            if (w + ln > ulen) { st = 7; break; }
            if (src + ln > cend) { st = 8; break; }
            typedef __attribute__((address_space(1))) const uint8_t gu8;
            for (uint32_t i0 = 0; i0 < ln; i0 += W_HALF) {     // (1 KiB at a time: the window ring holds 32 KiB)
                const uint32_t e = min(ln, i0 + (uint32_t)W_HALF);
                wave_lds_sync();
                for (uint32_t i = i0 + (uint32_t)lane; i < e; i += 64) win[(w + i - i0) & (W_WIN - 1)] = ((gu8 *)(in.g))[src + i];
                w += e - i0;
                wave_lds_sync();
                flush_to(w);
            }
            in.reset(src + ln);
            B.start(src + ln);
            continue;
        }
        if (type == 1) {
            if (!fixed_built) {
                if (lane == 0) {
                    for (int s2 = 0; s2 < 288; s2++) lens[s2] = s2 < 144 ? 8 : s2 < 256 ? 9 : s2 < 280 ? 7 : 8;
                    build(litp, lcnt, lsym, lens, 288, IB_LIT);
                    for (int s2 = 0; s2 < 32; s2++) lens[s2] = 5;
                    build(distp, dcnt, dsym, lens, 32, IB_DIST);
                }
                wave_lds_sync();
                fixed_built = true;
            }
        } else if (type == 2) {
            fixed_built = false;
            const int hlit = (int)B.get(5) + 257, hdist = (int)B.get(5) + 1, hclen = (int)B.get(4) + 4;
            uint8_t *const cl = lens;
            uint32_t clv[19];
            for (int i = 0; i < 19; i++) clv[i] = 0;
            for (int i = 0; i < hclen; i++) {
                const int ord = i < 3 ? 16 + i : i == 3 ? 0 : (i & 1) ? 7 - (i - 5) / 2 : 8 + (i - 4) / 2;
                clv[ord] = B.get(3);
            }
            bool ok = true;
            if (lane == 0) {
                for (int i = 0; i < 19; i++) cl[i] = (uint8_t)clv[i];
                ok = build(litp, dcnt, dsym, cl, 19, IB_CL);
            }
            wave_lds_sync();
            if (!__builtin_amdgcn_readfirstlane((int)ok)) { st = 3; break; }
            int k = 0;
            while (k < hlit + hdist) {
                B.fill();
                const int s2 = decode_w(B, litp, dcnt, dsym, IB_CL);
                if (s2 < 0) { st = 3; break; }
                if (s2 < 16) { if (lane == 0) lens[k] = (uint8_t)s2; k++; continue; }
                int rep;
                uint8_t v = 0;
                if (s2 == 16) {
                    if (k == 0) { st = 3; break; }
                    wave_lds_sync();
                    v = lens[k - 1];
                    rep = 3 + (int)B.get(2);
                } else if (s2 == 17) {
                    rep = 3 + (int)B.get(3);
                } else {
                    rep = 11 + (int)B.get(7);
                }
                if (k + rep > hlit + hdist) { st = 3; break; }
                if (lane == 0)
                    for (int r2 = 0; r2 < rep; r2++) lens[k + r2] = v;
                k += rep;
            }
            if (st) break;
            wave_lds_sync();
            bool ok2 = lens[256] != 0;
            if (lane == 0 && ok2)
                ok2 = build(distp, dcnt, dsym, lens + hlit, hdist, IB_DIST) && build(litp, lcnt, lsym, lens, hlit, IB_LIT);
            wave_lds_sync();
            if (!__builtin_amdgcn_readfirstlane((int)ok2)) { st = lens[256] == 0 ? 3 : 4; break; }
        } else {
            st = 1;
            break;
        }
        while (true) {                                   // the block's codes
            B.fill();
            const int s2 = decode_w(B, litp, lcnt, lsym, IB_LIT);
            if (s2 < 256) {
                if (s2 < 0) { st = 5; break; }
                if (w >= ulen) { st = 7; break; }
                if (lane == 0) win[w & (W_WIN - 1)] = (uint8_t)s2;
                w++;
                if ((w & (W_HALF - 1)) == 0) { wave_lds_sync(); flush_to(w); }
                continue;
            }
            if (s2 == 256) break;
            if (s2 > 285) { st = 5; break; }
            B.fill();
            const uint32_t len = len_base(s2 - 257) + B.peek((int)len_ext(s2 - 257));
            B.drop((int)len_ext(s2 - 257));
            const int ds = decode_w(B, distp, dcnt, dsym, IB_DIST);
            if (ds < 0 || ds > 29) { st = 5; break; }
            const uint32_t dist = dist_base(ds) + B.get((int)dist_ext(ds));
            if (dist > w) { st = 6; break; }
            if (w + len > ulen) { st = 7; break; }
            wave_lds_sync();                             // (literals lane 0 wrote since the last sync)
            // lanes copy bytes j = lane, lane + 64, ...: byte j of the match is the source's byte j mod dist
            for (uint32_t j0 = 0; j0 < len; j0 += 64) {
                const uint32_t j = j0 + (uint32_t)lane;
                uint8_t v = 0;
                if (j < len) v = win[(w - dist + (dist >= len ? j : j % dist)) & (W_WIN - 1)];
                if (j < len) win[(w + j) & (W_WIN - 1)] = v;
            }
            const uint32_t w0 = w;
            w += len;
            if ((w0 >> 10) != (w >> 10)) { wave_lds_sync(); flush_to(w); }
        }
        if (st) break;
        if (B.byte_pos() > cend) { st = 8; break; }
    } while (!bfinal);
    if (!st && w != ulen) st = 9;
    if (!st) {
        wave_lds_sync();
        flush_to(ulen);
    }
    if (lane == 0) status[m] = st;
}

// CRC-32 (zlib's reflected polynomial) arithmetic: a * b mod P and x^(8 n) mod P, as zlib's multmodp / x2nmodp
__device__ __forceinline__ uint32_t crc_multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (int i = 0; i < 32; i++) {
        if (a & m) p ^= b;
        m >>= 1;
        b = (b & 1u) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
    }
    return p;
}
__device__ __forceinline__ uint32_t crc_x8n(uint32_t n) {     // x^(8 n) mod P
    uint32_t r = 1u << 31, base = 1u << 30;                     // 1, x
    for (uint64_t e = 8ull * n; e; e >>= 1) {
        if (e & 1) r = crc_multmodp(base, r);
        base = crc_multmodp(base, base);
    }
    return r;
}

// Each member's output checked against the CRC32 in its BGZF trailer (a member the decoder got wrong with the right
// length would otherwise pass): one wave per member, lane j the CRC of bytes [1 KiB j, 1 KiB (j + 1)) through an LDS
// table, the 64 partial CRCs combined in order (crc32_combine: crc(A B) = crc(A) x^(8 |B|) + crc(B) mod P).
__global__ __launch_bounds__(256) void k_crc32(const uint8_t *__restrict__ comp, const spg_bgzf_member *__restrict__ mem,
                                               int64_t n, const uint8_t *__restrict__ out, uint32_t *__restrict__ status,
                                               uint32_t op1k) {
    // slice-by-4 tables: T[k][b] = the CRC register after byte b followed by k zero bytes
    __shared__ uint32_t T[4][256];
    __shared__ uint32_t part[4][64];
    {
        uint32_t c = (uint32_t)threadIdx.x;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        T[0][threadIdx.x] = c;
        __syncthreads();
        for (int k = 1; k < 4; k++) {
            c = T[0][c & 0xFFu] ^ (c >> 8);
            T[k][threadIdx.x] = c;
        }
        __syncthreads();
    }
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t m = (int64_t)blockIdx.x * 4 + w;
    if (m >= n) return;                                         // (wave-uniform; no barrier below)
    if (status[m] != 0) return;
    const spg_bgzf_member M = mem[m];
    const uint32_t a = (uint32_t)lane * 1024u, e = min(M.ulen, a + 1024u);
    uint32_t c = 0xFFFFFFFFu;
    if (a < e) {
        // four bytes per step from two aligned dwords (the segment starts at any byte), 16 dwords loaded per batch
        typedef __attribute__((address_space(1))) const uint32_t gu32;
        const uint64_t s0 = M.uoff + a;
        gu32 *d = (gu32 *)(const void *)(out + (s0 & ~3ull));
        const uint32_t ph = (uint32_t)(s0 & 3) * 8u, nw = (e - a) / 4;
        uint32_t prev = d[0];
        uint32_t i = 0;
        for (; i + 16 <= nw; i += 16) {
            uint32_t v[16];
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = d[i + k + 1];
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint32_t x = ph ? __builtin_amdgcn_alignbyte(v[k], prev, ph >> 3) : prev;
                prev = v[k];
                c ^= x;
                c = T[3][c & 0xFFu] ^ T[2][(c >> 8) & 0xFFu] ^ T[1][(c >> 16) & 0xFFu] ^ T[0][c >> 24];
            }
        }
        for (; i < nw; i++) {
            const uint32_t nx = d[i + 1];
            const uint32_t x = ph ? __builtin_amdgcn_alignbyte(nx, prev, ph >> 3) : prev;
            prev = nx;
            c ^= x;
            c = T[3][c & 0xFFu] ^ T[2][(c >> 8) & 0xFFu] ^ T[1][(c >> 16) & 0xFFu] ^ T[0][c >> 24];
        }
        typedef __attribute__((address_space(1))) const uint8_t gu8;
        for (uint32_t b = a + 4 * nw; b < e; b++) c = T[0][(c ^ ((gu8 *)(out + M.uoff))[b]) & 0xFFu] ^ (c >> 8);
    }
    part[w][lane] = ~c;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lane == 0) {
        const uint32_t nseg = (M.ulen + 1023u) / 1024u;
        uint32_t crc = 0;                                       // crc32 of the empty string
        for (uint32_t j = 0; j < nseg; j++) {
            const uint32_t len = min(1024u, M.ulen - 1024u * j);
            crc = crc_multmodp(len == 1024u ? op1k : crc_x8n(len), crc) ^ part[w][j];
        }
        const uint8_t *t = comp + M.coff + M.clen;
        const uint32_t want = (uint32_t)t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
        if (crc != want) status[m] = 10;
    }
}

// x^(8 * 1024) mod P on the host (the combine's operator for a whole 1 KiB segment)
static uint32_t host_crc_x8n(uint32_t n) {
    auto mul = [](uint32_t a, uint32_t b) {
        uint32_t m = 1u << 31, p = 0;
        for (int i = 0; i < 32; i++) {
            if (a & m) p ^= b;
            m >>= 1;
            b = (b & 1u) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
        }
        return p;
    };
    uint32_t r = 1u << 31, base = 1u << 30;
    for (uint64_t e = 8ull * n; e; e >>= 1) {
        if (e & 1) r = mul(base, r);
        base = mul(base, base);
    }
    return r;
}

hipError_t launch_inflate(const uint8_t *comp, uint64_t comp_bytes, const spg_bgzf_member *mem, int64_t n, uint8_t *out,
                          uint32_t *status, hipStream_t st) {
    if (n <= 0) return hipSuccess;
#if defined(SPG_INFLATE_WAVE)        // (A/B builds: one member per wave, its window in LDS — r05c: 73.7 ms vs 27.0 on the
                                     // 10,000x BAM: 4 members per CU leave the decode's dependent chain exposed)
    hipLaunchKernelGGL(k_inflate_w, dim3((unsigned)n), dim3(64), 0, st, comp, comp_bytes, mem, n, out, status);
#else
    (void)comp_bytes;
    hipLaunchKernelGGL(k_inflate, dim3((unsigned)((n + INFLATE_MPW - 1) / INFLATE_MPW)), dim3(64),
                       (size_t)INFLATE_MPW * SLICE, st, comp, mem, n, out, status, INFLATE_MPW);
#endif
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    static const uint32_t op1k = host_crc_x8n(1024);
    hipLaunchKernelGGL(k_crc32, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, comp, mem, n, (const uint8_t *)out, status,
                       op1k);
    return hipGetLastError();
}

}  // namespace spg

// ---------------------------------------------------------------------------------------------------------------
// C-ABI (include/spings_gpu.h): upload, inflate, download; per-device scratch kept between calls (grow-only)
// ---------------------------------------------------------------------------------------------------------------
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace {
struct InflateDev {
    hipStream_t st = nullptr;
    uint8_t *comp = nullptr, *out = nullptr;
    size_t comp_cap = 0, out_cap = 0, mem_bytes = 0, status_bytes = 0;
    spg_bgzf_member *mem = nullptr;
    uint32_t *status = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
};
std::mutex g_inf_mu;
std::vector<InflateDev> g_inf;
thread_local std::string g_inf_err;
int ifail(const std::string &m) { g_inf_err = m; return -1; }
#define ICHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return ifail(std::string("spg_bgzf_inflate: ") + #x + ": " + hipGetErrorString(e_)); } while (0)
template <class T> int grow(T *&p, size_t &cap, size_t need) {
    if (need <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, need) != hipSuccess) return -1;
    cap = need;
    return 0;
}
}  // namespace

extern "C" {
const char *spg_bgzf_last_error(void) { return g_inf_err.c_str(); }

// The device decoder compiled for the host, member by member (CPU tests of its logic; the product inflates on the GPU)
int spg_bgzf_inflate_check(const uint8_t *comp, size_t comp_bytes, const spg_bgzf_member *members, int64_t n,
                           uint8_t *out, size_t out_bytes, uint32_t *status) {
    if (n < 0 || (n && (!comp || !members || !out || !status))) return ifail("spg_bgzf_inflate_check: bad argument");
    for (int64_t i = 0; i < n; i++) {
        const spg_bgzf_member &m = members[i];
        if (m.coff + m.clen + 8 > comp_bytes || m.uoff + m.ulen > out_bytes || m.ulen > 65536)
            return ifail("spg_bgzf_inflate_check: member " + std::to_string(i) + " outside the buffers");
    }
    // the decoder reads whole aligned 16-byte chunks: a padded copy, aligned like the device buffer
    std::vector<uint64_t> padded((comp_bytes + 64) / 8 + 1, 0);
    std::memcpy(padded.data(), comp, comp_bytes);
    std::vector<uint64_t> slice(spg::SLICE / 8);
    for (int64_t i = 0; i < n; i++)
        status[i] = spg::inflate_member(reinterpret_cast<const uint8_t *>(padded.data()), members[i], out,
                                        reinterpret_cast<uint8_t *>(slice.data()));
    return 0;
}

int spg_bgzf_inflate(int device, const uint8_t *comp, size_t comp_bytes, const spg_bgzf_member *members, int64_t n,
                     uint8_t *out, size_t out_bytes, uint32_t *status, float *kernel_ms) {
    if (n < 0 || (n && (!comp || !members || !out || !status))) return ifail("spg_bgzf_inflate: bad argument");
    for (int64_t i = 0; i < n; i++) {
        const spg_bgzf_member &m = members[i];
        if (m.coff + m.clen + 8 > comp_bytes || m.uoff + m.ulen > out_bytes || m.ulen > 65536)
            return ifail("spg_bgzf_inflate: member " + std::to_string(i) + " outside the buffers");
    }
    if (kernel_ms) *kernel_ms = 0.f;
    if (n == 0) return 0;
    // one caller per device at a time (the device's scratch buffers are shared); the caller's current device is restored
    std::lock_guard<std::mutex> lk(g_inf_mu);
    int prev = 0, nd = 0;
    ICHK(hipGetDevice(&prev));
    ICHK(hipGetDeviceCount(&nd));
    if (device < 0 || device >= nd) return ifail("spg_bgzf_inflate: bad device");
    if ((int)g_inf.size() < nd) g_inf.resize((size_t)nd);
    InflateDev &D = g_inf[(size_t)device];
    struct Restore { int d; ~Restore() { (void)hipSetDevice(d); } } restore{prev};
    ICHK(hipSetDevice(device));
    if (!D.st) {
        ICHK(hipStreamCreateWithFlags(&D.st, hipStreamNonBlocking));
        ICHK(hipEventCreate(&D.ev[0]));
        ICHK(hipEventCreate(&D.ev[1]));
    }
    if (grow(D.comp, D.comp_cap, comp_bytes + 64) || grow(D.out, D.out_cap, out_bytes + 64) ||
        grow(D.mem, D.mem_bytes, (size_t)n * sizeof(spg_bgzf_member)) ||
        grow(D.status, D.status_bytes, (size_t)n * sizeof(uint32_t)))
        return ifail("spg_bgzf_inflate: out of device memory");
    // after the first enqueue every failure drains the stream before returning: the caller's `out` may be the target of a
    // queued copy, and it inflates failed members into it next
    auto drained = [&](int rc) { (void)hipStreamSynchronize(D.st); return rc; };
#define IQ(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return drained(ifail(std::string("spg_bgzf_inflate: ") + #x + ": " + hipGetErrorString(e_))); } while (0)
    IQ(hipMemcpyAsync(D.comp, comp, comp_bytes, hipMemcpyHostToDevice, D.st));
    IQ(hipMemsetAsync(D.comp + comp_bytes, 0, 64, D.st));
    IQ(hipMemcpyAsync(D.mem, members, (size_t)n * sizeof(spg_bgzf_member), hipMemcpyHostToDevice, D.st));
    IQ(hipEventRecord(D.ev[0], D.st));
    IQ(spg::launch_inflate(D.comp, comp_bytes, D.mem, n, D.out, D.status, D.st));
    IQ(hipEventRecord(D.ev[1], D.st));
    IQ(hipMemcpyAsync(out, D.out, out_bytes, hipMemcpyDeviceToHost, D.st));
    IQ(hipMemcpyAsync(status, D.status, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, D.st));
    IQ(hipStreamSynchronize(D.st));
#undef IQ
    if (kernel_ms && hipEventElapsedTime(kernel_ms, D.ev[0], D.ev[1]) != hipSuccess) *kernel_ms = -1.f;   // (timing only)
    // (the scratch only grows; after a BAM above 2 GiB inflated it is given back rather than held in HBM)
    if (D.out_cap > ((size_t)2 << 30)) {
        for (void *p : {(void *)D.comp, (void *)D.out}) (void)hipFree(p);
        D.comp = D.out = nullptr;
        D.comp_cap = D.out_cap = 0;
    }
    return 0;
}

// The device's inflate scratch freed (it only grows otherwise: one large BAM would keep its size in HBM)
int spg_bgzf_release(int device) {
    std::lock_guard<std::mutex> lk(g_inf_mu);
    if (device < 0 || (size_t)device >= g_inf.size()) return 0;
    InflateDev &D = g_inf[(size_t)device];
    if (!D.st) return 0;
    int prev = 0;
    ICHK(hipGetDevice(&prev));
    ICHK(hipSetDevice(device));
    (void)hipStreamSynchronize(D.st);
    for (void *p : {(void *)D.comp, (void *)D.out, (void *)D.mem, (void *)D.status})
        if (p) (void)hipFree(p);
    D.comp = D.out = nullptr;
    D.mem = nullptr;
    D.status = nullptr;
    D.comp_cap = D.out_cap = D.mem_bytes = D.status_bytes = 0;
    ICHK(hipSetDevice(prev));
    return 0;
}
}
