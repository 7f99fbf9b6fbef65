// spg_inflate.hip — BGZF members inflated on the GPU (process_bam's BAM read,
// live_variant_caller.py:54-72, which htslib's BGZF reader serves in the reference).
//
// A BGZF file is a sequence of independent raw-DEFLATE members (RFC 1951) of at most 64 KiB of output each.
// k_inflate_par (the product path): one wave per member, its blocks' data bits decoded by 64 lanes at once — segments
// that resynchronise on token starts — then the tokens resolved into the member's output through an LDS window ring
// (the comment above the kernel).  k_inflate: one lane per member, the whole member as one serial decode; it takes the
// members k_inflate_par leaves (stored blocks, token overflows, anything malformed) and reports real errors.  k_crc32
// checks every member's output against its trailer.  Both decoders share the bit reader, the two-level Huffman tables
// and the block-header code, compiled for the host too (spg_bgzf_inflate_check / _par_check: CPU tests against zlib).
// A member's status word is 0 when it inflated to exactly its ISIZE bytes with the trailer's CRC32; anything else (a
// corrupt stream) is reported and the caller inflates that member on the host (or plans the BAM there).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "spings_gpu.h"

#ifndef SPG_INFLATE_MATCH_HOOK
#define SPG_INFLATE_MATCH_HOOK(dist, len)     // (tools/inflate_stats.cpp: match statistics of a host run)
#endif
#ifndef SPG_INFLATE_SLOW_HOOK
#define SPG_INFLATE_SLOW_HOOK(pb)             // (tools/inflate_stats.cpp: codes longer than the root table)
#endif

namespace spg {

// Per-member decode tables: one slice of SLICE bytes (LDS on the device: one per member; a host array in the check).
// Two-level tables of u16 entries: a root table indexed by the next pb bits and, for codes longer than pb, sub-tables
// indexed by the bits after them (zlib's inflate_table layout), so every symbol is one or two lookups — no bit-by-bit
// walk whose loop would stall a whole wave whenever one lane meets a long code.  Entry: symbol | code length << 9
// (length 0: no code), or a link 0x8000 | sub-table bits << 11 | sub-table offset.  The counts and sorted symbols are
// build scratch; the code-length code's table borrows the literal table's area (it is done with before that is built);
// the code lengths are read into the lengths area.
constexpr int IB_LIT = 10, IB_DIST = 8, IB_CL = 7;      // root table bits
constexpr int TAB_LIT = 1536, TAB_DIST = 512;           // entries: root + sub-tables (zlib's bounds for these roots: 1332, 402)
constexpr int SL_LITP = 0, SL_DISTP = 2 * TAB_LIT, SL_CNT = SL_DISTP + 2 * TAB_DIST, SL_SYM = SL_CNT + 32,
              SL_LENS = SL_SYM + 576, SLICE = SL_LENS + 320;
static_assert(SLICE % 8 == 0 && SLICE == 5024, "slice layout");

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

// canonical Huffman tables from code lengths (RFC 1951 3.2.2) into tab (cap entries, root pb bits); false:
// over-subscribed, an incomplete code with more than one symbol (a single-code distance alphabet may be incomplete), or
// sub-tables past cap.  count[16] / sym[n]: scratch.
__host__ __device__ __forceinline__ bool build(uint16_t *tab, int cap, uint16_t *count, uint16_t *sym, const uint8_t *len,
                                               int n, int pb) {
    for (int i = 0; i < 16; i++) count[i] = 0;
    for (int s = 0; s < n; s++) count[len[s]]++;
    uint64_t *p8 = reinterpret_cast<uint64_t *>(tab);
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
    // codes in canonical order; count[l] becomes the codes of length l not yet placed (sub-table sizing, as zlib)
    uint32_t code = 0, prefix = ~0u, sub = 0, sbits = 0;
    int next = 1 << pb, k = 0;
    for (int l = 1; l <= 15; l++) {
        for (; count[l]; count[l]--, k++, code++) {
            const uint32_t rev = __builtin_bitreverse32(code) >> (32 - l);
            const uint16_t e = (uint16_t)(sym[k] | (l << 9));
            if (l <= pb) {
                for (uint32_t x = rev; x < (1u << pb); x += 1u << l) tab[x] = e;
                continue;
            }
            const uint32_t pre = rev & ((1u << pb) - 1);
            if (pre != prefix) {                         // a new sub-table for this root prefix
                uint32_t cur = (uint32_t)(l - pb);
                int lf = 1 << cur;
                while ((int)cur + pb < 15) {
                    lf -= count[cur + pb];
                    if (lf <= 0) break;
                    cur++;
                    lf <<= 1;
                }
                if (next + (1 << cur) > cap) return false;
                for (int x = 0; x < (1 << cur); x++) tab[next + x] = 0;
                tab[pre] = (uint16_t)(0x8000u | cur << 11 | (uint32_t)next);
                prefix = pre;
                sub = (uint32_t)next;
                sbits = cur;
                next += 1 << cur;
            }
            for (uint32_t x = rev >> pb; x < (1u << sbits); x += 1u << (l - pb)) tab[sub + x] = e;
        }
        code <<= 1;
    }
    return true;
}

#if defined(__HIP_DEVICE_COMPILE__)
// build() by the 64 lanes of a wave at once (k_inflate_par: every lane used to run the serial build, ~16 % of a member's
// time at 347k clocks per block, r06 tools/src_ab.py prof): lane l holds the lengths of symbols l, l + 64, ...; the
// counts per length by ballots, each symbol's canonical code from its rank among the symbols of its length (ballot +
// mbcnt), the root entries of codes <= pb bits written by their own lanes; the codes longer than pb (zlib's sub-table
// layout, usually a few dozen) then by the serial loop on every lane alike.  The same tables as build().
__device__ __forceinline__ bool build_wave(uint16_t *tab, int cap, uint16_t *count, uint16_t *sym, const uint8_t *len, int n,
                                           int pb) {
    // per-length values live in lanes 0..15 (lane l: length l), not in scalar arrays (which spilled SGPRs kernel-wide)
    constexpr int NCH = 5;                               // n <= 320 symbols
    const uint32_t lane = threadIdx.x & 63;
    uint32_t L[NCH];
#pragma unroll
    for (int i = 0; i < NCH; i++) L[i] = (int)lane + 64 * i < n ? len[lane + 64 * i] : 0xFFu;
    uint32_t cntv = 0;                                   // lane l: symbols of length l
#pragma unroll
    for (int i = 0; i < NCH; i++)
#pragma unroll 1
        for (uint32_t l = 0; l < 16; l++) {
            const uint32_t c = (uint32_t)__popcll(__ballot(L[i] == l));
            cntv += lane == l ? c : 0u;
        }
    uint64_t *p8 = reinterpret_cast<uint64_t *>(tab);
    for (int i = (int)lane; i < (1 << pb) / 4; i += 64) p8[i] = 0;
    if ((int)__builtin_amdgcn_readlane(cntv, 0) == n) return true;   // no codes: every lookup fails (only a distance code may)
    // Kraft (over-subscribed at any length; incomplete with more than one symbol), the lengths' first canonical codes and
    // offsets in the sorted symbol list, the codes longer than pb
    int left = 1;
    bool over = false;
    uint32_t o = 0, code = 0, offv = 0, fcv = 0, nlong = 0;
#pragma unroll 1
    for (uint32_t l = 1; l < 16; l++) {
        const uint32_t c = __builtin_amdgcn_readlane(cntv, l);
        left = (left << 1) - (int)c;
        over |= left < 0;
        offv = lane == l ? o : offv;
        fcv = lane == l ? code : fcv;
        o += c;
        code = (code + c) << 1;
        nlong += l > (uint32_t)pb ? c : 0u;
    }
    if (over) return false;
    if (left > 0 && n - (int)__builtin_amdgcn_readlane(cntv, 0) > 1) return false;
    // each symbol's rank among the symbols of its length (canonical order = by length, then by symbol): the earlier
    // chunks' count of its length (basev, lane l) + its rank in this chunk (mbcnt of the length's ballot)
    uint32_t code_of[NCH];
    uint32_t basev = 0;
#pragma unroll
    for (int i = 0; i < NCH; i++) {
        uint32_t rin = 0, chunkc = 0;
#pragma unroll 1
        for (uint32_t l = 1; l < 16; l++) {
            const uint64_t mk = __ballot(L[i] == l);
            const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
            rin = L[i] == l ? r : rin;
            chunkc = lane == l ? (uint32_t)__popcll(mk) : chunkc;
        }
        const int li = (int)(L[i] & 15u);
        const uint32_t b = (uint32_t)__shfl((int)basev, li, 64), of = (uint32_t)__shfl((int)offv, li, 64),
                       f = (uint32_t)__shfl((int)fcv, li, 64);
        code_of[i] = 0;
        if (L[i] >= 1 && L[i] < 16) {
            sym[of + b + rin] = (uint16_t)(lane + 64 * i);
            code_of[i] = f + b + rin;
        }
        basev += chunkc;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // root entries of the codes of <= pb bits, by their own lanes
#pragma unroll
    for (int i = 0; i < NCH; i++) {
        const uint32_t l = L[i];
        if (l >= 1 && l <= (uint32_t)pb) {
            const uint32_t rev = __builtin_bitreverse32(code_of[i]) >> (32 - l);
            const uint16_t e = (uint16_t)((lane + 64 * i) | (l << 9));
            for (uint32_t x = rev; x < (1u << pb); x += 1u << l) tab[x] = e;
        }
    }
    if (nlong) {
        // the codes longer than pb in canonical order, as build()'s loop places them (count[]: the codes of each length
        // not yet placed, which its sub-table sizing reads)
        if (lane < 16) count[lane] = (uint16_t)cntv;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t cd = __builtin_amdgcn_readlane(fcv, pb + 1), prefix = ~0u, sub = 0, sbits = 0;
        int next = 1 << pb, k = (int)__builtin_amdgcn_readlane(offv, pb + 1);
        for (int l = pb + 1; l <= 15; l++) {
            for (; count[l]; count[l]--, k++, cd++) {
                const uint32_t rev = __builtin_bitreverse32(cd) >> (32 - l);
                const uint16_t e = (uint16_t)(sym[k] | (l << 9));
                const uint32_t pre = rev & ((1u << pb) - 1);
                if (pre != prefix) {
                    uint32_t cur = (uint32_t)(l - pb);
                    int lf = 1 << cur;
                    while ((int)cur + pb < 15) {
                        lf -= count[cur + pb];
                        if (lf <= 0) break;
                        cur++;
                        lf <<= 1;
                    }
                    if (next + (1 << cur) > cap) return false;
                    for (int x = 0; x < (1 << cur); x++) tab[next + x] = 0;
                    tab[pre] = (uint16_t)(0x8000u | cur << 11 | (uint32_t)next);
                    prefix = pre;
                    sub = (uint32_t)next;
                    sbits = cur;
                    next += 1 << cur;
                }
                for (uint32_t x = rev >> pb; x < (1u << sbits); x += 1u << (l - pb)) tab[sub + x] = e;
            }
            cd <<= 1;
        }
    }
    return true;
}
#endif

template <bool WAVE>
__host__ __device__ __forceinline__ bool build_t(uint16_t *tab, int cap, uint16_t *count, uint16_t *sym, const uint8_t *len,
                                                 int n, int pb) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (WAVE) return build_wave(tab, cap, count, sym, len, n, pb);
#endif
    return build(tab, cap, count, sym, len, n, pb);
}

// one symbol; -1 on an invalid code.  Needs >= 15 bits in the buffer (the caller's fill()).
__host__ __device__ __forceinline__ int decode(IBits &B, const uint16_t *tab, int pb) {
    uint32_t e = tab[B.peek(pb)];
    if (e & 0x8000u) e = tab[(e & 0x7FFu) + (B.peek(pb + (int)((e >> 11) & 7u)) >> pb)];
    const int l = (int)((e >> 9) & 15u);
    if (!l) return -1;
    if (l > pb) SPG_INFLATE_SLOW_HOOK(pb);
    B.drop(l);
    return (int)(e & 0x1FFu);
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

// A fixed (type 1) or dynamic (type 2) block's header read after its 3 header bits, and its decode tables built into
// slice; status 0, 3 bad code lengths, 4 bad table.  fixed_built: the fixed tables are still in the slice (a member's
// later fixed blocks skip the rebuild).  The device's parallel inflater runs it on every lane of a wave alike (the same
// bits, the same LDS writes).
template <bool WAVE = false>
__host__ __device__ __forceinline__ uint32_t block_tables(IBits &B, uint8_t *slice, uint32_t type, bool &fixed_built) {
    uint16_t *const litp = reinterpret_cast<uint16_t *>(slice + SL_LITP);
    uint16_t *const distp = reinterpret_cast<uint16_t *>(slice + SL_DISTP);
    uint16_t *const cnt = reinterpret_cast<uint16_t *>(slice + SL_CNT);
    uint16_t *const sym = reinterpret_cast<uint16_t *>(slice + SL_SYM);
    uint8_t *const lens = slice + SL_LENS;
    if (type == 1) {                                     // the fixed codes (RFC 1951 3.2.6), built once per member
        if (!fixed_built) {
            for (int s = 0; s < 288; s++) lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
            build_t<WAVE>(litp, TAB_LIT, cnt, sym, lens, 288, IB_LIT);
            for (int s = 0; s < 32; s++) lens[s] = 5;    // (30 and 31 complete the code; decoding them fails)
            build_t<WAVE>(distp, TAB_DIST, cnt, sym, lens, 32, IB_DIST);
            fixed_built = true;
        }
        return 0;
    }
    fixed_built = false;
    const int hlit = (int)B.get(5) + 257, hdist = (int)B.get(5) + 1, hclen = (int)B.get(4) + 4;
    uint8_t *const cl = lens;                            // 19 code-length code lengths, in RFC order
    for (int i = 0; i < 19; i++) cl[i] = 0;
    for (int i = 0; i < hclen; i++) {
        const int ord = i < 3 ? 16 + i : i == 3 ? 0 : (i & 1) ? 7 - (i - 5) / 2 : 8 + (i - 4) / 2;   // RFC 1951 3.2.7
        cl[ord] = (uint8_t)B.get(3);
    }
    if (!build_t<WAVE>(litp, TAB_LIT, cnt, sym, cl, 19, IB_CL)) return 3;
    int k = 0;
    while (k < hlit + hdist) {
        B.fill();
        const int s = decode(B, litp, IB_CL);
        if (s < 0) return 3;
        if (s < 16) { lens[k++] = (uint8_t)s; continue; }
        int rep;
        uint8_t v = 0;
        if (s == 16) {
            if (k == 0) return 3;
            v = lens[k - 1];
            rep = 3 + (int)B.get(2);
        } else if (s == 17) {
            rep = 3 + (int)B.get(3);
        } else {
            rep = 11 + (int)B.get(7);
        }
        if (k + rep > hlit + hdist) return 3;
        while (rep--) lens[k++] = v;
    }
    if (lens[256] == 0) return 3;                        // no end-of-block code
    if (!build_t<WAVE>(distp, TAB_DIST, cnt, sym, lens + hlit, hdist, IB_DIST) ||
        !build_t<WAVE>(litp, TAB_LIT, cnt, sym, lens, hlit, IB_LIT))
        return 4;
    return 0;
}

// one member into out + M.uoff; status (see k_inflate).  slice: SLICE bytes, 8-byte aligned.
__host__ __device__ __forceinline__ uint32_t inflate_member(const uint8_t *comp, const spg_bgzf_member &M, uint8_t *out,
                                                            uint8_t *slice) {
    const uint16_t *const litp = reinterpret_cast<const uint16_t *>(slice + SL_LITP);
    const uint16_t *const distp = reinterpret_cast<const uint16_t *>(slice + SL_DISTP);
    uint8_t *o = out + M.uoff;
    const uint32_t ulen = M.ulen;
    const uint8_t *const cend = comp + M.coff + M.clen;
    IBits B;
    B.end = cend + 8;
    B.start(comp + M.coff);
    uint32_t w = 0;                                      // bytes written
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
        if (type == 3) { st = 1; break; }
        if ((st = block_tables(B, slice, type, fixed_built)) != 0) break;
        while (true) {                                   // the block's codes
            B.fill();
            const int s = decode(B, litp, IB_LIT);
            if (s < 256) {
                if (s < 0) { st = 5; break; }
                if (w >= ulen) { st = 7; break; }
                o[w++] = (uint8_t)s;
                continue;
            }
            if (s == 256) break;
            if (s > 285) { st = 5; break; }
            B.fill();                                    // <= 5 extra bits, then <= 15 of the distance code
            const uint32_t len = len_base(s - 257) + B.peek((int)len_ext(s - 257));
            B.drop((int)len_ext(s - 257));
            const int ds = decode(B, distp, IB_DIST);
            if (ds < 0 || ds > 29) { st = 5; break; }
            const uint32_t dist = dist_base(ds) + B.get((int)dist_ext(ds));
            SPG_INFLATE_MATCH_HOOK(dist, len);
            if (dist > w) { st = 6; break; }
            if (w + len > ulen) { st = 7; break; }
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
// (a member's symbols are a dependent chain; r04ze: 19.3 ms on the 10,000x BAM at 3 members per block).  Since r05 the
// fallback of k_inflate_par (only_fallback: the members it left).
constexpr int INFLATE_MPW = 3;
constexpr uint32_t ST_FALLBACK = 100;   // (k_inflate_par) this member is left to the lane kernel
__global__ __launch_bounds__(64) void k_inflate(const uint8_t *__restrict__ comp, const spg_bgzf_member *__restrict__ mem,
                                                int64_t n, uint8_t *__restrict__ out, uint32_t *__restrict__ status, int mpw,
                                                int only_fallback) {
    extern __shared__ __align__(16) uint8_t inf_lds[];
    if ((int)threadIdx.x >= mpw) return;
    const int64_t m = (int64_t)blockIdx.x * mpw + threadIdx.x;
    if (m >= n) return;
    if (only_fallback && status[m] != ST_FALLBACK) return;
    status[m] = inflate_member(comp, mem[m], out, inf_lds + (size_t)threadIdx.x * SLICE);
}

// ------------------------------------------------------------------------------------------------------------------
// k_inflate_par: one member per wave, its DEFLATE stream decoded by all 64 lanes at once.
//
// The lane-per-member kernel above runs a member's ~16k symbols as one dependent chain on one lane, three members per
// wave: every instruction of a symbol costs the wave its 4 issue cycles for one member's progress (r05h: the symbol decode
// alone 12 ms of 19.7 per 10,000x BAM).  Here a block's data bits are cut into K <= 64 equal segments (at least
// PAR_MIN_SEG bits each) and lane k decodes segment k on its own, starting at the segment's first bit as if a token began
// there.  Huffman codes self-synchronise: a decode begun at a wrong bit soon lands on a true token boundary and from there
// on reads the true tokens (measured on the 2,000x simulator BAM, /tmp-free harness in tests/test_inflate_check.py: ~95 %
// of lanes within 32 tokens, all within ~128 but for segments shorter than the distance).
//  * Phase A (every lane): the segment's tokens (literal, match (length, distance), end of block) and their start
//    positions; the lane's tokens end at the first token start past the segment (its `end`).
//  * Sync (every lane k >= 1): decode the true stream from the end of lane k - 1's true tokens until it meets one of lane
//    k's phase-A token starts; lane k's true tokens are these redo tokens plus its own tokens from that start on.  A lane
//    that never meets its own tokens (its redo covers the segment) moves its end: the lanes after it synchronise again
//    (rounds until no end moves).  More than PAR_RCAP redo tokens, a token overflow, a stored block or anything malformed
//    sends the member to the lane-per-member kernel (status ST_FALLBACK), which also reports real errors.
//  * The block ends at the first true end-of-block token; lanes past it decoded the next block with this block's tables
//    and are ignored; the next block's header follows the end-of-block code.
//  * Phase B (resolve): the true token lists in order, 64 tokens (at most PAR_BATCH output bytes) at a time, into an LDS
//    ring of the last PAR_RING output bytes (indexed by global output address): literals and matches whose source lies
//    before the batch are written at once (lane-parallel; matches longer than 32 bytes by the whole wave), then the
//    matches whose source is an earlier token of the batch, in order, each by the whole wave.  Completed 1 KiB blocks of
//    global memory are written from the ring with 16-byte stores; source bytes already flushed there (most matches of
//    BAM data: DEFLATE reaches 32 KiB back) are read from that written output.  A small ring keeps LDS per
//    wave low, so several waves per SIMD hide each other's latency: r05n 10,000x BAM 8.56 ms with an 8 KiB ring (13 KiB,
//    3 waves per SIMD; a 32 KiB ring allowed one: 14.0 ms); r06t, with 107 VGPRs since the whole-wave table builds, a
//    4 KiB ring (9.1 KiB: 4 waves per SIMD) 6.07 -> 5.81 ms; r06u, a 2 KiB ring (7.1 KiB) with the VGPRs held to 96 by
//    the waves-per-EU attribute (no spill): 5 waves per SIMD, 5.22 ms (6 waves, 80 VGPRs with spills: 5.3 ms).
// Token lists, positions and redo tokens live in global scratch (inflate_scratch_bytes: 12 B per compressed byte + 76 KiB
// per member).
// ------------------------------------------------------------------------------------------------------------------
constexpr uint32_t TK_EOB = 0x40000000u, TK_MATCH = 0x80000000u;   // tokens: literal byte | EOB | match (len-3)<<16 | dist-1
constexpr uint32_t PAR_RCAP = 256;                                  // redo tokens per lane
constexpr uint32_t PAR_MIN_SEG = 1024;                              // data bits per lane at least (fewer lanes for short blocks)
constexpr uint32_t PAR_RING = 2048, PAR_BATCH = 1024;               // LDS window ring (power of two), batch output cap
constexpr uint32_t PAR_RECENT = PAR_RING - PAR_BATCH;               // the ring holds every byte from w - PAR_RECENT on
static_assert(PAR_RECENT >= 1023, "an unflushed partial 1 KiB block must stay in the ring");
// scratch per member m (u32 units unless noted): token lists at 2 coff + 2048 m (2 clen + 2048 of them, split evenly
// over the block's lanes), token start positions (u16, relative to the lane's first bit) at the same index of a u16 array,
// redo tokens at 64 RCAP m
// (16-byte aligned: a lane's tokens are stored four at a time; a member's area ends before the next member's starts)
__host__ __device__ __forceinline__ uint64_t par_tok_at(const spg_bgzf_member &M, uint64_t m) {
    return (2ull * M.coff + 2048ull * m + 3) & ~3ull;
}
__host__ __device__ __forceinline__ uint32_t par_area(const spg_bgzf_member &M) { return 2u * M.clen + 2044u; }
// a lane's capacity (tokens) when the block's data is cut into K segments: a multiple of 4
__host__ __device__ __forceinline__ uint32_t par_cap(const spg_bgzf_member &M, uint32_t K) { return (par_area(M) / K) & ~3u; }

struct Tabs {
    const uint16_t *litp, *distp;
};
__host__ __device__ __forceinline__ Tabs tabs_of(const uint8_t *slice) {
    return Tabs{reinterpret_cast<const uint16_t *>(slice + SL_LITP), reinterpret_cast<const uint16_t *>(slice + SL_DISTP)};
}

// the next unread bit, relative to base (IBits: buf holds n bits, r rn bits, then the chunk at qa)
__host__ __device__ __forceinline__ uint32_t ib_pos(const IBits &B, const uint8_t *base) {
    return (uint32_t)(B.qa - base) * 8u - (uint32_t)B.rn - (uint32_t)B.n;
}
__host__ __device__ __forceinline__ void ib_seek(IBits &B, const uint8_t *base, uint32_t p) {
    B.start(base + (p >> 3));
    B.fill();
    B.drop((int)(p & 7u));
}

// one token at the reader's position; false: no valid token starts here
__host__ __device__ __forceinline__ bool next_token(IBits &B, const Tabs &T, uint32_t &t) {
    B.fill();
    const int s = decode(B, T.litp, IB_LIT);
    if (s < 256) {
        t = (uint32_t)s;
        return s >= 0;
    }
    if (s == 256) {
        t = TK_EOB;
        return true;
    }
    if (s > 285) return false;
    B.fill();
    const uint32_t len = len_base(s - 257) + B.peek((int)len_ext(s - 257));
    B.drop((int)len_ext(s - 257));
    const int ds = decode(B, T.distp, IB_DIST);
    if (ds < 0 || ds > 29) return false;
    const uint32_t dist = dist_base(ds) + B.get((int)dist_ext(ds));
    t = TK_MATCH | (len - 3u) << 16 | (dist - 1u);
    return true;
}

// phase A of one lane: tokens from bit s while they start before stop, with their start positions (pos[i] = start - s).
// A position where no valid token starts (only before the lane has synchronised) is skipped bit by bit.  The first
// end-of-block token is recorded (index, the bit after it); ne counts them.
struct SegOut {
    uint32_t end, n, ne, e0i, e0p;
    bool ovf;
};
__host__ __device__ __forceinline__ SegOut decode_seg(IBits &B, const uint8_t *base, uint32_t s, uint32_t stop, const Tabs &T,
                                                      uint32_t *tok, uint16_t *pos, uint32_t cap) {
    SegOut o{};
    uint32_t p = s, n = 0;
    // tokens and their positions staged four at a time in registers, then one 16-byte / 8-byte store each (tok and pos
    // are 16- / 8-byte aligned and cap is a multiple of 4): scattered 4-byte stores of 64 lanes made ~12x the
    // algorithmic write traffic (r05s PMC)
    uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, p01 = 0, p23 = 0;
    ib_seek(B, base, p);
    while (p < stop) {
        uint32_t t;
        if (!next_token(B, T, t)) {
            ib_seek(B, base, ++p);
            continue;
        }
        if (n >= cap) {
            o.ovf = true;
            break;
        }
        const uint32_t pr = p - s, sl = n & 3u;
        t0 = sl == 0 ? t : t0;
        t1 = sl == 1 ? t : t1;
        t2 = sl == 2 ? t : t2;
        t3 = sl == 3 ? t : t3;
        p01 = sl == 0 ? pr : sl == 1 ? (p01 | pr << 16) : p01;
        p23 = sl == 2 ? pr : sl == 3 ? (p23 | pr << 16) : p23;
        if (sl == 3) {
            *reinterpret_cast<uint4 *>(tok + (n - 3)) = make_uint4(t0, t1, t2, t3);
            *reinterpret_cast<uint2 *>(pos + (n - 3)) = make_uint2(p01, p23);
        }
        n++;
        p = ib_pos(B, base);
        if (t == TK_EOB) {
            if (o.ne == 0) { o.e0i = n - 1; o.e0p = p; }
            o.ne++;
        }
    }
    // the last 1-3 staged tokens
    const uint32_t r = n & 3u, b0 = n - r;
    if (r > 0) { tok[b0] = t0; pos[b0] = (uint16_t)p01; }
    if (r > 1) { tok[b0 + 1] = t1; pos[b0 + 1] = (uint16_t)(p01 >> 16); }
    if (r > 2) { tok[b0 + 2] = t2; pos[b0 + 2] = (uint16_t)p23; }
    o.end = p;
    o.n = n;
    return o;
}

// sync of lane k >= 1: the true stream from `start` (where the previous lane's true tokens end) until it meets one of
// the lane's phase-A token starts.  The lane's true tokens: redo[0, r) then its phase-A tokens [i, n).  end: where they
// end (phase A's end when they met, else the redo's).  eob >= 0: the true list's end-of-block token at that index (eobp:
// the bit after it).  fail: more than PAR_RCAP redo tokens, or no valid token on the true stream.
struct SyncOut {
    uint32_t i, r, end, eobp;
    int32_t eob;
    bool fail;
};
__host__ __device__ __forceinline__ SyncOut resync(IBits &B, const uint8_t *base, uint32_t s, uint32_t start, uint32_t stop,
                                                   const SegOut &so, const uint32_t *tok, const uint16_t *pos, const Tabs &T,
                                                   uint32_t *redo) {
    SyncOut y{};
    y.eob = -1;
    uint32_t cur = start, ii = 0, r = 0;
    bool seeked = false;
    // the recorded starts four at a time (one 8-byte load instead of a dependent 2-byte load per start)
    uint64_t pw = 0;
    uint32_t pb = ~0u;
    auto P = [&](uint32_t i) -> uint32_t {
        if ((i >> 2) != pb) {
            pb = i >> 2;
            pw = *reinterpret_cast<const uint64_t *>(pos + 4 * pb);
        }
        return (uint32_t)(pw >> (16 * (i & 3u))) & 0xFFFFu;
    };
    for (;;) {
        while (ii < so.n && s + P(ii) < cur) ii++;
        if (ii < so.n && s + P(ii) == cur) break;                  // met: the rest of phase A's tokens are true
        if (cur >= stop) {                                          // never met: the redo is the lane's whole list
            y.i = so.n;
            y.r = r;
            y.end = cur;
            return y;
        }
        if (r == PAR_RCAP) { y.fail = true; return y; }
        if (!seeked) {
            ib_seek(B, base, cur);
            seeked = true;
        }
        uint32_t t;
        if (!next_token(B, T, t)) { y.fail = true; return y; }
        redo[r++] = t;
        cur = ib_pos(B, base);
        if (t == TK_EOB) {
            y.eob = (int32_t)(r - 1);
            y.eobp = cur;
            y.i = so.n;
            y.r = r;
            y.end = cur;
            return y;
        }
    }
    y.i = ii;
    y.r = r;
    y.end = so.end;
    // the first end-of-block token among phase A's from index ii on
    if (so.ne && so.e0i >= ii) {
        y.eob = (int32_t)(r + so.e0i - ii);
        y.eobp = so.e0p;
    } else if (so.ne > 1) {                                         // (rare: an end of block in the lane's garbage prefix)
        for (uint32_t j = ii; j < so.n; j++)
            if (tok[j] == TK_EOB) {
                y.eob = (int32_t)(r + j - ii);
                y.eobp = j + 1 < so.n ? s + P(j + 1) : so.end;
                break;
            }
    }
    return y;
}

// lane 0 starts on the true stream: its list is its phase-A tokens
__host__ __device__ __forceinline__ SyncOut sync_lane0(const SegOut &so) {
    SyncOut y{};
    y.eob = -1;
    y.end = so.end;
    if (so.ne) {
        y.eob = (int32_t)so.e0i;
        y.eobp = so.e0p;
    }
    return y;
}

// The same algorithm on the host, lane after lane, with a plain sequential resolve (tests/test_inflate_check.py: the
// token lists against zlib, and how often a member would fall back).  stats[0] members inflated, [1] token overflow,
// [2] no sync, [3] stored block, [4] bad header, [5] no end of block, [6] bad resolve, [7] redo tokens, [8] blocks,
// [9] sync rounds beyond the first.
__host__ uint32_t par_member_host(const uint8_t *comp, const spg_bgzf_member &M, uint8_t *out, uint8_t *slice,
                                  uint64_t *stats, std::vector<uint32_t> &tok, std::vector<uint16_t> &pos,
                                  std::vector<uint32_t> &redo) {
    const uint8_t *const base = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(comp + M.coff) & ~(uintptr_t)15);
    const uint32_t pay0 = (uint32_t)((comp + M.coff) - base) * 8u, dend = pay0 + M.clen * 8u;
    IBits B;
    B.end = comp + M.coff + M.clen + 8;
    tok.assign(par_area(M), 0);
    pos.assign(par_area(M), 0);
    redo.assign(64ull * PAR_RCAP, 0);
    const Tabs T = tabs_of(slice);
    uint8_t *const o = out + M.uoff;
    uint32_t w = 0, p = pay0;
    bool fixed_built = false;
    int bfinal = 0;
    auto fb = [&](int why) {
        stats[why]++;
        return ST_FALLBACK;
    };
    do {
        ib_seek(B, base, p);
        bfinal = (int)B.get(1);
        const uint32_t type = B.get(2);
        if (type == 0 || type == 3) return fb(3);
        if (block_tables(B, slice, type, fixed_built) != 0) return fb(4);
        stats[8]++;
        const uint32_t d0 = ib_pos(B, base);
        if (d0 >= dend) return fb(4);
        const uint32_t K = std::min(64u, std::max(1u, (dend - d0) / PAR_MIN_SEG)), L = (dend - d0 + K - 1) / K;
        const uint32_t cap = par_cap(M, K);
        SegOut so[64];
        SyncOut sy[64];
        uint32_t used[64];
        for (uint32_t k = 0; k < K; k++) {
            const uint32_t s = d0 + k * L, stop = k + 1 == K ? dend : s + L;
            IBits Bk = B;
            so[k] = decode_seg(Bk, base, s, stop, T, &tok[k * cap], &pos[k * cap], cap);
            sy[k] = sync_lane0(so[k]);
            used[k] = s;                                            // (the start lane k's list was synchronised from)
        }
        // rounds: a lane whose predecessor's end moved synchronises again
        for (int round = 0;; round++) {
            bool any = false;
            for (uint32_t k = 1; k < K; k++) {
                if (sy[k - 1].end == used[k]) continue;
                any = true;
                const uint32_t s = d0 + k * L, stop = k + 1 == K ? dend : s + L;
                IBits Bk = B;
                used[k] = sy[k - 1].end;
                sy[k] = resync(Bk, base, s, used[k], stop, so[k], &tok[k * cap], &pos[k * cap], T, &redo[k * PAR_RCAP]);
                stats[7] += sy[k].r;
            }
            if (!any) break;
            if (round) stats[9]++;
        }
        int kend = -1;
        for (uint32_t k = 0; k < K; k++) {
            if (so[k].ovf) return fb(1);
            if (sy[k].fail) return fb(2);
            if (sy[k].eob >= 0) {
                kend = (int)k;
                break;
            }
        }
        if (kend < 0) return fb(5);
        for (int k = 0; k <= kend; k++) {
            const uint32_t c = k == kend ? (uint32_t)sy[k].eob : sy[k].r + so[k].n - sy[k].i;
            for (uint32_t g = 0; g < c; g++) {
                const uint32_t t = g < sy[k].r ? redo[k * PAR_RCAP + g] : tok[k * cap + sy[k].i + g - sy[k].r];
                if (!(t & TK_MATCH)) {
                    if (w >= M.ulen) return fb(6);
                    o[w++] = (uint8_t)t;
                    continue;
                }
                const uint32_t len = ((t >> 16) & 255u) + 3u, dist = (t & 0x7FFFu) + 1u;
                if (dist > w || w + len > M.ulen) return fb(6);
                for (uint32_t q = 0; q < len; q++, w++) o[w] = o[w - dist];
            }
        }
        p = sy[kend].eobp;
    } while (!bfinal);
    if (w != M.ulen) return fb(6);
    stats[0]++;
    return 0;
}

// inclusive prefix sum over the wave's 64 lanes: DPP row shifts within each row of 16, then the row totals broadcast
// (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3); disabled lanes take `old` = 0
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);    // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);    // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);    // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);    // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);    // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);    // row_bcast:31
    return v;
}

__device__ __forceinline__ uint32_t ring_slot(uint32_t g0, uint32_t x) { return (g0 + x) & (PAR_RING - 1); }

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void k_inflate_par(const uint8_t *__restrict__ comp, const spg_bgzf_member *__restrict__ mem,
                                                    int64_t n, uint8_t *__restrict__ out, uint32_t *__restrict__ status,
                                                    uint32_t *__restrict__ scr_tok, uint16_t *__restrict__ scr_pos,
                                                    uint32_t *__restrict__ scr_redo, uint32_t *__restrict__ n_fallback) {
    __shared__ __align__(16) uint8_t slice[SLICE];
    __shared__ __align__(16) uint8_t ring[PAR_RING];
    const int64_t m = blockIdx.x;
    if (m >= n) return;
    const int lane = threadIdx.x;
    const spg_bgzf_member M = mem[m];
    const uint8_t *const base = comp + (M.coff & ~15ull);
    const uint32_t pay0 = (uint32_t)(M.coff & 15ull) * 8u, dend = pay0 + M.clen * 8u;
    IBits B;
    B.end = comp + M.coff + M.clen + 8;
    uint32_t *const tok0 = scr_tok + par_tok_at(M, (uint64_t)m);                // lane k's list: tok0 + k cap
    uint16_t *const pos0 = scr_pos + par_tok_at(M, (uint64_t)m);
    uint32_t *const redo0 = scr_redo + (uint64_t)m * 64u * PAR_RCAP;            // lane k's redo: redo0 + k RCAP
    const Tabs T = tabs_of(slice);
    const uint32_t ulen = M.ulen;
    const uint64_t gbeg = M.uoff;                                               // the member's first global output byte
    const uint32_t g0 = (uint32_t)(gbeg & (PAR_RING - 1));
    typedef __attribute__((address_space(1))) const uint8_t gu8;
    gu8 *const gout = (gu8 *)(out + gbeg);                                      // the member's output written so far
    uint32_t w = 0, flushed = 0, p = pay0, st = 0;
    bool fixed_built = false;
    int bfinal = 0;

    // global bytes [flushed, upto) of the member from the ring: whole 16-byte aligned chunks of global memory per lane,
    // one aligned 1 KiB block of global memory per pass
    auto flush = [&](uint32_t upto) {
        while (flushed < upto) {
            const uint64_t ga = gbeg + flushed;
            const uint64_t blk = ga & ~1023ull;
            const uint32_t bend = (uint32_t)min((uint64_t)upto, blk + 1024 - gbeg);    // member coordinates
            const uint64_t c = blk + 16ull * (uint64_t)lane;                          // this lane's chunk (global)
            const uint64_t lo = max(c, ga), hi = min(c + 16, gbeg + bend);
            if (lo == c && hi == c + 16) {
                const uint4 v = *reinterpret_cast<const uint4 *>(ring + (uint32_t)(c & (PAR_RING - 1)));
                *reinterpret_cast<uint4 *>(out + c) = v;
            } else {
                for (uint64_t x = lo; x < hi; x++) out[x] = ring[(uint32_t)(x & (PAR_RING - 1))];
            }
            flushed = bend;
        }
    };

    do {
        ib_seek(B, base, p);
        bfinal = (int)B.get(1);
        const uint32_t type = B.get(2);
        if (type == 0 || type == 3) { st = ST_FALLBACK; break; }
        // (every lane reads the same header; the tables are built by the whole wave: build_wave)
        const uint32_t hs = block_tables<true>(B, slice, type, fixed_built);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (hs != 0) { st = ST_FALLBACK; break; }
        const uint32_t d0 = ib_pos(B, base);
        if (d0 >= dend) { st = ST_FALLBACK; break; }
        const uint32_t K = min(64u, max(1u, (dend - d0) / PAR_MIN_SEG)), L = (dend - d0 + K - 1) / K;
        const uint32_t cap = par_cap(M, K);
        const uint32_t s = d0 + (uint32_t)lane * L, stop = (uint32_t)lane + 1 == K ? dend : s + L;
        uint32_t *const tokl = tok0 + (uint64_t)lane * cap;
        uint16_t *const posl = pos0 + (uint64_t)lane * cap;
        SegOut so{};
        SyncOut sy{};
        sy.eob = -1;
        if ((uint32_t)lane < K) {
            so = decode_seg(B, base, s, stop, T, tokl, posl, cap);
            sy = sync_lane0(so);
        }
        __builtin_amdgcn_wave_barrier();
        // sync rounds: a lane whose predecessor's true tokens end elsewhere than where it last synchronised from runs again
        // (the first round: every lane but 0; later rounds only behind a lane that never met its own phase-A tokens)
        uint32_t used = s;
        for (;;) {
            const uint32_t eprev = (uint32_t)__shfl_up((int)sy.end, 1, 64);
            const bool again = lane >= 1 && (uint32_t)lane < K && eprev != used;
            if (!__ballot(again)) break;
            if (again) {
                used = eprev;
                sy = resync(B, base, s, used, stop, so, tokl, posl, T, redo0 + (uint32_t)lane * PAR_RCAP);
            }
        }
        __builtin_amdgcn_wave_barrier();
        const bool bad = (uint32_t)lane < K && (so.ovf || sy.fail);
        const uint64_t badm = __ballot(bad), eobm = __ballot((uint32_t)lane < K && sy.eob >= 0);
        // a lane past the first lane with an end of block decoded another block: only lanes up to it count
        const int kend = eobm ? __builtin_ctzll(eobm) : 64;
        if (kend == 64 || (badm & ((kend == 63 ? ~0ull : (2ull << kend) - 1)))) { st = ST_FALLBACK; break; }
        const uint32_t cnt = lane < kend ? sy.r + so.n - sy.i : lane == kend ? (uint32_t)sy.eob : 0u;
        const uint32_t pnext = (uint32_t)__builtin_amdgcn_readlane((int)sy.eobp, kend);
        // phase-A tokens and redo tokens were written by other lanes: visible to every lane from here
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

        // ---- phase B: the true token lists of lanes 0 .. kend, in order
        for (int k = 0; k <= kend && !st; k++) {
            const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cnt, k);
            const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)sy.r, k);
            const uint32_t i0 = (uint32_t)__builtin_amdgcn_readlane((int)sy.i, k);
            const uint32_t *const tl = tok0 + (int64_t)k * cap + (int64_t)i0 - (int64_t)r;   // (g >= r: tl[g])
            const uint32_t *const rl = redo0 + (uint32_t)k * PAR_RCAP;
            auto load = [&](uint32_t g) -> uint32_t { return g < c ? (g < r ? rl[g] : tl[g]) : 0u; };
            uint32_t t0 = 0, nxt = load((uint32_t)lane);
            while (t0 < c) {
                const bool valid = t0 + (uint32_t)lane < c;
                const uint32_t tk = nxt;
                const bool isM = (tk & TK_MATCH) != 0;
                const uint32_t len = valid ? (isM ? ((tk >> 16) & 255u) + 3u : 1u) : 0u;
                const uint32_t dist = (tk & 0x7FFFu) + 1u;
                const uint32_t incl = wave_incl_scan(len);
                const bool in = valid && incl <= PAR_BATCH;
                const uint64_t inm = __ballot(in);
                const uint32_t nb = (uint32_t)__builtin_popcountll(inm);                 // (a prefix of the lanes)
                const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)nb - 1);
                const uint32_t t1 = t0 + nb;
                nxt = load(t1 + (uint32_t)lane);                                         // the next batch, in flight
                const uint32_t excl = incl - len, o = w + excl;
                if (__ballot(in && isM && dist > o) || w + total > ulen) { st = ST_FALLBACK; break; }
                const uint32_t sb = o - dist;                                            // a match's source start
                // independent: a literal, or a match whose source lies before the batch.  A source byte already written
                // to global memory (before `flushed`) is read from there (L2), any later one from the LDS ring: the ring
                // keeps every byte from w - PAR_RECENT on through the batch, and at most one partial 1 KiB block (<= 1023
                // bytes <= PAR_RECENT) stays unflushed, so each byte is in one of the two (a match's source may straddle
                // `flushed` when PAR_RECENT is less than the longest match + 1 KiB)
                const bool indep = in && (!isM || sb + min(len, dist) <= w);
                // the independent tokens byte-parallel: lane l writes the batch's bytes [l CH, (l + 1) CH), each from
                // the token covering it (found by a search over the lanes, then one step per byte), literal or source
                // byte (read from global memory and from the ring unconditionally, selected after).  (r06ab: a lane per
                // token, short matches copied lane by lane and long ones by the whole wave, took 1.31 M + part of 0.77 M
                // of a member-wave's 2.24 M phase-B clocks: the lanes of short tokens idled while the longest copied.)
                {
                    const uint32_t ex_s = in ? excl : 0xFFFFFFFFu;                       // (past the batch: never found)
                    const uint32_t tkx = tk | (indep ? TK_EOB : 0u);                     // bit 30: independent (no EOB here)
                    const uint32_t CH = (total + 63u) / 64u, P0 = (uint32_t)lane * CH;
                    int t = 0;                                                           // the last token with excl <= P0
#pragma unroll
                    for (int st2 = 32; st2; st2 >>= 1) t += (uint32_t)__shfl((int)ex_s, t + st2, 64) <= P0 ? st2 : 0;
                    uint32_t et = (uint32_t)__shfl((int)ex_s, t, 64), kt = (uint32_t)__shfl((int)tkx, t, 64);
                    for (uint32_t i = 0; i < CH; i++) {
                        const uint32_t P = P0 + i;
                        const uint32_t lt = (kt & TK_MATCH) ? ((kt >> 16) & 255u) + 3u : 1u;
                        t = P >= et + lt ? t + 1 : t;                                    // (at most one token per byte)
                        et = (uint32_t)__shfl((int)ex_s, t & 63, 64);
                        kt = (uint32_t)__shfl((int)tkx, t & 63, 64);
                        const bool isMt = (kt & TK_MATCH) != 0;
                        const uint32_t dt = (kt & 0x7FFFu) + 1u;
                        uint32_t q = P - et;
                        if (isMt && q >= dt) q %= dt;
                        const uint32_t x = w + et - dt + q;                              // (a match's source byte)
                        const bool fg = x < flushed;
                        const uint32_t gv = gout[isMt && fg ? x : 0u], lv = ring[ring_slot(g0, isMt ? x : 0u)];
                        const uint32_t v = isMt ? (fg ? gv : lv) : (kt & 255u);
                        if (P < total && (kt & TK_EOB)) ring[ring_slot(g0, w + P)] = (uint8_t)v;
                    }
                }
                // then, in order, the matches whose source is an earlier token of this batch, one at a time by the whole
                // wave (every earlier token is written by then); byte q of a match is its source's byte q mod dist, so a
                // match never reads its own bytes
                uint64_t dm = __ballot(in && !indep);
                while (dm) {
                    const int j = __builtin_ctzll(dm);
                    dm &= dm - 1;
                    const uint32_t oj = (uint32_t)__builtin_amdgcn_readlane((int)o, j);
                    const uint32_t lj = (uint32_t)__builtin_amdgcn_readlane((int)len, j);
                    const uint32_t dj = (uint32_t)__builtin_amdgcn_readlane((int)dist, j);
                    for (uint32_t q0 = 0; q0 < lj; q0 += 64) {
                        const uint32_t q = q0 + (uint32_t)lane;
                        uint8_t v = 0;
                        const uint32_t x = oj - dj + (dj >= lj ? q : q % dj);
                        if (q < lj) v = x < flushed ? gout[x] : ring[ring_slot(g0, x)];
                        if (q < lj) ring[ring_slot(g0, oj + q)] = v;
                    }
                }
                if (st) break;
                w += total;
                t0 = t1;
                const uint64_t gb = (gbeg + w) & ~1023ull;    // whole global blocks only; the rest stays in the ring
                if (gb > gbeg + flushed) flush((uint32_t)(gb - gbeg));
            }
        }
        if (st) break;
        p = pnext;
    } while (!bfinal);
    if (!st && w != ulen) st = ST_FALLBACK;
    if (!st) flush(ulen);
    if (lane == 0) {
        status[m] = st;
        if (st) atomicAdd(n_fallback, 1u);
    }
}

// CRC-32 (zlib's reflected polynomial) arithmetic: a * b mod P, as zlib's multmodp (branch-free)
__device__ __forceinline__ uint32_t crc_multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll 8
    for (int i = 31; i >= 0; i--) {
        p ^= ((a >> i) & 1u) ? b : 0u;
        b = (b >> 1) ^ ((b & 1u) ? 0xEDB88320u : 0u);
    }
    return p;
}

// x^(8 * 1024 * 2^l) mod P for l = 0..5: the combine's operators for a right part of 2^l whole 1 KiB segments
struct CrcOps {
    uint32_t op[6];
};

// Each member's output checked against the CRC32 in its BGZF trailer (a member the decoder got wrong with the right
// length would otherwise pass): one wave per member, the member cut into 1 KiB segments aligned to its END (lane 63 the
// last 1 KiB, lane 0 the partial first segment), lane j the CRC of its segment through slice-by-4 LDS tables, then a
// 6-level tree over the lanes: crc(A B) = crc(A) x^(8 |B|) + crc(B) mod P (crc32_combine), where every right part B is a
// whole number of segments, so each level multiplies by one constant.  Lanes read their segment with 16-B loads (the
// lanes' starts share one alignment; at most 15 bytes at each end go byte by byte).  (r05: segments from the start,
// dword loads 1 KiB apart across the lanes, and lane 0 folding the 64 partial CRCs in turn with a shift-and-add
// multiply each: 0.49 ms per 10,000x BAM.)
__global__ __launch_bounds__(256) void k_crc32(const uint8_t *__restrict__ comp, const spg_bgzf_member *__restrict__ mem,
                                               int64_t n, const uint8_t *__restrict__ out, uint32_t *__restrict__ status,
                                               CrcOps ops) {
    // slice-by-4 tables: T[k][b] = the CRC register after byte b followed by k zero bytes
    __shared__ uint32_t T[4][256];
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
    // the lane's segment [a, e) of the member, aligned to its end (ulen <= 64 KiB)
    const int64_t e64 = (int64_t)M.ulen - 1024ll * (63 - lane), a64 = e64 - 1024;
    const uint32_t e = (uint32_t)max(e64, (int64_t)0), a = (uint32_t)max(a64, (int64_t)0);
    typedef __attribute__((address_space(1))) const uint8_t gu8;
    gu8 *src = (gu8 *)(const void *)(out + M.uoff);
    uint32_t c = 0xFFFFFFFFu;
    auto byte_step = [&](uint32_t x) { c = T[0][(c ^ x) & 0xFFu] ^ (c >> 8); };
    auto word_step = [&](uint32_t x) {
        c ^= x;
        c = T[3][c & 0xFFu] ^ T[2][(c >> 8) & 0xFFu] ^ T[1][(c >> 16) & 0xFFu] ^ T[0][c >> 24];
    };
    if (a < e) {
        // head bytes up to a 16-B aligned address, then 16-B blocks (eight loads in flight), then the tail bytes
        const uint64_t g0 = M.uoff + a;
        uint32_t b = a, h = (uint32_t)((16 - (g0 & 15)) & 15);
        if (h > e - a) h = e - a;
        for (uint32_t i = 0; i < h; i++) byte_step(src[b + i]);
        b += h;
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) const u32x4 gu128;
        gu128 *q = (gu128 *)(const void *)(out + M.uoff + b);      // (16-B aligned)
        const uint32_t nb = (e - b) / 16;
        uint32_t k = 0;
        for (; k + 8 <= nb; k += 8) {
            u32x4 v[8];
#pragma unroll
            for (int t = 0; t < 8; t++) v[t] = q[k + t];
#pragma unroll
            for (int t = 0; t < 8; t++) {
                word_step(v[t].x);
                word_step(v[t].y);
                word_step(v[t].z);
                word_step(v[t].w);
            }
        }
        for (; k < nb; k++) {
            const u32x4 v = q[k];
            word_step(v.x);
            word_step(v.y);
            word_step(v.z);
            word_step(v.w);
        }
        for (uint32_t i = b + 16 * nb; i < e; i++) byte_step(src[i]);
    }
    uint32_t crc = a < e ? ~c : 0u;                             // (an empty segment: crc32 of the empty string)
    // the tree: at level l, lane j (a multiple of 2^(l+1)) takes the right neighbour part (2^l whole segments)
#pragma unroll
    for (int l = 0; l < 6; l++) {
        const int s = 1 << l;
        const uint32_t r = __shfl_down(crc, s, 64);
        if ((lane & (2 * s - 1)) == 0) crc = crc_multmodp(ops.op[l], crc) ^ r;
    }
    if (lane == 0) {
        const uint8_t *t = comp + M.coff + M.clen;
        const uint32_t want = (uint32_t)t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
        if (crc != want) status[m] = 10;
    }
}

// x^(8 n) mod P on the host (the combine's operators)
static uint32_t host_crc_x8n(uint64_t n) {
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

// scratch of launch_inflate: the fallback counter, per member the parallel kernel's redo tokens (64 KiB), its token lists
// (u32) and their start positions (u16): 2 clen + 2048 each (par_area)
size_t inflate_scratch_bytes(uint64_t comp_bytes, int64_t n) {
    return 256 + 4 * (size_t)n * 64 * PAR_RCAP + 6 * (2 * (size_t)comp_bytes + 2048 * (size_t)n + 64);
}

// k_inflate_par over every member, the lane kernel over the members it left (status ST_FALLBACK), then every member's
// CRC32.  *fallbacks (device u32 at the start of scratch): members the lane kernel inflated.
hipError_t launch_inflate(const uint8_t *comp, uint64_t comp_bytes, const spg_bgzf_member *mem, int64_t n, uint8_t *out,
                          uint32_t *status, void *scratch, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    uint32_t *const cnt = static_cast<uint32_t *>(scratch);
    uint32_t *const redo = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(scratch) + 256);
    uint32_t *const tok = redo + (size_t)n * 64 * PAR_RCAP;
    uint16_t *const pos = reinterpret_cast<uint16_t *>(tok + 2 * (size_t)comp_bytes + 2048 * (size_t)n + 64);
    hipError_t e = hipMemsetAsync(cnt, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    (void)comp_bytes;
    hipLaunchKernelGGL(k_inflate_par, dim3((unsigned)n), dim3(64), 0, st, comp, mem, n, out, status, tok, pos, redo, cnt);
    hipLaunchKernelGGL(k_inflate, dim3((unsigned)((n + INFLATE_MPW - 1) / INFLATE_MPW)), dim3(64),
                       (size_t)INFLATE_MPW * SLICE, st, comp, mem, n, out, status, INFLATE_MPW, 1);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    static const CrcOps ops = [] {
        CrcOps o{};
        for (int l = 0; l < 6; l++) o.op[l] = host_crc_x8n(1024ull << l);
        return o;
    }();
    hipLaunchKernelGGL(k_crc32, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, comp, mem, n, (const uint8_t *)out, status,
                       ops);
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
    std::mutex mu;                // one caller per device at a time (the device's scratch buffers are shared)
    hipStream_t st = nullptr;
    uint8_t *comp = nullptr, *out = nullptr, *scr = nullptr;
    size_t comp_cap = 0, out_cap = 0, mem_bytes = 0, status_bytes = 0, scr_cap = 0;
    spg_bgzf_member *mem = nullptr;
    uint32_t *status = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    int64_t fallbacks = 0;        // the last call's members the parallel kernel left to the lane kernel
};
constexpr int MAX_INF_DEV = 64;
InflateDev g_inf[MAX_INF_DEV];
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

// The parallel inflater's algorithm on the host (k_inflate_par's phase A / sync functions lane after lane, a sequential
// resolve): status 0 or 100 (left to the lane kernel); stats[10] as spg::par_member_host (CPU tests)
int spg_bgzf_inflate_par_check(const uint8_t *comp, size_t comp_bytes, const spg_bgzf_member *members, int64_t n,
                               uint8_t *out, size_t out_bytes, uint32_t *status, uint64_t *stats) {
    if (n < 0 || !stats || (n && (!comp || !members || !out || !status))) return ifail("spg_bgzf_inflate_par_check: bad argument");
    for (int64_t i = 0; i < n; i++) {
        const spg_bgzf_member &m = members[i];
        if (m.coff + m.clen + 8 > comp_bytes || m.uoff + m.ulen > out_bytes || m.ulen > 65536)
            return ifail("spg_bgzf_inflate_par_check: member " + std::to_string(i) + " outside the buffers");
    }
    std::vector<uint64_t> padded((comp_bytes + 64) / 8 + 1, 0);
    std::memcpy(padded.data(), comp, comp_bytes);
    std::vector<uint64_t> slice(spg::SLICE / 8);
    std::vector<uint32_t> tok, redo;
    std::vector<uint16_t> pos;
    for (int k = 0; k < 10; k++) stats[k] = 0;
    for (int64_t i = 0; i < n; i++)
        status[i] = spg::par_member_host(reinterpret_cast<const uint8_t *>(padded.data()), members[i], out,
                                         reinterpret_cast<uint8_t *>(slice.data()), stats, tok, pos, redo);
    return 0;
}

int spg_bgzf_fallbacks(int device, int64_t *n) {
    if (!n || device < 0 || device >= MAX_INF_DEV) return ifail("spg_bgzf_fallbacks: bad argument");
    std::lock_guard<std::mutex> lk(g_inf[device].mu);
    *n = g_inf[device].fallbacks;
    return 0;
}

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
    int prev = 0, nd = 0;
    ICHK(hipGetDevice(&prev));
    ICHK(hipGetDeviceCount(&nd));
    if (device < 0 || device >= nd || device >= MAX_INF_DEV) return ifail("spg_bgzf_inflate: bad device");
    InflateDev &D = g_inf[device];
    std::lock_guard<std::mutex> lk(D.mu);
    struct Restore { int d; ~Restore() { (void)hipSetDevice(d); } } restore{prev};
    ICHK(hipSetDevice(device));
    if (!D.st) {
        ICHK(hipStreamCreateWithFlags(&D.st, hipStreamNonBlocking));
        ICHK(hipEventCreate(&D.ev[0]));
        ICHK(hipEventCreate(&D.ev[1]));
    }
    if (grow(D.comp, D.comp_cap, comp_bytes + 64) || grow(D.out, D.out_cap, out_bytes + 64) ||
        grow(D.mem, D.mem_bytes, (size_t)n * sizeof(spg_bgzf_member)) ||
        grow(D.status, D.status_bytes, (size_t)n * sizeof(uint32_t)) ||
        grow(D.scr, D.scr_cap, spg::inflate_scratch_bytes(comp_bytes, n)))
        return ifail("spg_bgzf_inflate: out of device memory");
    // after the first enqueue every failure drains the stream before returning: the caller's `out` may be the target of a
    // queued copy, and it inflates failed members into it next
    auto drained = [&](int rc) { (void)hipStreamSynchronize(D.st); return rc; };
#define IQ(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return drained(ifail(std::string("spg_bgzf_inflate: ") + #x + ": " + hipGetErrorString(e_))); } while (0)
    IQ(hipMemcpyAsync(D.comp, comp, comp_bytes, hipMemcpyHostToDevice, D.st));
    IQ(hipMemsetAsync(D.comp + comp_bytes, 0, 64, D.st));
    IQ(hipMemcpyAsync(D.mem, members, (size_t)n * sizeof(spg_bgzf_member), hipMemcpyHostToDevice, D.st));
    IQ(hipEventRecord(D.ev[0], D.st));
    IQ(spg::launch_inflate(D.comp, comp_bytes, D.mem, n, D.out, D.status, D.scr, D.st));
    IQ(hipEventRecord(D.ev[1], D.st));
    uint32_t fbk = 0;
    IQ(hipMemcpyAsync(out, D.out, out_bytes, hipMemcpyDeviceToHost, D.st));
    IQ(hipMemcpyAsync(status, D.status, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, D.st));
    IQ(hipMemcpyAsync(&fbk, D.scr, sizeof(uint32_t), hipMemcpyDeviceToHost, D.st));
    IQ(hipStreamSynchronize(D.st));
#undef IQ
    D.fallbacks = fbk;
    if (kernel_ms && hipEventElapsedTime(kernel_ms, D.ev[0], D.ev[1]) != hipSuccess) *kernel_ms = -1.f;   // (timing only)
    // (the scratch only grows; after a BAM above 2 GiB inflated it is given back rather than held in HBM)
    if (D.out_cap > ((size_t)2 << 30)) {
        for (void *p : {(void *)D.comp, (void *)D.out, (void *)D.scr}) (void)hipFree(p);
        D.comp = D.out = D.scr = nullptr;
        D.comp_cap = D.out_cap = D.scr_cap = 0;
    }
    return 0;
}

// The device's inflate scratch freed (it only grows otherwise: one large BAM would keep its size in HBM)
int spg_bgzf_release(int device) {
    if (device < 0 || device >= MAX_INF_DEV) return 0;
    InflateDev &D = g_inf[device];
    std::lock_guard<std::mutex> lk(D.mu);
    if (!D.st) return 0;
    int prev = 0;
    ICHK(hipGetDevice(&prev));
    ICHK(hipSetDevice(device));
    (void)hipStreamSynchronize(D.st);
    for (void *p : {(void *)D.comp, (void *)D.out, (void *)D.mem, (void *)D.status, (void *)D.scr})
        if (p) (void)hipFree(p);
    D.comp = D.out = D.scr = nullptr;
    D.mem = nullptr;
    D.status = nullptr;
    D.comp_cap = D.out_cap = D.mem_bytes = D.status_bytes = D.scr_cap = 0;
    ICHK(hipSetDevice(prev));
    return 0;
}
}
