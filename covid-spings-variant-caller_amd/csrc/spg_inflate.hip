// spg_inflate.hip — BGZF members inflated on the GPU (process_bam's BAM read,
// live_variant_caller.py:54-72, whose host BGZF inflate bounds the end-to-end stream at the GPU box's 16-CPU share).
//
// A BGZF file is a sequence of independent raw-DEFLATE members (RFC 1951) of at most 64 KiB of output each: one
// thread per member decodes its blocks (stored, fixed Huffman, dynamic Huffman) into the member's output range.
// Huffman decoding: a 10-bit primary table per code (entry = symbol | length << 9; codes longer than 10 bits, rare,
// take the canonical bit-serial walk over the code's length counts and sorted symbols), built per block in the
// thread's slice of a scratch buffer; the fixed-Huffman tables are built once into their own slice.  The bit buffer
// is refilled 32 bits at a time (unaligned dword loads; every member is followed by its 8-byte CRC32/ISIZE trailer
// and the uploaded file by 64 bytes of padding, so the refill may read past the payload).  A member's status word
// is 0 when it inflated to exactly its ISIZE bytes; anything else (a corrupt stream) is reported and the caller
// inflates that member on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spings_gpu.h"

namespace spg {

constexpr int IB_LIT = 10;                 // primary table bits, literal/length code
constexpr int IB_DIST = 8;                 // primary table bits, distance code
constexpr int IB_CL = 7;                   // the code-length code (max 7 bits: always primary)
struct HTab {                              // one Huffman code's decode tables (in the thread's scratch slice)
    uint16_t prim[1 << IB_LIT];            // (the distance / code-length codes use the first 2^8 / 2^7 entries)
    uint16_t count[16];                    // codes per length
    uint16_t sym[288];                     // symbols sorted by (length, value)
};
struct IScratch {
    HTab lit, dist, cl;
};

struct IBits {
    const uint8_t *p, *lim;                        // lim: the last dword load that stays inside payload + trailer
    uint64_t buf;
    int n;
    __host__ __device__ __forceinline__ void fill() {
        if (n <= 32) {
            uint32_t w = 0;                        // (past the member: zeros, and the overrun check fails it)
            if (p <= lim) __builtin_memcpy(&w, p, 4);
            buf |= (uint64_t)w << n;
            p += 4;
            n += 32;
        }
    }
    __host__ __device__ __forceinline__ uint32_t peek(int k) const { return (uint32_t)(buf & ((1ull << k) - 1)); }
    __host__ __device__ __forceinline__ void drop(int k) { buf >>= k; n -= k; }
    __host__ __device__ __forceinline__ uint32_t get(int k) {   // k <= 24 after fill()
        fill();
        const uint32_t v = peek(k);
        drop(k);
        return v;
    }
};

// canonical Huffman tables from code lengths (RFC 1951 3.2.2); false: over-subscribed or an incomplete code
// with more than one symbol (a single-symbol distance code is allowed incomplete)
__host__ __device__ bool build(HTab &T, const uint8_t *len, int n, int pb) {
    for (int i = 0; i < 16; i++) T.count[i] = 0;
    for (int s = 0; s < n; s++) T.count[len[s]]++;
    if (T.count[0] == n) {                             // no codes: every lookup fails (only a distance code may)
        for (int i = 0; i < (1 << pb); i++) T.prim[i] = 0;
        return true;
    }
    int left = 1;
    for (int l = 1; l < 16; l++) {
        left <<= 1;
        left -= T.count[l];
        if (left < 0) return false;
    }
    uint16_t offs[16];
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + T.count[l];
    for (int s = 0; s < n; s++)
        if (len[s]) T.sym[offs[len[s]]++] = (uint16_t)s;
    if (left > 0 && n - T.count[0] > 1) return false;   // incomplete with more than one code
    for (int i = 0; i < (1 << pb); i++) T.prim[i] = 0;
    // primary table: each code of length <= pb fills 2^(pb - len) entries at its bit-reversed code
    uint32_t code = 0;
    int k = 0;
    for (int l = 1; l <= 15; l++) {
        for (int c = 0; c < T.count[l]; c++, k++) {
            if (l <= pb) {
                const uint32_t rev = __builtin_bitreverse32(code) >> (32 - l);   // (clang builtin: host and device)
                const uint16_t e = (uint16_t)(T.sym[k] | (l << 9));
                for (uint32_t x = rev; x < (1u << pb); x += 1u << l) T.prim[x] = e;
            }
            code++;
        }
        code <<= 1;
    }
    return true;
}

// one symbol; -1 on an invalid code
__host__ __device__ __forceinline__ int decode(IBits &B, const HTab &T, int pb) {
    B.fill();
    const uint16_t e = T.prim[B.peek(pb)];
    if (e >> 9) {
        B.drop(e >> 9);
        return e & 0x1FF;
    }
    // longer than the primary table (or invalid): canonical walk, one bit at a time (the first bit read is the
    // code's most significant)
    int code = 0, first = 0, index = 0;
    for (int l = 1; l <= 15; l++) {
        code |= (int)B.peek(1);
        B.drop(1);
        const int c = T.count[l];
        if (code - first < c) return T.sym[index + (code - first)];
        index += c;
        first = (first + c) << 1;
        code <<= 1;
    }
    return -1;
}

struct InfTabs {                           // RFC 1951 3.2.5 / 3.2.7
    uint16_t lbase[29];
    uint8_t lext[29];
    uint16_t dbase[30];
    uint8_t dext[30];
    uint8_t clord[19];
};
#define SPG_INF_TABS {{3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258}, \
                      {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0},                      \
                      {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, \
                       6145, 8193, 12289, 16385, 24577},                                                                           \
                      {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13},          \
                      {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15}}
__constant__ InfTabs d_tabs = SPG_INF_TABS;
static const InfTabs h_tabs = SPG_INF_TABS;

__host__ __device__ void fixed_tables(IScratch *fx) {
    uint8_t len[288];
    for (int s = 0; s < 288; s++) len[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
    build(fx->lit, len, 288, IB_LIT);
    for (int s = 0; s < 30; s++) len[s] = 5;
    build(fx->dist, len, 30, IB_DIST);
}

// the fixed Huffman tables (RFC 1951 3.2.6), once
__global__ void k_inflate_fixed(IScratch *fx) {
    if (threadIdx.x == 0 && blockIdx.x == 0) fixed_tables(fx);
}

// one member: status (see k_inflate)
__host__ __device__ uint32_t inflate_member(const uint8_t *comp, const spg_bgzf_member &M, uint8_t *out, IScratch &S,
                                            const IScratch *fx, const InfTabs &TB) {
    uint8_t *o = out + M.uoff;
    const uint32_t ulen = M.ulen;
    const uint8_t *const cend = comp + M.coff + M.clen;
    IBits B{comp + M.coff, cend + 4, 0, 0};
    uint32_t w = 0;                                 // bytes written
    uint32_t st = 0;
    uint8_t lens[288 + 32];
    int bfinal = 0;
    do {
        bfinal = (int)B.get(1);
        const uint32_t type = B.get(2);
        if (type == 0) {                            // stored: to a byte boundary, LEN, NLEN, LEN bytes
            B.drop(B.n & 7);
            const uint32_t ln = B.get(16), nl = B.get(16);
            if ((ln ^ 0xFFFFu) != nl) { st = 2; break; }
            // the whole bytes still in the bit buffer come first
            const uint8_t *src = B.p - (B.n >> 3);
            B.buf = 0;
            B.n = 0;
            if (w + ln > ulen) { st = 7; break; }
            if (src + ln > cend) { st = 8; break; }
            for (uint32_t i = 0; i < ln; i++) o[w + i] = src[i];
            w += ln;
            B.p = src + ln;
            continue;
        }
        const HTab *L, *D;
        if (type == 1) {
            L = &fx->lit;
            D = &fx->dist;
        } else if (type == 2) {
            const int hlit = (int)B.get(5) + 257, hdist = (int)B.get(5) + 1, hclen = (int)B.get(4) + 4;
            uint8_t cl[19];
            for (int i = 0; i < 19; i++) cl[i] = 0;
            for (int i = 0; i < hclen; i++) cl[TB.clord[i]] = (uint8_t)B.get(3);
            if (!build(S.cl, cl, 19, IB_CL)) { st = 3; break; }
            int k = 0;
            while (k < hlit + hdist) {
                const int s = decode(B, S.cl, IB_CL);
                if (s < 0) { st = 3; break; }
                if (s < 16) { lens[k++] = (uint8_t)s; continue; }
                int rep = 0;
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
            if (lens[256] == 0) { st = 3; break; }          // no end-of-block code
            if (!build(S.lit, lens, hlit, IB_LIT) || !build(S.dist, lens + hlit, hdist, IB_DIST)) { st = 4; break; }
            L = &S.lit;
            D = &S.dist;
        } else {
            st = 1;
            break;
        }
        while (true) {                              // the block's codes
            const int s = decode(B, *L, IB_LIT);
            if (s < 0) { st = 5; break; }
            if (s < 256) {
                if (w >= ulen) { st = 7; break; }
                o[w++] = (uint8_t)s;
                continue;
            }
            if (s == 256) break;
            if (s > 285) { st = 5; break; }
            const uint32_t len = TB.lbase[s - 257] + B.get(TB.lext[s - 257]);
            const int ds = decode(B, *D, IB_DIST);
            if (ds < 0 || ds > 29) { st = 5; break; }
            const uint32_t dist = TB.dbase[ds] + B.get(TB.dext[ds]);
            if (dist > w) { st = 6; break; }
            if (w + len > ulen) { st = 7; break; }
            uint8_t *dst = o + w;
            const uint8_t *from = dst - dist;
            if (dist >= 4) {                        // four bytes at a time: each source dword was written before
                uint32_t i = 0;
                for (; i + 4 <= len; i += 4) {
                    uint32_t v;
                    __builtin_memcpy(&v, from + i, 4);
                    __builtin_memcpy(dst + i, &v, 4);
                }
                for (; i < len; i++) dst[i] = from[i];
            } else {                                // a 1-3 byte pattern repeated (runs of one quality value)
                uint32_t pat = 0;
                for (uint32_t j = 0; j < 4; j++) pat |= (uint32_t)from[j % dist] << (8 * j);
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
        if (B.p - (B.n >> 3) > cend) { st = 8; break; }
    } while (!bfinal);
    if (!st && w != ulen) st = 9;
    return st;
}

// status: 0 ok; 1 bad block type; 2 bad stored length; 3 bad code lengths; 4 bad table; 5 bad symbol;
// 6 distance too far back; 7 output overrun; 8 input overrun; 9 wrong size
// mpw members per wave (lanes >= mpw idle): fewer members in lockstep diverge less, and the members spread over more
// SIMDs (8,357 members of a 10,000x BAM are 131 full waves)
__global__ __launch_bounds__(64) void k_inflate(const uint8_t *__restrict__ comp, const spg_bgzf_member *__restrict__ mem,
                                                int64_t n, uint8_t *__restrict__ out, IScratch *__restrict__ scr,
                                                const IScratch *__restrict__ fx, uint32_t *__restrict__ status, int mpw) {
    if ((int)threadIdx.x >= mpw) return;
    const int64_t m = (int64_t)blockIdx.x * mpw + threadIdx.x;
    if (m >= n) return;
    status[m] = inflate_member(comp, mem[m], out, scr[m], fx, d_tabs);
}

}  // namespace spg

// ---------------------------------------------------------------------------------------------------------------
// C-ABI (include/spings_gpu.h): upload, inflate, download; per-device scratch kept between calls (grow-only)
// ---------------------------------------------------------------------------------------------------------------
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

namespace {
struct InflateDev {
    hipStream_t st = nullptr;
    uint8_t *comp = nullptr, *out = nullptr;
    size_t comp_cap = 0, out_cap = 0;
    spg_bgzf_member *mem = nullptr;
    spg::IScratch *scr = nullptr, *fx = nullptr;
    uint32_t *status = nullptr;
    int64_t mem_cap = 0;
    hipEvent_t ev[2] = {nullptr, nullptr};
    float ms = 0.f;
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
    std::vector<spg::IScratch> s(2);
    spg::fixed_tables(&s[1]);
    for (int64_t i = 0; i < n; i++) status[i] = spg::inflate_member(comp, members[i], out, s[0], &s[1], spg::h_tabs);
    return 0;
}

int spg_bgzf_inflate(int device, const uint8_t *comp, size_t comp_bytes, const spg_bgzf_member *members, int64_t n,
                     uint8_t *out, size_t out_bytes, uint32_t *status, float *kernel_ms) {
    if (n < 0 || (n && (!comp || !members || !out || !status))) return ifail("spg_bgzf_inflate: bad argument");
    std::lock_guard<std::mutex> lk(g_inf_mu);
    int nd = 0;
    ICHK(hipGetDeviceCount(&nd));
    if (device < 0 || device >= nd) return ifail("spg_bgzf_inflate: bad device");
    if ((int)g_inf.size() < nd) g_inf.resize((size_t)nd);
    InflateDev &D = g_inf[(size_t)device];
    ICHK(hipSetDevice(device));
    if (!D.st) {
        ICHK(hipStreamCreateWithFlags(&D.st, hipStreamNonBlocking));
        ICHK(hipEventCreate(&D.ev[0]));
        ICHK(hipEventCreate(&D.ev[1]));
        ICHK(hipMalloc(&D.fx, sizeof(spg::IScratch)));
        hipLaunchKernelGGL(spg::k_inflate_fixed, dim3(1), dim3(64), 0, D.st, D.fx);
        ICHK(hipGetLastError());
    }
    for (int64_t i = 0; i < n; i++) {
        const spg_bgzf_member &m = members[i];
        if (m.coff + m.clen + 8 > comp_bytes || m.uoff + m.ulen > out_bytes || m.ulen > 65536)
            return ifail("spg_bgzf_inflate: member " + std::to_string(i) + " outside the buffers");
    }
    if (n == 0) return 0;
    size_t mcap = (size_t)D.mem_cap * sizeof(spg_bgzf_member);
    if (grow(D.comp, D.comp_cap, comp_bytes + 64) || grow(D.out, D.out_cap, out_bytes + 64) ||
        grow(D.mem, mcap, (size_t)n * sizeof(spg_bgzf_member)))
        return ifail("spg_bgzf_inflate: out of device memory");
    if ((int64_t)(mcap / sizeof(spg_bgzf_member)) > D.mem_cap) {
        if (D.scr) (void)hipFree(D.scr);
        if (D.status) (void)hipFree(D.status);
        D.scr = nullptr;
        D.status = nullptr;
        D.mem_cap = (int64_t)(mcap / sizeof(spg_bgzf_member));
        ICHK(hipMalloc(&D.scr, sizeof(spg::IScratch) * (size_t)D.mem_cap));
        ICHK(hipMalloc(&D.status, sizeof(uint32_t) * (size_t)D.mem_cap));
    }
    ICHK(hipMemcpyAsync(D.comp, comp, comp_bytes, hipMemcpyHostToDevice, D.st));
    ICHK(hipMemsetAsync(D.comp + comp_bytes, 0, 64, D.st));
    ICHK(hipMemcpyAsync(D.mem, members, (size_t)n * sizeof(spg_bgzf_member), hipMemcpyHostToDevice, D.st));
    ICHK(hipEventRecord(D.ev[0], D.st));
    static const int mpw = [] { const char *e = getenv("SPG_INFLATE_MPW"); const int v = e ? atoi(e) : 16; return v >= 1 && v <= 64 ? v : 16; }();
    hipLaunchKernelGGL(spg::k_inflate, dim3((unsigned)((n + mpw - 1) / mpw)), dim3(64), 0, D.st, D.comp, D.mem, n, D.out, D.scr,
                       D.fx, D.status, mpw);
    ICHK(hipGetLastError());
    ICHK(hipEventRecord(D.ev[1], D.st));
    ICHK(hipMemcpyAsync(out, D.out, out_bytes, hipMemcpyDeviceToHost, D.st));
    ICHK(hipMemcpyAsync(status, D.status, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, D.st));
    ICHK(hipStreamSynchronize(D.st));
    if (kernel_ms) ICHK(hipEventElapsedTime(kernel_ms, D.ev[0], D.ev[1]));
    return 0;
}
}
