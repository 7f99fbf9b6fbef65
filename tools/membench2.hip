// membench2.hip — read-bandwidth ceiling of the deep accumulate kernel's access pattern (dev tool).
// Two arrays (code[], qual[]) at equal offsets, each wave streams a contiguous `seg`-byte segment of
// both in 1 KB steps (16 B per lane), 2 steps ahead, like k_acc_seg.  Swept: waves per CU (LDS pad),
// cache policy (aux 0 / nt), segment size, and a dependent descriptor load at wave start (the
// kernel reads its columns' CSR offsets before its first chunk load).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const void *p, uint32_t n) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0, (int)__builtin_amdgcn_readfirstlane(n), 0x00020000);
}

template <int AUX, int PADKB, bool DEP>
__global__ __launch_bounds__(256) void k(const uint8_t *a, const uint8_t *b, const uint64_t *offs, uint32_t seg,
                                         uint32_t nw, uint32_t *out) {
    __shared__ uint8_t pad[PADKB * 1024 + 16];
    if (threadIdx.x == 0) pad[PADKB * 1024] = 1;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= nw) return;
    uint64_t base = (uint64_t)w * seg;
    if (DEP) base = offs[w];                  // dependent start (CSR offsets)
    auto ra = rs(a + base, seg), rb = rs(b + base, seg);
    const uint32_t steps = seg / 1024;
    uint32_t acc = pad[lane];
    u32x4 x0 = __builtin_amdgcn_raw_buffer_load_b128(ra, lane * 16, 0, AUX);
    u32x4 y0 = __builtin_amdgcn_raw_buffer_load_b128(rb, lane * 16, 0, AUX);
    u32x4 x1 = __builtin_amdgcn_raw_buffer_load_b128(ra, 1024 + lane * 16, 0, AUX);
    u32x4 y1 = __builtin_amdgcn_raw_buffer_load_b128(rb, 1024 + lane * 16, 0, AUX);
    u32x4 x2, y2;
    for (uint32_t s = 0; s < steps; s += 3) {
        x2 = __builtin_amdgcn_raw_buffer_load_b128(ra, (s + 2) * 1024 + lane * 16, 0, AUX);
        y2 = __builtin_amdgcn_raw_buffer_load_b128(rb, (s + 2) * 1024 + lane * 16, 0, AUX);
        acc ^= x0.x ^ x0.y ^ x0.z ^ x0.w ^ y0.x ^ y0.y ^ y0.z ^ y0.w;
        x0 = __builtin_amdgcn_raw_buffer_load_b128(ra, (s + 3) * 1024 + lane * 16, 0, AUX);
        y0 = __builtin_amdgcn_raw_buffer_load_b128(rb, (s + 3) * 1024 + lane * 16, 0, AUX);
        acc ^= x1.x ^ x1.y ^ x1.z ^ x1.w ^ y1.x ^ y1.y ^ y1.z ^ y1.w;
        x1 = __builtin_amdgcn_raw_buffer_load_b128(ra, (s + 4) * 1024 + lane * 16, 0, AUX);
        y1 = __builtin_amdgcn_raw_buffer_load_b128(rb, (s + 4) * 1024 + lane * 16, 0, AUX);
        acc ^= x2.x ^ x2.y ^ x2.z ^ x2.w ^ y2.x ^ y2.y ^ y2.z ^ y2.w;
    }
    if (acc == 0x12345678u) out[w] = acc;
}

template <int AUX, int PADKB, bool DEP>
static float run(const uint8_t *a, const uint8_t *b, const uint64_t *offs, uint32_t seg, uint32_t nw, uint32_t *out) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    std::vector<float> t;
    for (int it = 0; it < 14; it++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<AUX, PADKB, DEP>), dim3((nw + 3) / 4), dim3(256), 0, 0, a, b, offs, seg, nw, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (it >= 4) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2] * 1e3f;
}

int main() {
    const size_t half = 299u << 20;          // ~ the 10,000x batch: 2 x 299 MiB
    uint8_t *a, *b;
    uint32_t *out;
    uint64_t *offs;
    hipMalloc(&a, half + (1 << 20));
    hipMalloc(&b, half + (1 << 20));
    hipMalloc(&out, 1 << 22);
    hipMalloc(&offs, 1 << 22);
    hipMemset(a, 1, half + (1 << 20));
    hipMemset(b, 2, half + (1 << 20));
    for (uint32_t seg : {20u << 10, 40u << 10, 80u << 10}) {
        const uint32_t nw = (uint32_t)(half / seg);
        std::vector<uint64_t> h(nw);
        for (uint32_t i = 0; i < nw; i++) h[i] = (uint64_t)i * seg;
        hipMemcpy(offs, h.data(), nw * 8, hipMemcpyHostToDevice);
        const double B = 2.0 * nw * seg;
        struct R { const char *name; float us; };
        std::vector<R> rs_;
        // LDS pads: 38 KB/block -> 4 blocks/CU (16 waves), 52 KB -> 3 (12 waves, the kernel's), 76 KB -> 2 (8)
        rs_.push_back({"12 waves/CU aux0      ", run<0, 52, false>(a, b, offs, seg, nw, out)});
        rs_.push_back({"12 waves/CU nt        ", run<2, 52, false>(a, b, offs, seg, nw, out)});
        rs_.push_back({"12 waves/CU nt dep    ", run<2, 52, true>(a, b, offs, seg, nw, out)});
        rs_.push_back({"16 waves/CU nt        ", run<2, 38, false>(a, b, offs, seg, nw, out)});
        rs_.push_back({" 8 waves/CU nt        ", run<2, 76, false>(a, b, offs, seg, nw, out)});
        rs_.push_back({"32 waves/CU nt        ", run<2, 0, false>(a, b, offs, seg, nw, out)});
        rs_.push_back({"32 waves/CU aux0      ", run<0, 0, false>(a, b, offs, seg, nw, out)});
        for (auto &r : rs_)
            printf("seg %3u KiB  %s  %7.1f us  %6.0f GB/s\n", seg >> 10, r.name, r.us, B / (r.us * 1e-6) / 1e9);
    }
    return 0;
}
