// membench3.hip — read-bandwidth ceiling of counted mode's access pattern (k_acc_lite_run<2,4>, dev tool).
// B per-BAM batches, each with its own base_code / qual arrays of `bsz` bytes (laid end to end, as the synthetic
// many-BAM batches are); an item = (tile of `tile` bytes, split of the batches); a wave walks its item's batches
// in order, per batch one dependent descriptor load (the batch's base, as the kernel's Hist) and then NCH 1 KiB
// chunks per array (16 B per lane; lanes past the tile's bytes reload its first block), two units in flight,
// no compute.  Swept: splits per tile.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <typename T> using gp = const __attribute__((address_space(1))) T *;

template <int NCH>
__global__ __launch_bounds__(256) void k(const uint8_t *code, const uint8_t *qual, const uint64_t *bases, int B,
                                         uint32_t tile, int n_tiles, int S, uint32_t *out) {
    const int64_t n_items = (int64_t)n_tiles * S;
    uint32_t acc = 0;
    const int lane = threadIdx.x & 63;
    for (int64_t item = blockIdx.x * 4 + (threadIdx.x >> 6); item < n_items; item += (int64_t)gridDim.x * 4) {
        const int g = (int)(item % n_tiles), sp = (int)(item / n_tiles);
        const int kper = (B + S - 1) / S, k0 = sp * kper, k1 = min(B, k0 + kper);
        u32x4 a[NCH], b[NCH], c[NCH], d[NCH];
        auto issue = [&](int kk, u32x4 *x, u32x4 *y) {
            const uint64_t base = ((gp<uint64_t>)bases)[min(kk, B - 1)] + (uint64_t)g * tile;
#pragma unroll
            for (int ch = 0; ch < NCH; ch++) {
                const uint32_t o = 1024u * ch + 16u * lane;
                const uint64_t at = base + (o < tile ? o : 0u);
                x[ch] = __builtin_nontemporal_load((gp<u32x4>)(code + at));
                y[ch] = __builtin_nontemporal_load((gp<u32x4>)(qual + at));
            }
        };
        issue(k0, a, b);
        issue(k0 + 1, c, d);
        for (int kk = k0; kk < k1; kk += 2) {
#pragma unroll
            for (int ch = 0; ch < NCH; ch++) acc ^= a[ch].x ^ a[ch].w ^ b[ch].y ^ b[ch].z;
            issue(kk + 2, a, b);
            if (kk + 1 >= k1) break;
#pragma unroll
            for (int ch = 0; ch < NCH; ch++) acc ^= c[ch].x ^ c[ch].w ^ d[ch].y ^ d[ch].z;
            issue(kk + 3, c, d);
        }
    }
    if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

int main() {
    const int B = 10000, L = 29903;
    const uint64_t bsz = (uint64_t)L * 100;          // 100x per BAM
    const uint64_t tot = (uint64_t)B * bsz + (1 << 20);
    uint8_t *code, *qual; uint64_t *bases; uint32_t *out;
    if (hipMalloc(&code, tot) || hipMalloc(&qual, tot) || hipMalloc(&bases, B * 8) || hipMalloc(&out, 4096)) {
        printf("alloc failed\n"); return 1;
    }
    hipMemset(code, 1, tot); hipMemset(qual, 2, tot);
    std::vector<uint64_t> h(B);
    for (int i = 0; i < B; i++) h[i] = (uint64_t)i * bsz;
    hipMemcpy(bases, h.data(), B * 8, hipMemcpyHostToDevice);
    const uint32_t tile = 3200;                      // 32 columns x 100 entries (LPC 2)
    const int n_tiles = (int)((bsz - 4096) / tile);
    const double bytes = 2.0 * (double)B * n_tiles * tile;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int S : {2, 4, 8, 16}) for (int blocks : {768, 1024, 2048}) {
        std::vector<float> t;
        for (int it = 0; it < 5; it++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL((k<4>), dim3(blocks), dim3(256), 0, 0, code, qual, bases, B, tile, n_tiles, S, out);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            if (it) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("splits %2d blocks %4d  %7.2f ms  %6.0f GB/s (%.1f GB)\n", S, blocks, t[t.size() / 2],
               bytes / (t[t.size() / 2] * 1e-3) / 1e9, bytes / 1e9);
        fflush(stdout);
    }
    return 0;
}
