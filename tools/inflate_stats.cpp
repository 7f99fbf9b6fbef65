// Match statistics of a BGZF file's DEFLATE streams (tools only): the device decoder (spg_inflate.hip) run on the
// host with a hook counting match distances / lengths and literals.  Build: hipcc -O2 -I include tools/inflate_stats.cpp
#include <cstdio>
#include <cstdint>
#include <vector>
#include <hip/hip_runtime.h>
static uint64_t g_dist[17], g_len[10], g_matches, g_mbytes;
__host__ __device__ inline void match_hook(uint32_t d, uint32_t l) {
#if !defined(__HIP_DEVICE_COMPILE__)
    int k = 0;
    while ((1u << (k + 1)) <= d) k++;
    g_dist[k]++;
    g_len[l < 16 ? 0 : l < 32 ? 1 : l < 64 ? 2 : l < 128 ? 3 : 4]++;
    g_matches++;
    g_mbytes += l;
#else
    (void)d; (void)l;
#endif
}
#define SPG_INFLATE_MATCH_HOOK(d, l) match_hook(d, l)
static uint64_t g_slow[16];
__host__ __device__ inline void slow_hook(int pb) {
#if !defined(__HIP_DEVICE_COMPILE__)
    g_slow[pb]++;
#else
    (void)pb;
#endif
}
#define SPG_INFLATE_SLOW_HOOK(pb) slow_hook(pb)
#include "../covid-spings-variant-caller_amd/csrc/spg_inflate.hip"

int main(int argc, char **argv) {
    if (argc < 2) return 1;
    FILE *f = fopen(argv[1], "rb");
    std::vector<uint8_t> b;
    uint8_t tmp[1 << 16];
    size_t n;
    while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + n);
    fclose(f);
    std::vector<spg_bgzf_member> mem;
    uint64_t uoff = 0;
    for (size_t q = 0; q + 18 <= b.size();) {
        const uint8_t *h = b.data() + q;
        const size_t xlen = h[10] | (h[11] << 8);
        size_t bsize = 0;
        for (size_t x = 12; x + 4 <= 12 + xlen;) {
            const size_t slen = h[x + 2] | (h[x + 3] << 8);
            if (h[x] == 66 && h[x + 1] == 67 && slen == 2) bsize = (h[x + 4] | (h[x + 5] << 8)) + 1;
            x += 4 + slen;
        }
        const uint32_t ulen = h[bsize - 4] | (h[bsize - 3] << 8) | (h[bsize - 2] << 16) | ((uint32_t)h[bsize - 1] << 24);
        mem.push_back({q + 12 + xlen, (uint32_t)(bsize - xlen - 20), ulen, uoff});
        uoff += ulen;
        q += bsize;
    }
    std::vector<uint8_t> out(uoff + 64);
    std::vector<uint32_t> st(mem.size());
    b.resize(b.size() + 64);
    spg_bgzf_inflate_check(b.data(), b.size() - 64, mem.data(), (int64_t)mem.size(), out.data(), out.size(), st.data());
    size_t bad = 0;
    for (auto s : st) bad += s != 0;
    printf("members %zu (bad %zu), inflated %llu, matches %llu (%.1f per member), match bytes %llu, literal bytes %llu\n",
           mem.size(), bad, (unsigned long long)uoff, (unsigned long long)g_matches, (double)g_matches / mem.size(),
           (unsigned long long)g_mbytes, (unsigned long long)(uoff - g_mbytes));
    uint64_t cum = 0;
    for (int k = 0; k < 16; k++) {
        cum += g_dist[k];
        printf("dist < %6u: %6.2f %% (cum %6.2f %%)\n", 2u << k, 100.0 * g_dist[k] / g_matches, 100.0 * cum / g_matches);
    }
    const char *ln[] = {"<16", "16-31", "32-63", "64-127", ">=128"};
    for (int k = 0; k < 5; k++) printf("len %s: %.2f %%\n", ln[k], 100.0 * g_len[k] / g_matches);
    printf("slow-path decodes: lit/len (10-bit table) %llu, dist (8-bit) %llu, code-length (7-bit) %llu\n",
           (unsigned long long)g_slow[10], (unsigned long long)g_slow[8], (unsigned long long)g_slow[7]);
    return 0;
}
