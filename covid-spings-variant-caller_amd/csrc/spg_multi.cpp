// spg_multi.cpp — one process, N devices (SURVEY §8 b/e): the path shards by coordinate range with no data-path
// collective; each device's context owns a contiguous range of positions, and the compact call tables come back
// to device 0 with one RCCL gather (ncclGather over xGMI).  This is the C-ABI form of shard.py's ShardedEngine
// (torch.distributed), for a host without torch (INTEGRATION.md Option B).
//
// The cuts are taken on the first batch of a sample (equal entries per device, from its CSR prefix sum; the
// positions before / after it go to the first / last device) and kept until reset, so every position's record
// lives on one device.  Each later batch is sliced at the cuts; a device whose slice is empty gets a batch of
// one empty column (no entries: no record changes), so every device numbers the batches alike and first visits
// (live_variant_caller.py:77-85) and the memory order stay global.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "spings_gpu.h"

struct spg_multi {
    int n = 0;
    int64_t n_pos = 0;
    std::vector<int> dev;
    std::vector<spg_ctx *> ctx;
    std::vector<ncclComm_t> comm;
    std::vector<int64_t> cut;              // n + 1 position cuts (empty until the sample's first batch)
    std::vector<void *> send;              // per device: [u64 count][cap x spg_candidate]
    void *recv = nullptr;                  // device 0: n x send size
    int64_t cap = 0;
    std::string err;
};

static thread_local std::string g_merr;
static int mfail(const std::string &m) {
    g_merr = m;
    return -1;
}
#define MHIP(x)                                                                                   \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) return mfail(std::string(#x) + ": " + hipGetErrorString(e_));       \
    } while (0)
#define MCCL(x)                                                                                   \
    do {                                                                                          \
        ncclResult_t r_ = (x);                                                                    \
        if (r_ != ncclSuccess) return mfail(std::string(#x) + ": " + ncclGetErrorString(r_));     \
    } while (0)
#define MCTX(x)                                                                                   \
    do {                                                                                          \
        if ((x) != 0) return mfail(std::string(#x) + ": " + spg_last_error());                    \
    } while (0)

extern "C" {

const char *spg_multi_last_error(void) { return g_merr.c_str(); }

int spg_multi_destroy(spg_multi *m) {
    if (!m) return 0;
    for (size_t i = 0; i < m->ctx.size(); i++) {
        if (m->send.size() > i && m->send[i]) { (void)hipSetDevice(m->dev[i]); (void)hipFree(m->send[i]); }
        if (m->ctx[i]) spg_destroy(m->ctx[i]);
    }
    if (m->recv) { (void)hipSetDevice(m->dev[0]); (void)hipFree(m->recv); }
    for (ncclComm_t c : m->comm)
        if (c) (void)ncclCommDestroy(c);
    delete m;
    return 0;
}

int spg_multi_create(const int *devices, int n, int64_t n_pos, const spg_params *p, spg_multi **out) {
    if (!devices || n < 1 || n > 64 || !p || !out || n_pos <= 0) return mfail("spg_multi_create: bad argument");
    spg_multi *m = new spg_multi();
    m->n = n;
    m->n_pos = n_pos;
    m->dev.assign(devices, devices + n);
    m->ctx.assign(n, nullptr);
    m->send.assign(n, nullptr);
    for (int i = 0; i < n; i++)
        if (spg_create(devices[i], n_pos, p, &m->ctx[i]) != 0) {
            const std::string e = spg_last_error();
            spg_multi_destroy(m);
            return mfail("spg_multi_create: device " + std::to_string(devices[i]) + ": " + e);
        }
    m->comm.assign(n, nullptr);
    if (ncclCommInitAll(m->comm.data(), n, devices) != ncclSuccess) {
        spg_multi_destroy(m);
        return mfail("spg_multi_create: ncclCommInitAll failed");
    }
    *out = m;
    return 0;
}

int spg_multi_set_eps_lut(spg_multi *m, const double lut[256]) {
    if (!m) return mfail("spg_multi_set_eps_lut: null");
    for (spg_ctx *c : m->ctx) MCTX(spg_set_eps_lut(c, lut));
    return 0;
}

int spg_multi_set_reference(spg_multi *m, const char *seq, int64_t len) {
    if (!m) return mfail("spg_multi_set_reference: null");
    for (spg_ctx *c : m->ctx) MCTX(spg_set_reference(c, seq, len));
    return 0;
}

int spg_multi_reset(spg_multi *m) {
    if (!m) return mfail("spg_multi_reset: null");
    for (spg_ctx *c : m->ctx) MCTX(spg_reset(c));
    m->cut.clear();
    return 0;
}

int spg_multi_partition(spg_multi *m, int64_t *cuts) {
    if (!m || !cuts) return mfail("spg_multi_partition: null");
    if (m->cut.empty()) return mfail("spg_multi_partition: no batch accumulated since reset");
    std::copy(m->cut.begin(), m->cut.end(), cuts);
    return 0;
}

// One host CSR batch (spg_accumulate's arguments; host memory only), sliced at the cuts.
int spg_multi_accumulate(spg_multi *m, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                         const uint8_t *base_code, const uint8_t *qual, uint64_t n_entries, uint32_t flags) {
    if (!m || !offsets || n_cols < 0) return mfail("spg_multi_accumulate: bad argument");
    if (flags & (SPG_IN_DEVICE | SPG_IN_BORROW)) return mfail("spg_multi_accumulate: host batches only");
    if (offsets[n_cols] != n_entries || offsets[0] != 0)
        return mfail("spg_multi_accumulate: offsets[0] must be 0 and offsets[n_cols] == n_entries");
    if (m->cut.empty()) {
        // equal entries per device on this batch's prefix sum
        m->cut.assign(m->n + 1, 0);
        m->cut[m->n] = m->n_pos;
        for (int d = 1; d < m->n; d++) {
            const uint64_t target = n_entries * (uint64_t)d / (uint64_t)m->n;
            const int64_t c = std::lower_bound(offsets, offsets + n_cols + 1, target) - offsets;
            m->cut[d] = std::max(m->cut[d - 1], std::min(m->n_pos, pos_begin + c));
        }
    }
    std::vector<uint64_t> sub;
    for (int d = 0; d < m->n; d++) {
        const int64_t lo = std::max(pos_begin, m->cut[d]), hi = std::min(pos_begin + n_cols, m->cut[d + 1]);
        if (hi <= lo) {
            static const uint64_t none[2] = {0, 0};
            MCTX(spg_accumulate_ex(m->ctx[d], std::min(m->cut[d], m->n_pos - 1), 1, none, nullptr, nullptr, 0, 0));
            continue;
        }
        const int64_t a = lo - pos_begin, b = hi - pos_begin;
        sub.resize((size_t)(b - a + 1));
        for (int64_t i = a; i <= b; i++) sub[(size_t)(i - a)] = offsets[i] - offsets[a];
        const uint64_t e = offsets[b] - offsets[a];
        MCTX(spg_accumulate_ex(m->ctx[d], lo, b - a, sub.data(), base_code + offsets[a], qual + offsets[a], e,
                               flags & SPG_IN_TRUSTED));
    }
    return 0;
}

int spg_multi_finalize(spg_multi *m) {
    if (!m) return mfail("spg_multi_finalize: null");
    for (spg_ctx *c : m->ctx) MCTX(spg_finalize(c));
    return 0;
}

// The merged call table: every device's table packed on its own stream, one ncclGather to device 0, then
// in memory order — (first_batch, pos, allele rank), as the shim orders one context's table.
int spg_multi_get_candidates(spg_multi *m, spg_candidate *out, int64_t cap, int64_t *n_out) {
    if (!m || !n_out) return mfail("spg_multi_get_candidates: null");
    int64_t need = 1;
    for (spg_ctx *c : m->ctx) {
        int64_t nc = 0, nd = 0;
        MCTX(spg_count(c, &nc, &nd));
        need = std::max(need, nc);
    }
    const size_t rec = sizeof(spg_candidate), per = 8 + rec * (size_t)need;
    if (need > m->cap) {                 // buffers sized for the largest table (KBs at these call rates)
        for (int d = 0; d < m->n; d++) {
            MHIP(hipSetDevice(m->dev[d]));
            if (m->send[d]) MHIP(hipFree(m->send[d]));
            MHIP(hipMalloc(&m->send[d], per));
        }
        MHIP(hipSetDevice(m->dev[0]));
        if (m->recv) MHIP(hipFree(m->recv));
        MHIP(hipMalloc(&m->recv, per * (size_t)m->n));
        m->cap = need;
    }
    const size_t per_cap = 8 + rec * (size_t)m->cap;
    std::vector<hipStream_t> st((size_t)m->n);
    for (int d = 0; d < m->n; d++) {
        MCTX(spg_stream(m->ctx[d], (void **)&st[(size_t)d]));
        MCTX(spg_copy_candidates_device(m->ctx[d], m->send[d], m->cap));
    }
    MCCL(ncclGroupStart());
    for (int d = 0; d < m->n; d++) {
        MHIP(hipSetDevice(m->dev[d]));
        MCCL(ncclGather(m->send[d], d == 0 ? m->recv : nullptr, per_cap, ncclUint8, 0, m->comm[d], st[(size_t)d]));
    }
    MCCL(ncclGroupEnd());
    std::vector<uint8_t> h(per_cap * (size_t)m->n);
    MHIP(hipSetDevice(m->dev[0]));
    MHIP(hipMemcpyAsync(h.data(), m->recv, h.size(), hipMemcpyDeviceToHost, st[0]));
    MHIP(hipStreamSynchronize(st[0]));
    std::vector<spg_candidate> all;
    for (int d = 0; d < m->n; d++) {
        uint64_t k = 0;
        memcpy(&k, h.data() + per_cap * (size_t)d, 8);
        const spg_candidate *r = reinterpret_cast<const spg_candidate *>(h.data() + per_cap * (size_t)d + 8);
        all.insert(all.end(), r, r + k);
    }
    std::stable_sort(all.begin(), all.end(), [](const spg_candidate &x, const spg_candidate &y) {
        if (x.first_batch != y.first_batch) return x.first_batch < y.first_batch;
        if (x.pos != y.pos) return x.pos < y.pos;
        return x.rank < y.rank;
    });
    *n_out = (int64_t)all.size();
    if (*n_out > cap) return mfail("spg_multi_get_candidates: output capacity too small");
    if (!all.empty() && out) memcpy(out, all.data(), rec * all.size());
    return 0;
}

int spg_multi_context(spg_multi *m, int i, spg_ctx **ctx) {
    if (!m || !ctx || i < 0 || i >= m->n) return mfail("spg_multi_context: bad argument");
    *ctx = m->ctx[(size_t)i];
    return 0;
}

}  // extern "C"
