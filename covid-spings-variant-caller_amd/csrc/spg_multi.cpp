// spg_multi.cpp — one process, N devices (SURVEY §8 b/e): the path shards by coordinate range with no data-path
// collective; each device's context owns a contiguous range of positions [cut[d], cut[d+1]) (its own coordinate
// space: Acc records, counted totals and reference slice only for that range), and the compact call tables come
// back to device 0 with one RCCL gather (ncclGather over xGMI).  The C-ABI form of shard.py's ShardedEngine
// (torch.distributed), for a host without torch (INTEGRATION.md Option B).
//
// Cuts: equal entries per device over a per-bucket entry histogram (spg_multi_plan_cuts).  A sample's cuts are
// planned at its first batch — from the previous sample's cumulative histogram when there is one (amplicon
// panels repeat their shape), else from that batch — and re-planned when the cumulative load drifts (an
// amplicon-shaped or partial first BAM): the history is re-sliced at the new cuts and re-accumulated (bounded by
// `rebalance_max_batches`).  Every device takes every batch, so batch numbers, first visits
// (live_variant_caller.py:77-85) and the memory order stay global; a device whose slice of a batch is empty
// gets one empty column (no entries: no record changes).
//
// Host batches, BAM records plans (spg_accumulate_records: the device pileup shards — each device gets the
// reads overlapping its range and their record bytes) and their sliced offsets are staged in per-device pinned
// rings, so the N devices' copies and kernels overlap.  Devices listed twice (one GPU standing in for several)
// share it without RCCL: the tables are gathered with device copies instead.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "spings_gpu.h"

namespace {

constexpr int NSTAGE = 4;                  // pinned staging sets per device (ring)

struct Stage {
    void *p = nullptr;
    size_t cap = 0;
    uint64_t ticket = 0;                   // the device context's input ticket of the copy that read it
};

struct MBatch {
    int64_t pos_begin, n_cols;
};

// One call table in flight (spg_multi_get_candidates_async): every device's table copied on its stream
// (spg_copy_table_device), gathered, and copied into this slot's pinned host buffer; `ev` marks the copies done.
struct TSlot {
    uint64_t ticket = 0;                   // 0: free
    bool collected = false;                // the host bytes were parsed (merged / bad)
    bool bad = false;                      // a table outgrew its copy or carried an error word
    std::vector<hipEvent_t> ev;            // per device (RCCL: [0] only, after the gather's copy)
    std::vector<int> ev_used;
    std::vector<int64_t> cut;              // the device ranges the tables were made over
    std::vector<spg_candidate> merged;     // memory order
};

constexpr size_t TABLE_HEAD = 16;          // spg_copy_table_device's header

}  // namespace

struct spg_multi {
    int n = 0;
    int64_t n_pos = 0;
    spg_params p{};
    std::vector<int> dev;
    std::vector<spg_ctx *> ctx;            // per device, over [cut[d], cut[d+1]) (created when a sample is planned)
    std::vector<ncclComm_t> comm;
    bool rccl = false;                     // distinct devices: RCCL gather (else device copies)
    std::vector<int64_t> cut;              // n + 1 (empty: not planned since reset)
    std::vector<int64_t> ctx_cut;          // the cuts the live contexts were created for
    double lut[256];
    bool lut_set = false;
    std::string ref;                       // padded with 'N' to n_pos (a device range past a shorter contig's end
    int64_t ref_len = 0;                   // still holds the one-column batch that keeps batch numbers global)
    bool ref_set = false;
    int64_t bucket = 1024;                 // positions per histogram bucket
    std::vector<uint64_t> w_cur, w_prev;   // entries per bucket: this sample, the previous sample
    std::vector<MBatch> batches;           // this sample's batches (extent), for re-plans
    std::vector<std::vector<Stage>> stage; // [device][NSTAGE]
    int stage_i = 0;
    double rebalance_ratio = 1.25;         // max device load / mean that triggers a re-plan
    int64_t rebalance_max_batches = 256;   // ... while the sample holds at most this many batches
    int64_t n_replans = 0;
    std::vector<void *> send;              // per table slot and device (slot * n + d): [16-B table header][cap records]
    void *recv[2] = {nullptr, nullptr};    // per table slot, on devices[0]: n x send size
    std::vector<hipStream_t> tstream;      // per device: the table's gather and copy down (off the context's stream)
    std::vector<hipEvent_t> tev;           // per device: the table copied out of the context's buffers
    int64_t cap = 0;                       // records per device table copy (grown from the tables seen)
    uint8_t *host[2] = {nullptr, nullptr}; // pinned: n x send size per table slot
    TSlot slot[2];
    uint64_t tseq = 0;                     // tickets handed out
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

// Entries per bucket of one CSR batch over reference positions [pos_begin, pos_begin + n_cols).
static void add_weights(std::vector<uint64_t> &w, int64_t bucket, int64_t pos_begin, int64_t n_cols, const uint64_t *off) {
    for (int64_t i = 0; i < n_cols;) {
        const int64_t b = (pos_begin + i) / bucket;
        const int64_t end = std::min<int64_t>(n_cols, (b + 1) * bucket - pos_begin);
        w[(size_t)b] += off[end] - off[i];
        i = end;
    }
}

extern "C" {

const char *spg_multi_last_error(void) { return g_merr.c_str(); }

// Cuts with equal entries per device over a bucket histogram (host only: no GPU needed).  cuts[0] = 0,
// cuts[n] = n_pos, every range non-empty, cut d at the first bucket boundary where the cumulative weight reaches
// d / n of the total; no weight at all: equal lengths.
int spg_multi_plan_cuts(const uint64_t *w, int64_t n_buckets, int64_t bucket, int64_t n_pos, int n, int64_t *cuts) {
    if (!cuts || n < 1 || n_pos < n || bucket < 1 || n_buckets < 0 || (n_buckets && !w))
        return mfail("spg_multi_plan_cuts: bad argument");
    long double tot = 0;
    for (int64_t b = 0; b < n_buckets; b++) tot += (long double)w[b];
    cuts[0] = 0;
    cuts[n] = n_pos;
    if (tot <= 0) {
        for (int d = 1; d < n; d++) cuts[d] = n_pos * d / n;
    } else {
        long double acc = 0;
        int64_t b = 0;
        for (int d = 1; d < n; d++) {
            const long double target = tot * d / n;
            while (b < n_buckets && acc + (long double)w[b] < target) acc += (long double)w[b++];
            // the bucket that crosses the target: cut inside it, proportionally (a bucket may hold one amplicon)
            int64_t c;
            if (b < n_buckets && w[b] > 0) {
                const long double f = (target - acc) / (long double)w[b];
                c = b * bucket + (int64_t)std::llround((double)(f * (long double)bucket));
            } else {
                c = b * bucket;
            }
            cuts[d] = c;
        }
    }
    for (int d = 1; d < n; d++)          // clamp: non-empty ranges, ascending
        cuts[d] = std::min(std::max(cuts[d], cuts[d - 1] + 1), n_pos - (n - d));
    return 0;
}

int spg_multi_destroy(spg_multi *m) {
    if (!m) return 0;
    for (TSlot &t : m->slot) {             // (copies in flight into the pinned buffers end first)
        for (size_t d = 0; d < t.ev.size(); d++)
            if (t.ev[d]) {
                if (t.ev_used[d]) (void)hipEventSynchronize(t.ev[d]);
                (void)hipEventDestroy(t.ev[d]);
            }
    }
    for (uint8_t *h : m->host)
        if (h) (void)hipHostFree(h);
    for (size_t i = 0; i < m->send.size(); i++)
        if (m->send[i]) { (void)hipSetDevice(m->dev[i % m->dev.size()]); (void)hipFree(m->send[i]); }
    for (size_t i = 0; i < m->tstream.size(); i++) {
        (void)hipSetDevice(m->dev[i]);
        if (m->tstream[i]) { (void)hipStreamSynchronize(m->tstream[i]); (void)hipStreamDestroy(m->tstream[i]); }
        if (m->tev[i]) (void)hipEventDestroy(m->tev[i]);
    }
    for (size_t i = 0; i < m->ctx.size(); i++)
        if (m->ctx[i]) spg_destroy(m->ctx[i]);
    for (auto &ring : m->stage)
        for (auto &s : ring)
            if (s.p) (void)hipHostFree(s.p);
    for (void *r : m->recv)
        if (r) { (void)hipSetDevice(m->dev[0]); (void)hipFree(r); }
    for (ncclComm_t c : m->comm)
        if (c) (void)ncclCommDestroy(c);
    delete m;
    return 0;
}

int spg_multi_create(const int *devices, int n, int64_t n_pos, const spg_params *p, spg_multi **out) {
    if (!devices || n < 1 || n > 64 || !p || !out || n_pos < n) return mfail("spg_multi_create: bad argument");
    spg_multi *m = new spg_multi();
    m->n = n;
    m->n_pos = n_pos;
    m->p = *p;
    m->dev.assign(devices, devices + n);
    m->ctx.assign(n, nullptr);
    m->send.assign(2 * (size_t)n, nullptr);
    m->stage.assign(n, std::vector<Stage>(NSTAGE));
    m->bucket = std::max<int64_t>(64, (n_pos + 65535) / 65536);
    m->w_cur.assign((size_t)((n_pos + m->bucket - 1) / m->bucket), 0);
    std::vector<int> sorted(devices, devices + n);
    std::sort(sorted.begin(), sorted.end());
    m->rccl = n > 1 && std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (m->rccl) {
        m->comm.assign(n, nullptr);
        if (ncclCommInitAll(m->comm.data(), n, devices) != ncclSuccess) {
            spg_multi_destroy(m);
            return mfail("spg_multi_create: ncclCommInitAll failed");
        }
    }
    *out = m;
    return 0;
}

int spg_multi_set_eps_lut(spg_multi *m, const double lut[256]) {
    if (!m || !lut) return mfail("spg_multi_set_eps_lut: null");
    memcpy(m->lut, lut, sizeof m->lut);
    m->lut_set = true;
    for (int d = 0; d < m->n; d++)
        if (m->ctx[d]) MCTX(spg_set_eps_lut(m->ctx[d], lut));
    return 0;
}

int spg_multi_set_reference(spg_multi *m, const char *seq, int64_t len) {
    if (!m || !seq || len < 0) return mfail("spg_multi_set_reference: bad argument");
    // a contig shorter than the positions: every device's range still lies inside the (padded) sequence, so the
    // one-column batch of an empty slice is accepted everywhere; batches past the contig's end are refused here
    m->ref.assign(seq, (size_t)std::min(len, m->n_pos));
    if (len < m->n_pos) m->ref.append((size_t)(m->n_pos - len), 'N');
    m->ref_len = std::min(len, m->n_pos);
    m->ref_set = true;
    for (int d = 0; d < m->n; d++)
        if (m->ctx[d]) MCTX(spg_set_reference(m->ctx[d], seq + m->ctx_cut[d], m->ctx_cut[d + 1] - m->ctx_cut[d]));
    return 0;
}

static int collect_all(spg_multi *m);

// (Re)create the device contexts over the current cuts (kept when the cuts did not change: a reset then suffices).
static int build_contexts(spg_multi *m) {
    if (!m->ctx_cut.empty() && m->ctx_cut == m->cut) {
        for (int d = 0; d < m->n; d++) MCTX(spg_reset(m->ctx[d]));
        return 0;
    }
    if (int rc = collect_all(m)) return rc;    // (tables in flight were enqueued on the streams destroyed here)
    for (int d = 0; d < m->n; d++) {
        if (m->ctx[d]) spg_destroy(m->ctx[d]);
        m->ctx[d] = nullptr;
        for (auto &s : m->stage[(size_t)d]) s.ticket = 0;      // tickets are per context
    }
    for (int d = 0; d < m->n; d++) {
        const int64_t lo = m->cut[d], hi = m->cut[d + 1];
        if (spg_create(m->dev[d], hi - lo, &m->p, &m->ctx[d]) != 0)
            return mfail("spg_multi: device " + std::to_string(m->dev[d]) + ": " + spg_last_error());
        if (m->lut_set) MCTX(spg_set_eps_lut(m->ctx[d], m->lut));
        if (m->ref_set) MCTX(spg_set_reference(m->ctx[d], m->ref.data() + lo, hi - lo));
    }
    m->ctx_cut = m->cut;
    return 0;
}

int spg_multi_reset(spg_multi *m) {
    if (!m) return mfail("spg_multi_reset: null");
    for (spg_ctx *c : m->ctx)
        if (c) MCTX(spg_reset(c));
    // the next sample is planned from this one's histogram (when it had entries)
    uint64_t tot = 0;
    for (uint64_t x : m->w_cur) tot += x;
    if (tot) m->w_prev = m->w_cur;
    std::fill(m->w_cur.begin(), m->w_cur.end(), 0);
    m->cut.clear();
    m->batches.clear();
    return 0;
}

int spg_multi_partition(spg_multi *m, int64_t *cuts) {
    if (!m || !cuts) return mfail("spg_multi_partition: null");
    if (m->cut.empty()) return mfail("spg_multi_partition: no batch accumulated since reset");
    std::copy(m->cut.begin(), m->cut.end(), cuts);
    return 0;
}

int spg_multi_set_rebalance(spg_multi *m, double ratio, int64_t max_batches) {
    if (!m || !(ratio >= 1.0) || max_batches < 0) return mfail("spg_multi_set_rebalance: bad argument");
    m->rebalance_ratio = ratio;
    m->rebalance_max_batches = max_batches;
    return 0;
}

int spg_multi_replans(spg_multi *m, int64_t *n) {
    if (!m || !n) return mfail("spg_multi_replans: null");
    *n = m->n_replans;
    return 0;
}

}  // extern "C"

// A pinned staging buffer of device d for the next batch (ring of NSTAGE; reused after its copy has landed).
static int stage_buf(spg_multi *m, int d, size_t bytes, Stage **out) {
    Stage &s = m->stage[(size_t)d][(size_t)m->stage_i];
    if (s.ticket) MCTX(spg_wait_ticket(m->ctx[d], s.ticket));
    if (s.cap < bytes) {
        if (s.p) MHIP(hipHostFree(s.p));
        s.p = nullptr;
        s.cap = 0;
        const size_t cap = std::max<size_t>(bytes + bytes / 8, 4096);
        MHIP(hipHostMalloc(&s.p, cap, hipHostMallocDefault));
        s.cap = cap;
    }
    *out = &s;
    return 0;
}

static int plan_sample(spg_multi *m, int64_t pos_begin, int64_t n_cols, const uint64_t *off) {
    std::vector<uint64_t> w;
    uint64_t prev = 0;
    for (uint64_t x : m->w_prev) prev += x;
    if (prev) {
        w = m->w_prev;
    } else {
        w.assign(m->w_cur.size(), 0);
        add_weights(w, m->bucket, pos_begin, n_cols, off);
    }
    m->cut.assign((size_t)m->n + 1, 0);
    if (spg_multi_plan_cuts(w.data(), (int64_t)w.size(), m->bucket, m->n_pos, m->n, m->cut.data()) != 0) return -1;
    return build_contexts(m);
}

static int accumulate_host(spg_multi *m, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                           const uint8_t *base_code, const uint8_t *qual, uint32_t flags);

// The sample's history re-sliced at new cuts: each batch reassembled from the devices' slices (their history copies),
// the contexts rebuilt over the new ranges, and every batch accumulated again in order.
static int replan(spg_multi *m, const std::vector<int64_t> &cuts) {
    std::vector<std::vector<uint64_t>> offs(m->batches.size());
    std::vector<std::vector<uint8_t>> codes(m->batches.size()), quals(m->batches.size());
    for (size_t i = 0; i < m->batches.size(); i++) {
        const MBatch &b = m->batches[i];
        std::vector<uint64_t> lens((size_t)b.n_cols, 0);
        std::vector<uint8_t> &cv = codes[i], &qv = quals[i];
        for (int d = 0; d < m->n; d++) {
            int64_t pb = 0, nc = 0;
            uint64_t ne = 0;
            MCTX(spg_history_info(m->ctx[d], (int64_t)i, &pb, &nc, &ne));
            if (ne == 0) continue;                         // an empty slice (or the one-column placeholder)
            std::vector<uint64_t> o((size_t)nc + 1);
            const size_t at = cv.size();
            cv.resize(at + ne);
            qv.resize(at + ne);
            MCTX(spg_history_copy(m->ctx[d], (int64_t)i, o.data(), cv.data() + at, qv.data() + at));
            const int64_t a = m->ctx_cut[d] + pb - b.pos_begin;   // the slice's first column in the batch
            for (int64_t k = 0; k < nc; k++) lens[(size_t)(a + k)] = o[(size_t)k + 1] - o[(size_t)k];
        }
        offs[i].assign((size_t)b.n_cols + 1, 0);
        for (int64_t k = 0; k < b.n_cols; k++) offs[i][(size_t)k + 1] = offs[i][(size_t)k] + lens[(size_t)k];
    }
    m->cut = cuts;
    if (int rc = build_contexts(m)) return rc;
    const std::vector<MBatch> keep = m->batches;
    m->batches.clear();
    for (size_t i = 0; i < keep.size(); i++)
        if (int rc = accumulate_host(m, keep[i].pos_begin, keep[i].n_cols, offs[i].data(), codes[i].data(), quals[i].data(),
                                     SPG_IN_TRUSTED))
            return rc;
    for (int d = 0; d < m->n; d++) MCTX(spg_wait_input(m->ctx[d]));   // (the host vectors go away)
    m->n_replans++;
    return 0;
}

// After a batch: re-plan when one device's cumulative load drifted past rebalance_ratio x the mean (an amplicon-
// shaped or partial first batch), while the history is short enough to re-slice.
static int maybe_rebalance(spg_multi *m) {
    // (not on a sample's first batch: its cuts may come from the previous sample's histogram, which one batch of an
    // amplicon-shaped BAM should not overturn)
    if (m->n < 2 || m->batches.size() < 2 || (int64_t)m->batches.size() > m->rebalance_max_batches ||
        m->rebalance_max_batches == 0)
        return 0;
    std::vector<long double> load((size_t)m->n, 0);
    long double tot = 0;
    for (size_t b = 0; b < m->w_cur.size(); b++) {
        const int64_t mid = (int64_t)b * m->bucket + m->bucket / 2;
        const int d = (int)(std::upper_bound(m->cut.begin() + 1, m->cut.end() - 1, mid) - (m->cut.begin() + 1));
        load[(size_t)d] += (long double)m->w_cur[b];
        tot += (long double)m->w_cur[b];
    }
    if (tot <= 0) return 0;
    const long double mx = *std::max_element(load.begin(), load.end());
    if (mx <= (long double)m->rebalance_ratio * tot / m->n) return 0;
    std::vector<int64_t> cuts((size_t)m->n + 1);
    if (spg_multi_plan_cuts(m->w_cur.data(), (int64_t)m->w_cur.size(), m->bucket, m->n_pos, m->n, cuts.data()) != 0) return -1;
    if (cuts == m->cut) return 0;
    return replan(m, cuts);
}

static int accumulate_host(spg_multi *m, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                           const uint8_t *base_code, const uint8_t *qual, uint32_t flags) {
    if (m->cut.empty())
        if (int rc = plan_sample(m, pos_begin, n_cols, offsets)) return rc;
    for (int d = 0; d < m->n; d++) {
        const int64_t lo = std::max(pos_begin, m->cut[d]), hi = std::min(pos_begin + n_cols, m->cut[d + 1]);
        if (hi <= lo) {
            static const uint64_t none[2] = {0, 0};
            MCTX(spg_accumulate_ex(m->ctx[d], 0, 1, none, nullptr, nullptr, 0, 0));
            continue;
        }
        const int64_t a = lo - pos_begin, b = hi - pos_begin;
        Stage *st = nullptr;
        if (int rc = stage_buf(m, d, sizeof(uint64_t) * (size_t)(b - a + 1), &st)) return rc;
        uint64_t *sub = static_cast<uint64_t *>(st->p);
        for (int64_t i = a; i <= b; i++) sub[(size_t)(i - a)] = offsets[i] - offsets[a];
        const uint64_t e = offsets[b] - offsets[a];
        MCTX(spg_accumulate_ex(m->ctx[d], lo - m->cut[d], b - a, sub, base_code + offsets[a], qual + offsets[a], e,
                               flags & SPG_IN_TRUSTED));
        MCTX(spg_input_ticket(m->ctx[d], &st->ticket));
    }
    m->stage_i = (m->stage_i + 1) % NSTAGE;
    m->batches.push_back(MBatch{pos_begin, n_cols});
    return 0;
}

extern "C" {

// One host CSR batch (spg_accumulate's arguments; host memory only), sliced at the cuts.  Pinned inputs are copied
// asynchronously on every device at once (the caller keeps them until spg_multi_wait_input).
int spg_multi_accumulate(spg_multi *m, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                         const uint8_t *base_code, const uint8_t *qual, uint64_t n_entries, uint32_t flags) {
    if (!m || !offsets || n_cols < 0 || pos_begin < 0 || pos_begin + n_cols > m->n_pos)
        return mfail("spg_multi_accumulate: bad argument");
    if (flags & (SPG_IN_DEVICE | SPG_IN_BORROW)) return mfail("spg_multi_accumulate: host batches only");
    if (!m->lut_set || !m->ref_set) return mfail("spg_multi_accumulate: eps LUT / reference not set");
    if (pos_begin + n_cols > m->ref_len)
        return mfail("spg_multi_accumulate: column range beyond the reference sequence (IndexError in the reference)");
    if (offsets[n_cols] != n_entries || offsets[0] != 0)
        return mfail("spg_multi_accumulate: offsets[0] must be 0 and offsets[n_cols] == n_entries");
    if (n_cols == 0) return 0;
    if (!(flags & SPG_IN_TRUSTED))
        for (int64_t i = 0; i < n_cols; i++)
            if (offsets[i + 1] < offsets[i]) return mfail("spg_multi_accumulate: offsets not monotone");
    if (int rc = accumulate_host(m, pos_begin, n_cols, offsets, base_code, qual, flags)) return rc;
    add_weights(m->w_cur, m->bucket, pos_begin, n_cols, offsets);
    return maybe_rebalance(m);
}

// One BAM records plan (spg_accumulate_records) sharded: device d gets the columns of its range, the reads that can
// reach them (rpos in [cut[d] - max_span, cut[d+1]); the plan's reads are in BAM = coordinate order), those reads'
// record bytes (a contiguous stretch of the inflated BAM) and rebased record offsets; positions stay reference
// positions (spg_records.pos_origin = cut[d]).  The device-side pileup runs on every device at once.
int spg_multi_accumulate_records(spg_multi *m, const spg_records *r, uint32_t flags) {
    (void)flags;
    if (!m || !r) return mfail("spg_multi_accumulate_records: null argument");
    if (!m->lut_set || !m->ref_set) return mfail("spg_multi_accumulate_records: eps LUT / reference not set");
    if (r->pos_origin != 0) return mfail("spg_multi_accumulate_records: plan positions must be reference positions");
    if (r->n_cols < 0 || r->pos_begin < 0 || r->pos_begin + r->n_cols > m->n_pos || r->n_reads < 0 || r->max_span < 0)
        return mfail("spg_multi_accumulate_records: bad extent");
    if (r->pos_begin + r->n_cols > m->ref_len)
        return mfail("spg_multi_accumulate_records: column range beyond the reference sequence");
    if (r->n_cols == 0) return 0;
    if (!r->offsets || r->offsets[0] != 0 || r->offsets[r->n_cols] != r->n_entries)
        return mfail("spg_multi_accumulate_records: offsets[0] must be 0 and offsets[n_cols] == n_entries");
    if (r->n_reads && (!r->data || !r->rec || !r->rpos || !r->rend || !r->tweak))
        return mfail("spg_multi_accumulate_records: null buffer");
    if (m->cut.empty())
        if (int rc = plan_sample(m, r->pos_begin, r->n_cols, r->offsets)) return rc;
    for (int64_t i = 1; i < r->n_reads; i++)
        if (r->rpos[i] < r->rpos[i - 1]) return mfail("spg_multi_accumulate_records: reads not in coordinate order");
    const int64_t pb = r->pos_begin, nc = r->n_cols;
    for (int d = 0; d < m->n; d++) {
        const int64_t lo = std::max(pb, m->cut[d]), hi = std::min(pb + nc, m->cut[d + 1]);
        if (hi <= lo) {
            static const uint64_t none[2] = {0, 0};
            MCTX(spg_accumulate_ex(m->ctx[d], 0, 1, none, nullptr, nullptr, 0, 0));
            continue;
        }
        const int64_t a = lo - pb, b = hi - pb;
        const int32_t *rp = r->rpos, *rp_end = r->rpos + r->n_reads;
        const int64_t r0 = std::lower_bound(rp, rp_end, (int32_t)std::max<int64_t>(INT32_MIN, lo - r->max_span)) - rp;
        const int64_t r1 = std::lower_bound(rp, rp_end, (int32_t)std::min<int64_t>(INT32_MAX, hi)) - rp;
        const int64_t nr = std::max<int64_t>(0, r1 - r0);
        Stage *st = nullptr;
        const size_t ob = sizeof(uint64_t) * (size_t)(b - a + 1);
        if (int rc = stage_buf(m, d, ob + sizeof(uint64_t) * (size_t)nr, &st)) return rc;
        uint64_t *sub = static_cast<uint64_t *>(st->p), *rec = sub + (b - a + 1);
        for (int64_t i = a; i <= b; i++) sub[(size_t)(i - a)] = r->offsets[i] - r->offsets[a];
        spg_records s = *r;
        s.pos_begin = lo - m->cut[d];
        s.n_cols = b - a;
        s.n_entries = r->offsets[b] - r->offsets[a];
        s.offsets = sub;
        s.pos_origin = m->cut[d];
        s.n_reads = nr;
        if (nr) {
            // the reads' record bytes: from the first read's record to the end of the last one (block_size in the 4
            // bytes before its refID field)
            const uint64_t base = r->rec[r0], last = r->rec[r1 - 1];
            int32_t bs = 0;
            memcpy(&bs, r->data + last - 4, 4);
            const uint64_t end = std::min<uint64_t>(r->data_bytes, last + (uint64_t)std::max(bs, 0));
            for (int64_t i = 0; i < nr; i++) rec[i] = r->rec[r0 + i] - base;
            s.data = r->data + base;
            s.data_bytes = end - base;
            s.rec = rec;
            s.rpos = r->rpos + r0;
            s.rend = r->rend + r0;
            s.tweak = r->tweak + r0;
        } else {
            s.data_bytes = 0;
            s.rec = nullptr;
        }
        MCTX(spg_accumulate_records(m->ctx[d], &s, 0));
        MCTX(spg_input_ticket(m->ctx[d], &st->ticket));
    }
    m->stage_i = (m->stage_i + 1) % NSTAGE;
    m->batches.push_back(MBatch{pb, nc});
    add_weights(m->w_cur, m->bucket, pb, nc, r->offsets);
    return maybe_rebalance(m);
}

// The cuts a batch over [pos_begin, pos_begin + n_cols) with these (host) offsets gets: the sample's cuts when it
// is already planned, else the plan spg_multi_accumulate would make for it (the contexts are created over them).
// A caller whose batch is already resident in HBM slices it at these cuts for spg_multi_accumulate_slices.
int spg_multi_plan(spg_multi *m, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets, int64_t *cuts) {
    if (!m || !offsets || !cuts || n_cols < 0 || pos_begin < 0 || pos_begin + n_cols > m->n_pos)
        return mfail("spg_multi_plan: bad argument");
    if (!m->lut_set || !m->ref_set) return mfail("spg_multi_plan: eps LUT / reference not set");
    if (m->cut.empty())
        if (int rc = plan_sample(m, pos_begin, n_cols, offsets)) return rc;
    std::copy(m->cut.begin(), m->cut.end(), cuts);
    return 0;
}

// One batch already resident in HBM, as one slice per device (slices[d]: device pointers on devices[d], pos_begin in
// reference coordinates, exactly the batch's columns inside [cuts[d], cuts[d+1]) — spg_multi_plan — with offsets
// rebased to 0; a device whose range the batch misses passes n_cols 0).  `offsets` is the whole batch's CSR on the
// host (n_cols + 1; it feeds the entry histogram that plans and re-plans the cuts).  flags: SPG_IN_DEVICE, optionally
// SPG_IN_BORROW (the slices stay the caller's and are the replay history: keep them until reset).
int spg_multi_accumulate_slices(spg_multi *m, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                                const spg_batch *slices, uint32_t flags) {
    if (!m || !offsets || !slices || n_cols < 0 || pos_begin < 0 || pos_begin + n_cols > m->n_pos)
        return mfail("spg_multi_accumulate_slices: bad argument");
    if (!(flags & SPG_IN_DEVICE) || (flags & ~(uint32_t)(SPG_IN_DEVICE | SPG_IN_BORROW | SPG_IN_TRUSTED)))
        return mfail("spg_multi_accumulate_slices: flags must be SPG_IN_DEVICE [| SPG_IN_BORROW]");
    if (!m->lut_set || !m->ref_set) return mfail("spg_multi_accumulate_slices: eps LUT / reference not set");
    if (pos_begin + n_cols > m->ref_len)
        return mfail("spg_multi_accumulate_slices: column range beyond the reference sequence");
    if (offsets[0] != 0) return mfail("spg_multi_accumulate_slices: offsets[0] must be 0");
    if (n_cols == 0) return 0;
    if (m->cut.empty())
        if (int rc = plan_sample(m, pos_begin, n_cols, offsets)) return rc;
    // every slice checked before anything is enqueued (a mismatch leaves no device with the batch)
    for (int d = 0; d < m->n; d++) {
        const int64_t lo = std::max(pos_begin, m->cut[d]), hi = std::min(pos_begin + n_cols, m->cut[d + 1]);
        const spg_batch &s = slices[d];
        if (hi <= lo) {
            if (s.n_cols != 0) return mfail("spg_multi_accumulate_slices: slice " + std::to_string(d) + " outside its cut");
            continue;
        }
        const uint64_t e = offsets[hi - pos_begin] - offsets[lo - pos_begin];
        if (s.pos_begin != lo || s.n_cols != hi - lo || s.n_entries != e || !s.offsets || (e && (!s.base_code || !s.qual)))
            return mfail("spg_multi_accumulate_slices: slice " + std::to_string(d) + " is not the batch's columns [" +
                         std::to_string(lo) + ", " + std::to_string(hi) + ") (spg_multi_plan)");
    }
    for (int d = 0; d < m->n; d++) {
        const spg_batch &s = slices[d];
        if (s.n_cols == 0) {
            static const uint64_t none[2] = {0, 0};
            MCTX(spg_accumulate_ex(m->ctx[d], 0, 1, none, nullptr, nullptr, 0, 0));
            continue;
        }
        MCTX(spg_accumulate_ex(m->ctx[d], s.pos_begin - m->cut[d], s.n_cols, s.offsets, s.base_code, s.qual, s.n_entries,
                               flags & (SPG_IN_DEVICE | SPG_IN_BORROW)));
    }
    m->batches.push_back(MBatch{pos_begin, n_cols});
    add_weights(m->w_cur, m->bucket, pos_begin, n_cols, offsets);
    return maybe_rebalance(m);
}

int spg_multi_wait_input(spg_multi *m) {
    if (!m) return mfail("spg_multi_wait_input: null");
    for (spg_ctx *c : m->ctx)
        if (c) MCTX(spg_wait_input(c));
    return 0;
}

int spg_multi_finalize(spg_multi *m) {
    if (!m) return mfail("spg_multi_finalize: null");
    if (m->cut.empty()) {                  // nothing accumulated since reset: an empty table
        if (!m->ctx[0]) {
            m->cut.assign((size_t)m->n + 1, 0);
            if (spg_multi_plan_cuts(nullptr, 0, m->bucket, m->n_pos, m->n, m->cut.data()) != 0) return -1;
            if (int rc = build_contexts(m)) return rc;
        }
    }
    for (spg_ctx *c : m->ctx) MCTX(spg_finalize(c));
    return 0;
}

}  // extern "C"

// The table copies sized for `need` records per device: send buffers on every device, the gather's receive buffer on
// devices[0], two pinned host slots.  Tables in flight are collected first (their buffers are replaced).
static int ensure_table_bufs(spg_multi *m, int64_t need) {
    if (need <= m->cap && m->host[0]) return 0;
    if (int rc = collect_all(m)) return rc;
    const int64_t cap = std::max<int64_t>({need, m->cap, 1024});
    const size_t per = TABLE_HEAD + sizeof(spg_candidate) * (size_t)cap;
    if (m->tstream.empty()) {
        m->tstream.assign((size_t)m->n, nullptr);
        m->tev.assign((size_t)m->n, nullptr);
        for (int d = 0; d < m->n; d++) {
            MHIP(hipSetDevice(m->dev[d]));
            MHIP(hipStreamCreateWithFlags(&m->tstream[(size_t)d], hipStreamNonBlocking));
            MHIP(hipEventCreateWithFlags(&m->tev[(size_t)d], hipEventDisableTiming));
        }
    }
    for (size_t i = 0; i < m->send.size(); i++) {
        MHIP(hipSetDevice(m->dev[i % (size_t)m->n]));
        if (m->send[i]) MHIP(hipFree(m->send[i]));
        m->send[i] = nullptr;
        MHIP(hipMalloc(&m->send[i], per));
    }
    MHIP(hipSetDevice(m->dev[0]));
    for (void *&r : m->recv) {
        if (r) MHIP(hipFree(r));
        r = nullptr;
        if (m->rccl) MHIP(hipMalloc(&r, per * (size_t)m->n));
    }
    for (uint8_t *&h : m->host) {
        if (h) MHIP(hipHostFree(h));
        h = nullptr;
        MHIP(hipHostMalloc((void **)&h, per * (size_t)m->n, hipHostMallocDefault));
    }
    m->cap = cap;
    return 0;
}

// Enqueue one table into slot t: per device the table + status copied out of the context's buffers by one small
// kernel on its stream (the next sample's kernels follow it there), then — on the device's table stream, off the
// context's — ONE ncclGather to devices[0] (distinct devices) or per-device copies, and the bytes into the slot's
// pinned buffer.  No host wait.
static int enqueue_table(spg_multi *m, TSlot &t) {
    const size_t per = TABLE_HEAD + sizeof(spg_candidate) * (size_t)m->cap;
    if (t.ev.empty()) {
        t.ev.assign((size_t)m->n, nullptr);
        t.ev_used.assign((size_t)m->n, 0);
    }
    const size_t si = (size_t)(&t - m->slot);
    uint8_t *h = m->host[si];
    void **send = m->send.data() + si * (size_t)m->n;
    for (int d = 0; d < m->n; d++) {
        hipStream_t st = nullptr;
        MCTX(spg_stream(m->ctx[d], (void **)&st));
        int64_t ncopy = 0;
        MCTX(spg_copy_table_device(m->ctx[d], send[d], m->cap, &ncopy));
        MHIP(hipSetDevice(m->dev[d]));
        MHIP(hipEventRecord(m->tev[(size_t)d], st));
        MHIP(hipStreamWaitEvent(m->tstream[(size_t)d], m->tev[(size_t)d], 0));
        if (!t.ev[(size_t)d]) MHIP(hipEventCreateWithFlags(&t.ev[(size_t)d], hipEventDisableTiming));
    }
    std::fill(t.ev_used.begin(), t.ev_used.end(), 0);
    if (m->rccl) {
        MCCL(ncclGroupStart());
        for (int d = 0; d < m->n; d++) {
            MHIP(hipSetDevice(m->dev[d]));
            MCCL(ncclGather(send[d], d == 0 ? m->recv[si] : nullptr, per, ncclUint8, 0, m->comm[d], m->tstream[(size_t)d]));
        }
        MCCL(ncclGroupEnd());
        MHIP(hipSetDevice(m->dev[0]));
        MHIP(hipMemcpyAsync(h, m->recv[si], per * (size_t)m->n, hipMemcpyDeviceToHost, m->tstream[0]));
    } else {
        for (int d = 0; d < m->n; d++) {
            MHIP(hipSetDevice(m->dev[d]));
            MHIP(hipMemcpyAsync(h + per * (size_t)d, send[d], per, hipMemcpyDeviceToHost, m->tstream[(size_t)d]));
        }
    }
    for (int d = 0; d < m->n; d++) {           // (every device's send buffer is free once its stream has passed here)
        MHIP(hipSetDevice(m->dev[d]));
        MHIP(hipEventRecord(t.ev[(size_t)d], m->tstream[(size_t)d]));
        t.ev_used[(size_t)d] = 1;
    }
    t.cut = m->ctx_cut;
    t.collected = false;
    t.bad = false;
    t.merged.clear();
    return 0;
}

// Wait for slot t's copies and parse them: the devices' tables merged in memory order — (first_batch, pos, allele
// rank), as the shim orders one context's table — with reference positions; `bad` when one outgrew its copy or carried
// an error word.
static int collect(spg_multi *m, TSlot &t) {
    if (t.collected || !t.ticket) return 0;
    for (size_t d = 0; d < t.ev.size(); d++)
        if (t.ev_used[d]) MHIP(hipEventSynchronize(t.ev[d]));
    const size_t per = TABLE_HEAD + sizeof(spg_candidate) * (size_t)m->cap;
    const uint8_t *h = m->host[&t - m->slot];
    size_t total = 0;
    t.bad = false;
    for (int d = 0; d < m->n; d++) {
        uint32_t head[4];
        memcpy(head, h + per * (size_t)d, sizeof head);
        if (head[1] != 0 || head[3] != head[0]) t.bad = true;
        total += head[3];
    }
    t.merged.clear();
    if (!t.bad) {
        t.merged.reserve(total);
        for (int d = 0; d < m->n; d++) {
            uint32_t head[4];
            memcpy(head, h + per * (size_t)d, sizeof head);
            const spg_candidate *r = reinterpret_cast<const spg_candidate *>(h + per * (size_t)d + TABLE_HEAD);
            const size_t at = t.merged.size();
            t.merged.insert(t.merged.end(), r, r + head[3]);
            for (size_t i = at; i < t.merged.size(); i++) t.merged[i].pos += t.cut[(size_t)d];
        }
        std::sort(t.merged.begin(), t.merged.end(), [](const spg_candidate &x, const spg_candidate &y) {
            if (x.first_batch != y.first_batch) return x.first_batch < y.first_batch;
            if (x.pos != y.pos) return x.pos < y.pos;
            return x.rank < y.rank;
        });
    }
    t.collected = true;
    return 0;
}

static int collect_all(spg_multi *m) {
    for (TSlot &t : m->slot)
        if (int rc = collect(m, t)) return rc;
    return 0;
}

// A free slot for the next table (the older one's ticket retired when both are in flight).
static TSlot &next_slot(spg_multi *m) {
    TSlot &a = m->slot[0], &b = m->slot[1];
    if (!a.ticket) return a;
    if (!b.ticket) return b;
    return a.ticket < b.ticket ? a : b;
}

static int finish_out(const std::vector<spg_candidate> &all, spg_candidate *out, int64_t cap, int64_t *n_out) {
    *n_out = (int64_t)all.size();
    if (*n_out > cap) return mfail("spg_multi_get_candidates: output capacity too small");
    if (!all.empty() && out) memcpy(out, all.data(), sizeof(spg_candidate) * all.size());
    return 0;
}

extern "C" {

int spg_multi_get_candidates(spg_multi *m, spg_candidate *out, int64_t cap, int64_t *n_out) {
    if (!m || !n_out) return mfail("spg_multi_get_candidates: null");
    *n_out = 0;
    if (!m->ctx[0]) return 0;
    if (int rc = ensure_table_bufs(m, m->cap)) return rc;
    for (int attempt = 0; attempt < 2; attempt++) {
        TSlot &t = next_slot(m);
        if (t.ticket && !t.collected) if (int rc = collect(m, t)) return rc;
        t.ticket = ++m->tseq;
        if (int rc = enqueue_table(m, t)) { t.ticket = 0; return rc; }
        if (int rc = collect(m, t)) { t.ticket = 0; return rc; }
        t.ticket = 0;                        // (a synchronous table: the slot is free again)
        if (!t.bad) return finish_out(t.merged, out, cap, n_out);
        // a table outgrew its copy, or an error word: settle every context (reports the error, or grows its buffers
        // and finalizes again), size the copies for the largest table, and take it once more
        int64_t need = 1;
        for (spg_ctx *c : m->ctx) {
            int64_t nc = 0, nd = 0;
            MCTX(spg_count(c, &nc, &nd));
            need = std::max(need, nc);
        }
        if (int rc = ensure_table_bufs(m, need)) return rc;
    }
    return mfail("spg_multi_get_candidates: the device tables did not settle");
}

int spg_multi_get_candidates_async(spg_multi *m, uint64_t *ticket) {
    if (!m || !ticket) return mfail("spg_multi_get_candidates_async: null");
    *ticket = 0;
    if (int rc = ensure_table_bufs(m, m->cap)) return rc;
    TSlot &t = next_slot(m);
    if (t.ticket && !t.collected) if (int rc = collect(m, t)) return rc;   // (retired: its wait fails)
    t.ticket = ++m->tseq;
    if (!m->ctx[0]) {                        // nothing accumulated, no contexts: an empty table
        std::fill(t.ev_used.begin(), t.ev_used.end(), 0);
        t.merged.clear();
        t.bad = false;
        t.collected = true;
    } else if (int rc = enqueue_table(m, t)) {
        t.ticket = 0;
        return rc;
    }
    *ticket = t.ticket;
    return 0;
}

int spg_multi_wait_candidates(spg_multi *m, uint64_t ticket, spg_candidate *out, int64_t cap, int64_t *n_out) {
    if (!m || !n_out) return mfail("spg_multi_wait_candidates: null");
    *n_out = 0;
    TSlot *t = nullptr;
    for (TSlot &s : m->slot)
        if (ticket && s.ticket == ticket) t = &s;
    if (!t) return mfail("spg_multi_wait_candidates: unknown or retired ticket (two tables at most in flight)");
    if (int rc = collect(m, *t)) return rc;
    if (t->bad) {
        t->ticket = 0;
        g_merr = "spg_multi_wait_candidates: a device table outgrew its copy or carried an error word; take this "
                 "sample's table with spg_multi_get_candidates before its reset";
        return 1;
    }
    if (int rc = finish_out(t->merged, out, cap, n_out)) return rc;   // (the ticket stays: wait again, larger cap)
    t->ticket = 0;
    t->merged.clear();
    return 0;
}

int spg_multi_context(spg_multi *m, int i, spg_ctx **ctx) {
    if (!m || !ctx || i < 0 || i >= m->n) return mfail("spg_multi_context: bad argument");
    if (!m->ctx[(size_t)i]) return mfail("spg_multi_context: no context yet (the sample's first batch creates them)");
    *ctx = m->ctx[(size_t)i];
    return 0;
}

}  // extern "C"
