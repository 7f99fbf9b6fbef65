// spg_api.cpp — C-ABI of the engine (include/spings_gpu.h): context, HBM buffers, stream-ordered
// copies and kernel launches.  Compiled by hipcc together with spg_kernels.hip into
// libspings_gpu.so.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "spg_device.h"

namespace spg {
hipError_t launch_accumulate(const KParams &P, const uint64_t *off, const uint8_t *code, const uint8_t *qual,
                             const uint8_t *ref, const Tables *T, Acc *acc, hipStream_t st);
hipError_t launch_finalize(const FParams &F, const Acc *acc, const Tables *T, const Out &O, const Hist *H,
                           hipStream_t st);
hipError_t launch_lite(const MParams &P, const Hist &hb, const uint8_t *ref, const Tables *T, Acc *acc, int64_t blocks,
                       hipStream_t st);
int lite_blocks_per_cu();
hipError_t launch_lite_fold(const MParams &P, const Hist &hb, const uint8_t *ref, const Tables *T, Acc *acc, int64_t blocks,
                            hipStream_t st);
hipError_t launch_count_run(const MParams &P, const Hist *H, const uint8_t *ref, uint32_t *cdep, uint32_t *cmcf, int lpc,
                            int64_t blocks, hipStream_t st);
int count_run_blocks_per_cu(int lpc);
hipError_t launch_count_cols(const MParams &P, const Hist &hb, const uint8_t *ref, uint32_t *dlist, int lpc, int64_t blocks,
                             hipStream_t st);
int count_cols_blocks_per_cu(int lpc);
hipError_t launch_count_list(const MParams &P, const uint8_t *ref, const uint32_t *cdep, const uint32_t *cmcf, hipStream_t st);
hipError_t launch_fold_hist(const MParams &P, const Hist *H, const uint8_t *ref, const Tables *T, Acc *acc, int64_t blocks,
                            void *part, uint32_t *arrived, int bpp, int cap, hipStream_t st);
size_t fold_part_bytes();
hipError_t launch_tile(const MParams &P, const Hist *H, const uint8_t *ref, int64_t ref_len, const Tables *T, Acc *acc,
                       int lpc, int64_t max_blocks, hipStream_t st);
hipError_t launch_merge(const MParams &P, const uint8_t *ref, Acc *acc, hipStream_t st);
int tile_blocks_per_cu(int lpc, bool one);
hipError_t launch_pileup_fill(const FillArgs &A, hipStream_t st);
size_t fill_scratch_bytes(int64_t n_cols, int64_t n_reads, int64_t max_span);
hipError_t launch_pos_bounds(const Hist *H, const int32_t *items, int32_t n, int64_t pos, uint64_t *rng, hipStream_t st);
hipError_t launch_pos_copy(const Hist *H, const int32_t *items, int32_t n, const uint64_t *rng, const uint64_t *dst,
                           uint8_t *oc, uint8_t *oq, hipStream_t st);
hipError_t launch_ck_compact(const Hist &h, uint32_t min_bq, uint64_t *kept, uint64_t *noff, void *scan_tmp,
                             size_t *scan_bytes, uint8_t *oc, uint8_t *oq, hipStream_t st);
hipError_t launch_ck_pack(uint8_t *oc, const uint8_t *oq, uint64_t m, uint64_t base, uint64_t *xi, uint8_t *xc, uint8_t *xq,
                          uint32_t *xn, uint32_t xcap, hipStream_t st);
hipError_t launch_table_copy(const Counters *ctr, const uint32_t *kerr, const uint32_t *ferr, const void *cand, int64_t cap,
                             int64_t detail_cap, void *dst, hipStream_t st);
size_t plan_temp_bytes(uint32_t n, int64_t span_n);
hipError_t launch_plan_reads(const PlanArgs &A, void *tmp, size_t tmp_bytes, hipStream_t st);
hipError_t launch_plan_cov(const PlanArgs &A, int all, int32_t *cov, void *tmp, size_t tmp_bytes, hipStream_t st);
hipError_t launch_plan_keep(const PlanArgs &A, bool sweep, hipStream_t st);
hipError_t launch_plan_rest(const PlanArgs &A, int32_t *cov, bool pairing, void *tmp, size_t tmp_bytes, hipStream_t st);
size_t inflate_scratch_bytes(uint64_t comp_bytes, int64_t n);
hipError_t launch_inflate(const uint8_t *comp, uint64_t comp_bytes, const spg_bgzf_member *mem, int64_t n, uint8_t *out,
                          uint32_t *status, void *scratch, hipStream_t st);
hipError_t launch_bam_scan(const BamArgs &A, int pass, hipStream_t st);
hipError_t launch_bam_pairs(const BamPairArgs &P, bool tweak, hipStream_t st);
hipError_t launch_bam_gather(const BamGatherArgs &G, hipStream_t st);
}  // namespace spg

using namespace spg;

static thread_local std::string g_err;

static int fail(const std::string &m) {
    g_err = m;
    return -1;
}

#define HIPCHK(x)                                                                                       \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_));              \
    } while (0)

// Timing events: 2 (default) around accumulate and finalize, 1 accumulate only, 0 none.  Each
// timestamped event costs a few microseconds of GPU idle between launches.
static int default_timing() {
    static const int lvl = [] { const char *e = getenv("SPG_TIMING"); return e ? atoi(e) : 2; }();
    return lvl;
}

struct HistBatch {
    int64_t pos_begin, n_cols;
    uint64_t n_entries;
    uint64_t *off;
    uint8_t *code, *qual;
    bool owned;            // in the context's arena (else borrowed device buffers)
    uint32_t seq0;         // batch_seq of its (first) sample
    int64_t n_samples;     // > 1: a multi-sample column-major batch (spg_accumulate_samples)
    uint32_t *fsamp;       // multi-sample: first sample holding entries, per column (device)
    int slab = -1;         // owned: the arena slab holding it
    size_t bytes = 0;      // owned: its bytes there (offsets + both padded arrays)
    uint8_t *dev0 = nullptr;   // owned: start of its arena block
    void *host = nullptr;      // spilled to pinned host memory (the descriptors point there, mapped)
};

// Device arena for the owned batch copies (the replay history): slabs allocated once and bump-
// allocated per batch, recycled at spg_reset (no hipMalloc / hipFree per batch).  Copies into a
// recycled slab are ordered after the kernels that read its old content (reset_fence below).
struct Arena {
    struct Slab { uint8_t *base; size_t cap, used; int64_t live; };
    std::vector<Slab> slabs;               // a released slab stays as a tombstone (base null): indices are stable
    size_t cur = 0;
    size_t max_slab = (size_t)8 << 30;     // smaller under a history cap (spilling frees whole slabs)
    hipError_t alloc(size_t n, uint8_t **out, int *slab) {
        n = (n + 255) & ~size_t(255);
        while (cur < slabs.size()) {
            Slab &s = slabs[cur];
            if (s.base && s.cap - s.used >= n) {
                *out = s.base + s.used; s.used += n; s.live++; *slab = (int)cur;
                return hipSuccess;
            }
            cur++;
        }
        // geometric slabs: 256 MiB, 512 MiB, 1 GiB, ... max_slab
        size_t cap = std::min((size_t)256 << 20, max_slab);
        for (size_t i = 0; i < slabs.size() && cap < max_slab; i++) cap <<= 1;
        cap = std::max(std::min(cap, max_slab), n);
        Slab s{nullptr, cap, 0, 0};
        hipError_t e = hipMalloc(&s.base, cap);
        if (e != hipSuccess) return e;
        slabs.push_back(s);
        cur = slabs.size() - 1;
        slabs[cur].used = n;
        slabs[cur].live = 1;
        *out = s.base;
        *slab = (int)cur;
        return hipSuccess;
    }
    void recycle() {
        for (auto &s : slabs) { s.used = 0; s.live = 0; }
        cur = 0;
    }
    void release() {
        for (auto &s : slabs)
            if (s.base) (void)hipFree(s.base);
        slabs.clear();
        cur = 0;
    }
    size_t bytes() const {
        size_t n = 0;
        for (auto &s : slabs)
            if (s.base) n += s.cap;
        return n;
    }
};

// Device buffers of spg_bam_* (one BAM at a time per context; grow-only, freed by spg_bam_release / spg_destroy)
struct DBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t need(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) { hipError_t e = hipFree(p); if (e != hipSuccess) return e; }
        p = nullptr;
        cap = 0;
        const size_t c = n + n / 8 + 256;
        hipError_t e = hipMalloc(&p, c);
        if (e == hipSuccess) cap = c;
        return e;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
    template <class T> T *as() const { return static_cast<T *>(p); }
};
struct BamDev {
    DBuf comp, out, mem, status, uoff, start, cnt, base, lohi, rec, fields, err;
    DBuf kept, pairs, orig, twof, recs_k, tile_first, iscr, rtmp;
    DBuf plan_rd, plan_sp, plan_tmp;   // spg_bam_plan_build: per-read arrays, per-column arrays, hipcub scratch
    int32_t tid = 0;                   // the contig spg_bam_open kept
    bool open = false;                 // a BAM is loaded (spg_bam_open succeeded)
    uint64_t total = 0;                // inflated bytes
    int64_t n_members = 0;
    uint32_t n_reads = 0;
    // field arrays inside `fields`
    int32_t *pos = nullptr, *end = nullptr, *mtid = nullptr, *mpos = nullptr, *isize = nullptr;
    uint16_t *flag = nullptr;
    uint32_t *l_seq = nullptr;
    uint64_t *nhash = nullptr;
    float inflate_ms = 0.f;
    int64_t inflate_fallbacks = 0;     // members k_inflate_par left to the lane kernel (the last spg_bam_open)
    hipEvent_t ev[2] = {nullptr, nullptr};
    hipEvent_t ev_up = nullptr;        // spg_bam_upload's copies into this slot done
    bool up_pending = false;           // comp / mem hold an upload of (up_comp, up_bytes, up_n) for the next spg_bam_open
    const uint8_t *up_comp = nullptr;
    uint64_t up_bytes = 0;
    int64_t up_n = 0;
    void release() {
        up_pending = false;
        for (DBuf *b : {&comp, &out, &mem, &status, &uoff, &start, &cnt, &base, &lohi, &rec, &fields, &err, &kept, &pairs,
                        &orig, &twof, &recs_k, &tile_first, &iscr, &rtmp, &plan_rd, &plan_sp, &plan_tmp})
            b->release();
        open = false;
    }
};

struct spg_ctx {
    int device = 0;
    int n_cu = 256;                     // compute units (the tile kernel's resident grid: 5 workgroups per CU)
    int64_t n_pos = 0;
    spg_params p{};
    hipStream_t stream = nullptr;       // kernels
    hipStream_t copy_stream = nullptr;  // host -> device batch copies
    hipStream_t up_stream = nullptr;    // spg_bam_upload: the next BAM's compressed bytes (created on first use)
    hipEvent_t copy_ev = nullptr;       // after the latest batch copy
    hipEvent_t compute_ev = nullptr;    // reset fence: recycled arena copies wait for the old kernels
    hipEvent_t hist_ev = nullptr;       // after the latest descriptor upload (pinned mirror -> d_hist)
    bool hist_up = false;               // an upload was enqueued since the last reset
    bool hist_fence = false;            // reset since that upload: the mirror's first rewrite waits for it
    static constexpr int NIN = 8;       // input tickets: an event per host-input batch copy (ring)
    hipEvent_t in_ev[NIN] = {};
    uint64_t in_seq = 0;
    bool copy_pending = false;          // the compute stream has not waited on copy_ev yet
    bool arena_fence = false;           // the arena was recycled: the next copy into it waits for the kernels
                                        // enqueued before the reset (recorded lazily: an event record per
                                        // step idled the GPU between steps)
    Acc *acc = nullptr;
    Tables *tables = nullptr;
    bool lut_set = false;
    uint8_t *ref = nullptr;
    int64_t ref_len = 0;
    std::vector<HistBatch> hist;
    Arena arena;
    Hist *d_hist = nullptr;             // device descriptors of every history batch
    int64_t d_hist_cap = 0;
    Hist *h_hist = nullptr;             // pinned host mirror (uploaded per run; append-only)
    int64_t h_hist_cap = 0;
    int64_t pend0 = 0;                  // history batches [pend0, size) are not accumulated yet (a run)
    uint64_t pend_entries = 0;
    uint32_t *kerr = nullptr;           // run kernels' error word (bit 0: a batch too deep for a run), compute stream
    bool kerr_dirty = false;            // a kernel that may set kerr was enqueued since it was last cleared
    uint32_t *ferr = nullptr;           // k_pileup_fill's error word (bit 2: the records disagree with the offsets):
                                        // written, read and cleared on the copy stream, where the fills run
    bool ferr_dirty = false;
    uint32_t *nlist = nullptr;          // fused run: positions listed for the sparse finalize (in `band`)
    uint32_t *deep_list = nullptr;      // single shallow batch: its long columns (for k_acc_seg<1>) ...
    int64_t deep_cap = 0;
    uint32_t *deep_n = nullptr;         // ... and their count
    bool stale = false;                 // records of history [0, stale_end) not written (fused run)
    bool stale_deep = false;            // ... the stale history is the sample's lone deep batch (k_count_cols)
    bool deep_pend = false;             // history batch 0 is a deep batch not accumulated yet: a calls-only
                                        // finalize runs it fused (k_acc_seg<..., FUSE>), anything else first
                                        // accumulates it on its own
    int64_t stale_end = 0;
    // counted mode (calls-only runs of shallow batches): per-position bq-passing / REF-code entry counts of history
    // [0, count_end), the records stale; see finalize_counted
    bool counted = false;
    int64_t count_end = 0;
    int64_t n_deep_hist = 0;            // deep / multi-sample batches since reset (counted mode needs none)
    uint32_t *cdep = nullptr, *cmcf = nullptr;
    uint64_t *fwm = nullptr;            // k_fold_hist's per-position fold watermarks ((generation << 32) | batches)
    RSlot *rcache = nullptr;            // replay cache (allocated once a history is long enough for replays to matter)
    uint8_t *pe_buf = nullptr;          // spg_position_entries' device scratch (grow-only)
    size_t pe_cap = 0;
    uint32_t count_gen = 0;             // generation of the current counted run (bumped whenever counted mode starts)
    void *fold_part = nullptr;          // k_fold_hist's multi-workgroup partials [FOLD_CAP][FOLD_BPP]
    uint32_t *fold_arrived = nullptr;   // ... and arrival counts (zero between launches)
    // bounded history: owned batches past `hist_cap` bytes of HBM are spilled, oldest folded first
    int64_t hist_cap = 0;               // 0 = no cap
    int64_t hist_dev_bytes = 0;         // owned history bytes resident in HBM
    int64_t n_spilled = 0;
    BamDev bams[2];                     // spg_bam_*: BAMs in HBM (two slots: process_bams opens the next BAM while the
    int bam_slot = 0;                   // host plans the last one), the current slot (spg_bam_slot)
    BamDev &bam_cur() { return bams[bam_slot]; }
    // spg_accumulate_records: HBM staging of the last records batch (inflated BAM + per-read index), grow-only
    uint8_t *rs = nullptr;
    size_t rs_cap = 0;
    MState *part = nullptr;             // split-run partial states
    size_t part_bytes = 0;
    // replay index: history batches per 2^RIDX_SHIFT-position bucket
    std::vector<std::vector<int32_t>> buckets;
    bool ridx_dirty = false;
    int64_t ridx_items = 0;
    uint32_t *h_ridx = nullptr, *d_ridx = nullptr;   // [n_buckets + 1 offsets | items]
    size_t ridx_cap = 0;
    hipEvent_t ridx_ev = nullptr;
    bool ridx_valid = false;
    uint32_t batch_seq = 0;
    uint32_t epoch = 1;        // Acc records of other epochs read as empty (reset = epoch bump)
    uint32_t cslot = 0;        // Counters slot of the last finalize
    // outputs
    uint32_t *o_depth = nullptr, *o_counts = nullptr, *o_order = nullptr, *o_first = nullptr;
    double *o_gl = nullptr;
    uint8_t *o_flags = nullptr;
    spg_candidate *cand = nullptr;
    int64_t cand_cap = 0;
    int64_t *band = nullptr;
    int64_t band_cap = 0;
    spg_detail *detail = nullptr;
    int64_t detail_cap = 0;
    Counters *ctr = nullptr;
    FusedArgs *d_fused = nullptr;       // the fused accumulate's finalize parameters [2 slots] (device) ...
    FusedArgs *h_fused = nullptr;       // ... and their pinned staging copy (re-uploaded when they change)
    bool fused_valid = false;
    bool finalized = false;
    // timing ring: one entry per finalize; events around the accumulate launches (first begin ..
    // last end) and around the finalize launch.  Read back without stalling the pipeline.
    static constexpr int NRING = 256;
    hipEvent_t ev[NRING][4] = {};
    int64_t ring_w = 0, ring_r = 0;     // entries [ring_r, ring_w) are complete
    uint8_t ring_tm[NRING] = {};        // bit 0: accumulate events recorded, bit 1: finalize events
    bool acc_open = false;
    bool last_acc = false, last_fin = false;
    bool table_valid = false;           // the SoA table matches the last finalize
    int timing = default_timing();
    int acc_timing = 0;                 // level the open / last accumulate interval was recorded at
    int64_t path[9] = {};               // spg_path_counters
};


extern "C" {

const char *spg_last_error(void) { return g_err.c_str(); }
int spg_abi_version(void) { return SPG_ABI_VERSION; }
size_t spg_sizeof_candidate(void) { return sizeof(spg_candidate); }
size_t spg_sizeof_detail(void) { return sizeof(spg_detail); }
size_t spg_sizeof_acc(void) { return sizeof(Acc); }

int spg_device_count(int *n) {
    if (!n) return fail("spg_device_count: null");
    HIPCHK(hipGetDeviceCount(n));
    return 0;
}

int spg_host_alloc(size_t bytes, void **out) {
    if (!out) return fail("spg_host_alloc: null argument");
    *out = nullptr;
    HIPCHK(hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocDefault));
    return 0;
}

int spg_host_free(void *p) {
    if (p) HIPCHK(hipHostFree(p));
    return 0;
}

static int alloc_outputs(spg_ctx *c) {
    const int64_t n = c->n_pos;
    HIPCHK(hipMalloc(&c->o_depth, sizeof(uint32_t) * (n + 1)));
    HIPCHK(hipMalloc(&c->o_counts, sizeof(uint32_t) * SPG_NCOUNT * (n + 1)));
    HIPCHK(hipMalloc(&c->o_order, sizeof(uint32_t) * (n + 1)));
    HIPCHK(hipMalloc(&c->o_first, sizeof(uint32_t) * (n + 1)));
    HIPCHK(hipMalloc(&c->o_gl, sizeof(double) * SPG_NSLOT * (n + 1)));
    HIPCHK(hipMalloc(&c->o_flags, n + 16));
    c->band_cap = n + 1;
    HIPCHK(hipMalloc(&c->band, sizeof(int64_t) * c->band_cap));
    c->cand_cap = std::max<int64_t>(4096, n / 4 + 1024);
    HIPCHK(hipMalloc(&c->cand, sizeof(spg_candidate) * c->cand_cap));
    c->detail_cap = std::max<int64_t>(1024, std::min<int64_t>(n + 1, 65536));
    HIPCHK(hipMalloc(&c->detail, sizeof(spg_detail) * c->detail_cap));
    HIPCHK(hipMalloc(&c->ctr, 2 * sizeof(Counters)));
    HIPCHK(hipMalloc(&c->d_fused, 2 * sizeof(FusedArgs)));
    HIPCHK(hipHostMalloc((void **)&c->h_fused, 2 * sizeof(FusedArgs), hipHostMallocDefault));
    memset(c->h_fused, 0, 2 * sizeof(FusedArgs));
    HIPCHK(hipMemsetAsync(c->ctr, 0, 2 * sizeof(Counters), c->stream));
    HIPCHK(hipMalloc(&c->kerr, sizeof(uint32_t)));
    HIPCHK(hipMalloc(&c->ferr, sizeof(uint32_t)));
    HIPCHK(hipMalloc(&c->nlist, sizeof(uint32_t)));
    HIPCHK(hipMalloc(&c->deep_n, sizeof(uint32_t)));
    HIPCHK(hipMemsetAsync(c->kerr, 0, sizeof(uint32_t), c->stream));
    HIPCHK(hipMemsetAsync(c->ferr, 0, sizeof(uint32_t), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));        // (ferr is then used on the copy stream)
    return 0;
}

int spg_create(int device, int64_t n_pos, const spg_params *p, spg_ctx **out) {
    if (!out || !p) return fail("spg_create: null argument");
    if (n_pos <= 0) return fail("spg_create: n_pos must be > 0");
    *out = nullptr;
    spg_ctx *c = new spg_ctx();
    c->device = device;
    c->n_pos = n_pos;
    c->p = *p;
    int rc = 0;
    auto bail = [&](int r) { spg_destroy(c); return r; };
    if (hipSetDevice(device) != hipSuccess) return bail(fail("spg_create: hipSetDevice failed"));
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->n_cu <= 0)
        c->n_cu = 256;
    if (const char *e = getenv("SPG_HIST_CAP")) {          // bytes of owned history kept in HBM (0 = no cap)
        c->hist_cap = atoll(e);
        if (c->hist_cap > 0)
            c->arena.max_slab = std::max<size_t>((size_t)16 << 20, std::min<size_t>((size_t)8 << 30, (size_t)c->hist_cap / 4));
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail("spg_create: stream"));
    if (hipEventCreateWithFlags(&c->copy_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->compute_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ridx_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->hist_ev, hipEventDisableTiming) != hipSuccess)
        return bail(fail("spg_create: event"));
    for (auto &e : c->in_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return bail(fail("spg_create: event"));
    if (hipMalloc(&c->acc, sizeof(Acc) * n_pos) != hipSuccess) return bail(fail("spg_create: acc alloc"));
    if (hipMalloc(&c->tables, sizeof(Tables)) != hipSuccess) return bail(fail("spg_create: tables alloc"));
    if (hipMemsetAsync(c->acc, 0, sizeof(Acc) * n_pos, c->stream) != hipSuccess) return bail(fail("memset"));
    if ((rc = alloc_outputs(c)) != 0) return bail(rc);
    for (auto &row : c->ev)
        for (auto &e : row)
            if (hipEventCreate(&e) != hipSuccess) return bail(fail("spg_create: event"));
    c->buckets.resize((size_t)((n_pos + (1 << RIDX_SHIFT) - 1) >> RIDX_SHIFT));
    *out = c;
    return 0;
}

static void free_spilled(spg_ctx *c);
static void clear_history(spg_ctx *c) {
    free_spilled(c);
    c->hist.clear();
    c->hist_dev_bytes = 0;
    c->arena.recycle();
    c->pend0 = 0;
    c->pend_entries = 0;
    for (auto &b : c->buckets) b.clear();
    c->ridx_items = 0;
    c->ridx_dirty = false;
    c->ridx_valid = false;
}

int spg_destroy(spg_ctx *c) {
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    if (c->up_stream) {
        (void)hipStreamSynchronize(c->up_stream);
        (void)hipStreamDestroy(c->up_stream);
    }
    free_spilled(c);
    c->arena.release();
    for (BamDev &b : c->bams) {
        b.release();
        for (hipEvent_t e : b.ev)
            if (e) (void)hipEventDestroy(e);
        if (b.ev_up) (void)hipEventDestroy(b.ev_up);
    }
    void *bufs[] = {c->acc, c->tables, c->ref, c->d_hist, c->o_depth, c->o_counts, c->o_order, c->o_first,
                    c->o_gl, c->o_flags, c->cand, c->band, c->detail, c->ctr, c->part, c->d_ridx, c->kerr, c->nlist,
                    c->d_fused, c->deep_list, c->deep_n, c->cdep, c->cmcf, c->fwm, c->fold_part, c->fold_arrived, c->rs,
                    c->ferr, c->rcache, c->pe_buf};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (c->h_hist) (void)hipHostFree(c->h_hist);
    if (c->h_ridx) (void)hipHostFree(c->h_ridx);
    if (c->h_fused) (void)hipHostFree(c->h_fused);
    for (auto &row : c->ev)
        for (auto &e : row)
            if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {c->copy_ev, c->compute_ev, c->ridx_ev, c->hist_ev})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->in_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    delete c;
    return 0;
}

int spg_reset(spg_ctx *c) {
    if (!c) return fail("spg_reset: null ctx");
    HIPCHK(hipSetDevice(c->device));
    c->stale = false;
    c->stale_deep = false;
    c->deep_pend = false;
    c->counted = false;
    c->count_end = 0;
    c->n_deep_hist = 0;
    // batches still pending belong to the old sample: dropped.  Copies into the recycled arena are
    // ordered after every kernel enqueued so far (add_batch records that fence before its first copy).
    if (!c->arena.slabs.empty()) c->arena_fence = true;
    // descriptor uploads still queued read the pinned mirror, which the next sample rewrites from index 0
    if (c->hist_up) c->hist_fence = true;
    clear_history(c);
    // a new sample starts error-free (only the run and records kernels write the word, and settle clears what it
    // reports: no per-step memset launch for the deep path)
    if (c->kerr_dirty) {
        HIPCHK(hipMemsetAsync(c->kerr, 0, sizeof(uint32_t), c->stream));
        c->kerr_dirty = false;
    }
    // (on the copy stream: ordered after the dropped sample's records fills, before the next sample's)
    if (c->ferr_dirty) {
        HIPCHK(hipMemsetAsync(c->ferr, 0, sizeof(uint32_t), c->copy_stream));
        c->ferr_dirty = false;
    }
    if (++c->epoch == 0) {     // wrapped: clear the records once and restart at epoch 1
        HIPCHK(hipMemsetAsync(c->acc, 0, sizeof(Acc) * c->n_pos, c->stream));
        c->epoch = 1;
    }
    c->batch_seq = 0;
    c->finalized = false;
    return 0;
}

int spg_set_eps_lut(spg_ctx *c, const double lut[256]) {
    if (!c || !lut) return fail("spg_set_eps_lut: null argument");
    Tables *t = (Tables *)calloc(1, sizeof(Tables));
    for (int q = 0; q < 256; q++) {
        t->eps[q] = lut[q];
        t->l1m[q] = q == 0 ? 0.0 : std::log1p(-lut[q]);
        if (!(lut[q] > 0.0 && lut[q] <= 1.0)) {
            free(t);
            return fail("spg_set_eps_lut: eps out of (0,1]");
        }
    }
    if (lut[0] != 1.0) { free(t); return fail("spg_set_eps_lut: eps[0] must be 1.0 (10^-0)"); }
    for (int k = 0; k < 336; k++) {
        char buf[32];
        snprintf(buf, sizeof buf, "1e-%d", k);
        t->p10k[k] = strtod(buf, nullptr);   // correctly rounded decimal -> binary
    }
    t->fast[0][0] = 0.0;
    t->fast[0][1] = 0.0;
    for (int q = 1; q < 256; q++) {
        t->fast[q][0] = t->l1m[q];
        t->fast[q][1] = t->eps[q];
    }
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = hipMemcpyAsync(c->tables, t, sizeof(Tables), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    free(t);
    if (e != hipSuccess) return fail(std::string("spg_set_eps_lut: ") + hipGetErrorString(e));
    c->lut_set = true;
    return 0;
}

static int flush_run(spg_ctx *c, int64_t h1 = -1, bool fused = false);
static int flush_deep(spg_ctx *c);
static int materialize(spg_ctx *c);

int spg_set_reference(spg_ctx *c, const char *seq, int64_t len) {
    if (!c || !seq || len < 0) return fail("spg_set_reference: bad argument");
    HIPCHK(hipSetDevice(c->device));
    // pending batches take their first-visit REF chars from the reference they were accumulated under, and
    // so do the records a fused finalize left unwritten (materialize re-folds them under this reference)
    if (int rc = materialize(c)) return rc;
    if (int rc = flush_deep(c)) return rc;
    if (int rc = flush_run(c)) return rc;
    if (c->ref) {
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipFree(c->ref));
        c->ref = nullptr;
    }
    HIPCHK(hipMalloc(&c->ref, len + 16));
    HIPCHK(hipMemcpyAsync(c->ref, seq, len, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->ref_len = len;
    return 0;
}

// SPG_TRACE=1 (debugging): synchronise after every launch and name the kernel that failed
static bool trace_on() {
    static const bool on = [] { const char *e = getenv("SPG_TRACE"); return e && atoi(e) > 0; }();
    return on;
}
static uint32_t *trace_dbg() {      // device words the kernels record range violations in
    static uint32_t *d = [] { uint32_t *p = nullptr; if (hipMalloc(&p, 64) == hipSuccess) (void)hipMemset(p, 0, 64); return p; }();
    return d;
}
static uint4 *g_prog = nullptr;      // SPG_TRACE: host-mapped per-wave progress of the last accumulate
static size_t g_prog_n = 0;
static uint4 *trace_prog(int64_t n_waves) {
    if (!trace_on()) return nullptr;
    if ((size_t)n_waves > g_prog_n) {
        if (g_prog) (void)hipHostFree(g_prog);
        g_prog = nullptr;
        g_prog_n = 0;
        if (hipHostMalloc((void **)&g_prog, sizeof(uint4) * n_waves, hipHostMallocMapped) != hipSuccess) return nullptr;
        g_prog_n = (size_t)n_waves;
    }
    memset(g_prog, 0, sizeof(uint4) * g_prog_n);
    uint4 *d = nullptr;
    if (hipHostGetDevicePointer((void **)&d, g_prog, 0) != hipSuccess) return nullptr;
    return d;
}
static int trace_sync(spg_ctx *c, const char *what) {
    if (!trace_on()) return 0;
    const hipError_t e = hipStreamSynchronize(c->stream);
    if (g_prog && e != hipSuccess) {     // which waves were where when the kernel faulted
        size_t hist[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int shown = 0;
        for (size_t w = 0; w < g_prog_n; w++) {
            const volatile uint32_t *r = reinterpret_cast<volatile uint32_t *>(g_prog + w);
            const uint32_t st = r[0];
            hist[st < 8 ? st : 7]++;
            if (st != 0 && st != 6 && shown < 32) {
                fprintf(stderr, "[spg trace] wave %zu stage %u: %u %u %u\n", w, st, r[1], r[2], r[3]);
                shown++;
            }
        }
        fprintf(stderr, "[spg trace] stages 0-7: %zu %zu %zu %zu %zu %zu %zu %zu\n", hist[0], hist[1], hist[2],
                hist[3], hist[4], hist[5], hist[6], hist[7]);
    }
    uint32_t h[4] = {0, 0, 0, 0};
    if (e == hipSuccess && trace_dbg()) (void)hipMemcpy(h, trace_dbg(), sizeof(h), hipMemcpyDeviceToHost);
    fprintf(stderr, "[spg trace] %s: %s dbg %u %u %u %08x\n", what, hipGetErrorString(e), h[0], h[1], h[2], h[3]);
    fflush(stderr);
    return e == hipSuccess ? 0 : fail(std::string("spg trace: ") + what + ": " + hipGetErrorString(e));
}

static constexpr int64_t NB_RING = SPG_NB;   // k_acc_seg's finishing ring (columns per wave when fused)

static int64_t env_i64(const char *name, int64_t dflt) {
    const char *e = getenv(name);
    return e ? std::max<int64_t>(1, atoll(e)) : dflt;
}

// Device descriptor table and its pinned host mirror, grown geometrically.
static int grow_history_table(spg_ctx *c) {
    const int64_t n = (int64_t)c->hist.size();
    if (n > c->h_hist_cap) {
        int64_t cap = std::max<int64_t>(64, c->h_hist_cap * 2);
        while (cap < n) cap *= 2;
        Hist *nh = nullptr;
        HIPCHK(hipHostMalloc((void **)&nh, sizeof(Hist) * cap, hipHostMallocDefault));
        if (c->h_hist) {
            memcpy(nh, c->h_hist, sizeof(Hist) * c->h_hist_cap);
            HIPCHK(hipStreamSynchronize(c->stream));      // in-flight uploads may still read the old mirror
            HIPCHK(hipHostFree(c->h_hist));
        }
        c->h_hist = nh;
        c->h_hist_cap = cap;
    }
    if (n > c->d_hist_cap) {
        int64_t cap = std::max<int64_t>(64, c->d_hist_cap * 2);
        while (cap < n) cap *= 2;
        Hist *nd = nullptr;
        HIPCHK(hipMalloc(&nd, sizeof(Hist) * cap));
        if (c->d_hist) {
            HIPCHK(hipMemcpyAsync(nd, c->d_hist, sizeof(Hist) * c->d_hist_cap, hipMemcpyDeviceToDevice, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            HIPCHK(hipFree(c->d_hist));
        }
        c->d_hist = nd;
        c->d_hist_cap = cap;
    }
    return 0;
}

// accumulate timing interval: ev[0] before the first accumulate launch since the last finalize
static int acc_begin(spg_ctx *c) {
    if (c->acc_open) return 0;
    c->acc_timing = c->timing;
    if (c->acc_timing >= 1) HIPCHK(hipEventRecord(c->ev[c->ring_w % spg_ctx::NRING][0], c->stream));
    c->acc_open = true;
    return 0;
}
static int acc_end(spg_ctx *c) {
    if (c->acc_timing >= 1) HIPCHK(hipEventRecord(c->ev[c->ring_w % spg_ctx::NRING][1], c->stream));
    return 0;
}

// kernels read batch data only after its copy (copy stream) has landed
static int wait_copies(spg_ctx *c) {
    if (!c->copy_pending) return 0;
    HIPCHK(hipStreamWaitEvent(c->stream, c->copy_ev, 0));
    c->copy_pending = false;
    return 0;
}

static void fill_swar(const spg_ctx *c, int32_t &min_bq, int32_t &qlo, uint32_t &kpass, uint32_t &kok) {
    const int mb = c->p.min_base_quality;
    min_bq = mb;
    qlo = std::max(mb, 4);
    kpass = mb <= 0 ? 0x80808080u : (mb >= 128 ? 0u : (uint32_t)(0x80 - mb) * 0x01010101u);
    kok = qlo >= 128 ? 0u : (uint32_t)(0x80 - qlo) * 0x01010101u;
}

// k_acc_seg over one batch (every column of a deep batch; the long columns of a shallow one).  F/O:
// fused with the calls-only finalize (FRESH deep batch, the sample's only one).
static int launch_seg(spg_ctx *c, int64_t idx, bool deep_batch, const FParams *F = nullptr, const Out *O = nullptr,
                      bool listed = false, bool *list_mode = nullptr, uint32_t t_listed = 128u) {
    if (list_mode) *list_mode = false;
    const HistBatch &hb0 = c->hist[(size_t)idx];
    constexpr int64_t target_waves = 16384;
    // Each wave owns G consecutive columns.  A new wave costs a workgroup dispatch (median 1.4 us from
    // the previous wave's end in its slot) and its setup (LUT + CSR offsets, then its first chunk: two
    // memory round trips), so a deep wave gets ~22-30 chunks where that still leaves one grid generation
    // of <= 4,096 waves (16 per CU) to fill the chip; otherwise G targets 16,384 waves.  10,000x: G = 3
    // (interleaved A/B on one box: 109.5 us vs 114.7 us for G = 2, 113.5 us for G = 5).
    int64_t g = std::max<int64_t>(1, (hb0.n_cols + target_waves - 1) / target_waves);
    if (deep_batch) {
        // ~22-30 chunks per wave: G = 3 at both 10,000x (10 chunks a column) and the 8000-capped
        // 7,960x (8 chunks; G = 4 there measured 103.5 vs 95.9 us); 1,000x: G = 16 (list mode below)
        const double avg0 = (double)hb0.n_entries / (double)std::max<int64_t>(1, hb0.n_cols);
        const int64_t g_chunks = (int64_t)std::ceil(22528.0 / std::max(avg0, 1.0));
        const int64_t g_fill = std::max<int64_t>(1, (hb0.n_cols + 4095) / 4096);           // one generation
        g = std::max<int64_t>(g, std::min(g_chunks, g_fill));
    }
    // fused (records kept in the wave's finishing ring for the finalize) only when a wave's columns fit the ring;
    // a wider group finishes its ring NB columns at a time, lists the positions that may call, and the caller
    // runs the sparse k_finalize over them (list mode: mid-depth batches such as 1,000x, G = 16)
    if (F && g > NB_RING && deep_batch && !listed) {
        if (list_mode) *list_mode = true;
        F = nullptr;
        O = nullptr;
    }
    if (F) {
        // finalize parameters in device memory (the kernel reads them after its loop), one copy per
        // Counters slot; they change only when the result buffers grow
        FusedArgs fa[2];
        memset(fa, 0, sizeof fa);               // padding included: compared bytewise below
        for (uint32_t k = 0; k < 2; k++) {
            memcpy(&fa[k].F, F, sizeof *F);
            memcpy(&fa[k].O, O, sizeof *O);
            fa[k].F.epoch = 0;
            fa[k].F.cslot = k;
        }
        if (!c->fused_valid || memcmp(fa, c->h_fused, sizeof fa) != 0) {
            HIPCHK(hipStreamSynchronize(c->stream));        // an earlier upload may still read the staging copy
            memcpy(c->h_fused, fa, sizeof fa);
            HIPCHK(hipMemcpyAsync(c->d_fused, c->h_fused, sizeof fa, hipMemcpyHostToDevice, c->stream));
            c->fused_valid = true;
        }
    }
    const HistBatch &hb = c->hist[(size_t)idx];
    const int64_t n_cols = hb.n_cols;
    // fused: a wave's columns fit its finishing ring (its records stay in LDS for the finalize)
    const uint32_t G = (uint32_t)std::min<int64_t>(F ? NB_RING : (deep_batch ? SPG_GMAX_DEEP : SPG_GMAX), g);
    KParams P{};
    P.pos_begin = hb.pos_begin;
    P.n_cols = n_cols;
    fill_swar(c, P.min_bq, P.qlo, P.kpass, P.kok);
    P.batch_seq = hb.seq0;
    P.fsamp = hb.fsamp;
    P.epoch = c->epoch;
    P.hdesc = Hist{hb.pos_begin, n_cols, hb.off, hb.code, hb.qual};
    P.hslot = c->d_hist + idx;
    P.G = G;
    P.G2 = G;
    P.w1 = (uint32_t)std::min<int64_t>(UINT32_MAX, (n_cols + G - 1) / G);
    // Deep batches with G >= 2: the last grid generation (#CUs x 16 waves) gets groups of G / 2 columns,
    // so the waves that start last end sooner (the launch's tail)
    constexpr int64_t tail_waves = 4096;
    if (deep_batch && G >= 2) {
        const int64_t G2 = G / 2;
        const int64_t tail_cols = std::min<int64_t>(n_cols, tail_waves * G2);
        const int64_t w1 = (n_cols - tail_cols + G - 1) / G;
        if (w1 > 0 && w1 * G < n_cols) {
            P.w1 = (uint32_t)w1;
            P.G2 = (uint32_t)G2;
        }
    }
    int64_t n_launch_waves = 0;
    P.t_deep = deep_batch ? 1u : 128u;
    P.calls_only = (c->p.flags & SPG_P_CALLS_ONLY) ? 1u : 0u;
    P.n_entries = hb.n_entries;
    P.dbg = trace_on() ? trace_dbg() : nullptr;
    if (list_mode && *list_mode) {
        HIPCHK(hipMemsetAsync(c->nlist, 0, sizeof(uint32_t), c->stream));
        P.list = c->band;
        P.n_list = c->nlist;
        P.min_td = c->p.min_total_depth;
        P.min_ad = c->p.min_allele_depth;
        P.ratio_lo = c->p.min_evidence_ratio * (1.0 - 1e-9);
    }
    if (listed) {                 // the long columns the run kernel listed (k_count_cols: every listed column), one per wave
        P.t_deep = t_listed;
        P.G = 1;
        P.G2 = 1;
        P.deep_list = c->deep_list;
        P.deep_n = c->deep_n;
    }
    P.prog = trace_prog(listed ? 2048 * 4 + 4 : std::max<int64_t>(n_launch_waves, 2 * ((n_cols + G - 1) / G) + 4));
    // SPG_WAVE_TIMES=<file> (profiling, tools/wavetimes.py): per-wave timeline of each deep launch
    // appended to <file> (the launch is synchronised)
    static const char *wt_file = getenv("SPG_WAVE_TIMES");
    static uint4 *wt_buf = nullptr;
    static int64_t wt_cap = 0;
    const int64_t n_waves = P.w1 >= (n_cols + G - 1) / G ? (n_cols + G - 1) / G
                                                        : P.w1 + (n_cols - (int64_t)P.w1 * G + P.G2 - 1) / P.G2;
    if (wt_file && deep_batch) {
        if (n_waves > wt_cap) {
            if (wt_buf) HIPCHK(hipFree(wt_buf));
            HIPCHK(hipMalloc(&wt_buf, sizeof(uint4) * n_waves));
            wt_cap = n_waves;
        }
        HIPCHK(hipMemsetAsync(wt_buf, 0, sizeof(uint4) * n_waves, c->stream));
        P.wtime = wt_buf;
    }
    if (F) P.fused = c->d_fused + F->cslot;
    P.min_td = c->p.min_total_depth;
    P.min_ad = c->p.min_allele_depth;
    P.ratio_lo = c->p.min_evidence_ratio * (1.0 - 1e-9);
    HIPCHK(launch_accumulate(P, hb.off, hb.code, hb.qual, c->ref, c->tables, c->acc, c->stream));
    if (P.wtime) {
        std::vector<uint4> h((size_t)n_waves);
        HIPCHK(hipMemcpyAsync(h.data(), P.wtime, sizeof(uint4) * n_waves, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (FILE *f = fopen(wt_file, "ab")) {
            const int64_t hdr[2] = {n_waves, (int64_t)G};
            fwrite(hdr, sizeof hdr, 1, f);
            fwrite(h.data(), sizeof(uint4), h.size(), f);
            fclose(f);
        }
    }
    return trace_sync(c, F ? "accumulate + finalize (k_acc_seg, fused)" : "accumulate (k_acc_seg)");
}

// The deferred deep batch, accumulated on its own (something other than a calls-only finalize of the
// sample needs its records)
static int flush_deep(spg_ctx *c) {
    if (!c->deep_pend) return 0;
    c->deep_pend = false;
    if (int rc = wait_copies(c)) return rc;
    if (int rc = acc_begin(c)) return rc;
    if (int rc = launch_seg(c, 0, true)) return rc;
    return acc_end(c);
}

// How a run of shallow batches [h0, h1) over positions [u0, u1) is folded by k_acc_tile: LPC lanes per
// column so that a tile's bytes of one batch fit a 2 KiB DMA slot (TC = 64 / LPC columns per tile), and the
// batch range split S ways when the tiles alone cannot fill the resident grid (items of equal work: S is the
// smallest split whose last round keeps >= 90 % of the waves busy).
struct RunPlan {
    int lpc;
    int64_t n_groups, S, kper, tc;
};
static int64_t tile_blocks(const spg_ctx *c, int lpc, bool one) {
    return (int64_t)c->n_cu * tile_blocks_per_cu(lpc, one);
}
static RunPlan plan_run(const spg_ctx *c, int64_t h0, int64_t h1, int64_t u0, int64_t u1, uint64_t run_entries) {
    const int64_t K = h1 - h0, L = u1 - u0;
    RunPlan R{1, 0, 1, K, 64};
    // bytes of one batch in a tile: TC x mean column length (whole 16-B blocks around it)
    constexpr double fill = 1984.0;
    const double mean = (double)run_entries / ((double)K * (double)std::max<int64_t>(1, L));
    while (R.lpc < 8 && (64.0 / R.lpc) * mean > fill) R.lpc *= 2;
    R.tc = 64 / R.lpc;
    R.n_groups = (L + R.tc - 1) / R.tc;
    const int64_t waves = tile_blocks(c, R.lpc, false) * 2;
    int64_t best = 1;
    if (K > 1 && R.n_groups < waves) {
        double best_eff = -1.0;
        for (int64_t S = 1; S <= std::min<int64_t>(K, 64); S++) {
            const int64_t kper = (K + S - 1) / S, s_eff = (K + kper - 1) / kper;
            const double items = (double)(R.n_groups * s_eff);
            const double rounds = std::ceil(items / (double)waves);
            const double eff = items / (rounds * (double)waves);
            if (eff > best_eff + 1e-9) { best_eff = eff; best = S; }
            if (eff >= 0.9) { best = S; break; }
        }
    }
    R.kper = (K + best - 1) / best;
    R.S = (K + R.kper - 1) / R.kper;
    return R;
}

// Fold the pending run [pend0, size) into the records: k_acc_tile (+ k_merge_parts when split), and for a
// single batch the long columns through k_acc_seg<1>.
static int flush_run(spg_ctx *c, int64_t h1, bool fused) {
    if (h1 < 0) h1 = (int64_t)c->hist.size();
    const int64_t h0 = c->pend0;
    if (h1 <= h0) return 0;
    const int32_t K = (int32_t)(h1 - h0);
    int64_t u0 = INT64_MAX, u1 = INT64_MIN;
    for (int64_t i = h0; i < h1; i++) {
        u0 = std::min(u0, c->hist[(size_t)i].pos_begin);
        u1 = std::max(u1, c->hist[(size_t)i].pos_begin + c->hist[(size_t)i].n_cols);
    }
    c->pend0 = h1;
    c->pend_entries = 0;
    if (int rc = wait_copies(c)) return rc;
    if (int rc = acc_begin(c)) return rc;
    // descriptors of the run (pinned mirror -> device table)
    HIPCHK(hipMemcpyAsync(c->d_hist + h0, c->h_hist + h0, sizeof(Hist) * K, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipEventRecord(c->hist_ev, c->stream));
    c->hist_up = true;
    uint64_t run_entries = 0;
    for (int64_t i = h0; i < h1; i++) run_entries += c->hist[(size_t)i].n_entries;
    const RunPlan R = plan_run(c, h0, h1, u0, u1, run_entries);
    MParams P{};
    P.u0 = u0;
    P.u1 = u1;
    P.h0 = (int32_t)h0;
    P.K = K;
    P.n_groups = (int32_t)R.n_groups;
    P.S = (int32_t)R.S;
    P.kper = (int32_t)R.kper;
    P.pstride = R.n_groups * R.tc;
    fill_swar(c, P.min_bq, P.qlo, P.kpass, P.kok);
    P.seq0 = c->hist[(size_t)h0].seq0;
    P.epoch = c->epoch;
    P.calls_only = (c->p.flags & SPG_P_CALLS_ONLY) ? 1u : 0u;
    P.t_deep = K == 1 ? 128u : 0u;
    P.fresh = h0 == 0 ? 1u : 0u;
    P.ref_sl = P.calls_only && (double)run_entries < 200.0 * (double)(u1 - u0) ? 1u : 0u;
    P.err = c->kerr;
    c->kerr_dirty = true;
    if (fused) {
        if (K != 1 || h0 != 0 || (double)run_entries > 40.0 * (double)(u1 - u0))
            return fail("spg: internal: a fused run is one FRESH shallow batch (k_acc_lite)");
        P.min_td = c->p.min_total_depth;
        P.min_ad = c->p.min_allele_depth;
        P.ratio_lo = c->p.min_evidence_ratio * (1.0 - 1e-9);
        P.list = c->band;
        P.n_list = c->nlist;
        HIPCHK(hipMemsetAsync(c->nlist, 0, sizeof(uint32_t), c->stream));
    }
    // partial states folded by k_merge_parts: a split run, or (k_acc_tile) any run into records that may
    // already hold this sample's earlier batches
    const bool use_part = P.S > 1 || !P.fresh;
    if (use_part) {
        const size_t need = sizeof(MState) * (size_t)P.S * (size_t)P.pstride;
        if (need > c->part_bytes) {
            if (c->part) { HIPCHK(hipStreamSynchronize(c->stream)); HIPCHK(hipFree(c->part)); }
            c->part = nullptr;
            c->part_bytes = 0;
            HIPCHK(hipMalloc(&c->part, need));
            c->part_bytes = need;
        }
        P.part = c->part;
    }
    if (K == 1) {
        // list of the batch's long columns (each has >= 128 entries: at most E / 128 of them)
        const HistBatch &hb = c->hist[(size_t)h0];
        const int64_t cap = std::min<int64_t>(hb.n_cols, (int64_t)(hb.n_entries / 128) + 1);
        if (cap > c->deep_cap) {
            if (c->deep_list) { HIPCHK(hipStreamSynchronize(c->stream)); HIPCHK(hipFree(c->deep_list)); }
            c->deep_list = nullptr;
            c->deep_cap = 0;
            HIPCHK(hipMalloc(&c->deep_list, sizeof(uint32_t) * cap));
            c->deep_cap = cap;
        }
        HIPCHK(hipMemsetAsync(c->deep_n, 0, sizeof(uint32_t), c->stream));
        P.deep_list = c->deep_list;
        P.deep_n = c->deep_n;
    }
    // a FUSED single shallow batch into a FRESH memory (process_bam + prepare_variants; mean column <= 40
    // entries): k_acc_lite, counts + the exact fold of the columns that may call
    const bool lite = fused;
    if (lite) {
        P.n_groups = (int32_t)((u1 - u0 + 63) / 64);
        HIPCHK(launch_lite(P, c->h_hist[h0], c->ref, c->tables, c->acc, (int64_t)c->n_cu * lite_blocks_per_cu(), c->stream));
        // the listed positions' exact fold (their records; deep columns are k_acc_seg<1>'s below)
        HIPCHK(launch_lite_fold(P, c->h_hist[h0], c->ref, c->tables, c->acc, 2 * (int64_t)c->n_cu, c->stream));
    } else {
        c->path[0]++;
        HIPCHK(launch_tile(P, c->d_hist, c->ref, c->ref_len, c->tables, c->acc, R.lpc, tile_blocks(c, R.lpc, K == 1), c->stream));
        if (use_part) HIPCHK(launch_merge(P, c->ref, c->acc, c->stream));
    }
    if (int rc = trace_sync(c, lite ? "accumulate (k_acc_lite)" : "accumulate (k_acc_tile)")) return rc;
    if (K == 1) {
        // a single shallow batch: its long columns (>= 128 entries), listed by the run kernel, go through the
        // wave-wide kernel
        if (int rc = launch_seg(c, h0, false, nullptr, nullptr, true)) return rc;
    }
    return acc_end(c);
}

// A fused run at spg_finalize wrote records only for positions that could produce a call: before
// anything reads the records again (another batch, the table, a full finalize), fold the run once more
// with every record written.
static int materialize(spg_ctx *c) {
    if (!c->stale) return 0;
    c->stale = false;
    c->counted = false;            // the records hold history [0, stale_end) again; pending batches fold into them
    c->path[1]++;
    if (c->stale_deep) {           // the lone deep batch k_count_cols counted: every column through k_acc_seg
        c->stale_deep = false;
        if (int rc = wait_copies(c)) return rc;
        if (int rc = acc_begin(c)) return rc;
        if (int rc = launch_seg(c, 0, true)) return rc;
        // the listed columns' records again through k_acc_seg<1> (deep_list / deep_n still hold count_cols' list:
        // nothing lists between it and this materialize), so every later finalize reads the very records (fp64
        // sums in the same order) the sparse finalize after the count read: calls stay bit-identical across
        // finalizes, as the reference's prepare_variants over an unchanged memory
        if (int rc = launch_seg(c, 0, false, nullptr, nullptr, true, nullptr, 1u)) return rc;
        return acc_end(c);
    }
    const int64_t keep = c->pend0;
    c->pend0 = 0;
    const int rc = flush_run(c, c->stale_end, false);
    c->pend0 = keep;
    return rc;
}

// Counted mode (count_pending) may take a calls-only sample of shallow single-sample batches whose records are
// not needed as they stand: none written yet (pend0 == 0), or stale (a fused finalize or counted mode left them
// unwritten; counting reads the history, not the records).  vc_queue.py:142-144 finalizes after every BAM: each
// finalize counts (a lone chr1-like batch of <= 40 entries per column takes k_acc_lite instead).
static bool countable(const spg_ctx *c) {
    return (c->p.flags & SPG_P_CALLS_ONLY) && c->n_deep_hist == 0 && !c->deep_pend &&
           (c->counted || c->stale || c->pend0 == 0);
}

static bool is_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
    return a.type == hipMemoryTypeHost;
}
static bool is_device_mem(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
    return a.type == hipMemoryTypeDevice;
}

// One batch: validation, its history copy (arena) or borrowed device buffers, descriptors, bucket
// index; a deep batch is accumulated right away, a shallow one joins the pending run.
// ---- bounded history ------------------------------------------------------------------
// Owned batches live in the device arena so that the exact replay, the counted mode's exact fold and a
// re-materialization can read them.  Past the cap, the oldest batches whose entries are already folded (into
// the records, or into the counted totals) move to pinned host memory: their descriptors then point at the
// mapped host copy, so those rare readers stream the few columns they need over PCIe, and a slab whose
// batches have all moved is freed.
static int count_pending(spg_ctx *c);

static int spill_batch(spg_ctx *c, int64_t i) {
    HistBatch &b = c->hist[(size_t)i];
    void *h = nullptr;
    HIPCHK(hipHostMalloc(&h, b.bytes, hipHostMallocMapped));
    void *hd = nullptr;
    HIPCHK(hipHostGetDevicePointer(&hd, h, 0));
    // after every kernel enqueued so far (some may read the batch), before any later one
    if (int rc = wait_copies(c)) return rc;
    HIPCHK(hipMemcpyAsync(h, b.dev0, b.bytes, hipMemcpyDeviceToHost, c->stream));
    uint8_t *d = (uint8_t *)hd;
    b.code = d + (b.code - b.dev0);
    b.qual = d + (b.qual - b.dev0);
    b.off = reinterpret_cast<uint64_t *>(d + ((uint8_t *)b.off - b.dev0));
    b.host = h;
    // the pinned descriptor mirror: an upload still queued may read it (it would pick up the new pointers
    // before the copy above ran)
    if (c->hist_up) HIPCHK(hipEventSynchronize(c->hist_ev));
    c->h_hist[i] = Hist{b.pos_begin, b.n_cols, b.off, b.code, b.qual};
    HIPCHK(hipMemcpyAsync(c->d_hist + i, c->h_hist + i, sizeof(Hist), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipEventRecord(c->hist_ev, c->stream));
    c->hist_up = true;
    c->hist_dev_bytes -= (int64_t)b.bytes;
    c->n_spilled++;
    Arena::Slab &sl = c->arena.slabs[(size_t)b.slab];
    if (--sl.live == 0 && (size_t)b.slab != c->arena.cur) {
        HIPCHK(hipStreamSynchronize(c->stream));      // the copies out of it have run
        HIPCHK(hipFree(sl.base));
        sl.base = nullptr;
        sl.cap = sl.used = 0;
    }
    b.dev0 = nullptr;
    return 0;
}

static int enforce_history_cap(spg_ctx *c) {
    if (c->hist_cap <= 0 || c->hist_dev_bytes <= c->hist_cap) return 0;
    // batches [0, folded) are in the records / the counted totals
    int64_t folded = c->counted ? c->count_end : c->pend0;
    const int64_t nh = (int64_t)c->hist.size();
    int64_t movable = 0;
    for (int64_t i = 0; i < folded; i++)
        if (c->hist[(size_t)i].dev0 && c->hist[(size_t)i].n_samples == 1) movable += (int64_t)c->hist[(size_t)i].bytes;
    if (c->hist_dev_bytes - movable > c->hist_cap && nh > folded) {
        // fold the pending batches first (all but the newest: it stays pending for the next finalize)
        if (countable(c)) {
            if (int rc = count_pending(c)) return rc;
            folded = c->count_end;
        } else {
            if (int rc = materialize(c)) return rc;
            if (int rc = flush_run(c)) return rc;
            folded = c->pend0;
        }
    }
    for (int64_t i = 0; i < folded && c->hist_dev_bytes > c->hist_cap; i++) {
        const HistBatch &b = c->hist[(size_t)i];
        if (!b.dev0 || b.n_samples != 1) continue;
        if (int rc = spill_batch(c, i)) return rc;
    }
    return 0;
}

static void free_spilled(spg_ctx *c) {
    bool any = false;
    for (auto &b : c->hist) any |= b.host != nullptr;
    if (!any) return;
    (void)hipStreamSynchronize(c->stream);             // kernels reading the mapped copies are done
    for (auto &b : c->hist)
        if (b.host) { (void)hipHostFree(b.host); b.host = nullptr; }
}

// Records batch (spg_accumulate_records): the inflated BAM and its per-read index to HBM, then the device-side
// pileup writes the batch's entries (all on the copy stream, so the batch is ready where a copied one would be).
static int upload_records(spg_ctx *c, const spg_records *R, const HistBatch &hb, hipStream_t cs) {
    const uint64_t n = (uint64_t)R->n_reads, nt = (uint64_t)R->n_tweaks;
    const int64_t n_tiles = (R->n_cols + 63) / 64;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_data = 0, o_rec = al(R->data_bytes + 64), o_pos = al(o_rec + 8 * n), o_end = al(o_pos + 4 * n),
                 o_tw = al(o_end + 4 * n), o_tcol = al(o_tw + 4 * n), o_tq = al(o_tcol + 8 * nt),
                 o_orig = al(o_tq + 8 * nt), o_tf = al(o_orig + R->orig_bytes),
                 need = al(o_tf + fill_scratch_bytes(R->n_cols, (int64_t)n, R->max_span));
    if (need > c->rs_cap) {
        if (c->rs) HIPCHK(hipFree(c->rs));      // (synchronous: the previous fill has run)
        c->rs = nullptr;
        c->rs_cap = need + need / 8;
        HIPCHK(hipMalloc(&c->rs, c->rs_cap));
    }
    uint8_t *m = c->rs;
    const hipMemcpyKind k = hipMemcpyHostToDevice;
    if (R->data_bytes) HIPCHK(hipMemcpyAsync(m + o_data, R->data, R->data_bytes, k, cs));
    HIPCHK(hipMemsetAsync(m + o_data + R->data_bytes, 0, 64, cs));
    if (n) {
        HIPCHK(hipMemcpyAsync(m + o_rec, R->rec, 8 * n, k, cs));
        HIPCHK(hipMemcpyAsync(m + o_pos, R->rpos, 4 * n, k, cs));
        HIPCHK(hipMemcpyAsync(m + o_end, R->rend, 4 * n, k, cs));
        HIPCHK(hipMemcpyAsync(m + o_tw, R->tweak, 4 * n, k, cs));
    }
    if (nt) {
        HIPCHK(hipMemcpyAsync(m + o_tcol, R->tweak_col, 8 * nt, k, cs));
        HIPCHK(hipMemcpyAsync(m + o_tq, R->tweak_qual, 8 * nt, k, cs));
    }
    if (R->orig_bytes) HIPCHK(hipMemcpyAsync(m + o_orig, R->orig_qual, R->orig_bytes, k, cs));
    FillArgs A{};
    A.data = m + o_data;
    A.data_bytes = R->data_bytes;
    A.rec = reinterpret_cast<const uint64_t *>(m + o_rec);
    A.rpos = reinterpret_cast<const int32_t *>(m + o_pos);
    A.rend = reinterpret_cast<const int32_t *>(m + o_end);
    A.tweak = reinterpret_cast<const int32_t *>(m + o_tw);
    A.tw_col = reinterpret_cast<const int64_t *>(m + o_tcol);
    A.tw_q = reinterpret_cast<const uint64_t *>(m + o_tq);
    A.orig = m + o_orig;
    A.orig_bytes = R->orig_bytes;
    A.scratch = m + o_tf;
    A.scratch_bytes = need - o_tf;
    A.off = hb.off;
    A.code = hb.code;
    A.qual = hb.qual;
    A.pos_begin = R->pos_begin + R->pos_origin;     // (the fill compares reference positions)
    A.n_cols = (int32_t)R->n_cols;
    A.n_tiles = (int32_t)n_tiles;
    A.n_reads = (uint32_t)n;
    A.back = (int32_t)((R->max_span + 63) / 64);
    A.err = c->ferr;
    c->ferr_dirty = true;
    HIPCHK(launch_pileup_fill(A, cs));
    return 0;
}

static int add_batch(spg_ctx *c, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                     const uint8_t *base_code, const uint8_t *qual, uint64_t n_entries, uint32_t flags,
                     bool *pageable_copy, int64_t n_samples = 1, const uint32_t *first_sample = nullptr,
                     const spg_records *recs = nullptr, const FillArgs *dfill = nullptr) {
    if (n_samples < 1 || n_samples > (1 << 30)) return fail("spg_accumulate_samples: n_samples out of range");
    constexpr double deep_min = 256.0;
    const bool deep_batch = (n_cols > 0 && (double)n_entries / (double)n_cols >= deep_min) || n_samples > 1 || first_sample;
    // a shallow batch into a countable sample leaves the records stale (it is counted at the next finalize)
    if (deep_batch || n_samples > 1 || !countable(c))
        if (int rc = materialize(c)) return rc;
    if (int rc = flush_deep(c)) return rc;
    if (n_cols < 0 || pos_begin < 0 || pos_begin + n_cols > c->n_pos)
        return fail("spg_accumulate: column range outside the context's positions");
    if (pos_begin + n_cols > c->ref_len)
        return fail("spg_accumulate: column range beyond the reference sequence (IndexError in the reference)");
    if (n_cols == 0) return 0;
    if (!offsets || (n_entries && !recs && !dfill && (!base_code || !qual))) return fail("spg_accumulate: null buffer");
    if (n_entries >= (1ull << 40)) return fail("spg_accumulate: batch too large");
    const bool dev = !recs && !dfill && (flags & SPG_IN_DEVICE);
    const bool borrow = dev && (flags & SPG_IN_BORROW);
    if (!dev && !recs && !dfill && !(flags & SPG_IN_TRUSTED)) {
        // validate the host CSR (offsets O(n_cols), codes O(E)); device inputs are trusted
        if (offsets[0] != 0 || offsets[n_cols] != n_entries)
            return fail("spg_accumulate: offsets[0] must be 0 and offsets[n_cols] == n_entries");
        for (int64_t i = 0; i < n_cols; i++)
            if (offsets[i + 1] < offsets[i]) return fail("spg_accumulate: offsets not monotone");
        uint8_t hi = 0;
        for (uint64_t i = 0; i < n_entries; i++) hi = std::max(hi, base_code[i]);
        if (hi > SPG_CODE_SKIP) {
            for (uint64_t i = 0; i < n_entries; i++)
                if (base_code[i] > SPG_CODE_SKIP) return fail("spg_accumulate: base_code > 17 at entry " + std::to_string(i));
        }
    }
    HistBatch hb{pos_begin, n_cols, n_entries, nullptr, nullptr, nullptr, !borrow, c->batch_seq + 1, n_samples, nullptr};
    if (first_sample && !dev) {
        for (int64_t i = 0; i < n_cols; i++)
            if (first_sample[i] >= (uint64_t)n_samples) return fail("spg_accumulate_samples: first_sample >= n_samples");
    }
    if (borrow) {
        hb.off = const_cast<uint64_t *>(offsets);
        hb.code = const_cast<uint8_t *>(base_code);
        hb.qual = const_cast<uint8_t *>(qual);
        hb.fsamp = const_cast<uint32_t *>(first_sample);
    } else {
        const size_t pad = (n_entries + 16 + 15) & ~size_t(15);
        uint8_t *m = nullptr;
        if (c->arena_fence) {
            HIPCHK(hipEventRecord(c->compute_ev, c->stream));
            HIPCHK(hipStreamWaitEvent(c->copy_stream, c->compute_ev, 0));
            c->arena_fence = false;
        }
        hb.bytes = sizeof(uint64_t) * (n_cols + 1) + 2 * pad;
        HIPCHK(c->arena.alloc(hb.bytes, &m, &hb.slab));
        hb.dev0 = m;
        c->hist_dev_bytes += (int64_t)hb.bytes;
        hb.code = m;
        hb.qual = m + pad;
        hb.off = reinterpret_cast<uint64_t *>(m + 2 * pad);
        const hipMemcpyKind k = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
        hipStream_t cs = c->copy_stream;
        // (a device plan's offsets are in HBM: spg_bam_plan_build)
        HIPCHK(hipMemcpyAsync(hb.off, offsets, sizeof(uint64_t) * (n_cols + 1), dfill ? hipMemcpyDefault : k, cs));
        if (recs) {
            if (int rc = upload_records(c, recs, hb, cs)) return rc;
        } else if (dfill) {                    // spg_bam_accumulate: the records are in HBM already
            FillArgs A = *dfill;
            A.off = hb.off;
            A.code = hb.code;
            A.qual = hb.qual;
            A.err = c->ferr;
            c->ferr_dirty = true;
            HIPCHK(launch_pileup_fill(A, cs));
        } else if (n_entries) {
            HIPCHK(hipMemcpyAsync(hb.code, base_code, n_entries, k, cs));
            HIPCHK(hipMemcpyAsync(hb.qual, qual, n_entries, k, cs));
        }
        HIPCHK(hipMemsetAsync(hb.code + n_entries, 0xFF, pad - n_entries, cs));
        HIPCHK(hipMemsetAsync(hb.qual + n_entries, 0, pad - n_entries, cs));
        if (first_sample) {
            uint8_t *fs = nullptr;
            int fslab = -1;
            HIPCHK(c->arena.alloc(sizeof(uint32_t) * n_cols, &fs, &fslab));
            hb.fsamp = reinterpret_cast<uint32_t *>(fs);
            HIPCHK(hipMemcpyAsync(hb.fsamp, first_sample, sizeof(uint32_t) * n_cols, k, cs));
        }
        HIPCHK(hipEventRecord(c->copy_ev, cs));
        HIPCHK(hipEventRecord(c->in_ev[c->in_seq % spg_ctx::NIN], cs));
        c->in_seq++;
        c->copy_pending = true;
        // pageable host buffers are the caller's again on return; pinned ones after spg_wait_input
        if (recs) {
            if (!(is_pinned(offsets) && (!recs->data_bytes || is_pinned(recs->data)) && (!recs->n_reads || is_pinned(recs->rec))))
                *pageable_copy = true;
        } else if (dfill) {
            if (!is_pinned(offsets) && !is_device_mem(offsets)) *pageable_copy = true;
        } else if (!dev && !(is_pinned(offsets) && (!n_entries || (is_pinned(base_code) && is_pinned(qual))))) {
            *pageable_copy = true;
        }
    }
    c->hist.push_back(hb);
    const int64_t idx = (int64_t)c->hist.size() - 1;
    if (int rc = grow_history_table(c)) return rc;
    if (c->hist_fence) {       // the previous sample's last upload may still read these mirror entries
        HIPCHK(hipEventSynchronize(c->hist_ev));
        c->hist_fence = false;
        c->hist_up = false;
    }
    c->h_hist[idx] = Hist{pos_begin, n_cols, hb.off, hb.code, hb.qual};
    for (int64_t b = pos_begin >> RIDX_SHIFT; b <= (pos_begin + n_cols - 1) >> RIDX_SHIFT; b++) {
        c->buckets[(size_t)b].push_back((int32_t)idx);
        c->ridx_items++;
    }
    c->ridx_dirty = true;
    c->batch_seq += (uint32_t)n_samples;
    c->finalized = false;
    if (deep_batch) {
        c->n_deep_hist++;
        // a deep (or multi-sample) batch: the run before it first (accumulate order), then k_acc_seg on
        // its own (a run folds single-sample batches with consecutive batch numbers)
        if (int rc = flush_run(c, idx)) return rc;
        c->pend0 = idx + 1;
        if (idx == 0 && (c->p.flags & SPG_P_CALLS_ONLY)) {
            c->deep_pend = true;               // the sample's first batch: launched by spg_finalize
            return 0;
        }
        if (int rc = wait_copies(c)) return rc;
        if (int rc = acc_begin(c)) return rc;
        if (int rc = launch_seg(c, idx, true)) return rc;
        if (int rc = acc_end(c)) return rc;
        return enforce_history_cap(c);         // every batch is folded now: any of them may move
    }
    c->pend_entries += n_entries;
    // (calls-only: the pending run waits for the finalize, which counts it — see finalize_counted)
    constexpr int64_t run_max = 4096;
    if (!(c->p.flags & SPG_P_CALLS_ONLY) && (int64_t)c->hist.size() - c->pend0 >= run_max)
        if (int rc = flush_run(c)) return rc;
    return enforce_history_cap(c);
}

static int accumulate_many(spg_ctx *c, const spg_batch *b, int64_t n, uint32_t flags) {
    if (!c) return fail("spg_accumulate: null ctx");
    if (!c->lut_set) return fail("spg_accumulate: spg_set_eps_lut not called");
    if (!c->ref) return fail("spg_accumulate: spg_set_reference not called");
    if (n < 0 || (n > 0 && !b)) return fail("spg_accumulate_batches: bad batch list");
    HIPCHK(hipSetDevice(c->device));
    bool pageable = false;
    int rc = 0;
    for (int64_t i = 0; i < n && rc == 0; i++)
        rc = add_batch(c, b[i].pos_begin, b[i].n_cols, b[i].offsets, b[i].base_code, b[i].qual, b[i].n_entries,
                       flags, &pageable);
    if (pageable) HIPCHK(hipStreamSynchronize(c->copy_stream));
    return rc;
}

int spg_accumulate_ex(spg_ctx *c, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                      const uint8_t *base_code, const uint8_t *qual, uint64_t n_entries, uint32_t flags) {
    const spg_batch b{pos_begin, n_cols, offsets, base_code, qual, n_entries};
    return accumulate_many(c, &b, 1, flags);
}

int spg_accumulate(spg_ctx *c, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets, const uint8_t *base_code,
                   const uint8_t *qual, uint64_t n_entries) {
    return spg_accumulate_ex(c, pos_begin, n_cols, offsets, base_code, qual, n_entries, 0);
}

int spg_accumulate_batches(spg_ctx *c, const spg_batch *batches, int64_t n, uint32_t flags) {
    return accumulate_many(c, batches, n, flags);
}

int spg_accumulate_samples(spg_ctx *c, int64_t pos_begin, int64_t n_cols, int64_t n_samples, const uint64_t *offsets,
                           const uint32_t *first_sample, const uint8_t *base_code, const uint8_t *qual,
                           uint64_t n_entries, uint32_t flags) {
    if (!c) return fail("spg_accumulate_samples: null ctx");
    if (!c->lut_set) return fail("spg_accumulate: spg_set_eps_lut not called");
    if (!c->ref) return fail("spg_accumulate: spg_set_reference not called");
    HIPCHK(hipSetDevice(c->device));
    bool pageable = false;
    int rc = add_batch(c, pos_begin, n_cols, offsets, base_code, qual, n_entries, flags, &pageable, n_samples,
                       first_sample);
    if (pageable) HIPCHK(hipStreamSynchronize(c->copy_stream));
    return rc;
}

int spg_accumulate_records(spg_ctx *c, const spg_records *r, uint32_t flags) {
    if (!c || !r) return fail("spg_accumulate_records: null argument");
    if (!c->lut_set) return fail("spg_accumulate: spg_set_eps_lut not called");
    if (!c->ref) return fail("spg_accumulate: spg_set_reference not called");
    if (r->n_cols < 0 || r->n_cols > ((int64_t)1 << 31) - 128) return fail("spg_accumulate_records: n_cols out of range");
    if (r->n_reads < 0 || r->n_reads >= ((int64_t)1 << 31)) return fail("spg_accumulate_records: n_reads out of range");
    if (r->n_tweaks < 0 || r->n_tweaks > r->n_reads || r->max_span < 0 || r->pos_origin < 0)
        return fail("spg_accumulate_records: bad tweak count / span / origin");
    if (r->n_cols > 0 && (!r->offsets || (r->n_reads && (!r->data || !r->rec || !r->rpos || !r->rend || !r->tweak)) ||
                          (r->n_tweaks && (!r->tweak_col || !r->tweak_qual || (r->orig_bytes && !r->orig_qual)))))
        return fail("spg_accumulate_records: null buffer");
    if (r->n_cols > 0 && (r->offsets[0] != 0 || r->offsets[r->n_cols] != r->n_entries))
        return fail("spg_accumulate_records: offsets[0] must be 0 and offsets[n_cols] == n_entries");
    // the fill writes column c's entries at [offsets[c], offsets[c + 1]) and reads each read's fixed fields at
    // rec[i] + 0..35: both bounded here (O(n_cols + n_reads) branch-free scans)
    if (r->n_cols > 0) {
        uint64_t desc = 0;
        for (int64_t i = 0; i < r->n_cols; i++) desc |= (uint64_t)(r->offsets[i + 1] < r->offsets[i]);
        if (desc) return fail("spg_accumulate_records: offsets not monotone");
    }
    if (r->n_reads > 0) {
        uint64_t hi = 0;
        int32_t thi = -1;
        for (int64_t i = 0; i < r->n_reads; i++) {
            hi = std::max(hi, r->rec[i]);
            thi = std::max(thi, r->tweak[i]);
        }
        if (r->data_bytes < 36 || hi > r->data_bytes - 36)
            return fail("spg_accumulate_records: a record offset points past the records buffer");
        if (thi >= (int32_t)r->n_tweaks) return fail("spg_accumulate_records: tweak index >= n_tweaks");
    }
    (void)flags;
    HIPCHK(hipSetDevice(c->device));
    bool pageable = false;
    int rc = add_batch(c, r->pos_begin, r->n_cols, r->offsets, nullptr, nullptr, r->n_entries, SPG_IN_TRUSTED, &pageable,
                       1, nullptr, r);
    if (pageable) HIPCHK(hipStreamSynchronize(c->copy_stream));
    return rc;
}

int spg_history_samples(spg_ctx *c, int64_t i, int64_t *n_samples, uint32_t *first_sample) {
    if (!c) return fail("spg_history_samples: null ctx");
    if (i < 0 || i >= (int64_t)c->hist.size()) return fail("spg_history_samples: batch index out of range");
    HIPCHK(hipSetDevice(c->device));
    const HistBatch &h = c->hist[(size_t)i];
    if (n_samples) *n_samples = h.n_samples;
    if (first_sample) {
        if (h.fsamp) {
            if (int rc = wait_copies(c)) return rc;
            HIPCHK(hipMemcpyAsync(first_sample, h.fsamp, sizeof(uint32_t) * h.n_cols, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
        } else {
            memset(first_sample, 0, sizeof(uint32_t) * h.n_cols);
        }
    }
    return 0;
}

int spg_input_ticket(spg_ctx *c, uint64_t *ticket) {
    if (!c || !ticket) return fail("spg_input_ticket: null argument");
    *ticket = c->in_seq;
    return 0;
}

int spg_wait_ticket(spg_ctx *c, uint64_t ticket) {
    if (!c) return fail("spg_wait_ticket: null ctx");
    if (ticket == 0) return 0;
    if (ticket > c->in_seq) return fail("spg_wait_ticket: ticket from the future");
    HIPCHK(hipSetDevice(c->device));
    // the ring slot of copy #ticket; if it has been re-recorded since, the wait covers a later copy too
    HIPCHK(hipEventSynchronize(c->in_ev[(ticket - 1) % spg_ctx::NIN]));
    return 0;
}

int spg_wait_input(spg_ctx *c) {
    if (!c) return fail("spg_wait_input: null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->copy_stream));
    return 0;
}

// Replay index upload: CSR of the bucket lists (only when more than a few batches are kept: with
// few, the replay scans them all).
static int upload_ridx(spg_ctx *c, RIndex &R) {
    R = RIndex{nullptr, nullptr, 0};
    if ((int64_t)c->hist.size() <= 8) return 0;
    if (c->ridx_dirty || !c->ridx_valid) {
        const int64_t nb = (int64_t)c->buckets.size();
        const size_t words = (size_t)(nb + 1 + c->ridx_items);
        if (c->h_ridx) HIPCHK(hipEventSynchronize(c->ridx_ev));   // the previous upload has read it
        if (words > c->ridx_cap) {
            size_t cap = std::max<size_t>(words, c->ridx_cap * 2);
            if (c->h_ridx) HIPCHK(hipHostFree(c->h_ridx));
            if (c->d_ridx) { HIPCHK(hipStreamSynchronize(c->stream)); HIPCHK(hipFree(c->d_ridx)); }
            c->h_ridx = nullptr;
            c->d_ridx = nullptr;
            c->ridx_cap = 0;
            HIPCHK(hipHostMalloc((void **)&c->h_ridx, sizeof(uint32_t) * cap, hipHostMallocDefault));
            HIPCHK(hipMalloc(&c->d_ridx, sizeof(uint32_t) * cap));
            c->ridx_cap = cap;
        }
        uint32_t *off = c->h_ridx;
        int32_t *items = reinterpret_cast<int32_t *>(c->h_ridx + nb + 1);
        uint32_t at = 0;
        for (int64_t b = 0; b < nb; b++) {
            off[b] = at;
            for (int32_t i : c->buckets[(size_t)b]) items[at++] = i;
        }
        off[nb] = at;
        HIPCHK(hipMemcpyAsync(c->d_ridx, c->h_ridx, sizeof(uint32_t) * words, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipEventRecord(c->ridx_ev, c->stream));
        c->ridx_dirty = false;
        c->ridx_valid = true;
    }
    R.off = c->d_ridx;
    R.items = reinterpret_cast<const int32_t *>(c->d_ridx + c->buckets.size() + 1);
    R.n_buckets = (int64_t)c->buckets.size();
    return 0;
}

static Out make_out(spg_ctx *c) {
    Out O;
    O.depth = c->o_depth; O.counts = c->o_counts; O.order = c->o_order; O.first = c->o_first;
    O.gl = c->o_gl; O.flags = c->o_flags; O.cand = c->cand; O.band = c->band; O.detail = c->detail;
    O.ctr = c->ctr;
    return O;
}

static FParams make_fparams(spg_ctx *c) {
    FParams F{};
    F.n_pos = c->n_pos;
    F.min_td = c->p.min_total_depth;
    F.min_ad = c->p.min_allele_depth;
    F.ratio = c->p.min_evidence_ratio;
    F.cand_cap = c->cand_cap;
    F.band_cap = c->band_cap;
    F.detail_cap = c->detail_cap;
    F.min_bq = c->p.min_base_quality;
    F.n_hist = (int32_t)c->hist.size();
    F.epoch = c->epoch;
    F.cslot = c->cslot;
    return F;
}

// Counted mode (a calls-only finalize of a sample of shallow batches, e.g. one process_bam per BAM): count the
// batches not counted yet into the per-position totals (k_acc_lite_run), list the positions whose totals can
// pass prepare_variants' filters (k_count_list), build their records exactly from the whole history
// (k_fold_hist); the sparse finalize then decides them.  The other records stay stale (materialize() re-folds
// the history if anything reads them).
static int count_pending(spg_ctx *c) {
    const int64_t nh = (int64_t)c->hist.size();
    if (!c->counted) {
        if (!c->cdep) {
            HIPCHK(hipMalloc(&c->cdep, sizeof(uint32_t) * c->n_pos));
            HIPCHK(hipMalloc(&c->cmcf, sizeof(uint32_t) * c->n_pos));
            HIPCHK(hipMalloc(&c->fwm, sizeof(uint64_t) * c->n_pos));
            HIPCHK(hipMemsetAsync(c->fwm, 0, sizeof(uint64_t) * c->n_pos, c->stream));
        }
        // a new counted run: records folded before it (by other paths) carry no watermark of this generation
        if (++c->count_gen == 0) {
            HIPCHK(hipMemsetAsync(c->fwm, 0, sizeof(uint64_t) * c->n_pos, c->stream));
            c->count_gen = 1;
        }
        HIPCHK(hipMemsetAsync(c->cdep, 0, sizeof(uint32_t) * c->n_pos, c->stream));
        HIPCHK(hipMemsetAsync(c->cmcf, 0, sizeof(uint32_t) * c->n_pos, c->stream));
        c->count_end = 0;
    }
    const int64_t h0 = c->count_end;
    int64_t u0 = INT64_MAX, u1 = INT64_MIN;            // positions of the batches counted now
    uint64_t run_entries = 0;
    for (int64_t i = h0; i < nh; i++) {
        const HistBatch &b = c->hist[(size_t)i];
        u0 = std::min(u0, b.pos_begin);
        u1 = std::max(u1, b.pos_begin + b.n_cols);
        run_entries += b.n_entries;
    }
    if (int rc = wait_copies(c)) return rc;
    if (int rc = acc_begin(c)) return rc;
    // descriptors of every batch not uploaded yet (pinned mirror -> device table)
    const int64_t up0 = std::min(h0, c->pend0);
    if (nh > up0) {
        if (c->hist_fence) { HIPCHK(hipEventSynchronize(c->hist_ev)); c->hist_fence = false; }
        HIPCHK(hipMemcpyAsync(c->d_hist + up0, c->h_hist + up0, sizeof(Hist) * (nh - up0), hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipEventRecord(c->hist_ev, c->stream));
        c->hist_up = true;
    }
    if (nh > h0) {
        // one wave per (tile, batch split): LPC lanes per column so that a tile's bytes of one batch fit the
        // 3 KiB slot; splits until the items fill the resident grid twice over
        MParams P{};
        fill_swar(c, P.min_bq, P.qlo, P.kpass, P.kok);
        const int64_t K = nh - h0, L = u1 - u0;
        const double mean = (double)run_entries / ((double)K * (double)std::max<int64_t>(1, L));
        // (LPC 2 stages 4 KiB per array: up to ~3,500 B of a batch per 32-column tile)
        int lpc = 1;
        while (lpc < 8 && (64.0 / lpc) * mean > (lpc == 2 ? 3500.0 : 2200.0)) lpc *= 2;
        const int64_t tc = lpc ? 64 / lpc : 64, n_tiles = (L + tc - 1) / tc;
        const int64_t blocks = (int64_t)c->n_cu * count_run_blocks_per_cu(lpc);
        const int64_t want_items = 2 * blocks * 4;
        const int64_t S = std::min<int64_t>(K, std::max<int64_t>(1, (want_items + n_tiles - 1) / n_tiles));
        P.u0 = u0;
        P.u1 = u1;
        P.h0 = (int32_t)h0;
        P.K = (int32_t)K;
        P.kper = (int32_t)((K + S - 1) / S);
        P.S = (int32_t)((K + P.kper - 1) / P.kper);
        P.n_groups = (int32_t)n_tiles;
        HIPCHK(launch_count_run(P, c->d_hist, c->ref, c->cdep, c->cmcf, lpc, blocks, c->stream));
        c->path[7] += K;
        if (int rc = trace_sync(c, "accumulate (k_acc_lite_run)")) return rc;
    }
    c->count_end = nh;
    c->counted = true;
    c->pend0 = nh;
    c->pend_entries = 0;
    c->stale = true;                   // records of history [0, nh) are not written
    c->stale_end = nh;
    return acc_end(c);
}

// Counted mode (a calls-only finalize of a sample of shallow batches, e.g. one process_bam per BAM): count the
// batches not counted yet into the per-position totals (k_acc_lite_run), list the positions whose totals can
// pass prepare_variants' filters (k_count_list), build their records exactly from the whole history
// (k_fold_hist); the sparse finalize then decides them.  The other records stay stale (materialize() re-folds
// the history if anything reads them).
static int finalize_counted(spg_ctx *c) {
    if (int rc = count_pending(c)) return rc;
    const int64_t nh = (int64_t)c->hist.size();
    int64_t ua = INT64_MAX, ub = INT64_MIN;            // positions of the whole history (listing)
    for (int64_t i = 0; i < nh; i++) {
        const HistBatch &b = c->hist[(size_t)i];
        ua = std::min(ua, b.pos_begin);
        ub = std::max(ub, b.pos_begin + b.n_cols);
    }
    if (int rc = acc_begin(c)) return rc;
    MParams P{};
    fill_swar(c, P.min_bq, P.qlo, P.kpass, P.kok);
    P.epoch = c->epoch;
    P.calls_only = 1u;
    P.min_td = c->p.min_total_depth;
    P.min_ad = c->p.min_allele_depth;
    P.ratio_lo = c->p.min_evidence_ratio * (1.0 - 1e-9);
    P.list = c->band;
    P.n_list = c->nlist;
    P.wm = c->fwm;
    P.wm_gen = c->count_gen;
    // list, then the exact records of the listed positions over the whole history (incremental: a listed
    // position's record from an earlier counted finalize takes only the batches since)
    HIPCHK(hipMemsetAsync(c->nlist, 0, sizeof(uint32_t), c->stream));
    P.u0 = ua;
    P.u1 = ub;
    HIPCHK(launch_count_list(P, c->ref, c->cdep, c->cmcf, c->stream));
    P.h0 = 0;
    P.K = (int32_t)nh;
    P.seq0 = c->hist[0].seq0;
    // thousands of batches: up to 8 workgroups per listed position (the first FOLD_CAP of them), so a few dozen
    // positions still spread over the chip
    constexpr int FOLD_BPP = 8, FOLD_CAP = 4096;
    const int bpp = (int)std::min<int64_t>(FOLD_BPP, nh / 1024);
    if (bpp > 1 && !c->fold_part) {
        HIPCHK(hipMalloc(&c->fold_part, fold_part_bytes() * FOLD_BPP * FOLD_CAP));
        HIPCHK(hipMalloc(&c->fold_arrived, sizeof(uint32_t) * FOLD_CAP));
        HIPCHK(hipMemsetAsync(c->fold_arrived, 0, sizeof(uint32_t) * FOLD_CAP, c->stream));
    }
    HIPCHK(launch_fold_hist(P, c->d_hist, c->ref, c->tables, c->acc, 4 * (int64_t)c->n_cu, bpp > 1 ? c->fold_part : nullptr,
                            c->fold_arrived, bpp, FOLD_CAP, c->stream));
    if (int rc = trace_sync(c, "accumulate (k_fold_hist)")) return rc;
    return acc_end(c);
}

static int finalize_impl(spg_ctx *c, bool table);

// k_count_cols' lanes per column for the sample's lone deep batch (0: the fused k_acc_seg takes it).  Mid-depth
// single-sample batches (mean column < 4,096 entries, e.g. 1,000x) are counted: the fused kernel's waves would own
// more columns than its finishing ring holds, and its per-column work dominates at one or two chunks a column.
// SPG_COUNT_COLS=0 disables, =1 takes every lone deep batch (A/B; 10,000x: 127 us vs the fused kernel's 111 us).
// LPC: two or three 16-B blocks per lane (SPG_COUNT_LPC forces one: tests).
static int mid_count_lpc(const spg_ctx *c) {
    const char *me = getenv("SPG_COUNT_COLS");        // (read per call: tests compare both paths)
    const int mode = me ? atoi(me) : -1;
    if (mode == 0 || c->hist.empty()) return 0;
    const HistBatch &b = c->hist[0];
    if (b.n_samples != 1 || b.fsamp || b.n_cols == 0) return 0;
    const double mean = (double)b.n_entries / (double)b.n_cols;
    if (mode != 1 && mean >= 4096.0) return 0;
    const int64_t force = env_i64("SPG_COUNT_LPC", 0);          // (read per call: tests switch it)
    if (force == 4 || force == 8 || force == 16 || force == 32 || force == 64) return (int)force;
    int lpc = 4;                        // (1,000x: LPC 32, two rounds: 0.683 ms vs 0.714 ms for LPC 16, r04l)
    while (lpc < 64 && mean / 16.0 / lpc > 2.5) lpc *= 2;
    return lpc;
}

// The lone deep batch of a calls-only sample at its finalize, counted (mid_count_lpc): k_count_cols lists the positions
// whose counts pass prepare_variants' filters (band: positions; deep_list: columns; deep_n: their number), then
// k_acc_seg<1> builds exactly those records (FRESH).  The batch's records are left stale.
static int count_cols(spg_ctx *c) {
    const HistBatch &hb = c->hist[0];
    const int lpc = mid_count_lpc(c);
    if (hb.n_cols > c->deep_cap) {
        if (c->deep_list) { HIPCHK(hipStreamSynchronize(c->stream)); HIPCHK(hipFree(c->deep_list)); }
        c->deep_list = nullptr;
        c->deep_cap = 0;
        HIPCHK(hipMalloc(&c->deep_list, sizeof(uint32_t) * hb.n_cols));
        c->deep_cap = hb.n_cols;
    }
    if (int rc = wait_copies(c)) return rc;
    if (int rc = acc_begin(c)) return rc;
    HIPCHK(hipMemsetAsync(c->deep_n, 0, sizeof(uint32_t), c->stream));
    MParams P{};
    fill_swar(c, P.min_bq, P.qlo, P.kpass, P.kok);
    P.epoch = c->epoch;
    P.calls_only = 1u;
    P.min_td = c->p.min_total_depth;
    P.min_ad = c->p.min_allele_depth;
    P.ratio_lo = c->p.min_evidence_ratio * (1.0 - 1e-9);
    P.list = c->band;
    P.n_list = c->deep_n;
    const int64_t blocks = (int64_t)c->n_cu * count_cols_blocks_per_cu(lpc);
    HIPCHK(launch_count_cols(P, c->h_hist[0], c->ref, c->deep_list, lpc, blocks, c->stream));
    if (int rc = trace_sync(c, "accumulate (k_count_cols)")) return rc;
    // the listed columns' records (every listed column, whatever its length: t_deep 1)
    if (int rc = launch_seg(c, 0, false, nullptr, nullptr, true, nullptr, 1u)) return rc;
    if (int rc = acc_end(c)) return rc;
    c->stale = true;
    c->stale_deep = true;
    c->stale_end = 1;
    return 0;
}

// The replay cache for a finalize: a history of >= 16 batches (a live memory) keeps each replayed position's exact
// fold state, so its next replay folds only the batches added since (RSlot, spg_device.h)
static int replay_cache(spg_ctx *c, RCache &rc) {
    rc = RCache{nullptr, 0, 0};
    if ((int64_t)c->hist.size() < 16) return 0;
    if (!c->rcache) {
        HIPCHK(hipMalloc(&c->rcache, sizeof(RSlot) * RCACHE_SLOTS));
        HIPCHK(hipMemsetAsync(c->rcache, 0, sizeof(RSlot) * RCACHE_SLOTS, c->stream));
    }
    rc = RCache{c->rcache, (uint32_t)RCACHE_SLOTS - 1, 0};
    return 0;
}

int spg_finalize(spg_ctx *c) {
    if (!c) return fail("spg_finalize: null ctx");
    // calls-only contexts write the per-position table lazily (spg_get_table)
    return finalize_impl(c, !(c->p.flags & SPG_P_CALLS_ONLY));
}

static int finalize_impl(spg_ctx *c, bool table) {
    if (!c->lut_set) return fail("spg_finalize: spg_set_eps_lut not called");
    HIPCHK(hipSetDevice(c->device));
    // A calls-only finalize of a sample whose every batch is still pending (one FRESH run): fold and
    // pre-filter in one pass, finalize only the listed positions.  Otherwise: records complete, every
    // position.
    const int64_t nh = (int64_t)c->hist.size();
    // one deep batch pending: accumulate + finalize in one launch
    const bool fused_deep = !table && c->deep_pend && nh == 1;
    if (!fused_deep)
        if (int rc = flush_deep(c)) return rc;
    // a calls-only sample of shallow batches is counted — except a lone batch of <= 40 entries per column (chr1 30x:
    // one process_bam then prepare_variants), which k_acc_lite counts and folds in one pass
    const bool lone_lite = nh == 1 && c->pend0 == 0 &&
                           (double)c->hist[0].n_entries <= 40.0 * (double)std::max<int64_t>(1, c->hist[0].n_cols);
    const bool counted = !fused_deep && !table && nh >= 1 && !lone_lite && countable(c);
    const bool fused = !counted && !fused_deep && !table && (c->p.flags & SPG_P_CALLS_ONLY) && lone_lite;
    if (fused_deep) {
        c->deep_pend = false;
        c->path[5]++;
    } else if (counted) {
        if (int rc = finalize_counted(c)) return rc;
        c->path[4]++;
    } else if (fused) {
        c->path[6]++;
        if (int rc = flush_run(c, -1, true)) return rc;
        c->stale = true;
        c->stale_end = nh;
    } else {
        if (int rc = materialize(c)) return rc;
        if (int rc = flush_run(c)) return rc;     // the pending run of shallow batches
    }
    c->cslot ^= 1u;            // this call counts in slot cslot (zeroed by the previous call / creation)
    hipEvent_t *ev = c->ev[c->ring_w % spg_ctx::NRING];
    if (!c->acc_open && !fused_deep) {   // no accumulate since the last finalize: empty accumulate interval
        c->acc_timing = c->timing;
        if (c->acc_timing >= 1) {
            HIPCHK(hipEventRecord(ev[0], c->stream));
            HIPCHK(hipEventRecord(ev[1], c->stream));
        }
    }
    const int ft = c->timing;
    FParams F = make_fparams(c);
    F.table = table ? 1u : 0u;
    if (fused_deep && mid_count_lpc(c) > 0) {
        // a lone mid-depth batch (1,000x): k_count_cols counts every column and lists the positions that may
        // call, k_acc_seg<1> folds exactly the listed columns' records, the sparse k_finalize decides them; the
        // other records stay stale (materialize() accumulates the batch through k_acc_seg if anything reads them)
        if (int rc = count_cols(c)) return rc;
        if (ft >= 2) HIPCHK(hipEventRecord(ev[2], c->stream));
        F.list = c->band;
        F.n_list = c->deep_n;
        c->path[3]++;
        c->path[8]++;
        if (int rc = upload_ridx(c, F.ridx)) return rc;
        if (int rc = replay_cache(c, F.rc)) return rc;
        HIPCHK(launch_finalize(F, c->acc, c->tables, make_out(c), c->d_hist, c->stream));
        if (trace_sync(c, "finalize (sparse, listed by k_count_cols)")) return -1;
    } else if (fused_deep) {
        // the accumulate interval holds the fused kernel; the finalize interval is empty (list mode: the sparse
        // k_finalize over the positions the accumulate listed)
        const Out O = make_out(c);
        if (int rc = wait_copies(c)) return rc;
        if (int rc = acc_begin(c)) return rc;
        bool list_mode = false;
        if (int rc = launch_seg(c, 0, true, &F, &O, false, &list_mode)) return rc;
        if (int rc = acc_end(c)) return rc;
        if (ft >= 2) HIPCHK(hipEventRecord(ev[2], c->stream));
        if (list_mode) {
            F.list = c->band;
            F.n_list = c->nlist;
            c->path[3]++;
            if (int rc = upload_ridx(c, F.ridx)) return rc;
            if (int rc = replay_cache(c, F.rc)) return rc;
            HIPCHK(launch_finalize(F, c->acc, c->tables, make_out(c), c->d_hist, c->stream));
            if (trace_sync(c, "finalize (sparse, listed by k_acc_seg)")) return -1;
        }
    } else {
        if (ft >= 2) HIPCHK(hipEventRecord(ev[2], c->stream));
        if (fused || counted) { F.list = c->band; F.n_list = c->nlist; }
        c->path[(fused || counted) ? 3 : 2]++;
        if (int rc = upload_ridx(c, F.ridx)) return rc;
        if (int rc = replay_cache(c, F.rc)) return rc;
        HIPCHK(launch_finalize(F, c->acc, c->tables, make_out(c), c->d_hist, c->stream));
        if (trace_sync(c, "finalize")) return -1;
    }
    c->table_valid = table;
    if (ft >= 2) HIPCHK(hipEventRecord(ev[3], c->stream));
    c->last_acc = c->acc_open && c->acc_timing >= 1;
    c->last_fin = ft >= 2;
    c->ring_tm[c->ring_w % spg_ctx::NRING] = (c->last_acc ? 1 : 0) | (c->last_fin ? 2 : 0);
    c->acc_open = false;
    c->ring_w++;
    if (c->ring_w - c->ring_r > spg_ctx::NRING) c->ring_r = c->ring_w - spg_ctx::NRING;
    c->finalized = true;
    return 0;
}

int spg_stream(spg_ctx *c, void **stream) {
    if (!c || !stream) return fail("spg_stream: null argument");
    *stream = (void *)c->stream;
    return 0;
}

int spg_sync(spg_ctx *c) {
    if (!c) return fail("spg_sync: null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->copy_stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

// Grow the candidate / detail buffers and re-run finalize when the last one overflowed.
static int settle(spg_ctx *c, Counters &h) {
    if (!c->finalized) return fail("spg: spg_finalize has not been called since the last accumulate/reset");
    HIPCHK(hipSetDevice(c->device));
    for (int iter = 0; iter < 4; iter++) {
        HIPCHK(hipMemcpyAsync(&h, c->ctr + c->cslot, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (h.err) return fail("spg: replay found a depth mismatch between history and accumulators");
        if (c->ferr_dirty) {
            // every records fill enqueued so far has run (the ones this finalize read, and any enqueued since)
            uint32_t ferr = 0;
            HIPCHK(hipMemcpyAsync(&ferr, c->ferr, sizeof(ferr), hipMemcpyDeviceToHost, c->copy_stream));
            HIPCHK(hipStreamSynchronize(c->copy_stream));
            c->ferr_dirty = false;
            if (ferr) {
                HIPCHK(hipMemsetAsync(c->ferr, 0, sizeof(uint32_t), c->copy_stream));   // reported once
                return fail("spg: spg_accumulate_records: the records disagree with the batch's offsets (inconsistent plan)");
            }
        }
        uint32_t kerr = 0;
        HIPCHK(hipMemcpyAsync(&kerr, c->kerr, sizeof(kerr), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        c->kerr_dirty = false;         // the stream is idle: zero, or cleared below (reported once)
        if (kerr) {
            HIPCHK(hipMemsetAsync(c->kerr, 0, sizeof(uint32_t), c->stream));   // reported once
            return fail("spg: a shallow batch held >= 2^30 entries in 64 consecutive columns; accumulate it "
                        "on its own as a deep batch (spg_accumulate on a context without a pending run)");
        }
        bool again = false;
        if ((int64_t)h.n_cand > c->cand_cap) {
            HIPCHK(hipFree(c->cand));
            c->cand_cap = (int64_t)h.n_cand * 2;
            HIPCHK(hipMalloc(&c->cand, sizeof(spg_candidate) * c->cand_cap));
            again = true;
        }
        if ((int64_t)h.n_detail > c->detail_cap) {
            HIPCHK(hipFree(c->detail));
            c->detail_cap = (int64_t)h.n_detail * 2;
            HIPCHK(hipMalloc(&c->detail, sizeof(spg_detail) * c->detail_cap));
            again = true;
        }
        if (!again) return 0;
        int rc = finalize_impl(c, c->table_valid);
        if (rc) return rc;
    }
    return fail("spg: result buffers did not settle");
}

int spg_count(spg_ctx *c, int64_t *n_candidates, int64_t *n_details) {
    if (!c) return fail("spg_count: null ctx");
    Counters h{};
    int rc = settle(c, h);
    if (rc) return rc;
    if (n_candidates) *n_candidates = h.n_cand;
    if (n_details) *n_details = h.n_detail;
    return 0;
}

int spg_get_candidates(spg_ctx *c, spg_candidate *out, int64_t cap, int64_t *n_out) {
    if (!c || !n_out) return fail("spg_get_candidates: null argument");
    Counters h{};
    int rc = settle(c, h);
    if (rc) return rc;
    *n_out = h.n_cand;
    if ((int64_t)h.n_cand > cap) return fail("spg_get_candidates: output capacity too small");
    if (h.n_cand) {
        HIPCHK(hipMemcpyAsync(out, c->cand, sizeof(spg_candidate) * h.n_cand, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return 0;
}

int spg_get_details(spg_ctx *c, spg_detail *out, int64_t cap, int64_t *n_out) {
    if (!c || !n_out) return fail("spg_get_details: null argument");
    Counters h{};
    int rc = settle(c, h);
    if (rc) return rc;
    *n_out = h.n_detail;
    if ((int64_t)h.n_detail > cap) return fail("spg_get_details: output capacity too small");
    if (h.n_detail) {
        HIPCHK(hipMemcpyAsync(out, c->detail, sizeof(spg_detail) * h.n_detail, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return 0;
}

int spg_get_table(spg_ctx *c, int64_t pos0, int64_t n, uint32_t *depth, uint32_t *counts, double *gl,
                  uint8_t *flags, uint32_t *order, uint32_t *first_batch) {
    if (!c) return fail("spg_get_table: null ctx");
    if (pos0 < 0 || n < 0 || pos0 + n > c->n_pos) return fail("spg_get_table: range outside the context");
    Counters h{};
    int rc = settle(c, h);
    if (rc) return rc;
    if (!c->table_valid) {                  // calls-only finalize: build the table now
        rc = finalize_impl(c, true);
        if (rc) return rc;
        rc = settle(c, h);
        if (rc) return rc;
    }
    const hipMemcpyKind k = hipMemcpyDeviceToHost;
    if (depth) HIPCHK(hipMemcpyAsync(depth, c->o_depth + pos0, 4 * n, k, c->stream));
    if (counts) HIPCHK(hipMemcpyAsync(counts, c->o_counts + pos0 * SPG_NCOUNT, 4 * SPG_NCOUNT * n, k, c->stream));
    if (gl) HIPCHK(hipMemcpyAsync(gl, c->o_gl + pos0 * SPG_NSLOT, 8 * SPG_NSLOT * n, k, c->stream));
    if (flags) HIPCHK(hipMemcpyAsync(flags, c->o_flags + pos0, n, k, c->stream));
    if (order) HIPCHK(hipMemcpyAsync(order, c->o_order + pos0, 4 * n, k, c->stream));
    if (first_batch) HIPCHK(hipMemcpyAsync(first_batch, c->o_first + pos0, 4 * n, k, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int spg_device_results(spg_ctx *c, void **candidates, void **n_candidates) {
    if (!c) return fail("spg_device_results: null ctx");
    if (candidates) *candidates = c->cand;
    if (n_candidates) *n_candidates = &c->ctr[c->cslot].n_cand;
    return 0;
}

int spg_copy_candidates_device(spg_ctx *c, void *dst, int64_t cap) {
    if (!c || !dst || cap < 0) return fail("spg_copy_candidates_device: bad argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemsetAsync(dst, 0, 8, c->stream));
    HIPCHK(hipMemcpyAsync(dst, &c->ctr[c->cslot].n_cand, sizeof(uint32_t), hipMemcpyDeviceToDevice, c->stream));
    const int64_t n = std::min<int64_t>(cap, c->cand_cap);
    if (n) HIPCHK(hipMemcpyAsync((char *)dst + 8, c->cand, sizeof(spg_candidate) * n, hipMemcpyDeviceToDevice, c->stream));
    return 0;
}

int spg_copy_table_device(spg_ctx *c, void *dst, int64_t cap, int64_t *n_copy_cap) {
    if (!c || !dst || cap < 0) return fail("spg_copy_table_device: bad argument");
    if (!c->finalized) return fail("spg_copy_table_device: spg_finalize has not been called since the last accumulate/reset");
    HIPCHK(hipSetDevice(c->device));
    const int64_t n = std::min<int64_t>(cap, c->cand_cap);
    HIPCHK(launch_table_copy(c->ctr + c->cslot, c->kerr, c->ferr, c->cand, n, c->detail_cap, dst, c->stream));
    if (n_copy_cap) *n_copy_cap = n;
    return 0;
}

int spg_last_kernel_ms(spg_ctx *c, float *acc_ms, float *fin_ms) {
    if (!c) return fail("spg_last_kernel_ms: null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (acc_ms) *acc_ms = 0.f;
    if (fin_ms) *fin_ms = 0.f;
    if (c->acc_open) {         // accumulates since the last finalize
        if (acc_ms && c->acc_timing >= 1) HIPCHK(hipEventElapsedTime(acc_ms, c->ev[c->ring_w % spg_ctx::NRING][0],
                                               c->ev[c->ring_w % spg_ctx::NRING][1]));
        return 0;
    }
    if (c->ring_w == 0) return 0;
    hipEvent_t *ev = c->ev[(c->ring_w - 1) % spg_ctx::NRING];
    if (acc_ms && c->last_acc) HIPCHK(hipEventElapsedTime(acc_ms, ev[0], ev[1]));
    if (fin_ms && c->last_fin) HIPCHK(hipEventElapsedTime(fin_ms, ev[2], ev[3]));
    return 0;
}

int spg_set_timing(spg_ctx *c, int level) {
    if (!c) return fail("spg_set_timing: null ctx");
    if (level < 0 || level > 2) return fail("spg_set_timing: level must be 0, 1 or 2");
    c->timing = level;
    return 0;
}

int spg_kernel_times(spg_ctx *c, float *acc_ms, float *fin_ms, int64_t cap, int64_t *n_out) {
    if (!c || !n_out) return fail("spg_kernel_times: null argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    int64_t n = 0;
    for (int64_t i = c->ring_r; i < c->ring_w && n < cap; i++, n++) {
        hipEvent_t *ev = c->ev[i % spg_ctx::NRING];
        const uint8_t tm = c->ring_tm[i % spg_ctx::NRING];
        if (acc_ms) {
            acc_ms[n] = 0.f;
            if (tm & 1) HIPCHK(hipEventElapsedTime(acc_ms + n, ev[0], ev[1]));
        }
        if (fin_ms) {
            fin_ms[n] = 0.f;
            if (tm & 2) HIPCHK(hipEventElapsedTime(fin_ms + n, ev[2], ev[3]));
        }
    }
    c->ring_r += n;
    *n_out = n;
    return 0;
}

int spg_path_counters(spg_ctx *c, int64_t *out, int64_t n) {
    if (!c || (!out && n > 0)) return fail("spg_path_counters: bad argument");
    for (int64_t i = 0; i < std::min<int64_t>(n, 9); i++) out[i] = c->path[i];
    return 0;
}

// The context's device scratch for the history readers (spg_position_entries, spg_history_copy_compact): grows with
// headroom (doubled while small, +1/8 past 64 MiB) so a lookup does not allocate and free per call
static constexpr size_t SCRATCH_BIG = (size_t)64 << 20;
static int grow_scratch(spg_ctx *c, size_t need) {
    if (need <= c->pe_cap) return 0;
    if (c->pe_buf) { HIPCHK(hipStreamSynchronize(c->stream)); HIPCHK(hipFree(c->pe_buf)); }
    c->pe_buf = nullptr;
    c->pe_cap = 0;
    const size_t cap = need < SCRATCH_BIG ? need * 2 : need + need / 8;
    HIPCHK(hipMalloc(&c->pe_buf, cap));
    c->pe_cap = cap;
    return 0;
}

// A context with a history cap (spg_set_history_cap) budgets its HBM by that cap: a large scratch taken by one
// compaction (~0.6 GB for a 10,000x batch) is not kept behind the cap's back
static int trim_scratch(spg_ctx *c) {
    if (!c->hist_cap || c->pe_cap <= SCRATCH_BIG) return 0;
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipFree(c->pe_buf));
    c->pe_buf = nullptr;
    c->pe_cap = 0;
    return 0;
}

int spg_position_entries(spg_ctx *c, int64_t pos, uint8_t *codes, uint8_t *quals, int64_t cap, int64_t *n_out) {
    return spg_position_entries_upto(c, pos, INT64_MAX, codes, quals, cap, n_out);
}

int spg_position_entries_upto(spg_ctx *c, int64_t pos, int64_t n_batches, uint8_t *codes, uint8_t *quals, int64_t cap,
                              int64_t *n_out) {
    if (!c || !n_out || cap < 0 || (cap > 0 && (!codes || !quals)) || n_batches < 0)
        return fail("spg_position_entries: bad argument");
    if (pos < 0 || pos >= c->n_pos) return fail("spg_position_entries: position outside the context");
    HIPCHK(hipSetDevice(c->device));
    *n_out = 0;
    // the batches that may cover pos (bucket list, accumulate order), the first n_batches of the history only (a view
    // taken before later batches)
    const std::vector<int32_t> &all = c->buckets[(size_t)(pos >> RIDX_SHIFT)];
    const std::vector<int32_t> items(all.begin(), std::lower_bound(all.begin(), all.end(),
                                                                   (int32_t)std::min<int64_t>(n_batches, INT32_MAX)));
    const int32_t n = (int32_t)items.size();
    if (n == 0) return 0;
    if (int rc = wait_copies(c)) return rc;
    // every descriptor on the device (a pending batch's may not be yet)
    const int64_t nh = (int64_t)c->hist.size();
    if (c->hist_fence) { HIPCHK(hipEventSynchronize(c->hist_ev)); c->hist_fence = false; }
    HIPCHK(hipMemcpyAsync(c->d_hist, c->h_hist, sizeof(Hist) * nh, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipEventRecord(c->hist_ev, c->stream));
    c->hist_up = true;
    const size_t need = sizeof(int32_t) * n + 3 * sizeof(uint64_t) * n + 64;
    if (int rc = grow_scratch(c, need)) return rc;
    uint64_t *d_rng = reinterpret_cast<uint64_t *>(c->pe_buf);
    uint64_t *d_dst = d_rng + 2 * n;
    int32_t *d_items = reinterpret_cast<int32_t *>(d_dst + n);
    HIPCHK(hipMemcpyAsync(d_items, items.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_pos_bounds(c->d_hist, d_items, n, pos, d_rng, c->stream));
    std::vector<uint64_t> rng(2 * (size_t)n), dst((size_t)n);
    HIPCHK(hipMemcpyAsync(rng.data(), d_rng, sizeof(uint64_t) * 2 * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    uint64_t tot = 0;
    for (int32_t i = 0; i < n; i++) { dst[(size_t)i] = tot; tot += rng[2 * (size_t)i + 1] - rng[2 * (size_t)i]; }
    *n_out = (int64_t)tot;
    if ((int64_t)tot > cap) return cap == 0 ? 0 : fail("spg_position_entries: output capacity too small");
    if (tot == 0) return 0;
    // the output in the same scratch, after the index arrays (grown when needed: no allocation per lookup)
    const size_t ob = (need + 255) & ~(size_t)255;
    if (ob + 2 * tot > c->pe_cap) {
        std::vector<int32_t> keep(items);          // (the scratch is reallocated: the index arrays go up again)
        if (int rc = grow_scratch(c, ob + 2 * tot)) return rc;
        d_rng = reinterpret_cast<uint64_t *>(c->pe_buf);
        d_dst = d_rng + 2 * n;
        d_items = reinterpret_cast<int32_t *>(d_dst + n);
        HIPCHK(hipMemcpyAsync(d_items, keep.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(d_rng, rng.data(), sizeof(uint64_t) * 2 * n, hipMemcpyHostToDevice, c->stream));
    }
    uint8_t *oc = c->pe_buf + ob;
    HIPCHK(hipMemcpyAsync(d_dst, dst.data(), sizeof(uint64_t) * n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_pos_copy(c->d_hist, d_items, n, d_rng, d_dst, oc, oc + tot, c->stream));
    HIPCHK(hipMemcpyAsync(codes, oc, tot, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(quals, oc + tot, tot, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int spg_history_count(spg_ctx *c, int64_t *n_batches) {
    if (!c || !n_batches) return fail("spg_history_count: null argument");
    *n_batches = (int64_t)c->hist.size();
    return 0;
}

int spg_history_info(spg_ctx *c, int64_t i, int64_t *pos_begin, int64_t *n_cols, uint64_t *n_entries) {
    if (!c) return fail("spg_history_info: null ctx");
    if (i < 0 || i >= (int64_t)c->hist.size()) return fail("spg_history_info: batch index out of range");
    const HistBatch &h = c->hist[(size_t)i];
    if (pos_begin) *pos_begin = h.pos_begin;
    if (n_cols) *n_cols = h.n_cols;
    if (n_entries) *n_entries = h.n_entries;
    return 0;
}

int spg_set_history_cap(spg_ctx *c, int64_t bytes) {
    if (!c || bytes < 0) return fail("spg_set_history_cap: bad argument");
    HIPCHK(hipSetDevice(c->device));
    c->hist_cap = bytes;
    // spilling frees whole slabs: keep them a fraction of the cap
    c->arena.max_slab = bytes ? std::max<size_t>((size_t)16 << 20, std::min<size_t>((size_t)8 << 30, (size_t)bytes / 4))
                              : (size_t)8 << 30;
    return enforce_history_cap(c);
}

int spg_history_resident(spg_ctx *c, int64_t *device_bytes, int64_t *n_spilled, int64_t *arena_bytes) {
    if (!c) return fail("spg_history_resident: null ctx");
    if (device_bytes) *device_bytes = c->hist_dev_bytes;
    if (n_spilled) {
        int64_t n = 0;
        for (auto &b : c->hist) n += b.host != nullptr;
        *n_spilled = n;
    }
    if (arena_bytes) *arena_bytes = (int64_t)c->arena.bytes();
    return 0;
}

// Batch i as the checkpoint keeps it (live_variant_caller.py:40-45, :89, :77-85): the entries with q >= min_bq plus a
// first-entry marker per column whose entries all fail it, compacted on the device (spg_ckpt.hip) in column ranges of
// at most ~256 M entries (bounded scratch); only the kept bytes cross PCIe.
// spg_history_copy_compact and spg_history_copy_packed: the compaction in HBM, then either both arrays down or, packed,
// one byte per entry (k_ck_pack) plus the exception list
static int history_compact(spg_ctx *c, int64_t i, int32_t min_bq, uint64_t *offsets, uint8_t *base_code, uint8_t *qual,
                           uint64_t *n_kept, uint8_t *packed, uint64_t *exc_index, uint8_t *exc_code, uint8_t *exc_qual,
                           int64_t exc_cap, int64_t *n_exc) {
    if (!c || !offsets || !n_kept) return fail("spg_history_copy_compact: null argument");
    if (i < 0 || i >= (int64_t)c->hist.size()) return fail("spg_history_copy_compact: batch index out of range");
    if (min_bq < 0 || min_bq > 256) return fail("spg_history_copy_compact: min_bq out of range");
    HIPCHK(hipSetDevice(c->device));
    if (int rc = wait_copies(c)) return rc;
    const HistBatch &h = c->hist[(size_t)i];
    *n_kept = 0;
    // the batch's offsets first (the chunk boundaries come from them), then overwritten by the compact ones
    HIPCHK(hipMemcpyAsync(offsets, h.off, sizeof(uint64_t) * (h.n_cols + 1), hipMemcpyDefault, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (h.n_entries && !packed && (!base_code || !qual)) return fail("spg_history_copy_compact: null output buffer");
    if (h.n_entries && packed && exc_cap > 0 && (!exc_index || !exc_code || !exc_qual))
        return fail("spg_history_copy_packed: null exception buffer");
    const uint64_t chunk_entries = (uint64_t)256 << 20;
    std::vector<int64_t> cuts{0};
    for (int64_t k = 0; k < h.n_cols;) {
        // the next cut: the last column start within chunk_entries of this one (at least one column)
        const uint64_t lim = offsets[k] + chunk_entries;
        int64_t lo = k + 1, hi = h.n_cols;
        while (lo < hi) {
            const int64_t mid = lo + (hi - lo + 1) / 2;
            if (offsets[mid] <= lim) lo = mid; else hi = mid - 1;
        }
        k = lo;
        cuts.push_back(k);
    }
    int64_t max_cols = 1;
    uint64_t max_e = 16;
    for (size_t k = 1; k < cuts.size(); k++) {
        max_cols = std::max(max_cols, cuts[k] - cuts[k - 1]);
        max_e = std::max<uint64_t>(max_e, offsets[cuts[k]] - offsets[cuts[k - 1]]);
    }
    size_t scan_bytes = 0;
    Hist probe{0, max_cols, nullptr, nullptr, nullptr};
    HIPCHK(launch_ck_compact(probe, 0, nullptr, nullptr, nullptr, &scan_bytes, nullptr, nullptr, c->stream));
    const size_t ob = ((sizeof(uint64_t) * (size_t)(max_cols + 1)) + 255) & ~size_t(255);
    const size_t sb = (scan_bytes + 255) & ~size_t(255), eb = ((size_t)max_e + 255) & ~size_t(255);
    // (packed: a device exception list of up to 1 Mi entries; more than the caller's capacity reports the count only)
    const uint32_t xcap = packed ? (uint32_t)std::min<int64_t>(std::max<int64_t>(exc_cap, 0), (int64_t)1 << 20) : 0u;
    const size_t xb = packed ? (((size_t)xcap * 10 + 256 + 255) & ~size_t(255)) : 0;
    if (int rc = grow_scratch(c, 2 * ob + sb + 2 * eb + xb)) return rc;
    uint64_t *kept = reinterpret_cast<uint64_t *>(c->pe_buf), *noff = reinterpret_cast<uint64_t *>(c->pe_buf + ob);
    void *tmp = c->pe_buf + 2 * ob;
    uint8_t *oc = c->pe_buf + 2 * ob + sb, *oq = oc + eb;
    uint32_t *xn = reinterpret_cast<uint32_t *>(oq + eb);
    uint64_t *xi = reinterpret_cast<uint64_t *>(oq + eb + 256);
    uint8_t *xc = reinterpret_cast<uint8_t *>(xi + xcap), *xq = xc + xcap;
    if (packed) HIPCHK(hipMemsetAsync(xn, 0, sizeof(uint32_t), c->stream));
    std::vector<uint64_t> loc((size_t)max_cols + 1);
    uint64_t base = 0;
    for (size_t k = 1; k < cuts.size(); k++) {
        const int64_t c0 = cuts[k - 1], n = cuts[k] - c0;
        Hist sub{h.pos_begin + c0, n, h.off + c0, h.code, h.qual};
        size_t tb = sb;
        HIPCHK(launch_ck_compact(sub, (uint32_t)min_bq, kept, noff, tmp, &tb, oc, oq, c->stream));
        HIPCHK(hipMemcpyAsync(loc.data(), noff, sizeof(uint64_t) * (size_t)(n + 1), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        const uint64_t m = loc[(size_t)n];
        if (m && packed) {
            HIPCHK(launch_ck_pack(oc, oq, m, base, xi, xc, xq, xn, xcap, c->stream));
            HIPCHK(hipMemcpyAsync(packed + base, oc, m, hipMemcpyDeviceToHost, c->stream));
        } else if (m) {
            HIPCHK(hipMemcpyAsync(base_code + base, oc, m, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(qual + base, oq, m, hipMemcpyDeviceToHost, c->stream));
        }
        for (int64_t j = 0; j < n; j++) offsets[c0 + j] = base + loc[(size_t)j];
        base += m;
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    offsets[h.n_cols] = base;
    *n_kept = base;
    if (packed) {
        uint32_t nx = 0;
        HIPCHK(hipMemcpyAsync(&nx, xn, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        *n_exc = nx;
        if ((int64_t)nx <= exc_cap && nx <= xcap && nx) {
            HIPCHK(hipMemcpyAsync(exc_index, xi, sizeof(uint64_t) * nx, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(exc_code, xc, nx, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(exc_qual, xq, nx, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
        } else if (nx > xcap) {
            *n_exc = std::max<int64_t>((int64_t)nx, exc_cap + 1);   // (more than the device list held: not usable)
        }
    }
    return trim_scratch(c);
}

int spg_history_copy_compact(spg_ctx *c, int64_t i, int32_t min_bq, uint64_t *offsets, uint8_t *base_code, uint8_t *qual,
                             uint64_t *n_kept) {
    return history_compact(c, i, min_bq, offsets, base_code, qual, n_kept, nullptr, nullptr, nullptr, nullptr, 0, nullptr);
}

int spg_history_copy_packed(spg_ctx *c, int64_t i, int32_t min_bq, uint64_t *offsets, uint8_t *packed, uint64_t *n_kept,
                            uint64_t *exc_index, uint8_t *exc_code, uint8_t *exc_qual, int64_t exc_cap, int64_t *n_exc) {
    if (!packed || !n_exc) return fail("spg_history_copy_packed: null argument");
    *n_exc = 0;
    return history_compact(c, i, min_bq, offsets, nullptr, nullptr, n_kept, packed, exc_index, exc_code, exc_qual, exc_cap,
                           n_exc);
}


int spg_history_copy(spg_ctx *c, int64_t i, uint64_t *offsets, uint8_t *base_code, uint8_t *qual) {
    if (!c) return fail("spg_history_copy: null ctx");
    if (i < 0 || i >= (int64_t)c->hist.size()) return fail("spg_history_copy: batch index out of range");
    HIPCHK(hipSetDevice(c->device));
    if (int rc = wait_copies(c)) return rc;
    const HistBatch &h = c->hist[(size_t)i];
    // (hipMemcpyDefault: a spilled batch is in pinned host memory)
    if (offsets) HIPCHK(hipMemcpyAsync(offsets, h.off, sizeof(uint64_t) * (h.n_cols + 1), hipMemcpyDefault, c->stream));
    if (base_code && h.n_entries) HIPCHK(hipMemcpyAsync(base_code, h.code, h.n_entries, hipMemcpyDefault, c->stream));
    if (qual && h.n_entries) HIPCHK(hipMemcpyAsync(qual, h.qual, h.n_entries, hipMemcpyDefault, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}


// ------------------------------------------------------------------------------------------------------------------
// spg_bam_*: a BAM kept in HBM (include/spings_gpu.h; kernels in spg_bam.hip, spg_inflate.hip, spg_fill.hip)
// ------------------------------------------------------------------------------------------------------------------
static int bam_fallback(const std::string &m) {
    g_err = m;
    return 1;
}

int spg_bam_release(spg_ctx *c) {
    if (!c) return fail("spg_bam_release: null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->copy_stream));
    // an spg_bam_upload still in flight reads the caller's host buffer: done before the caller may free it, and the
    // slot forgets it (a later BAM at the same address and size must not take it for its own upload)
    if (c->up_stream) HIPCHK(hipStreamSynchronize(c->up_stream));
    for (BamDev &b : c->bams) b.release();
    return 0;
}

int spg_bam_slot(spg_ctx *c, int slot) {
    if (!c || slot < 0 || slot > 1) return fail("spg_bam_slot: bad argument");
    c->bam_slot = slot;
    return 0;
}

int spg_bam_inflate_ms(spg_ctx *c, float *ms) {
    if (!c || !ms) return fail("spg_bam_inflate_ms: null argument");
    *ms = c->bam_cur().inflate_ms;
    return 0;
}

int spg_bam_inflate_fallbacks(spg_ctx *c, int64_t *n) {
    if (!c || !n) return fail("spg_bam_inflate_fallbacks: null argument");
    *n = c->bam_cur().inflate_fallbacks;
    return 0;
}

int spg_bam_upload(spg_ctx *c, int slot, const uint8_t *comp, uint64_t comp_bytes, const spg_bgzf_member *members,
                   int64_t n) {
    if (!c || !comp || !members || n < 1 || slot < 0 || slot > 1) return fail("spg_bam_upload: bad argument");
    for (int64_t i = 0; i < n; i++)
        if (members[i].coff + members[i].clen + 8 > comp_bytes || members[i].ulen > 65536)
            return fail("spg_bam_upload: member outside the file");
    HIPCHK(hipSetDevice(c->device));
    if (!c->up_stream) HIPCHK(hipStreamCreateWithFlags(&c->up_stream, hipStreamNonBlocking));
    BamDev &B = c->bams[slot];
    B.up_pending = false;
    if (!B.ev_up) HIPCHK(hipEventCreateWithFlags(&B.ev_up, hipEventDisableTiming));
    // (the slot's previous BAM: its inflate read comp / mem on the kernel stream, and spg_bam_open synchronised on it
    // before returning; growing a buffer frees the old one, which waits for the device)
    HIPCHK(B.comp.need(comp_bytes + 64));
    HIPCHK(B.mem.need(sizeof(spg_bgzf_member) * (size_t)n));
    HIPCHK(hipMemcpyAsync(B.comp.p, comp, comp_bytes, hipMemcpyHostToDevice, c->up_stream));
    HIPCHK(hipMemsetAsync(B.comp.as<uint8_t>() + comp_bytes, 0, 64, c->up_stream));
    HIPCHK(hipMemcpyAsync(B.mem.p, members, sizeof(spg_bgzf_member) * (size_t)n, hipMemcpyHostToDevice, c->up_stream));
    HIPCHK(hipEventRecord(B.ev_up, c->up_stream));
    B.up_pending = true;
    B.up_comp = comp;
    B.up_bytes = comp_bytes;
    B.up_n = n;
    return 0;
}

int spg_bam_open(spg_ctx *c, const uint8_t *comp, uint64_t comp_bytes, const spg_bgzf_member *members, int64_t n,
                 uint64_t body, int32_t tid, int32_t n_ref, const spg_bam_filter *flt, int64_t *n_reads) {
    if (!c || !comp || !members || !flt || !n_reads || n < 1 || tid < 0 || tid >= n_ref)
        return fail("spg_bam_open: bad argument");
    if (flt->stepper < 0 || flt->stepper > 2) return fail("spg_bam_open: bad stepper");
    HIPCHK(hipSetDevice(c->device));
    BamDev &B = c->bam_cur();
    B.open = false;
    *n_reads = 0;
    std::vector<uint64_t> uoff((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; i++) {
        const spg_bgzf_member &m = members[i];
        if (m.coff + m.clen + 8 > comp_bytes || m.ulen > 65536) return fail("spg_bam_open: member outside the file");
        if (m.uoff != uoff[(size_t)i]) return fail("spg_bam_open: members' inflated offsets are not contiguous");
        uoff[(size_t)i + 1] = uoff[(size_t)i] + m.ulen;
    }
    const uint64_t total = uoff[(size_t)n];
    if (body >= total || total >= ((uint64_t)1 << 40)) return fail("spg_bam_open: bad header end");
    hipStream_t cs = c->copy_stream;
    if (!B.ev[0]) { HIPCHK(hipEventCreate(&B.ev[0])); HIPCHK(hipEventCreate(&B.ev[1])); }
    const size_t nm = (size_t)n;
    HIPCHK(B.comp.need(comp_bytes + 64));
    HIPCHK(B.out.need(total + 64));
    HIPCHK(B.mem.need(sizeof(spg_bgzf_member) * nm));
    HIPCHK(B.status.need(sizeof(uint32_t) * nm));
    HIPCHK(B.uoff.need(sizeof(uint64_t) * (nm + 1)));
    HIPCHK(B.start.need(sizeof(uint64_t) * nm));
    HIPCHK(B.cnt.need(sizeof(uint32_t) * nm));
    HIPCHK(B.base.need(sizeof(uint32_t) * (nm + 1)));
    HIPCHK(B.lohi.need(sizeof(int64_t) * 2 * nm));
    HIPCHK(B.err.need(64));
    HIPCHK(B.iscr.need(inflate_scratch_bytes(comp_bytes, n)));
    HIPCHK(B.rtmp.need(sizeof(uint64_t) * BAM_RTMP * nm));
    // the compressed bytes and member table: already on their way when spg_bam_upload sent this same file to this slot
    // (process_bams sends BAM i + 1 while BAM i inflates); else copied here
    const bool up = B.up_pending && B.up_comp == comp && B.up_bytes == comp_bytes && B.up_n == n;
    B.up_pending = false;
    if (up) {
        HIPCHK(hipStreamWaitEvent(cs, B.ev_up, 0));
    } else {
        HIPCHK(hipMemcpyAsync(B.comp.p, comp, comp_bytes, hipMemcpyHostToDevice, cs));
        HIPCHK(hipMemsetAsync(B.comp.as<uint8_t>() + comp_bytes, 0, 64, cs));
        HIPCHK(hipMemcpyAsync(B.mem.p, members, sizeof(spg_bgzf_member) * nm, hipMemcpyHostToDevice, cs));
    }
    HIPCHK(hipMemcpyAsync(B.uoff.p, uoff.data(), sizeof(uint64_t) * (nm + 1), hipMemcpyHostToDevice, cs));
    HIPCHK(hipMemsetAsync(B.out.as<uint8_t>() + total, 0, 64, cs));
    HIPCHK(hipMemsetAsync(B.err.p, 0, 64, cs));
    HIPCHK(hipEventRecord(B.ev[0], cs));
    HIPCHK(launch_inflate(B.comp.as<uint8_t>(), comp_bytes, B.mem.as<spg_bgzf_member>(), n, B.out.as<uint8_t>(),
                          B.status.as<uint32_t>(), B.iscr.p, cs));
    HIPCHK(hipEventRecord(B.ev[1], cs));
    BamArgs A{};
    A.data = B.out.as<uint8_t>();
    A.total = total;
    A.body = body;
    A.uoff = B.uoff.as<uint64_t>();
    A.n_members = n;
    A.tid = tid;
    A.n_ref = n_ref;
    A.stepper = flt->stepper;
    A.flag_filter = flt->flag_filter;
    A.min_mapq = flt->min_mapping_quality;
    A.start = B.start.as<uint64_t>();
    A.cnt = B.cnt.as<uint32_t>();
    A.base = B.base.as<uint32_t>();
    A.pos_lo = B.lohi.as<int64_t>();
    A.pos_hi = A.pos_lo + nm;
    A.err = B.err.as<uint32_t>();
    A.rtmp = B.rtmp.as<uint64_t>();
    HIPCHK(launch_bam_scan(A, 0, cs));
    HIPCHK(launch_bam_scan(A, 1, cs));
    std::vector<uint32_t> st(nm), cnt(nm), err(1), fbk(1);
    std::vector<int64_t> lohi(2 * nm);
    HIPCHK(hipMemcpyAsync(st.data(), B.status.p, sizeof(uint32_t) * nm, hipMemcpyDeviceToHost, cs));
    HIPCHK(hipMemcpyAsync(cnt.data(), B.cnt.p, sizeof(uint32_t) * nm, hipMemcpyDeviceToHost, cs));
    HIPCHK(hipMemcpyAsync(lohi.data(), B.lohi.p, sizeof(int64_t) * 2 * nm, hipMemcpyDeviceToHost, cs));
    HIPCHK(hipMemcpyAsync(err.data(), B.err.p, sizeof(uint32_t), hipMemcpyDeviceToHost, cs));
    HIPCHK(hipMemcpyAsync(fbk.data(), B.iscr.p, sizeof(uint32_t), hipMemcpyDeviceToHost, cs));
    HIPCHK(hipStreamSynchronize(cs));
    B.inflate_fallbacks = fbk[0];
    if (hipEventElapsedTime(&B.inflate_ms, B.ev[0], B.ev[1]) != hipSuccess) B.inflate_ms = -1.f;
    for (size_t i = 0; i < nm; i++)
        if (st[i] != 0)
            return bam_fallback("spg_bam_open: member " + std::to_string(i) + " did not inflate on the GPU (status " +
                                std::to_string(st[i]) + ")");
    if (err[0] & 1u) return bam_fallback("spg_bam_open: the record chains of the members disagree");
    int64_t last = -1;
    for (size_t i = 0; i < nm; i++) {
        if (lohi[i] == INT64_MAX) continue;
        if (lohi[i] < last || (err[0] & 2u)) return fail("spg_bam_open: BAM is not coordinate-sorted");
        last = lohi[nm + i];
    }
    std::vector<uint32_t> base(nm + 1, 0);
    uint64_t tot = 0;
    for (size_t i = 0; i < nm; i++) { base[i] = (uint32_t)tot; tot += cnt[i]; }
    if (tot >= ((uint64_t)1 << 31)) return fail("spg_bam_open: more than 2^31 reads");
    base[nm] = (uint32_t)tot;
    const size_t nr = (size_t)tot;
    HIPCHK(B.rec.need(sizeof(uint64_t) * (nr + 1)));
    // fields: pos end mtid mpos isize (i32), l_seq (u32), nhash (u64), flag (u16)
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t f32 = al(4 * (nr + 1)), f64 = al(8 * (nr + 1)), f16 = al(2 * (nr + 1));
    HIPCHK(B.fields.need(6 * f32 + f64 + f16));
    uint8_t *fb = B.fields.as<uint8_t>();
    B.pos = reinterpret_cast<int32_t *>(fb);
    B.end = reinterpret_cast<int32_t *>(fb + f32);
    B.mtid = reinterpret_cast<int32_t *>(fb + 2 * f32);
    B.mpos = reinterpret_cast<int32_t *>(fb + 3 * f32);
    B.isize = reinterpret_cast<int32_t *>(fb + 4 * f32);
    B.l_seq = reinterpret_cast<uint32_t *>(fb + 5 * f32);
    B.nhash = reinterpret_cast<uint64_t *>(fb + 6 * f32);
    B.flag = reinterpret_cast<uint16_t *>(fb + 6 * f32 + f64);
    HIPCHK(hipMemcpyAsync(B.base.p, base.data(), sizeof(uint32_t) * (nm + 1), hipMemcpyHostToDevice, cs));
    A.rec = B.rec.as<uint64_t>();
    A.n_reads = (uint32_t)nr;
    A.pos = B.pos; A.end = B.end; A.mtid = B.mtid; A.mpos = B.mpos; A.isize = B.isize;
    A.flag = B.flag; A.l_seq = B.l_seq; A.nhash = B.nhash;
    // the counting walk listed each member's records (<= BAM_RTMP of them): copy the lists; else walk again
    const bool lists = std::all_of(cnt.begin(), cnt.end(), [](uint32_t v) { return v <= BAM_RTMP; });
    HIPCHK(launch_bam_scan(A, lists ? 4 : 2, cs));
    HIPCHK(launch_bam_scan(A, 3, cs));
    HIPCHK(hipMemcpyAsync(err.data(), B.err.p, sizeof(uint32_t), hipMemcpyDeviceToHost, cs));
    HIPCHK(hipStreamSynchronize(cs));
    if (err[0] & 4u) return fail("spg_bam_open: corrupt BAM record (field lengths exceed block_size)");
    B.total = total;
    B.n_members = n;
    B.n_reads = (uint32_t)nr;
    B.tid = tid;
    B.open = true;
    *n_reads = (int64_t)nr;
    return 0;
}

int spg_bam_reads_copy(spg_ctx *c, const spg_bam_reads *o) {
    if (!c || !o) return fail("spg_bam_reads_copy: null argument");
    BamDev &B = c->bam_cur();
    if (!B.open) return fail("spg_bam_reads_copy: no BAM open (spg_bam_open)");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t cs = c->copy_stream;
    const size_t n = B.n_reads;
    if (n) {
        struct { void *h; const void *d; size_t w; } cp[] = {
            {o->pos, B.pos, 4}, {o->end, B.end, 4}, {o->mtid, B.mtid, 4}, {o->mpos, B.mpos, 4}, {o->isize, B.isize, 4},
            {o->flag, B.flag, 2}, {o->l_seq, B.l_seq, 4}, {o->name_hash, B.nhash, 8}};
        for (auto &x : cp)
            if (x.h) HIPCHK(hipMemcpyAsync(x.h, x.d, x.w * n, hipMemcpyDeviceToHost, cs));
    }
    HIPCHK(hipStreamSynchronize(cs));
    return 0;
}

// The open BAM's pileup plan built in HBM (spg_plan.hip): htslib's depth cap and mate pairing over the reads'
// fixed fields, the kept list, the CSR offsets and the pairs — what spp_pileup_plan_fields computes on the host from
// spg_bam_reads_copy's fields, without the fields coming down.  Returns 1 (nothing built) when the device declines.
int spg_bam_plan_build(spg_ctx *c, int64_t max_depth, int32_t ignore_overlaps, spg_bam_plan *out) {
    if (!c || !out) return fail("spg_bam_plan_build: null argument");
    if (max_depth < 0) return fail("spg_bam_plan_build: max_depth < 0");
    BamDev &B = c->bam_cur();
    if (!B.open) return fail("spg_bam_plan_build: no BAM open (spg_bam_open)");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t cs = c->copy_stream;
    *out = spg_bam_plan{};
    const uint32_t n = B.n_reads;
    if (n == 0) return 0;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    // per-read arrays (one buffer): first, didx, dfirst (n + 1), dpos, kept, sval, pairb, pb_list, pa, pbv (n), keep (u8),
    // skey, pcol, porig, lsa (8-byte), the head
    const size_t u4 = al(4 * ((size_t)n + 1)), u8 = al(8 * (size_t)n), b1 = al(n);
    const size_t rd = 10 * u4 + b1 + 4 * u8 + al(sizeof(PlanHead));
    HIPCHK(B.plan_rd.need(rd));
    uint8_t *m = B.plan_rd.as<uint8_t>();
    PlanArgs A{};
    A.n = n;
    A.pos = B.pos; A.end = B.end; A.mtid = B.mtid; A.mpos = B.mpos; A.isize = B.isize;
    A.flag = B.flag; A.l_seq = B.l_seq; A.nhash = B.nhash;
    A.tid = B.tid;
    A.olap = ignore_overlaps ? 1 : 0;
    A.maxcnt = max_depth > 0 ? max_depth : INT64_MAX;
    uint32_t *w4[10];
    for (int i = 0; i < 10; i++) w4[i] = reinterpret_cast<uint32_t *>(m + (size_t)i * u4);
    A.first = w4[0]; A.didx = w4[1]; A.dfirst = w4[2]; A.dpos = reinterpret_cast<int32_t *>(w4[3]); A.kept = w4[4];
    A.sval = w4[5]; A.pairb = w4[6]; A.pb_list = w4[7]; A.pa = w4[8]; A.pbv = w4[9];
    uint8_t *q = m + 10 * u4;
    A.keep = q;
    q += b1;
    A.skey = reinterpret_cast<uint64_t *>(q);
    A.pcol = reinterpret_cast<int64_t *>(q + u8);
    A.porig = reinterpret_cast<uint64_t *>(q + 2 * u8);
    A.lsa = reinterpret_cast<uint64_t *>(q + 3 * u8);
    A.head = reinterpret_cast<PlanHead *>(q + 4 * u8);
    size_t tb = plan_temp_bytes(n, 0);
    HIPCHK(B.plan_tmp.need(tb));
    HIPCHK(launch_plan_reads(A, B.plan_tmp.p, tb, cs));
    PlanHead h{};
    HIPCHK(hipMemcpyAsync(&h, A.head, sizeof h, hipMemcpyDeviceToHost, cs));
    HIPCHK(hipStreamSynchronize(cs));
    if (h.err & 1u) return bam_fallback("spg_bam_plan_build: a read without reference span, or reads out of order");
    const bool capped = max_depth > 0;
    if (capped && (int64_t)h.max_span + 128 > 8192)
        return bam_fallback("spg_bam_plan_build: a read spans more than the depth-cap sweep's ring");
    // per-column arrays over [min_pos, max_end]: the coverage difference array, the coverage, the offsets
    A.span_lo = h.min_pos;
    A.span_n = h.max_end - h.min_pos;
    if (A.span_n < 1 || A.span_n > ((int64_t)1 << 31) - 256) return bam_fallback("spg_bam_plan_build: column span out of range");
    const size_t sn = (size_t)A.span_n + 1;
    HIPCHK(B.plan_sp.need(2 * al(4 * sn) + al(8 * sn)));
    uint8_t *sp = B.plan_sp.as<uint8_t>();
    A.diff = reinterpret_cast<int32_t *>(sp);
    int32_t *cov = reinterpret_cast<int32_t *>(sp + al(4 * sn));
    A.offsets = reinterpret_cast<uint64_t *>(sp + 2 * al(4 * sn));
    tb = plan_temp_bytes(n, A.span_n);
    HIPCHK(B.plan_tmp.need(tb));
    bool sweep = capped;
    if (capped && h.n_distinct > (1u << 22)) {
        // a long contig: the sweep only when the cap can bite somewhere (U_p <= cov(p) + cov(p - 1) <= 2 max cov)
        HIPCHK(launch_plan_cov(A, 1, cov, B.plan_tmp.p, tb, cs));
        HIPCHK(hipMemcpyAsync(&h, A.head, sizeof h, hipMemcpyDeviceToHost, cs));
        HIPCHK(hipStreamSynchronize(cs));
        if (2 * (int64_t)h.max_cov > max_depth)
            return bam_fallback("spg_bam_plan_build: the depth cap bites on a contig with > 4 M start positions");
        sweep = false;
    }
    HIPCHK(launch_plan_keep(A, sweep, cs));
    HIPCHK(launch_plan_rest(A, cov, A.olap && h.n_cand > 0, B.plan_tmp.p, tb, cs));
    HIPCHK(hipMemcpyAsync(&h, A.head, sizeof h, hipMemcpyDeviceToHost, cs));
    HIPCHK(hipStreamSynchronize(cs));
    if (h.err & 2u) return bam_fallback("spg_bam_plan_build: more than 16 reads share a name hash");
    if (h.n_kept && h.lo != A.span_lo) return fail("spg_bam_plan_build: internal error (first read not kept)");
    out->pos_begin = h.lo;
    out->n_cols = h.hi - h.lo;
    out->n_entries = h.n_entries;
    out->offsets = A.offsets;
    out->n_kept = h.n_kept;
    out->kept = A.kept;
    out->n_pairs = h.n_pairs;
    out->pair_a = A.pa;
    out->pair_b = A.pbv;
    out->pair_col = A.pcol;
    out->pair_orig = A.porig;
    out->orig_bytes = h.orig_bytes;
    out->max_span = h.max_span_kept;
    return 0;
}

// spg_bam_plan_build's arrays copied to host memory (tests: the device plan against spp_pileup_plan_fields')
int spg_bam_plan_download(spg_ctx *c, const spg_bam_plan *P, uint64_t *offsets, uint32_t *kept, uint32_t *pair_a,
                          uint32_t *pair_b, int64_t *pair_col, uint64_t *pair_orig) {
    if (!c || !P) return fail("spg_bam_plan_download: null argument");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t cs = c->copy_stream;
    const size_t nc = (size_t)std::max<int64_t>(0, P->n_cols), nk = (size_t)P->n_kept, np = (size_t)P->n_pairs;
    if (offsets && P->offsets && nc) HIPCHK(hipMemcpyAsync(offsets, P->offsets, 8 * (nc + 1), hipMemcpyDeviceToHost, cs));
    if (kept && nk) HIPCHK(hipMemcpyAsync(kept, P->kept, 4 * nk, hipMemcpyDeviceToHost, cs));
    if (np) {
        if (pair_a) HIPCHK(hipMemcpyAsync(pair_a, P->pair_a, 4 * np, hipMemcpyDeviceToHost, cs));
        if (pair_b) HIPCHK(hipMemcpyAsync(pair_b, P->pair_b, 4 * np, hipMemcpyDeviceToHost, cs));
        if (pair_col) HIPCHK(hipMemcpyAsync(pair_col, P->pair_col, 8 * np, hipMemcpyDeviceToHost, cs));
        if (pair_orig) HIPCHK(hipMemcpyAsync(pair_orig, P->pair_orig, 8 * np, hipMemcpyDeviceToHost, cs));
    }
    HIPCHK(hipStreamSynchronize(cs));
    return 0;
}

int spg_bam_accumulate(spg_ctx *c, const spg_bam_plan *P, uint32_t flags) {
    // SPG_IN_DEVICE: the plan's arrays are in HBM (spg_bam_plan_build, trusted); else host arrays (validated here)
    const bool devp = (flags & SPG_IN_DEVICE) != 0;
    if (!c || !P) return fail("spg_bam_accumulate: null argument");
    if (!c->lut_set) return fail("spg_accumulate: spg_set_eps_lut not called");
    if (!c->ref) return fail("spg_accumulate: spg_set_reference not called");
    BamDev &B = c->bam_cur();
    if (!B.open) return fail("spg_bam_accumulate: no BAM open (spg_bam_open)");
    if (P->n_cols < 0 || P->n_cols > ((int64_t)1 << 31) - 128) return fail("spg_bam_accumulate: n_cols out of range");
    if (P->n_kept < 0 || P->n_kept > (int64_t)B.n_reads || P->n_pairs < 0 || P->n_pairs > P->n_kept || P->max_span < 0)
        return fail("spg_bam_accumulate: bad read / pair counts");
    if (P->n_cols > 0 && (!P->offsets || (P->n_kept && !P->kept) ||
                          (P->n_pairs && (!P->pair_a || !P->pair_b || !P->pair_col || !P->pair_orig))))
        return fail("spg_bam_accumulate: null buffer");
    if (P->n_cols == 0) { B.open = false; return 0; }
    if (!devp) {
        if (P->offsets[0] != 0 || P->offsets[P->n_cols] != P->n_entries)
            return fail("spg_bam_accumulate: offsets[0] must be 0 and offsets[n_cols] == n_entries");
        uint64_t desc = 0;
        for (int64_t i = 0; i < P->n_cols; i++) desc |= (uint64_t)(P->offsets[i + 1] < P->offsets[i]);
        if (desc) return fail("spg_bam_accumulate: offsets not monotone");
        uint64_t need_orig = 0;
        for (int64_t j = 0; j < P->n_pairs; j++) {
            if (P->pair_a[j] >= B.n_reads || P->pair_b[j] >= B.n_reads)
                return fail("spg_bam_accumulate: pair read out of range");
            need_orig = std::max<uint64_t>(need_orig, P->pair_orig[j]);
        }
        if (P->n_pairs && P->orig_bytes < need_orig) return fail("spg_bam_accumulate: orig_bytes too small");
    }
    HIPCHK(hipSetDevice(c->device));
    hipStream_t cs = c->copy_stream;
    const size_t nk = (size_t)P->n_kept, np = (size_t)P->n_pairs, nr = B.n_reads;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    HIPCHK(B.kept.need(4 * nk + 16));
    const size_t o_pb = al(4 * np), o_col = o_pb + al(4 * np), o_oq = o_col + al(8 * np);
    HIPCHK(B.pairs.need(o_oq + al(8 * np) + 16));
    HIPCHK(B.orig.need(P->orig_bytes + 64));
    HIPCHK(B.twof.need(4 * nr + 16));
    const size_t o_pos = al(8 * nk), o_end = o_pos + al(4 * nk), o_tw = o_end + al(4 * nk);
    HIPCHK(B.recs_k.need(o_tw + al(4 * nk) + 16));
    const int64_t n_tiles = (P->n_cols + 63) / 64;
    const size_t fsb = fill_scratch_bytes(P->n_cols, P->n_kept, P->max_span);
    HIPCHK(B.tile_first.need(fsb));
    const hipMemcpyKind pk = devp ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (nk) HIPCHK(hipMemcpyAsync(B.kept.p, P->kept, 4 * nk, pk, cs));
    uint8_t *pb = B.pairs.as<uint8_t>();
    if (np) {
        HIPCHK(hipMemcpyAsync(pb, P->pair_a, 4 * np, pk, cs));
        HIPCHK(hipMemcpyAsync(pb + o_pb, P->pair_b, 4 * np, pk, cs));
        HIPCHK(hipMemcpyAsync(pb + o_col, P->pair_col, 8 * np, pk, cs));
        HIPCHK(hipMemcpyAsync(pb + o_oq, P->pair_orig, 8 * np, pk, cs));
        BamPairArgs Q{};
        Q.data = B.out.as<uint8_t>();
        Q.wdata = B.out.as<uint8_t>();
        Q.rec = B.rec.as<uint64_t>();
        Q.n_reads = (uint32_t)nr;
        Q.n_pairs = (uint32_t)np;
        Q.pa = reinterpret_cast<const uint32_t *>(pb);
        Q.pb = reinterpret_cast<const uint32_t *>(pb + o_pb);
        Q.oq = reinterpret_cast<const uint64_t *>(pb + o_oq);
        Q.orig = B.orig.as<uint8_t>();
        Q.err = B.err.as<uint32_t>() + 1;
        // names first (a hash collision must not tweak anything): the plan is refused before any change
        uint32_t e = 0;
        HIPCHK(hipMemsetAsync(Q.err, 0, 4, cs));
        HIPCHK(launch_bam_pairs(Q, false, cs));
        HIPCHK(hipMemcpyAsync(&e, Q.err, 4, hipMemcpyDeviceToHost, cs));
        HIPCHK(hipStreamSynchronize(cs));
        if (e & 8u) return bam_fallback("spg_bam_accumulate: paired reads with equal name hashes have different names");
        HIPCHK(launch_bam_pairs(Q, true, cs));
    }
    uint8_t *rk = B.recs_k.as<uint8_t>();
    BamGatherArgs G{};
    G.n_reads = (uint32_t)nr;
    G.n_kept = (uint32_t)nk;
    G.n_pairs = (uint32_t)np;
    G.kept = B.kept.as<uint32_t>();
    G.pa = reinterpret_cast<const uint32_t *>(pb);
    G.rec = B.rec.as<uint64_t>();
    G.pos = B.pos;
    G.end = B.end;
    G.twof = B.twof.as<int32_t>();
    G.rec_k = reinterpret_cast<uint64_t *>(rk);
    G.rpos_k = reinterpret_cast<int32_t *>(rk + o_pos);
    G.rend_k = reinterpret_cast<int32_t *>(rk + o_end);
    G.tw_k = reinterpret_cast<int32_t *>(rk + o_tw);
    G.err = c->ferr;
    HIPCHK(hipMemsetAsync(G.twof, 0xFF, 4 * nr, cs));
    HIPCHK(launch_bam_gather(G, cs));
    FillArgs F{};
    F.data = B.out.as<uint8_t>();
    F.data_bytes = B.total;
    F.rec = G.rec_k;
    F.rpos = G.rpos_k;
    F.rend = G.rend_k;
    F.tweak = G.tw_k;
    F.tw_col = reinterpret_cast<const int64_t *>(pb + o_col);
    F.tw_q = reinterpret_cast<const uint64_t *>(pb + o_oq);
    F.orig = B.orig.as<uint8_t>();
    F.orig_bytes = P->orig_bytes;
    F.scratch = B.tile_first.p;
    F.scratch_bytes = fsb;
    F.pos_begin = P->pos_begin;
    F.n_cols = (int32_t)P->n_cols;
    F.n_tiles = (int32_t)n_tiles;
    F.n_reads = (uint32_t)nk;
    F.back = (int32_t)((P->max_span + 63) / 64);
    c->ferr_dirty = true;
    bool pageable = false;
    B.open = false;                        // (the next spg_bam_open reuses the buffers after this fill: same stream)
    int rc = add_batch(c, P->pos_begin, P->n_cols, P->offsets, nullptr, nullptr, P->n_entries, SPG_IN_TRUSTED, &pageable,
                       1, nullptr, nullptr, &F);
    if (pageable) HIPCHK(hipStreamSynchronize(c->copy_stream));
    return rc;
}

}  // extern "C"
