// spp_pileup.cpp — host BAM/SAM reader + htslib-faithful pileup emulator (include/spings_pileup.h).
//
// Replaces pysam.AlignmentFile.pileup() as driven by LiveVariantCaller.process_bam
// (variant_caller/live_variant_caller.py:54-72).  Two stages:
//   1. read: stream the file (BGZF blocks inflated in parallel, or SAM text), keep the reads of
//      one contig (position, reference end, flags, mate fields, CIGAR, base nibbles, qualities);
//   2. pileup: replay htslib's bam_plp_push / bam_plp_next bookkeeping exactly where it decides
//      anything (the maxcnt drop rule depends on when buffered reads are freed), apply the mate
//      overlap tweak, then write the CSR columns — every kept read contributes one entry to each
//      column of [pos, end) in read order, which is htslib's per-column order.
// Semantics restated from the published htslib sam.c / pysam libcalignmentfile.pyx (absent here:
// parity unpinned; oracle/pileup_port.py is the independent restatement the tests compare with).
#include "spings_pileup.h"
#include "spings_gpu.h"      // spg_records (the device-decode plan's view)

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <dlfcn.h>
#include <sys/mman.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <queue>
#include <random>
#include <cmath>
#include <stdexcept>
#include <string>
#include <string_view>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

thread_local std::string g_err;
int fail(const std::string &m) {
    g_err = m;
    return -1;
}

enum : uint32_t {   // SAM flags
    F_PAIRED = 0x1, F_PROPER = 0x2, F_UNMAP = 0x4, F_MUNMAP = 0x8, F_SECONDARY = 0x100,
    F_QCFAIL = 0x200, F_DUP = 0x400,
};
enum : uint32_t { C_M = 0, C_I = 1, C_D = 2, C_N = 3, C_S = 4, C_H = 5, C_P = 6, C_EQ = 7, C_X = 8 };

inline bool consumes_ref(uint32_t op) { return op == C_M || op == C_D || op == C_N || op == C_EQ || op == C_X; }
inline bool consumes_query(uint32_t op) { return op == C_M || op == C_I || op == C_S || op == C_EQ || op == C_X; }

// htslib seq_nt16_table: text base -> 4-bit code
struct Nt16 {
    uint8_t t[256];
    Nt16() {
        std::fill(t, t + 256, 15);
        const char *s = "=ACMGRSVTWYHKDBN";
        for (int i = 0; i < 16; i++) {
            t[(uint8_t)s[i]] = (uint8_t)i;
            t[(uint8_t)tolower(s[i])] = (uint8_t)i;
        }
        t[(uint8_t)'U'] = t[(uint8_t)'u'] = 8;
    }
} const NT16;

// resize() without value-initialisation: the parallel decoders write every element, and the first
// touch of fresh pages then happens on those threads rather than in a serial zero fill.
template <class T>
struct NoInit : std::allocator<T> {
    template <class U> struct rebind { using other = NoInit<U>; };
    NoInit() = default;
    template <class U> NoInit(const NoInit<U> &) {}
    template <class U, class... A> void construct(U *p, A &&...a) {
        if constexpr (sizeof...(A) == 0) ::new ((void *)p) U;
        else ::new ((void *)p) U(std::forward<A>(a)...);
    }
};
template <class T> using Vec = std::vector<T, NoInit<T>>;

// Process-wide pool of 2 MiB-aligned blocks (up to SPP_POOL_MB, default 4096 MiB, kept resident)
// (the pools are never destroyed: detached release threads may still return blocks / plans while
// the process exits)
std::mutex &g_pool_mu = *new std::mutex;
std::vector<std::pair<uint8_t *, size_t>> &g_pool = *new std::vector<std::pair<uint8_t *, size_t>>;
size_t g_pool_bytes = 0;
size_t pool_cap() {
    static const size_t cap = [] { const char *e = getenv("SPP_POOL_MB"); return (size_t)(e ? atoll(e) : 4096) << 20; }();
    return cap;
}
uint8_t *block_pool_get(size_t sz) {
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); i++)
            if (g_pool[i].second == sz) {
                uint8_t *b = g_pool[i].first;
                g_pool.erase(g_pool.begin() + (long)i);
                g_pool_bytes -= sz;
                return b;
            }
    }
    uint8_t *b = (uint8_t *)aligned_alloc(2u << 20, sz);
    if (!b) throw std::runtime_error("out of host memory for the reads");
    madvise(b, sz, MADV_HUGEPAGE);
    return b;
}
void block_pool_put(uint8_t *b, size_t sz) {
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (g_pool_bytes + sz <= pool_cap()) {
        g_pool.emplace_back(b, sz);
        g_pool_bytes += sz;
    } else {
        free(b);
    }
}

struct Reads {                 // one contig's reads, structure of arrays
    Vec<int64_t> pos, end, mpos, isize;
    Vec<int32_t> mtid;
    Vec<uint16_t> flag;
    Vec<uint8_t> mapq;
    Vec<uint64_t> cig_off, name_off;
    Vec<uint32_t> n_cig, l_seq;
    Vec<uint32_t> cigar;
    Vec<uint8_t *> bases;     // per read: l_seq nibble codes, then l_seq qualities (in `arena`);
                              // null for reads outside the decode window (spp_pileup_region)
    int64_t dlo = INT64_MIN, dhi = INT64_MAX;   // decode window: reads overlapping it keep bases
    int64_t max_span = 0;                       // longest reference span of any read of the contig
    bool decode(int64_t pos, int64_t end) const { return end > dlo && pos < dhi; }
    Vec<char> names;
    // bases storage: 2 MiB-aligned 64 MiB blocks (transparent huge pages requested), never moved, so
    // the decoders can fill a window's records in parallel without a serial grow-and-copy.  Blocks
    // come from a process-wide pool and go back to it: the next BAM reuses resident pages (no page
    // faults, no munmap on the critical path).
    struct Arena {
        std::vector<std::pair<uint8_t *, size_t>> blocks;
        uint8_t *cur = nullptr;
        size_t left = 0;
        Arena() = default;
        Arena(const Arena &) = delete;
        Arena &operator=(const Arena &) = delete;
        ~Arena() { clear(); }
        void clear() {                  // the blocks go back to the process-wide pool
            for (auto &b : blocks) block_pool_put(b.first, b.second);
            blocks.clear();
            cur = nullptr;
            left = 0;
        }
        uint8_t *alloc(size_t n) {
            if (n > left) {
                const size_t sz = std::max<size_t>(n + (2u << 20) - 1, 64u << 20) & ~(size_t)((2u << 20) - 1);
                cur = block_pool_get(sz);
                blocks.emplace_back(cur, sz);
                left = sz;
            }
            uint8_t *r = cur;
            cur += n;
            left -= n;
            return r;
        }
    } arena;
    // records plans (spp_pileup_plan_records): bases stay packed in the inflated BAM bytes `raw`; rec[r] is the
    // offset of read r's refID field there and bases[r] only marks reads inside the decode window
    uint8_t *raw = nullptr;
    Vec<uint64_t> rec;
    size_t qual_off(size_t r) const {
        return rec[r] + 32 + raw[rec[r] + 8] + 4 * (size_t)n_cig[r] + (l_seq[r] + 1) / 2;
    }
    // CIGAR op i / read name of read r (records plans: read in place, nothing copied)
    uint32_t cig(size_t r, uint32_t i) const {
        if (!raw) return cigar[cig_off[r] + i];
        uint32_t v;
        memcpy(&v, raw + rec[r] + 32 + raw[rec[r] + 8] + 4 * (size_t)i, 4);
        return v;
    }
    // device plans (spp_pileup_plan_fields): names known by their 64-bit hash only (pairs verified on the device)
    Vec<uint64_t> nhash;
    bool hashed = false;
    std::string name(size_t r) const { return std::string(name_view(r)); }
    std::string_view name_view(size_t r) const {        // (valid while the reads are: no copy)
        if (hashed) return std::string_view(reinterpret_cast<const char *>(nhash.data() + r), sizeof(uint64_t));
        if (!raw) return std::string_view(names.data() + name_off[r]);
        const uint8_t ln = raw[rec[r] + 8];
        return std::string_view((const char *)raw + rec[r] + 32, ln ? ln - 1u : 0u);
    }
    uint8_t *seq(size_t r) const { return bases[r]; }
    uint8_t *qual(size_t r) const { return raw ? raw + qual_off(r) : bases[r] + l_seq[r]; }
    uint8_t base(size_t r, uint32_t i) const {
        if (!raw) return bases[r][i];
        const uint8_t b = raw[rec[r] + 32 + raw[rec[r] + 8] + 4 * (size_t)n_cig[r] + i / 2];
        return (i & 1) ? (b & 15) : (b >> 4);
    }
    size_t size() const { return pos.size(); }
    void clear() {                      // empty, keeping every array's capacity (and its resident pages)
        pos.clear(); end.clear(); mpos.clear(); isize.clear(); mtid.clear(); flag.clear(); mapq.clear();
        cig_off.clear(); name_off.clear(); n_cig.clear(); l_seq.clear(); cigar.clear(); bases.clear();
        names.clear(); rec.clear(); nhash.clear();
        raw = nullptr;
        hashed = false;
        dlo = INT64_MIN; dhi = INT64_MAX; max_span = 0;
        arena.clear();
    }
};

struct Target {
    std::string name;
    int64_t len;
};

}  // namespace

struct spp_file {
    std::string path;
    bool bam = false;
    std::vector<Target> targets;
    std::unordered_map<std::string, int32_t> tid_of;
};

struct spp_plan;                   // the parsed reads between spp_pileup_plan and spp_batch_fill
void release_plan(spp_plan *p);

struct spp_batch {
    int64_t pos_begin = 0, n_cols = 0;
    uint64_t n_entries = 0;
    int64_t n_used = 0, n_dropped = 0;
    std::vector<uint64_t> off;
    uint8_t *code = nullptr, *qual = nullptr;
    bool owns = true;              // code / qual allocated here (else the caller's buffers)
    spp_plan *plan = nullptr;
    int threads = 1;
    ~spp_batch() {
        if (owns) {
            free(code);
            free(qual);
        }
        release_plan(plan);
    }
};

namespace {


// ---------------------------------------------------------------------------------------------
// Raw-deflate block decoder: libdeflate when the image has its runtime library (its whole-buffer
// decoder inflated this repository's 10,000x BAMs 1.4x faster than zlib's streaming inflate on one
// core; no header ships, so its three C entry points are bound with dlopen), else zlib.
// SPP_NO_LIBDEFLATE=1 forces zlib.
struct Inflater {
    using alloc_fn = void *(*)();
    using free_fn = void (*)(void *);
    using dec_fn = int (*)(void *, const void *, size_t, void *, size_t, size_t *);
    struct Api { alloc_fn alloc = nullptr; free_fn free = nullptr; dec_fn dec = nullptr; };
    static const Api &api() {
        static const Api a = [] {
            Api r;
            if (getenv("SPP_NO_LIBDEFLATE")) return r;
            void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
            if (!h) return r;
            r.alloc = (alloc_fn)dlsym(h, "libdeflate_alloc_decompressor");
            r.free = (free_fn)dlsym(h, "libdeflate_free_decompressor");
            r.dec = (dec_fn)dlsym(h, "libdeflate_deflate_decompress");
            if (!r.alloc || !r.free || !r.dec) r = Api{};
            return r;
        }();
        return a;
    }
    Inflater() {
        if (api().dec) ld_ = api().alloc();
        if (!ld_) {
            memset(&zs_, 0, sizeof(zs_));
            zok_ = inflateInit2(&zs_, -15) == Z_OK;
        }
    }
    ~Inflater() {
        if (ld_) api().free(ld_);
        else if (zok_) inflateEnd(&zs_);
    }
    // exactly ulen bytes from one raw-deflate member
    bool run(const uint8_t *in, size_t clen, uint8_t *out, size_t ulen) {
        if (ld_) {
            size_t got = 0;
            return api().dec(ld_, in, clen, out, ulen, &got) == 0 && got == ulen;
        }
        if (!zok_) return false;
        inflateReset(&zs_);
        zs_.next_in = const_cast<uint8_t *>(in);
        zs_.avail_in = (uInt)clen;
        zs_.next_out = out;
        zs_.avail_out = (uInt)ulen;
        return inflate(&zs_, Z_FINISH) == Z_STREAM_END && zs_.avail_out == 0;
    }
    void *ld_ = nullptr;
    z_stream zs_;
    bool zok_ = false;
};

// BGZF: blocks are independent raw-deflate members; inflate a window of blocks in parallel.
// ---------------------------------------------------------------------------------------------
class BgzfReader {
  public:
    BgzfReader(const std::string &path, int threads, size_t window = 0) : threads_(std::max(1, threads)) {
        if (window) window_ = std::max<size_t>(window, 65554);
        // SPP_BGZF_WINDOW (bytes, >= 65554): a smaller read window, for the boundary tests
        if (const char *w = getenv("SPP_BGZF_WINDOW")) window_ = std::max<size_t>(strtoull(w, nullptr, 10), 65554);
        f_ = fopen(path.c_str(), "rb");
        if (!f_) throw std::runtime_error("cannot open " + path);
    }
    ~BgzfReader() {
        if (f_) fclose(f_);
    }
    // Inflate the next window of blocks into out[gap:] (out is resized); false at EOF.
    bool next(Vec<uint8_t> &out, size_t gap) {
        Vec<uint8_t> &comp = comp_;
        comp.resize(window_);
        size_t n = carry_.size();
        std::copy(carry_.begin(), carry_.end(), comp.begin());
        n += fread(comp.data() + n, 1, window_ - n, f_);
        if (n == 0) return false;
        struct Blk { size_t off, clen, ulen; };
        std::vector<Blk> blks;
        size_t p = 0;
        while (p + 18 <= n) {
            const uint8_t *h = comp.data() + p;
            if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) throw std::runtime_error("not a BGZF block");
            const size_t xlen = h[10] | (h[11] << 8);
            size_t bsize = 0;
            for (size_t x = 12; x + 4 <= 12 + xlen;) {
                const size_t slen = h[x + 2] | (h[x + 3] << 8);
                if (h[x] == 66 && h[x + 1] == 67 && slen == 2) bsize = (h[x + 4] | (h[x + 5] << 8)) + 1;
                x += 4 + slen;
            }
            if (!bsize) throw std::runtime_error("BGZF block without BSIZE");
            if (p + bsize > n) break;
            const size_t ulen = (size_t)h[bsize - 4] | ((size_t)h[bsize - 3] << 8) | ((size_t)h[bsize - 2] << 16) |
                                ((size_t)h[bsize - 1] << 24);
            blks.push_back({p + 12 + xlen, bsize - xlen - 20, ulen});
            p += bsize;
        }
        if (blks.empty()) {
            if (feof(f_)) {
                if (n) throw std::runtime_error("truncated BGZF file");
                return false;
            }
            throw std::runtime_error("BGZF block larger than the read window");
        }
        carry_.assign(comp.begin() + p, comp.begin() + n);
        std::vector<size_t> uoff(blks.size() + 1, 0);
        for (size_t i = 0; i < blks.size(); i++) uoff[i + 1] = uoff[i] + blks[i].ulen;
        const size_t base = gap;
        out.resize(base + uoff.back());
        std::atomic<size_t> next_blk{0};
        std::atomic<bool> bad{false};
        auto work = [&]() {
            Inflater inf;
            for (size_t i; (i = next_blk++) < blks.size();) {
                if (blks[i].ulen == 0) continue;
                if (!inf.run(comp.data() + blks[i].off, blks[i].clen, out.data() + base + uoff[i], blks[i].ulen))
                    bad = true;
            }
        };
        const int nt = (int)std::min<size_t>(threads_, blks.size());
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(work);
        work();
        for (auto &t : pool) t.join();
        if (bad) throw std::runtime_error("BGZF inflate failed");
        return true;
    }

  private:
    size_t window_ = 16u << 20;      // compressed bytes read per window
    FILE *f_ = nullptr;
    int threads_;
    std::vector<uint8_t> carry_;
    Vec<uint8_t> comp_;
};

// Byte source over the decompressed BAM stream.  The next window is inflated on a helper thread
// while the caller parses the current one (refill() joins it); windows are inflated behind a
// kGap-byte head room into which the unparsed tail of the previous window (a partial record) is
// copied, so a refill swaps buffers instead of moving the window.
class BamStream {
  public:
    BamStream(const std::string &path, int threads, size_t window = 0) : z_(path, threads, window) { launch(); }
    ~BamStream() {
        if (pending_.joinable()) pending_.join();
    }
    size_t avail() const { return buf_.size() - cur_; }
    bool need(size_t n) {            // ensure n bytes available at cur_
        while (avail() < n)
            if (!refill()) return false;
        return true;
    }
    // Append the next inflated window (dropping the consumed prefix); false at EOF.  Pointers
    // from ptr() are invalidated.
    bool refill() {
        pending_.join();
        if (err_) std::rethrow_exception(err_);
        if (!more_) return false;
        const size_t carry = avail();
        if (carry <= kGap) {
            memcpy(next_.data() + kGap - carry, ptr(), carry);
            buf_.swap(next_);
            cur_ = kGap - carry;
        } else {                        // a record longer than the head room: concatenate
            Vec<uint8_t> joined(carry + next_.size() - kGap);
            memcpy(joined.data(), ptr(), carry);
            memcpy(joined.data() + carry, next_.data() + kGap, next_.size() - kGap);
            buf_.swap(joined);
            cur_ = 0;
        }
        launch();
        return true;
    }
    const uint8_t *ptr() const { return buf_.data() + cur_; }
    void skip(size_t n) { cur_ += n; }

  private:
    void launch() {
        pending_ = std::thread([this] {
            try {
                more_ = z_.next(next_, kGap);
            } catch (...) {
                err_ = std::current_exception();
            }
        });
    }
    static constexpr size_t kGap = 1u << 20;
    BgzfReader z_;
    Vec<uint8_t> buf_, next_;
    size_t cur_ = 0;
    bool more_ = false;
    std::exception_ptr err_;
    std::thread pending_;
};

inline int32_t rd32(const uint8_t *p) { int32_t v; memcpy(&v, p, 4); return v; }
inline uint32_t rdu32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint16_t rdu16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

bool is_bgzf(const std::string &path) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open " + path);
    uint8_t h[4] = {0, 0, 0, 0};
    const size_t n = fread(h, 1, 4, f);
    fclose(f);
    return n == 4 && h[0] == 31 && h[1] == 139;
}

void bam_header(BamStream &s, spp_file *f) {
    if (!s.need(12) || memcmp(s.ptr(), "BAM\1", 4) != 0) throw std::runtime_error("not a BAM file");
    const int32_t l_text = rd32(s.ptr() + 4);
    s.skip(8);
    if (!s.need((size_t)l_text + 4)) throw std::runtime_error("truncated BAM header");
    s.skip((size_t)l_text);
    const int32_t n_ref = rd32(s.ptr());
    s.skip(4);
    for (int32_t i = 0; i < n_ref; i++) {
        if (!s.need(4)) throw std::runtime_error("truncated BAM header");
        const int32_t l_name = rd32(s.ptr());
        if (!s.need((size_t)l_name + 8)) throw std::runtime_error("truncated BAM header");
        Target t;
        t.name.assign((const char *)s.ptr() + 4, (size_t)std::max(0, l_name - 1));
        t.len = rd32(s.ptr() + 4 + l_name);
        s.skip((size_t)l_name + 8);
        f->tid_of[t.name] = (int32_t)f->targets.size();
        f->targets.push_back(t);
    }
}

int64_t ref_len(const uint32_t *cig, uint32_t n) {
    int64_t l = 0;
    for (uint32_t i = 0; i < n; i++)
        if (consumes_ref(cig[i] & 0xF)) l += cig[i] >> 4;
    return l;
}

void push_read(Reads &R, int64_t pos, uint16_t flag, uint8_t mapq, int32_t mtid, int64_t mpos, int64_t isize,
               const uint32_t *cig, uint32_t n_cig, const char *name, size_t l_name) {
    R.pos.push_back(pos);
    R.end.push_back(pos + ref_len(cig, n_cig));
    R.flag.push_back(flag);
    R.mapq.push_back(mapq);
    R.mtid.push_back(mtid);
    R.mpos.push_back(mpos);
    R.isize.push_back(isize);
    R.cig_off.push_back(R.cigar.size());
    R.n_cig.push_back(n_cig);
    R.cigar.insert(R.cigar.end(), cig, cig + n_cig);
    R.name_off.push_back(R.names.size());
    R.names.insert(R.names.end(), name, name + l_name);
    R.names.push_back('\0');
}

// stepper read filter (pysam __advance_all / __advance_nofilter / __advance_samtools) + htslib's
// own unmapped skip in bam_plp_push
bool stepper_keeps(const spp_params &p, uint16_t flag, uint8_t mapq) {
    if (flag & F_UNMAP) return false;
    if (p.stepper == SPP_STEPPER_NOFILTER) return true;
    if (p.stepper == SPP_STEPPER_ALL) return !(flag & (F_UNMAP | F_SECONDARY | F_QCFAIL | F_DUP));
    if (flag & p.flag_filter) return false;
    if (mapq < p.min_mapping_quality) return false;
    if ((flag & F_PAIRED) && !(flag & F_PROPER)) return false;   // orphan (ignore_orphans default)
    return true;
}

// BAM records: the complete records of each inflated window are located serially (block_size
// hops; contig, sort order and the stepper filter read from the fixed header), then decoded into
// the Reads arrays in parallel.
void read_bam(const spp_file *f, int32_t tid, const spp_params &p, Reads &R) {
    const int nt = std::max(1, std::min(p.n_threads, 64));
    BamStream s(f->path, nt);
    spp_file tmp;
    bam_header(s, &tmp);
    // two 4-bit codes per packed byte, high nibble first
    static const auto pair_tab = [] {
        std::vector<uint16_t> t(256);
        for (int v = 0; v < 256; v++) t[(size_t)v] = (uint16_t)((v >> 4) | ((v & 0xF) << 8));
        return t;
    }();
    int64_t last_pos = -1;
    std::vector<const uint8_t *> recs;
    static const bool timing = getenv("SPP_TIMING") != nullptr;
    double t_scan = 0, t_dec = 0, t_wait = 0;
    auto now = [] { return std::chrono::steady_clock::now(); };
    for (;;) {
        auto ta = now();
        recs.clear();
        const uint8_t *pf = s.ptr();                   // linear prefetch ahead of the record hops
        while (s.avail() >= 4) {
            if (s.ptr() + 4096 > pf && s.avail() > 8192) {
                pf = s.ptr() + 8192;
                for (int l = 0; l < 4096; l += 64) __builtin_prefetch(pf - 4096 + l);
            }
            const uint32_t bs = rdu32(s.ptr());
            if (s.avail() < 4 + (size_t)bs) break;
            const uint8_t *b = s.ptr() + 4;
            if (bs < 32) throw std::runtime_error("truncated BAM record");
            if (rd32(b) == tid) {
                const int64_t pos = rd32(b + 4);
                if (pos < last_pos) throw std::runtime_error("BAM is not coordinate-sorted");
                last_pos = pos;
                if (stepper_keeps(p, rdu16(b + 14), b[9])) recs.push_back(b);
            }
            s.skip(4 + (size_t)bs);
        }
        const size_t k = recs.size(), n0 = R.size();
        auto tb = now();
        t_scan += std::chrono::duration<double>(tb - ta).count();
        if (k) {
            // per-read offsets into the variable-length arrays (serial prefix sums)
            R.pos.resize(n0 + k); R.end.resize(n0 + k); R.flag.resize(n0 + k); R.mapq.resize(n0 + k);
            R.mtid.resize(n0 + k); R.mpos.resize(n0 + k); R.isize.resize(n0 + k);
            R.cig_off.resize(n0 + k); R.n_cig.resize(n0 + k); R.name_off.resize(n0 + k);
            R.bases.resize(n0 + k); R.l_seq.resize(n0 + k);
            size_t co = R.cigar.size(), so = 0, no = R.names.size();
            std::vector<uint8_t> dec(k, 1);
            for (size_t i = 0; i < k; i++) {
                const uint8_t *b = recs[i];
                const uint32_t n_cig = rdu16(b + 12), l_seq = (uint32_t)rd32(b + 16), l_name = b[8];
                R.cig_off[n0 + i] = co; R.n_cig[n0 + i] = n_cig; co += n_cig;
                R.l_seq[n0 + i] = l_seq;
                R.name_off[n0 + i] = no; no += (l_name ? l_name - 1u : 0u) + 1u;
                if (R.dlo != INT64_MIN || R.dhi != INT64_MAX) {   // region: bases of the window's reads only
                    uint32_t cg[64];
                    int64_t span = 0;
                    for (uint32_t c0 = 0; c0 < n_cig; c0 += 64) {
                        const uint32_t m = std::min<uint32_t>(64, n_cig - c0);
                        memcpy(cg, b + 32 + l_name + 4u * c0, 4u * m);
                        span += ref_len(cg, m);
                    }
                    const int64_t pos = rd32(b + 4);
                    R.max_span = std::max(R.max_span, span);
                    dec[i] = R.decode(pos, pos + span) ? 1 : 0;
                }
                if (dec[i]) so += 2 * (size_t)l_seq;
            }
            R.cigar.resize(co); R.names.resize(no);
            uint8_t *bp = so ? R.arena.alloc(so) : nullptr;
            for (size_t i = 0; i < k; i++) {
                R.bases[n0 + i] = dec[i] ? bp : nullptr;
                if (dec[i]) bp += 2 * (size_t)R.l_seq[n0 + i];
            }
            auto work = [&](size_t i0, size_t i1) {
                for (size_t i = i0; i < i1; i++) {
                    const uint8_t *b = recs[i];
                    const size_t r = n0 + i;
                    const uint8_t l_name = b[8];
                    const uint32_t n_cig = R.n_cig[r], l_seq = R.l_seq[r];
                    R.pos[r] = rd32(b + 4);
                    R.mapq[r] = b[9];
                    R.flag[r] = rdu16(b + 14);
                    R.mtid[r] = rd32(b + 20);
                    R.mpos[r] = rd32(b + 24);
                    R.isize[r] = rd32(b + 28);
                    const uint8_t *name = b + 32;
                    const size_t ln = l_name ? l_name - 1u : 0u;
                    memcpy(R.names.data() + R.name_off[r], name, ln);
                    R.names[R.name_off[r] + ln] = '\0';
                    uint32_t *cg = R.cigar.data() + R.cig_off[r];
                    memcpy(cg, name + l_name, 4u * n_cig);
                    R.end[r] = R.pos[r] + ref_len(cg, n_cig);
                    if (!R.bases[r]) continue;                  // outside the decode window
                    const uint8_t *sq = name + l_name + 4u * n_cig;
                    const uint8_t *ql = sq + (l_seq + 1) / 2;
                    uint8_t *dst = R.seq(r);
                    for (uint32_t j = 0; j < l_seq / 2; j++) memcpy(dst + 2 * j, &pair_tab[sq[j]], 2);
                    if (l_seq & 1) dst[l_seq - 1] = sq[l_seq / 2] >> 4;
                    memcpy(R.qual(r), ql, l_seq);
                }
            };
            const size_t nw = std::min<size_t>((size_t)nt, (k + 4095) / 4096);
            std::vector<std::thread> pool;
            for (size_t t = 1; t < nw; t++) pool.emplace_back(work, k * t / nw, k * (t + 1) / nw);
            work(0, nw ? k / nw : k);
            for (auto &t : pool) t.join();
        }
        auto tc = now();
        t_dec += std::chrono::duration<double>(tc - tb).count();
        const bool more = s.refill();
        t_wait += std::chrono::duration<double>(now() - tc).count();
        if (!more) break;
    }
    if (timing) fprintf(stderr, "[spp timing] read_bam: scan %.1f ms, decode %.1f ms, wait for inflate %.1f ms\n",
                        t_scan * 1e3, t_dec * 1e3, t_wait * 1e3);
    if (s.avail()) throw std::runtime_error("truncated BAM record");
}

// ---------------------------------------------------------------------------------------------
// Records plans (spp_pileup_plan_records): the whole BAM inflated into one host buffer that goes to HBM
// as is; the GPU decodes bases / qualities and walks the CIGARs (spg_accumulate_records).
// ---------------------------------------------------------------------------------------------
spp_alloc_fn g_alloc = nullptr;
spp_free_fn g_free = nullptr;
std::atomic<spp_inflate_fn> g_inflate{nullptr};  // GPU inflater of the records plans (spp_set_inflater)

struct HostBuf {
    uint8_t *p = nullptr;
    size_t cap = 0;
    spp_free_fn fr = nullptr;      // allocator hook's release (null: free())
    void release() {
        if (!p) return;
        if (fr) fr(p);
        else free(p);
        p = nullptr;
        cap = 0;
    }
};
// Recycled buffers (pinned allocations cost ~0.2 s per GB; a 10,000x SARS-CoV-2 BAM inflates to ~0.6 GB)
std::mutex &g_buf_mu = *new std::mutex;
std::vector<HostBuf> &g_bufs = *new std::vector<HostBuf>;

HostBuf buf_get(size_t need, bool pinned = true) {
    const spp_free_fn want = pinned ? g_free : nullptr;
    {
        std::lock_guard<std::mutex> lk(g_buf_mu);
        size_t best = SIZE_MAX;
        for (size_t i = 0; i < g_bufs.size(); i++)
            if (g_bufs[i].cap >= need && g_bufs[i].fr == want && (best == SIZE_MAX || g_bufs[i].cap < g_bufs[best].cap))
                best = i;
        if (best != SIZE_MAX) {
            HostBuf b = g_bufs[best];
            g_bufs.erase(g_bufs.begin() + (long)best);
            return b;
        }
    }
    HostBuf b;
    b.cap = ((need + need / 16) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    if (g_alloc && pinned) {
        void *q = nullptr;
        if (g_alloc(b.cap, &q) != 0 || !q) throw std::runtime_error("host allocator failed");
        b.p = (uint8_t *)q;
        b.fr = g_free;
    } else {
        b.p = (uint8_t *)aligned_alloc(4096, b.cap);
        if (!b.p) throw std::runtime_error("out of host memory for the BAM records");
    }
    return b;
}

void buf_put(HostBuf &b) {
    if (!b.p) return;
    std::lock_guard<std::mutex> lk(g_buf_mu);
    size_t held = 0;
    for (auto &x : g_bufs) held += x.cap;
    if ((b.fr == g_free || !b.fr) && g_bufs.size() < 12 && held + b.cap <= ((size_t)6 << 30)) g_bufs.push_back(b);
    else b.release();
    b = HostBuf{};
}

// Persistent worker threads for par_chunks (a BAM's plan runs ~6 parallel loops; spawning 15 threads for each cost
// ~0.3-0.5 ms a loop).  A job's chunks are taken from its counter by its caller and by the workers that pop one of its
// queue entries; several host threads may run jobs at once (process_bams: the reader and the planner).  The caller
// returns only after every worker that took an entry of its job has left it (entries still queued are withdrawn).
struct ParJob {
    const std::function<void(int)> *run;
    int nt;
    std::atomic<int> next{1};
    std::mutex m;                        // guards left; the caller sleeps on cv until it is 0 (no spinning: the
    std::condition_variable cv;          // process's CPU quota is the workers')
    int left = 0;                        // queue entries not yet finished or withdrawn
    void leave(int k) {
        std::lock_guard<std::mutex> lk(m);
        left -= k;
        if (left == 0) cv.notify_one();
    }
};
struct ParPool {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<ParJob *> q;
    size_t n_threads = 0;
    static void work(ParJob *j) {
        for (int t; (t = j->next.fetch_add(1)) < j->nt;) (*j->run)(t);
    }
    void grow(size_t want) {              // (called under mu)
        for (; n_threads < want; n_threads++)
            std::thread([this] {
                for (;;) {
                    ParJob *j;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return !q.empty(); });
                        j = q.front();
                        q.pop_front();
                    }
                    work(j);
                    j->leave(1);
                }
            }).detach();
    }
};
ParPool &g_par = *new ParPool;           // (never destroyed: its detached workers wait on it until the process ends)

// Parallel chunked loop: fn(t, i0, i1) on nt threads over [0, n)
template <class Fn> void par_chunks(size_t n, int nt, Fn &&fn) {
    nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, (n + 16383) / 16384));
    std::exception_ptr err;
    std::mutex emu;
    const std::function<void(int)> run = [&](int t) {
        try {
            fn(t, n * (size_t)t / (size_t)nt, n * (size_t)(t + 1) / (size_t)nt);
        } catch (...) {
            std::lock_guard<std::mutex> lk(emu);
            if (!err) err = std::current_exception();
        }
    };
    if (nt == 1) {
        run(0);
    } else {
        ParJob j;
        j.run = &run;
        j.nt = nt;
        j.left = nt - 1;
        {
            std::lock_guard<std::mutex> lk(g_par.mu);
            g_par.grow((size_t)std::min(nt - 1, 63));
            for (int t = 1; t < nt; t++) g_par.q.push_back(&j);
        }
        g_par.cv.notify_all();
        run(0);
        ParPool::work(&j);
        {
            int withdrawn = 0;
            std::lock_guard<std::mutex> lk(g_par.mu);     // withdraw the entries no worker took
            for (auto it = g_par.q.begin(); it != g_par.q.end();) {
                if (*it == &j) { it = g_par.q.erase(it); withdrawn++; }
                else ++it;
            }
            if (withdrawn) j.leave(withdrawn);
        }
        std::unique_lock<std::mutex> lk(j.m);
        j.cv.wait(lk, [&] { return j.left == 0; });
    }
    if (err) std::rethrow_exception(err);
}

// n tasks on up to nt threads (no minimum work per thread, unlike par_chunks: a task here is a whole range)
template <class Fn> void par_tasks(size_t n, int nt, Fn &&fn) {
    nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, n));
    std::atomic<size_t> next{0};
    par_chunks((size_t)nt * 16384, nt, [&](int, size_t, size_t) {
        for (size_t i; (i = next++) < n;) fn(i);
    });
}

// The BAM mapped, its BGZF members located, inflated in parallel straight into `out` (the helpers take
// members in file order; this thread scans the records as the inflated prefix grows, inflating members
// itself while it waits), then the kept records' fixed fields parsed in parallel.  Bases and qualities
// stay packed in `out`.
// A BGZF BAM mapped and its members located (each member's payload offset / length and inflated length; uoff: the
// members' offsets in the inflated stream).  The mapping is released on a helper thread.
struct Blk { size_t off, clen, ulen; };
struct BamMap {
    const uint8_t *m = nullptr;
    size_t fsz = 0;
    std::vector<Blk> blks;
    std::vector<size_t> uoff;
    size_t total = 0;
    std::chrono::steady_clock::time_point tmm, tms;      // (SPP_TIMING) after the page touch / the parallel search
    BamMap() = default;
    BamMap(const BamMap &) = delete;
    BamMap &operator=(const BamMap &) = delete;
    bool mapped = true;                                   // (false: m is the caller's buffer)
    ~BamMap() {
        if (!m || !mapped) return;
        // (unmapped on a helper thread: tearing down the mapped pages took 5-12 ms per 0.2 GB; parallel preads into a
        // buffer instead of the mapping were slower still, 4 GB/s)
        void *mp = const_cast<uint8_t *>(m);
        const size_t n = fsz;
        try { std::thread([mp, n] { munmap(mp, n); }).detach(); } catch (...) { munmap(mp, n); }
    }
};

// preloaded: the file's bytes already in memory (fsz of them; spp_bam_map_open reads them into pinned memory), else
// the file is mapped
void map_bam(const std::string &path, int nt, BamMap &M, const uint8_t *preloaded = nullptr, size_t pre_size = 0) {
    size_t fsz = pre_size;
    if (!preloaded) {
        const int fd = open(path.c_str(), O_RDONLY);
        if (fd < 0) throw std::runtime_error("cannot open " + path);
        struct stat st;
        if (fstat(fd, &st) != 0) { close(fd); throw std::runtime_error("cannot stat " + path); }
        fsz = (size_t)st.st_size;
        if (fsz == 0) { close(fd); throw std::runtime_error("not a BAM file"); }
        void *mp = mmap(nullptr, fsz, PROT_READ, MAP_PRIVATE, fd, 0);
        close(fd);
        if (mp == MAP_FAILED) throw std::runtime_error("cannot map " + path);
        M.m = (const uint8_t *)mp;
    } else {
        if (fsz == 0) throw std::runtime_error("not a BAM file");
        M.m = preloaded;
        M.mapped = false;
    }
    M.fsz = fsz;
    const uint8_t *m = M.m;
    // The mapped file's pages faulted in by all threads at once, one touch per page: the member walk below
    // (a dependent chain per thread) and the inflate then run on mapped pages
    static const bool pretouch = [] { const char *e = getenv("SPP_PRETOUCH"); return !e || atoi(e) != 0; }();
    if (pretouch && !preloaded) {
        par_chunks((fsz + 4095) >> 12, nt, [&](int, size_t i0, size_t i1) {
            uint32_t acc = 0;
            for (size_t i = i0; i < i1; i++) acc += ((const volatile uint8_t *)m)[i << 12];
            (void)acc;
        });
    }
    const auto tmm = std::chrono::steady_clock::now();
    auto tms = tmm;
    std::vector<Blk> &blks = M.blks;
    // Members located in parallel: each thread finds the first member header in its byte range (a BGZF header
    // whose BSIZE chain reaches the next header), walks the chain to the next thread's start, and the chains
    // must meet exactly; otherwise (a false header inside compressed data, a damaged file) the serial walk
    // below locates them and reports the error.
    auto member = [&](size_t q, Blk *bk) -> size_t {      // member size at q, 0 if no valid header there
        if (q + 18 > fsz) return 0;
        const uint8_t *h = m + q;
        if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return 0;
        const size_t xlen = h[10] | (h[11] << 8);
        size_t bsize = 0;
        for (size_t x = 12; x + 4 <= 12 + xlen && q + x + 4 <= fsz;) {
            const size_t slen = h[x + 2] | (h[x + 3] << 8);
            if (h[x] == 66 && h[x + 1] == 67 && slen == 2 && q + x + 6 <= fsz) bsize = (h[x + 4] | (h[x + 5] << 8)) + 1;
            x += 4 + slen;
        }
        if (!bsize || q + bsize > fsz || bsize < xlen + 20) return 0;
        if (bk) *bk = {q + 12 + xlen, bsize - xlen - 20, (size_t)h[bsize - 4] | ((size_t)h[bsize - 3] << 8) |
                                                             ((size_t)h[bsize - 2] << 16) | ((size_t)h[bsize - 1] << 24)};
        return bsize;
    };
    {
        const int np = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, fsz >> 22));
        std::vector<size_t> start((size_t)np + 1, fsz);
        std::vector<std::vector<Blk>> part((size_t)np);
        std::atomic<bool> ok{np > 1};
        if (np > 1) {
            par_tasks((size_t)np, np, [&](size_t t) {
                {
                    if (t == 0) { start[0] = 0; return; }
                    for (size_t q = fsz * t / (size_t)np, e = fsz * (t + 1) / (size_t)np; q < e; q++) {
                        const size_t bs = member(q, nullptr);
                        if (bs && (q + bs == fsz || member(q + bs, nullptr))) { start[t] = q; break; }
                    }
                }
            });
            tms = std::chrono::steady_clock::now();
            for (int t = np - 1; t >= 1; t--) start[(size_t)t] = std::min(start[(size_t)t], start[(size_t)t + 1]);
            par_tasks((size_t)np, np, [&](size_t t) {
                {
                    size_t q = start[t];
                    Blk bk;
                    while (q < start[t + 1]) {
                        const size_t bs = member(q, &bk);
                        if (!bs) { ok = false; break; }
                        part[t].push_back(bk);
                        q += bs;
                    }
                    if (q != start[t + 1]) ok = false;
                }
            });
        }
        if (ok)
            for (auto &v : part) blks.insert(blks.end(), v.begin(), v.end());
    }
    for (size_t q = blks.empty() ? 0 : fsz; q < fsz;) {
        if (q + 18 > fsz) throw std::runtime_error("truncated BGZF file");
        const uint8_t *h = m + q;
        if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) throw std::runtime_error("not a BGZF block");
        const size_t xlen = h[10] | (h[11] << 8);
        size_t bsize = 0;
        for (size_t x = 12; x + 4 <= 12 + xlen && q + x + 4 <= fsz;) {
            const size_t slen = h[x + 2] | (h[x + 3] << 8);
            if (h[x] == 66 && h[x + 1] == 67 && slen == 2 && q + x + 6 <= fsz) bsize = (h[x + 4] | (h[x + 5] << 8)) + 1;
            x += 4 + slen;
        }
        if (!bsize) throw std::runtime_error("BGZF block without BSIZE");
        if (q + bsize > fsz || bsize < xlen + 20) throw std::runtime_error("truncated BGZF file");
        const size_t ulen = (size_t)h[bsize - 4] | ((size_t)h[bsize - 3] << 8) | ((size_t)h[bsize - 2] << 16) |
                            ((size_t)h[bsize - 1] << 24);
        blks.push_back({q + 12 + xlen, bsize - xlen - 20, ulen});
        q += bsize;
    }
    const size_t nb = blks.size();
    M.uoff.assign(nb + 1, 0);
    for (size_t i = 0; i < nb; i++) M.uoff[i + 1] = M.uoff[i] + blks[i].ulen;
    M.total = M.uoff[nb];
    M.tmm = tmm;
    M.tms = tms;
}

// Offset of the first record in the inflated stream (the header's end) and the header's reference count: the first
// members inflated on this thread until the header is complete
uint64_t header_end(const BamMap &M, int32_t *n_ref) {
    std::vector<uint8_t> h;
    Inflater inf;
    size_t k = 0;
    auto need = [&](size_t n) -> bool {
        while (h.size() < n) {
            if (k >= M.blks.size()) return false;
            const Blk &b = M.blks[k++];
            const size_t at = h.size();
            h.resize(at + b.ulen);
            if (b.ulen && !inf.run(M.m + b.off, b.clen, h.data() + at, b.ulen)) throw std::runtime_error("BGZF inflate failed");
        }
        return true;
    };
    if (!need(12) || memcmp(h.data(), "BAM\1", 4) != 0) throw std::runtime_error("not a BAM file");
    size_t cur = 8 + (size_t)(uint32_t)rd32(h.data() + 4);
    if (!need(cur + 4)) throw std::runtime_error("truncated BAM header");
    const int32_t nr = rd32(h.data() + cur);
    cur += 4;
    for (int32_t i = 0; i < nr; i++) {
        if (!need(cur + 4)) throw std::runtime_error("truncated BAM header");
        const size_t l_name = (size_t)(uint32_t)rd32(h.data() + cur);
        if (!need(cur + 8 + l_name)) throw std::runtime_error("truncated BAM header");
        cur += 8 + l_name;
    }
    *n_ref = nr;
    return cur;
}

size_t read_bam_raw(const spp_file *f, int32_t tid, const spp_params &p, Reads &R, HostBuf &out) {
    const int nt = std::max(1, std::min(p.n_threads, 64));
    const auto tm0 = std::chrono::steady_clock::now();
    BamMap M;
    map_bam(f->path, nt, M);
    const uint8_t *m = M.m;
    const size_t fsz = M.fsz;
    const std::vector<Blk> &blks = M.blks;
    const std::vector<size_t> &uoff = M.uoff;
    const size_t nb = blks.size(), total = M.total;
    const auto tmm = M.tmm, tms = M.tms;
    const auto tm1 = std::chrono::steady_clock::now();
    out = buf_get(total + 64);
    const auto tm2 = std::chrono::steady_clock::now();
    uint8_t *buf = out.p;
    memset(buf + total, 0, 64);
    std::unique_ptr<std::atomic<uint8_t>[]> done(new std::atomic<uint8_t>[nb ? nb : 1]);
    for (size_t i = 0; i < nb; i++) done[i].store(0, std::memory_order_relaxed);
    std::atomic<size_t> next{0};
    std::atomic<bool> bad{false};
    auto inflate_one = [&](Inflater &inf, size_t i) {
        if (blks[i].ulen && !inf.run(m + blks[i].off, blks[i].clen, buf + uoff[i], blks[i].ulen)) bad = true;
        done[i].store(1, std::memory_order_release);
    };
    // GPU inflate (spp_set_inflater): the mapped file's bytes copied into pinned staging in parallel, every member
    // inflated on the device (one call: upload, kernel, download into `buf`); members it reports bad — and all of them
    // if the call fails — are inflated here below.  The host's threads are then free for the record scan.
    // Only BAMs of many members: a member is a dependent chain of ~17k symbols on the GPU (~19 ms however few there
    // are), the host's threads inflate ~80 members per ms (r04zf); SPP_GPU_INFLATE_MIN overrides the 4096 floor.
    const size_t gpu_min = p.inflate_min_members > 0 ? (size_t)p.inflate_min_members : (size_t)4096;
    bool gpu_inflated = false;
    if (const spp_inflate_fn gfn = g_inflate.load(); gfn && p.inflate_device >= 0 && nb > 0 && nb >= gpu_min) {
        struct GM { uint64_t coff; uint32_t clen, ulen; uint64_t uoff; };
        std::vector<GM> gm(nb);
        for (size_t i = 0; i < nb; i++) gm[i] = {blks[i].off, (uint32_t)blks[i].clen, (uint32_t)blks[i].ulen, uoff[i]};
        auto gms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
        const auto g0 = std::chrono::steady_clock::now();
        HostBuf cb = buf_get(fsz + 64);
        const auto g1 = std::chrono::steady_clock::now();
        par_chunks(fsz, nt, [&](int, size_t a, size_t b) { memcpy(cb.p + a, m + a, b - a); });
        const auto g2 = std::chrono::steady_clock::now();
        std::vector<uint32_t> gst(nb, 1);
        float kms = 0.f;
        const bool ok_call = gfn(p.inflate_device, cb.p, fsz, gm.data(), (int64_t)nb, buf, total, gst.data(), &kms) == 0;
        const auto g3 = std::chrono::steady_clock::now();
        buf_put(cb);
        size_t nbad = nb;
        if (ok_call) {
            gpu_inflated = true;
            nbad = 0;
            for (size_t i = 0; i < nb; i++) {
                if (gst[i] == 0) done[i].store(1, std::memory_order_relaxed);
                else nbad++;
            }
        }
        if (getenv("SPP_TIMING"))
            fprintf(stderr, "[spp timing] gpu inflate: staging buffer %.1f ms, copy %.1f ms, call %.1f ms (kernel %.1f ms), "
                    "%zu of %zu members left to the host\n", gms(g0, g1), gms(g1, g2), gms(g2, g3), kms, nbad, nb);
    }
    std::vector<std::thread> pool;
    struct Join { std::vector<std::thread> &v; std::atomic<size_t> &nx; size_t n;
                  ~Join() { nx = n; for (auto &t : v) if (t.joinable()) t.join(); } } join{pool, next, nb};
    // (after a GPU inflate the helpers only redo the members it reported bad)
    if (gpu_inflated) {
        std::vector<size_t> redo;
        for (size_t i = 0; i < nb; i++)
            if (!done[i].load(std::memory_order_relaxed)) redo.push_back(i);
        Inflater rinf;
        for (size_t i : redo) inflate_one(rinf, i);
        next = nb;
    }
    for (int t = 1; t < nt && !gpu_inflated; t++)
        pool.emplace_back([&] {
            Inflater inf;
            for (size_t i; (i = next++) < nb;) inflate_one(inf, i);
        });
    Inflater minf;
    size_t ready = 0, nready = 0;
    auto avail_to = [&](size_t end) -> bool {   // bytes [0, end) inflated (false: past the end of the BAM)
        while (ready < end) {
            if (bad) throw std::runtime_error("BGZF inflate failed");
            if (nready < nb && done[nready].load(std::memory_order_acquire)) { ready = uoff[++nready]; continue; }
            if (nready == nb) return false;
            const size_t i = next++;
            if (i < nb) inflate_one(minf, i);
            else std::this_thread::yield();
        }
        return true;
    };
    if (!avail_to(12) || memcmp(buf, "BAM\1", 4) != 0) throw std::runtime_error("not a BAM file");
    size_t cur = 8 + (size_t)(uint32_t)rd32(buf + 4);
    if (!avail_to(cur + 4)) throw std::runtime_error("truncated BAM header");
    const int32_t n_ref = rd32(buf + cur);
    cur += 4;
    for (int32_t i = 0; i < n_ref; i++) {
        if (!avail_to(cur + 4)) throw std::runtime_error("truncated BAM header");
        const size_t l_name = (size_t)(uint32_t)rd32(buf + cur);
        if (!avail_to(cur + 8 + l_name)) throw std::runtime_error("truncated BAM header");
        cur += 8 + l_name;
    }
    int64_t last_pos = -1;
    static const bool timing = getenv("SPP_TIMING") != nullptr;
    // (off by default: under the GPU box's 16-CPU quota the second pass over the inflated stream cost more than the serial
    // scan that follows the inflate frontier, 85.6 vs 73.3 ms per 10,000x BAM, profiles/r04s; SPP_PAR_SCAN=1 enables)
    static const bool par_scan = [] { const char *e = getenv("SPP_PAR_SCAN"); return e && atoi(e) != 0; }();
    const auto t0 = std::chrono::steady_clock::now();
    // Record boundaries in parallel: the inflated stream (once every member is in) split into nt ranges; each range's
    // first record is found by a validated chain — a block_size hop whose fixed fields are plausible (refIDs in range,
    // lengths inside block_size, a NUL-terminated name) eight records in a row — the ranges are scanned at once, and
    // the chains must meet exactly (each range's scan ends on the next range's start).  Otherwise (a false start
    // inside a record, a damaged file) the serial scan below walks the stream from the header, as before.
    bool scanned = false;
    const size_t body = cur;
    auto tps = t0;                               // (SPP_TIMING) start of the parallel record scan
    if ((par_scan || gpu_inflated) && nt > 1 && nb > 0 && total > body + ((size_t)nt << 20) && avail_to(total)) {
        auto rec_len = [&](size_t x) -> size_t {        // plausible record at x: 4 + block_size, else 0
            if (x + 40 > total) return 0;
            const uint32_t bs = rdu32(buf + x);
            if (bs < 32 || bs > (1u << 26) || x + 4 + (size_t)bs > total) return 0;
            const uint8_t *b = buf + x + 4;
            const int32_t ref = rd32(b), mref = rd32(b + 20), pos = rd32(b + 4);
            if (ref < -1 || ref >= n_ref || mref < -1 || mref >= n_ref || pos < -1) return 0;
            const uint32_t l_name = b[8], n_cig = rdu16(b + 12);
            const int32_t l_seq = rd32(b + 16);
            if (l_name < 1 || l_seq < 0 || 32ull + l_name + 4ull * n_cig + ((uint64_t)l_seq + 1) / 2 + (uint64_t)l_seq > bs)
                return 0;
            if (b[32 + l_name - 1] != 0) return 0;
            return 4 + (size_t)bs;
        };
        // np ranges, CH of them per thread: a thread steps its CH chains in turn, so CH record-header loads (each the
        // next hop of a dependent walk over bytes no CPU cache holds yet) are in flight at once instead of one
        tps = std::chrono::steady_clock::now();
        static const int CH = [] { const char *e = getenv("SPP_SCAN_CHAINS"); const int v = e ? atoi(e) : 8; return v >= 1 && v <= 32 ? v : 8; }();
        const int np = total > body + ((size_t)nt * (size_t)CH << 20) ? nt * CH : nt;
        const int ch = np / nt;
        std::vector<size_t> start((size_t)np + 1, total);
        start[0] = body;
        par_tasks((size_t)np - 1, nt, [&](size_t t1) {
            {
                const size_t t = t1 + 1;
                const size_t b0 = body + (total - body) * t / (size_t)np, lim = std::min(total, b0 + ((size_t)1 << 20));
                for (size_t x = b0; x < lim; x++) {
                    size_t y = x;
                    int k = 0;
                    for (; k < 8 && y < total; k++) {
                        const size_t len = rec_len(y);
                        if (!len) break;
                        y += len;
                    }
                    if (k == 8 || y == total) { start[t] = x; break; }
                }
            }
        });
        for (int t = np - 1; t >= 1; t--) start[(size_t)t] = std::min(start[(size_t)t], start[(size_t)t + 1]);
        std::vector<Vec<uint64_t>> part((size_t)np);
        std::vector<int64_t> first_pos((size_t)np, INT64_MAX), last_p((size_t)np, -1);
        std::atomic<bool> ok{true}, unsorted{false};
        par_tasks((size_t)nt, nt, [&](size_t w) {
            {
                const size_t r0 = w * (size_t)ch;
                size_t q[32];
                int64_t lp[32];
                int live = 0;
                for (int j = 0; j < ch; j++) { q[j] = start[r0 + (size_t)j]; lp[j] = -1; live += q[j] < start[r0 + (size_t)j + 1]; }
                while (live > 0) {
                    for (int j = 0; j < ch; j++) {
                        const size_t t = r0 + (size_t)j, qq = q[j];
                        if (qq >= start[t + 1]) continue;
                        const uint32_t bs = rdu32(buf + qq);
                        if (bs < 32 || qq + 4 + (size_t)bs > total) { ok = false; q[j] = start[t + 1] + 1; live--; continue; }
                        const uint8_t *b = buf + qq + 4;
                        if (rd32(b) == tid) {
                            const int64_t pos = rd32(b + 4);
                            if (pos < lp[j]) unsorted = true;
                            if (first_pos[t] == INT64_MAX) first_pos[t] = pos;
                            lp[j] = pos;
                            if (stepper_keeps(p, rdu16(b + 14), b[9])) part[t].push_back(qq + 4);
                        }
                        q[j] = qq + 4 + (size_t)bs;
                        if (q[j] >= start[t + 1]) { live--; if (q[j] != start[t + 1]) ok = false; }
                    }
                }
                for (int j = 0; j < ch; j++) last_p[r0 + (size_t)j] = lp[j];
            }
        });
        if (ok) {
            for (int t = 0; t < np; t++) {
                if (first_pos[(size_t)t] != INT64_MAX && first_pos[(size_t)t] < last_pos) unsorted = true;
                if (last_p[(size_t)t] >= 0) last_pos = last_p[(size_t)t];
            }
            if (unsorted) throw std::runtime_error("BAM is not coordinate-sorted");
            size_t nrec = 0;
            for (auto &v : part) nrec += v.size();
            R.rec.resize(nrec);
            size_t at = 0;
            for (auto &v : part) { if (!v.empty()) memcpy(R.rec.data() + at, v.data(), v.size() * sizeof(uint64_t)); at += v.size(); }
            cur = total;
            scanned = true;
        }
    }
    while (!scanned && avail_to(cur + 4)) {
        const uint32_t bs = rdu32(buf + cur);
        if (bs < 32 || !avail_to(cur + 4 + (size_t)bs)) throw std::runtime_error("truncated BAM record");
        const uint8_t *b = buf + cur + 4;
        if (rd32(b) == tid) {
            const int64_t pos = rd32(b + 4);
            if (pos < last_pos) throw std::runtime_error("BAM is not coordinate-sorted");
            last_pos = pos;
            if (stepper_keeps(p, rdu16(b + 14), b[9])) R.rec.push_back(cur + 4);
        }
        cur += 4 + (size_t)bs;
    }
    if (cur != total) throw std::runtime_error("truncated BAM record");
    const auto t1 = std::chrono::steady_clock::now();
    R.raw = buf;
    // fixed fields of the kept records, in parallel (names and CIGARs stay in place: Reads::name / Reads::cig)
    const size_t k = R.rec.size();
    R.pos.resize(k); R.end.resize(k); R.flag.resize(k); R.mapq.resize(k); R.mtid.resize(k); R.mpos.resize(k);
    R.isize.resize(k); R.n_cig.resize(k); R.bases.resize(k); R.l_seq.resize(k);
    const int nw = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, (k + 16383) / 16384));
    std::vector<int64_t> spans((size_t)nw, 0);
    par_chunks(k, nw, [&](int t, size_t i0, size_t i1) {
        int64_t span = 0;
        for (size_t i = i0; i < i1; i++) {
            const uint8_t *b = buf + R.rec[i];
            const uint32_t bs = rdu32(b - 4), n_cig = rdu16(b + 12), l_name = b[8];
            const int32_t l_seq = rd32(b + 16);
            if (l_seq < 0 || 32ull + l_name + 4ull * n_cig + ((uint64_t)l_seq + 1) / 2 + (uint64_t)l_seq > bs)
                throw std::runtime_error("corrupt BAM record (field lengths exceed block_size)");
            R.n_cig[i] = n_cig;
            R.l_seq[i] = (uint32_t)l_seq;
            R.pos[i] = rd32(b + 4);
            R.mapq[i] = b[9];
            R.flag[i] = rdu16(b + 14);
            R.mtid[i] = rd32(b + 20);
            R.mpos[i] = rd32(b + 24);
            R.isize[i] = rd32(b + 28);
            const uint8_t *cg = b + 32 + l_name;
            int64_t rl = 0;
            for (uint32_t j = 0; j < n_cig; j++) {
                const uint32_t c = rdu32(cg + 4 * (size_t)j);
                if (consumes_ref(c & 0xF)) rl += c >> 4;
            }
            R.end[i] = R.pos[i] + rl;
            span = std::max(span, rl);
            R.bases[i] = R.decode(R.pos[i], R.end[i]) ? const_cast<uint8_t *>(b) : nullptr;
        }
        spans[(size_t)t] = span;
    });
    for (int64_t v : spans) R.max_span = std::max(R.max_span, v);
    if (timing)
        fprintf(stderr, "[spp timing] read_bam_raw: %zu members, map %.1f ms + search %.1f ms + members %.1f ms, buffer %.1f ms, inflate+scan %.1f ms "
                "(parallel scan %.1f ms), fields %.1f ms\n", nb, std::chrono::duration<double, std::milli>(tmm - tm0).count(),
                std::chrono::duration<double, std::milli>(tms - tmm).count(),
                std::chrono::duration<double, std::milli>(tm1 - tms).count(),
                std::chrono::duration<double, std::milli>(tm2 - tm1).count(),
                std::chrono::duration<double, std::milli>(t1 - t0).count(),
                scanned ? std::chrono::duration<double, std::milli>(t1 - tps).count() : 0.0,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
    return total;
}

void sam_header_line(spp_file *f, const std::string &line) {
    if (line.compare(0, 3, "@SQ") != 0) return;
    Target t;
    t.len = 0;
    size_t p = 0;
    while ((p = line.find('\t', p)) != std::string::npos) {
        ++p;
        const size_t q = line.find('\t', p);
        const std::string fld = line.substr(p, q == std::string::npos ? std::string::npos : q - p);
        if (fld.compare(0, 3, "SN:") == 0) t.name = fld.substr(3);
        if (fld.compare(0, 3, "LN:") == 0) t.len = atoll(fld.c_str() + 3);
    }
    f->tid_of[t.name] = (int32_t)f->targets.size();
    f->targets.push_back(t);
}

template <class F>
void for_lines(const std::string &path, F &&fn) {
    FILE *fp = fopen(path.c_str(), "rb");
    if (!fp) throw std::runtime_error("cannot open " + path);
    std::string line;
    std::vector<char> buf(1 << 20);
    std::string carry;
    size_t n;
    bool stop = false;
    while (!stop && (n = fread(buf.data(), 1, buf.size(), fp)) > 0) {
        size_t s = 0;
        for (size_t i = 0; i < n; i++)
            if (buf[i] == '\n') {
                carry.append(buf.data() + s, i - s);
                if (!carry.empty() && carry.back() == '\r') carry.pop_back();
                if (!fn(carry)) { stop = true; break; }
                carry.clear();
                s = i + 1;
            }
        if (!stop) carry.append(buf.data() + s, n - s);
    }
    if (!stop && !carry.empty()) fn(carry);
    fclose(fp);
}

void read_sam(const spp_file *f, int32_t tid, const spp_params &p, Reads &R) {
    const std::string &want = f->targets[(size_t)tid].name;
    int64_t last_pos = -1;
    std::vector<uint32_t> cig;
    for_lines(f->path, [&](const std::string &line) {
        if (line.empty() || line[0] == '@') return true;
        const char *fld[11];
        size_t len[11];
        size_t s = 0;
        for (int k = 0; k < 11; k++) {
            const size_t e = line.find('\t', s);
            if (e == std::string::npos && k < 10) throw std::runtime_error("SAM record with < 11 fields");
            fld[k] = line.data() + s;
            len[k] = (e == std::string::npos ? line.size() : e) - s;
            s = e + 1;
        }
        if (std::string(fld[2], len[2]) != want) return true;
        const uint16_t flag = (uint16_t)atoi(fld[1]);
        const int64_t pos = atoll(fld[3]) - 1;
        const uint8_t mapq = (uint8_t)atoi(fld[4]);
        if (pos < last_pos) throw std::runtime_error("SAM is not coordinate-sorted");
        last_pos = pos;
        if (!stepper_keeps(p, flag, mapq)) return true;
        cig.clear();
        if (!(len[5] == 1 && fld[5][0] == '*')) {
            uint32_t v = 0;
            for (size_t i = 0; i < len[5]; i++) {
                const char c = fld[5][i];
                if (c >= '0' && c <= '9') { v = v * 10 + (uint32_t)(c - '0'); continue; }
                const char *ops = "MIDNSHP=X";
                const char *o = strchr(ops, c);
                if (!o || !*o) throw std::runtime_error("bad CIGAR");
                cig.push_back(v << 4 | (uint32_t)(o - ops));
                v = 0;
            }
        }
        const std::string rnext(fld[6], len[6]);
        int32_t mtid = -1;
        if (rnext == "=") mtid = tid;
        else if (rnext != "*") { auto it = f->tid_of.find(rnext); mtid = it == f->tid_of.end() ? -1 : it->second; }
        const int64_t mpos = atoll(fld[7]) - 1, isize = atoll(fld[8]);
        push_read(R, pos, flag, mapq, mtid, mpos, isize, cig.data(), (uint32_t)cig.size(), fld[0], len[0]);
        const bool noseq = len[9] == 1 && fld[9][0] == '*';
        const uint32_t l_seq = noseq ? 0u : (uint32_t)len[9];
        R.l_seq.push_back(l_seq);
        R.max_span = std::max(R.max_span, R.end.back() - pos);
        if (!R.decode(pos, R.end.back())) { R.bases.push_back(nullptr); return true; }
        uint8_t *bp = R.arena.alloc(2 * (size_t)l_seq);
        R.bases.push_back(bp);
        for (uint32_t i = 0; i < l_seq; i++) bp[i] = NT16.t[(uint8_t)fld[9][i]];
        const bool noq = len[10] == 1 && fld[10][0] == '*';
        if (!noq && len[10] != l_seq) throw std::runtime_error("SAM QUAL length differs from SEQ");
        for (uint32_t i = 0; i < l_seq; i++) bp[l_seq + i] = noq ? 0xFF : (uint8_t)(fld[10][i] - 33);
        return true;
    });
}

// htslib mate-overlap quality tweak (sam.c tweak_overlap_quality): at every reference position
// where both mates have an aligned M/=/X base, equal bases -> a.q = min(a.q + b.q, 200), b.q = 0;
// different bases -> the higher (a on ties) keeps 0.8 * q (truncated), the other gets 0.
void tweak_overlap(Reads &R, size_t a, size_t b) {
    auto aligned = [&](size_t r, std::vector<std::pair<int64_t, uint32_t>> &out) {
        int64_t x = R.pos[r];
        uint32_t y = 0;
        for (uint32_t i = 0; i < R.n_cig[r]; i++) {
            const uint32_t c = R.cig(r, i), op = c & 0xF, l = c >> 4;
            if (op == C_M || op == C_EQ || op == C_X)
                for (uint32_t k = 0; k < l; k++) out.emplace_back(x + k, y + k);
            if (consumes_ref(op)) x += l;
            if (consumes_query(op)) y += l;
        }
    };
    std::vector<std::pair<int64_t, uint32_t>> pa, pb;
    aligned(a, pa);
    aligned(b, pb);
    size_t i = 0, j = 0;
    while (i < pa.size() && j < pb.size()) {
        if (pa[i].first < pb[j].first) { i++; continue; }
        if (pb[j].first < pa[i].first) { j++; continue; }
        const uint32_t ia = pa[i].second, ib = pb[j].second;
        if (ia >= R.l_seq[a] || ib >= R.l_seq[b]) return;
        uint8_t &qa = R.qual(a)[ia], &qb = R.qual(b)[ib];
        if (R.base(a, ia) == R.base(b, ib)) {
            const int q = qa + qb;
            qa = (uint8_t)(q > 200 ? 200 : q);
            qb = 0;
        } else if (qa >= qb) {
            qa = (uint8_t)(0.8 * qa);
            qb = 0;
        } else {
            qb = (uint8_t)(0.8 * qb);
            qa = 0;
        }
        i++;
        j++;
    }
}

// Overlap tweaks happen when the second mate is pushed; columns before the iterator's pending
// position were already handed out by then (pysam reads qual[qpos] at that time).  Only the D/N
// entries of the first mate can point (next query base) at a tweaked base in such a column, so
// the first mate's original qualities are kept for the columns before `col`.
struct Tweaks {
    std::vector<int64_t> col;                                   // per read; INT64_MAX = none
    std::unordered_map<size_t, std::vector<uint8_t>> orig;      // first mate -> qualities before
    bool defer = false;                                         // device plans: record the pairs, tweak nothing here
    std::vector<std::pair<size_t, size_t>> pairs;               // (first mate, second mate) in push order
};

// The live buffer's reads keyed by end, for "free every read with end <= col" (the order among equal
// ends is immaterial).  A bucket ring over end positions: a live read's end lies within its span of
// the scan position, so ends in [lo, lo + S) index the ring directly (O(1) push and pop; a binary
// heap took ~45 % of the reads at 10,000x, whose ends are not monotone); ends beyond the ring (after
// a coverage gap) wait in an overflow heap.
struct EndQueue {
    using E = std::pair<int64_t, size_t>;
    std::vector<std::vector<size_t>> ring;
    size_t mask = 0;
    int64_t lo = INT64_MIN;             // every end < lo has been popped
    size_t cnt = 0;                     // reads in the ring
    std::priority_queue<E, std::vector<E>, std::greater<E>> ov;
    explicit EndQueue(int64_t max_span) {
        size_t S = 64;
        while ((int64_t)S < max_span + 2 && S < ((size_t)1 << 20)) S <<= 1;
        ring.resize(S);
        mask = S - 1;
    }
    size_t size() const { return cnt + ov.size(); }
    void emplace(int64_t end, size_t r) {
        if (cnt == 0 && end >= lo) lo = end;          // empty ring: start it at this end
        if (end >= lo && end - lo < (int64_t)ring.size()) {
            ring[(size_t)end & mask].push_back(r);
            cnt++;
        } else {
            ov.emplace(end, r);
        }
    }
    template <class Fn> void pop_upto(int64_t col, Fn &&fn) {
        while (!ov.empty() && ov.top().first <= col) {
            const size_t r = ov.top().second;
            ov.pop();
            fn(r);
        }
        if (cnt == 0) {
            if (col >= lo) lo = col + 1;
            return;
        }
        for (; lo <= col && cnt; lo++) {
            std::vector<size_t> &b = ring[(size_t)lo & mask];
            for (size_t r : b) fn(r);
            cnt -= b.size();
            b.clear();
        }
        if (cnt == 0 && col >= lo) lo = col + 1;
    }
};

// htslib's overlap hash (read name -> the first mate still waiting for its partner) as a flat open-addressing table:
// linear probing over 64-bit name keys (the reads' FNV-1a name hashes when the names are hashed, a hash of the name
// otherwise, equal keys confirmed by comparing the names), backward-shift deletion, no allocation per entry.  The
// node-based map it replaces cost ~10 ms per 10,000x BAM at max_depth 8000 (every read the cap drops is looked up).
struct OlapTable {
    std::vector<uint64_t> key;
    std::vector<uint32_t> val;                 // read index + 1; 0 = empty slot
    size_t mask = 0, n = 0;
    explicit OlapTable(size_t cap = (size_t)1 << 16) { reset(cap); }
    void reset(size_t cap) {
        key.assign(cap, 0);
        val.assign(cap, 0);
        mask = cap - 1;
        n = 0;
    }
    static size_t slot0(uint64_t k) { return (size_t)((k * 0x9E3779B97F4A7C15ull) >> 20); }
    // the slot holding a read whose name equals r's (same key, eq(read) true), or SIZE_MAX
    template <class Eq> size_t find(uint64_t k, Eq &&eq) const {
        for (size_t i = slot0(k) & mask;; i = (i + 1) & mask) {
            if (!val[i]) return SIZE_MAX;
            if (key[i] == k && eq((size_t)val[i] - 1)) return i;
        }
    }
    void insert(uint64_t k, size_t r) {
        if (2 * (n + 1) > mask + 1) grow();
        size_t i = slot0(k) & mask;
        while (val[i]) i = (i + 1) & mask;
        key[i] = k;
        val[i] = (uint32_t)(r + 1);
        n++;
    }
    size_t at(size_t i) const { return (size_t)val[i] - 1; }
    void erase(size_t i) {                     // backward shift: later entries of the probe run move up
        size_t j = i;
        while (true) {
            j = (j + 1) & mask;
            if (!val[j]) break;
            const size_t h = slot0(key[j]) & mask;
            // entry j may fill the hole at i when its home slot h is not cyclically in (i, j]
            if ((j > i && (h <= i || h > j)) || (j < i && (h <= i && h > j))) {
                key[i] = key[j];
                val[i] = val[j];
                i = j;
            }
        }
        val[i] = 0;
        n--;
    }
    bool empty() const { return n == 0; }
    void grow() {
        std::vector<uint64_t> k0;
        std::vector<uint32_t> v0;
        k0.swap(key);
        v0.swap(val);
        reset(2 * (mask + 1));
        for (size_t i = 0; i < v0.size(); i++)
            if (v0[i]) insert(k0[i], (size_t)v0[i] - 1);
    }
};

// The depth cap alone, per position instead of per read, when nothing else of simulate() below applies: reads sorted,
// each spanning >= 1 column, and no read a mate-overlap candidate (single-end data, or ignore_overlaps off).  Then the
// replay reduces to: the iterator stands at the previous read position when the first read at p is pushed (never
// dropped), and at p for the others, with every read ending before p freed; so the i-th read at p (i >= 1) is dropped
// iff B_p + i + 1 > maxcnt, where B_p counts the kept reads with pos < p and end >= p — k_p = min(n_p, max(1, maxcnt -
// B_p)) reads kept at p, in BAM order.  B_p is carried in a ring of kept-read ends.  ~5x faster than the per-read
// replay at 10,000x (the ring, the push list and the iterator walk per read); false: take the general replay.
bool capped_no_pairs(const Reads &R, const spp_params &p, int32_t tid, int64_t maxcnt, std::vector<uint8_t> &keep) {
    const size_t n = R.size();
    const int nt = std::max(1, std::min(p.n_threads, 64));
    std::atomic<bool> ok{true};
    std::vector<int64_t> spans((size_t)nt, 1);
    par_chunks(n, nt, [&](int t, size_t i0, size_t i1) {
        int64_t sp = 1;
        for (size_t r = i0; r < i1 && ok.load(std::memory_order_relaxed); r++) {
            bool bad = R.end[r] <= R.pos[r] || (r && R.pos[r] < R.pos[r - 1]);
            if (p.ignore_overlaps) {
                const uint16_t fl = R.flag[r];
                bad |= !(fl & F_MUNMAP) && (fl & F_PROPER) && !(R.mtid[r] >= 0 && R.mtid[r] != tid) &&
                       !(std::llabs(R.isize[r]) >= 2 * (int64_t)R.l_seq[r] && R.mpos[r] >= R.end[r]);
            }
            if (bad) ok = false;
            sp = std::max(sp, R.end[r] - R.pos[r]);
        }
        spans[(size_t)t] = sp;
    });
    if (!ok) return false;
    const int64_t max_span = *std::max_element(spans.begin(), spans.end());
    keep.assign(n, 0);
    size_t ring = 2;
    while ((int64_t)ring < max_span + 2) ring <<= 1;
    const size_t mask = ring - 1;
    std::vector<int64_t> ends(ring, 0);          // kept reads ending at e (slot e & mask), e >= the current position
    int64_t alive = 0, at = INT64_MIN;           // kept reads with end >= at
    for (size_t r0 = 0; r0 < n;) {
        const int64_t pos = R.pos[r0];
        size_t r1 = r0 + 1;
        while (r1 < n && R.pos[r1] == pos) r1++;
        if (alive > 0) {                          // free the reads ending in [at, pos)
            if (pos - at >= (int64_t)ring) {
                std::fill(ends.begin(), ends.end(), 0);
                alive = 0;
            } else {
                for (int64_t e = at; e < pos; e++) {
                    int64_t &c = ends[(size_t)e & mask];
                    alive -= c;
                    c = 0;
                }
            }
        }
        at = pos;
        const int64_t k = std::min<int64_t>((int64_t)(r1 - r0), std::max<int64_t>(1, maxcnt - alive));
        for (size_t r = r0; r < r0 + (size_t)k; r++) {
            keep[r] = 1;
            ends[(size_t)R.end[r] & mask]++;
        }
        alive += k;
        r0 = r1;
    }
    return true;
}

// Replay of bam_plp_push / bam_plp_next: which reads enter the buffer (maxcnt) and the overlap
// pairing.  Returns keep[r].
std::vector<uint8_t> simulate(Reads &R, const spp_params &p, int32_t tid, Tweaks &T) {
    const size_t n = R.size();
    T.col.clear();                             // (empty: no read tweaked; else one column per read, INT64_MAX: none)
    // Uncapped, every read spans >= 1 column and no overlap pairing can happen: every read is pushed
    // (sorted starts keep the pending position <= each read's start < its end) and nothing is tweaked
    if (p.max_depth <= 0) {
        std::atomic<bool> simple{true};
        par_chunks(n, std::max(1, std::min(p.n_threads, 64)), [&](int, size_t i0, size_t i1) {
            for (size_t r = i0; r < i1 && simple.load(std::memory_order_relaxed); r++)
                if (!(R.end[r] > R.pos[r] && !(p.ignore_overlaps && (R.flag[r] & F_PROPER)))) simple = false;
        });
        if (simple) return std::vector<uint8_t>(n, 1);
    }
    const int64_t maxcnt = p.max_depth > 0 ? p.max_depth : INT64_MAX;
    if (p.max_depth > 0) {
        std::vector<uint8_t> keep;
        if (capped_no_pairs(R, p, tid, maxcnt, keep)) return keep;
    }
    T.col.assign(n, INT64_MAX);
    std::vector<uint8_t> keep(n, 0);
    // live buffer: reads pushed and not yet freed.  Freed while scanning column c when end <= c.
    int64_t max_span = 0;
    for (size_t r = 0; r < n; r++) max_span = std::max(max_span, R.end[r] - R.pos[r]);
    EndQueue by_end(max_span);
    std::vector<uint8_t> freed(n, 0);
    size_t head = 0;                          // oldest pushed read not yet freed (list head)
    std::vector<size_t> pushed;               // kept reads in push order
    // bam_plp_init leaves iter->tid = iter->pos = 0: for contig 0 the depth check is live from the
    // first read; for a later contig the first push sees another tid and the iterator then jumps
    // to that read's position.
    int64_t it_pos = 0, max_pos = -1;
    bool started = tid == 0;
    // (keyed by the names in place: no string built per read — the std::string keys cost about half of this sweep at
    // 10,000x)
    OlapTable olap(p.ignore_overlaps ? (size_t)1 << 16 : 2);
    auto name = [&](size_t r) { return R.name_view(r); };
    auto name_key = [&](size_t r) -> uint64_t {
        if (R.hashed) return R.nhash[r];
        const std::string_view v = R.name_view(r);
        uint64_t h = 0xcbf29ce484222325ull;
        for (const char ch : v) h = (h ^ (uint8_t)ch) * 0x100000001b3ull;
        return h;
    };
    auto olap_find = [&](size_t r, uint64_t k) {
        if (R.hashed) return olap.find(k, [](size_t) { return true; });
        const std::string_view nm = name(r);
        return olap.find(k, [&](size_t a) { return name(a) == nm; });
    };
    auto olap_remove = [&](size_t r) {
        if (!p.ignore_overlaps || olap.empty()) return;
        const size_t i = olap_find(r, name_key(r));
        if (i != SIZE_MAX) olap.erase(i);
    };
    auto scan = [&](int64_t col) {            // free reads with end <= col (bam_plp_next)
        by_end.pop_upto(col, [&](size_t r) {
            freed[r] = 1;
            olap_remove(r);
        });
        while (head < pushed.size() && freed[pushed[head]]) head++;
    };
    auto advance = [&]() {                     // bam_plp_next loop while max_pos > pos
        while (max_pos > it_pos) {
            scan(it_pos);
            if (head < pushed.size()) {
                const int64_t hb = R.pos[pushed[head]];
                if (it_pos < hb) it_pos = hb;
                else ++it_pos;
            } else break;
        }
    };
    for (size_t r = 0; r < n; r++) {
        // bam_plp_push
        const int64_t cnt = (int64_t)by_end.size() + 1;      // mempool nodes: buffered + tail
        if (started && it_pos == R.pos[r] && cnt > maxcnt) { olap_remove(r); continue; }
        max_pos = R.pos[r];
        if (R.end[r] > it_pos || !started) {
            keep[r] = 1;
            pushed.push_back(r);
            by_end.emplace(R.end[r], r);
            if (p.ignore_overlaps) {            // overlap_push
                const uint16_t fl = R.flag[r];
                const bool cand = !(fl & F_MUNMAP) && (fl & F_PROPER) &&
                                  !(R.mtid[r] >= 0 && R.mtid[r] != tid) &&
                                  !(std::llabs(R.isize[r]) >= 2 * (int64_t)R.l_seq[r] && R.mpos[r] >= R.end[r]);
                if (cand) {
                    const uint64_t k = name_key(r);
                    const size_t itr = olap_find(r, k);
                    if (itr == SIZE_MAX) {
                        if (R.mpos[r] >= R.pos[r] || ((fl & F_PAIRED) && R.mpos[r] == -1)) olap.insert(k, r);
                    } else {
                        const size_t a = olap.at(itr);
                        // region pileups decode the reads within a read span of the region: a pair with
                        // an undecoded mate shares no aligned base with the region's reads
                        if (R.bases[a] && R.bases[r]) {
                            T.col[a] = it_pos;
                            if (T.defer) {
                                T.pairs.emplace_back(a, r);     // (the device applies it: spg_bam_accumulate)
                            } else {
                                T.orig.emplace(a, std::vector<uint8_t>(R.qual(a), R.qual(a) + R.l_seq[a]));
                                tweak_overlap(R, a, r);
                            }
                        }
                        olap.erase(itr);
                    }
                }
            }
        }
        if (!started) {                        // first read: the iterator jumps to its contig/pos
            started = true;
            if (head < pushed.size()) it_pos = R.pos[pushed[head]];
        }
        advance();
    }
    return keep;
}

}  // namespace

struct spp_plan {
    Reads R;
    std::vector<uint8_t> keep;
    Tweaks T;
    std::vector<size_t> kept;      // reads with entries in the batch's columns, in BAM order
    int64_t rlo = INT64_MIN, rhi = INT64_MAX;
    // records plan: the inflated BAM (R.raw) and the per-read index + CSR offsets handed to the GPU
    bool raw = false;
    HostBuf data, idx;
    size_t data_len = 0;           // inflated bytes in `data`
    spg_records view{};
    // device plan (spp_pileup_plan_fields): the reads live in HBM (spg_bam_open); `idx` holds the plan's arrays
    bool device = false;
    spg_bam_plan dview{};
    void clear() {
        R.clear(); keep.clear(); T.col.clear(); T.orig.clear(); T.pairs.clear(); T.defer = false; kept.clear();
        rlo = INT64_MIN; rhi = INT64_MAX;
        buf_put(data);
        buf_put(idx);
        raw = false;
        device = false;
        view = spg_records{};
        dview = spg_bam_plan{};
    }
};

// Plans are recycled (up to two kept): a 10,000x BAM's parsed-read arrays are ~150 MB, and fresh ones
// cost the parallel decoders page faults and grow-and-copy reallocations on every BAM.  A released
// plan is emptied on a helper thread, so the pipeline's next BAM does not wait for it (the arena's
// blocks go back to the block pool).
std::mutex &g_plan_mu = *new std::mutex;
std::vector<spp_plan *> &g_plan_pool = *new std::vector<spp_plan *>;

spp_plan *plan_get() {
    {
        std::lock_guard<std::mutex> lk(g_plan_mu);
        if (!g_plan_pool.empty()) {
            spp_plan *p = g_plan_pool.back();
            g_plan_pool.pop_back();
            return p;
        }
    }
    return new spp_plan();
}

void release_plan(spp_plan *p) {
    if (!p) return;
    auto recycle = [p] {
        p->clear();
        std::lock_guard<std::mutex> lk(g_plan_mu);
        if (g_plan_pool.size() < 2) g_plan_pool.push_back(p);
        else delete p;
    };
    try {
        std::thread(recycle).detach();
    } catch (...) {
        recycle();
    }
}

namespace {

// CSR offsets of the kept reads' columns (the batch's entry count is known after this).  Parallel over read
// chunks: the column range by reduction, the coverage difference array per thread when it is small (else one
// shared array, serially), the kept list by chunk counts.
void plan_csr(spp_plan &P, spp_batch *B, int threads) {
    const Reads &R = P.R;
    const std::vector<uint8_t> &keep = P.keep;
    const int64_t rlo = P.rlo, rhi = P.rhi;
    const size_t n = R.size();
    auto inreg = [&](size_t r) { return keep[r] && R.end[r] > R.pos[r] && R.end[r] > rlo && R.pos[r] < rhi; };
    const int nw = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), (n + 65535) / 65536));
    std::vector<int64_t> tlo((size_t)nw, INT64_MAX), thi((size_t)nw, INT64_MIN);
    std::vector<size_t> tcnt((size_t)nw + 1, 0);
    par_chunks(n, nw, [&](int t, size_t i0, size_t i1) {
        int64_t a = INT64_MAX, z = INT64_MIN;
        size_t k = 0;
        for (size_t r = i0; r < i1; r++)
            if (inreg(r)) { a = std::min(a, std::max(R.pos[r], rlo)); z = std::max(z, std::min(R.end[r], rhi)); k++; }
        tlo[(size_t)t] = a;
        thi[(size_t)t] = z;
        tcnt[(size_t)t + 1] = k;
    });
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (int t = 0; t < nw; t++) { lo = std::min(lo, tlo[(size_t)t]); hi = std::max(hi, thi[(size_t)t]); }
    for (int t = 0; t < nw; t++) tcnt[(size_t)t + 1] += tcnt[(size_t)t];
    if (lo == INT64_MAX) { lo = 0; hi = 0; }
    const int64_t C = hi - lo;
    B->pos_begin = lo;
    B->n_cols = C;
    const bool per_thread = nw > 1 && (uint64_t)(C + 1) * (uint64_t)nw <= ((uint64_t)1 << 24);
    std::vector<std::vector<int64_t>> tdiff(per_thread ? (size_t)nw : 1);
    P.kept.resize(tcnt[(size_t)nw]);
    auto scatter = [&](int t, size_t i0, size_t i1, std::vector<int64_t> &diff) {
        size_t k = tcnt[(size_t)t];
        for (size_t r = i0; r < i1; r++)
            if (inreg(r)) {
                diff[(size_t)(std::max(R.pos[r], lo) - lo)]++;
                diff[(size_t)(std::min(R.end[r], hi) - lo)]--;
                P.kept[k++] = r;
            }
    };
    if (per_thread) {
        par_chunks(n, nw, [&](int t, size_t i0, size_t i1) {
            tdiff[(size_t)t].assign((size_t)C + 1, 0);
            scatter(t, i0, i1, tdiff[(size_t)t]);
        });
    } else {
        tdiff[0].assign((size_t)C + 1, 0);
        for (int t = 0; t < nw; t++) scatter(t, n * (size_t)t / (size_t)nw, n * (size_t)(t + 1) / (size_t)nw, tdiff[0]);
    }
    B->off.assign((size_t)C + 1, 0);
    int64_t run = 0;
    for (int64_t c = 0; c < C; c++) {
        for (auto &d : tdiff) run += d[(size_t)c];
        B->off[(size_t)c + 1] = B->off[(size_t)c] + (uint64_t)run;
    }
    B->n_entries = B->off[(size_t)C];
}

// base_code / qual of every entry into code / qual (>= n_entries + 16 bytes each)
void fill_csr(const spp_plan &P, spp_batch *B, uint8_t *code, uint8_t *qual, int threads) {
    const Reads &R = P.R;
    const Tweaks &T = P.T;
    const std::vector<size_t> &kept = P.kept;
    const int64_t lo = B->pos_begin, C = B->n_cols;
    const uint64_t E = B->n_entries;
    B->code = code;
    B->qual = qual;
    memset(B->code + E, 0xFF, 16);
    memset(B->qual + E, 0, 16);
    // Column-range parallel fill: a thread owns columns [c0, c1) and walks the reads overlapping
    // them in read order, so each column's entries keep htslib's order.
    const int nt = std::max(1, std::min(threads, 64));
    auto work = [&](int t) {
        const int64_t c0 = C * t / nt, c1 = C * (t + 1) / nt;
        if (c0 >= c1) return;
        std::vector<uint64_t> cur(B->off.begin() + c0, B->off.begin() + c1);
        // reads are sorted by pos: those starting before lo + c1 can overlap
        const auto last = std::lower_bound(kept.begin(), kept.end(), lo + c1,
                                           [&](size_t r, int64_t v) { return R.pos[r] < v; });
        for (auto itr = kept.begin(); itr != last; ++itr) {
            const size_t r = *itr;
            if (R.end[r] <= lo + c0) continue;
            int64_t x = R.pos[r];
            uint32_t y = 0;
            const uint32_t *cg = R.cigar.data() + R.cig_off[r];
            const uint8_t *sq = R.seq(r), *ql = R.qual(r);
            const uint32_t ls = R.l_seq[r];
            const int64_t tcol = T.col.empty() ? INT64_MAX : T.col[r];
            const uint8_t *ql0 = tcol == INT64_MAX ? ql : T.orig.at(r).data();
            for (uint32_t i = 0; i < R.n_cig[r] && x < lo + c1; i++) {
                const uint32_t op = cg[i] & 0xF, l = cg[i] >> 4;
                if (consumes_ref(op)) {
                    const int64_t a = std::max<int64_t>(x, lo + c0), e = std::min<int64_t>(x + l, lo + c1);
                    for (int64_t col = a; col < e; col++) {
                        const size_t k = (size_t)(col - lo - c0);
                        uint8_t code, q;
                        if (op == C_D || op == C_N) {            // resolve_cigar2: qpos = next query base
                            code = op == C_D ? 16 : 17;
                            q = y < ls ? (col < tcol ? ql0[y] : ql[y]) : 0;
                        } else {
                            const uint32_t qp = y + (uint32_t)(col - x);
                            code = qp < ls ? sq[qp] : 15;
                            q = qp < ls ? ql[qp] : 0;
                        }
                        B->code[cur[k]] = code;
                        B->qual[cur[k]] = q;
                        cur[k]++;
                    }
                    x += l;
                }
                if (consumes_query(op)) y += l;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work, t);
    work(0);
    for (auto &t : pool) t.join();
}

// The records plan's GPU view: per kept read its record offset, span and tweak index; the tweaked reads'
// original qualities; the CSR offsets — one host buffer (pinned under the allocator hook).
void plan_records(spp_plan &P, spp_batch *B, int threads) {
    const Reads &R = P.R;
    const std::vector<size_t> &kept = P.kept;
    const size_t n = kept.size();
    if (n >= ((size_t)1 << 31)) throw std::runtime_error("more than 2^31 reads in one batch");
    std::vector<int32_t> tw;            // per kept read: tweak index (only when some read was tweaked)
    std::vector<size_t> tw_read;
    uint64_t orig_bytes = 0;
    if (!P.T.orig.empty()) {
        tw.assign(n, -1);
        for (size_t i = 0; i < n; i++) {
            const size_t r = kept[i];
            if (P.T.col[r] != INT64_MAX) {
                tw[i] = (int32_t)tw_read.size();
                tw_read.push_back(r);
                orig_bytes += R.l_seq[r];
            }
        }
    }
    const size_t nt = tw_read.size(), C = (size_t)B->n_cols;
    auto al = [](size_t x) { return (x + 63) & ~(size_t)63; };
    const size_t o_off = 0, o_rec = al(o_off + 8 * (C + 1)), o_pos = al(o_rec + 8 * n), o_end = al(o_pos + 4 * n),
                 o_tw = al(o_end + 4 * n), o_tcol = al(o_tw + 4 * n), o_tq = al(o_tcol + 8 * nt),
                 o_orig = al(o_tq + 8 * nt), bytes = al(o_orig + orig_bytes) + 64;
    P.idx = buf_get(bytes);
    uint8_t *m = P.idx.p;
    uint64_t *off = (uint64_t *)(m + o_off), *rec = (uint64_t *)(m + o_rec), *tq = (uint64_t *)(m + o_tq);
    int32_t *rpos = (int32_t *)(m + o_pos), *rend = (int32_t *)(m + o_end), *twi = (int32_t *)(m + o_tw);
    int64_t *tcol = (int64_t *)(m + o_tcol);
    uint8_t *orig = m + o_orig;
    memcpy(off, B->off.data(), 8 * (C + 1));
    const int nw = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), (n + 65535) / 65536));
    std::vector<int64_t> spans((size_t)nw, 0);
    par_chunks(n, nw, [&](int t, size_t i0, size_t i1) {
        int64_t sp = 0;
        for (size_t i = i0; i < i1; i++) {
            const size_t r = kept[i];
            rec[i] = R.rec[r];
            rpos[i] = (int32_t)R.pos[r];
            rend[i] = (int32_t)R.end[r];
            twi[i] = tw.empty() ? -1 : tw[i];
            sp = std::max(sp, R.end[r] - R.pos[r]);
        }
        spans[(size_t)t] = sp;
    });
    int64_t span = 0;
    for (int64_t v : spans) span = std::max(span, v);
    uint64_t oq = 0;
    for (size_t j = 0; j < nt; j++) {
        const size_t r = tw_read[j];
        tcol[j] = P.T.col[r];
        tq[j] = oq;
        const std::vector<uint8_t> &o = P.T.orig.at(r);
        memcpy(orig + oq, o.data(), o.size());
        oq += o.size();
    }
    spg_records &v = P.view;
    v = spg_records{};
    v.pos_begin = B->pos_begin;
    v.n_cols = B->n_cols;
    v.n_entries = B->n_entries;
    v.offsets = off;
    v.data = P.data.p;
    v.data_bytes = P.data_len;
    v.n_reads = (int64_t)n;
    v.rec = rec;
    v.rpos = rpos;
    v.rend = rend;
    v.tweak = twi;
    v.n_tweaks = (int64_t)nt;
    v.tweak_col = tcol;
    v.tweak_qual = tq;
    v.orig_qual = orig;
    v.orig_bytes = orig_bytes;
    v.max_span = span;
}


// The device plan's arrays (spg_bam_plan): kept reads (u32 read indices), CSR offsets, the overlapping mate pairs with
// their tweak columns and the offsets of the first mates' saved qualities — one host buffer (pinned under the hook).
void plan_device(spp_plan &P, spp_batch *B) {
    const Reads &R = P.R;
    const std::vector<size_t> &kept = P.kept;
    const size_t n = kept.size(), np = P.T.pairs.size(), C = (size_t)B->n_cols;
    auto al = [](size_t x) { return (x + 63) & ~(size_t)63; };
    const size_t o_off = 0, o_kept = al(8 * (C + 1)), o_pa = al(o_kept + 4 * n), o_pb = al(o_pa + 4 * np),
                 o_col = al(o_pb + 4 * np), o_oq = al(o_col + 8 * np), bytes = al(o_oq + 8 * np) + 64;
    P.idx = buf_get(bytes);
    uint8_t *m = P.idx.p;
    uint64_t *off = (uint64_t *)(m + o_off), *oq = (uint64_t *)(m + o_oq);
    uint32_t *kp = (uint32_t *)(m + o_kept), *pa = (uint32_t *)(m + o_pa), *pb = (uint32_t *)(m + o_pb);
    int64_t *col = (int64_t *)(m + o_col);
    memcpy(off, B->off.data(), 8 * (C + 1));
    const int nw = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, B->threads), (n + 65535) / 65536));
    std::vector<int64_t> spans((size_t)nw, 0);
    par_chunks(n, nw, [&](int t, size_t i0, size_t i1) {
        int64_t sp = 0;
        for (size_t i = i0; i < i1; i++) {
            kp[i] = (uint32_t)kept[i];
            sp = std::max(sp, R.end[kept[i]] - R.pos[kept[i]]);
        }
        spans[(size_t)t] = sp;
    });
    int64_t span = 0;
    for (int64_t v : spans) span = std::max(span, v);
    uint64_t o = 0;
    for (size_t j = 0; j < np; j++) {
        const size_t a = P.T.pairs[j].first, b = P.T.pairs[j].second;
        pa[j] = (uint32_t)a;
        pb[j] = (uint32_t)b;
        col[j] = P.T.col[a];
        oq[j] = o;
        o += R.l_seq[a];
    }
    spg_bam_plan &v = P.dview;
    v = spg_bam_plan{};
    v.pos_begin = B->pos_begin;
    v.n_cols = B->n_cols;
    v.n_entries = B->n_entries;
    v.offsets = off;
    v.n_kept = (int64_t)n;
    v.kept = kp;
    v.n_pairs = (int64_t)np;
    v.pair_a = pa;
    v.pair_b = pb;
    v.pair_col = col;
    v.pair_orig = oq;
    v.orig_bytes = o;
    v.max_span = span;
}

// ---------------------------------------------------------------------------------------------
// Read simulator -> BGZF BAM
// ---------------------------------------------------------------------------------------------
class BgzfWriter {
  public:
    BgzfWriter(const std::string &path, int threads, int level) : threads_(std::max(1, threads)), level_(level) {
        f_ = fopen(path.c_str(), "wb");
        if (!f_) throw std::runtime_error("cannot create " + path);
    }
    ~BgzfWriter() {
        if (f_) fclose(f_);
    }
    void write(const void *p, size_t n) {
        const uint8_t *b = (const uint8_t *)p;
        buf_.insert(buf_.end(), b, b + n);
        if (buf_.size() >= kFlush) flush(false);
    }
    void close() {
        flush(true);
        static const uint8_t eof[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        fwrite(eof, 1, 28, f_);
        fclose(f_);
        f_ = nullptr;
    }

  private:
    static constexpr size_t kBlock = 65280, kFlush = 64u << 20;
    void flush(bool all) {
        const size_t nb = all ? (buf_.size() + kBlock - 1) / kBlock : buf_.size() / kBlock;
        if (!nb) return;
        std::vector<std::vector<uint8_t>> out(nb);
        std::atomic<size_t> next{0};
        std::atomic<bool> bad{false};
        auto work = [&]() {
            for (size_t i; (i = next++) < nb;) {
                const size_t off = i * kBlock, len = std::min(kBlock, buf_.size() - off);
                z_stream zs;
                memset(&zs, 0, sizeof(zs));
                if (deflateInit2(&zs, level_, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) { bad = true; return; }
                std::vector<uint8_t> &o = out[i];
                o.resize(18 + deflateBound(&zs, len) + 8);
                zs.next_in = buf_.data() + off;
                zs.avail_in = (uInt)len;
                zs.next_out = o.data() + 18;
                zs.avail_out = (uInt)(o.size() - 26);
                if (deflate(&zs, Z_FINISH) != Z_STREAM_END) bad = true;
                const size_t clen = zs.total_out;
                deflateEnd(&zs);
                const size_t bsize = clen + 26;
                const uint8_t hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0,
                                         (uint8_t)((bsize - 1) & 0xFF), (uint8_t)((bsize - 1) >> 8)};
                memcpy(o.data(), hdr, 18);
                const uint32_t crc = (uint32_t)crc32(0, buf_.data() + off, (uInt)len), isz = (uint32_t)len;
                memcpy(o.data() + 18 + clen, &crc, 4);
                memcpy(o.data() + 22 + clen, &isz, 4);
                o.resize(bsize);
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < threads_; t++) pool.emplace_back(work);
        work();
        for (auto &t : pool) t.join();
        if (bad) throw std::runtime_error("BGZF deflate failed");
        for (auto &o : out) fwrite(o.data(), 1, o.size(), f_);
        const size_t used = std::min(buf_.size(), nb * kBlock);
        buf_.erase(buf_.begin(), buf_.begin() + (ptrdiff_t)used);
    }
    FILE *f_ = nullptr;
    int threads_, level_;
    std::vector<uint8_t> buf_;
};

}  // namespace

extern "C" {

const char *spp_last_error(void) { return g_err.c_str(); }

const char *spp_host_inflater(void) { return Inflater::api().dec ? "libdeflate" : "zlib"; }

void spp_default_params(spp_params *p) {
    memset(p, 0, sizeof(*p));
    p->stepper = SPP_STEPPER_ALL;
    p->min_mapping_quality = 0;
    p->max_depth = 8000;
    p->ignore_overlaps = 1;
    p->flag_filter = F_UNMAP | F_SECONDARY | F_QCFAIL | F_DUP;
    p->n_threads = 1;
    p->inflate_device = -1;
    p->inflate_min_members = 0;
}

int spp_open(const char *path, spp_file **out) {
    if (!path || !out) return fail("spp_open: null argument");
    *out = nullptr;
    try {
        auto *f = new spp_file();
        f->path = path;
        f->bam = is_bgzf(path);
        if (f->bam) {
            // the header only: a small inflate window (the default 16 MiB one inflated ~40 MB of reads
            // just to read it, 0.2-0.5 s per BAM)
            BamStream s(path, 1, 256u << 10);
            bam_header(s, f);
        } else {
            for_lines(path, [&](const std::string &line) {
                if (line.empty() || line[0] != '@') return false;
                sam_header_line(f, line);
                return true;
            });
        }
        *out = f;
        return 0;
    } catch (const std::exception &e) {
        return fail(std::string("spp_open: ") + e.what());
    }
}

int spp_close(spp_file *f) {
    delete f;
    return 0;
}

int spp_n_targets(spp_file *f, int32_t *n) {
    if (!f || !n) return fail("spp_n_targets: null argument");
    *n = (int32_t)f->targets.size();
    return 0;
}

int spp_target(spp_file *f, int32_t tid, const char **name, int64_t *length) {
    if (!f) return fail("spp_target: null file");
    if (tid < 0 || (size_t)tid >= f->targets.size()) return fail("spp_target: tid out of range");
    if (name) *name = f->targets[(size_t)tid].name.c_str();
    if (length) *length = f->targets[(size_t)tid].len;
    return 0;
}

int spp_target_id(spp_file *f, const char *name, int32_t *tid) {
    if (!f || !name || !tid) return fail("spp_target_id: null argument");
    auto it = f->tid_of.find(name);
    if (it == f->tid_of.end()) return fail(std::string("invalid contig `") + name + "`");
    *tid = it->second;
    return 0;
}

static int plan_impl(spp_file *f, int32_t tid, const spp_params *p, int64_t lo, int64_t hi, spp_batch **out,
                     bool raw = false) {
    if (!f || !p || !out) return fail("spp_pileup: null argument");
    if (raw && !f->bam) return fail("spp_pileup_plan_records: the device-decode plan needs a BAM (this is SAM text)");
    if (tid < 0 || (size_t)tid >= f->targets.size()) return fail("spp_pileup: tid out of range");
    if (lo >= hi) return fail("spp_pileup_region: empty region");
    *out = nullptr;
    spp_plan *P = nullptr;
    try {
        const bool region = lo != INT64_MIN || hi != INT64_MAX;
        // region: bases of reads within a read span of [lo, hi) (mates that can overlap a region read);
        // the span bound is checked against the longest read and the pass redone if it was too short
        int64_t pad = 16384;
        for (;;) {
            // SPP_TIMING=1: phase times on stderr (read / depth-cap simulation / offsets)
            static const bool timing = getenv("SPP_TIMING") != nullptr;
            auto now = [] { return std::chrono::steady_clock::now(); };
            const auto t0 = now();
            P = plan_get();
            Reads &R = P->R;
            if (region) { R.dlo = lo == INT64_MIN ? lo : lo - pad; R.dhi = hi == INT64_MAX ? hi : hi + pad; }
            if (raw) {
                P->raw = true;
                P->data_len = read_bam_raw(f, tid, *p, R, P->data);
            } else if (f->bam) {
                read_bam(f, tid, *p, R);
            } else {
                read_sam(f, tid, *p, R);
            }
            if (region && R.max_span > pad) {
                pad = 2 * R.max_span;
                release_plan(P);
                P = nullptr;
                continue;
            }
            const auto t1 = now();
            P->keep = simulate(R, *p, tid, P->T);      // every read: exact depth cap
            const auto t2 = now();
            auto *B = new spp_batch();
            int64_t used = 0;
            for (uint8_t k : P->keep) used += k;
            B->n_used = used;
            B->n_dropped = (int64_t)R.size() - used;
            B->threads = std::max(1, p->n_threads);
            P->rlo = lo;
            P->rhi = hi;
            plan_csr(*P, B, B->threads);
            const auto t3 = now();
            if (raw) plan_records(*P, B, B->threads);
            B->plan = P;
            P = nullptr;
            if (timing) {
                const auto t4 = now();
                auto ms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
                fprintf(stderr, "[spp timing] read %.1f ms, simulate %.1f ms, offsets %.1f ms, records index %.1f ms "
                        "(%zu reads, %d threads)\n", ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4),
                        (size_t)B->plan->R.size(), p->n_threads);
            }
            *out = B;
            return 0;
        }
    } catch (const std::exception &e) {
        release_plan(P);
        return fail(std::string("spp_pileup: ") + e.what());
    }
}

int spp_batch_fill(spp_batch *b, uint8_t *base_code, uint8_t *qual) {
    if (!b) return fail("spp_batch_fill: null batch");
    if (!b->plan) return fail("spp_batch_fill: the batch is already filled");
    if (b->plan->raw) return fail("spp_batch_fill: a records plan is filled on the GPU (spg_accumulate_records)");
    if (b->plan->device) return fail("spp_batch_fill: a device plan is filled on the GPU (spg_bam_accumulate)");
    if ((base_code == nullptr) != (qual == nullptr)) return fail("spp_batch_fill: give both buffers or neither");
    try {
        static const bool timing = getenv("SPP_TIMING") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        const uint64_t E = b->n_entries;
        if (!base_code) {
            base_code = (uint8_t *)malloc(E + 16);
            qual = (uint8_t *)malloc(E + 16);
            if (!base_code || !qual) {
                free(base_code);
                free(qual);
                return fail("spp_batch_fill: out of host memory for the pileup");
            }
            b->owns = true;
        } else {
            b->owns = false;
        }
        fill_csr(*b->plan, b, base_code, qual, b->threads);
        release_plan(b->plan);       // helper thread
        b->plan = nullptr;
        if (timing)
            fprintf(stderr, "[spp timing] fill %.1f ms (%s buffers)\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                    b->owns ? "own" : "caller");
        return 0;
    } catch (const std::exception &e) {
        return fail(std::string("spp_batch_fill: ") + e.what());
    }
}

int spp_pileup_plan(spp_file *f, int32_t tid, int64_t lo, int64_t hi, const spp_params *p, spp_batch **out) {
    return plan_impl(f, tid, p, lo, hi, out);
}

int spp_pileup_plan_records(spp_file *f, int32_t tid, int64_t lo, int64_t hi, const spp_params *p, spp_batch **out) {
    return plan_impl(f, tid, p, lo, hi, out, true);
}

int spp_batch_records(spp_batch *b, spg_records *out) {
    if (!b || !out) return fail("spp_batch_records: null argument");
    if (!b->plan || !b->plan->raw) return fail("spp_batch_records: not a records plan (spp_pileup_plan_records)");
    *out = b->plan->view;
    return 0;
}

struct spp_bam_map {
    HostBuf comp;                                  // the file's bytes (pinned under the allocator hook)
    std::vector<spg_bgzf_member> mem;
};

int spp_bam_map_open(spp_file *f, int n_threads, spp_bam_map **out, spp_bam_map_info *info) {
    if (!f || !out || !info) return fail("spp_bam_map_open: null argument");
    if (!f->bam) return fail("spp_bam_map_open: not a BAM (BGZF) file");
    *out = nullptr;
    spp_bam_map *h = nullptr;
    try {
        const int nt = std::max(1, std::min(n_threads, 64));
        // the file read straight into the (pinned) buffer by every thread (pread: no mapping, no page-table set-up and
        // tear-down; the mapped form cost 10-11 ms per 10,000x BAM, r05e), then its members walked there
        const int fd = open(f->path.c_str(), O_RDONLY);
        if (fd < 0) throw std::runtime_error("cannot open " + f->path);
        struct stat st;
        if (fstat(fd, &st) != 0) { close(fd); throw std::runtime_error("cannot stat " + f->path); }
        const size_t fsz = (size_t)st.st_size;
        h = new spp_bam_map();
        try {
            h->comp = buf_get(fsz + 64);
        } catch (...) {
            close(fd);
            throw;
        }
        std::atomic<bool> rd_ok{true};
        par_tasks((fsz + ((size_t)1 << 20) - 1) >> 20, nt, [&](size_t i) {   // (1 MiB blocks, taken in turn)
            size_t a = i << 20;
            const size_t e = std::min(fsz, a + ((size_t)1 << 20));
            while (a < e && rd_ok) {
                const ssize_t r = pread(fd, h->comp.p + a, e - a, (off_t)a);
                if (r <= 0) { rd_ok = false; break; }
                a += (size_t)r;
            }
        });
        close(fd);
        if (!rd_ok) throw std::runtime_error("cannot read " + f->path);
        memset(h->comp.p + fsz, 0, 64);
        BamMap M;
        map_bam(f->path, nt, M, h->comp.p, fsz);
        int32_t n_ref = 0;
        const uint64_t body = header_end(M, &n_ref);
        h->mem.resize(M.blks.size());
        for (size_t i = 0; i < M.blks.size(); i++)
            h->mem[i] = spg_bgzf_member{M.blks[i].off, (uint32_t)M.blks[i].clen, (uint32_t)M.blks[i].ulen, M.uoff[i]};
        *info = spp_bam_map_info{};
        info->comp = h->comp.p;
        info->comp_bytes = M.fsz;
        info->members = h->mem.data();
        info->n_members = (int64_t)h->mem.size();
        info->inflated_bytes = M.total;
        info->body = body;
        info->n_ref = n_ref;
        *out = h;
        return 0;
    } catch (const std::exception &e) {
        if (h) { buf_put(h->comp); delete h; }
        return fail(std::string("spp_bam_map_open: ") + e.what());
    }
}

int spp_bam_map_close(spp_bam_map *h) {
    if (!h) return 0;
    buf_put(h->comp);
    delete h;
    return 0;
}

int spp_pileup_plan_fields(spp_file *f, int32_t tid, const spp_read_fields *F, const spp_params *p, spp_batch **out) {
    if (!f || !F || !p || !out) return fail("spp_pileup_plan_fields: null argument");
    if (tid < 0 || (size_t)tid >= f->targets.size()) return fail("spp_pileup_plan_fields: tid out of range");
    if (F->n < 0 || (F->n && (!F->pos || !F->end || !F->mtid || !F->mpos || !F->isize || !F->flag || !F->l_seq ||
                              !F->name_hash)))
        return fail("spp_pileup_plan_fields: null field array");
    *out = nullptr;
    spp_plan *P = nullptr;
    try {
        static const bool timing = getenv("SPP_TIMING") != nullptr;
        auto now = [] { return std::chrono::steady_clock::now(); };
        const auto t0 = now();
        P = plan_get();
        Reads &R = P->R;
        const size_t n = (size_t)F->n;
        static uint8_t present = 0;               // (bases stay in HBM: a non-null mark that the read is decoded)
        R.pos.resize(n); R.end.resize(n); R.mpos.resize(n); R.isize.resize(n); R.mtid.resize(n); R.flag.resize(n);
        R.l_seq.resize(n); R.nhash.resize(n); R.bases.resize(n);
        const int nt = std::max(1, std::min(p->n_threads, 64));
        std::vector<int64_t> spans((size_t)nt, 0);
        par_chunks(n, nt, [&](int t, size_t i0, size_t i1) {
            int64_t sp = 0;
            for (size_t i = i0; i < i1; i++) {
                R.pos[i] = F->pos[i];
                R.end[i] = F->end[i];
                R.mpos[i] = F->mpos[i];
                R.isize[i] = F->isize[i];
                R.mtid[i] = F->mtid[i];
                R.flag[i] = F->flag[i];
                R.l_seq[i] = F->l_seq[i];
                R.nhash[i] = F->name_hash[i];
                R.bases[i] = &present;
                sp = std::max(sp, R.end[i] - R.pos[i]);
            }
            spans[(size_t)t] = sp;
        });
        for (int64_t v : spans) R.max_span = std::max(R.max_span, v);
        R.hashed = true;
        P->device = true;
        P->T.defer = true;
        const auto t1 = now();
        P->keep = simulate(R, *p, tid, P->T);
        const auto t2 = now();
        auto *B = new spp_batch();
        int64_t used = 0;
        for (uint8_t k : P->keep) used += k;
        B->n_used = used;
        B->n_dropped = (int64_t)n - used;
        B->threads = nt;
        plan_csr(*P, B, B->threads);
        const auto t3 = now();
        plan_device(*P, B);
        B->plan = P;
        P = nullptr;
        if (timing) {
            auto ms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
            fprintf(stderr, "[spp timing] plan_fields: fields %.1f ms, simulate %.1f ms, offsets %.1f ms, device plan %.1f ms "
                    "(%zu reads, %zu pairs)\n", ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, now()), n,
                    B->plan->T.pairs.size());
        }
        *out = B;
        return 0;
    } catch (const std::exception &e) {
        release_plan(P);
        return fail(std::string("spp_pileup_plan_fields: ") + e.what());
    }
}

int spp_batch_device_plan(spp_batch *b, spg_bam_plan *out) {
    if (!b || !out) return fail("spp_batch_device_plan: null argument");
    if (!b->plan || !b->plan->device) return fail("spp_batch_device_plan: not a device plan (spp_pileup_plan_fields)");
    *out = b->plan->dview;
    return 0;
}

int spp_set_inflater(spp_inflate_fn fn, int device) {
    (void)device;
    g_inflate = fn;
    return 0;
}

int spp_set_host_allocator(spp_alloc_fn alloc, spp_free_fn release) {
    if ((alloc == nullptr) != (release == nullptr)) return fail("spp_set_host_allocator: give both or neither");
    std::lock_guard<std::mutex> lk(g_buf_mu);
    for (auto &b : g_bufs) b.release();     // pooled buffers of the previous allocator
    g_bufs.clear();
    g_alloc = alloc;
    g_free = release;
    return 0;
}

static int pileup_impl(spp_file *f, int32_t tid, const spp_params *p, int64_t lo, int64_t hi, spp_batch **out) {
    if (int rc = plan_impl(f, tid, p, lo, hi, out)) return rc;
    if (int rc = spp_batch_fill(*out, nullptr, nullptr)) {
        delete *out;
        *out = nullptr;
        return rc;
    }
    return 0;
}

int spp_pileup(spp_file *f, int32_t tid, const spp_params *p, spp_batch **out) {
    return pileup_impl(f, tid, p, INT64_MIN, INT64_MAX, out);
}

int spp_pileup_region(spp_file *f, int32_t tid, int64_t lo, int64_t hi, const spp_params *p, spp_batch **out) {
    return pileup_impl(f, tid, p, lo, hi, out);
}

int spp_batch_info(spp_batch *b, int64_t *pos_begin, int64_t *n_cols, uint64_t *n_entries, int64_t *n_reads_used,
                   int64_t *n_reads_dropped) {
    if (!b) return fail("spp_batch_info: null batch");
    if (pos_begin) *pos_begin = b->pos_begin;
    if (n_cols) *n_cols = b->n_cols;
    if (n_entries) *n_entries = b->n_entries;
    if (n_reads_used) *n_reads_used = b->n_used;
    if (n_reads_dropped) *n_reads_dropped = b->n_dropped;
    return 0;
}

int spp_batch_arrays(spp_batch *b, const uint64_t **offsets, const uint8_t **base_code, const uint8_t **qual) {
    if (!b) return fail("spp_batch_arrays: null batch");
    if (offsets) *offsets = b->off.data();
    if (base_code) *base_code = b->code;
    if (qual) *qual = b->qual;
    return 0;
}

int spp_batch_free(spp_batch *b) {
    delete b;
    return 0;
}

}  // extern "C"

namespace {

int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

// One chunk of reads (consecutive in sorted order) -> BAM records; its own RNG stream, so the
// output does not depend on the thread count.
void sim_chunk(const spp_sim_params &p, const char *ref, int64_t L, const std::vector<int64_t> &starts, size_t r0,
               size_t r1, uint64_t seed, std::vector<uint8_t> &out) {
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::normal_distribution<double> Nq(p.q_mean, p.q_sd);
    static const char ACGT[4] = {'A', 'C', 'G', 'T'};
    auto idx_of = [](char c) { c = (char)toupper(c); return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1; };
    const int R = p.read_len;
    std::vector<char> seq((size_t)R + 8);
    std::vector<uint8_t> qual((size_t)R + 8);
    for (size_t r = r0; r < r1; r++) {
        int64_t pos = starts[r];
        const double u = U(rng);
        int kind = u < p.del_frac ? 1 : (u < p.del_frac + p.ins_frac ? 2 : 0);
        if (R < 74) kind = 0;
        if (kind == 1 && pos + R + 2 > L) kind = 0;
        uint32_t cig[3];
        int ncig = 1;
        if (kind == 0) cig[0] = (uint32_t)R << 4 | C_M;
        else if (kind == 1) { cig[0] = 70u << 4 | C_M; cig[1] = 2u << 4 | C_D; cig[2] = (uint32_t)(R - 70) << 4 | C_M; ncig = 3; }
        else { cig[0] = 70u << 4 | C_M; cig[1] = 2u << 4 | C_I; cig[2] = (uint32_t)(R - 72) << 4 | C_M; ncig = 3; }
        // query bases
        int y = 0;
        int64_t x = pos;
        for (int k = 0; k < ncig; k++) {
            const uint32_t op = cig[k] & 0xF, l = cig[k] >> 4;
            for (uint32_t j = 0; j < l; j++) {
                if (op == C_D) { x++; continue; }
                char b;
                if (op == C_I) b = ACGT[rng() & 3];
                else {
                    b = (char)toupper(ref[x]);
                    if (p.snv_every > 0 && x % p.snv_every == p.snv_every / 2) {
                        static const double afs[4] = {1.0, 0.5, 0.2, 0.05};
                        const int bi = idx_of(b);
                        if (bi >= 0 && U(rng) < afs[(x / p.snv_every) % 4]) b = ACGT[(bi + 1 + (int)(x % 3)) % 4];
                    }
                    x++;
                }
                int q = (int)std::lround(Nq(rng));
                q = std::min(std::max(q, p.q_min), p.q_max);
                const int bi = idx_of(b);
                if (bi >= 0 && U(rng) < std::pow(10.0, -q / 10.0)) b = ACGT[(bi + 1 + (int)(rng() % 3)) % 4];
                if (U(rng) < p.n_rate) b = 'N';
                seq[(size_t)y] = b;
                qual[(size_t)y] = (uint8_t)q;
                y++;
            }
        }
        const int64_t end = x;
        char name[32];
        const int ln = snprintf(name, sizeof(name), "r%zu", r) + 1;
        const int lseq = y;
        const uint32_t bs = 32 + (uint32_t)ln + 4u * (uint32_t)ncig + (uint32_t)((lseq + 1) / 2) + (uint32_t)lseq;
        const size_t o = out.size();
        out.resize(o + 4 + bs);
        uint8_t *b = out.data() + o;
        auto w32 = [&](size_t at, uint32_t v) { memcpy(b + at, &v, 4); };
        auto w16 = [&](size_t at, uint16_t v) { memcpy(b + at, &v, 2); };
        w32(0, bs);
        w32(4, 0);                                     // refID
        w32(8, (uint32_t)pos);
        b[12] = (uint8_t)ln;
        b[13] = 60;                                    // MAPQ
        w16(14, (uint16_t)reg2bin(pos, std::max(end, pos + 1)));
        w16(16, (uint16_t)ncig);
        w16(18, 0);                                    // flag
        w32(20, (uint32_t)lseq);
        w32(24, 0xFFFFFFFFu);                          // next refID
        w32(28, 0xFFFFFFFFu);                          // next pos
        w32(32, 0);                                    // tlen
        memcpy(b + 36, name, (size_t)ln);
        size_t at = 36 + (size_t)ln;
        for (int k = 0; k < ncig; k++, at += 4) w32(at, cig[k]);
        for (int i = 0; i < lseq; i += 2) {
            const uint8_t hi = NT16.t[(uint8_t)seq[(size_t)i]], lo = i + 1 < lseq ? NT16.t[(uint8_t)seq[(size_t)i + 1]] : 0;
            b[at++] = (uint8_t)(hi << 4 | lo);
        }
        memcpy(b + at, qual.data(), (size_t)lseq);
    }
}

}  // namespace

extern "C" {

void spp_default_sim_params(spp_sim_params *p) {
    memset(p, 0, sizeof(*p));
    p->depth = 1000.0;
    p->read_len = 150;
    p->snv_every = 997;
    p->q_mean = 33.0;
    p->q_sd = 6.0;
    p->q_min = 2;
    p->q_max = 41;
    p->del_frac = 0.01;
    p->ins_frac = 0.01;
    p->n_rate = 1e-4;
    p->seed = 2;
    p->n_threads = 8;
    p->level = 1;
}

int spp_simulate_bam(const char *path, const char *contig, const char *ref_seq, int64_t ref_len,
                     const spp_sim_params *p, int64_t *n_reads_out) {
    if (!path || !contig || !ref_seq || !p) return fail("spp_simulate_bam: null argument");
    if (ref_len < p->read_len + 4 || p->read_len < 1) return fail("spp_simulate_bam: reference shorter than a read");
    try {
        const int64_t L = ref_len;
        const int64_t n = (int64_t)std::llround(p->depth * (double)L / p->read_len);
        std::vector<int64_t> starts((size_t)n);
        {
            std::mt19937_64 rng(p->seed);
            std::uniform_int_distribution<int64_t> S(0, L - p->read_len);
            for (auto &s : starts) s = S(rng);
            std::sort(starts.begin(), starts.end());
        }
        BgzfWriter w(path, p->n_threads, p->level);
        const std::string text = std::string("@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:") + contig + "\tLN:" +
                                 std::to_string(L) + "\n";
        std::vector<uint8_t> hdr;
        auto put32 = [&](uint32_t v) { const uint8_t *q = (const uint8_t *)&v; hdr.insert(hdr.end(), q, q + 4); };
        hdr.insert(hdr.end(), {'B', 'A', 'M', 1});
        put32((uint32_t)text.size());
        hdr.insert(hdr.end(), text.begin(), text.end());
        put32(1);
        put32((uint32_t)strlen(contig) + 1);
        hdr.insert(hdr.end(), contig, contig + strlen(contig) + 1);
        put32((uint32_t)L);
        w.write(hdr.data(), hdr.size());
        const size_t chunk = 1 << 16;
        const size_t nchunks = ((size_t)n + chunk - 1) / chunk;
        const int nt = std::max(1, p->n_threads);
        for (size_t c0 = 0; c0 < nchunks; c0 += (size_t)nt) {         // nt chunks in parallel, written in order
            const size_t c1 = std::min(nchunks, c0 + (size_t)nt);
            std::vector<std::vector<uint8_t>> bufs(c1 - c0);
            std::vector<std::thread> pool;
            for (size_t c = c0; c < c1; c++)
                pool.emplace_back([&, c]() {
                    sim_chunk(*p, ref_seq, L, starts, c * chunk, std::min((size_t)n, (c + 1) * chunk),
                              p->seed * 1000003ull + c, bufs[c - c0]);
                });
            for (auto &t : pool) t.join();
            for (auto &b : bufs) w.write(b.data(), b.size());
        }
        w.close();
        if (n_reads_out) *n_reads_out = n;
        return 0;
    } catch (const std::exception &e) {
        return fail(std::string("spp_simulate_bam: ") + e.what());
    }
}

}  // extern "C"

extern "C" int spp_synth_batch(const char *ref_seq, int64_t ref_len, int64_t lo, int64_t hi, const spp_sim_params *p,
                               int64_t max_depth, spp_batch **out) {
    if (!ref_seq || !p || !out) return fail("spp_synth_batch: null argument");
    if (lo < 0 || hi > ref_len || hi < lo) return fail("spp_synth_batch: bad column range");
    *out = nullptr;
    try {
        const int64_t L = ref_len, R = p->read_len, C = hi - lo;
        const int64_t n = (int64_t)std::llround(p->depth * (double)L / (double)R);
        std::vector<int64_t> starts((size_t)n);
        {
            std::mt19937_64 rng(p->seed);
            std::uniform_int_distribution<int64_t> S(0, std::max<int64_t>(0, L - R));
            for (auto &x : starts) x = S(rng);
            std::sort(starts.begin(), starts.end());
        }
        auto *B = new spp_batch();
        B->pos_begin = lo;
        B->n_cols = C;
        B->off.assign((size_t)C + 1, 0);
        for (int64_t c = 0; c < C; c++) {          // reads covering lo + c: starts in [lo+c-R+1, lo+c]
            const int64_t col = lo + c;
            const auto a = std::lower_bound(starts.begin(), starts.end(), col - R + 1);
            const auto b = std::upper_bound(starts.begin(), starts.end(), col);
            int64_t d = b - a;
            if (max_depth > 0) d = std::min(d, max_depth);
            B->off[(size_t)c + 1] = B->off[(size_t)c] + (uint64_t)d;
        }
        const uint64_t E = B->off[(size_t)C];
        B->n_entries = E;
        B->n_used = n;
        B->code = (uint8_t *)malloc(E + 16);
        B->qual = (uint8_t *)malloc(E + 16);
        if (!B->code || !B->qual) { delete B; return fail("spp_synth_batch: out of host memory"); }
        memset(B->code + E, 0xFF, 16);
        memset(B->qual + E, 0, 16);
        // quality -> error probability, the discrete q distribution (clip(round(N(mean, sd))))
        double eps[256];
        for (int q = 0; q < 256; q++) eps[q] = std::pow(10.0, -q / 10.0);
        const int nt = std::max(1, p->n_threads);
        const int64_t blk = 4096;                  // columns per RNG stream: deterministic for any nt
        const int64_t nblk = (C + blk - 1) / blk;
        std::atomic<int64_t> next{0};
        auto work = [&]() {
            static const uint8_t ACGT[4] = {1, 2, 4, 8};
            for (int64_t bi; (bi = next++) < nblk;) {
                std::mt19937_64 rng(p->seed * 0x9E3779B97F4A7C15ull + (uint64_t)bi * 7919u + 17u);
                std::uniform_real_distribution<double> U(0.0, 1.0);
                std::normal_distribution<double> Nq(p->q_mean, p->q_sd);
                const double del_rate = p->del_frac * 2.0 / (double)R;
                for (int64_t c = bi * blk; c < std::min(C, (bi + 1) * blk); c++) {
                    const int64_t col = lo + c;
                    const char rc = (char)toupper(ref_seq[col]);
                    const int ri = rc == 'A' ? 0 : rc == 'C' ? 1 : rc == 'G' ? 2 : rc == 'T' ? 3 : -1;
                    const bool planted = p->snv_every > 0 && col % p->snv_every == p->snv_every / 2 && ri >= 0;
                    static const double afs[4] = {1.0, 0.5, 0.2, 0.05};
                    const double af = planted ? afs[(col / p->snv_every) % 4] : 0.0;
                    const uint8_t alt = planted ? ACGT[(ri + 1 + (int)(col % 3)) % 4] : 0;
                    for (uint64_t e = B->off[(size_t)c]; e < B->off[(size_t)c + 1]; e++) {
                        uint8_t b = ri >= 0 ? ACGT[ri] : 15;
                        if (planted && U(rng) < af) b = alt;
                        int q = (int)std::lround(Nq(rng));
                        q = std::min(std::max(q, p->q_min), p->q_max);
                        if (b != 15 && U(rng) < eps[q]) {
                            const int bi2 = b == 1 ? 0 : b == 2 ? 1 : b == 4 ? 2 : 3;
                            b = ACGT[(bi2 + 1 + (int)(rng() % 3)) % 4];
                        }
                        if (U(rng) < p->n_rate) b = 15;
                        if (U(rng) < del_rate) b = 16;
                        B->code[e] = b;
                        B->qual[e] = (uint8_t)q;
                    }
                }
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(work);
        work();
        for (auto &t : pool) t.join();
        *out = B;
        return 0;
    } catch (const std::exception &e) {
        return fail(std::string("spp_synth_batch: ") + e.what());
    }
}
