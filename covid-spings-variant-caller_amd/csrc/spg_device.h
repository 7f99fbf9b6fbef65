// spg_device.h — device-side data layout shared by the engine kernels (gfx950) and the host API.
//
// Layout in HBM (one context = one contiguous reference range of n_pos positions):
//   Acc      acc[n_pos]      160 B AoS record per position (accumulators of LiveVariantCaller.memory)
//   Tables   *tables         eps / ln(1-eps) / 10^-k LUTs (from the reference's from_phred_scale)
//   Hist     hist[n_batches] descriptors of the accumulated CSR batches (the exact replay walks them)
//   batch CSR                offsets u64[n_cols+1], base_code u8[E], qual u8[E] (16-B padded)
//   outputs (SoA)            depth u32, counts u32[8], gl f64[5], flags u8, order u32, first_batch u32,
//                            candidates, details, Counters[2]
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spings_gpu.h"

namespace spg {

constexpr int NSLOT = SPG_NSLOT;          // A C G T N
constexpr uint32_t INF32 = 0xFFFFFFFFu;
constexpr uint32_t MISC_EXOTIC = 0x100u;  // acc.misc bit: an allele outside A,C,G,T,N was seen
// acc.misc bits 9..13: slot k's sum(ln(1-eps)) and sum(eps) are incomplete (SPG_P_CALLS_ONLY: the deep
// kernel skips them for a column's major allele when it is the REF char; finalize treats that
// allele's hypothesis product as unknown and replays a position whose calls would depend on it)
constexpr int MISC_SKIP_SHIFT = 9;
// acc.misc bits 14..18: slot k's sum(eps) IS complete although its skip bit is set (only its
// sum(ln(1-eps)) is not: the fused deep kernel's second allele in dual mode keeps QUAL's sum)
constexpr int MISC_SEONLY_SHIFT = 14;

// k_acc_seg's per-wave LDS: a finishing ring of SPG_NB columns (fused: a wave's whole group) and the
// descriptors of its group (at most SPG_GMAX_DEEP columns per wave of a deep batch, SPG_GMAX for the
// W = 1 kernel).  Sized so a 4-wave workgroup stays under 32 KiB: 5 workgroups per CU, so the waves of
// a fifth start in the slots of finished waves while their workgroups' longest wave still runs.
#ifndef SPG_NB
#define SPG_NB 4
#endif
#ifndef SPG_GMAX
#define SPG_GMAX 64
#endif
#ifndef SPG_GMAX_DEEP
#define SPG_GMAX_DEEP 16
#endif

// Accumulators replacing Site (structs.py:2-6).  The q lists are replaced by sufficient
// statistics: counts, the integer sum of q (log10 of the eps product up to fp64 rounding), the sum
// of ln(1-eps) (the hypothesis product), the sum of eps (QUAL), a lower bound on q (H == 0 iff a
// Q0 entry; q >= 4 makes every eps factor < 1/2, which the underflow proof needs) and the dict
// insertion order of the alleles.  The exact ordered lists live on as the batch history that the
// replay walks for the rare positions where the order of fp64 roundings matters.
// A record belongs to the current sample only when `epoch` matches the context's epoch: reset is
// an epoch bump, not a memset.
struct __align__(16) Acc {
    uint32_t depth;        // totalDepth (:75, :87)
    uint32_t first_batch;  // batch seq of first visit (dict insertion order); 0 = not in memory
    uint32_t order;        // bits 0-2 n alleles; bits 3+3i.. slot of i-th allele (snvs dict order)
    uint32_t misc;         // bits 0-7 REF char stored at first visit (:81); MISC_EXOTIC
    uint32_t n_del, n_skip, n_other, epoch;
    uint32_t cnt[NSLOT];
    uint32_t sq[NSLOT];    // sum q, saturating at 2^31
    uint8_t qf[8];         // q lower bound per slot (exact below 4)
    double sl[NSLOT];      // sum ln(1 - eps)
    double se[NSLOT];      // sum eps
};
static_assert(sizeof(Acc) == 160, "Acc layout");

struct Tables {
    double eps[256];       // from_phred_scale(q), bit-identical to the reference (host-supplied)
    double l1m[256];       // log1p(-eps[q]); l1m[0] = 0 (Q0 handled through qf == 0)
    double p10k[336];      // 10^-k, correctly rounded, k = 0..335
    double fast[256][2];   // {l1m, eps} for q = 1..255; row 0 = {0, 0} ("not selected" / Q0)
};

struct Hist {               // one accumulated batch, kept for the exact replay
    int64_t pos_begin, n_cols;
    const uint64_t *off;
    const uint8_t *code;
    const uint8_t *qual;
};

struct KParams {
    int64_t pos_begin, n_cols;
    int32_t min_bq, qlo;   // qlo = max(min_bq, 4): fast-path floor
    uint32_t kpass, kok;   // SWAR compare constants
    uint32_t batch_seq;    // 1-based within the epoch
    uint32_t epoch;
    uint32_t G;            // columns per wave group
    uint32_t w1, G2;       // waves >= w1 own G2 (< G) columns: the last grid generation's waves are
                           // shorter, so the launch's tail is (w1 = all waves: no split)
    uint32_t t_deep;       // columns with >= t_deep raw entries are processed wave-wide
    uint32_t calls_only;   // SPG_P_CALLS_ONLY
    uint32_t rot;          // SPG_WAVE_ROT (profiling): block b takes block (b + rot) % grid's work (XCD placement)
    uint64_t n_entries;    // entries of the batch (launch shape only)
    Hist hdesc;            // this batch's history descriptor ...
    Hist *hslot;           // ... written here by the first thread of the launch
    const struct FusedArgs *fused;   // k_acc_seg<..., FUSE>: finalize parameters of this Counters slot (device
                                     // memory: read only for the positions that pass the pre-check below)
    int32_t min_td, min_ad;          // FUSE: prepare_variants' filters (:131, :151-157) for the division-free
    double ratio_lo;                 // pre-check (ratio_lo = min_evidence_ratio * (1 - 1e-9))
    const uint32_t *fsamp; // multi-sample batch: per column, the first sample holding entries (else null)
    uint32_t *dbg;         // SPG_TRACE: range violations recorded here instead of faulting (else null)
    uint4 *prog;           // SPG_TRACE: per-wave progress records in host-mapped memory (else null)
    const uint32_t *deep_list;   // W = 1: the long columns the run kernel listed (batch-relative) ...
    const uint32_t *deep_n;      // ... and their count (null: one group of G columns per wave)
    uint4 *wtime;          // SPG_WAVE_TIMES: per wave {start, first column, lifetime} (s_memrealtime, 100 MHz), hw id
    // calls-only listing (a FRESH deep batch, the sample's only one, whose waves own more columns than the finishing
    // ring holds — mid-depth columns, e.g. 1,000x): each finished ring's records pass the division-free pre-check
    // of prepare_variants' filters (:131, :151-157) and the positions that may call are listed here for the
    // sparse k_finalize (null: no listing)
    int64_t *list;
    uint32_t *n_list;
};

// Per-position state of a run of batches folded by one lane group (k_acc_tile), and
// the partial record one batch split hands to k_merge_parts (same 176-B layout in HBM).
struct __align__(16) MState {
    uint32_t depth, n_del, n_skip, n_other;
    uint32_t cnt[NSLOT], sq[NSLOT];
    uint32_t first[NSLOT];   // stream index (raw entries of this position in the split) of the slot's
                             // first entry; INF32 if absent
    uint32_t fb;             // launch-relative index of the first batch holding raw entries (INF32: none)
    uint8_t qf[NSLOT];       // q lower bound per slot (255 = none)
    uint8_t skip;            // slots whose sum(ln(1-eps)) / sum(eps) were skipped (calls-only REF)
    uint8_t flags;           // image bits after the record is assembled: 1 write, 2 write the sums half
    uint8_t pad0;
    uint32_t pad1[2];
    double sl[NSLOT], se[NSLOT];
};
static_assert(sizeof(MState) == 176, "MState layout");

struct MParams {             // one run-kernel launch: history batches [h0, h0 + K) over positions [u0, u1)
    int64_t u0, u1;
    int32_t h0, K;
    int32_t S, kper;         // batch splits (partial records merged by k_merge_parts when S > 1)
    int32_t n_groups;        // 64-position groups
    int32_t min_bq, qlo;
    uint32_t kpass, kok;
    uint32_t seq0;           // batch_seq of batch h0 (1-based within the epoch)
    uint32_t epoch;
    uint32_t calls_only;
    uint32_t t_deep;         // K == 1: columns with >= t_deep entries are left to k_acc_seg (0 = none)
    uint32_t fresh;          // seq0 == 1: no record of this epoch exists yet
    uint32_t ref_sl;         // calls-only, shallow run: still sum ln(1-eps) for a REF-char major (at such
                             // depths a call's GL is not 0, its SCORE needs S = sum(GL), which needs the
                             // REF allele's H; skipping it would send every call to the exact replay)
    MState *part;            // S > 1: partial records [S][pstride]
    int64_t pstride;         // positions per split in `part` (>= u1 - u0)
    uint32_t *err;           // bit 0: a 64-column window of a run's batch held >= 2^30 entries (not run)
    uint32_t *deep_list;     // K == 1: columns with >= t_deep entries, listed for k_acc_seg<1> ...
    uint32_t *deep_n;        // ... and their count
    // fused (k_acc_lite: a lone FRESH shallow batch folded at spg_finalize, calls-only) and counted mode
    // (k_count_list): a record is written only for positions that can produce a call (prepare_variants' filters
    // :131, :151-157) or need the exact replay; they are listed for the sparse finalize
    int32_t min_td, min_ad;
    double ratio_lo;         // min_evidence_ratio * (1 - 1e-9): the conservative AD/DP pre-check
    int64_t *list;           // positions whose record was written (the sparse finalize's input)
    uint32_t *n_list;
    // counted mode's exact fold (k_fold_hist), incremental: wm[p] = (wm_gen << 32) | n says position p's record
    // already holds history batches [0, n) (written by an earlier counted finalize of this sample; any other
    // generation: fold from batch 0)
    uint64_t *wm;
    uint32_t wm_gen;
    uint32_t pad_wm;
};

// Replay index: history batches overlapping each 2^RIDX_SHIFT-position bucket, in accumulate order.
constexpr int RIDX_SHIFT = 12;
struct RIndex {
    const uint32_t *off;     // [n_buckets + 1]
    const int32_t *items;    // history indices
    int64_t n_buckets;       // 0: no index, scan every batch
};

// Replay cache: the exact sequential fold state of a replayed position after history batches [0, upto), so the
// next finalize's replay of it (the live loop finalizes after every BAM, vc_queue.py:142-144) folds only the
// batches since.  Open addressing, one slot per position per epoch, claimed by atomicCAS on `key`
// ((epoch << 32) | (pos + 1)); slots of older epochs are reclaimed.  H folds are kept only for the codes whose
// N_h = prod over the other alleles' P was non-zero at the last replay ("alive"): P products only shrink as
// entries arrive, so a code whose N_h reached exactly 0 never needs its H again (H * 0 == 0).
struct RSlot {
    uint64_t key;
    uint32_t upto, alive;   // history batches folded (0: no state yet); codes whose H fold is tracked
    uint32_t depth, pad;
    uint64_t ord;           // raw entries of the position folded so far (stream index of the next one)
    uint32_t cnt[16];
    uint64_t first[16];
    double P[16], H[16], se[16];
};
constexpr int RCACHE_SLOTS = 8192;
constexpr int RCACHE_PROBE = 16;
struct RCache {
    RSlot *slot;            // null: no cache (every replay folds the whole history)
    uint32_t mask, pad;
};

struct Counters {           // per finalize; two slots, the kernel zeroes the other one
    uint32_t n_cand, n_band, n_detail, err;   // n_band: positions queued for the exact replay
};

struct FParams {
    int64_t n_pos;
    int32_t min_td, min_ad;
    double ratio;
    int64_t cand_cap, band_cap, detail_cap;
    int32_t min_bq, n_hist;
    uint32_t epoch, cslot;
    uint32_t table;        // write the per-position SoA table (else: calls only, early exits)
    uint32_t pad_;
    RIndex ridx;
    const int64_t *list;   // sparse finalize: only these positions (*n_list of them); null = every position
    const uint32_t *n_list;
    RCache rc;             // replay cache (null slot: none)
};

struct Out {                // SoA result table
    uint32_t *depth, *counts, *order, *first;
    double *gl;
    uint8_t *flags;
    spg_candidate *cand;
    int64_t *band;
    spg_detail *detail;
    Counters *ctr;          // Counters[2]
};

struct FusedArgs {          // the fused accumulate's finalize (one per Counters slot; F.epoch unused)
    FParams F;
    Out O;
};

__device__ __forceinline__ int slot_of(uint32_t c) {
    return c == 1u ? 0 : c == 2u ? 1 : c == 4u ? 2 : c == 8u ? 3 : c == 15u ? 4 : -1;
}
__host__ __device__ __forceinline__ uint32_t slot_code(int s) {
    return s == 0 ? 1u : s == 1 ? 2u : s == 2 ? 4u : s == 3 ? 8u : 15u;
}
__host__ __device__ __forceinline__ uint8_t nibble_char(uint32_t c) {
    // "=ACMGRSVTWYHKDBN"[c & 15] from two immediates (no memory load in the device code)
    const uint64_t t = (c & 8u) ? 0x4E42444B48595754ull : 0x565352474D43413Dull;
    return (uint8_t)(t >> (8u * (c & 7u)));
}

// spg_accumulate_records: the device-side pileup (spg_fill.hip)
struct FillArgs {
    const uint8_t *data;           // the inflated BAM (64 readable pad bytes past data_bytes)
    uint64_t data_bytes;
    const uint64_t *rec;           // per read: offset of its refID field in data
    const int32_t *rpos, *rend, *tweak;
    const int64_t *tw_col;
    const uint64_t *tw_q;
    const uint8_t *orig;
    uint64_t orig_bytes;
    void *scratch;                 // fill_scratch_bytes(): tile_first [n_tiles + 1] (first read starting at or after
                                   // the tile), item offsets [n_tiles + 1], the scan's temporary, group starts
    size_t scratch_bytes;
    const uint64_t *off;           // CSR offsets [n_cols + 1]
    uint8_t *code, *qual;
    int64_t pos_begin;
    int32_t n_cols, n_tiles;
    uint32_t n_reads;
    int32_t back;                  // tiles to look back: ceil(max_span / 64)
    uint32_t *err;                 // |= 2: the records disagree with the offsets (inconsistent plan)
};

// The pileup plan of a BAM in HBM built on the GPU (spg_plan.hip, spg_bam_plan_build): htslib's depth cap and mate
// pairing over the kept reads' fixed fields (what spp_pileup_plan_fields replays on the host).
struct PlanHead {                  // reductions and counts (zeroed / initialised by launch_plan_init)
    int32_t min_span, max_span;    // over every read
    int32_t max_span_kept, pad0;
    uint32_t err;                  // 1: a read without reference span or out of order; 2: a name group too large
    uint32_t n_distinct;           // distinct start positions
    uint32_t n_kept, n_pairs;
    int64_t min_pos, max_end;      // over every read
    int64_t lo, hi;                // kept reads' column range [lo, hi)
    uint64_t n_entries, orig_bytes;
    int32_t max_cov, n_cand;       // coverage maximum over every read; pair candidates
};
struct PlanArgs {
    uint32_t n;                    // reads, BAM (= coordinate) order
    const int32_t *pos, *end, *mtid, *mpos, *isize;
    const uint16_t *flag;
    const uint32_t *l_seq;
    const uint64_t *nhash;
    int32_t tid;
    int32_t olap;                  // ignore_overlaps: mate pairing
    int64_t maxcnt;                // max_depth (INT64_MAX: uncapped)
    int64_t span_lo;               // column range the diff arrays cover: [span_lo, span_lo + span_n)
    int64_t span_n;
    PlanHead *head;
    uint32_t *first;               // [n + 1] 1 at a read that starts a new position; then (scanned) its distinct index
    uint32_t *didx;                // [n + 1] exclusive scan of first
    int32_t *dpos;                 // [n_distinct] distinct start positions
    uint32_t *dfirst;              // [n_distinct + 1] their first read
    uint8_t *keep;                 // [n] htslib keeps the read (max_depth)
    uint32_t *kept;                // [n] kept reads in BAM order
    int32_t *diff;                 // [span_n + 1] coverage difference array, then coverage
    uint64_t *offsets;             // [span_n + 1] CSR offsets of the kept reads' columns
    uint64_t *skey;                // [n] name hashes sorted (with sval: read index)
    uint32_t *sval;
    uint32_t *pairb;               // [n] first mate + 1 of a second mate (0: none)
    uint32_t *pb_list;             // [n] second mates in BAM order
    uint32_t *pa, *pbv;            // [n_pairs] pairs (first mate, second mate) in push order
    int64_t *pcol;                 // [n_pairs] tweak column (htslib's iterator position at the second mate's push)
    uint64_t *porig;               // [n_pairs] offset of the first mate's saved qualities
    uint64_t *lsa;                 // [n_pairs] the first mates' l_seq (scanned into porig)
};

// A BAM in HBM (spg_bam.hip, include/spings_gpu.h spg_bam_*)
constexpr uint64_t BAM_NONE = ~0ull;
constexpr uint32_t BAM_RTMP = 2048;  // kept records the counting walk lists per member (a 64 KiB member holds <= 1,821)
struct BamArgs {
    const uint8_t *data;           // the inflated stream (64 readable pad bytes past total)
    uint64_t total, body;          // its length; the first record's offset (after the header)
    const uint64_t *uoff;          // [n_members + 1] members' inflated offsets
    int64_t n_members;
    int32_t tid, n_ref;
    int32_t stepper;               // SPP_STEPPER_*: 0 all, 1 nofilter, 2 samtools
    uint32_t flag_filter;
    int32_t min_mapq;
    uint32_t n_reads;              // fields pass: listed reads
    uint64_t *start;               // [n_members] first record start in the member's range (BAM_NONE: none)
    uint32_t *cnt, *base;          // kept records per member's chain; their exclusive prefix
    int64_t *pos_lo, *pos_hi;      // first / last position of the contig's records per chain (sort order)
    uint64_t *rec;                 // listed reads: offset of the refID field
    uint64_t *rtmp;                // [n_members * BAM_RTMP] the counting walk's kept records per member (pass 4 copies)
    int32_t *pos, *end, *mtid, *mpos, *isize;
    uint16_t *flag;
    uint32_t *l_seq;
    uint64_t *nhash;
    uint32_t *err;                 // 1: chains disagree / truncated record; 2: not sorted; 4: corrupt lengths
};
struct BamPairArgs {
    const uint8_t *data;
    uint8_t *wdata;                // the same stream, written (tweak)
    const uint64_t *rec;
    uint32_t n_reads, n_pairs;
    const uint32_t *pa, *pb;       // pair j: first mate's / second mate's read index
    const uint64_t *oq;            // pair j: offset of the first mate's saved qualities in orig
    uint8_t *orig;
    uint32_t *err;                 // 8: a pair's names differ (a name-hash collision)
};
struct BamGatherArgs {
    uint32_t n_reads, n_kept, n_pairs;
    const uint32_t *kept, *pa;
    const uint64_t *rec;
    const int32_t *pos, *end;
    int32_t *twof;                 // [n_reads] pair index of a first mate (-1: none)
    uint64_t *rec_k;
    int32_t *rpos_k, *rend_k, *tw_k;
    uint32_t *err;
};

}  // namespace spg
