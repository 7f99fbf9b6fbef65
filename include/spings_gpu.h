/*
 * spings_gpu.h — C-ABI of the MI355X (gfx950) pileup + genotype-likelihood engine.
 *
 * Drop-in boundary for the hot path of COVID-SpiNGS/covid-spings-variant-caller
 * (SURVEY.md §8 b).  The reference has no FFI for this path (it is pure Python over pysam);
 * these entry points are what its `LiveVariantCaller` (variant_caller/live_variant_caller.py)
 * binds through ctypes — see INTEGRATION.md for the binding stub.  Every function cites the
 * reference interface it replaces.
 *
 * Conventions
 *   - Plain pointers and sizes only; no torch or HIP types in signatures.
 *   - Every function returns int status: 0 = ok, < 0 = error; spg_last_error() returns the
 *     thread-local message of the last failing call (replaces pysam's Python exceptions, which
 *     the reference lets propagate uncaught).
 *   - A context is NOT re-entrant: callers serialise calls on one context (the Python shim
 *     holds a lock; the reference calls the engine from daemon threads, vc_queue.py:99-111).
 *   - Work is enqueued on the context's own HIP stream; spg_sync() blocks.  Every spg_get_*
 *     call synchronises the stream before copying.
 *
 * Column boundary (CSR): a batch is `n_cols` consecutive reference positions
 * starting at `pos_begin`; `offsets[n_cols+1]` (u64) delimit each column's pileup entries in
 * `base_code[]` / `qual[]` (u8 each).  base_code is the BAM 4-bit nibble (0..15,
 * "=ACMGRSVTWYHKDBN"), 16 = CIGAR D (is_del), 17 = CIGAR N (is_refskip).  For D/N entries
 * `qual` is the quality of the next aligned query base (0 if none) — the value pysam's
 * base-quality filter tests.  Entries are in htslib pileup order (surviving reads in BAM order);
 * the maxcnt cap and the read filters (flags, MAPQ) are applied before the boundary; the
 * base-quality filter is applied by the engine.  A column with no entries is "not emitted"
 * (htslib never yields an empty column).
 */
#ifndef SPINGS_GPU_H
#define SPINGS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPG_ABI_VERSION 1

/* Allele slots of the per-position table (dict keys of Site.snvs, structs.py:2-6).
 * Other IUPAC nibbles / '=' are exact too, but reported through spg_detail records. */
#define SPG_NSLOT 5           /* A C G T N */
#define SPG_NCOUNT 8          /* A C G T N DEL REFSKIP OTHER */
#define SPG_CODE_DEL 16
#define SPG_CODE_SKIP 17

/* per-position flags (spg_get_table) */
#define SPG_F_PRESENT 0x01    /* position is in LiveVariantCaller.memory */
#define SPG_F_EVALUATED 0x02  /* totalDepth >= minTotalDepth: GLs computed (:131) */
#define SPG_F_REPLAYED 0x04   /* resolved by the exact sequential replay (subnormal band / exotic) */
#define SPG_F_EXOTIC 0x08     /* has alleles outside A,C,G,T,N (see spg_detail) */
#define SPG_F_CANDIDATE 0x10  /* produced >= 1 variant */
#define SPG_F_PARTIAL 0x20    /* SPG_P_CALLS_ONLY: some table GL of this position not computed (NaN) */

/* accumulate flags */
#define SPG_IN_DEVICE 0x1     /* offsets/base_code/qual are device pointers on the ctx device */
#define SPG_IN_BORROW 0x2     /* with SPG_IN_DEVICE: keep the caller's device buffers as replay
                                 history without copying; they must stay valid until
                                 spg_reset/spg_destroy, and base_code / qual must be readable for
                                 16 bytes past the last entry (the kernels load 16-B blocks) */
#define SPG_IN_TRUSTED 0x4    /* host input produced by spp_pileup / spp_batch_fill (already valid CSR):
                               skip the O(E) host validation scan */

/* spg_params.flags */
#define SPG_P_CALLS_ONLY 0x1  /* compute what prepare_variants() emits and nothing it cannot see: the
                                 deep kernel does not accumulate sum(ln(1-eps)) / sum(eps) of a
                                 column's major allele when it is the REF char (never a candidate).
                                 Candidates stay exact (positions whose calls would depend on the
                                 missing terms are replayed); table GL entries that depend on them
                                 read NaN and the position carries SPG_F_PARTIAL. */

/* LiveVariantCaller ctor thresholds (live_variant_caller.py:22-29); minMappingQuality and
 * maxVariants act before the boundary / are unused by the reference, so they are not here. */
typedef struct {
    int32_t min_base_quality;    /* pileup min_base_quality -> pysam pileup_base_qual_skip */
    int32_t min_total_depth;     /* :131 */
    int32_t min_allele_depth;    /* :153 */
    int32_t flags;               /* SPG_P_* */
    double min_evidence_ratio;   /* :154 */
    int64_t reserved1[4];
} spg_params;

/* One emitted variant (a row of prepare_variants(), live_variant_caller.py:170-185). */
typedef struct {
    int64_t pos;           /* 'start' (0-based); 'stop' = pos + 1 */
    int32_t dp;            /* info DP  = totalDepth */
    int32_t ad;            /* info AD  = len(snvs[allele]) */
    int32_t pl;            /* info PL  = round(-10*gl), 0 when GL == 0 */
    int32_t score;         /* info SCORE = to_phred_scale(1 - GL/sum(GL)) */
    uint8_t ref;           /* alleles[0]: reference char as stored at first visit (case kept) */
    uint8_t alt;           /* alleles[1]: allele char "=ACMGRSVTWYHKDBN"[code] */
    uint8_t gl_zero;       /* 1 when GL == 0 (then info GL is the int 0) */
    uint8_t rank;          /* index of the allele in snvs dict order */
    uint32_t first_batch;  /* batch sequence number (1-based) of the position's first visit:
                              prepare_variants iterates memory in insertion order */
    double gl;             /* info GL = log10(GL) (0 when GL == 0) */
    double gl_linear;      /* GL itself (utils.genotype_likelihood) */
    double qual;           /* 'qual' = np.mean(eps list) */
} spg_candidate;           /* 56 bytes */

/* Full per-allele record of a replayed position (exotic alleles, subnormal band). */
typedef struct {
    int64_t pos;
    uint32_t depth;
    uint8_t n_alleles;     /* alleles in dict order */
    uint8_t pad[3];
    uint8_t code[16];      /* nibble codes in dict order */
    uint32_t count[16];
    double gl[16];         /* exact reference-order GL per allele (NaN if not evaluated) */
} spg_detail;              /* 224 bytes */

typedef struct spg_ctx spg_ctx;

/* thread-local message of the last failing call ("" if none) */
const char *spg_last_error(void);
int spg_abi_version(void);

/* LiveVariantCaller.__init__ (live_variant_caller.py:22-32): device accumulators for n_pos
 * reference positions on HIP device `device`. */
int spg_create(int device, int64_t n_pos, const spg_params *p, spg_ctx **out);
int spg_destroy(spg_ctx *ctx);                             /* __del__ (:34-35) */
int spg_reset(spg_ctx *ctx);                               /* reset_memory (:37-38) */

/* from_phred_scale (utils.py:9-10): the 256 eps values, produced by the caller with the
 * reference's own math.pow so device eps are bit-identical. */
int spg_set_eps_lut(spg_ctx *ctx, const double lut[256]);

/* fastaFile.fetch(reference_name) (:78): the contig the next batches belong to; the char at
 * a position is stored on its first visit (memory[pos]['reference'], :81). */
int spg_set_reference(spg_ctx *ctx, const char *seq, int64_t len);

/* process_bam / process_pileup_column / process_svn (:54-103) for one CSR batch.
 * Accumulates across calls like `memory` does.  Host pointers by default (copied on the ctx
 * stream); see SPG_IN_* flags.  Returns after enqueue. */
int spg_accumulate(spg_ctx *ctx, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                   const uint8_t *base_code, const uint8_t *qual, uint64_t n_entries);
int spg_accumulate_ex(spg_ctx *ctx, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                      const uint8_t *base_code, const uint8_t *qual, uint64_t n_entries, uint32_t flags);

/* Many batches (BAMs) in one call: exactly n successive spg_accumulate_ex calls, without n trips
 * through the binding (process_bam over a list of BAMs, vc_queue.py:142-144 repeated).  Shallow
 * batches (mean < 256 entries per column) are not launched one by one: the context folds a run of
 * them per position in one pass (each record read and written once per run), when the run reaches
 * 4,096 batches, before a deep batch, and at spg_finalize. */
typedef struct {
    int64_t pos_begin, n_cols;
    const uint64_t *offsets;       /* n_cols + 1 */
    const uint8_t *base_code, *qual;
    uint64_t n_entries;
} spg_batch;
int spg_accumulate_batches(spg_ctx *ctx, const spg_batch *batches, int64_t n, uint32_t flags);

/* BASELINE config 4 ingest: n_samples BAMs over one coordinate range in ONE column-major CSR batch,
 * the layout a multi-BAM pileup (samtools mpileup style) emits: column c's entries are sample 0's
 * pileup entries at that position, then sample 1's, ..., each in its own BAM order.  Accumulating it
 * equals n_samples successive spg_accumulate calls, one per sample in sample order (the reference's
 * process_bam per BAM, live_variant_caller.py:54-103): dict order follows the concatenated stream,
 * batch numbers advance by n_samples, and a position first visited here gets first_batch =
 * (first batch number) + first_sample[c], the first sample with an entry at c (NULL: 0 for every
 * column).  Each position's stream is one long column, so the deep kernel streams it. */
int spg_accumulate_samples(spg_ctx *ctx, int64_t pos_begin, int64_t n_cols, int64_t n_samples,
                           const uint64_t *offsets, const uint32_t *first_sample, const uint8_t *base_code,
                           const uint8_t *qual, uint64_t n_entries, uint32_t flags);

/* Device-side pileup (replaces the host CIGAR walk of process_bam, live_variant_caller.py:54-72
 * driving pysam's pileup): one BAM contig's inflated records plus the host's per-read decisions
 * (spp_pileup_plan_records: stepper filter, htslib depth cap, mate-overlap tweak, CSR offsets).  The
 * engine copies the record bytes to HBM and a kernel decodes the packed bases / qualities, walks each
 * read's CIGAR and writes the batch's base_code / qual in htslib column order (reads in BAM order per
 * column; D = 16 / N = 17 with the next query base's quality, 0 past the read end) — bit-identical to
 * spp_batch_fill of the same plan.  The batch is then accumulated like spg_accumulate_ex's. */
typedef struct spg_records {
    int64_t pos_begin, n_cols;     /* the batch's columns */
    uint64_t n_entries;
    const uint64_t *offsets;       /* n_cols + 1 */
    const uint8_t *data;           /* inflated BAM bytes holding the records (64 readable bytes of padding past
                                      data_bytes) */
    uint64_t data_bytes;
    int64_t n_reads;               /* the reads with entries in the columns, in BAM order (< 2^31) */
    const uint64_t *rec;           /* per read: offset in data of its record's refID field */
    const int32_t *rpos, *rend;    /* per read: first reference position, one past its CIGAR's last */
    const int32_t *tweak;          /* per read: index into tweak_col / tweak_qual, or -1 */
    int64_t n_tweaks;
    const int64_t *tweak_col;      /* the read's D/N entries in columns < tweak_col read orig_qual (the
                                      qualities before htslib's mate-overlap tweak; data holds the tweaked ones) */
    const uint64_t *tweak_qual;    /* offset of the read's original qualities in orig_qual */
    const uint8_t *orig_qual;
    uint64_t orig_bytes;
    int64_t max_span;              /* max(rend - rpos) */
    int64_t pos_origin;            /* rpos / rend / tweak_col are reference positions; the context's position of
                                      reference position x is x - pos_origin (0 for a context over the whole contig;
                                      spg_multi passes each device's cut) */
    int64_t reserved[3];
} spg_records;
int spg_accumulate_records(spg_ctx *ctx, const spg_records *r, uint32_t flags);

/* Pinned (page-locked) host staging buffers for the CSR inputs (north_star: "SoA pinned buffers").
 * Inputs in pinned memory are copied asynchronously on the context's copy stream: spg_accumulate
 * returns after enqueue and the caller must not modify them until spg_wait_input (or spg_sync)
 * returns.  Pageable inputs are copied before spg_accumulate returns. */
int spg_host_alloc(size_t bytes, void **out);
int spg_host_free(void *p);
/* Block until every input copy enqueued so far has completed (the host buffers are free again). */
int spg_wait_input(spg_ctx *ctx);
/* Per-batch input tracking for double-buffered staging: spg_input_ticket returns the number of host-input
 * batch copies enqueued so far (the ticket of the latest one); spg_wait_ticket(t) blocks until copy #t has
 * landed (not the copies enqueued after it), so staging set A can be refilled while set B's copy runs. */
int spg_input_ticket(spg_ctx *ctx, uint64_t *ticket);
int spg_wait_ticket(spg_ctx *ctx, uint64_t ticket);

/* prepare_variants (:120-231) + genotype_likelihood / to_phred_scale (utils.py:12-24):
 * per-position table and the candidate list, on device.  Returns after enqueue. */
int spg_finalize(spg_ctx *ctx);

int spg_sync(spg_ctx *ctx);
/* The context's HIP stream (hipStream_t as void*), so a caller can order its own work against the
 * engine's without host synchronisation (e.g. torch.cuda.ExternalStream + wait_stream). */
int spg_stream(spg_ctx *ctx, void **stream);

/* Copy table rows [pos0, pos0+n) to host; any pointer may be NULL.
 *   depth[n] u32; counts[n*8] u32 (A C G T N DEL REFSKIP OTHER); gl[n*5] f64 (A C G T N,
 *   NaN where not evaluated / allele absent); flags[n] u8 (SPG_F_*); order[n] u32 (snvs dict
 *   order: bits 0-2 = k, bits 3+3i..5+3i = slot of the i-th allele); first_batch[n] u32. */
int spg_get_table(spg_ctx *ctx, int64_t pos0, int64_t n, uint32_t *depth, uint32_t *counts, double *gl,
                  uint8_t *flags, uint32_t *order, uint32_t *first_batch);
/* Number of candidates / replayed details produced by the last spg_finalize. */
int spg_count(spg_ctx *ctx, int64_t *n_candidates, int64_t *n_details);
/* Candidates in device append order (the shim orders them by (first_batch, pos, rank)). */
int spg_get_candidates(spg_ctx *ctx, spg_candidate *out, int64_t cap, int64_t *n_out);
int spg_get_details(spg_ctx *ctx, spg_detail *out, int64_t cap, int64_t *n_out);

/* Device pointers of the result buffers (for zero-copy consumers on the same device, e.g. a
 * torch.distributed gather).  Valid until the next spg_finalize / spg_reset / spg_destroy. */
int spg_device_results(spg_ctx *ctx, void **candidates, void **n_candidates);

/* Device-to-device copy of the call table into caller memory on the ctx device: dst[0..8) gets the
 * candidate count (u64), dst + 8 up to `cap` spg_candidate records.  Enqueued on the ctx stream:
 * order a consumer on another stream (e.g. an RCCL gather) after it through spg_stream. */
int spg_copy_candidates_device(spg_ctx *ctx, void *dst, int64_t cap);

/* The call table and its status in one device-side copy into caller memory on the ctx device (no host wait; the
 * multi-device gather's per-context step): dst[0..16) = {u32 candidates (true count), u32 status, u32 details,
 * u32 records copied}, then min(candidates, *n_copy_cap) spg_candidate records, *n_copy_cap = min(cap, the context's
 * candidate buffer).  status bits: 1 replay depth mismatch, 2 run error word, 4 fill error word, 8 more candidates
 * than the copy holds, 16 more details than the context's buffer.  Any bit set: take this finalize's table through
 * spg_count / spg_get_candidates (they report the error, or grow the buffers and finalize again). */
int spg_copy_table_device(spg_ctx *ctx, void *dst, int64_t cap, int64_t *n_copy_cap);

/* Bound the HBM held by the context's own copies of accumulated batches (the replay history; borrowed
 * batches are the caller's).  Past `bytes`, the oldest batches already folded into the records (or, calls-only,
 * into the counted totals) move to pinned host memory; the rare readers (exact replay, the exact fold of the
 * positions that may call, re-materialization) read them there over PCIe.  0 = no cap (default; env
 * SPG_HIST_CAP sets it at spg_create).  Replaces nothing in the reference: its `memory` grows in host RAM
 * (live_variant_caller.py:100-103); this keeps the engine from being the first thing to run out. */
int spg_set_history_cap(spg_ctx *ctx, int64_t bytes);
/* Owned history bytes resident in HBM, batches spilled to host, arena bytes allocated (any may be NULL). */
int spg_history_resident(spg_ctx *ctx, int64_t *device_bytes, int64_t *n_spilled, int64_t *arena_bytes);

/* The accumulated batches (replay history) since the last spg_reset, in accumulate order: the
 * exact state behind LiveVariantCaller.memory, used for create_checkpoint (:40-45) and the
 * memory view.  spg_history_copy copies batch i to host buffers (offsets n_cols+1, base_code /
 * qual n_entries each; any may be NULL) and synchronises. */
int spg_history_count(spg_ctx *ctx, int64_t *n_batches);
int spg_history_info(spg_ctx *ctx, int64_t i, int64_t *pos_begin, int64_t *n_cols, uint64_t *n_entries);
int spg_history_copy(spg_ctx *ctx, int64_t i, uint64_t *offsets, uint8_t *base_code, uint8_t *qual);
/* Batch i as create_checkpoint keeps it (live_variant_caller.py:40-45; the pickled memory holds only the qualities
 * that passed the base-quality filter, :89/:96-103, and every first visit, :77-85): its entries with q >= min_bq, plus
 * the first entry of a column whose entries all fail the filter (a marker that records the visit; the engine filters
 * it again on resume).  Compacted on the device; offsets (n_cols + 1, host) always, base_code / qual (host, room
 * for the batch's n_entries) get *n_kept entries.  Synchronises. */
int spg_history_copy_compact(spg_ctx *ctx, int64_t i, int32_t min_bq, uint64_t *offsets, uint8_t *base_code,
                             uint8_t *qual, uint64_t *n_kept);
/* The same kept entries packed one byte each (the checkpoint shard's packed form): (b << 6) | q for base A/C/G/T
 * (BAM nibble 1/2/4/8 -> b 0..3) with q <= 62; any other entry is byte 63 plus an exception (its index in the batch's
 * kept entries, its code, its quality) in exc_* — *n_exc of them, in no particular order.  packed: room for the batch's
 * n_entries; when *n_exc > exc_cap the exceptions were not copied (call again with more room, or use
 * spg_history_copy_compact).  Synchronises. */
int spg_history_copy_packed(spg_ctx *ctx, int64_t i, int32_t min_bq, uint64_t *offsets, uint8_t *packed, uint64_t *n_kept,
                            uint64_t *exc_index, uint8_t *exc_code, uint8_t *exc_qual, int64_t exc_cap, int64_t *n_exc);
/* One position's entries over the whole history, in accumulate order (the q list behind memory[pos], before the
 * base-quality filter): *n_out = their number; codes / quals get them when n_out <= cap (cap 0: count only).
 * Synchronises.  LiveVariantCaller.memory builds a Site from this per lookup instead of expanding every entry. */
int spg_position_entries(spg_ctx *ctx, int64_t pos, uint8_t *codes, uint8_t *quals, int64_t cap, int64_t *n_out);
/* The same over the first n_batches batches of the history only (a memory view taken before later batches). */
int spg_position_entries_upto(spg_ctx *ctx, int64_t pos, int64_t n_batches, uint8_t *codes, uint8_t *quals, int64_t cap,
                              int64_t *n_out);
/* Samples of history batch i (1 unless it came from spg_accumulate_samples) and, if first_sample is
 * not NULL, its per-column first samples (n_cols; zeros for a single-sample batch). */
int spg_history_samples(spg_ctx *ctx, int64_t i, int64_t *n_samples, uint32_t *first_sample);

/* Timing hooks (bench): HIP events around the accumulate launches of one finalize step (first
 * begin .. last end) and around the finalize launch, ms.  spg_last_kernel_ms: the latest step.
 * spg_kernel_times: every step completed since the previous spg_kernel_times call (at most 64
 * are kept), oldest first, without timing-induced stalls between steps.  Both synchronise. */
int spg_last_kernel_ms(spg_ctx *ctx, float *accumulate_ms, float *finalize_ms);
/* Which timing events are recorded from now on: 2 = accumulate + finalize (default, or env
 * SPG_TIMING), 1 = accumulate only, 0 = none; unrecorded intervals read as 0 ms.  Each event pair
 * costs a few microseconds of GPU idle time between launches. */
int spg_set_timing(spg_ctx *ctx, int level);
int spg_kernel_times(spg_ctx *ctx, float *accumulate_ms, float *finalize_ms, int64_t cap, int64_t *n_out);

/* Which engine paths ran since spg_create (tests / profiling; counters only grow):
 *   out[0] record-path runs (k_acc_tile over a run of shallow batches, incl. re-materializations)
 *   out[1] re-materializations (records a fused / counted finalize left stale, re-folded from batch 0)
 *   out[2] full-range finalizes (k_finalize over every position)      out[3] sparse finalizes (listed positions)
 *   out[4] counted finalizes (k_acc_lite_run + k_count_list + k_fold_hist)
 *   out[5] fused deep finalizes (k_acc_seg FUSE, or list mode)           out[6] fused shallow finalizes (k_acc_lite)
 *   out[7] batches counted by k_acc_lite_run
 *   out[8] lone mid-depth batches counted by k_count_cols (+ k_acc_seg<1> over the listed columns)
 * Writes min(n, 9) values. */
int spg_path_counters(spg_ctx *ctx, int64_t *out, int64_t n);

/* BGZF members inflated on the GPU (the records plan's BAM read).  comp: the file's bytes (each
 * member's raw-DEFLATE payload at coff, clen bytes, followed by its 8-byte CRC32/ISIZE trailer); out: the inflated
 * stream (member m at uoff, exactly ulen <= 65536 bytes).  status[m] = 0 when member m inflated to ulen bytes whose
 * CRC32 matches the trailer's (else the caller inflates it on the host).  kernel_ms: the inflate + CRC kernels' time
 * (may be null; -1 when the timing failed).  Synchronous; the caller's current device is kept. */
typedef struct spg_bgzf_member {
    uint64_t coff;
    uint32_t clen;
    uint32_t ulen;
    uint64_t uoff;
} spg_bgzf_member;
int spg_bgzf_inflate(int device, const uint8_t *comp, size_t comp_bytes, const spg_bgzf_member *members, int64_t n,
                     uint8_t *out, size_t out_bytes, uint32_t *status, float *kernel_ms);
const char *spg_bgzf_last_error(void);
/* Free spg_bgzf_inflate's scratch on `device` (grow-only otherwise). */
int spg_bgzf_release(int device);
/* The same decoder compiled for the host (CPU tests of its logic only; comp needs 8 readable bytes past each
 * member's payload, as in a BGZF file). */
int spg_bgzf_inflate_check(const uint8_t *comp, size_t comp_bytes, const spg_bgzf_member *members, int64_t n,
                           uint8_t *out, size_t out_bytes, uint32_t *status);
/* The parallel inflater (k_inflate_par: 64 lanes per member, self-synchronising segment decode) run on the host lane
 * after lane (CPU tests of its algorithm only): status[m] 0, or 100 when the GPU would leave member m to the
 * one-lane-per-member decoder; stats[10]: members inflated, token overflows, segments that did not synchronise, stored
 * blocks, bad headers, no end of block, bad resolve, redo tokens, blocks, phase-A tokens before the meeting points. */
int spg_bgzf_inflate_par_check(const uint8_t *comp, size_t comp_bytes, const spg_bgzf_member *members, int64_t n,
                               uint8_t *out, size_t out_bytes, uint32_t *status, uint64_t *stats);
/* Members of the last spg_bgzf_inflate on `device` that the parallel kernel left to the one-lane-per-member decoder. */
int spg_bgzf_fallbacks(int device, int64_t *n);

/* ---- a BAM kept in HBM (the lone process_bam, live_variant_caller.py:54-72) ---------------------------
 * Only the compressed file goes up and the reads' fixed fields come down: spg_bam_open copies the BGZF bytes to the
 * context's device, inflates every member there (k_inflate + a CRC32 check per member), locates the records of contig
 * `tid` in the inflated stream (parallel block_size chains from each member's first record, which must meet exactly)
 * and applies the stepper's read filter; spg_bam_reads_copy hands the kept reads' fields to the host, which replays
 * htslib's depth cap and mate pairing on them (spp_pileup_plan_fields, include/spings_pileup.h); spg_bam_accumulate
 * takes that plan — the kept reads, the CSR offsets, the overlapping mate pairs — applies the mate-overlap quality
 * tweak in HBM and writes the batch's entries with k_pileup_fill, then accumulates it like spg_accumulate_records
 * (bit-identical batch).  One BAM per slot at a time (spg_bam_slot: two slots per context); its device buffers are
 * reused by the slot's next spg_bam_open (stream-ordered after this BAM's fill).  Return 1 (not < 0) means "not handled here, nothing accumulated": a member
 * the GPU could not inflate (corrupt, CRC mismatch), record chains that disagree, or two paired reads whose names
 * differ behind an equal name hash — the caller then plans the BAM on the host (spp_pileup_plan_records). */
typedef struct {
    int32_t stepper;               /* SPP_STEPPER_*: 0 all, 1 nofilter, 2 samtools */
    uint32_t flag_filter;          /* samtools stepper */
    int32_t min_mapping_quality;   /* samtools stepper */
    int32_t reserved;
} spg_bam_filter;
/* comp: the whole file (each member's payload at members[m].coff with its 8-byte trailer after it); body: offset of the
 * first record in the inflated stream (after the header); n_ref: the header's reference count.  *n_reads: the kept
 * reads of contig tid. */
int spg_bam_open(spg_ctx *ctx, const uint8_t *comp, uint64_t comp_bytes, const spg_bgzf_member *members, int64_t n_members,
                 uint64_t body, int32_t tid, int32_t n_ref, const spg_bam_filter *filter, int64_t *n_reads);
/* Optional prefetch: start copying a BAM's compressed bytes and member table into device slot `slot` on the context's
 * upload stream and return; a later spg_bam_open of the same (comp, comp_bytes, n_members) in that slot waits for these
 * copies instead of making its own.  comp must stay valid until that spg_bam_open returns.  process_bams sends BAM i + 1
 * this way (into the other slot) before opening BAM i, so the upload overlaps BAM i's inflate. */
int spg_bam_upload(spg_ctx *ctx, int slot, const uint8_t *comp, uint64_t comp_bytes, const spg_bgzf_member *members,
                   int64_t n_members);
typedef struct {                   /* host arrays with room for n_reads values each, in BAM order */
    int32_t *pos, *end, *mtid, *mpos, *isize;   /* end: pos + the CIGAR's reference length */
    uint16_t *flag;
    uint32_t *l_seq;
    uint64_t *name_hash;           /* FNV-1a 64 of the read name */
} spg_bam_reads;
int spg_bam_reads_copy(spg_ctx *ctx, const spg_bam_reads *out);
typedef struct spg_bam_plan {
    int64_t pos_begin, n_cols;
    uint64_t n_entries;
    const uint64_t *offsets;       /* n_cols + 1 */
    int64_t n_kept;
    const uint32_t *kept;          /* reads (indices into spg_bam_open's reads) with entries, BAM order */
    int64_t n_pairs;
    const uint32_t *pair_a, *pair_b;   /* overlapping mates: a (pushed first) and b */
    const int64_t *pair_col;       /* a's D / N entries in columns < pair_col read its qualities before the tweak */
    const uint64_t *pair_orig;     /* offset of a's saved qualities (sum of the earlier pairs' a l_seq) */
    uint64_t orig_bytes;
    int64_t max_span;              /* max(end - pos) over the kept reads */
    int64_t reserved[4];
} spg_bam_plan;
/* flags: SPG_IN_DEVICE when the plan's arrays are in HBM (spg_bam_plan_build), else host arrays. */
int spg_bam_accumulate(spg_ctx *ctx, const spg_bam_plan *plan, uint32_t flags);
/* The open BAM's plan built on the GPU — htslib's depth cap (max_depth 0: none) and, with ignore_overlaps, its mate
 * pairing over the kept reads' fixed fields: the arrays spp_pileup_plan_fields computes on the host from
 * spg_bam_reads_copy, here without the fields leaving HBM.  *plan gets device pointers (valid until this slot's next
 * spg_bam_open / spg_bam_plan_build) for spg_bam_accumulate(..., SPG_IN_DEVICE).  Returns 1 (nothing built, reason in
 * spg_last_error) when the device declines: a read without reference span, a read spanning more than 8,000 columns
 * under a cap, more than 16 reads sharing a name hash, a capped contig of > 4 M start positions where the cap bites;
 * the caller then plans the BAM on the host (spg_bam_reads_copy + spp_pileup_plan_fields). */
int spg_bam_plan_build(spg_ctx *ctx, int64_t max_depth, int32_t ignore_overlaps, spg_bam_plan *plan);
/* A built plan's arrays copied to host memory (n_cols + 1 offsets, n_kept reads, n_pairs of each pair array; any may
 * be NULL). */
int spg_bam_plan_download(spg_ctx *ctx, const spg_bam_plan *plan, uint64_t *offsets, uint32_t *kept, uint32_t *pair_a,
                          uint32_t *pair_b, int64_t *pair_col, uint64_t *pair_orig);
/* ms of the last spg_bam_open's inflate + CRC kernels (HIP events) */
int spg_bam_inflate_ms(spg_ctx *ctx, float *ms);
/* members of the last spg_bam_open that the parallel inflater left to the one-lane-per-member decoder */
int spg_bam_inflate_fallbacks(spg_ctx *ctx, int64_t *n);
/* Free the BAM buffers of both slots (the next spg_bam_open allocates them again). */
int spg_bam_release(spg_ctx *ctx);
/* The BAM slot (0 or 1, default 0) the next spg_bam_* calls use: each slot holds one open BAM's device buffers, so a
 * caller can open the next BAM in the other slot while the host plans this one (LiveVariantCaller.process_bams); a
 * slot's buffers are reused by its next spg_bam_open, ordered after that slot's spg_bam_accumulate on the context's
 * copy stream. */
int spg_bam_slot(spg_ctx *ctx, int slot);

/* Introspection for tests. */
int spg_device_count(int *n);
size_t spg_sizeof_candidate(void);
size_t spg_sizeof_detail(void);
size_t spg_sizeof_acc(void);

/* ---- one process, N devices (SURVEY §8 b/e; shard.py's ShardedEngine without torch) ----------------------
 * Each device's context owns a contiguous coordinate range [cuts[d], cuts[d+1]) in its own coordinate space
 * (records, counted totals and reference slice for that range only).  Cuts give every device equal entries over a
 * per-bucket entry histogram: a sample is planned at its first batch (from the previous sample's histogram when
 * there is one, else from that batch) and re-planned — its history re-sliced and re-accumulated — when one device's
 * cumulative load exceeds `ratio` x the mean while the sample holds at most `max_batches` batches
 * (spg_multi_set_rebalance; default 1.25, 256).  Every device takes every batch (an empty slice becomes one empty
 * column), so batch numbers and first visits stay global; the compact call tables come back to devices[0] with ONE
 * RCCL ncclGather over xGMI (a device listed twice — one GPU standing in for several — uses device copies instead)
 * and are merged in memory order (first_batch, pos, allele rank), positions in reference coordinates.  Sliced
 * offsets and record indices are staged in per-device pinned rings, so the devices' copies overlap.  Replaces the
 * reference's single-process loop (live_variant_caller.py:54-185) for multi-GPU hosts. */
typedef struct spg_multi spg_multi;
int spg_multi_create(const int *devices, int n, int64_t n_pos, const spg_params *params, spg_multi **out);
int spg_multi_destroy(spg_multi *m);
const char *spg_multi_last_error(void);
int spg_multi_set_eps_lut(spg_multi *m, const double lut[256]);
/* A contig shorter than n_pos is padded with 'N' internally; batches past its end are refused. */
int spg_multi_set_reference(spg_multi *m, const char *seq, int64_t len);
int spg_multi_reset(spg_multi *m);
/* Host CSR batch, as spg_accumulate (SPG_IN_TRUSTED allowed; no device / borrowed input).  Pinned inputs are copied
 * asynchronously: keep them until spg_multi_wait_input. */
int spg_multi_accumulate(spg_multi *m, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                         const uint8_t *base_code, const uint8_t *qual, uint64_t n_entries, uint32_t flags);
/* A BAM records plan (spg_accumulate_records, pos_origin 0), sharded: each device decodes the reads that reach its
 * range on the GPU.  The plan's buffers are read asynchronously: keep them until spg_multi_wait_input. */
int spg_multi_accumulate_records(spg_multi *m, const spg_records *r, uint32_t flags);
/* The cuts a batch (host offsets) gets — the sample's, planned now when it has none yet (cuts: n + 1 values). */
int spg_multi_plan(spg_multi *m, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets, int64_t *cuts);
/* A batch already resident in HBM, one slice per device (slices[d]: device pointers on devices[d], pos_begin in
 * reference coordinates, exactly the batch's columns inside [cuts[d], cuts[d+1]) with offsets rebased to 0, n_cols 0
 * where the batch misses the device's range); offsets: the whole batch's CSR on the host (the entry histogram).
 * flags: SPG_IN_DEVICE [| SPG_IN_BORROW].  The per-rank shards of north_star's "positions shard by coordinate
 * range" when each GPU already holds its part of the pileup. */
int spg_multi_accumulate_slices(spg_multi *m, int64_t pos_begin, int64_t n_cols, const uint64_t *offsets,
                                const spg_batch *slices, uint32_t flags);
int spg_multi_wait_input(spg_multi *m);
int spg_multi_finalize(spg_multi *m);
/* The merged call table (needs n_out <= cap; *n_out is set either way).  One host wait per call: every device's table
 * and status are copied on the device (spg_copy_table_device), gathered, and brought down in one copy; only a table that
 * outgrew the copy (or an error word) takes the settling path per device. */
int spg_multi_get_candidates(spg_multi *m, spg_candidate *out, int64_t cap, int64_t *n_out);
/* The same table without waiting (replaces vc_queue.py:142-144's blocking prepare_variants per BAM when the caller
 * pipelines samples): everything is enqueued — the device copies, the gather, one copy into pinned host memory — and
 * *ticket names it.  The next sample's spg_multi_reset / accumulate / finalize may be enqueued before its wait.  Two
 * tables may be in flight; a third enqueue retires the oldest (its wait then fails).  A ticket is waited for once
 * (repeat the wait with a larger cap while it returns -1 with *n_out > cap). */
int spg_multi_get_candidates_async(spg_multi *m, uint64_t *ticket);
/* Wait for a ticket's table and merge it in memory order.  Returns 1 (nothing written, *n_out = 0) when a device's
 * table did not fit the copy or carried an error word: that sample's table must be taken with spg_multi_get_candidates
 * before its contexts move on (reset); the copies are sized from every table seen, so this happens at most while the
 * first tables of a run grow. */
int spg_multi_wait_candidates(spg_multi *m, uint64_t ticket, spg_candidate *out, int64_t cap, int64_t *n_out);
/* cuts[0..n]: device i owns positions [cuts[i], cuts[i+1]) (after the sample's first batch). */
int spg_multi_partition(spg_multi *m, int64_t *cuts);
int spg_multi_set_rebalance(spg_multi *m, double ratio, int64_t max_batches);
/* Re-plans (history re-sliced) since creation. */
int spg_multi_replans(spg_multi *m, int64_t *n);
/* Equal-entry cuts over a bucket histogram (w[b] = entries in positions [b bucket, (b+1) bucket)): cuts[0] = 0,
 * cuts[n] = n_pos, every range non-empty.  Host only (no GPU). */
int spg_multi_plan_cuts(const uint64_t *w, int64_t n_buckets, int64_t bucket, int64_t n_pos, int n, int64_t *cuts);
/* The context of device index i, in its own coordinates (position x of the contig is x - cuts[i] there). */
int spg_multi_context(spg_multi *m, int i, spg_ctx **ctx);

#ifdef __cplusplus
}
#endif
#endif /* SPINGS_GPU_H */
