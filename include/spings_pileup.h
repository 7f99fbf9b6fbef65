/*
 * spings_pileup.h — C-ABI of the host BAM/SAM reader and pileup emulator (libspings_pileup.so).
 *
 * Replaces the third-party pysam/htslib pileup that LiveVariantCaller.process_bam drives
 * (variant_caller/live_variant_caller.py:54-72): it turns one contig of a
 * coordinate-sorted BAM (or SAM) file into the CSR batch that spg_accumulate consumes
 * (include/spings_gpu.h): offsets u64[n_cols+1], base_code u8[E], qual u8[E].
 *
 * Semantics restated from htslib sam.c / pysam libcalignmentfile.pyx (not vendored, absent from
 * this image — parity unpinned):
 *   - reads of the contig in file order; the stepper's read filter (pysam "all": skip
 *     flag & (UNMAP|SECONDARY|QCFAIL|DUP); "samtools": also MAPQ < min_mapping_quality and
 *     paired-but-not-proper reads; "nofilter": none); htslib itself skips unmapped reads;
 *   - htslib's depth cap (bam_plp_push): a read starting at the pending column is dropped when
 *     the iterator's node count (buffered reads + 1) exceeds max_depth (pysam default 8000);
 *   - htslib's mate-overlap quality tweak when ignore_overlaps is set (pysam default True);
 *   - per column, the buffered reads covering it in buffer (file) order: CIGAR M/=/X give the
 *     base (BAM nibble) and its quality; D gives code 16, N code 17, each with the quality of
 *     the next query base (0 when past the end) — the value pysam's min_base_quality filter
 *     tests.  The base-quality filter itself is applied by the GPU engine.
 *   - columns with no buffered read are not emitted (offsets[c] == offsets[c+1]).
 * Every function returns 0 on success, < 0 on error (message: spp_last_error()).
 */
#ifndef SPINGS_PILEUP_H
#define SPINGS_PILEUP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPP_STEPPER_ALL 0        /* pysam stepper="all" (its default) */
#define SPP_STEPPER_NOFILTER 1   /* stepper="nofilter" */
#define SPP_STEPPER_SAMTOOLS 2   /* stepper="samtools" (MAPQ + orphan filter; no BAQ: no fastafile) */

typedef struct {
    int32_t stepper;               /* SPP_STEPPER_* */
    int32_t min_mapping_quality;   /* applied by the samtools stepper (pileup(min_mapping_quality=)) */
    int32_t max_depth;             /* htslib maxcnt; pysam default 8000; <= 0 = unlimited (extension) */
    int32_t ignore_overlaps;       /* 1 = htslib overlap quality tweak (pysam default) */
    uint32_t flag_filter;          /* samtools stepper flag filter (pysam default 0x704) */
    int32_t n_threads;             /* BGZF inflate / CSR fill threads (<= 0: 1) */
    int32_t inflate_device;        /* records plans: inflate the BGZF members with the inflater spp_set_inflater
                                      registered, on this GPU (-1, the default: on the host's threads) ... */
    int32_t inflate_min_members;   /* ... when the BAM has at least this many members (<= 0: 4096) */
    int64_t reserved[1];
} spp_params;

typedef struct spp_file spp_file;
typedef struct spp_batch spp_batch;

const char *spp_last_error(void);
/* The host BGZF inflater this process uses for records plans and host fills: "libdeflate" (its runtime library is
 * loaded with dlopen when present) or "zlib" (absent, or SPP_NO_LIBDEFLATE set before the first inflate). */
const char *spp_host_inflater(void);
void spp_default_params(spp_params *p);

/* Open a BAM (BGZF) or SAM file and parse its header. */
int spp_open(const char *path, spp_file **out);
int spp_close(spp_file *f);
int spp_n_targets(spp_file *f, int32_t *n);
/* name pointer valid until spp_close */
int spp_target(spp_file *f, int32_t tid, const char **name, int64_t *length);
int spp_target_id(spp_file *f, const char *name, int32_t *tid);

/* AlignmentFile.pileup(reference=<contig tid>, ...) over the whole contig -> one CSR batch.
 * The batch covers columns [pos_begin, pos_begin + n_cols) (first..last emitted column). */
int spp_pileup(spp_file *f, int32_t tid, const spp_params *p, spp_batch **out);
/* The columns [lo, hi) of spp_pileup's batch (bit-identical to slicing it), for a coordinate shard
 * (SURVEY §8 e): every read's fixed fields are parsed (htslib's depth cap depends on all pushes), but
 * bases and qualities are decoded only for reads within a read span of the region, and the CSR
 * holds only the region's columns. */
int spp_pileup_region(spp_file *f, int32_t tid, int64_t lo, int64_t hi, const spp_params *p, spp_batch **out);
int spp_batch_info(spp_batch *b, int64_t *pos_begin, int64_t *n_cols, uint64_t *n_entries,
                   int64_t *n_reads_used, int64_t *n_reads_dropped);
/* Arrays owned by the batch (valid until spp_batch_free).  base_code and qual are allocated
 * with 16 bytes of padding past n_entries (code 0xFF, qual 0) so they can be handed to the GPU
 * engine without a copy. */
int spp_batch_arrays(spp_batch *b, const uint64_t **offsets, const uint8_t **base_code, const uint8_t **qual);
int spp_batch_free(spp_batch *b);

/* Two-phase pileup for an ingest pipeline: spp_pileup_plan parses the reads, applies the depth cap /
 * overlap rules and computes the CSR offsets (n_entries known: spp_batch_info); spp_batch_fill then
 * writes base_code / qual into caller buffers of >= n_entries + 16 bytes each (e.g. pinned memory from
 * spg_host_alloc, reused across BAMs: no page faults, DMA-able), or into its own allocation when both
 * are null.  The batch keeps the caller's pointers (spp_batch_arrays) and does not free them.  Region
 * form: lo/hi as in spp_pileup_region (INT64_MIN / INT64_MAX = whole contig). */
int spp_pileup_plan(spp_file *f, int32_t tid, int64_t lo, int64_t hi, const spp_params *p, spp_batch **out);
int spp_batch_fill(spp_batch *b, uint8_t *base_code, uint8_t *qual);

/* Device-decode form of spp_pileup_plan (BAM only): the BGZF members are inflated in parallel
 * straight into one buffer, the records' fixed fields are parsed on the host (what the stepper filter, the
 * depth cap and the overlap pairing decide on), and the packed bases / qualities are NOT decoded: the batch
 * exposes the raw record bytes and per-read index as an spg_records (include/spings_gpu.h) for
 * spg_accumulate_records, whose kernel writes the CSR entries.  The record buffer comes from the host
 * allocator below when one is set (spg_host_alloc: pinned, so the copy to HBM is a DMA), else malloc; it is
 * reused across plans.  spp_batch_fill is not available on such a batch. */
struct spg_records;
int spp_pileup_plan_records(spp_file *f, int32_t tid, int64_t lo, int64_t hi, const spp_params *p, spp_batch **out);
int spp_batch_records(spp_batch *b, struct spg_records *out);
/* Allocator for the record buffers (e.g. spg_host_alloc / spg_host_free); NULLs restore malloc/free. */
typedef int (*spp_alloc_fn)(size_t bytes, void **out);
typedef int (*spp_free_fn)(void *p);
int spp_set_host_allocator(spp_alloc_fn alloc, spp_free_fn release);
/* BGZF inflater for the records plans (e.g. spg_bgzf_inflate): called once per BAM with the plan's
 * spp_params.inflate_device, the mapped file, its members ({u64 coff, u32 clen, u32 ulen, u64 uoff}, layout of
 * spg_bgzf_member) and the record buffer; members whose status is not 0 are inflated on the host.  Each plan chooses
 * through its spp_params (inflate_device >= 0, at least inflate_min_members members: fewer inflate faster on the
 * host's threads), so callers with different choices do not override one another; NULL unregisters it.  `device` is
 * kept for the ABI and ignored. */
typedef int (*spp_inflate_fn)(int device, const uint8_t *comp, size_t comp_bytes, const void *members, int64_t n,
                              uint8_t *out, size_t out_bytes, uint32_t *status, float *kernel_ms);
int spp_set_inflater(spp_inflate_fn fn, int device);

/* A BAM kept in HBM (include/spings_gpu.h spg_bam_*).  spp_bam_map_open reads the file (parallel pread)
 * into one host buffer (pinned under the allocator hook) for spg_bam_open, and locates its BGZF members there
 * (parallel header search, chains that must meet) and the header's end; the handle keeps the buffer until
 * spp_bam_map_close.
 * spp_pileup_plan_fields replays htslib's depth cap and mate pairing (spp_pileup_plan's rules) on the reads' fixed
 * fields as spg_bam_reads_copy returns them — names compared by their 64-bit hash (the device verifies every pair's
 * names) — computes the CSR offsets, and returns the overlapping mate pairs instead of tweaking qualities on the host;
 * spp_batch_device_plan exposes the plan as an spg_bam_plan for spg_bam_accumulate.  spp_batch_fill / records are not
 * available on such a batch. */
typedef struct {
    const uint8_t *comp;           /* the file's bytes (64 zero bytes of padding past comp_bytes) */
    uint64_t comp_bytes;
    const void *members;           /* spg_bgzf_member[n_members] (include/spings_gpu.h), in file order */
    int64_t n_members;
    uint64_t inflated_bytes;       /* the inflated stream's length */
    uint64_t body;                 /* offset of the first record in it (the header's end) */
    int32_t n_ref;                 /* the header's reference count */
    int32_t reserved;
} spp_bam_map_info;
typedef struct spp_bam_map spp_bam_map;
int spp_bam_map_open(spp_file *f, int n_threads, spp_bam_map **out, spp_bam_map_info *info);
int spp_bam_map_close(spp_bam_map *h);
typedef struct {                   /* one contig's reads after the stepper filter, in BAM order (spg_bam_reads) */
    int64_t n;
    const int32_t *pos, *end, *mtid, *mpos, *isize;
    const uint16_t *flag;
    const uint32_t *l_seq;
    const uint64_t *name_hash;
} spp_read_fields;
int spp_pileup_plan_fields(spp_file *f, int32_t tid, const spp_read_fields *reads, const spp_params *p, spp_batch **out);
struct spg_bam_plan;
int spp_batch_device_plan(spp_batch *b, struct spg_bam_plan *out);

/* Synthetic read simulator (SURVEY.md §8 d "Synthetic inputs"): writes a coordinate-sorted BGZF
 * BAM of single-end reads (flag 0, MAPQ 60) over one contig — starts uniform on [0, L-read_len],
 * CIGAR read_len M (a del_frac share "70M2D..M", an ins_frac share "70M2I..M"), q =
 * clip(round(N(q_mean, q_sd)), q_min, q_max), a sequencing error replaces the base with a uniform
 * other base with probability eps(q), N with probability n_rate, planted SNVs every snv_every-th
 * position (offset snv_every/2) with allele fractions cycling {1.0, 0.5, 0.2, 0.05}.  Seeded. */
typedef struct {
    double depth;          /* mean coverage */
    int32_t read_len;      /* 150 */
    int32_t snv_every;     /* 997; 0 = none */
    double q_mean, q_sd;   /* 33, 6 */
    int32_t q_min, q_max;  /* 2, 41 */
    double del_frac, ins_frac, n_rate;   /* 0.01, 0.01, 1e-4 */
    uint64_t seed;
    int32_t n_threads;     /* BGZF deflate threads */
    int32_t level;         /* zlib level (1 = fast) */
    int64_t reserved[2];
} spp_sim_params;

void spp_default_sim_params(spp_sim_params *p);
int spp_simulate_bam(const char *path, const char *contig, const char *ref_seq, int64_t ref_len,
                     const spp_sim_params *p, int64_t *n_reads_out);

/* Synthetic pileup straight to CSR (no BAM), for the large benchmark configs (100,000x, chr1 30x):
 * the read model of spp_simulate_bam at column level — reads of read_len start uniformly (sorted),
 * column c holds the reads covering it in start order; per entry q, sequencing error, N and planted
 * SNVs as above, CIGAR D entries (code 16, quality of the next base) at rate del_frac*2/read_len.
 * Columns [lo, hi) of a reference of ref_len; multi-threaded, deterministic for a seed. */
int spp_synth_batch(const char *ref_seq, int64_t ref_len, int64_t lo, int64_t hi, const spp_sim_params *p,
                    int64_t max_depth, spp_batch **out);

#ifdef __cplusplus
}
#endif
#endif /* SPINGS_PILEUP_H */
