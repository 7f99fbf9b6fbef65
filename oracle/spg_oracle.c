/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 * Never linked into, loaded by, or called from the product path.
 *
 * Plain-C restatement of the reference's per-position pileup + genotype-likelihood path
 * (COVID-SpiNGS/covid-spings-variant-caller), driven by the build's CSR column boundary
 * (SURVEY §8 a3).  It reproduces the reference's fp64 arithmetic operation-for-operation:
 *
 *   spo_accumulate  <- variant_caller/live_variant_caller.py:74-103  (process_pileup_column,
 *                      process_svn) + pysam's access-time base-quality filter of
 *                      PileupColumn.pileups (pileup_base_qual_skip, restated)
 *   spo_finalize    <- live_variant_caller.py:120-185 (prepare_variants; the indel branch
 *                      :187-229 is dead because process_indel's call is commented out at :94)
 *   prod_seq        <- np.prod == strict left fold (utils.py:17,19)
 *   gl chain        <- utils.py:16-24: H_h * ((1.0 * P_a1) * P_a2 ...) in dict order
 *   mean_np         <- np.mean == numpy pairwise_sum(all) / n (live_variant_caller.py:168)
 *   to_phred        <- utils.py:12-13, Python round() == rint() (half-to-even)
 *   eps             <- utils.py:9-10 via a 256-entry LUT produced by math.pow in Python
 *
 * Pinned against golden vectors from the reference's own code: tests/test_oracle_golden.py.
 * Build: make -C oracle   (-> oracle/_build/libspg_oracle.so)
 */
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NCODE 16
#define CODE_DEL 16
#define CODE_SKIP 17

static const char NIBBLE[17] = "=ACMGRSVTWYHKDBN";

typedef struct {
    uint8_t n_all;          /* alleles in dict insertion order */
    uint8_t code[NCODE];
    uint32_t len[NCODE], cap[NCODE];
    uint8_t *q[NCODE];
} site_t;

typedef struct {
    int64_t n_pos;
    char *ref;
    int min_bq, min_td, min_ad;
    double ratio;
    double eps[256];
    /* memory */
    uint8_t *present;
    uint64_t *depth;        /* totalDepth */
    uint64_t *n_del, *n_skip;
    site_t **site;
    int64_t *ins;           /* positions in dict insertion order */
    int64_t n_ins;
    /* finalize outputs */
    int64_t n_var, cap_var;
    struct spo_variant *var;
    double *gl;             /* [n_pos*16] by dict-order index; NaN if not evaluated */
} spo_ctx;

typedef struct spo_variant {
    int64_t start;
    int32_t dp, ad, pl, score;
    uint8_t ref, alt, gl_zero, pad[5];
    double gl;              /* log10(GL) or 0 */
    double gl_linear;       /* GL */
    double qual;            /* np.mean(eps) */
} spo_variant;

spo_ctx *spo_create(int64_t n_pos, const char *ref, int min_bq, int min_td, int min_ad, double ratio,
                    const double *eps_lut) {
    spo_ctx *c = (spo_ctx *)calloc(1, sizeof(spo_ctx));
    c->n_pos = n_pos;
    c->ref = (char *)malloc((size_t)n_pos + 1);
    memcpy(c->ref, ref, (size_t)n_pos);
    c->ref[n_pos] = 0;
    c->min_bq = min_bq; c->min_td = min_td; c->min_ad = min_ad; c->ratio = ratio;
    memcpy(c->eps, eps_lut, sizeof(c->eps));
    c->present = (uint8_t *)calloc((size_t)n_pos, 1);
    c->depth = (uint64_t *)calloc((size_t)n_pos, 8);
    c->n_del = (uint64_t *)calloc((size_t)n_pos, 8);
    c->n_skip = (uint64_t *)calloc((size_t)n_pos, 8);
    c->site = (site_t **)calloc((size_t)n_pos, sizeof(site_t *));
    c->ins = (int64_t *)malloc((size_t)n_pos * 8);
    c->gl = (double *)malloc((size_t)n_pos * NCODE * 8);
    return c;
}

static void free_sites(spo_ctx *c) {
    for (int64_t i = 0; i < c->n_pos; i++) {
        site_t *s = c->site[i];
        if (!s) continue;
        for (int k = 0; k < NCODE; k++) free(s->q[k]);
        free(s);
        c->site[i] = NULL;
    }
}

void spo_reset(spo_ctx *c) {   /* reset_memory, live_variant_caller.py:37-38 */
    free_sites(c);
    memset(c->present, 0, (size_t)c->n_pos);
    memset(c->depth, 0, (size_t)c->n_pos * 8);
    memset(c->n_del, 0, (size_t)c->n_pos * 8);
    memset(c->n_skip, 0, (size_t)c->n_pos * 8);
    c->n_ins = 0;
    c->n_var = 0;
}

void spo_destroy(spo_ctx *c) {
    if (!c) return;
    free_sites(c);
    free(c->ref); free(c->present); free(c->depth); free(c->n_del); free(c->n_skip);
    free(c->site); free(c->ins); free(c->gl); free(c->var);
    free(c);
}

static inline void site_append(site_t *s, uint8_t code, uint8_t q) {
    int k;
    for (k = 0; k < s->n_all; k++)
        if (s->code[k] == code) break;
    if (k == s->n_all) { s->code[k] = code; s->n_all++; }   /* :100-101 first-seen order */
    if (s->len[k] == s->cap[k]) {
        s->cap[k] = s->cap[k] ? s->cap[k] * 2 : 16;
        s->q[k] = (uint8_t *)realloc(s->q[k], s->cap[k]);
    }
    s->q[k][s->len[k]++] = q;                               /* :103 */
}

/* Threads for spo_accumulate / spo_finalize (OpenMP; 1 = the sequential restatement).  Positions are
 * independent, so the per-position arithmetic (and every output bit) is the same for any count. */
static int g_threads = 1;
void spo_set_threads(int n) { g_threads = n > 0 ? n : 1; }
int spo_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* live_variant_caller.py:74-103 over one CSR batch */
int spo_accumulate(spo_ctx *c, int64_t pos_begin, int64_t n_cols, const uint64_t *off, const uint8_t *code,
                   const uint8_t *qual) {
    if (pos_begin < 0 || pos_begin + n_cols > c->n_pos) return -1;
    /* first visits in column order (:77-85): memory insertion order */
    for (int64_t i = 0; i < n_cols; i++) {
        int64_t pos = pos_begin + i;
        if (off[i + 1] == off[i] || c->present[pos]) continue;   /* htslib emits no empty column */
        c->present[pos] = 1;
        c->ins[c->n_ins++] = pos;
        c->site[pos] = (site_t *)calloc(1, sizeof(site_t));
    }
    int err = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 256) num_threads(g_threads) reduction(| : err)
#endif
    for (int64_t i = 0; i < n_cols; i++) {
        uint64_t lo = off[i], hi = off[i + 1];
        if (hi == lo) continue;
        int64_t pos = pos_begin + i;
        uint64_t total = 0;
        for (uint64_t e = lo; e < hi; e++)
            if (!(c->min_bq > 0 && qual[e] < c->min_bq)) total++;   /* :75 len(pileups) */
        c->depth[pos] += total;                             /* :81 / :87 */
        site_t *s = c->site[pos];
        for (uint64_t e = lo; e < hi; e++) {                /* :89-103 */
            uint8_t q = qual[e], cd = code[e];
            if (c->min_bq > 0 && q < c->min_bq) continue;
            if (cd == CODE_DEL) { c->n_del[pos]++; continue; }
            if (cd == CODE_SKIP) { c->n_skip[pos]++; continue; }
            if (cd >= NCODE) { err = 1; break; }
            site_append(s, cd, q);
        }
    }
    return err ? -2 : 0;
}

/* numpy pairwise_sum_DOUBLE (PW_BLOCKSIZE 128, unroll 8) */
static double pairwise(const double *a, int64_t n) {
    if (n < 8) {
        double r = 0.;
        for (int64_t i = 0; i < n; i++) r += a[i];
        return r;
    } else if (n <= 128) {
        double r[8];
        int64_t i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise(a, n2) + pairwise(a + n2, n - n2);
    }
}

static int to_phred(double p) {                             /* utils.py:12-13 */
    if (!(p > 0.0)) return 99;
    double r = rint(-10.0 * log10(p));
    return r < 99.0 ? (int)r : 99;
}

static void push_var(spo_ctx *c, spo_variant *v) {
    if (c->n_var == c->cap_var) {
        c->cap_var = c->cap_var ? c->cap_var * 2 : 1024;
        c->var = (spo_variant *)realloc(c->var, (size_t)c->cap_var * sizeof(spo_variant));
    }
    c->var[c->n_var++] = *v;
}

/* One position of prepare_variants (:131-185): GL per allele (utils.py:16-24) into glp, the emitted
 * variants into out (at most NCODE); returns their number. */
static int finalize_pos(const spo_ctx *c, int64_t pos, double **eps, size_t *eps_cap, spo_variant *out) {
    double *glp = c->gl + pos * NCODE;
    for (int k = 0; k < NCODE; k++) glp[k] = NAN;
    if (c->depth[pos] < (uint64_t)(c->min_td < 0 ? 0 : c->min_td)) return 0;   /* :131 */
    const site_t *s = c->site[pos];
    int n = s->n_all;
    double P[NCODE], H[NCODE], Q[NCODE];
    for (int k = 0; k < n; k++) {
        uint32_t m = s->len[k];
        if (m > *eps_cap) { *eps_cap = m * 2; *eps = (double *)realloc(*eps, *eps_cap * 8); }
        double *e = *eps;
        for (uint32_t j = 0; j < m; j++) e[j] = c->eps[s->q[k][j]];     /* :132-138 */
        double p = e[0], h = 1.0 - e[0];                                /* np.prod left fold */
        for (uint32_t j = 1; j < m; j++) { p *= e[j]; h *= (1.0 - e[j]); }
        P[k] = p; H[k] = h;
        Q[k] = pairwise(e, m) / (double)m;                               /* np.mean */
    }
    double G[NCODE];
    double S = 0.0;
    for (int h = 0; h < n; h++) {                                       /* :140-143 */
        double non = 1.0;
        for (int a = 0; a < n; a++)
            if (a != h) non = non * P[a];
        G[h] = H[h] * non;
        glp[h] = G[h];
    }
    for (int h = 0; h < n; h++) S = S + G[h];                           /* :145 */
    if (S == 0) S = 1.0;                                                /* :146 */
    char refc = c->ref[pos];
    int nv = 0;
    for (int k = 0; k < n; k++) {                                       /* :148-185 */
        uint32_t ad = s->len[k];
        char allele = NIBBLE[s->code[k]];
        if (refc != allele && (int64_t)ad >= c->min_ad &&
            (double)ad / (double)c->depth[pos] >= c->ratio) {
            spo_variant v;
            memset(&v, 0, sizeof(v));
            v.start = pos;
            v.dp = (int32_t)c->depth[pos];
            v.ad = (int32_t)ad;
            v.ref = (uint8_t)refc;
            v.alt = (uint8_t)allele;
            v.gl_linear = G[k];
            if (G[k] != 0) { v.gl = log10(G[k]); v.pl = (int32_t)rint(-10.0 * v.gl); v.gl_zero = 0; }
            else { v.gl = 0; v.pl = 0; v.gl_zero = 1; }
            v.score = to_phred(1.0 - (G[k] / S));
            v.qual = Q[k];
            out[nv++] = v;
        }
    }
    return nv;
}

/* live_variant_caller.py:120-185 + utils.py:16-24; returns the number of variants.  Positions in
 * memory insertion order, evaluated in chunks (in parallel when threads > 1), emitted in order. */
int64_t spo_finalize(spo_ctx *c) {
    c->n_var = 0;
    enum { CHUNK = 65536 };
    spo_variant *buf = (spo_variant *)malloc((size_t)CHUNK * NCODE * sizeof(spo_variant));
    int *nv = (int *)malloc((size_t)CHUNK * sizeof(int));
    for (int64_t c0 = 0; c0 < c->n_ins; c0 += CHUNK) {
        int64_t c1 = c0 + CHUNK < c->n_ins ? c0 + CHUNK : c->n_ins;
#ifdef _OPENMP
#pragma omp parallel num_threads(g_threads)
#endif
        {
            double *eps = NULL;
            size_t eps_cap = 0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
            for (int64_t ii = c0; ii < c1; ii++)
                nv[ii - c0] = finalize_pos(c, c->ins[ii], &eps, &eps_cap, buf + (ii - c0) * NCODE);
            free(eps);
        }
        for (int64_t ii = c0; ii < c1; ii++)
            for (int k = 0; k < nv[ii - c0]; k++) push_var(c, buf + (ii - c0) * NCODE + k);
    }
    free(buf);
    free(nv);
    return c->n_var;
}

/* ---- accessors (ctypes) ---- */
int64_t spo_n_present(const spo_ctx *c) { return c->n_ins; }

/* per present position in dict insertion order: pos, depth, n_del, n_skip, n_alleles,
 * codes[16], counts[16] (by dict index), gl[16] (by dict index, NaN when not evaluated) */
void spo_memory(const spo_ctx *c, int64_t *pos, uint64_t *depth, uint64_t *n_del, uint64_t *n_skip,
                uint8_t *n_all, uint8_t *codes, uint32_t *counts, double *gl) {
    for (int64_t i = 0; i < c->n_ins; i++) {
        int64_t p = c->ins[i];
        const site_t *s = c->site[p];
        pos[i] = p;
        depth[i] = c->depth[p];
        n_del[i] = c->n_del[p];
        n_skip[i] = c->n_skip[p];
        n_all[i] = s->n_all;
        for (int k = 0; k < NCODE; k++) {
            codes[i * NCODE + k] = k < s->n_all ? s->code[k] : 0xFF;
            counts[i * NCODE + k] = k < s->n_all ? s->len[k] : 0;
            gl[i * NCODE + k] = c->gl[p * NCODE + k];
        }
    }
}

void spo_variants(const spo_ctx *c, spo_variant *out) { memcpy(out, c->var, (size_t)c->n_var * sizeof(spo_variant)); }
int spo_variant_size(void) { return (int)sizeof(spo_variant); }
