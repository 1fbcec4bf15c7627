/*
 * bsr_oracle.c -- CPU restatement of the better-search-rag-rust search hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see bsr_oracle.h): the checker for tests/, smoke() and the
 * CPU baseline of bench.py.  Never linked into or called by the product library.
 *
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math -fPIC -shared (oracle/Makefile).  On
 * x86-64 float arithmetic is SSE single precision, so every `*` and `+` below rounds to
 * f32 exactly as Rust's (which never contracts to FMA and never reorders a float sum).
 *
 * Each function cites the reference line it restates.  Parity status: see the header
 * ("parity unpinned" against the reference binary; pinned by hand-derived known answers
 * and an independent numpy restatement).
 */
#include "bsr_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* src/metrics.rs:7-19 -- `(a[i] - b[i]).abs() > 1e-10` on f32 (the literal is rounded to
 * f32 by Rust's type inference). */
static int vectors_are_identical(const float* a, size_t la, const float* b, size_t lb) {
    if (la != lb) return 0;
    const float tol = 1e-10f;
    for (size_t i = 0; i < la; ++i) {
        float d = a[i] - b[i];
        if (fabsf(d) > tol) return 0;
    }
    return 1;
}

/* Rust's `impl Sum for f32` folds from -0.0 in recent std (older: +0.0).  The two differ
 * only when every term is -0.0, which cannot change a returned distance (a +-0 dot gives
 * s = +-0 and 1 - s = 1; a sum of squares is never -0.0 unless empty).  We follow -0.0. */
static float seq_dot(const float* a, const float* b, size_t n) {
    float acc = -0.0f;
    for (size_t i = 0; i < n; ++i) {
        float p = a[i] * b[i]; /* separate rounding: no FMA (-ffp-contract=off) */
        acc = acc + p;
    }
    return acc;
}

/* src/metrics.rs:143-165 */
float bsr_oracle_cosine_distance(const float* a, size_t len_a, const float* b, size_t len_b) {
    if (len_a != len_b || len_a == 0) return 1.0f;                    /* :144-146 */
    if (vectors_are_identical(a, len_a, b, len_b)) return 0.0f;       /* :149-151 */
    float dot = seq_dot(a, b, len_a);                                  /* :153 */
    float mag_a = sqrtf(seq_dot(a, a, len_a));                         /* :154 */
    float mag_b = sqrtf(seq_dot(b, b, len_b));                         /* :155 */
    if (mag_a == 0.0f || mag_b == 0.0f) return 1.0f;                  /* :157-159 */
    float denom = mag_a * mag_b;
    float s = dot / denom;                                             /* :161 */
    s = fmaxf(s, -1.0f);                                               /* :162 .max(-1.0) */
    s = fminf(s, 1.0f);                                                /*      .min(1.0)  */
    return 1.0f - s;                                                   /* :164 */
}

/* src/mpi_helpers/load_balance.rs:24-42.  `end` may be < `start` (e.g. count=5,size=4,
 * rank=3); the reference then slices an empty block, which callers here treat as
 * [start, max(start,end)) clipped to count. */
void bsr_oracle_interval_by_rank(int32_t rank, int32_t size, uint64_t count,
                                 uint64_t* start_index, uint64_t* end_index) {
    uint64_t per_rank = ((uint64_t)size > count) ? 1 : (count + (uint64_t)size - 1) / (uint64_t)size;
    uint64_t start = per_rank * (uint64_t)rank;
    uint64_t end;
    if (rank == size - 1) {
        end = count;
    } else {
        end = start + per_rank;
        if (end > count) end = count;
    }
    *start_index = start;
    *end_index = end;
}

typedef struct {
    uint64_t idx;
    float dist;
} pair_t;

/* Stable merge sort by `dist` only, as Rust's `sort_by(|(_, a), (_, b)| a.partial_cmp(b))`
 * (src/mpi_helpers/metrics.rs:47,153).  Equal distances keep their input order. */
static void stable_sort_by_dist(pair_t* v, size_t n) {
    if (n < 2) return;
    pair_t* tmp = (pair_t*)malloc(n * sizeof(pair_t));
    for (size_t width = 1; width < n; width *= 2) {
        for (size_t lo = 0; lo < n; lo += 2 * width) {
            size_t mid = lo + width < n ? lo + width : n;
            size_t hi = lo + 2 * width < n ? lo + 2 * width : n;
            size_t i = lo, j = mid, o = lo;
            while (i < mid && j < hi) {
                if (v[j].dist < v[i].dist) tmp[o++] = v[j++]; /* take right only if strictly less */
                else tmp[o++] = v[i++];
            }
            while (i < mid) tmp[o++] = v[i++];
            while (j < hi) tmp[o++] = v[j++];
        }
        memcpy(v, tmp, n * sizeof(pair_t));
    }
    free(tmp);
}

static int has_nan(const pair_t* v, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (isnan(v[i].dist)) return 1;
    return 0;
}

/* src/mpi_helpers/metrics.rs:16-53 */
size_t bsr_oracle_local_top_k(const float* rows, uint64_t n_rows, uint32_t dim,
                              int32_t rank, int32_t size, uint32_t top_k,
                              const float* query, uint64_t* out_idx, float* out_dist) {
    uint64_t start, end;
    bsr_oracle_interval_by_rank(rank, size, n_rows, &start, &end); /* :27 */
    if (start >= n_rows || end <= start) return 0;                 /* empty slice, §8a-3 */
    size_t cnt = (size_t)(end - start);
    pair_t* d = (pair_t*)malloc(cnt * sizeof(pair_t));
    for (size_t i = 0; i < cnt; ++i) {                              /* :36-44 */
        d[i].idx = start + i;
        d[i].dist = bsr_oracle_cosine_distance(rows + (start + i) * (uint64_t)dim, dim, query, dim);
    }
    if (has_nan(d, cnt)) { free(d); return (size_t)-1; }          /* reference panics */
    stable_sort_by_dist(d, cnt);                                    /* :47 */
    size_t keep = cnt > top_k ? top_k : cnt;                        /* :48-50 */
    for (size_t i = 0; i < keep; ++i) { out_idx[i] = d[i].idx; out_dist[i] = d[i].dist; }
    free(d);
    return keep;
}

/* src/mpi_helpers/metrics.rs:141-171 */
size_t bsr_oracle_global_top_k(const uint64_t* idx, const float* dist, size_t n,
                               uint32_t top_k, uint64_t* out_idx, float* out_dist) {
    if (n == 0) return 0;
    pair_t* v = (pair_t*)malloc(n * sizeof(pair_t));
    for (size_t i = 0; i < n; ++i) { v[i].idx = idx[i]; v[i].dist = dist[i]; } /* :147-150 */
    if (has_nan(v, n)) { free(v); return (size_t)-1; }
    stable_sort_by_dist(v, n);                                                 /* :153 */
    size_t out = 0;
    for (size_t i = 0; i < n && out < top_k; ++i) {                            /* :156-168 */
        int seen = 0;
        for (size_t j = 0; j < out; ++j)
            if (out_idx[j] == v[i].idx) { seen = 1; break; }
        if (seen) continue;
        out_idx[out] = v[i].idx;
        out_dist[out] = v[i].dist;
        ++out;
    }
    free(v);
    return out;
}

typedef struct {
    const float* rows;
    uint64_t n_rows;
    uint32_t dim;
    int32_t size;
    uint32_t top_k;
    const float* queries;
    uint32_t n_queries;
    int32_t first_rank, rank_stride;
    uint64_t* part_idx;   /* [size][n_queries][top_k] */
    float* part_dist;
    size_t* part_cnt;     /* [size][n_queries] */
} job_t;

static void* rank_worker(void* p) {
    job_t* j = (job_t*)p;
    for (int32_t r = j->first_rank; r < j->size; r += j->rank_stride) {
        for (uint32_t q = 0; q < j->n_queries; ++q) {
            size_t off = ((size_t)r * j->n_queries + q) * j->top_k;
            j->part_cnt[(size_t)r * j->n_queries + q] = bsr_oracle_local_top_k(
                j->rows, j->n_rows, j->dim, r, j->size, j->top_k,
                j->queries + (size_t)q * j->dim, j->part_idx + off, j->part_dist + off);
        }
    }
    return NULL;
}

void bsr_oracle_parallel_top_k_batch(const float* rows, uint64_t n_rows, uint32_t dim,
                                     int32_t size, uint32_t top_k, const float* queries,
                                     uint32_t n_queries, uint64_t* out_idx, float* out_dist,
                                     uint32_t* out_count, int32_t threads) {
    if (size < 1) size = 1;
    if (threads < 1) threads = 1;
    if (threads > size) threads = size;
    size_t slots = (size_t)size * n_queries * (top_k ? top_k : 1);
    uint64_t* pidx = (uint64_t*)malloc(slots * sizeof(uint64_t));
    float* pdist = (float*)malloc(slots * sizeof(float));
    size_t* pcnt = (size_t*)calloc((size_t)size * n_queries, sizeof(size_t));
    job_t* jobs = (job_t*)malloc((size_t)threads * sizeof(job_t));
    pthread_t* th = (pthread_t*)malloc((size_t)threads * sizeof(pthread_t));
    for (int t = 0; t < threads; ++t) {
        job_t j = {rows, n_rows, dim, size, top_k, queries, n_queries, t, threads, pidx, pdist, pcnt};
        jobs[t] = j;
        if (threads == 1) rank_worker(&jobs[t]);
        else pthread_create(&th[t], NULL, rank_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);

    /* gather_top_k_results: concatenate rank lists in rank order (:86-126). */
    uint64_t* gidx = (uint64_t*)malloc(slots * sizeof(uint64_t));
    float* gdist = (float*)malloc(slots * sizeof(float));
    for (uint32_t q = 0; q < n_queries; ++q) {
        size_t n = 0;
        int nan = 0;
        for (int32_t r = 0; r < size; ++r) {
            size_t c = pcnt[(size_t)r * n_queries + q];
            if (c == (size_t)-1) { nan = 1; continue; }
            size_t off = ((size_t)r * n_queries + q) * top_k;
            memcpy(gidx + n, pidx + off, c * sizeof(uint64_t));
            memcpy(gdist + n, pdist + off, c * sizeof(float));
            n += c;
        }
        size_t got = nan ? (size_t)-1
                         : bsr_oracle_global_top_k(gidx, gdist, n, top_k,
                                                   out_idx + (size_t)q * top_k,
                                                   out_dist + (size_t)q * top_k);
        out_count[q] = (got == (size_t)-1) ? 0xFFFFFFFFu : (uint32_t)got;
    }
    free(gidx); free(gdist); free(pidx); free(pdist); free(pcnt); free(jobs); free(th);
}

size_t bsr_oracle_parallel_top_k(const float* rows, uint64_t n_rows, uint32_t dim,
                                 int32_t size, uint32_t top_k, const float* query,
                                 uint64_t* out_idx, float* out_dist, int32_t threads) {
    uint32_t cnt = 0;
    bsr_oracle_parallel_top_k_batch(rows, n_rows, dim, size, top_k, query, 1, out_idx,
                                    out_dist, &cnt, threads);
    return cnt == 0xFFFFFFFFu ? (size_t)-1 : cnt;
}
