/*
 * bsr.h -- C ABI of the MI355X-native search engine for the better-search-rag-rust hot path:
 * block-distributed exact cosine-distance scan + global top-k reduction.
 *
 * One process per GPU (the reference's one process per MPI rank).  Every entry point
 * returns 0 (BSR_OK) or a negative bsr_status (BSR_PARTIAL, positive, only from the
 * parallel search's root: see there); bsr_last_error() gives a thread-local message.  No
 * C++ exception or panic crosses this boundary.  Plain pointers only: query, row and
 * output pointers may be host or device (hipMalloc) memory, detected per call.
 * Device inputs: bsr_index_load / bsr_index_append synchronize the device before reading
 * device rows (one-time calls).  The search entry points do not: the library's streams are
 * blocking streams, so their work waits for work issued before the call on the legacy
 * default (NULL) stream (e.g. PyTorch's default stream); queries produced on any other
 * stream must be complete (synchronized) first.
 *
 * Each entry point names the reference item it replaces (paths relative to the reference
 * repository nichmorgan/better-search-rag-rust):
 *   bsr_cosine_distance               src/metrics.rs:143-165 (cosine_distance)
 *   bsr_interval_by_rank              src/mpi_helpers/load_balance.rs:24-42 (interval_by_rank)
 *   bsr_index_*                       src/vectorstore/polars.rs:79-91,121-169,243-246
 *                                     (PolarsVectorstore::new/get_many/get/get_count: the
 *                                     rank's corpus slab, resident in HBM)
 *   bsr_local_top_k                   src/mpi_helpers/metrics.rs:16-53 (compute_local_top_k)
 *   bsr_gather_top_k                  src/mpi_helpers/metrics.rs:56-138 (gather_top_k_results)
 *   bsr_global_top_k                  src/mpi_helpers/metrics.rs:141-171 (compute_global_top_k)
 *   bsr_gather_global_top_k           src/mpi_helpers/metrics.rs:56-171 (a-4 + a-5: the
 *                                     exchange and root merge of a-6, :194-202)
 *   bsr_parallel_top_k_similarity_search
 *                                     src/mpi_helpers/metrics.rs:174-206
 *                                     (parallel_top_k_similarity_search)
 *   bsr_broadcast                     src/main.rs:123-125 (broadcast_into of the query)
 *   bsr_allgather_bytes               src/mpi_helpers/benchmark.rs:131-293 (timing gather)
 *
 * Results are bit-identical to the reference's: indices in (distance asc, index asc)
 * order, each distance the exact f32 the reference computes (sequential f32 sums, no FMA,
 * correctly rounded sqrt/div, identical-vector shortcut).  Deviations (documented in
 * DESIGN.md): non-finite inputs return BSR_E_NONFINITE where the reference panics; a query
 * whose length differs from the index dimension returns BSR_E_DIM where the reference
 * scores every row 1.0.
 */
#ifndef BSR_H
#define BSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    BSR_PARTIAL = 1,      /* parallel search root: result valid but its own block is missing */
    BSR_OK = 0,
    BSR_E_INVALID = -1,   /* bad argument / null pointer / k out of range */
    BSR_E_NONFINITE = -2, /* NaN or Inf in a query or row (the reference panics) */
    BSR_E_HIP = -3,       /* HIP runtime error (message in bsr_last_error) */
    BSR_E_NOMEM = -4,     /* device allocation failed */
    BSR_E_RCCL = -5,      /* RCCL error */
    BSR_E_DIM = -6,       /* query length != index dimension */
    BSR_E_STATE = -7,     /* call out of order (e.g. search before load) */
    BSR_E_NODEVICE = -8   /* no HIP device visible: the engine has no CPU fallback */
} bsr_status;

typedef enum { BSR_F32 = 0, BSR_BF16 = 1 } bsr_dtype;

typedef struct {
    uint32_t dim;    /* embedding length (768 in the reference, src/main.rs:117) */
    uint32_t dtype;  /* bsr_dtype of the stored rows */
    uint32_t max_k;  /* largest top_k a search may ask for (<= BSR_MAX_K) */
    uint32_t flags;  /* BSR_FLAG_* */
    int32_t device;  /* HIP device ordinal; -1 = current device */
} bsr_config;

#define BSR_MAX_K 256u
#define BSR_FLAG_EXACT_ONLY 1u /* never use the MFMA candidate stage (always full exact scan) */
#define BSR_FLAG_PROFILE 2u    /* record per-kernel HIP events (bsr_index_profile) */
/* The MFMA candidate filter's operand is int8 (v_mfma_i32_16x16x64_i8 for rows of up to 768
 * bytes, v_mfma_i32_32x32x32_i8 otherwise; per-32-row-block and per-query scales, certified
 * with a measured Cauchy-Schwarz bound).  Every returned list is exact; the filter only
 * decides how much exact work a query needs.  The bf16 filter operand of earlier rounds is
 * retired: bsr_index_create with this flag returns BSR_E_INVALID (a bf16 CORPUS, cfg.dtype =
 * BSR_BF16, is served on the int8 filter). */
#define BSR_FLAG_FILTER_BF16 4u

/* Mirrors RankInterval {start_index, end_index} (load_balance.rs:8-17). end < start means
 * an empty block, as in the reference's release build. */
typedef struct {
    uint64_t start_index;
    uint64_t end_index;
} bsr_rank_interval;

typedef struct bsr_index bsr_index; /* one rank's corpus shard, resident in HBM */
typedef struct bsr_comm bsr_comm;   /* the rank group: RCCL (one GPU each), a host transport or a loopback */

/* Per-search statistics of the last bsr_local_top_k on an index. */
typedef struct {
    uint32_t n_queries;
    uint32_t n_exact_direct;   /* queries answered by the full exact scan by design */
    uint32_t n_fallback;       /* queries whose MFMA candidate set failed certification */
    uint32_t n_candidates;     /* k' candidates rescored per query */
    uint64_t n_emitted;        /* candidates emitted by the MFMA filter (all queries) */
    uint32_t filter_op;        /* 0 = int8 filter (the only operand since round 4) */
    float row_ebound;          /* max over rows of ||a/|a| - s q||_2 (int8 quantisation) */
    uint32_t n_rescued;        /* queries certified by the second chance (all emitted rows) */
    uint32_t graph_replay;     /* 1: the search replayed a captured hipGraph (every filtered batch
                                  from the second search of its shape on, at profile level 0) */
    uint32_t search_path;      /* BSR_PATH_* bits: which branches the last search took */
} bsr_search_stats;

/* bsr_search_stats.search_path: which branches the last search took (bits 1-16: the parallel
 * search; 32, 64: a batch of <= 16 queries on the self-thresholded path) */
#define BSR_PATH_COLLECTIVE 1u   /* the collectives ran (size > 1, or BSR_FORCE_COLLECTIVES=1) */
#define BSR_PATH_GLOBAL_TAU 2u   /* the global-threshold search */
#define BSR_PATH_DIRECT_OUT 4u   /* root: merged rows written straight into coherent pinned outputs */
#define BSR_PATH_DEVICE_MERGE 8u /* root of the standard path: the device merge (k_merge_lists) */
#define BSR_PATH_FALLBACK 16u    /* global threshold: uncertified queries took the collective fallback */
#define BSR_PATH_SKINNY_TOP 32u  /* no sample pass: every filter wave's 4 best keys per query */
#define BSR_PATH_TOP_RERUN 64u   /* ... left a query uncertified: the batch ran again, thresholded */

/* Per-kernel timing (BSR_FLAG_PROFILE): cumulative device milliseconds and launch counts
 * since the last reset, measured with hipEvents on the index's stream. */
typedef struct {
    double gemm_emit_ms;  uint64_t gemm_emit_launches;  /* dominant kernel */
    double gemm_sample_ms; uint64_t gemm_sample_launches;
    double select_ms;     uint64_t select_launches;
    double rescore_ms;    uint64_t rescore_launches;
    double scan_ms;       uint64_t scan_launches;
    double search_ms;     uint64_t searches;             /* whole bsr_local_top_k */
} bsr_profile;

/* ---- errors / device -------------------------------------------------------------- */
const char* bsr_last_error(void);
const char* bsr_status_string(int status);
int bsr_device_count(int* out_count);
const char* bsr_version(void);

/* ---- a-1: src/metrics.rs:143-165, one pair, computed on the GPU ------------------ */
int bsr_cosine_distance(const float* a, uint32_t len_a, const float* b, uint32_t len_b,
                        float* out);

/* ---- a-3: src/mpi_helpers/load_balance.rs:24-42 ---------------------------------- */
int bsr_interval_by_rank(int32_t rank, int32_t size, uint64_t count, bsr_rank_interval* out);

/* ---- the rank's shard (read side of src/vectorstore/polars.rs) ------------------- */
int bsr_index_create(const bsr_config* cfg, bsr_index** out);
void bsr_index_destroy(bsr_index* ix);
/* Copy n_rows row-major rows (f32, or bf16 bits when cfg.dtype == BSR_BF16) into HBM and
 * precompute per-row state.  global_offset is the global index of local row 0
 * (interval_by_rank(rank,size,N).start_index).  Replaces any previous contents.  Device rows
 * may come from any stream: load and append synchronize the device before reading them. */
int bsr_index_load(bsr_index* ix, const void* rows, uint64_t n_rows, uint64_t global_offset);
/* Append rows after the current ones (PolarsVectorstore::append_many, polars.rs:101-119). */
int bsr_index_append(bsr_index* ix, const void* rows, uint64_t n_rows);
int bsr_index_count(const bsr_index* ix, uint64_t* out);                /* get_count */
int bsr_index_dim(const bsr_index* ix, uint32_t* out);                  /* row length */
int bsr_index_global_offset(const bsr_index* ix, uint64_t* out);
/* Copy `count` rows starting at local row `offset` into out (f32, host or device):
 * PolarsVectorstore::get_many(SliceArgs{offset,length}) / get (polars.rs:121-169). */
int bsr_index_get_many(const bsr_index* ix, uint64_t offset, uint64_t count, float* out);

/* ---- a-2: compute_local_top_k for n_queries queries (row-major [n_queries][dim] f32).
 * out_idx/out_dist are [n_queries][k]; row q holds out_count[q] = min(k, n_rows) entries
 * in (distance asc, global index asc) order.  Indices are global (offset added). ------ */
int bsr_local_top_k(bsr_index* ix, const float* queries, uint32_t n_queries, uint32_t k,
                    uint64_t* out_idx, float* out_dist, uint32_t* out_count);

/* ---- a-5: compute_global_top_k over n_lists per-rank lists, for n_queries queries.
 * Input list l of query q: idx[(l*n_queries+q)*k_in ..] with count[l*n_queries+q]
 * entries.  Rank-order concatenation + stable sort by distance + dedupe, keep k.
 * Host arrays: merged on the host (threads over queries).  Every array in device memory
 * (n_lists <= 64, n_lists * k_in <= 1024, k <= 256): merged on the GPU, one wave per query
 * (the RCCL path's root merge).  Rows past out_count[q] are (~0, +inf). -------------- */
int bsr_global_top_k(const uint64_t* idx, const float* dist, const uint32_t* count,
                     uint32_t n_lists, uint32_t n_queries, uint32_t k_in, uint32_t k,
                     uint64_t* out_idx, float* out_dist, uint32_t* out_count);

/* ---- communicator (replaces the MPI world; RCCL over xGMI) ----------------------- */
#define BSR_UNIQUE_ID_BYTES 128
int bsr_comm_unique_id(uint8_t out_id[BSR_UNIQUE_ID_BYTES]); /* on rank 0; broadcast it */
int bsr_comm_init(const uint8_t id[BSR_UNIQUE_ID_BYTES], int32_t rank, int32_t size,
                  int32_t device, bsr_comm** out);
void bsr_comm_destroy(bsr_comm* comm);
int bsr_comm_rank(const bsr_comm* comm, int32_t* rank, int32_t* size);

/* Host transport for bsr_comm_init_host: an all-gather of `bytes` bytes from every rank
 * into recv (size * bytes, rank order), called collectively by every rank.  Returns 0 on
 * success.  Lets a caller run the exchange over its own transport (MPI, gloo, a test
 * harness) with the same gather + merge code as the RCCL path. */
typedef int (*bsr_host_allgather_fn)(const void* send, void* recv, uint64_t bytes, void* user);
int bsr_comm_init_host(int32_t rank, int32_t size, bsr_host_allgather_fn fn, void* user,
                       bsr_comm** out);

/* Loopback communicator (measurement and tests, not a transport): ONE process on one GPU acting
 * as rank `rank` of `size`.  Every all-gather is emulated by one device kernel enqueued exactly
 * where ncclAllGather would be (same stream, no host wait), so a parallel search runs the RCCL
 * path's enqueue-only control flow and its per-rank device timeline.  Without a script
 * (n_calls = 0) each all-gather gives every slot this rank's own contribution.  With one, the
 * all-gathers of each bsr_parallel_top_k_similarity_search replay, in order, the contributions
 * recorded in a real size-rank run of the same batch (call i: call_bytes[i] bytes per rank,
 * script holds its [size][call_bytes[i]] receive buffer, calls concatenated); this rank's slot
 * is always its live contribution, and a call that does not match the recording (another
 * size, past its end) replicates from then on in that search.  Broadcasts are no-ops. */
int bsr_comm_init_loopback(int32_t rank, int32_t size, int32_t device, uint32_t n_calls,
                           const uint64_t* call_bytes, const void* script, bsr_comm** out);
/* All-gathers replayed from the script and calls that missed it, since creation. */
int bsr_comm_loopback_stats(const bsr_comm* comm, uint64_t* replayed, uint64_t* missed);

/* ---- a-4: gather_top_k_results.  Every rank passes its [n_queries][k] local lists;
 * the root (rank 0) receives [size][n_queries][k] lists + counts in rank order
 * (host buffers, may be NULL on non-root ranks).  Collective: every rank calls it. ---- */
int bsr_gather_top_k(bsr_comm* comm, const uint64_t* local_idx, const float* local_dist,
                     const uint32_t* local_count, uint32_t n_queries, uint32_t k,
                     uint64_t* root_idx, float* root_dist, uint32_t* root_count);

/* ---- a-4 + a-5 composed (the exchange step of a-6): every rank passes its
 * [n_queries][k] local lists (host or device; all three NULL = an empty contribution, what
 * the reference sends after a local error, src/mpi_helpers/metrics.rs:185-191); the root
 * gets the global top-k (rank-order concatenation, stable sort by distance, dedupe by
 * index, :141-171) in out_*; other ranks get out_count[q] = 0.  Collective. ---------- */
int bsr_gather_global_top_k(bsr_comm* comm, const uint64_t* local_idx, const float* local_dist,
                            const uint32_t* local_count, uint32_t n_queries, uint32_t k,
                            uint64_t* out_idx, float* out_dist, uint32_t* out_count);

/* ---- a-6: parallel_top_k_similarity_search (src/mpi_helpers/metrics.rs:174-206) for a batch
 * of n_queries queries.  The root (rank 0) gets the global top-k in out_* (the reference's
 * Some(global_top_k)); other ranks get out_count[q] = 0 (its None).  comm may be NULL for a
 * single-rank run (the local lists are the result).  Collective: every rank calls it.
 *
 * With size > 1 every rank first all-gathers a 32-byte header {n_queries, k, local status,
 * magic, eligible for the global threshold, shard rows (2 words), 0}.  Ranks that disagree on
 * n_queries or k all return BSR_E_INVALID and no lists move.  Then one of two paths, the same
 * on every rank:
 *   - the global-threshold path (every rank eligible: n_queries > 16, k <= 200, a shard of
 *     more rows than one query's candidate list, size <= 64, size * k <= 1024; the library
 *     setting BSR_GLOBAL_TAU=0 turns it off): every rank all-gathers its best sample keys,
 *     emits against the threshold the whole corpus's sample selects, rescores every row it
 *     emitted exactly and all-gathers its packed result (lists, status words, per-query
 *     exclusion bounds).  EVERY rank merges the gathered lists on its GPU and certifies each
 *     merged list against every rank's bound; the uncertified queries (usually none) take the
 *     standard path below, collectively, and replace the root's rows;
 *   - the standard path: each rank's certified local top-k (bsr_local_top_k), the all-gather
 *     of the [n_queries][k] lists and the root's merge on its GPU (bsr_gather_global_top_k).
 * A rank whose local step fails (bad arguments, device mismatch, a failed search) still takes
 * part in every collective with an empty list (:185-191): a non-root rank then returns its
 * error; the root returns BSR_PARTIAL with the other ranks' global top-k in out_* (the
 * reference's root still returns Some(..), :199-202) and the message in bsr_last_error().
 * Over RCCL every step is enqueued on the device with one host wait at the end; over a host
 * transport each all-gather is a host round trip. ------------------------------------------ */
int bsr_parallel_top_k_similarity_search(bsr_comm* comm, bsr_index* ix, const float* queries,
                                         uint32_t n_queries, uint32_t k, uint64_t* out_idx,
                                         float* out_dist, uint32_t* out_count);

/* ---- pinned host buffers for results (round 5): coherent (fine-grained) pinned host memory.  Root
 * outputs of bsr_parallel_top_k_similarity_search in such memory are written by the GPU directly
 * on the global-threshold path (no staging copy after the search); any other host memory works
 * everywhere, through a copy. -------------------------------------------------------------- */
int bsr_host_alloc(uint64_t bytes, void** out);
void bsr_host_free(void* p);

/* ---- driver collectives: src/main.rs:123-125 (process_at_rank(ROOT).broadcast_into of the
 * query) and the timing gather of src/mpi_helpers/benchmark.rs:131-293.  Host or device
 * buffers; collective over the comm (RCCL or host transport). ------------------------ */
int bsr_broadcast(bsr_comm* comm, void* buf, uint64_t bytes, int32_t root);
int bsr_allgather_bytes(bsr_comm* comm, const void* send, void* recv, uint64_t bytes);

/* ---- diagnostics ------------------------------------------------------------------ */
int bsr_index_last_stats(const bsr_index* ix, bsr_search_stats* out);
int bsr_index_profile(bsr_index* ix, bsr_profile* out, int reset);
/* Which stages of a BSR_FLAG_PROFILE index record HIP events: 0 = none (the product path:
 * filtered batches replay a captured hipGraph), 1 = the filter / scan kernels only, 2 = every
 * stage (the default).  At levels 1 and 2 a search launches its kernels directly, with the
 * events recorded on the stream around them (how kernel durations are timed). */
int bsr_index_set_profile(bsr_index* ix, int level);

/* ---- synthetic data (bench / tests): U(-1,1) f32 from a counter-based hash of
 * (seed, global element index), written on the device: value(row, col) for rows
 * [row0, row0+n_rows).  Identical on every rank and GPU. --------------------------- */
int bsr_synth_uniform(float* dev_out, uint64_t row0, uint64_t n_rows, uint32_t dim,
                      uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif /* BSR_H */
