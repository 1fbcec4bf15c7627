/*
 * bsr_oracle.h -- CPU restatement of the better-search-rag-rust search hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (better-search-rag-rust_amd/) links,
 * loads or calls this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, as the checker / the timed CPU baseline.
 *
 * Parity status: the reference is Rust and cannot be built or run in this image (no
 * cargo/rustc, crates not vendored, no MPI), and none of its own tests cover this path
 * (SURVEY.md F6, §8c).  This restatement is therefore pinned by (1) hand-derived
 * known-answer vectors that follow directly from the reference source
 * (tests/golden/known_answers.json), and (2) an independent numpy restatement
 * (tests/oracle_np.py) that must agree bit-for-bit.  No reference-executed fixture
 * exists: "parity unpinned" against the reference binary itself.
 */
#ifndef BSR_ORACLE_H
#define BSR_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/metrics.rs:143-165 (+ vectors_are_identical, src/metrics.rs:7-19).  a = stored row,
 * b = query (src/mpi_helpers/metrics.rs:42). */
float bsr_oracle_cosine_distance(const float* a, size_t len_a, const float* b, size_t len_b);

/* src/mpi_helpers/load_balance.rs:24-42 (release-mode semantics; a start past end is an
 * empty block). */
void bsr_oracle_interval_by_rank(int32_t rank, int32_t size, uint64_t count,
                                 uint64_t* start_index, uint64_t* end_index);

/* src/mpi_helpers/metrics.rs:16-53 for one query: the rank's block of a row-major
 * n_rows x dim slab, stable sort by distance, truncate to top_k.  Returns the length. */
size_t bsr_oracle_local_top_k(const float* rows, uint64_t n_rows, uint32_t dim,
                              int32_t rank, int32_t size, uint32_t top_k,
                              const float* query, uint64_t* out_idx, float* out_dist);

/* src/mpi_helpers/metrics.rs:141-171: stable sort by distance, dedupe by index, keep
 * top_k.  Returns the length.  Returns (size_t)-1 when a distance is NaN (the reference
 * panics in partial_cmp().unwrap()). */
size_t bsr_oracle_global_top_k(const uint64_t* idx, const float* dist, size_t n,
                               uint32_t top_k, uint64_t* out_idx, float* out_dist);

/* src/mpi_helpers/metrics.rs:174-206 with `size` simulated ranks: each rank runs
 * local_top_k on its block, lists are concatenated in rank order (gather_top_k_results,
 * :56-138), then global_top_k.  `threads` > 1 runs the ranks on that many POSIX threads
 * (the mpiexec analogue used for the CPU baseline). */
size_t bsr_oracle_parallel_top_k(const float* rows, uint64_t n_rows, uint32_t dim,
                                 int32_t size, uint32_t top_k, const float* query,
                                 uint64_t* out_idx, float* out_dist, int32_t threads);

/* Many queries: query q's result goes to out_idx[q*top_k ..], out_count[q]. */
void bsr_oracle_parallel_top_k_batch(const float* rows, uint64_t n_rows, uint32_t dim,
                                     int32_t size, uint32_t top_k, const float* queries,
                                     uint32_t n_queries, uint64_t* out_idx, float* out_dist,
                                     uint32_t* out_count, int32_t threads);

#ifdef __cplusplus
}
#endif
#endif
