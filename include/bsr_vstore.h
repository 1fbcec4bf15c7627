/*
 * bsr_vstore.h -- C ABI of the vector-store adapter: the reference's
 * parquet vector store, read and written natively (Apache Arrow C++ / Parquet), feeding the
 * rank's corpus block straight into a bsr_index.
 *
 * Mirrors, item for item (paths relative to nichmorgan/better-search-rag-rust):
 *   bsr_vstore_open          PolarsVectorstore::new + read_parquet  src/vectorstore/polars.rs:50-91
 *   bsr_vstore_get_count     PolarsVectorstore::get_count           src/vectorstore/polars.rs:243-246
 *   bsr_vstore_get_many      PolarsVectorstore::get_many            src/vectorstore/polars.rs:121-156
 *   bsr_vstore_get           PolarsVectorstore::get                 src/vectorstore/polars.rs:158-169
 *   bsr_vstore_append_many   PolarsVectorstore::append/append_many  src/vectorstore/polars.rs:97-119
 *   bsr_vstore_persist       PolarsVectorstore::persist             src/vectorstore/polars.rs:183-241
 *   bsr_vstore_reload        PolarsVectorstore::reload              src/vectorstore/polars.rs:171-181
 *   bsr_vstore_reset         PolarsVectorstore::reset               src/vectorstore/polars.rs:93-95
 *   bsr_vstore_*_path        get_global_vstore / get_local_vstore   src/mpi_helpers/vectorstore.rs:5-20
 *   bsr_index_load_vstore    the read half of compute_local_top_k   src/mpi_helpers/metrics.rs:23-33
 *
 * File format: one column "embeddings" of List(Float32) (polars.rs:17-37).  Files written by
 * polars (or pyarrow) are read; files written here are readable by polars.  Row semantics
 * follow the reference: get_count counts every row (null rows included); get_many slices
 * with polars' DataFrame::slice rules (a negative offset counts from the end, the length is
 * clamped), drops null rows and skips null elements inside a row (filter_map + flatten).
 * Every call returns 0 or a negative bsr_status (bsr.h); bsr_last_error() has the message.
 */
#ifndef BSR_VSTORE_H
#define BSR_VSTORE_H

#include <stddef.h>
#include <stdint.h>

#include "bsr.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bsr_vstore bsr_vstore;

/* empty != 0: an empty in-memory store bound to `path` (nothing read or written).
 * empty == 0: read `path`; a missing file is created (parent directories too) holding an
 * empty "embeddings" column, as read_parquet does. */
int bsr_vstore_open(const char* path, int empty, bsr_vstore** out);
void bsr_vstore_close(bsr_vstore* vs);
const char* bsr_vstore_path(const bsr_vstore* vs);

int bsr_vstore_get_count(const bsr_vstore* vs, uint64_t* out);

/* Rows of DataFrame::slice(offset, length) (null rows dropped, null elements skipped),
 * written back to back into `out` (capacity in floats); row_len[i] receives each row's
 * length (capacity `len_capacity` rows).  *out_rows / *out_floats: rows / floats written.
 * BSR_E_INVALID if a capacity is too small (nothing is partially reported as success).
 * A caller that only needs the sizes passes out = NULL and row_len = NULL. */
int bsr_vstore_get_many(const bsr_vstore* vs, int64_t offset, uint64_t length, float* out,
                        uint64_t out_capacity, uint32_t* row_len, uint64_t len_capacity,
                        uint64_t* out_rows, uint64_t* out_floats);
/* The same slice as a dense [rows][dim] f32 slab; BSR_E_DIM if a returned row's length is
 * not dim.  out may be host or device memory (hipMemcpy'd when device). */
int bsr_vstore_read_slab(const bsr_vstore* vs, int64_t offset, uint64_t length, uint32_t dim,
                         float* out, uint64_t capacity_rows, uint64_t* out_rows);
/* get(index): BSR_E_INVALID ("Index not found") when the slice has no row. */
int bsr_vstore_get(const bsr_vstore* vs, uint64_t index, float* out, uint32_t capacity,
                   uint32_t* out_len);

int bsr_vstore_append_many(bsr_vstore* vs, const float* rows, uint64_t n_rows, uint32_t dim);
int bsr_vstore_persist(bsr_vstore* vs);
/* Re-read the file; an empty (or invalid) file is an error unless force != 0. */
int bsr_vstore_reload(bsr_vstore* vs, int force);
int bsr_vstore_reset(bsr_vstore* vs);

/* <dir>/global.parquet, <dir>/rank_{rank}.parquet; BSR_E_INVALID if cap is too small. */
int bsr_vstore_global_path(const char* dir, char* out, size_t cap);
int bsr_vstore_local_path(const char* dir, int32_t rank, char* out, size_t cap);

/* Load this rank's block of the store into the index: interval_by_rank(rank, size,
 * get_count) (an empty block gives an empty shard), get_many of that block, then
 * bsr_index_load with global_offset = the block start -- exactly the rows the reference's
 * rank scans.  The block must be dense (every row length == the index dimension). */
int bsr_index_load_vstore(bsr_index* ix, const bsr_vstore* vs, int32_t rank, int32_t size);

#ifdef __cplusplus
}
#endif
#endif /* BSR_VSTORE_H */
