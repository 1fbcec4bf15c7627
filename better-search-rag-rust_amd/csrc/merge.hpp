// merge.hpp -- the root's merge of partial top-k lists (compute_global_top_k for a batch).
#pragma once

#include <stdint.h>

namespace bsr {

// n_lists partial lists per query, laid out [list][query][k_in] with counts [list][query]
// (the all-gather's receive layout and bsr_global_top_k's input layout).
struct ListsView {
    const uint64_t* idx;
    const float* dist;
    const uint32_t* count;
    uint32_t n_lists, n_queries, k_in;
    uint32_t count_of(uint32_t l, uint32_t q) const {
        const uint32_t c = count[(uint64_t)l * n_queries + q];
        return c < k_in ? c : k_in;
    }
    const uint64_t* idx_of(uint32_t l, uint32_t q) const { return idx + ((uint64_t)l * n_queries + q) * k_in; }
    const float* dist_of(uint32_t l, uint32_t q) const { return dist + ((uint64_t)l * n_queries + q) * k_in; }
};

// src/mpi_helpers/metrics.rs:141-171 for every query: rank-order concatenation, stable sort
// by distance, first top_k distinct indices.  Rows of out_* are [n_queries][k]; entries past
// out_count[q] are (~0, +inf).  A NaN distance returns BSR_E_NONFINITE (the reference panics).
int merge_top_k_lists(const ListsView& in, uint32_t n_queries, uint32_t k, uint64_t* out_idx, float* out_dist,
                      uint32_t* out_count);

}  // namespace bsr
