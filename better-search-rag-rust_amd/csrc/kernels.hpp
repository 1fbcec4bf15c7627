// kernels.hpp -- host-side launchers for the gfx950 kernels in kernels.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bsr {

// Layout constants shared by the host orchestration and the kernels.
constexpr uint32_t kLdAlign = 64;      // f32/bf16 row leading dimension multiple (elements)
constexpr uint32_t kRowPad = 256;      // rows are padded to a multiple of this (zero rows)
constexpr uint32_t kGemmBM = 128;      // MFMA filter tile: corpus rows
constexpr uint32_t kGemmBN = 128;      // MFMA filter tile: queries
constexpr uint32_t kScanQF = 8;        // queries per exact-scan launch (max)
constexpr uint32_t kSampleStride = 32; // candidate-threshold sample: every 32nd row

// Row-state flags (index load).
constexpr uint32_t kRowNonFinite = 1u;  // a NaN/Inf element
constexpr uint32_t kRowNormOvf = 2u;    // sum of squares overflowed
constexpr uint32_t kRowNormRange = 4u;  // nonzero norm outside [1e-18, 1e18]: no MFMA stage

// Query flags.
constexpr uint32_t kQueryNonFinite = 1u;
constexpr uint32_t kQueryNoApprox = 2u;   // norm zero/tiny/huge: answered by the exact scan

hipError_t launch_synth_uniform(float* out, uint64_t row0, uint64_t n_rows, uint32_t dim,
                                uint32_t ld, uint64_t seed, hipStream_t s);
hipError_t launch_copy_rows_f32(const float* src, uint64_t n, uint32_t dim, uint32_t ld,
                                float* dst, hipStream_t s);
hipError_t launch_widen_bf16_rows(const uint16_t* src, uint64_t n, uint32_t dim, uint32_t ld,
                                  float* dst, hipStream_t s);
hipError_t launch_row_norms(const float* rows, uint64_t n, uint32_t dim, uint32_t ld,
                            float* na, uint32_t* flags, hipStream_t s);
hipError_t launch_rows_to_bf16n(const float* rows, const float* na, uint64_t n, uint64_t n_pad,
                                uint32_t dim, uint32_t ld, uint16_t* out, hipStream_t s);
hipError_t launch_query_prep(const float* q, uint32_t nq, uint32_t qpad, uint32_t dim,
                             uint32_t ld, float* qf32, float* nb, uint16_t* qbf,
                             uint32_t* qflags, hipStream_t s);

struct GemmArgs {
    const uint16_t* A;      // normalised bf16 corpus [n_pad][ld]
    uint64_t a_row_stride;  // elements between consecutive tile rows (ld or ld*sample stride)
    uint32_t n_rows;        // valid tile rows (n for emit, n_sample for the sample pass)
    const uint16_t* B;      // normalised bf16 queries [qpad][ld]
    uint32_t ld;
    uint32_t n_rt, n_qt;    // row tiles, query tiles
    float* S;               // sample: scores [qpad][s_ld]
    uint32_t s_ld;
    const float* tau;       // emit: per-query threshold
    uint64_t* cand;         // emit: [qpad][cap] score keys
    uint32_t* cnt;          // emit: [qpad] counters
    uint32_t cap;
};
// Tile geometry of the active filter kernel (BSR_GEMM_VARIANT=1 selects the v1 128x128
// kernel for A/B comparisons; default v2 = persistent 256x256).
uint32_t gemm_query_pad();
uint32_t gemm_row_tile();
hipError_t launch_gemm_sample(const GemmArgs& a, hipStream_t s);
hipError_t launch_gemm_emit(const GemmArgs& a, hipStream_t s);

hipError_t launch_select_tau(const float* S, uint32_t s_ld, uint32_t n_s, uint32_t nq,
                             uint32_t qpad, const uint32_t* qflags, uint32_t ks, float* tau,
                             hipStream_t s);
hipError_t launch_select_cand(const uint64_t* cand, const uint32_t* cnt, uint32_t cap,
                              uint32_t nq, const float* tau, uint32_t kp, uint32_t* cand_rows,
                              uint32_t* ncand, float* tau_excl, hipStream_t s);
hipError_t launch_rescore(const float* rows, uint32_t ld, uint32_t dim, const float* na,
                          const float* qf32, const float* nb, uint32_t nq,
                          const uint32_t* cand_rows, const uint32_t* ncand, uint32_t kp,
                          const float* tau_excl, uint32_t k, double ebound,
                          uint64_t* out_keys, uint32_t* fail_cnt, uint32_t* fail_list,
                          hipStream_t s);
// Exact full scan for up to kScanQF queries (ids in qids, device).  part must hold
// grid * kScanQF * k keys; returns the grid used through *grid_out.
hipError_t launch_scan_exact(const float* rows, uint32_t ld, uint32_t dim, uint64_t n,
                             const float* na, const float* qf32, const int32_t* qids,
                             uint32_t nqf, const float* nb, uint32_t k, uint32_t grid,
                             uint64_t* part, hipStream_t s);
hipError_t launch_merge_parts(const uint64_t* part, uint32_t grid, const int32_t* qids,
                              uint32_t nqf, uint32_t k, uint64_t* out_keys, hipStream_t s);
hipError_t launch_finalize(const uint64_t* keys, uint32_t nq, uint32_t k, uint64_t n,
                           uint64_t offset, uint64_t* out_idx, float* out_dist,
                           uint32_t* out_count, hipStream_t s);
hipError_t launch_cosine_pair(const float* a, uint32_t la, const float* b, uint32_t lb,
                              float* out, hipStream_t s);
hipError_t launch_check_finite(const float* x, uint64_t count, uint32_t* flag, hipStream_t s);

uint32_t scan_grid_for(uint64_t n);

}  // namespace bsr
