// kernels.hpp -- host-side launchers for the gfx950 kernels (k_prep.hip, k_filter.hip,
// k_exact.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bsr {

// Layout constants shared by the host orchestration and the kernels.
constexpr uint32_t kLdAlign = 64;      // f32 row leading dimension multiple (elements)
constexpr uint32_t kRowPad = 256;      // rows are padded to a multiple of this (zero rows)
constexpr uint32_t kScanQF = 8;        // queries per exact-scan launch (max)
constexpr uint32_t kSampleStride = 32; // candidate-threshold sample: every 32nd row
constexpr uint32_t kQuantBlock = 32;   // rows sharing one int8 scale (one 32-row MFMA block)
constexpr uint32_t kSampleScaleRows = 128; // int8 sample rows sharing one scale (one filter tile)
constexpr uint32_t kFilterTile = 256;  // MFMA filter tile: 256 corpus rows x 256 queries

// Row-state flags (index load).
constexpr uint32_t kRowNonFinite = 1u;  // a NaN/Inf element
constexpr uint32_t kRowNormOvf = 2u;    // sum of squares overflowed
constexpr uint32_t kRowNormRange = 4u;  // nonzero norm outside [1e-18, 1e18]: no MFMA stage

// Query flags.
constexpr uint32_t kQueryNonFinite = 1u;
constexpr uint32_t kQueryNoApprox = 2u;   // norm zero/tiny/huge: answered by the exact scan

// Search status words (device, one small D2H copy per search).
enum StatusWord : uint32_t { kStFail = 0, kStEmitted = 1, kStQueryFlags = 2, kStFail2 = 3, kStWords = 4 };

// ---- data movement / load-time preparation (k_prep.hip) -------------------------------
hipError_t launch_synth_uniform(float* out, uint64_t row0, uint64_t n_rows, uint32_t dim,
                                uint32_t ld, uint64_t seed, hipStream_t s);
hipError_t launch_copy_rows_f32(const float* src, uint64_t n, uint32_t dim, uint32_t ld,
                                float* dst, hipStream_t s);
hipError_t launch_widen_bf16_rows(const uint16_t* src, uint64_t n, uint32_t dim, uint32_t ld,
                                  float* dst, hipStream_t s);
hipError_t launch_row_norms(const float* rows, uint64_t n, uint32_t dim, uint32_t ld,
                            float* na, uint32_t* flags, hipStream_t s);
// int8 filter operand: per 32-row block scale s (127*s >= max |a_i|/|a| over the block),
// q_i = rint(a_i/(|a| s)); ea_max (u32 bits of a non-negative float, atomicMax) receives
// an upper bound of max_row || a/|a| - s q ||_2.
hipError_t launch_rows_to_i8(const float* rows, uint64_t n, uint64_t n_pad, uint32_t dim,
                             uint32_t ld, int8_t* out, float* scales, uint32_t* ea_max,
                             hipStream_t s);
// The sample pass's operand: rows 0, kSampleStride, 2 kSampleStride, ... of the corpus,
// contiguous, int8 with one scale per kSampleScaleRows of them (the sample pass only sets the
// emission threshold; no certification depends on its quantization).  out: [n_s_pad][ld],
// scales: [n_s_pad / kSampleScaleRows], n_s_pad = round_up(n_s, kSampleScaleRows).
hipError_t launch_rows_to_i8_sample(const float* rows, uint64_t n, uint32_t dim, uint32_t ld,
                                    int8_t* out, float* scales, hipStream_t s);
// Query preparation: exact |b| (src/metrics.rs:155), flags, padded f32 copy, the filter
// operand (int8 + scale) and the per-query certification bound ebound[q].
struct QueryPrepArgs {
    const float* q;        // caller's queries [nq][dim]
    uint32_t nq, qpad, dim, ld;
    const uint32_t* ea_max;  // row-side error bound (device word)
    float* qf32;           // [qpad][ld]
    float* nb;             // [qpad]
    void* qop;             // int8 [qpad][ld]
    float* qscale;         // [qpad]
    float* ebound;         // [qpad]
    uint32_t* qflags;      // [qpad]
    int32_t* qids;         // [qpad]: min(q, nq-1), the exact scan's query-id list
    uint32_t* status;      // kStQueryFlags word receives the OR of the flags
    bool with_op;          // build the filter operand (false: exact scan only)
};
hipError_t launch_query_prep(const QueryPrepArgs& a, hipStream_t s);
// The parallel search's header exchange without host copies: this rank's 8 words into the device
// send buffer; the P received headers into fine-grained pinned host memory, then host_flag = seq
// (system-scope release) -- the host polls the flag.
hipError_t launch_header_put(const int32_t w[8], int32_t* dst, hipStream_t s);
hipError_t launch_header_publish(const int32_t* src, uint32_t words, int32_t* host, uint32_t* host_flag, uint32_t seq,
                                 hipStream_t s);
// The loopback communicator's all-gather: recv[r] = script[r] (a recorded contribution of a real
// P-rank run) for r != rank, this rank's send otherwise (every slot when script is null).
hipError_t launch_gather_emulate(const void* send, const void* script, void* recv, uint64_t bytes, uint32_t P,
                                 uint32_t rank, hipStream_t s);

// ---- MFMA candidate filter (k_filter.hip) ---------------------------------------------
struct GemmArgs {
    const uint8_t* A;       // filter rows [n_pad][row_bytes]
    uint64_t a_stride;      // bytes between consecutive tile rows (row_bytes, or x sample stride)
    uint32_t n_rows;        // valid tile rows (n for emit, n_sample for the sample pass)
    uint32_t a_scale_rows;  // int8: tile rows per a_scale entry (kQuantBlock emit, kSampleScaleRows sample)
    const uint8_t* B;       // filter queries [qpad][row_bytes]
    uint32_t row_bytes;     // bytes of one operand row (multiple of 64)
    uint32_t n_rt, n_qt;    // row tiles, query tiles
    const float* a_scale;   // i8: [n_pad / 32] block scales
    const float* b_scale;   // i8: [qpad] query scales
    float* S;               // sample: scores [qpad][s_ld]
    uint32_t s_ld;
    uint32_t s_compact;     // sample: 1 = one maximum per 32 sampled rows, 0 = every score
    const float* tau;       // emit: per-query threshold
    uint64_t* cand;         // emit: [qpad][cap] score keys
    uint32_t* cnt;          // emit: [qpad] counters
    uint32_t cap;
    // emit, int8 query-stationary kernel: all but the last 1/kTailDiv of its 128-row tiles go
    // to the workgroups' row streams round-robin, the rest are claimed one at a time per query
    // tile from tail[qt] (zeroed by k_select_tau); tail = nullptr: every tile static
    uint32_t* tail;
    // skinny TOP: the search's status words (zeroed by the kernel: no k_select_tau runs) and
    // the batch's query count (padding queries keep no list)
    uint32_t* status;
    uint32_t n_q;
    uint32_t top_layout;  // the skinny TOP row layout: 2 = the product strided pairs (0: lab, k_filter.hip)
};
// Dynamic tail of the emit filter: 1/kTailDiv of the row tiles; counters per (XCD pool, query
// tile) (<= kTailCounters query tiles) after the per-query counters, cnt[qpad + x * n_qt + qt].
constexpr uint32_t kTailDiv = 8;
constexpr uint32_t kTailCounters = 64;
// Row-stream gangs of the emit filter (GANG > 0): one 64-bit progress word per row stream (its
// n_qt <= 4 workgroups' static tile counts, 16 bits each) after the tail counters,
// cnt[qpad + 8 * kTailCounters ...], zeroed with them.
constexpr uint32_t kGangWords = 2 * 256;
// (static tiles per row stream: gangs from ~5.6M rows at 1000 queries.  Round 5, the filter
// builds in one process at the global threshold's rate: the gang build 2.4% slower than the
// small-shard build at 2.5M rows, 0.8% at 5M, 0-1% faster at 10M -- profiles/r05hm_hist_*,
// r05e_hist_10m.txt; the threshold was 256, ~2.5M rows)
constexpr uint32_t kGangMinTiles = 600;
// e0 / e1 (optional): events recorded at the kernel's own dispatch and completion
// (hipExtLaunchKernel), i.e. its device duration without the stream's launch gaps.
hipError_t launch_filter_sample(const GemmArgs& a, hipStream_t s, hipEvent_t e0 = nullptr,
                                hipEvent_t e1 = nullptr);
hipError_t launch_filter_emit(const GemmArgs& a, hipStream_t s, hipEvent_t e0 = nullptr,
                              hipEvent_t e1 = nullptr);
// int8 only, batches of <= 16 queries (query tile rows 0..15), HBM-bound: the same
// contract as the two launches above.
constexpr uint32_t kSkinnyMaxQ = 16;
hipError_t launch_filter_skinny_sample(const GemmArgs& a, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t launch_filter_skinny_emit(const GemmArgs& a, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
// The self-thresholded single-query path (round 6; rows of <= 16 K slices): no sample pass and no
// tau0 -- each of the skinny2 grid's W = skinny_top_lists(n) workgroups writes its 4 best keys per
// query to cand[q][W][4] (ascending; every other row of the workgroup scores at most the 4th), and
// cnt[q] = 4 W for q < 16; the status words kStFail / kStEmitted / kStFail2 are zeroed.
hipError_t launch_filter_skinny_top(const GemmArgs& a, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
uint32_t skinny_top_lists(uint32_t n_rows);
bool skinny_glds_on();  // the LDS-DMA skinny filter for 768-byte rows (BSR_SKINNY_GLDS=0: off; read per call)
// Shards of at least this many rows take the self-thresholded path for batches of <= 16 queries
// and k' <= 63 (every wave of the 512-workgroup grid then holds >= 64 units of 16 rows).
constexpr uint64_t kSkinnyTopMinRows = 2u << 20;

// tau[q] = the ks-th best sampled score (ks <= 128); also zeroes cnt[0..qpad) and the status
// words kStFail / kStEmitted / kStFail2 for the emit pass and rescores that follow.
// smax (optional): the query's ks best sample keys [qpad][ks] (kKeyNone where there are none),
// the input of the global threshold of a parallel search.
hipError_t launch_select_tau(const float* S, uint32_t s_ld, uint32_t n_s, uint32_t nq,
                             uint32_t qpad, const uint32_t* qflags, uint32_t ks, float* tau,
                             uint32_t* cnt, uint32_t* status, hipStream_t s, uint64_t* smax = nullptr);
// tau[q] = the ks-th best of the all-gathered sample keys g[P][qpad][ks] (parallel search,
// DESIGN.md §6); INFINITY for padding / no-filter queries.
hipError_t launch_global_tau(const uint64_t* g, uint32_t P, uint32_t qpad, uint32_t nq, uint32_t ks,
                             const uint32_t* qflags, float* tau, hipStream_t s);
// The k' = kp best emitted candidates (rows) and tau_excl = the (kp+1)-th score, for lists
// larger than kFusedSelectCap (smaller ones are selected inside the rescore).
hipError_t launch_select_cand(const uint64_t* cand, const uint32_t* cnt, uint32_t cap,
                              uint32_t nq, const float* tau, uint32_t kp, uint32_t* cand_rows,
                              uint32_t* ncand, float* tau_excl, hipStream_t s);

// ---- exact arithmetic (k_exact.hip) ---------------------------------------------------
// Exact rescoring of candidates + certification (one wave per query, or device-counted
// 8-wave workgroups for the second chance).
struct RescoreArgs {
    const float* rows;          // f32 [n_pad][ld]
    uint32_t ld, dim;
    const float* na;            // row magnitudes
    const float* qf32;          // queries [qpad][ld]
    const float* nb;            // query magnitudes
    uint32_t n_items;           // queries to process (the grid), or the bound on *n_items_dev
    const uint32_t* n_items_dev;  // non-null: the item count is read on the device (a status
                                  // word written by an earlier kernel of the same stream)
    const uint32_t* qlist;      // query id of item b (nullptr: b)
    // mode A, the k' selected candidates: cand_rows[q*kp + i], i < ncand[q]; tau_excl[q]
    const uint32_t* cand_rows;
    const uint32_t* ncand;
    uint32_t kp;
    const float* tau_excl;
    // mode B (cand_keys != nullptr), every emitted candidate: key_row(cand_keys[q*cap + i]),
    // i < cnt[q] <= cap (an overflowed list fails); certified against tau0[q]
    const uint64_t* cand_keys;
    const uint32_t* cnt;
    uint32_t cap;
    const float* tau0;
    // mode S (sel != 0, one-wave launch, cap <= 1024): the k' candidates selected in the
    // rescore kernel itself from cand_keys / cnt (radix select; tau_x = the (k'+1)-th score,
    // or tau0 when fewer were emitted) -- k_select_cand is not launched
    uint32_t sel;
    // mode S of the self-thresholded single-query path (top_w != 0; the tiny-batch kernel
    // k_rescore_kp only): cand_keys[q * cap ..] holds top_w ascending 4-lists (cap = 4 top_w <=
    // 64 kTopKeysPerLane, launch_filter_skinny_top); its wave 0 radix-selects the k' best of them.  The bound on the rows outside the lists -- the best score among the
    // lists' 4th keys -- goes to top_tau[q], and the keys above it are compacted to the front of
    // the query's list, their count to top_cnt[q]: the second chance's mode-B input (a query the
    // filter cannot serve: count 0, bound +inf).
    uint32_t top_w;
    const uint32_t* qflags;
    float* top_tau;
    uint32_t* top_cnt;
    uint32_t k;
    const float* ebound;        // per-query certification bound E_q
    uint64_t* out_keys;         // [nq][k]
    uint32_t* fail_cnt;         // uncertified queries: count (a status word) and list
    uint32_t* fail_list;
    // Fused finalize (the filter path: no k_finalize launch): the list of a query becomes its
    // (global index, distance) result rows here -- modes S / A for the certified queries, mode
    // B for every item it rescored (the uncertified ones are rewritten after the exact scan).
    uint64_t* res_idx;          // [nq][k] (nullptr: no fused finalize)
    float* res_dist;
    uint32_t* res_cnt;          // [nq]
    uint64_t offset, n_rows;    // global index of local row 0; shard rows (count = min(k, n))
    // (optional) the host mirror of the same rows (fine-grained pinned memory): every result row
    // is written there too, by the wave that finalizes it, so the publish copies only the status
    // words (the standard path; the global-threshold path publishes its whole buffer)
    uint64_t* hres_idx;
    float* hres_dist;
    uint32_t* hres_cnt;
    // mode B: block 0 also zeroes the NEXT search's status words and sums the emitted counts
    // into cur_status[kStEmitted] (what k_finalize does on the other paths)
    uint32_t* next_status;
    const uint32_t* emit_cnt;
    uint32_t* cur_status;
    uint32_t n_queries;
    // Parallel search with a global threshold (mode B, one wave per query): no
    // local certification -- every query's list of its rescored emitted rows becomes its
    // result (count = min(k, rows rescored)) and excl_out[q] receives the distance below which
    // no row left out can lie (1 - tau0 - E_q - 2.5e-7 rounded down; -inf when nothing can be
    // certified, +inf when every row was a candidate); the root certifies the merged lists.
    float* excl_out;
    // (optional, block 0) the parallel search merge's two words, set before its launch:
    // merge_words[0] = 0 (uncertified count), merge_words[1] = ~0 (lowest query with a NaN)
    uint32_t* merge_words;
    // Publish (optional, the batch's last kernel): the workgroup that finishes last copies
    // pub_bytes of the packed result buffer pub_src to host memory pub_dst (fine-grained pinned)
    // and then sets *pub_flag = 1 with a system-scope release, so the host sees the result
    // without waiting for the stream's completion signal and without a D2H copy node.
    const uint8_t* pub_src;
    uint8_t* pub_dst;
    size_t pub_bytes;
    uint32_t* pub_flag;
    uint32_t* pub_ticket;       // kTicketWords device words, 0 between launches
    uint32_t solo;              // (set by launch_rescore) a one-workgroup grid: its own last arrival
};
// The publishing kernels' arrival ticket: kTicketLeaves leaf counters and one root counter,
// each on a 64-byte line of its own (a workgroup adds to its leaf, blockIdx % kTicketLeaves; the
// last of a leaf adds to the root), all zero between launches.
constexpr uint32_t kTicketLeaves = 8, kTicketStride = 16, kTicketWords = (kTicketLeaves + 1) * kTicketStride;
// Workgroups of the device-counted rescore (failed certifications, usually a few queries).
constexpr uint32_t kRescoreAllGrid = 128;
// Candidate lists up to this many keys (k <= 10) are selected inside the rescore kernel.
constexpr uint32_t kFusedSelectCap = 1024;
hipError_t launch_rescore(const RescoreArgs& a, hipStream_t s);
// whether launch_rescore takes k_rescore_kp for a tiny batch's first pass (BSR_RESCORE_KP != 0)
bool rescore_kp_enabled();
// The self-thresholded path's lists per query are selected by one wave, this many keys per lane.
constexpr uint32_t kTopKeysPerLane = 32;
// Exact full scan for up to kScanQF queries (ids in qids, device).  part must hold
// grid * kScanQF * k keys.
hipError_t launch_scan_exact(const float* rows, uint32_t ld, uint32_t dim, uint64_t n,
                             const float* na, const float* qf32, const int32_t* qids,
                             uint32_t nqf, const float* nb, uint32_t k, uint32_t grid,
                             uint64_t* part, hipStream_t s);
hipError_t launch_merge_parts(const uint64_t* part, uint32_t grid, const int32_t* qids,
                              uint32_t nqf, uint32_t k, uint64_t* out_keys, hipStream_t s);
// The root's merge of gathered [P][nq][k_in] lists (counts [P][nq]) into [nq][k] outputs on
// the device (compute_global_top_k); P <= 64, P * k_in <= kMergeMaxEntries, k <= 256.
// *first_nan must hold ~0 before the launch; afterwards the lowest query with a NaN distance.
constexpr uint32_t kMergeMaxEntries = 1024;
hipError_t launch_merge_lists(const uint64_t* idx, const float* dist, const uint32_t* cnt, uint32_t P, uint32_t nq,
                              uint32_t k_in, uint32_t k, uint64_t* out_idx, float* out_dist, uint32_t* out_count,
                              uint32_t* first_nan, hipStream_t s);
// The general form: strided lists (the all-gathered packed result buffers of a parallel search)
// and, with excl, the certification of a global-threshold search.
struct MergeArgs {
    const uint64_t* idx;        // list l of query q: idx + l * idx_stride + q * k_in
    const float* dist;          // dist + l * dist_stride + q * k_in
    const uint32_t* cnt;        // cnt[l * cnt_stride + q]
    uint64_t idx_stride, dist_stride, cnt_stride;
    uint32_t P, nq, k_in, k;
    uint64_t* out_idx;          // [nq][k]
    float* out_dist;
    uint32_t* out_count;        // [nq]
    uint32_t* first_nan;        // ~0 before the launch
    // certification (optional): list l's exclusion bounds excl[l * excl_stride + q]; a query
    // is certified iff its merged list holds need = min(k, corpus rows) entries and the k-th
    // distance is below every bound -- the others are appended to fail_list / *fail_cnt
    const float* excl;
    uint64_t excl_stride;
    uint32_t need;
    uint32_t* fail_cnt;
    uint32_t* fail_list;
    // (optional) each list's kStWords status words, st[l * st_stride + w] -> st_all[l][w]
    const uint32_t* st;
    uint64_t st_stride;
    uint32_t* st_all;
    // (optional) the host mirror of out_idx / out_dist / out_count: the merged rows are written
    // there too, by the wave that merges them (pub_bytes then covers the part before them)
    uint64_t* hout_idx;
    float* hout_dist;
    uint32_t* hout_count;
    // (optional) publish the merged result buffer to host memory, as RescoreArgs::pub_*
    const uint8_t* pub_src;
    uint8_t* pub_dst;
    size_t pub_bytes;
    uint32_t* pub_flag;
    uint32_t* pub_ticket;
    uint32_t force_hash;  // (lab, set by launch_merge from BSR_MERGE_HASH) no disjoint-lists shortcut
    // every list is one search's own top-k (no index twice within a list): lists whose index ranges
    // are pairwise disjoint then skip the first-occurrence filter
    uint32_t lists_unique;
};
hipError_t launch_merge(const MergeArgs& a, hipStream_t s);
// Keys -> (global index, distance) rows; also zeroes `status`, the status words of the
// result buffer the next search will use.
// status: the NEXT search's status words (zeroed); emit_cnt (optional): per-query emitted
// counts, summed into cur_status[kStEmitted].
hipError_t launch_finalize(const uint64_t* keys, uint32_t nq, uint32_t k, uint64_t n,
                           uint64_t offset, uint64_t* out_idx, float* out_dist,
                           uint32_t* out_count, uint32_t* status, const uint32_t* emit_cnt,
                           uint32_t* cur_status, hipStream_t s);
hipError_t launch_cosine_pair(const float* a, uint32_t la, const float* b, uint32_t lb,
                              float* out, hipStream_t s);

uint32_t scan_grid_for(uint64_t n);

}  // namespace bsr
