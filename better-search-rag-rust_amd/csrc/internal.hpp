// internal.hpp -- host-side state shared by the C-ABI translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>

#include <atomic>

#include <string>
#include <vector>

#include "bsr.h"
#include "kernels.hpp"

namespace bsr {

int set_error(int code, const char* fmt, ...);
void clear_error();

#define BSR_HIP(call)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess)                                                               \
            return ::bsr::set_error(BSR_E_HIP, "%s failed: %s (%s:%d)", #call,              \
                                    hipGetErrorString(e_), __FILE__, __LINE__);             \
    } while (0)

#define BSR_TRY(call)               \
    do {                            \
        int r_ = (call);            \
        if (r_ != BSR_OK) return r_; \
    } while (0)

// Bumped by every device / pinned (re)allocation: a captured search graph is valid only
// for the generation it was captured in.
extern std::atomic<uint64_t> g_alloc_gen;

// Growable device allocation (never shrinks).
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t need);
    void release();
    template <class T> T* as() const { return static_cast<T*>(p); }
    ~DevBuf() { release(); }
};

bool is_device_ptr(const void* p);
void* coherent_host_alias(const void* p);  // device address of coherent pinned host memory, or nullptr
hipError_t stream_wait(hipStream_t s);  // poll until the stream's work is done
// Poll a host flag a publishing kernel raises (checking the stream now and then): hipSuccess,
// the stream's error, or hipErrorUnknown when the stream finished without raising it.
hipError_t flag_wait(const uint32_t* flag, hipStream_t s);
int select_device(int device);

static inline uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

struct Events {
    hipEvent_t a = nullptr, b = nullptr;
    bool armed = false;
    ~Events();
    int create();
};

}  // namespace bsr

struct bsr_index {
    bsr_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t dim = 0, ld = 0;
    uint64_t n = 0, n_pad = 0, global_offset = 0;
    bool loaded = false;
    bool approx_ok = false;
    uint32_t row_flags = 0;
    uint32_t op_row_bytes = 0;          // bytes of one filter operand row
    float row_ebound = 0.0f;            // int8: max_row ||a/|a| - s q||_2 (certification)

    bsr::DevBuf rows;   // f32 [n_pad][ld], zero padded: the reference's values
    bsr::DevBuf na;     // f32 [n_pad]: exact magnitudes (src/metrics.rs:154)
    bsr::DevBuf fop;    // filter operand rows: int8 [n_pad][ld]
    bsr::DevBuf fop_s;  // every kSampleStride-th row as the sample pass's operand, contiguous
    bsr::DevBuf ascale_s; // int8: f32 [n_s_pad / kSampleScaleRows] sample operand scales
    bsr::DevBuf ascale; // int8: f32 [n_pad/32] block scales
    bsr::DevBuf flags;  // u32 [2]: row flags, int8 row error bound (f32 bits)

    // per-search scratch
    bsr::DevBuf q_in, qf32, nb, qop, qscale, ebound, qflags, tau, S, cand, cnt, cand_rows, ncand,
        tau_excl, keys, fail, fail2, part, qids, qids_id, tmp;

    // Packed per-search result, double-buffered: [status words | counts | distances |
    // indices].  One D2H copy per search reads it all back (into pinned memory); the
    // finalize kernel of search i zeroes the status words of the buffer search i+1 uses.
    bsr::DevBuf res[2];
    uint8_t* h_res = nullptr;  // pinned, fine-grained (hipHostMallocCoherent) mirror of one result buffer
    uint8_t* h_res_dev = nullptr;   // its device-side address (the publishing kernel writes it)
    size_t h_res_bytes = 0;
    uint32_t* h_flag = nullptr;     // fine-grained host word raised by the publishing kernel
    uint32_t* h_flag_dev = nullptr;
    bsr::DevBuf pub_ticket;         // device word: workgroups finished in the publishing kernel
    uint32_t cur = 0;          // result buffer of the last search
    bool next_status_clean = false;  // status words of res[cur ^ 1] are known to be zero
    size_t res_off_cnt = 0, res_off_dist = 0, res_off_idx = 0, res_off_x = 0, res_bytes = 0;
    uint32_t* d_status = nullptr;
    uint32_t* d_cnt = nullptr;
    float* d_dist = nullptr;
    uint64_t* d_idx = nullptr;
    float* d_x = nullptr;      // global-threshold search: per-query exclusion bounds

    std::vector<uint32_t> h_qflags, h_fail;

    bsr_search_stats stats{};
    bsr_profile prof{};
    bsr::Events ev_emit, ev_sample, ev_select, ev_rescore, ev_scan, ev_total;
    int prof_level = 2;  // bsr_index_set_profile

    // Filtered batches replay a captured hipGraph of query prep -> filter -> select -> rescore
    // -> finalize -> D2H instead of ~9 launches.  One graph per result buffer; captured on the second search of a shape
    // (the first sizes every buffer), dropped when the shape or any allocation changes.
    struct SearchGraph {
        hipGraphExec_t exec = nullptr;
        uint32_t nq = 0, k = 0;
        const float* qsrc = nullptr;
        uint64_t n = 0, gen = 0;
        int timed = 0;  // profile level it was captured at (always 0: timed searches launch directly)
        bool top = false;  // the self-thresholded single-query path (round 6)
        uint32_t top_layout = 2;  // its row layout (BSR_TOP_LAYOUT, lab: read per search)
    };
    // (round 6) the batch is searched again on the thresholded path: the self-thresholded path
    // left a query uncertified (direct launches, no graph)
    bool force_threshold = false;
    bool capturing = false;    // a search is being captured into a graph
    SearchGraph graphs[2];
    SearchGraph warm;  // the last direct search of a graphable shape (no exec)
    uint64_t graph_replays = 0;
    ~bsr_index();

    // Run the local search; results stay in d_idx / d_dist / d_cnt (device, [nq][k]) and in
    // the pinned host mirror h_res at the same offsets.  after_launch (optional) runs once the
    // search's GPU work is enqueued, before the host waits for it (the parallel search issues
    // its shape-agreement collective there); its non-OK status is returned after the wait.
    int search_device(const float* queries, uint32_t nq, uint32_t k, int (*after_launch)(void*) = nullptr,
                      void* ctx = nullptr);
    int prepare_result(uint32_t nq, uint32_t k);

    // Parallel search with a global emission threshold (P > 1), in two halves
    // around the all-gather of every rank's ks best sample keys:
    //   phase A: query prep, the sample pass, tau0 and the keys (smax [qpad][gt_ks]);
    //   phase B: the global threshold from the gathered keys g[P][qpad][gt_ks], the emit pass
    //            and the exact rescore of EVERY emitted row, its top-k written as the result
    //            rows with the per-query exclusion bound d_x (no local certification).
    // Both enqueue only (no host wait); gtau_prepare sizes every buffer of phase A first.
    // gtau_eligible: the filter path with a sample pass.
    bool gtau_eligible(uint32_t nq, uint32_t k) const;
    int gtau_prepare(const float* queries, uint32_t nq, uint32_t k);  // buffers only (before the header)
    int gtau_phase_a(const float* queries, int part);  // launches only: part 0 query prep, 1 sample + tau0
    int gtau_phase_b(const uint64_t* g_smax, uint32_t P, uint32_t* merge_words = nullptr);
    bsr::DevBuf smax;
    uint32_t gt_nq = 0, gt_k = 0, gt_qpad = 0, gt_ks = 0;
};
