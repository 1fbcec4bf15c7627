// index.cpp -- the rank's corpus shard in HBM and the local search pipeline
// (compute_local_top_k, src/mpi_helpers/metrics.rs:16-53, for a batch of queries).
//
// Pipeline for a batch, all on the index's stream:
//   1. query prep     exact |b| (src/metrics.rs:155), flags, the filter operand (int8 + scale)
//                     and the per-query certification bound E_q
//   2. sample filter  MFMA scores of every 32nd row -> tau0 (per query)
//   3. emit filter    MFMA scores of every row; rows with score >= tau0 -> candidates
//   4. select         top-(k'+1) candidates by approximate score
//   5. rescore        exact sequential-f32 distances of k' candidates, top-k, certify
//   6. one status readback; fallback: exact full scan of any uncertified / ineligible query
// k > 200, or an index with out-of-range norms, use the exact scan only.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "internal.hpp"
#include "kernels.hpp"

namespace bsr {

constexpr uint32_t kMaxKForFilter = 200;

static thread_local std::string g_err;

int set_error(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
void clear_error() { g_err.clear(); }
const char* last_error_cstr() { return g_err.c_str(); }

std::atomic<uint64_t> g_alloc_gen{0};

int DevBuf::ensure(size_t need) {
    if (need <= bytes && p) return BSR_OK;
    release();
    ++g_alloc_gen;
    if (need == 0) need = 16;
    hipError_t e = hipMalloc(&p, need);
    if (e != hipSuccess) {
        p = nullptr;
        bytes = 0;
        (void)hipGetLastError();
        return set_error(BSR_E_NOMEM, "hipMalloc(%zu bytes) failed: %s", need, hipGetErrorString(e));
    }
    bytes = need;
    return BSR_OK;
}
void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
}

// Completion of a search's work on its stream, polled (hipStreamQuery) rather than blocked on:
// a blocking synchronize wakes the host ~15 us after the GPU finishes (measured: the D2H copy
// ends, the next host call comes 15 us later), which is idle GPU time between batches.
hipError_t stream_wait(hipStream_t s) {
    for (;;) {
        const hipError_t r = hipStreamQuery(s);
        if (r != hipErrorNotReady) return r;
        __builtin_ia32_pause();
    }
}

// A published search (its last kernel raises *flag after copying the result to host memory):
// spin on the flag, and now and then ask the stream -- a stream that has finished (or failed)
// without raising it is an error, never an endless wait.
hipError_t flag_wait(const uint32_t* flag, hipStream_t s) {
    for (uint32_t i = 1;; ++i) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE)) return hipSuccess;
        if ((i & 4095) == 0) {
            const hipError_t r = hipStreamQuery(s);
            if (r == hipSuccess) return __atomic_load_n(flag, __ATOMIC_ACQUIRE) ? hipSuccess : hipErrorUnknown;
            if (r != hipErrorNotReady) return r;
        }
        __builtin_ia32_pause();
    }
}

bool is_device_ptr(const void* p) {
    if (!p) return false;
    // no device visible (host-only entry points on a CPU machine): every pointer is host
    static const bool have_device = [] {
        int n = 0;
        const bool ok = hipGetDeviceCount(&n) == hipSuccess && n > 0;
        (void)hipGetLastError();
        return ok;
    }();
    if (!have_device) return false;
    hipPointerAttribute_t attr;
    hipError_t e = hipPointerGetAttributes(&attr, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// The device address of coherent (fine-grained) pinned host memory -- hipHostMalloc with
// hipHostMallocCoherent, e.g. bsr_host_alloc -- else nullptr (pageable memory, device memory,
// or non-coherent pinned memory, which the host could read stale from its caches).
void* coherent_host_alias(const void* p) {
    if (!p) return nullptr;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (attr.type != hipMemoryTypeHost || !(attr.allocationFlags & hipHostMallocCoherent) || !attr.devicePointer)
        return nullptr;
    return attr.devicePointer;
}

int select_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        (void)hipGetLastError();
        return set_error(BSR_E_NODEVICE, "no HIP device visible (this engine has no CPU path)");
    }
    if (device >= 0) {
        if (device >= n) return set_error(BSR_E_INVALID, "device %d out of range (%d visible)", device, n);
        BSR_HIP(hipSetDevice(device));
    }
    return BSR_OK;
}

Events::~Events() {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
}
int Events::create() {
    if (!a) BSR_HIP(hipEventCreate(&a));
    if (!b) BSR_HIP(hipEventCreate(&b));
    return BSR_OK;
}

}  // namespace bsr

using namespace bsr;

// ---------------------------------------------------------------------------------------
// profiling helpers
// ---------------------------------------------------------------------------------------
// Events exist when the index was created with BSR_FLAG_PROFILE; prof_level (bsr_index_set_profile)
// picks which stages record them: 1 = the emit filter / scan kernels only (the bench's timed
// steps: each recorded event is one more node in the search graph), 2 = every stage.
static inline bool profiling(const bsr_index* ix) { return (ix->cfg.flags & BSR_FLAG_PROFILE) != 0; }
static inline void ev_begin(bsr_index* ix, Events& e, int level = 2) {
    if (profiling(ix) && ix->prof_level >= level && e.a) { (void)hipEventRecord(e.a, ix->stream); e.armed = true; }
}
static inline void ev_end(bsr_index* ix, Events& e) {
    if (profiling(ix) && e.armed) (void)hipEventRecord(e.b, ix->stream);
}
// A filter / scan kernel launch timed at profile level >= 1: HIP events recorded on the stream
// around a direct launch (so the start event completes when the stream reaches the kernel).
// Two other forms were measured wrong on ROCm 7.2 (profiles/r04m_*): the events bound to the
// launch by hipExtLaunchKernel start at the kernel's submission -- behind the sample pass and
// tau selection still running, +0.2 ms on a 5.57 ms kernel -- and event-record nodes inside a
// replayed graph timed from the graph's start (6.12 ms).  Timed searches are therefore never
// graph-replayed (level 0 is the product path).
template <class F>
static inline hipError_t launch_timed(bsr_index* ix, Events& e, F&& launch, int level = 1) {
    const bool timed = !ix->capturing && profiling(ix) && ix->prof_level >= level && e.a;
    if (!timed) return launch((hipEvent_t) nullptr, (hipEvent_t) nullptr);
    hipError_t r = hipEventRecord(e.a, ix->stream);
    if (r == hipSuccess) r = launch((hipEvent_t) nullptr, (hipEvent_t) nullptr);
    if (r == hipSuccess) r = hipEventRecord(e.b, ix->stream);
    e.armed = r == hipSuccess;
    return r;
}
static inline void ev_collect(Events& e, double& ms, uint64_t& n, uint64_t launches) {
    if (!e.armed) return;
    float t = 0.0f;
    if (hipEventElapsedTime(&t, e.a, e.b) == hipSuccess) { ms += t; n += launches; }
    e.armed = false;
}

// ---------------------------------------------------------------------------------------
// load / append
// ---------------------------------------------------------------------------------------
static int index_prepare_rows(bsr_index* ix, const void* rows, uint64_t n_rows, uint64_t first_row) {
    // Copy rows [first_row, first_row+n_rows) of the padded slab from the caller's buffer.
    float* dst = ix->rows.as<float>() + first_row * ix->ld;
    const bool dev = is_device_ptr(rows);
    const size_t elem = ix->cfg.dtype == BSR_BF16 ? 2 : 4;
    const void* src = rows;
    // Device rows may still be in flight on ANY stream of the caller (a torch side stream, a
    // communication stream): the ABI has no stream argument, and a load runs once, outside
    // any timed region, so a full device synchronize costs nothing and removes the hazard.
    if (dev) BSR_HIP(hipDeviceSynchronize());
    if (!dev) {
        BSR_TRY(ix->tmp.ensure(n_rows * (size_t)ix->dim * elem));
        BSR_HIP(hipMemcpyAsync(ix->tmp.p, rows, n_rows * (size_t)ix->dim * elem, hipMemcpyHostToDevice,
                               ix->stream));
        src = ix->tmp.p;
    }
    if (ix->cfg.dtype == BSR_BF16)
        BSR_HIP(launch_widen_bf16_rows(static_cast<const uint16_t*>(src), n_rows, ix->dim, ix->ld, dst, ix->stream));
    else
        BSR_HIP(launch_copy_rows_f32(static_cast<const float*>(src), n_rows, ix->dim, ix->ld, dst, ix->stream));
    return BSR_OK;
}

// Per-row state: the reference's magnitudes, row flags and the filter operand.
static int index_finish_load(bsr_index* ix) {
    BSR_TRY(ix->na.ensure(ix->n_pad * sizeof(float)));
    BSR_TRY(ix->fop.ensure((size_t)ix->n_pad * ix->op_row_bytes));
    BSR_TRY(ix->flags.ensure(2 * sizeof(uint32_t)));
    BSR_HIP(hipMemsetAsync(ix->flags.p, 0, 2 * sizeof(uint32_t), ix->stream));
    BSR_HIP(hipMemsetAsync(ix->na.p, 0, ix->n_pad * sizeof(float), ix->stream));
    if (ix->n) BSR_HIP(launch_row_norms(ix->rows.as<float>(), ix->n, ix->dim, ix->ld, ix->na.as<float>(),
                                        ix->flags.as<uint32_t>(), ix->stream));
    BSR_TRY(ix->ascale.ensure(ix->n_pad / kQuantBlock * sizeof(float)));
    BSR_HIP(launch_rows_to_i8(ix->rows.as<float>(), ix->n, ix->n_pad, ix->dim, ix->ld, ix->fop.as<int8_t>(),
                              ix->ascale.as<float>(), ix->flags.as<uint32_t>() + 1, ix->stream));
    // The sample pass reads every kSampleStride-th row: those rows, contiguous (1/32 of the
    // operand bytes), so that it streams whole rows, quantized with one scale per filter tile
    // of sampled rows (its epilogue then takes integer maxima).
    const uint64_t n_s = (ix->n + kSampleStride - 1) / kSampleStride;
    const uint64_t n_s_pad = round_up(std::max<uint64_t>(n_s, 1), kSampleScaleRows);
    BSR_TRY(ix->fop_s.ensure((size_t)n_s_pad * ix->op_row_bytes));
    BSR_TRY(ix->ascale_s.ensure((size_t)(n_s_pad / kSampleScaleRows) * sizeof(float)));
    BSR_HIP(launch_rows_to_i8_sample(ix->rows.as<float>(), ix->n, ix->dim, ix->ld, ix->fop_s.as<int8_t>(),
                                     ix->ascale_s.as<float>(), ix->stream));
    uint32_t f[2] = {0, 0};
    BSR_HIP(hipMemcpyAsync(f, ix->flags.p, sizeof f, hipMemcpyDeviceToHost, ix->stream));
    BSR_HIP(hipStreamSynchronize(ix->stream));
    ix->row_flags = f[0];
    memcpy(&ix->row_ebound, &f[1], sizeof(float));
    if (f[0] & kRowNonFinite) {
        ix->loaded = false;
        ix->n = 0;
        return set_error(BSR_E_NONFINITE, "corpus contains NaN/Inf (the reference panics on NaN distances)");
    }
    ix->approx_ok = !(f[0] & (kRowNormOvf | kRowNormRange)) && !(ix->cfg.flags & BSR_FLAG_EXACT_ONLY);
    ix->loaded = true;
    return BSR_OK;
}

int bsr_index_create_impl(const bsr_config* cfg, bsr_index** out) {
    if (!cfg || !out) return set_error(BSR_E_INVALID, "null argument");
    *out = nullptr;
    if (cfg->dim == 0) return set_error(BSR_E_INVALID, "dim must be >= 1");
    if (cfg->dtype != BSR_F32 && cfg->dtype != BSR_BF16) return set_error(BSR_E_INVALID, "unknown dtype");
    // The bf16 filter operand (rounds 1-3) is retired: the int8 operand runs at twice the MFMA
    // rate with an equally tight certification bound; a bf16 CORPUS (dtype)
    // is still served, on the int8 filter.
    if (cfg->flags & BSR_FLAG_FILTER_BF16)
        return set_error(BSR_E_INVALID, "BSR_FLAG_FILTER_BF16 is retired (the filter operand is int8)");
    if (cfg->max_k == 0 || cfg->max_k > BSR_MAX_K)
        return set_error(BSR_E_INVALID, "max_k must be in [1, %u]", BSR_MAX_K);
    BSR_TRY(select_device(cfg->device));
    bsr_index* ix = new (std::nothrow) bsr_index();
    if (!ix) return set_error(BSR_E_NOMEM, "host allocation failed");
    ix->cfg = *cfg;
    int dev = 0;
    (void)hipGetDevice(&dev);
    ix->device = dev;
    ix->dim = cfg->dim;
    ix->ld = (uint32_t)round_up(cfg->dim, kLdAlign);
    ix->op_row_bytes = ix->ld;  // int8 filter operand rows
    // A blocking stream: its work waits for work issued earlier on the legacy default (NULL)
    // stream -- PyTorch's default stream -- so device rows or queries a caller has just
    // produced there are complete before the library reads them (the ABI has no stream
    // argument).  Round 3's 50M test loaded shards whose bf16 conversion was still running on
    // torch's stream into a non-blocking stream: stale rows, wrong results.
    if (hipStreamCreateWithFlags(&ix->stream, hipStreamDefault) != hipSuccess) {
        delete ix;
        return set_error(BSR_E_HIP, "hipStreamCreate failed");
    }
    if (cfg->flags & BSR_FLAG_PROFILE) {
        for (Events* e : {&ix->ev_emit, &ix->ev_sample, &ix->ev_select, &ix->ev_rescore, &ix->ev_scan, &ix->ev_total}) {
            int r = e->create();
            if (r != BSR_OK) { delete ix; return r; }
        }
    }
    *out = ix;
    return BSR_OK;
}

bsr_index::~bsr_index() {
    for (SearchGraph& g : graphs)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (h_res) (void)hipHostFree(h_res);
    if (h_flag) (void)hipHostFree(h_flag);
}

void bsr_index_destroy_impl(bsr_index* ix) {
    if (!ix) return;
    (void)hipSetDevice(ix->device);
    (void)hipStreamSynchronize(ix->stream);
    (void)hipStreamDestroy(ix->stream);
    delete ix;
}

int bsr_index_load_impl(bsr_index* ix, const void* rows, uint64_t n_rows, uint64_t global_offset) {
    if (!ix) return set_error(BSR_E_INVALID, "null index");
    if (n_rows && !rows) return set_error(BSR_E_INVALID, "null rows");
    if (n_rows >= (1ull << 31)) return set_error(BSR_E_INVALID, "shard too large (the reference slices with i32 offsets)");
    BSR_HIP(hipSetDevice(ix->device));
    ix->loaded = false;
    ix->n = n_rows;
    ix->n_pad = round_up(n_rows ? n_rows : 1, kRowPad);
    ix->global_offset = global_offset;
    BSR_TRY(ix->rows.ensure(ix->n_pad * (size_t)ix->ld * sizeof(float)));
    BSR_HIP(hipMemsetAsync(ix->rows.p, 0, ix->n_pad * (size_t)ix->ld * sizeof(float), ix->stream));
    if (n_rows) BSR_TRY(index_prepare_rows(ix, rows, n_rows, 0));
    return index_finish_load(ix);
}

int bsr_index_append_impl(bsr_index* ix, const void* rows, uint64_t n_rows) {
    if (!ix) return set_error(BSR_E_INVALID, "null index");
    if (!n_rows) return BSR_OK;
    if (!rows) return set_error(BSR_E_INVALID, "null rows");
    BSR_HIP(hipSetDevice(ix->device));
    const uint64_t old_n = ix->loaded ? ix->n : 0;
    const uint64_t new_n = old_n + n_rows;
    if (new_n >= (1ull << 31)) return set_error(BSR_E_INVALID, "shard too large");
    const uint64_t new_pad = round_up(new_n, kRowPad);
    if (new_pad * (size_t)ix->ld * sizeof(float) > ix->rows.bytes) {
        DevBuf grown;
        BSR_TRY(grown.ensure(new_pad * (size_t)ix->ld * sizeof(float)));
        BSR_HIP(hipMemsetAsync(grown.p, 0, new_pad * (size_t)ix->ld * sizeof(float), ix->stream));
        if (old_n)
            BSR_HIP(hipMemcpyAsync(grown.p, ix->rows.p, old_n * (size_t)ix->ld * sizeof(float),
                                   hipMemcpyDeviceToDevice, ix->stream));
        BSR_HIP(hipStreamSynchronize(ix->stream));
        std::swap(ix->rows.p, grown.p);
        std::swap(ix->rows.bytes, grown.bytes);
    }
    ix->n = new_n;
    ix->n_pad = new_pad;
    BSR_TRY(index_prepare_rows(ix, rows, n_rows, old_n));
    return index_finish_load(ix);
}

int bsr_index_get_many_impl(const bsr_index* ix, uint64_t offset, uint64_t count, float* out) {
    if (!ix || (!out && count)) return set_error(BSR_E_INVALID, "null argument");
    if (!ix->loaded) return set_error(BSR_E_STATE, "index not loaded");
    if (offset > ix->n || count > ix->n - offset) return set_error(BSR_E_INVALID, "slice out of range");
    if (!count) return BSR_OK;
    BSR_HIP(hipSetDevice(ix->device));
    const hipMemcpyKind kind = is_device_ptr(out) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    BSR_HIP(hipMemcpy2DAsync(out, ix->dim * sizeof(float), ix->rows.as<float>() + offset * ix->ld,
                             ix->ld * sizeof(float), ix->dim * sizeof(float), count, kind, ix->stream));
    BSR_HIP(hipStreamSynchronize(ix->stream));
    return BSR_OK;
}

// ---------------------------------------------------------------------------------------
// search
// ---------------------------------------------------------------------------------------
// Exact full scan of n_ids queries whose ids are the device list `ids` (groups of kScanQF;
// an id list padded to a multiple of kScanQF with valid ids).
static int run_exact_scan(bsr_index* ix, const int32_t* ids, uint32_t n_ids, uint32_t k) {
    if (!n_ids) return BSR_OK;
    const uint32_t groups = (n_ids + kScanQF - 1) / kScanQF;
    const uint32_t grid = scan_grid_for(ix->n);
    BSR_TRY(ix->part.ensure((size_t)grid * kScanQF * k * sizeof(uint64_t)));
    ev_begin(ix, ix->ev_scan, 1);
    for (uint32_t g = 0; g < groups; ++g) {
        const uint32_t nqf = std::min(kScanQF, n_ids - g * kScanQF);
        const int32_t* qid = ids + (size_t)g * kScanQF;
        BSR_HIP(launch_scan_exact(ix->rows.as<float>(), ix->ld, ix->dim, ix->n, ix->na.as<float>(),
                                  ix->qf32.as<float>(), qid, nqf, ix->nb.as<float>(), k, grid,
                                  ix->part.as<uint64_t>(), ix->stream));
        BSR_HIP(launch_merge_parts(ix->part.as<uint64_t>(), grid, qid, nqf, k, ix->keys.as<uint64_t>(), ix->stream));
    }
    ev_end(ix, ix->ev_scan);
    return BSR_OK;
}

// The same for a host list of query ids (the fallback queries of a batch).
static int run_exact_scan_list(bsr_index* ix, const std::vector<int32_t>& ids, uint32_t k) {
    if (ids.empty()) return BSR_OK;
    const uint32_t groups = (uint32_t)((ids.size() + kScanQF - 1) / kScanQF);
    std::vector<int32_t> padded((size_t)groups * kScanQF);
    for (uint32_t g = 0; g < groups; ++g)
        for (uint32_t j = 0; j < kScanQF; ++j) {
            const size_t i = (size_t)g * kScanQF + j;
            padded[i] = i < ids.size() ? ids[i] : ids[(size_t)g * kScanQF];
        }
    BSR_TRY(ix->qids.ensure(padded.size() * sizeof(int32_t)));
    BSR_HIP(hipMemcpyAsync(ix->qids.p, padded.data(), padded.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                           ix->stream));
    return run_exact_scan(ix, ix->qids.as<int32_t>(), (uint32_t)ids.size(), k);
}

static uint32_t kp_for(uint32_t k) { return 64u * ((3u * k + 34u + 63u) / 64u) - 1u; }
static uint32_t cap_for(uint32_t k) { return 16u * (kp_for(k) + 1u); }

static uint32_t ks_for(uint32_t k) { return (kp_for(k) + 1u) / 8u; }

// Steps 2-3 of the candidate stage: the sample pass and tau0 (smax: also the ks best sample
// keys per query, the input of a parallel search's global threshold), then the emit pass.
// Batches of at most 16 queries use the skinny (HBM-bound, no LDS) filter kernels.
static int sample_pass(bsr_index* ix, uint32_t nq, uint32_t qpad, uint32_t k, uint64_t* smax);
static int emit_pass(bsr_index* ix, uint32_t nq, uint32_t qpad, uint32_t k);


// The self-thresholded single-query path (round 6, DESIGN.md §5 tiny batches): batches of <= 16
// queries over shards of >= kSkinnyTopMinRows rows, k' <= 63, rows of <= 16 K slices, with the
// tiny-batch rescore kernel (BSR_SKINNY_TOP=0 turns it off, for A/B runs).  No sample pass and
// no tau0: the skinny filter keeps every wave's 4 best keys per query, the rescore selects the k'
// best of them.  Returns the lists' slots per query (0: the thresholded path).
static uint32_t top_slots(const bsr_index* ix, uint32_t nq, uint32_t k) {
    const char* v = getenv("BSR_SKINNY_TOP");
    if ((v && v[0] == '0') || ix->force_threshold) return 0;
    if (nq > kSkinnyMaxQ || ix->n < kSkinnyTopMinRows || kp_for(k) > 63 || k > 64 || ix->op_row_bytes > 16 * 64 ||
        ix->ld % 64 != 0 || ix->ld > 1024 || !rescore_kp_enabled())
        return 0;
    const uint32_t slots = 4 * skinny_top_lists((uint32_t)ix->n);
    return slots <= 64u * kTopKeysPerLane ? slots : 0;  // (k_rescore_kp's wave 0 holds the lists)
}

// Buffers of the candidate stage for a batch (k' = kp_for(k) candidates, lists of cap keys).
static int filter_buffers(bsr_index* ix, uint32_t nq, uint32_t qpad, uint32_t k) {
    // k' candidates, (k'+1) % 64 == 0, about 3k: the k-th exact score must clear the (k'+1)-th
    // approximate one by E_q, and in a Gaussian-like tail that takes ~3x as many rows at
    // E_q/sigma ~ 0.26.  63 for k <= 10, 191 for k = 50, 383 for k = 100.
    const uint32_t kp = kp_for(k);
    const uint32_t cap = std::max(cap_for(k), top_slots(ix, nq, k));
    ix->stats.n_candidates = kp;
    BSR_TRY(ix->tau.ensure((size_t)qpad * sizeof(float)));
    BSR_TRY(ix->cand.ensure((size_t)qpad * cap * sizeof(uint64_t)));
    BSR_TRY(ix->cnt.ensure(((size_t)qpad + 8 * kTailCounters + kGangWords) * sizeof(uint32_t)));  // + tail, gangs
    BSR_TRY(ix->cand_rows.ensure((size_t)nq * kp * sizeof(uint32_t)));
    BSR_TRY(ix->ncand.ensure((size_t)nq * sizeof(uint32_t)));
    BSR_TRY(ix->tau_excl.ensure((size_t)nq * sizeof(float)));
    BSR_TRY(ix->fail.ensure((size_t)nq * sizeof(uint32_t)));
    BSR_TRY(ix->fail2.ensure((size_t)nq * sizeof(uint32_t)));
    return BSR_OK;
}

static GemmArgs gemm_args(bsr_index* ix, uint32_t qpad) {
    GemmArgs g{};
    g.A = ix->fop.as<uint8_t>();
    g.B = ix->qop.as<uint8_t>();
    g.row_bytes = ix->op_row_bytes;
    g.n_qt = qpad / kFilterTile;
    g.a_scale = ix->ascale.as<float>();
    g.b_scale = ix->qscale.as<float>();
    return g;
}

static int sample_pass(bsr_index* ix, uint32_t nq, uint32_t qpad, uint32_t k, uint64_t* smax) {
    BSR_TRY(filter_buffers(ix, nq, qpad, k));
    const bool skinny = nq <= kSkinnyMaxQ;
    const uint32_t cap = cap_for(k);
    // (k'+1)/8: about 8 x 32 = 256 rows reach tau0 for k <= 10.  Fewer (ks = (k'+1)/12, /16)
    // measured 1-2% less filter time and up to 1.3% of the queries falling back to the exact
    // scan (profiles/r02f_*): not worth it.
    const uint32_t ks = ks_for(k);
    const uint32_t BM = kFilterTile;
    const uint64_t n = ix->n;
    GemmArgs g = gemm_args(ix, qpad);
    uint32_t* status = ix->d_status;
    if (n > cap) {
        // tau0 from every 32nd row: the ks-th best sampled score, or (large shards) the
        // ks-th best maximum over 32 sampled rows -- never above the former, so at least
        // ~ks*32 rows of the shard reach it.
        const uint32_t n_s = (uint32_t)((n + kSampleStride - 1) / kSampleStride);
        const uint32_t n_rt_s = (n_s + BM - 1) / BM;
        const bool compact = n_s >= 32u * 8u * ks;
        const uint32_t s_ld = compact ? n_rt_s * (BM / 32) : n_rt_s * BM;
        const uint32_t n_vals = compact ? (n_s + 31) / 32 : n_s;
        BSR_TRY(ix->S.ensure((size_t)qpad * s_ld * sizeof(float)));
        g.A = ix->fop_s.as<uint8_t>();  // the sampled rows, contiguous
        g.a_stride = ix->op_row_bytes;
        g.a_scale = ix->ascale_s.as<float>();
        g.a_scale_rows = kSampleScaleRows;
        g.n_rows = n_s;
        g.n_rt = n_rt_s;
        g.S = ix->S.as<float>();
        g.s_ld = s_ld;
        g.s_compact = compact ? 1u : 0u;
        BSR_HIP(launch_timed(ix, ix->ev_sample, [&](hipEvent_t e0, hipEvent_t e1) {
            return skinny ? launch_filter_skinny_sample(g, ix->stream, e0, e1)
                          : launch_filter_sample(g, ix->stream, e0, e1);
        }, 2));
        BSR_HIP(launch_select_tau(ix->S.as<float>(), s_ld, n_vals, nq, qpad, ix->qflags.as<uint32_t>(), ks,
                                  ix->tau.as<float>(), ix->cnt.as<uint32_t>(), status, ix->stream, smax));
    } else {
        BSR_HIP(launch_select_tau(nullptr, 0, 0, nq, qpad, ix->qflags.as<uint32_t>(), ks, ix->tau.as<float>(),
                                  ix->cnt.as<uint32_t>(), status, ix->stream, smax));
    }
    return BSR_OK;
}

static int emit_pass(bsr_index* ix, uint32_t nq, uint32_t qpad, uint32_t k) {
    const bool skinny = nq <= kSkinnyMaxQ;
    const uint32_t BM = kFilterTile;
    const uint64_t n = ix->n;
    GemmArgs g = gemm_args(ix, qpad);
    g.a_stride = ix->op_row_bytes;
    g.a_scale_rows = kQuantBlock;
    g.n_rows = (uint32_t)n;
    g.n_rt = (uint32_t)((n + BM - 1) / BM);
    g.tau = ix->tau.as<float>();
    g.cand = ix->cand.as<uint64_t>();
    g.cnt = ix->cnt.as<uint32_t>();
    g.cap = cap_for(k);
    // the last 1/kTailDiv of the row tiles are balanced dynamically (k_filter_qs16)
    g.tail = g.n_qt <= kTailCounters ? ix->cnt.as<uint32_t>() + qpad : nullptr;
    BSR_HIP(launch_timed(ix, ix->ev_emit, [&](hipEvent_t e0, hipEvent_t e1) {
        return skinny ? launch_filter_skinny_emit(g, ix->stream, e0, e1)
                      : launch_filter_emit(g, ix->stream, e0, e1);
    }));
    return BSR_OK;
}

// the skinny TOP row layout: 2, the strided pairs (BSR_TOP_LAYOUT=0: contiguous units, lab A/B only)
static uint32_t top_layout_lab() {
    const char* lay = getenv("BSR_TOP_LAYOUT");
    return lay && lay[0] == '0' ? 0u : 2u;
}

// The self-thresholded filter pass: every wave's 4 best keys per query (launch_filter_skinny_top).
static int top_pass(bsr_index* ix, uint32_t nq, uint32_t qpad, uint32_t k) {
    BSR_TRY(filter_buffers(ix, nq, qpad, k));
    GemmArgs g = gemm_args(ix, qpad);
    g.a_stride = ix->op_row_bytes;
    g.a_scale_rows = kQuantBlock;
    g.n_rows = (uint32_t)ix->n;
    g.n_rt = (uint32_t)((ix->n + kFilterTile - 1) / kFilterTile);
    g.cand = ix->cand.as<uint64_t>();
    g.cnt = ix->cnt.as<uint32_t>();
    g.cap = top_slots(ix, nq, k);
    g.status = ix->d_status;
    g.n_q = nq;
    g.top_layout = top_layout_lab();
    BSR_HIP(launch_timed(ix, ix->ev_emit, [&](hipEvent_t e0, hipEvent_t e1) {
        return launch_filter_skinny_top(g, ix->stream, e0, e1);
    }));
    return BSR_OK;
}

// Candidate stage (steps 2-5) for every query of the batch.
static int run_filter(bsr_index* ix, uint32_t nq, uint32_t qpad, uint32_t k, uint32_t* next_status, bool publish) {
    const uint32_t top = top_slots(ix, nq, k);
    if (top) {
        BSR_TRY(top_pass(ix, nq, qpad, k));
    } else {
        BSR_TRY(sample_pass(ix, nq, qpad, k, nullptr));
        BSR_TRY(emit_pass(ix, nq, qpad, k));
    }
    const uint32_t kp = kp_for(k);
    const uint32_t cap = top ? top : cap_for(k);
    uint32_t* status = ix->d_status;
    // lists of <= 1024 keys (k <= 10): the rescore kernel selects its own k' candidates (the
    // self-thresholded path: always, every wave of the tiny-batch kernel taking part)
    const bool fused_select = top || cap <= kFusedSelectCap;
    if (!fused_select) {
        ev_begin(ix, ix->ev_select);
        BSR_HIP(launch_select_cand(ix->cand.as<uint64_t>(), ix->cnt.as<uint32_t>(), cap, nq, ix->tau.as<float>(),
                                   kp, ix->cand_rows.as<uint32_t>(), ix->ncand.as<uint32_t>(),
                                   ix->tau_excl.as<float>(), ix->stream));
        ev_end(ix, ix->ev_select);
    }
    ev_begin(ix, ix->ev_rescore);
    RescoreArgs ra{};
    ra.rows = ix->rows.as<float>();
    ra.ld = ix->ld;
    ra.dim = ix->dim;
    ra.na = ix->na.as<float>();
    ra.qf32 = ix->qf32.as<float>();
    ra.nb = ix->nb.as<float>();
    ra.n_items = nq;
    ra.cand_rows = ix->cand_rows.as<uint32_t>();
    ra.ncand = ix->ncand.as<uint32_t>();
    ra.kp = kp;
    ra.tau_excl = ix->tau_excl.as<float>();
    ra.k = k;
    ra.ebound = ix->ebound.as<float>();
    ra.out_keys = ix->keys.as<uint64_t>();
    ra.fail_cnt = status + kStFail;
    ra.fail_list = ix->fail.as<uint32_t>();
    // the result rows are written by the rescore kernels themselves (no k_finalize launch)
    ra.res_idx = ix->d_idx;
    ra.res_dist = ix->d_dist;
    ra.res_cnt = ix->d_cnt;
    if (publish) {  // the result rows also go straight to the host mirror (published below)
        ra.hres_idx = reinterpret_cast<uint64_t*>(ix->h_res_dev + ix->res_off_idx);
        ra.hres_dist = reinterpret_cast<float*>(ix->h_res_dev + ix->res_off_dist);
        ra.hres_cnt = reinterpret_cast<uint32_t*>(ix->h_res_dev + ix->res_off_cnt);
    }
    ra.offset = ix->global_offset;
    ra.n_rows = ix->n;
    if (fused_select) {
        ra.sel = 1;
        ra.cand_keys = ix->cand.as<uint64_t>();
        ra.cnt = ix->cnt.as<uint32_t>();
        ra.cap = cap;
        ra.tau0 = ix->tau.as<float>();
    }
    if (top) {
        ra.top_w = top / 4;  // (lists: one per workgroup of the skinny filter)
        ra.qflags = ix->qflags.as<uint32_t>();
        ra.top_tau = ix->tau.as<float>();  // (the second chance's tau0)
        ra.top_cnt = ix->cnt.as<uint32_t>();
    }
    BSR_HIP(launch_rescore(ra, ix->stream));
    // Second chance, in the same stream (and graph): a query that failed certification is
    // rescored over EVERY row it emitted (~4k'), certified against tau0 -- far less than a
    // scan.  The failed count is read on the device, so no host round trip; what fails here
    // too goes to fail2 (exact scan, host-driven).
    RescoreArgs rb = ra;
    rb.sel = 0;
    rb.top_w = 0;
    rb.n_items = nq;
    rb.n_items_dev = status + kStFail;
    rb.qlist = ix->fail.as<uint32_t>();
    rb.cand_rows = nullptr;
    rb.ncand = nullptr;
    rb.tau_excl = nullptr;
    rb.cand_keys = ix->cand.as<uint64_t>();
    rb.cnt = ix->cnt.as<uint32_t>();
    rb.cap = cap;
    rb.tau0 = ix->tau.as<float>();
    rb.fail_cnt = status + kStFail2;
    rb.fail_list = ix->fail2.as<uint32_t>();
    rb.next_status = next_status;
    rb.emit_cnt = ix->cnt.as<uint32_t>();
    rb.cur_status = status;
    rb.n_queries = nq;
    if (publish) {  // the batch's last kernel: the status words to host memory, then the flag
        rb.pub_src = ix->res[ix->cur].as<uint8_t>();
        rb.pub_dst = ix->h_res_dev;
        rb.pub_bytes = kStWords * sizeof(uint32_t);  // (the rows: written through by both passes)
        rb.pub_flag = ix->h_flag_dev;
        rb.pub_ticket = ix->pub_ticket.as<uint32_t>();
    }
    BSR_HIP(launch_rescore(rb, ix->stream));
    ev_end(ix, ix->ev_rescore);
    return BSR_OK;
}

// The packed result buffer of a batch (status words | counts | distances | indices | the
// global-threshold search's exclusion bounds), double-buffered; d_* point into res[cur].
int bsr_index::prepare_result(uint32_t nq, uint32_t k) {
    const size_t nqk = (size_t)std::max(nq, 1u) * k;
    res_off_cnt = 16;
    res_off_dist = round_up(res_off_cnt + (size_t)std::max(nq, 1u) * sizeof(uint32_t), 16);
    res_off_idx = round_up(res_off_dist + nqk * sizeof(float), 16);
    res_off_x = round_up(res_off_idx + nqk * sizeof(uint64_t), 16);
    res_bytes = round_up(res_off_x + (size_t)std::max(nq, 1u) * sizeof(float), 16);
    if (res[0].bytes < res_bytes || res[1].bytes < res_bytes) {
        for (DevBuf& r : res) {
            BSR_TRY(r.ensure(res_bytes));
            BSR_HIP(hipMemsetAsync(r.p, 0, r.bytes, stream));  // status words start at zero
        }
        next_status_clean = true;
    }
    if (h_res_bytes < res_bytes) {
        if (h_res) BSR_HIP(hipHostFree(h_res));
        h_res = nullptr;
        h_res_bytes = 0;
        // fine-grained: the rescore kernels write the result rows into it and the publishing
        // kernel the status words, and the host reads it while the stream may still be
        // finishing (the flag, not the completion signal, says the bytes are there)
        BSR_HIP(hipHostMalloc((void**)&h_res, res_bytes, hipHostMallocCoherent));
        BSR_HIP(hipHostGetDevicePointer((void**)&h_res_dev, h_res, 0));
        h_res_bytes = res_bytes;
        ++g_alloc_gen;
    }
    if (!h_flag) {
        BSR_HIP(hipHostMalloc((void**)&h_flag, 64, hipHostMallocCoherent));
        BSR_HIP(hipHostGetDevicePointer((void**)&h_flag_dev, h_flag, 0));
        *h_flag = 0;
        BSR_TRY(pub_ticket.ensure(kTicketWords * sizeof(uint32_t)));
        BSR_HIP(hipMemsetAsync(pub_ticket.p, 0, kTicketWords * sizeof(uint32_t), stream));
        ++g_alloc_gen;
    }
    cur ^= 1u;
    uint8_t* rb = res[cur].as<uint8_t>();
    d_status = reinterpret_cast<uint32_t*>(rb);
    d_cnt = reinterpret_cast<uint32_t*>(rb + res_off_cnt);
    d_dist = reinterpret_cast<float*>(rb + res_off_dist);
    d_idx = reinterpret_cast<uint64_t*>(rb + res_off_idx);
    d_x = reinterpret_cast<float*>(rb + res_off_x);
    if (!next_status_clean) BSR_HIP(hipMemsetAsync(d_status, 0, kStWords * sizeof(uint32_t), stream));
    next_status_clean = false;
    return BSR_OK;
}

int bsr_index::search_device(const float* queries, uint32_t nq, uint32_t k, int (*after_launch)(void*),
                             void* ctx) {
    bsr_index* ix = this;
    if (!ix->loaded) return set_error(BSR_E_STATE, "index not loaded");
    if (k == 0 || k > ix->cfg.max_k) return set_error(BSR_E_INVALID, "k=%u outside [1, max_k=%u]", k, ix->cfg.max_k);
    BSR_HIP(hipSetDevice(ix->device));
    stats = bsr_search_stats{};
    stats.n_queries = nq;
    stats.filter_op = 0;  // int8
    stats.row_ebound = row_ebound;
    BSR_TRY(prepare_result(nq, k));
    uint32_t* next_status = res[cur ^ 1u].as<uint32_t>();
    if (nq == 0) return BSR_OK;
    if (!queries) return set_error(BSR_E_INVALID, "null queries");

    // queries padded to the filter's 256-query tile; batches of <= 16 (the skinny kernels read
    // query rows 0..15 only) to 16, so that the per-query kernels launch 16 workgroups, not 256
    const uint32_t qpad = nq <= kSkinnyMaxQ ? kSkinnyMaxQ : (uint32_t)round_up(nq, kFilterTile);
    BSR_TRY(qf32.ensure((size_t)qpad * ld * sizeof(float)));
    BSR_TRY(nb.ensure((size_t)qpad * sizeof(float)));
    BSR_TRY(qop.ensure((size_t)qpad * op_row_bytes));
    BSR_TRY(qscale.ensure((size_t)qpad * sizeof(float)));
    BSR_TRY(ebound.ensure((size_t)qpad * sizeof(float)));
    BSR_TRY(qflags.ensure((size_t)qpad * sizeof(uint32_t)));
    BSR_TRY(qids_id.ensure((size_t)qpad * sizeof(int32_t)));
    BSR_TRY(keys.ensure((size_t)nq * k * sizeof(uint64_t)));

    ev_begin(ix, ev_total);
    const float* qsrc = queries;
    if (!is_device_ptr(queries)) {
        BSR_TRY(q_in.ensure((size_t)nq * dim * sizeof(float)));
        BSR_HIP(hipMemcpyAsync(q_in.p, queries, (size_t)nq * dim * sizeof(float), hipMemcpyHostToDevice, stream));
        qsrc = q_in.as<float>();
    }
    // (the status words of res[cur] were zeroed by the previous search's finalize)
    // every batch is filtered (batches of <= 16 queries by the skinny kernels)
    const bool use_filter = n > 0 && approx_ok && k <= kMaxKForFilter;
    QueryPrepArgs qa{};
    qa.q = qsrc;
    qa.nq = nq;
    qa.qpad = qpad;
    qa.dim = dim;
    qa.ld = ld;
    qa.ea_max = flags.as<uint32_t>() + 1;
    qa.qf32 = qf32.as<float>();
    qa.nb = nb.as<float>();
    qa.qop = qop.p;
    qa.qscale = qscale.as<float>();
    qa.ebound = ebound.as<float>();
    qa.qflags = qflags.as<uint32_t>();
    qa.qids = qids_id.as<int32_t>();
    qa.status = d_status;
    qa.with_op = use_filter;
    // The filtered path publishes its result: the rescore kernels write every result row into
    // the pinned host mirror as well, and the last kernel copies the status words there and
    // raises a host flag, which the host polls -- no D2H copy node, no wait for the stream's
    // completion signal.  Profile level 2 (every stage evented) keeps the D2H
    // copy and the stream wait.
    const bool publish = use_filter && n > 0 && (!profiling(ix) || prof_level <= 1);
    // prep -> local search -> finalize -> one D2H copy of the packed result (graph-capturable:
    // no allocation and no host synchronisation once the buffers are sized)
    auto enqueue_search = [&]() -> int {
        BSR_HIP(launch_query_prep(qa, stream));
        if (n == 0) {
            // Empty shard (e.g. a rank whose interval_by_rank block is empty): no results.
            BSR_HIP(hipMemsetAsync(keys.p, 0xff, (size_t)nq * k * sizeof(uint64_t), stream));
        } else if (!use_filter) {
            stats.n_exact_direct = nq;
            BSR_TRY(run_exact_scan(ix, qids_id.as<int32_t>(), nq, k));
        } else {
            // (the rescore kernels write the result rows and the status bookkeeping)
            BSR_TRY(run_filter(ix, nq, qpad, k, next_status, publish));
        }
        if (!(use_filter && n > 0))
            BSR_HIP(launch_finalize(keys.as<uint64_t>(), nq, k, n, global_offset, d_idx, d_dist, d_cnt, next_status,
                                    nullptr, d_status, stream));
        ev_end(ix, ev_total);
        if (!publish) BSR_HIP(hipMemcpyAsync(h_res, res[cur].p, res_bytes, hipMemcpyDeviceToHost, stream));
        return BSR_OK;
    };
    if (publish) __atomic_store_n(h_flag, 0u, __ATOMIC_RELEASE);  // (before any launch of this search)

    // Every filtered batch is graph-capturable; a timed search (profile level >= 1) launches
    // directly, its events recorded on the stream (launch_timed).
    const bool top = use_filter && top_slots(ix, nq, k) != 0;
    if (top) stats.search_path |= BSR_PATH_SKINNY_TOP;
    const bool graphable = use_filter && n > 0 && (!profiling(ix) || prof_level == 0) && !force_threshold;
    SearchGraph& gs = graphs[cur];
    // (the graph key: the TOP row layout and the skinny filter's A/B switch, both read per search)
    const uint32_t lay = (top ? top_layout_lab() : 2u) | (skinny_glds_on() ? 0x100u : 0u);
    const bool same_shape = warm.nq == nq && warm.k == k && warm.qsrc == qsrc && warm.n == n &&
                            warm.timed == (profiling(ix) ? prof_level : 0) && warm.top == top &&
                            warm.top_layout == lay;
    const int timed_level = profiling(ix) ? prof_level : 0;
    if (graphable && gs.exec && gs.nq == nq && gs.k == k && gs.qsrc == qsrc && gs.n == n && gs.gen == g_alloc_gen &&
        gs.timed == timed_level && gs.top == top && gs.top_layout == lay) {
        BSR_HIP(hipGraphLaunch(gs.exec, stream));
        stats.n_candidates = kp_for(k);
        ++graph_replays;
        stats.graph_replay = 1;
    } else if (graphable && same_shape && warm.gen == g_alloc_gen) {
        // capture (every buffer already sized by the direct search of this shape), then replay
        if (gs.exec) { (void)hipGraphExecDestroy(gs.exec); gs.exec = nullptr; }
        BSR_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
        const uint64_t gen0 = g_alloc_gen;
        capturing = true;
        const int rc = enqueue_search();
        capturing = false;
        hipGraph_t graph = nullptr;
        const hipError_t ec = hipStreamEndCapture(stream, &graph);
        if (rc != BSR_OK) { if (graph) (void)hipGraphDestroy(graph); return rc; }
        if (ec != hipSuccess || g_alloc_gen != gen0) {
            if (graph) (void)hipGraphDestroy(graph);
            return set_error(BSR_E_HIP, "search graph capture failed: %s", hipGetErrorString(ec));
        }
        hipGraphExec_t exec = nullptr;
        const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (ei != hipSuccess) return set_error(BSR_E_HIP, "hipGraphInstantiate: %s", hipGetErrorString(ei));
        gs = SearchGraph{exec, nq, k, qsrc, n, g_alloc_gen, timed_level, top, lay};
        BSR_HIP(hipGraphLaunch(gs.exec, stream));
        ++graph_replays;
        stats.graph_replay = 1;
    } else {
        BSR_TRY(enqueue_search());
        if (graphable) warm = SearchGraph{nullptr, nq, k, qsrc, n, g_alloc_gen, timed_level, top, lay};
    }
    next_status_clean = true;
    int hook_st = BSR_OK;
    if (after_launch) hook_st = after_launch(ctx);
    if (publish) {
        const hipError_t r = flag_wait(h_flag, stream);
        if (r == hipErrorUnknown) return set_error(BSR_E_HIP, "the search's stream finished without publishing its result");
        BSR_HIP(r);
    } else {
        BSR_HIP(stream_wait(stream));
    }
    if (hook_st != BSR_OK) return hook_st;
    // Later rounds (second-chance rescore, scan) finalize and read back again, directly.
    auto finalize_and_read = [&]() -> int {
        BSR_HIP(launch_finalize(keys.as<uint64_t>(), nq, k, n, global_offset, d_idx, d_dist, d_cnt, next_status,
                                nullptr, d_status, stream));
        next_status_clean = true;
        BSR_HIP(hipMemcpyAsync(h_res, res[cur].p, res_bytes, hipMemcpyDeviceToHost, stream));
        BSR_HIP(hipStreamSynchronize(stream));
        return BSR_OK;
    };
    std::vector<int32_t> exact_ids;
    const uint32_t* st = reinterpret_cast<const uint32_t*>(h_res);
    if (st[kStQueryFlags] & kQueryNonFinite) {
        h_qflags.resize(nq);
        BSR_HIP(hipMemcpy(h_qflags.data(), qflags.p, (size_t)nq * sizeof(uint32_t), hipMemcpyDeviceToHost));
        uint32_t bad = 0;
        while (bad < nq && !(h_qflags[bad] & kQueryNonFinite)) ++bad;
        return set_error(BSR_E_NONFINITE, "query %u contains NaN/Inf (the reference panics)", bad);
    }
    if (use_filter) {
        stats.n_emitted = st[kStEmitted];
        // st[kStFail] queries failed the first certification and were rescored over every
        // emitted row in the same launch sequence; st[kStFail2] of them failed again.
        const uint32_t nfail = st[kStFail2];
        const uint32_t* fail_dev = fail2.as<uint32_t>();
        stats.n_rescued = st[kStFail] - nfail;
        if (nfail) {
            // Uncertified queries, and queries the filter cannot serve (zero/tiny/huge |b|),
            // take the exact full scan: the reference's arithmetic on every row.
            h_fail.resize(nfail);
            h_qflags.resize(nq);
            BSR_HIP(hipMemcpyAsync(h_fail.data(), fail_dev, (size_t)nfail * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   stream));
            BSR_HIP(hipMemcpyAsync(h_qflags.data(), qflags.p, (size_t)nq * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   stream));
            BSR_HIP(hipStreamSynchronize(stream));
            bool served_failed = false;
            for (uint32_t q : h_fail) served_failed |= !(h_qflags[q] & kQueryNoApprox);
            if (top && served_failed) {
                // The self-thresholded path left a query it serves uncertified (more than a wave's 4
                // best of its rows lie near the top: a cluster of near-duplicates): the batch again
                // on the thresholded path, directly launched, whose own failures take the exact scan.
                force_threshold = true;
                const int r = search_device(queries, nq, k);
                force_threshold = false;
                stats.search_path |= BSR_PATH_SKINNY_TOP | BSR_PATH_TOP_RERUN;
                return r;
            }
            std::sort(h_fail.begin(), h_fail.end());
            for (uint32_t q : h_fail) {
                exact_ids.push_back((int32_t)q);
                if (h_qflags[q] & kQueryNoApprox) ++stats.n_exact_direct;
                else ++stats.n_fallback;
            }
            BSR_TRY(run_exact_scan_list(ix, exact_ids, k));
            BSR_TRY(finalize_and_read());
        }
    }
    return BSR_OK;
}

// ---------------------------------------------------------------------------------------
// The parallel search's global emission threshold: phase A / phase B
// ---------------------------------------------------------------------------------------
bool bsr_index::gtau_eligible(uint32_t nq, uint32_t k) const {
    // the filter path with a sample pass (a shard of more rows than one query's candidate list)
    return loaded && nq > 0 && k >= 1 && k <= cfg.max_k && k <= kMaxKForFilter && approx_ok && n > cap_for(k);
}

// Phase A's buffers (the result buffer of this search, the query and filter scratch, the sample
// scores, the ks best keys): everything that can fail short of a device error, done before the
// parallel search posts its header -- which is then posted before phase A's kernels, so that
// its round trip overlaps them (round 5: posted after them it could finish behind the sample
// pass and hold the host's enqueue of phase B, +25 us per search in the loopback timeline).
int bsr_index::gtau_prepare(const float* queries, uint32_t nq, uint32_t k) {
    if (!gtau_eligible(nq, k)) return set_error(BSR_E_STATE, "global-threshold search not applicable");
    if (!queries) return set_error(BSR_E_INVALID, "null queries");
    BSR_HIP(hipSetDevice(device));
    stats = bsr_search_stats{};
    stats.n_queries = nq;
    stats.row_ebound = row_ebound;
    BSR_TRY(prepare_result(nq, k));
    const uint32_t qpad = (uint32_t)round_up(nq, kFilterTile);
    const uint32_t ks = ks_for(k);
    BSR_TRY(qf32.ensure((size_t)qpad * ld * sizeof(float)));
    BSR_TRY(nb.ensure((size_t)qpad * sizeof(float)));
    BSR_TRY(qop.ensure((size_t)qpad * op_row_bytes));
    BSR_TRY(qscale.ensure((size_t)qpad * sizeof(float)));
    BSR_TRY(ebound.ensure((size_t)qpad * sizeof(float)));
    BSR_TRY(qflags.ensure((size_t)qpad * sizeof(uint32_t)));
    BSR_TRY(qids_id.ensure((size_t)qpad * sizeof(int32_t)));
    BSR_TRY(keys.ensure((size_t)nq * k * sizeof(uint64_t)));
    BSR_TRY(smax.ensure((size_t)qpad * ks * sizeof(uint64_t)));
    if (!is_device_ptr(queries)) BSR_TRY(q_in.ensure((size_t)nq * dim * sizeof(float)));
    BSR_TRY(filter_buffers(this, nq, qpad, k));
    const uint32_t n_s = (uint32_t)((n + kSampleStride - 1) / kSampleStride);
    const uint32_t n_rt_s = (n_s + kFilterTile - 1) / kFilterTile;
    const bool compact = n_s >= 32u * 8u * ks;
    const uint32_t s_ld = compact ? n_rt_s * (kFilterTile / 32) : n_rt_s * kFilterTile;
    BSR_TRY(S.ensure((size_t)qpad * s_ld * sizeof(float)));  // (sample_pass's size)
    gt_nq = nq;
    gt_k = k;
    gt_qpad = qpad;
    gt_ks = ks;
    return BSR_OK;
}

// Phase A's work, enqueued (after gtau_prepare sized every buffer: nothing is allocated here), in
// two parts so that the parallel search can post its header between them: the query prep (the
// GPU starts on it while the host issues the header's launches), then the sample pass and tau0.
int bsr_index::gtau_phase_a(const float* queries, int part) {
    bsr_index* ix = this;
    const uint32_t nq = gt_nq, k = gt_k, qpad = gt_qpad;
    if (part == 1) {
        BSR_TRY(sample_pass(ix, nq, qpad, k, smax.as<uint64_t>()));
        return BSR_OK;
    }
    const float* qsrc = queries;
    if (!is_device_ptr(queries)) {
        BSR_HIP(hipMemcpyAsync(q_in.p, queries, (size_t)nq * dim * sizeof(float), hipMemcpyHostToDevice, stream));
        qsrc = q_in.as<float>();
    }
    ev_begin(ix, ev_total);
    QueryPrepArgs qa{};
    qa.q = qsrc;
    qa.nq = nq;
    qa.qpad = qpad;
    qa.dim = dim;
    qa.ld = ld;
    qa.ea_max = flags.as<uint32_t>() + 1;
    qa.qf32 = qf32.as<float>();
    qa.nb = nb.as<float>();
    qa.qop = qop.p;
    qa.qscale = qscale.as<float>();
    qa.ebound = ebound.as<float>();
    qa.qflags = qflags.as<uint32_t>();
    qa.qids = qids_id.as<int32_t>();
    qa.status = d_status;
    qa.with_op = true;
    BSR_HIP(launch_query_prep(qa, stream));
    return BSR_OK;
}

int bsr_index::gtau_phase_b(const uint64_t* g_smax, uint32_t P, uint32_t* merge_words) {
    bsr_index* ix = this;
    const uint32_t nq = gt_nq, k = gt_k, qpad = gt_qpad;
    BSR_HIP(launch_global_tau(g_smax, P, qpad, nq, gt_ks, qflags.as<uint32_t>(), tau.as<float>(), stream));
    BSR_TRY(emit_pass(ix, nq, qpad, k));
    // every emitted row rescored exactly, one wave per query (mode B); the list is this rank's
    // contribution, its exclusion bound goes with it (the root certifies the merged lists)
    ev_begin(ix, ev_rescore);
    RescoreArgs ra{};
    ra.rows = rows.as<float>();
    ra.ld = ld;
    ra.dim = dim;
    ra.na = na.as<float>();
    ra.qf32 = qf32.as<float>();
    ra.nb = nb.as<float>();
    ra.n_items = nq;
    ra.cand_keys = cand.as<uint64_t>();
    ra.cnt = cnt.as<uint32_t>();
    ra.cap = cap_for(k);
    ra.tau0 = tau.as<float>();
    ra.kp = kp_for(k);
    ra.k = k;
    ra.ebound = ebound.as<float>();
    ra.out_keys = keys.as<uint64_t>();
    ra.res_idx = d_idx;
    ra.res_dist = d_dist;
    ra.res_cnt = d_cnt;
    ra.offset = global_offset;
    ra.n_rows = n;
    ra.excl_out = d_x;
    ra.next_status = res[cur ^ 1u].as<uint32_t>();
    ra.emit_cnt = cnt.as<uint32_t>();
    ra.cur_status = d_status;
    ra.n_queries = nq;
    ra.merge_words = merge_words;  // (the merge's two words: no memset launches before it)
    BSR_HIP(launch_rescore(ra, stream));
    ev_end(ix, ev_rescore);
    ev_end(ix, ev_total);  // (the local part: phases A and B, the all-gather between them included)
    next_status_clean = true;
    return BSR_OK;
}

// Results of the last search to the caller's arrays: from the pinned host mirror for host
// arrays, device-to-device for device arrays.
static int copy_out(bsr_index* ix, uint32_t nq, uint32_t k, uint64_t* out_idx, float* out_dist, uint32_t* out_count) {
    const size_t nk = (size_t)nq * k;
    const bool dev = is_device_ptr(out_idx) || is_device_ptr(out_dist) || is_device_ptr(out_count);
    if (!dev) {
        if (out_idx) memcpy(out_idx, ix->h_res + ix->res_off_idx, nk * sizeof(uint64_t));
        if (out_dist) memcpy(out_dist, ix->h_res + ix->res_off_dist, nk * sizeof(float));
        if (out_count) memcpy(out_count, ix->h_res + ix->res_off_cnt, (size_t)nq * sizeof(uint32_t));
        return BSR_OK;
    }
    if (out_idx) BSR_HIP(hipMemcpyAsync(out_idx, ix->d_idx, nk * sizeof(uint64_t), hipMemcpyDefault, ix->stream));
    if (out_dist) BSR_HIP(hipMemcpyAsync(out_dist, ix->d_dist, nk * sizeof(float), hipMemcpyDefault, ix->stream));
    if (out_count) BSR_HIP(hipMemcpyAsync(out_count, ix->d_cnt, (size_t)nq * sizeof(uint32_t), hipMemcpyDefault, ix->stream));
    BSR_HIP(hipStreamSynchronize(ix->stream));
    return BSR_OK;
}

int bsr_copy_out_impl(bsr_index* ix, uint32_t nq, uint32_t k, uint64_t* out_idx, float* out_dist,
                      uint32_t* out_count) {
    return copy_out(ix, nq, k, out_idx, out_dist, out_count);
}

static void collect_profile(bsr_index* ix) {
    if (!profiling(ix)) return;
    bsr_profile& p = ix->prof;
    ev_collect(ix->ev_emit, p.gemm_emit_ms, p.gemm_emit_launches, 1);
    ev_collect(ix->ev_sample, p.gemm_sample_ms, p.gemm_sample_launches, 1);
    ev_collect(ix->ev_select, p.select_ms, p.select_launches, 1);
    ev_collect(ix->ev_rescore, p.rescore_ms, p.rescore_launches, 1);
    ev_collect(ix->ev_scan, p.scan_ms, p.scan_launches, 1);
    ev_collect(ix->ev_total, p.search_ms, p.searches, 1);
}

int bsr_local_top_k_impl(bsr_index* ix, const float* queries, uint32_t nq, uint32_t k, uint64_t* out_idx,
                         float* out_dist, uint32_t* out_count) {
    if (!ix) return set_error(BSR_E_INVALID, "null index");
    if (nq && (!out_idx || !out_dist || !out_count)) return set_error(BSR_E_INVALID, "null output");
    BSR_TRY(ix->search_device(queries, nq, k));
    BSR_TRY(copy_out(ix, nq, k, out_idx, out_dist, out_count));
    collect_profile(ix);
    return BSR_OK;
}

int bsr_index_collect_profile_impl(bsr_index* ix) {
    collect_profile(ix);
    return BSR_OK;
}
