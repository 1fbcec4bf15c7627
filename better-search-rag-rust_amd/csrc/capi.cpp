// capi.cpp -- the C ABI (include/bsr.h): argument checks, exception firewall, the RCCL
// communicator, gather (src/mpi_helpers/metrics.rs:56-138), the host merge
// (:141-171) and the composed parallel search (:174-206).
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "internal.hpp"
#include "kernels.hpp"
#include "merge.hpp"

namespace bsr {
const char* last_error_cstr();
}
using namespace bsr;

int bsr_index_create_impl(const bsr_config* cfg, bsr_index** out);
void bsr_index_destroy_impl(bsr_index* ix);
int bsr_index_load_impl(bsr_index* ix, const void* rows, uint64_t n_rows, uint64_t global_offset);
int bsr_index_append_impl(bsr_index* ix, const void* rows, uint64_t n_rows);
int bsr_index_get_many_impl(const bsr_index* ix, uint64_t offset, uint64_t count, float* out);
int bsr_local_top_k_impl(bsr_index* ix, const float* queries, uint32_t nq, uint32_t k, uint64_t* out_idx,
                         float* out_dist, uint32_t* out_count);
int bsr_index_collect_profile_impl(bsr_index* ix);
int bsr_copy_out_impl(bsr_index* ix, uint32_t nq, uint32_t k, uint64_t* out_idx, float* out_dist,
                      uint32_t* out_count);

#define BSR_GUARD(expr)                                                        \
    try {                                                                      \
        clear_error();                                                         \
        return (expr);                                                         \
    } catch (const std::bad_alloc&) {                                          \
        return set_error(BSR_E_NOMEM, "host allocation failed");               \
    } catch (...) {                                                            \
        return set_error(BSR_E_INVALID, "internal error (exception)");         \
    }

// Host memory for the gathered lists that grows on demand: pinned when a HIP device is
// present (the RCCL path copies into it; pageable vectors would make those copies staged and
// synchronous), plain memory otherwise (a host-transport communicator on a CPU-only node).
template <class T>
struct PinnedVec {
    T* p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    PinnedVec() = default;
    PinnedVec(const PinnedVec&) = delete;
    PinnedVec& operator=(const PinnedVec&) = delete;
    ~PinnedVec() { release(); }
    void release() {
        if (p && pinned) (void)hipHostFree(p);
        else free(p);
        p = nullptr;
        cap = 0;
    }
    int resize(size_t n) {
        if (n <= cap) return BSR_OK;
        release();
        const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
        void* q = nullptr;
        pinned = hipHostMalloc(&q, bytes, hipHostMallocDefault) == hipSuccess;
        if (!pinned) {
            (void)hipGetLastError();  // (no device: clear the sticky error)
            q = malloc(bytes);
        }
        if (!q) return set_error(BSR_E_NOMEM, "host allocation of %zu bytes failed", bytes);
        p = static_cast<T*>(q);
        cap = n;
        return BSR_OK;
    }
    T* data() { return p; }
    const T* data() const { return p; }
};

// The rank group of the exchange step: RCCL over xGMI (one GPU per rank), or a host
// transport given by the caller (bsr_comm_init_host: e.g. gloo/MPI stand-ins on CPU).
struct bsr_comm {
    ncclComm_t comm = nullptr;
    int32_t rank = 0, size = 1, device = -1;
    hipStream_t stream = nullptr;
    bsr_host_allgather_fn host_fn = nullptr;  // non-null: host transport
    void* host_user = nullptr;
    DevBuf send_idx, send_dist, send_cnt, recv_idx, recv_dist, recv_cnt;
    PinnedVec<uint64_t> h_idx;     // root: gathered [size][nq][k]
    PinnedVec<float> h_dist;
    PinnedVec<uint32_t> h_cnt;     // root: [size][nq]
    std::vector<uint8_t> h_send, h_recv;  // host transport packing
    std::vector<uint64_t> m_idx;   // root merge output staging (device outputs)
    std::vector<float> m_dist;
    std::vector<uint32_t> m_cnt;
    DevBuf nan_word;               // device merge: the lowest query with a NaN distance
    PinnedVec<uint32_t> h_nan;
    DevBuf hdr_send, hdr_recv;     // the parallel search's shape agreement (RCCL)
    PinnedVec<int32_t> h_hdr;      // [1 + size][kHdrWords]: this rank's words, then every rank's
    bool hdr_posted = false;       // this search's header all-gather has been issued
    // (device transports) the received headers, published by k_header_publish into fine-grained
    // pinned memory [size][kHdrWords], and the flag it raises to the search's sequence number
    int32_t* hdr_host = nullptr;
    int32_t* hdr_host_dev = nullptr;
    uint32_t* hdr_flag = nullptr;
    uint32_t* hdr_flag_dev = nullptr;
    uint32_t hdr_seq = 0;
    // the global-threshold search (parallel_gtau): gathered sample keys, gathered result
    // buffers, the merged result (device and pinned host)
    DevBuf g_smax, g_res, m_res, pub_ticket;
    PinnedVec<uint8_t> h_stage;
    uint8_t* h_mres = nullptr;      // fine-grained pinned: the merge kernel publishes into it
    uint8_t* h_mres_dev = nullptr;
    size_t h_mres_bytes = 0;
    uint32_t* h_flag = nullptr;     // fine-grained host word the merge kernel raises
    uint32_t* h_flag_dev = nullptr;
    // the uncertified queries' staging (parallel_gtau), reserved before the header is posted
    std::vector<float> f_q, f_dist;
    std::vector<uint64_t> f_idx;
    std::vector<uint32_t> f_cnt, f_list;
    // bsr_comm_init_loopback: one process, every collective emulated on the device (no RCCL).
    // Without a script each all-gather replicates this rank's contribution P times; with one,
    // the parallel search's all-gathers replay the recorded contributions of a real P-rank run
    // (lb_bytes[i] bytes per rank, [P][bytes] at lb_script + lb_off[i]) in their order, this
    // rank's own slot always live.
    bool loopback = false;
    DevBuf lb_script;
    std::vector<uint64_t> lb_bytes, lb_off;
    size_t lb_cursor = 0;
    bool lb_search = false, lb_live = false;
    int32_t lb_nq = -1, lb_k = -1;  // the recorded search's batch shape (its header): replayed only for it
    uint64_t lb_replayed = 0, lb_missed = 0;
    uint64_t lb_qdigest = 0;  // FNV-1a of the first host query batch replayed
    bool lb_qdigest_set = false;
    ~bsr_comm() {
        if (h_mres) (void)hipHostFree(h_mres);
        if (h_flag) (void)hipHostFree(h_flag);
        if (hdr_host) (void)hipHostFree(hdr_host);
        if (hdr_flag) (void)hipHostFree(hdr_flag);
    }
};

// The parallel search's header, all-gathered before the lists: every rank's batch shape
// and local status, so that no rank issues a list exchange the others do not match.
constexpr size_t kHdrWords = 8;  // {n_queries, k, local status, magic, gtau, rows lo, rows hi, 0}
constexpr int32_t kHdrMagic = 0x42535231;

// Copy to a caller buffer that may be host or device memory.
#define BSR_HIP_OR_HOST_COPY(dst, src, bytes)                                            \
    do {                                                                                 \
        if (is_device_ptr(dst)) BSR_HIP(hipMemcpy((dst), (src), (bytes), hipMemcpyHostToDevice)); \
        else memcpy((dst), (src), (bytes));                                              \
    } while (0)

#define BSR_HIP_OR_HOST_COPY_FROM(dst, src, bytes)                                       \
    do {                                                                                 \
        if (is_device_ptr(src)) BSR_HIP(hipMemcpy((dst), (src), (bytes), hipMemcpyDeviceToHost)); \
        else memcpy((dst), (src), (bytes));                                              \
    } while (0)

#define BSR_NCCL(call)                                                                          \
    do {                                                                                        \
        ncclResult_t r_ = (call);                                                               \
        if (r_ != ncclSuccess)                                                                  \
            return set_error(BSR_E_RCCL, "%s failed: %s", #call, ncclGetErrorString(r_));       \
    } while (0)

// One all-gather of `bytes` device bytes per rank on `stream`: RCCL, or the loopback
// communicator's emulation (one kernel on the same stream, where ncclAllGather would sit).
static int coll_allgather(bsr_comm* c, const void* send, void* recv, size_t bytes, hipStream_t stream) {
    if (!c->loopback) {
        BSR_NCCL(ncclAllGather(send, recv, bytes, ncclUint8, c->comm, stream));
        return BSR_OK;
    }
    const void* script = nullptr;
    if (c->lb_search && c->lb_live && !c->lb_bytes.empty()) {
        if (c->lb_cursor < c->lb_bytes.size() && c->lb_bytes[c->lb_cursor] == bytes) {
            script = c->lb_script.as<uint8_t>() + c->lb_off[c->lb_cursor++];
            ++c->lb_replayed;
        } else {  // (the recording ends, or another call sequence: replicate from here on)
            c->lb_live = false;
            ++c->lb_missed;
        }
    }
    BSR_HIP(launch_gather_emulate(send, script, recv, bytes, (uint32_t)c->size, (uint32_t)c->rank, stream));
    return BSR_OK;
}
static int coll_group(bsr_comm* c, bool start) {
    if (c->loopback) return BSR_OK;
    if (start) BSR_NCCL(ncclGroupStart());
    else BSR_NCCL(ncclGroupEnd());
    return BSR_OK;
}

// The parallel search's header buffers, allocated with the communicator: posting a header can
// then fail only in the transport, which every rank sees.
constexpr size_t kHdrWordsInit = 8;
static int alloc_header(bsr_comm* c) {
    const size_t P = (size_t)c->size, hb = kHdrWordsInit * sizeof(int32_t);
    BSR_TRY(c->h_hdr.resize(kHdrWordsInit * (1 + P)));
    if (!c->host_fn) {
        BSR_TRY(c->hdr_send.ensure(hb));
        BSR_TRY(c->hdr_recv.ensure(hb * P));
        BSR_HIP(hipHostMalloc((void**)&c->hdr_host, hb * P, hipHostMallocCoherent));
        BSR_HIP(hipHostGetDevicePointer((void**)&c->hdr_host_dev, c->hdr_host, 0));
        BSR_HIP(hipHostMalloc((void**)&c->hdr_flag, 64, hipHostMallocCoherent));
        BSR_HIP(hipHostGetDevicePointer((void**)&c->hdr_flag_dev, c->hdr_flag, 0));
        __atomic_store_n(c->hdr_flag, 0u, __ATOMIC_RELEASE);
    }
    return BSR_OK;
}

// ---------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------
extern "C" {

const char* bsr_last_error(void) { return last_error_cstr(); }

const char* bsr_status_string(int s) {
    switch (s) {
        case BSR_OK: return "BSR_OK";
        case BSR_PARTIAL: return "BSR_PARTIAL";
        case BSR_E_INVALID: return "BSR_E_INVALID";
        case BSR_E_NONFINITE: return "BSR_E_NONFINITE";
        case BSR_E_HIP: return "BSR_E_HIP";
        case BSR_E_NOMEM: return "BSR_E_NOMEM";
        case BSR_E_RCCL: return "BSR_E_RCCL";
        case BSR_E_DIM: return "BSR_E_DIM";
        case BSR_E_STATE: return "BSR_E_STATE";
        case BSR_E_NODEVICE: return "BSR_E_NODEVICE";
        default: return "BSR_E_UNKNOWN";
    }
}

const char* bsr_version(void) { return "bsr-mi355x 0.1.0 (gfx950)"; }

int bsr_device_count(int* out_count) {
    if (!out_count) return set_error(BSR_E_INVALID, "null argument");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        n = 0;
    }
    *out_count = n;
    return BSR_OK;
}

static int cosine_distance_impl(const float* a, uint32_t la, const float* b, uint32_t lb, float* out) {
    if (!out || (la && !a) || (lb && !b)) return set_error(BSR_E_INVALID, "null argument");
    BSR_TRY(select_device(-1));
    DevBuf da, db, dout;
    const float* pa = a;
    const float* pb = b;
    if (la && !is_device_ptr(a)) {
        BSR_TRY(da.ensure(la * sizeof(float)));
        BSR_HIP(hipMemcpy(da.p, a, la * sizeof(float), hipMemcpyHostToDevice));
        pa = da.as<float>();
    }
    if (lb && !is_device_ptr(b)) {
        BSR_TRY(db.ensure(lb * sizeof(float)));
        BSR_HIP(hipMemcpy(db.p, b, lb * sizeof(float), hipMemcpyHostToDevice));
        pb = db.as<float>();
    }
    BSR_TRY(dout.ensure(sizeof(float)));
    BSR_HIP(launch_cosine_pair(pa, la, pb, lb, dout.as<float>(), nullptr));
    BSR_HIP(hipMemcpy(out, dout.p, sizeof(float), hipMemcpyDefault));
    return BSR_OK;
}

int bsr_cosine_distance(const float* a, uint32_t len_a, const float* b, uint32_t len_b, float* out) {
    BSR_GUARD(cosine_distance_impl(a, len_a, b, len_b, out));
}

int bsr_interval_by_rank(int32_t rank, int32_t size, uint64_t count, bsr_rank_interval* out) {
    // src/mpi_helpers/load_balance.rs:24-42
    if (!out || size < 1 || rank < 0 || rank >= size) return set_error(BSR_E_INVALID, "bad rank/size");
    const uint64_t per = ((uint64_t)size > count) ? 1 : (count + (uint64_t)size - 1) / (uint64_t)size;
    const uint64_t start = per * (uint64_t)rank;
    uint64_t end = (rank == size - 1) ? count : std::min(start + per, count);
    out->start_index = start;
    out->end_index = end;
    return BSR_OK;
}

int bsr_index_create(const bsr_config* cfg, bsr_index** out) { BSR_GUARD(bsr_index_create_impl(cfg, out)); }
void bsr_index_destroy(bsr_index* ix) {
    try { bsr_index_destroy_impl(ix); } catch (...) {}
}
int bsr_index_load(bsr_index* ix, const void* rows, uint64_t n_rows, uint64_t global_offset) {
    BSR_GUARD(bsr_index_load_impl(ix, rows, n_rows, global_offset));
}
int bsr_index_append(bsr_index* ix, const void* rows, uint64_t n_rows) {
    BSR_GUARD(bsr_index_append_impl(ix, rows, n_rows));
}
int bsr_index_count(const bsr_index* ix, uint64_t* out) {
    if (!ix || !out) return set_error(BSR_E_INVALID, "null argument");
    *out = ix->loaded ? ix->n : 0;
    return BSR_OK;
}
int bsr_index_dim(const bsr_index* ix, uint32_t* out) {
    if (!ix || !out) return set_error(BSR_E_INVALID, "null argument");
    *out = ix->dim;
    return BSR_OK;
}
int bsr_index_global_offset(const bsr_index* ix, uint64_t* out) {
    if (!ix || !out) return set_error(BSR_E_INVALID, "null argument");
    *out = ix->global_offset;
    return BSR_OK;
}
int bsr_index_get_many(const bsr_index* ix, uint64_t offset, uint64_t count, float* out) {
    BSR_GUARD(bsr_index_get_many_impl(ix, offset, count, out));
}

int bsr_local_top_k(bsr_index* ix, const float* queries, uint32_t n_queries, uint32_t k, uint64_t* out_idx,
                    float* out_dist, uint32_t* out_count) {
    BSR_GUARD(bsr_local_top_k_impl(ix, queries, n_queries, k, out_idx, out_dist, out_count));
}

// The device merge's limits (k_merge_lists: one wave per query, the concatenation in LDS).
static bool device_merge_fits(uint32_t P, uint32_t k_in, uint32_t k) {
    return P <= 64 && (uint64_t)P * k_in <= kMergeMaxEntries && k <= 256;
}

static int global_top_k_impl(const uint64_t* idx, const float* dist, const uint32_t* count, uint32_t n_lists,
                             uint32_t n_queries, uint32_t k_in, uint32_t k, uint64_t* out_idx, float* out_dist,
                             uint32_t* out_count) {
    if (!n_queries) return BSR_OK;
    if (!count || !out_idx || !out_dist || !out_count || (n_lists && k_in && (!idx || !dist)))
        return set_error(BSR_E_INVALID, "null argument");
    if (k == 0) return set_error(BSR_E_INVALID, "k must be >= 1");
    if (is_device_ptr(count)) {
        // every array in device memory: the merge kernel (the RCCL root's merge), on the
        // current device's null stream
        if (!is_device_ptr(out_idx) || !is_device_ptr(out_dist) || !is_device_ptr(out_count) ||
            (n_lists && k_in && (!is_device_ptr(idx) || !is_device_ptr(dist))))
            return set_error(BSR_E_INVALID, "device lists need device outputs");
        if (!device_merge_fits(n_lists, k_in, k))
            return set_error(BSR_E_INVALID, "device merge: n_lists <= 64, n_lists * k_in <= %u, k <= 256",
                             kMergeMaxEntries);
        DevBuf nan_word;
        BSR_TRY(nan_word.ensure(sizeof(uint32_t)));
        BSR_HIP(hipMemset(nan_word.p, 0xff, sizeof(uint32_t)));
        BSR_HIP(launch_merge_lists(idx, dist, count, n_lists, n_queries, k_in, k, out_idx, out_dist, out_count,
                                   nan_word.as<uint32_t>(), nullptr));
        uint32_t bad = 0;
        BSR_HIP(hipMemcpy(&bad, nan_word.p, sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (bad != ~0u) return set_error(BSR_E_NONFINITE, "NaN distance in query %u (the reference panics)", bad);
        return BSR_OK;
    }
    // host counts: every array must be host memory (the host merge dereferences them all)
    if (is_device_ptr(out_idx) || is_device_ptr(out_dist) || is_device_ptr(out_count) ||
        (n_lists && k_in && (is_device_ptr(idx) || is_device_ptr(dist))))
        return set_error(BSR_E_INVALID, "host counts need host lists and outputs (or pass every array on the device)");
    return merge_top_k_lists(ListsView{idx, dist, count, n_lists, n_queries, k_in}, n_queries, k, out_idx, out_dist,
                             out_count);
}

int bsr_global_top_k(const uint64_t* idx, const float* dist, const uint32_t* count, uint32_t n_lists,
                     uint32_t n_queries, uint32_t k_in, uint32_t k, uint64_t* out_idx, float* out_dist,
                     uint32_t* out_count) {
    BSR_GUARD(global_top_k_impl(idx, dist, count, n_lists, n_queries, k_in, k, out_idx, out_dist, out_count));
}

int bsr_comm_unique_id(uint8_t out_id[BSR_UNIQUE_ID_BYTES]) {
    if (!out_id) return set_error(BSR_E_INVALID, "null argument");
    static_assert(sizeof(ncclUniqueId) == BSR_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    BSR_NCCL(ncclGetUniqueId(&id));
    memcpy(out_id, &id, sizeof id);
    return BSR_OK;
}

static int comm_init_impl(const uint8_t id[BSR_UNIQUE_ID_BYTES], int32_t rank, int32_t size, int32_t device,
                          bsr_comm** out) {
    if (!id || !out || size < 1 || rank < 0 || rank >= size) return set_error(BSR_E_INVALID, "bad argument");
    *out = nullptr;
    BSR_TRY(select_device(device));
    bsr_comm* c = new bsr_comm();
    (void)hipGetDevice(&c->device);
    c->rank = rank;
    c->size = size;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    ncclResult_t r = ncclCommInitRank(&c->comm, size, uid, rank);
    if (r != ncclSuccess) {
        delete c;
        return set_error(BSR_E_RCCL, "ncclCommInitRank failed: %s", ncclGetErrorString(r));
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess) {  // blocking: see bsr_index
        ncclCommDestroy(c->comm);
        delete c;
        return set_error(BSR_E_HIP, "hipStreamCreate failed");
    }
    const int ra = alloc_header(c);
    if (ra != BSR_OK) {
        bsr_comm_destroy(c);
        return ra;
    }
    *out = c;
    return BSR_OK;
}

int bsr_comm_init(const uint8_t id[BSR_UNIQUE_ID_BYTES], int32_t rank, int32_t size, int32_t device,
                  bsr_comm** out) {
    BSR_GUARD(comm_init_impl(id, rank, size, device, out));
}

static int comm_init_host_impl(int32_t rank, int32_t size, bsr_host_allgather_fn fn, void* user, bsr_comm** out) {
    if (!out || !fn || size < 1 || rank < 0 || rank >= size) return set_error(BSR_E_INVALID, "bad argument");
    bsr_comm* c = new bsr_comm();
    c->rank = rank;
    c->size = size;
    c->host_fn = fn;
    c->host_user = user;
    const int ra = alloc_header(c);
    if (ra != BSR_OK) {
        delete c;
        return ra;
    }
    *out = c;
    return BSR_OK;
}

int bsr_comm_init_host(int32_t rank, int32_t size, bsr_host_allgather_fn fn, void* user, bsr_comm** out) {
    BSR_GUARD(comm_init_host_impl(rank, size, fn, user, out));
}

static int comm_init_loopback_impl(int32_t rank, int32_t size, int32_t device, uint32_t n_calls,
                                   const uint64_t* call_bytes, const void* script, bsr_comm** out) {
    if (!out || size < 1 || rank < 0 || rank >= size || (n_calls && (!call_bytes || !script)))
        return set_error(BSR_E_INVALID, "bad argument");
    *out = nullptr;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n_calls; ++i) {
        if (call_bytes[i] % 4) return set_error(BSR_E_INVALID, "recorded all-gather %u: bytes %% 4 != 0", i);
        total += call_bytes[i] * (uint64_t)size;
    }
    BSR_TRY(select_device(device));
    bsr_comm* c = new bsr_comm();
    (void)hipGetDevice(&c->device);
    c->rank = rank;
    c->size = size;
    c->loopback = true;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess) {
        delete c;
        return set_error(BSR_E_HIP, "hipStreamCreate failed");
    }
    int r = alloc_header(c);
    if (r == BSR_OK && n_calls) {
        r = c->lb_script.ensure(total);
        if (r == BSR_OK && hipMemcpy(c->lb_script.p, script, total, hipMemcpyHostToDevice) != hipSuccess)
            r = set_error(BSR_E_HIP, "loopback script upload failed");
        if (call_bytes[0] == 8 * sizeof(int32_t)) {  // the recorded header: this rank's {n_queries, k, ...}
            const int32_t* h = static_cast<const int32_t*>(script) + 8 * (size_t)rank;
            c->lb_nq = h[0];
            c->lb_k = h[1];
        }
        uint64_t off = 0;
        for (uint32_t i = 0; r == BSR_OK && i < n_calls; ++i) {
            c->lb_bytes.push_back(call_bytes[i]);
            c->lb_off.push_back(off);
            off += call_bytes[i] * (uint64_t)size;
        }
    }
    if (r != BSR_OK) {
        bsr_comm_destroy(c);
        return r;
    }
    *out = c;
    return BSR_OK;
}

int bsr_comm_init_loopback(int32_t rank, int32_t size, int32_t device, uint32_t n_calls, const uint64_t* call_bytes,
                           const void* script, bsr_comm** out) {
    BSR_GUARD(comm_init_loopback_impl(rank, size, device, n_calls, call_bytes, script, out));
}

int bsr_host_alloc(uint64_t bytes, void** out) {
    if (!out) return set_error(BSR_E_INVALID, "null argument");
    *out = nullptr;
    BSR_TRY(select_device(-1));
    BSR_HIP(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocCoherent));
    return BSR_OK;
}

void bsr_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int bsr_comm_loopback_stats(const bsr_comm* c, uint64_t* replayed, uint64_t* missed) {
    if (!c || !replayed || !missed) return set_error(BSR_E_INVALID, "null argument");
    if (!c->loopback) return set_error(BSR_E_INVALID, "not a loopback communicator");
    *replayed = c->lb_replayed;
    *missed = c->lb_missed;
    return BSR_OK;
}

void bsr_comm_destroy(bsr_comm* c) {
    if (!c) return;
    try {
        if (c->stream) {
            (void)hipSetDevice(c->device);
            (void)hipStreamSynchronize(c->stream);
            (void)hipStreamDestroy(c->stream);
        }
        if (c->comm) ncclCommDestroy(c->comm);
        delete c;
    } catch (...) {}
}

int bsr_comm_rank(const bsr_comm* c, int32_t* rank, int32_t* size) {
    if (!c || !rank || !size) return set_error(BSR_E_INVALID, "null argument");
    *rank = c->rank;
    *size = c->size;
    return BSR_OK;
}

// ---------------------------------------------------------------------------------------
// The exchange step (gather_top_k_results, src/mpi_helpers/metrics.rs:56-138): every rank's
// [nq][k] partial lists (+ counts) reach the root in rank order, as c->h_idx / h_dist /
// h_cnt laid out [rank][nq][k].  RCCL: one group of three all-gathers on `stream` (lists on
// the device, or staged there); host transport: one packed all-gather through the caller's
// function.  `empty`: this rank contributes empty lists (its local search failed:
// :185-191 sends an empty vector and the gather still completes).
// ---------------------------------------------------------------------------------------
static int exchange_lists(bsr_comm* c, const uint64_t* idx, const float* dist, const uint32_t* cnt, bool empty,
                          uint32_t nq, uint32_t k, hipStream_t stream, bool to_host = true) {
    const size_t nk = (size_t)nq * k, P = (size_t)c->size;
    const bool root = c->rank == 0;
    if (c->host_fn) {
        // message per rank: counts [nq] u32 | dists [nq][k] f32 | indices [nq][k] u64
        const size_t o_dist = (size_t)nq * 4, o_idx = o_dist + nk * 4, bytes = o_idx + nk * 8;
        c->h_send.assign(bytes, 0);
        c->h_recv.resize(bytes * P);
        if (!empty) {
            const bool dev = is_device_ptr(idx) || is_device_ptr(dist) || is_device_ptr(cnt);
            if (dev) {
                BSR_HIP(hipMemcpy(c->h_send.data(), cnt, (size_t)nq * 4, hipMemcpyDefault));
                BSR_HIP(hipMemcpy(c->h_send.data() + o_dist, dist, nk * 4, hipMemcpyDefault));
                BSR_HIP(hipMemcpy(c->h_send.data() + o_idx, idx, nk * 8, hipMemcpyDefault));
            } else {
                memcpy(c->h_send.data(), cnt, (size_t)nq * 4);
                memcpy(c->h_send.data() + o_dist, dist, nk * 4);
                memcpy(c->h_send.data() + o_idx, idx, nk * 8);
            }
        }
        if (c->host_fn(c->h_send.data(), c->h_recv.data(), bytes, c->host_user) != 0)
            return set_error(BSR_E_RCCL, "host all-gather callback failed");
        if (root) {
            BSR_TRY(c->h_cnt.resize((size_t)nq * P));
            BSR_TRY(c->h_dist.resize(nk * P));
            BSR_TRY(c->h_idx.resize(nk * P));
            for (size_t r = 0; r < P; ++r) {
                const uint8_t* m = c->h_recv.data() + r * bytes;
                memcpy(c->h_cnt.data() + r * nq, m, (size_t)nq * 4);
                memcpy(c->h_dist.data() + r * nk, m + o_dist, nk * 4);
                memcpy(c->h_idx.data() + r * nk, m + o_idx, nk * 8);
            }
        }
        return BSR_OK;
    }
    BSR_HIP(hipSetDevice(c->device));
    const uint64_t* s_idx = idx;
    const float* s_dist = dist;
    const uint32_t* s_cnt = cnt;
    if (empty || !is_device_ptr(idx) || !is_device_ptr(dist) || !is_device_ptr(cnt)) {
        BSR_TRY(c->send_idx.ensure(nk * sizeof(uint64_t)));
        BSR_TRY(c->send_dist.ensure(nk * sizeof(float)));
        BSR_TRY(c->send_cnt.ensure((size_t)nq * sizeof(uint32_t)));
        if (empty) {
            BSR_HIP(hipMemsetAsync(c->send_cnt.p, 0, (size_t)nq * sizeof(uint32_t), stream));
        } else {
            BSR_HIP(hipMemcpyAsync(c->send_idx.p, idx, nk * sizeof(uint64_t), hipMemcpyDefault, stream));
            BSR_HIP(hipMemcpyAsync(c->send_dist.p, dist, nk * sizeof(float), hipMemcpyDefault, stream));
            BSR_HIP(hipMemcpyAsync(c->send_cnt.p, cnt, (size_t)nq * sizeof(uint32_t), hipMemcpyDefault, stream));
        }
        s_idx = c->send_idx.as<uint64_t>();
        s_dist = c->send_dist.as<float>();
        s_cnt = c->send_cnt.as<uint32_t>();
    }
    BSR_TRY(c->recv_idx.ensure(nk * P * sizeof(uint64_t)));
    BSR_TRY(c->recv_dist.ensure(nk * P * sizeof(float)));
    BSR_TRY(c->recv_cnt.ensure((size_t)nq * P * sizeof(uint32_t)));
    BSR_TRY(coll_group(c, true));
    BSR_TRY(coll_allgather(c, s_idx, c->recv_idx.p, nk * sizeof(uint64_t), stream));
    BSR_TRY(coll_allgather(c, s_dist, c->recv_dist.p, nk * sizeof(float), stream));
    BSR_TRY(coll_allgather(c, s_cnt, c->recv_cnt.p, (size_t)nq * sizeof(uint32_t), stream));
    BSR_TRY(coll_group(c, false));
    if (!to_host) return BSR_OK;  // the lists stay in recv_* (stream-ordered consumers follow)
    if (root) {
        BSR_TRY(c->h_idx.resize(nk * P));
        BSR_TRY(c->h_dist.resize(nk * P));
        BSR_TRY(c->h_cnt.resize((size_t)nq * P));
        BSR_HIP(hipMemcpyAsync(c->h_idx.data(), c->recv_idx.p, nk * P * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
        BSR_HIP(hipMemcpyAsync(c->h_dist.data(), c->recv_dist.p, nk * P * sizeof(float), hipMemcpyDeviceToHost, stream));
        BSR_HIP(hipMemcpyAsync(c->h_cnt.data(), c->recv_cnt.p, (size_t)nq * P * sizeof(uint32_t), hipMemcpyDeviceToHost,
                               stream));
    }
    BSR_HIP(hipStreamSynchronize(stream));
    return BSR_OK;
}

// Non-root outputs: the reference returns None; counts read 0 (host or device memory).
static int clear_counts(uint32_t* out_count, uint32_t nq) {
    if (!out_count || !nq) return BSR_OK;
    if (is_device_ptr(out_count)) BSR_HIP(hipMemset(out_count, 0, (size_t)nq * sizeof(uint32_t)));
    else memset(out_count, 0, (size_t)nq * sizeof(uint32_t));
    return BSR_OK;
}

// The root's merge (compute_global_top_k, :200-202) of the gathered lists into out_*.
static int root_merge(bsr_comm* c, uint32_t nq, uint32_t k, uint64_t* out_idx, float* out_dist, uint32_t* out_count) {
    const ListsView v{c->h_idx.data(), c->h_dist.data(), c->h_cnt.data(), (uint32_t)c->size, nq, k};
    const bool dev = is_device_ptr(out_idx) || is_device_ptr(out_dist) || is_device_ptr(out_count);
    if (!dev) return merge_top_k_lists(v, nq, k, out_idx, out_dist, out_count);
    const size_t nk = (size_t)nq * k;
    c->m_idx.resize(nk);
    c->m_dist.resize(nk);
    c->m_cnt.resize(nq);
    BSR_TRY(merge_top_k_lists(v, nq, k, c->m_idx.data(), c->m_dist.data(), c->m_cnt.data()));
    BSR_HIP(hipMemcpy(out_idx, c->m_idx.data(), nk * sizeof(uint64_t), hipMemcpyHostToDevice));
    BSR_HIP(hipMemcpy(out_dist, c->m_dist.data(), nk * sizeof(float), hipMemcpyHostToDevice));
    BSR_HIP(hipMemcpy(out_count, c->m_cnt.data(), (size_t)nq * sizeof(uint32_t), hipMemcpyHostToDevice));
    return BSR_OK;
}

// The root's merge on the device (RCCL path): the gathered lists in c->recv_* are merged by
// k_merge_lists into the index's result buffer (where the local lists were), read back with
// one D2H copy, then handed to the caller's arrays -- instead of P lists to the host and a
// host merge (at 8 ranks x 1000 queries: a 1 MB copy and 0.15-0.3 ms of host merge, against
// a 10 us kernel).
static int root_merge_device(bsr_comm* c, bsr_index* ix, uint32_t nq, uint32_t k, uint64_t* out_idx,
                             float* out_dist, uint32_t* out_count) {
    hipStream_t s = ix->stream;
    if (c->host_fn) {
        // host transport: the gathered lists arrived in c->h_* (pinned); 1 MB up at P = 8
        const size_t nk = (size_t)nq * k * c->size;
        BSR_TRY(c->recv_idx.ensure(nk * sizeof(uint64_t)));
        BSR_TRY(c->recv_dist.ensure(nk * sizeof(float)));
        BSR_TRY(c->recv_cnt.ensure((size_t)nq * c->size * sizeof(uint32_t)));
        BSR_HIP(hipMemcpyAsync(c->recv_idx.p, c->h_idx.data(), nk * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        BSR_HIP(hipMemcpyAsync(c->recv_dist.p, c->h_dist.data(), nk * sizeof(float), hipMemcpyHostToDevice, s));
        BSR_HIP(hipMemcpyAsync(c->recv_cnt.p, c->h_cnt.data(), (size_t)nq * c->size * sizeof(uint32_t),
                               hipMemcpyHostToDevice, s));
    }
    BSR_TRY(c->nan_word.ensure(sizeof(uint32_t)));
    BSR_TRY(c->h_nan.resize(1));
    BSR_HIP(hipMemsetAsync(c->nan_word.p, 0xff, sizeof(uint32_t), s));
    BSR_HIP(launch_merge_lists(c->recv_idx.as<uint64_t>(), c->recv_dist.as<float>(), c->recv_cnt.as<uint32_t>(),
                               (uint32_t)c->size, nq, k, k, ix->d_idx, ix->d_dist, ix->d_cnt,
                               c->nan_word.as<uint32_t>(), s));
    BSR_HIP(hipMemcpyAsync(ix->h_res, ix->res[ix->cur].p, ix->res_bytes, hipMemcpyDeviceToHost, s));
    BSR_HIP(hipMemcpyAsync(c->h_nan.data(), c->nan_word.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    BSR_HIP(stream_wait(s));
    if (c->h_nan.data()[0] != ~0u)
        return set_error(BSR_E_NONFINITE, "NaN distance in query %u (the reference panics)", c->h_nan.data()[0]);
    return bsr_copy_out_impl(ix, nq, k, out_idx, out_dist, out_count);
}

static int gather_impl(bsr_comm* c, const uint64_t* local_idx, const float* local_dist, const uint32_t* local_count,
                       uint32_t nq, uint32_t k, uint64_t* root_idx, float* root_dist, uint32_t* root_count) {
    if (!c) return set_error(BSR_E_INVALID, "null communicator");
    if (!nq) return BSR_OK;
    if (k == 0) return set_error(BSR_E_INVALID, "k must be >= 1");
    // bad local or root arguments: still take part (an empty contribution), then fail, so
    // that no other rank is left blocked in the collective
    const bool empty = !local_idx || !local_dist || !local_count;
    const bool bad_root = c->rank == 0 && (!root_idx || !root_dist || !root_count);
    BSR_TRY(exchange_lists(c, local_idx, local_dist, local_count, empty, nq, k, c->stream));
    if (empty) return set_error(BSR_E_INVALID, "null local list (an empty contribution was sent)");
    if (bad_root) return set_error(BSR_E_INVALID, "null root output");
    if (c->rank == 0) {
        const size_t nk = (size_t)nq * k * c->size;
        BSR_HIP_OR_HOST_COPY(root_idx, c->h_idx.data(), nk * sizeof(uint64_t));
        BSR_HIP_OR_HOST_COPY(root_dist, c->h_dist.data(), nk * sizeof(float));
        BSR_HIP_OR_HOST_COPY(root_count, c->h_cnt.data(), (size_t)nq * c->size * sizeof(uint32_t));
    }
    return BSR_OK;
}

int bsr_gather_top_k(bsr_comm* c, const uint64_t* local_idx, const float* local_dist, const uint32_t* local_count,
                     uint32_t n_queries, uint32_t k, uint64_t* root_idx, float* root_dist, uint32_t* root_count) {
    BSR_GUARD(gather_impl(c, local_idx, local_dist, local_count, n_queries, k, root_idx, root_dist, root_count));
}

static int gather_global_impl(bsr_comm* c, const uint64_t* local_idx, const float* local_dist,
                              const uint32_t* local_count, uint32_t nq, uint32_t k, uint64_t* out_idx,
                              float* out_dist, uint32_t* out_count) {
    if (!c) return set_error(BSR_E_INVALID, "null communicator");
    if (!nq) return BSR_OK;
    if (k == 0) return set_error(BSR_E_INVALID, "k must be >= 1");
    const bool root = c->rank == 0;
    const bool empty = !local_idx || !local_dist || !local_count;  // an empty contribution
    BSR_TRY(exchange_lists(c, local_idx, local_dist, local_count, empty, nq, k, c->stream));
    if (!root) return clear_counts(out_count, nq);
    // (checked after the exchange: no other rank is left blocked in the collective)
    if (!out_idx || !out_dist || !out_count) return set_error(BSR_E_INVALID, "null root output");
    return root_merge(c, nq, k, out_idx, out_dist, out_count);
}

int bsr_gather_global_top_k(bsr_comm* comm, const uint64_t* local_idx, const float* local_dist,
                            const uint32_t* local_count, uint32_t n_queries, uint32_t k, uint64_t* out_idx,
                            float* out_dist, uint32_t* out_count) {
    BSR_GUARD(gather_global_impl(comm, local_idx, local_dist, local_count, n_queries, k, out_idx, out_dist, out_count));
}

// All-gather of every rank's header {nq, k, status of the local checks, magic, global-threshold
// capable, shard rows} into c->h_hdr[1 + r]: through the host transport (synchronous), or as a
// 32-byte RCCL all-gather on c->stream that header_wait() completes.
// Fault injection for the collective-safety tests (BSR_INJECT_FAULT=header_hook[:rank]): the
// first header all-gather of a search fails before it is posted, as a buffer that cannot be
// sized would make it fail; the rank must then post it again with its error status.
static bool inject_header_fault(const bsr_comm* c) {
    const char* v = getenv("BSR_INJECT_FAULT");  // (read per search: tests set it in-process)
    if (!v || strncmp(v, "header_hook", 11) != 0) return false;
    return v[11] != ':' || atoi(v + 12) == c->rank;
}

static int header_start(bsr_comm* c, uint32_t nq, uint32_t k, int32_t st, bool gtau, uint64_t n_rows,
                        bool first = false) {
    const size_t P = (size_t)c->size, hb = kHdrWords * sizeof(int32_t);
    if (first && inject_header_fault(c))
        return set_error(BSR_E_NOMEM, "injected fault: header buffers (BSR_INJECT_FAULT)");
    static_assert(kHdrWords == kHdrWordsInit, "header buffers sized at init");
    BSR_TRY(c->h_hdr.resize(kHdrWords * (1 + P)));  // (allocated at init: never fails here)
    int32_t* h = c->h_hdr.data();
    h[0] = (int32_t)nq;
    h[1] = (int32_t)k;
    h[2] = st;
    h[3] = kHdrMagic;
    h[4] = gtau ? 1 : 0;
    h[5] = (int32_t)(uint32_t)n_rows;
    h[6] = (int32_t)(uint32_t)(n_rows >> 32);
    h[7] = 0;
    c->hdr_seq = c->hdr_seq + 1 ? c->hdr_seq + 1 : 1;  // (the published flag's value: never 0)
    if (c->host_fn) {
        c->hdr_posted = true;  // (a failing transport fails on every rank)
        if (c->host_fn(h, h + kHdrWords, hb, c->host_user) != 0)
            return set_error(BSR_E_RCCL, "host all-gather callback failed");
        return BSR_OK;
    }
    // device transports: kernels only (no host copies, which would hold the host until done)
    BSR_HIP(hipSetDevice(c->device));
    BSR_HIP(launch_header_put(h, c->hdr_send.as<int32_t>(), c->stream));
    BSR_TRY(coll_allgather(c, c->hdr_send.p, c->hdr_recv.p, hb, c->stream));
    c->hdr_posted = true;
    BSR_HIP(launch_header_publish(c->hdr_recv.as<int32_t>(), (uint32_t)(kHdrWords * P), c->hdr_host_dev,
                                  c->hdr_flag_dev, c->hdr_seq, c->stream));
    return BSR_OK;
}
static int header_wait(bsr_comm* c) {
    if (c->host_fn) return BSR_OK;  // (synchronous)
    // poll the published flag (checking the stream now and then: one that finished or failed
    // without raising it is an error, never an endless wait)
    for (uint32_t i = 1;; ++i) {
        if (__atomic_load_n(c->hdr_flag, __ATOMIC_ACQUIRE) == c->hdr_seq) return BSR_OK;
        if ((i & 4095) == 0) {
            const hipError_t r = hipStreamQuery(c->stream);
            if (r == hipSuccess) {
                if (__atomic_load_n(c->hdr_flag, __ATOMIC_ACQUIRE) == c->hdr_seq) return BSR_OK;
                return set_error(BSR_E_HIP, "the header exchange finished without publishing");
            }
            if (r != hipErrorNotReady) BSR_HIP(r);
        }
        __builtin_ia32_pause();
    }
}
static const int32_t* header_of(const bsr_comm* c, int32_t r) {
    // (host transport: c->h_hdr after this rank's words; device transports: the published copy)
    if (!c->host_fn) return c->hdr_host + kHdrWords * (size_t)r;
    return c->h_hdr.data() + kHdrWords * (1 + (size_t)r);
}
// Post this search's header exactly once: a first attempt that failed before it was posted (the
// injected fault; the buffers exist since the communicator was created) is posted again carrying
// that failure, returned in *local_err.  Returns a transport error, which every rank sees.
static int post_header(bsr_comm* c, uint32_t nq, uint32_t k, int st, bool gt, uint64_t n, int* local_err) {
    *local_err = BSR_OK;
    const int hs = header_start(c, nq, k, st, gt, n, true);
    if (hs == BSR_OK || c->hdr_posted) return hs;
    *local_err = hs;
    return header_start(c, nq, k, st != BSR_OK ? st : hs, false, n);
}

// An all-gather of `bytes` device bytes per rank on `stream` (RCCL), or through the host
// transport (staged through pinned memory: a host round trip).
static int allgather_device(bsr_comm* c, const void* send, void* recv, size_t bytes, hipStream_t stream) {
    if (!c->host_fn) return coll_allgather(c, send, recv, bytes, stream);
    const size_t P = (size_t)c->size;
    BSR_TRY(c->h_stage.resize(bytes * (1 + P)));
    uint8_t* hs = c->h_stage.data();
    BSR_HIP(hipMemcpyAsync(hs, send, bytes, hipMemcpyDeviceToHost, stream));
    BSR_HIP(stream_wait(stream));
    if (c->host_fn(hs, hs + bytes, bytes, c->host_user) != 0)
        return set_error(BSR_E_RCCL, "host all-gather callback failed");
    BSR_HIP(hipMemcpyAsync(recv, hs + bytes, bytes * P, hipMemcpyHostToDevice, stream));
    return BSR_OK;
}

static int parallel_impl(bsr_comm* c, bsr_index* ix, const float* queries, uint32_t nq, uint32_t k,
                         uint64_t* out_idx, float* out_dist, uint32_t* out_count, bool allow_gtau);

// The merged result of the global-threshold search: [fail count, NaN word | status words
// [P][4] | fail list [nq] | counts [nq] | distances [nq][k] | indices [nq][k]]
struct MresLayout { size_t o_st, o_fail, o_cnt, o_dist, o_idx, bytes; };
static MresLayout mres_layout(uint32_t P, uint32_t nq, uint32_t k) {
    const size_t nqk = (size_t)nq * k;
    MresLayout L;
    L.o_st = 16;
    L.o_fail = round_up(L.o_st + (size_t)P * kStWords * 4, 16);
    L.o_cnt = round_up(L.o_fail + (size_t)nq * 4, 16);
    L.o_dist = round_up(L.o_cnt + (size_t)nq * 4, 16);
    L.o_idx = round_up(L.o_dist + nqk * 4, 16);
    L.bytes = round_up(L.o_idx + nqk * 8, 16);
    return L;
}

// Every buffer the global-threshold search uses after the header, allocated BEFORE the header
// is posted (after phase A, which sized the rank's result buffer): an allocation that fails here
// takes the rank -- and so every rank -- off the path through its header, where one failing
// between two all-gathers would leave the other ranks waiting in the next.
static int gtau_reserve(bsr_comm* c, const bsr_index* ix, uint32_t nq, uint32_t k) {
    const size_t P = (size_t)c->size;
    const size_t kb = (size_t)ix->gt_qpad * ix->gt_ks * sizeof(uint64_t), rbytes = ix->res_bytes;
    const size_t mbytes = mres_layout((uint32_t)P, nq, k).bytes;
    BSR_HIP(hipSetDevice(ix->device));
    BSR_TRY(c->g_smax.ensure(kb * P));
    BSR_TRY(c->g_res.ensure(rbytes * P));
    BSR_TRY(c->m_res.ensure(mbytes));
    if (c->host_fn) BSR_TRY(c->h_stage.resize(std::max(kb, rbytes) * (1 + P)));
    // (the uncertified queries' staging: sized now, so that no allocation can fail between the
    // merge and the fallback's collectives; bad_alloc becomes an error return, which takes the
    // rank off the path through its header instead of past it to BSR_GUARD -- ADVICE r05)
    try {
        c->f_q.reserve((size_t)nq * ix->dim);
        c->f_idx.reserve((size_t)nq * k);
        c->f_dist.reserve((size_t)nq * k);
        c->f_cnt.reserve(nq);
        c->f_list.reserve(nq);
    } catch (const std::bad_alloc&) {
        return set_error(BSR_E_NOMEM, "host allocation of the fallback staging failed");
    }
    if (c->h_mres_bytes < mbytes) {
        if (c->h_mres) BSR_HIP(hipHostFree(c->h_mres));
        c->h_mres = nullptr;
        c->h_mres_bytes = 0;
        BSR_HIP(hipHostMalloc((void**)&c->h_mres, mbytes, hipHostMallocCoherent));
        BSR_HIP(hipHostGetDevicePointer((void**)&c->h_mres_dev, c->h_mres, 0));
        c->h_mres_bytes = mbytes;
    }
    if (!c->h_flag) {
        BSR_TRY(c->pub_ticket.ensure(kTicketWords * sizeof(uint32_t)));
        BSR_HIP(hipMemsetAsync(c->pub_ticket.p, 0, kTicketWords * sizeof(uint32_t), ix->stream));
        BSR_HIP(hipHostMalloc((void**)&c->h_flag, 64, hipHostMallocCoherent));
        BSR_HIP(hipHostGetDevicePointer((void**)&c->h_flag_dev, c->h_flag, 0));
    }
    return BSR_OK;
}

// The rest of a parallel search with the global emission threshold, every rank
// having enqueued phase A (query prep, sample pass, its ks best sample keys per query) and
// every header saying so:
//   1. all-gather of the sample keys -> phase B: the global tau (the threshold one shard of the
//      whole corpus would select), the emit pass, the exact rescore of every emitted row, the
//      rank's top-k of them with its exclusion bound per query;
//   2. all-gather of the packed result buffers (lists, status words, bounds);
//   3. EVERY rank merges them (compute_global_top_k, :141-171) and certifies the merged lists
//      against the ranks' bounds -- the same deterministic kernel on the same bytes, so every
//      rank knows the same uncertified set F;
//   4. F (usually empty) takes the standard parallel search (local certified searches, their
//      exchange and merge), collectively, and its rows replace the root's.
// RCCL: every step is enqueued behind phase A on the index's stream, one host wait at the end.
// `a_err` != BSR_OK: this rank's phase A failed after its header put it on the path.
// It still takes part in every collective, poisoned: no sample keys (kKeyNone) and an empty result
// whose exclusion bounds are NaN, so that no merged list certifies and every query takes step 4,
// the standard collective search (where this rank searches again, or contributes an empty list).
// A non-root rank then returns a_err; the root returns the fallback's status, its rows complete.
static int parallel_gtau(bsr_comm* c, bsr_index* ix, const float* queries, uint32_t nq, uint32_t k,
                         uint64_t* out_idx, float* out_dist, uint32_t* out_count, int a_err,
                         const std::string& a_msg) {
    const uint32_t P = (uint32_t)c->size;
    const bool root = c->rank == 0;
    const bool poisoned = a_err != BSR_OK;
    hipStream_t s = ix->stream;
    uint64_t n_total = 0;
    for (int32_t r = 0; r < c->size; ++r) {
        const int32_t* h = header_of(c, r);
        n_total += (uint64_t)(uint32_t)h[5] | ((uint64_t)(uint32_t)h[6] << 32);
    }
    uint32_t need = (uint64_t)k < n_total ? k : (uint32_t)n_total;
    {  // (test hook, BSR_INJECT_FAULT=gtau_uncertified: no merged list certifies -- F is every query)
        const char* v = getenv("BSR_INJECT_FAULT");
        if (v && strcmp(v, "gtau_uncertified") == 0) need = k + 1;
    }
    BSR_HIP(hipSetDevice(ix->device));
    // 1. the sample keys of every rank, then phase B
    const size_t kb = (size_t)ix->gt_qpad * ix->gt_ks * sizeof(uint64_t);
    const size_t rbytes = ix->res_bytes;
    if (poisoned) BSR_HIP(hipMemsetAsync(ix->smax.p, 0xff, kb, s));  // (kKeyNone: no sample keys)
    BSR_TRY(allgather_device(c, ix->smax.p, c->g_smax.p, kb, s));
    if (!poisoned) {
        // (phase B's rescore also sets the merge's fail count and NaN word in m_res: two memset
        // launches fewer on the critical path)
        BSR_TRY(ix->gtau_phase_b(c->g_smax.as<uint64_t>(), P, c->m_res.as<uint32_t>()));
    } else {
        // an empty, uncertifiable contribution: status words and counts 0, exclusion bounds NaN;
        // the merge's fail count 0 and NaN word ~0 (what phase B's rescore would have set)
        uint8_t* rb = ix->res[ix->cur].as<uint8_t>();
        BSR_HIP(hipMemsetAsync(rb, 0, rbytes, s));
        BSR_HIP(hipMemsetAsync(rb + ix->res_off_x, 0xff, (size_t)nq * sizeof(float), s));
        BSR_HIP(hipMemsetAsync(c->m_res.p, 0, sizeof(uint32_t), s));
        BSR_HIP(hipMemsetAsync(c->m_res.as<uint8_t>() + sizeof(uint32_t), 0xff, sizeof(uint32_t), s));
    }
    // 2. the packed result buffers
    BSR_TRY(allgather_device(c, ix->res[ix->cur].p, c->g_res.p, rbytes, s));
    // 3. merge + certify into m_res (mres_layout)
    const size_t nqk = (size_t)nq * k;
    const MresLayout L = mres_layout(P, nq, k);
    const size_t o_st = L.o_st, o_fail = L.o_fail, o_cnt = L.o_cnt, o_dist = L.o_dist, o_idx = L.o_idx;
    __atomic_store_n(c->h_flag, 0u, __ATOMIC_RELEASE);
    uint8_t* md = c->m_res.as<uint8_t>();  // (its fail count and NaN word were set by phase B's rescore)
    const uint8_t* g = c->g_res.as<uint8_t>();
    MergeArgs ma{};
    ma.idx = reinterpret_cast<const uint64_t*>(g + ix->res_off_idx);
    ma.dist = reinterpret_cast<const float*>(g + ix->res_off_dist);
    ma.cnt = reinterpret_cast<const uint32_t*>(g + ix->res_off_cnt);
    ma.idx_stride = rbytes / 8;
    ma.dist_stride = rbytes / 4;
    ma.cnt_stride = rbytes / 4;
    ma.P = P;
    ma.nq = nq;
    ma.k_in = k;
    ma.k = k;
    ma.out_idx = reinterpret_cast<uint64_t*>(md + o_idx);
    ma.out_dist = reinterpret_cast<float*>(md + o_dist);
    ma.out_count = reinterpret_cast<uint32_t*>(md + o_cnt);
    ma.first_nan = reinterpret_cast<uint32_t*>(md) + 1;
    ma.excl = reinterpret_cast<const float*>(g + ix->res_off_x);
    ma.excl_stride = rbytes / 4;
    ma.need = need;
    ma.fail_cnt = reinterpret_cast<uint32_t*>(md);
    ma.fail_list = reinterpret_cast<uint32_t*>(md + o_fail);
    ma.st = reinterpret_cast<const uint32_t*>(g);
    ma.st_stride = rbytes / 4;
    ma.st_all = reinterpret_cast<uint32_t*>(md + o_st);
    // the merge publishes its result into host memory and raises the flag (no D2H copy, no
    // wait for the completion signal: index.cpp flag_wait)
    ma.pub_src = md;
    ma.pub_dst = c->h_mres_dev;
    // (the status words and F; the root's merged rows are written through by the merging waves)
    ma.pub_bytes = o_cnt;
    // Root outputs in coherent pinned host memory (bsr_host_alloc): the merging waves write the
    // merged rows straight into them -- no staging copy after the flag (round 5)
    uint64_t* d_oi = nullptr;
    float* d_od = nullptr;
    uint32_t* d_oc = nullptr;
    if (root && nq) {
        d_oi = static_cast<uint64_t*>(coherent_host_alias(out_idx));
        d_od = static_cast<float*>(coherent_host_alias(out_dist));
        d_oc = static_cast<uint32_t*>(coherent_host_alias(out_count));
    }
    const bool direct = d_oi && d_od && d_oc;
    const uint32_t path = BSR_PATH_COLLECTIVE | BSR_PATH_GLOBAL_TAU | (root && direct ? BSR_PATH_DIRECT_OUT : 0u);
    if (root) {
        ma.hout_idx = direct ? d_oi : reinterpret_cast<uint64_t*>(c->h_mres_dev + o_idx);
        ma.hout_dist = direct ? d_od : reinterpret_cast<float*>(c->h_mres_dev + o_dist);
        ma.hout_count = direct ? d_oc : reinterpret_cast<uint32_t*>(c->h_mres_dev + o_cnt);
    }
    ma.pub_flag = c->h_flag_dev;
    ma.pub_ticket = c->pub_ticket.as<uint32_t>();
    ma.lists_unique = 1;  // (each rank's list: its own search's top-k)
    BSR_HIP(launch_merge(ma, s));
    uint8_t* hm = c->h_mres;
    {
        const hipError_t r = flag_wait(c->h_flag, s);
        if (r == hipErrorUnknown) return set_error(BSR_E_HIP, "the merge finished without publishing its result");
        BSR_HIP(r);
    }
    bsr_index_collect_profile_impl(ix);
    const uint32_t* hw = reinterpret_cast<const uint32_t*>(hm);
    const uint32_t* st_all = reinterpret_cast<const uint32_t*>(hm + o_st);
    ix->stats.n_emitted = st_all[(size_t)c->rank * kStWords + kStEmitted];
    ix->stats.n_candidates = 0;  // (every emitted row was rescored)
    for (uint32_t r = 0; r < P; ++r)
        if (st_all[(size_t)r * kStWords + kStQueryFlags] & kQueryNonFinite)
            return set_error(BSR_E_NONFINITE, "a query contains NaN/Inf (the reference panics; rank %u)", r);
    if (hw[1] != ~0u) return set_error(BSR_E_NONFINITE, "NaN distance in query %u (the reference panics)", hw[1]);
    // 4. the uncertified queries, collectively (every rank holds the same F)
    const uint32_t nf = hw[0];
    ix->stats.n_fallback = nf;
    ix->stats.search_path = path;
    uint32_t* m_cnt = direct ? out_count : reinterpret_cast<uint32_t*>(hm + o_cnt);
    float* m_dist = direct ? out_dist : reinterpret_cast<float*>(hm + o_dist);
    uint64_t* m_idx = direct ? out_idx : reinterpret_cast<uint64_t*>(hm + o_idx);
    int fr = BSR_OK;  // the fallback's status (BSR_PARTIAL on a root whose own search failed)
    if (nf) {
        // (staging reserved by gtau_reserve: these resizes do not allocate.  A local failure
        // here still takes part in the fallback's collectives -- with no queries, i.e. an empty
        // contribution -- and is returned after them.)
        std::vector<uint32_t>& fl = c->f_list;
        fl.assign(reinterpret_cast<const uint32_t*>(hm + o_fail), reinterpret_cast<const uint32_t*>(hm + o_fail) + nf);
        std::sort(fl.begin(), fl.end());
        const uint32_t d = ix->dim;
        c->f_q.resize((size_t)nf * d);
        const bool qdev = is_device_ptr(queries);
        int staged = BSR_OK;
        for (uint32_t i = 0; i < nf && staged == BSR_OK; ++i) {
            if (!qdev) memcpy(c->f_q.data() + (size_t)i * d, queries + (size_t)fl[i] * d, d * sizeof(float));
            else if (hipMemcpyAsync(c->f_q.data() + (size_t)i * d, queries + (size_t)fl[i] * d, d * sizeof(float),
                                    hipMemcpyDeviceToHost, s) != hipSuccess)
                staged = set_error(BSR_E_HIP, "staging the uncertified queries failed");
        }
        if (qdev && staged == BSR_OK && stream_wait(s) != hipSuccess)
            staged = set_error(BSR_E_HIP, "staging the uncertified queries failed");
        std::string staged_err = staged == BSR_OK ? std::string() : std::string(last_error_cstr());
        c->f_idx.resize((size_t)nf * k);
        c->f_dist.resize((size_t)nf * k);
        c->f_cnt.resize(nf);
        const bsr_search_stats keep = ix->stats;
        fr = parallel_impl(c, ix, staged == BSR_OK ? c->f_q.data() : nullptr, nf, k, c->f_idx.data(),
                           c->f_dist.data(), c->f_cnt.data(), false);
        ix->stats.n_emitted = keep.n_emitted;
        ix->stats.n_candidates = 0;  // (this search's path: every emitted row rescored)
        ix->stats.n_fallback = nf;
        ix->stats.n_queries = nq;
        ix->stats.search_path = path | BSR_PATH_FALLBACK;
        if (poisoned && !root) return set_error(a_err, "%s", a_msg.c_str());
        if (staged != BSR_OK && !root) return set_error(staged, "%s", staged_err.c_str());
        // (the root's staging failed: its fallback search had no queries; report the real cause)
        if (staged != BSR_OK && fr == BSR_PARTIAL)
            set_error(BSR_PARTIAL, "this rank's local search failed (%s); the result covers the other ranks' blocks",
                      staged_err.c_str());
        // a root whose own fallback search failed still has the other ranks' rows (BSR_PARTIAL):
        // they are patched in and the merged result is handed out with that status
        if (fr != BSR_OK && !(root && fr == BSR_PARTIAL)) return fr;
        if (root)
            for (uint32_t i = 0; i < nf; ++i) {
                const uint32_t q = fl[i];
                m_cnt[q] = c->f_cnt[i];
                memcpy(m_idx + (size_t)q * k, c->f_idx.data() + (size_t)i * k, k * sizeof(uint64_t));
                memcpy(m_dist + (size_t)q * k, c->f_dist.data() + (size_t)i * k, k * sizeof(float));
            }
    }
    if (poisoned && !root) return set_error(a_err, "%s", a_msg.c_str());
    if (!root) return clear_counts(out_count, nq);
    if (direct) return fr;  // (the merged rows, and any fallback rows patched above, are in out_*)
    if (is_device_ptr(out_idx) || is_device_ptr(out_dist) || is_device_ptr(out_count)) {
        BSR_HIP_OR_HOST_COPY(out_idx, m_idx, nqk * sizeof(uint64_t));
        BSR_HIP_OR_HOST_COPY(out_dist, m_dist, nqk * sizeof(float));
        BSR_HIP_OR_HOST_COPY(out_count, m_cnt, (size_t)nq * sizeof(uint32_t));
    } else {
        memcpy(out_idx, m_idx, nqk * sizeof(uint64_t));
        memcpy(out_dist, m_dist, nqk * sizeof(float));
        memcpy(out_count, m_cnt, (size_t)nq * sizeof(uint32_t));
    }
    return fr;  // (BSR_OK, or BSR_PARTIAL with bsr_last_error() from the fallback)
}

// Test switch (BSR_FORCE_COLLECTIVES=1, read per search): a one-rank communicator takes the
// multi-rank branch, so a one-rank RCCL communicator runs every collective of the parallel search
// -- the header all-gather on the communicator's stream, the global threshold's key and result
// all-gathers on the index's stream, the standard path's group of three -- through real RCCL.
static bool force_collectives() {
    const char* v = getenv("BSR_FORCE_COLLECTIVES");
    return v && v[0] == '1';
}

// Fault injection for the collective-safety tests (BSR_INJECT_FAULT=phase_a0[:rank] or
// phase_a1[:rank]): the global-threshold search's phase A fails in its first part (before the
// header) or its second (after it).
static bool inject_phase_a_fault(const bsr_comm* c, int part) {
    const char* v = getenv("BSR_INJECT_FAULT");
    const char* want = part == 0 ? "phase_a0" : "phase_a1";
    if (!v || strncmp(v, want, 8) != 0) return false;
    return v[8] != ':' || atoi(v + 9) == c->rank;
}

// parallel_top_k_similarity_search (src/mpi_helpers/metrics.rs:174-206).  Collective-safe:
// every rank reaches the same collectives whatever fails locally.
//   1. local checks; (size > 1) the rank's eligibility for the global threshold and, when
//      eligible, phase A enqueued; the all-gather of every rank's header {nq, k, status,
//      eligible, shard rows}; ranks that disagree on the batch shape all return BSR_E_INVALID
//      and no list exchange happens (mismatched all-gathers are undefined);
//   2. every rank eligible and fine: the global-threshold search (parallel_gtau);
//   3. otherwise compute_local_top_k (:185) on each rank, gather_top_k_results (:194) -- a rank
//      whose search or checks failed contributes an empty list, as the reference's error
//      branch does (:185-191) -- and the root's merge (:200-202).
// Returns: BSR_OK; on a non-root rank whose local step failed, that error; on a root whose
// own local step failed but whose outputs are usable, BSR_PARTIAL with the other ranks'
// global top-k in out_* (the reference's root returns Some(..) there, :199-202).
static int parallel_impl(bsr_comm* c, bsr_index* ix, const float* queries, uint32_t nq, uint32_t k,
                         uint64_t* out_idx, float* out_dist, uint32_t* out_count, bool allow_gtau) {
    const bool root = !c || c->rank == 0;
    const bool outs_ok = !nq || (out_idx && out_dist && out_count);
    int st = BSR_OK;
    if (!ix) st = set_error(BSR_E_INVALID, "null index");
    else if (root && !outs_ok) st = set_error(BSR_E_INVALID, "null output");
    else if (c && !c->host_fn && c->device != ix->device)
        st = set_error(BSR_E_INVALID, "communicator and index on different devices");
    const bool multi = c && (c->size > 1 || force_collectives());
    bool searched = false;
    if (multi) {
        // global threshold: this rank's filter path with a sample pass, lists the device merge
        // takes, and the library setting (BSR_GLOBAL_TAU=0 turns it off)
        const char* gv = getenv("BSR_GLOBAL_TAU");  // (read per search, as the test switches)
        const bool gtau_on = !(gv && gv[0] == '0');
        // (batches of <= 16 queries -- the latency path -- keep the per-rank threshold: their
        // emission is light, and the standard path overlaps the header with the search)
        bool gt = allow_gtau && gtau_on && st == BSR_OK && nq > kSkinnyMaxQ && ix->gtau_eligible(nq, k) &&
                  device_merge_fits((uint32_t)c->size, k, k);
        if (gt) {
            // every buffer of the path sized first: an allocation failure takes this rank (so every
            // rank) off the path through its header
            const int r = ix->gtau_prepare(queries, nq, k);
            if (r != BSR_OK) { st = r; gt = false; }
            else if (gtau_reserve(c, ix, nq, k) != BSR_OK) gt = false;  // (the standard path then)
        }
        c->hdr_posted = false;
        const uint64_t n_rows = ix ? ix->n : 0;
        int lerr = BSR_OK;
        int a_err = BSR_OK;  // phase A's second part failed after a header that put this rank on the path
        std::string a_msg;
        if (gt) {
            // the query prep, then the header, then the rest of phase A: the GPU starts on the prep
            // while the host issues the header's launches, and the header's round trip (to the
            // transport and back to the host, which enqueues phase B when it has it) overlaps phase A
            // instead of following it.  A failure of the prep (e.g. staging pageable host queries)
            // goes into the header, which takes every rank off the path.
            const int ra = inject_phase_a_fault(c, 0)
                               ? set_error(BSR_E_HIP, "injected fault: phase A, query prep (BSR_INJECT_FAULT)")
                               : ix->gtau_phase_a(queries, 0);
            if (ra != BSR_OK) {
                st = ra;
                gt = false;
            }
        }
        if (gt) {
            BSR_TRY(post_header(c, nq, k, st, true, n_rows, &lerr));  // (a transport error: every rank sees it)
            if (lerr != BSR_OK) {  // reposted with the failure: this rank, so every rank, is off the path
                st = lerr;
                gt = false;
            } else {
                // (past the header: a failure here keeps this rank in every collective, poisoned)
                a_err = inject_phase_a_fault(c, 1)
                            ? set_error(BSR_E_HIP, "injected fault: phase A, sample pass (BSR_INJECT_FAULT)")
                            : ix->gtau_phase_a(queries, 1);
                if (a_err != BSR_OK) a_msg = last_error_cstr();
            }
        }
        if (!gt) {
            // No rank is on the global-threshold path: the standard search starts now and the header
            // is posted and waited for from the search's hook, after the persistent filter has been
            // launched (an RCCL kernel waiting for a late peer then cannot hold a CU the filter's
            // one-workgroup-per-CU grid needs), overlapping the search.
            struct HookCtx {
                bsr_comm* c;
                uint32_t nq, k;
                uint64_t n;
                int lerr, hst;
                bool ran;
            } hc{c, nq, k, n_rows, BSR_OK, BSR_OK, false};
            auto hook = [](void* p) -> int {
                HookCtx* h = static_cast<HookCtx*>(p);
                h->ran = true;
                if (!h->c->hdr_posted) h->hst = post_header(h->c, h->nq, h->k, BSR_OK, false, h->n, &h->lerr);
                if (h->hst == BSR_OK) h->hst = header_wait(h->c);
                return h->hst;
            };
            if (st == BSR_OK) {
                st = ix->search_device(queries, nq, k, +hook, &hc);
                if (hc.ran && hc.hst != BSR_OK) return hc.hst;  // (a transport error: every rank sees it)
                if (st == BSR_OK && hc.lerr != BSR_OK) st = hc.lerr;  // (an empty contribution, then this error)
            }
            if (!c->hdr_posted) {  // the search failed before its launch, or never ran
                BSR_TRY(post_header(c, nq, k, st, false, n_rows, &lerr));
                if (st == BSR_OK) st = lerr;
            }
            if (!hc.ran) BSR_TRY(header_wait(c));
            searched = true;
        } else {
            BSR_TRY(header_wait(c));
        }
        const int32_t* h0 = header_of(c, 0);
        bool all_gt = true;
        for (int32_t r = 0; r < c->size; ++r) {
            const int32_t* hr = header_of(c, r);
            if (hr[3] != kHdrMagic || hr[0] != h0[0] || hr[1] != h0[1])
                return set_error(BSR_E_INVALID,
                                 "ranks disagree on the batch shape: rank 0 (n_queries %d, k %d), rank %d "
                                 "(n_queries %d, k %d); no rank exchanged lists",
                                 h0[0], h0[1], r, hr[0], hr[1]);
            all_gt &= hr[4] == 1 && hr[2] == BSR_OK;
        }
        if (gt && all_gt)
            return parallel_gtau(c, ix, queries, nq, k, out_idx, out_dist, out_count, a_err, a_msg);
        if (gt) {  // (phase A ran for nothing: the standard path; a failed phase A, an empty contribution)
            if (a_err != BSR_OK) st = set_error(a_err, "%s", a_msg.c_str());
            else if (stream_wait(ix->stream) != hipSuccess) st = set_error(BSR_E_HIP, "phase A failed on the device");
        }
    }
    // compute_local_top_k (:185-191)
    if (st == BSR_OK && !searched) st = ix->search_device(queries, nq, k);
    if (!c) {  // one rank, no communicator: the local lists are the result
        BSR_TRY(st);
        if (!nq) return BSR_OK;
        BSR_TRY(bsr_copy_out_impl(ix, nq, k, out_idx, out_dist, out_count));
        bsr_index_collect_profile_impl(ix);
        return BSR_OK;
    }
    std::string local_err;
    if (st != BSR_OK) local_err = last_error_cstr();
    if (!nq) return st;
    if (k == 0) return st != BSR_OK ? st : set_error(BSR_E_INVALID, "k must be >= 1");
    const bool ok = st == BSR_OK;
    // gather_top_k_results (:194) on the index's stream (ordered after the search), then the
    // root's merge (:200-202)
    // (RCCL: the device lists; host transport: their pinned host mirror)
    const uint64_t* li = nullptr;
    const float* ld = nullptr;
    const uint32_t* lc = nullptr;
    if (ok && c->host_fn) {
        li = reinterpret_cast<const uint64_t*>(ix->h_res + ix->res_off_idx);
        ld = reinterpret_cast<const float*>(ix->h_res + ix->res_off_dist);
        lc = reinterpret_cast<const uint32_t*>(ix->h_res + ix->res_off_cnt);
    } else if (ok) {
        li = ix->d_idx;
        ld = ix->d_dist;
        lc = ix->d_cnt;
    }
    // (the root merges on the device into its own result buffer: only after its own search
    // succeeded, i.e. that buffer is sized for this batch; host transport: the root's lists
    // come up to its GPU for the same merge)
    const bool dev_merge = ok && device_merge_fits((uint32_t)c->size, k, k);
    if (ix) ix->stats.search_path |= BSR_PATH_COLLECTIVE | (root && dev_merge ? BSR_PATH_DEVICE_MERGE : 0u);
    hipStream_t xs = c->host_fn ? nullptr : (ok ? ix->stream : c->stream);
    BSR_TRY(exchange_lists(c, li, ld, lc, !ok, nq, k, xs, !dev_merge || c->host_fn));
    if (ok) bsr_index_collect_profile_impl(ix);
    if (root && dev_merge) {
        BSR_TRY(root_merge_device(c, ix, nq, k, out_idx, out_dist, out_count));
    } else if (root && outs_ok) {
        BSR_TRY(root_merge(c, nq, k, out_idx, out_dist, out_count));
    } else if (!root && dev_merge) {
        BSR_HIP(stream_wait(ix->stream));  // the all-gather has read this rank's lists
        BSR_TRY(clear_counts(out_count, nq));
    } else if (!root) {
        BSR_TRY(clear_counts(out_count, nq));
    }
    if (ok) return BSR_OK;
    if (root && outs_ok) {
        set_error(BSR_PARTIAL, "this rank's local search failed (%s); the result covers the other ranks' blocks",
                  local_err.c_str());
        return BSR_PARTIAL;
    }
    return set_error(st, "%s", local_err.c_str());
}

static int parallel_top(bsr_comm* c, bsr_index* ix, const float* queries, uint32_t nq, uint32_t k, uint64_t* out_idx,
                        float* out_dist, uint32_t* out_count) {
    if (c && c->loopback) {  // a loopback script replays the recorded search's all-gathers, from its first
        c->lb_search = true;
        c->lb_live = c->lb_nq == (int32_t)nq && c->lb_k == (int32_t)k;  // (another batch shape: replicate)
        c->lb_cursor = 0;
        // The replayed contributions are the other ranks' for the RECORDED query batch: replay is
        // valid only for that batch.  Host batches are checked by digest against the first one
        // replayed (another batch: a miss, replicated); device batches are taken on trust (the
        // bench's loopback step replays its one recorded batch).
        if (c->lb_live && !c->lb_bytes.empty() && queries && !is_device_ptr(queries)) {
            uint64_t h = 1469598103934665603ull;
            const uint8_t* b = reinterpret_cast<const uint8_t*>(queries);
            const size_t nb = (size_t)nq * (ix ? ix->dim : 0) * sizeof(float);
            for (size_t i = 0; i < nb; ++i) h = (h ^ b[i]) * 1099511628211ull;
            if (!c->lb_qdigest_set) {
                c->lb_qdigest = h;
                c->lb_qdigest_set = true;
            } else if (h != c->lb_qdigest) {
                c->lb_live = false;
                ++c->lb_missed;
            }
        }
    }
    const int r = parallel_impl(c, ix, queries, nq, k, out_idx, out_dist, out_count, true);
    if (c) c->lb_search = false;
    return r;
}

int bsr_parallel_top_k_similarity_search(bsr_comm* comm, bsr_index* ix, const float* queries, uint32_t n_queries,
                                         uint32_t k, uint64_t* out_idx, float* out_dist, uint32_t* out_count) {
    BSR_GUARD(parallel_top(comm, ix, queries, n_queries, k, out_idx, out_dist, out_count));
}

// ---------------------------------------------------------------------------------------
// Small collectives of the driver (src/main.rs:123-125 broadcast_into; the timing gather of
// src/mpi_helpers/benchmark.rs:131-293): host or device buffers, either transport.
// ---------------------------------------------------------------------------------------
static int allgather_bytes_impl(bsr_comm* c, const void* send, void* recv, uint64_t bytes) {
    if (!c || (bytes && (!send || !recv))) return set_error(BSR_E_INVALID, "bad argument");
    if (!bytes) return BSR_OK;
    const size_t P = (size_t)c->size;
    if (c->host_fn) {
        std::vector<uint8_t> hs(bytes), hr(bytes * P);
        BSR_HIP_OR_HOST_COPY_FROM(hs.data(), send, bytes);
        if (c->host_fn(hs.data(), hr.data(), bytes, c->host_user) != 0)
            return set_error(BSR_E_RCCL, "host all-gather callback failed");
        BSR_HIP_OR_HOST_COPY(recv, hr.data(), bytes * P);
        return BSR_OK;
    }
    BSR_HIP(hipSetDevice(c->device));
    DevBuf ds, dr;
    BSR_TRY(ds.ensure(bytes));
    BSR_TRY(dr.ensure(bytes * P));
    BSR_HIP(hipMemcpyAsync(ds.p, send, bytes, hipMemcpyDefault, c->stream));
    BSR_TRY(coll_allgather(c, ds.p, dr.p, bytes, c->stream));
    BSR_HIP(hipMemcpyAsync(recv, dr.p, bytes * P, hipMemcpyDefault, c->stream));
    BSR_HIP(hipStreamSynchronize(c->stream));
    return BSR_OK;
}

int bsr_allgather_bytes(bsr_comm* comm, const void* send, void* recv, uint64_t bytes) {
    BSR_GUARD(allgather_bytes_impl(comm, send, recv, bytes));
}

static int broadcast_impl(bsr_comm* c, void* buf, uint64_t bytes, int32_t root) {
    if (!c || (bytes && !buf) || root < 0 || root >= c->size) return set_error(BSR_E_INVALID, "bad argument");
    if (!bytes) return BSR_OK;
    if (c->host_fn) {  // a broadcast as an all-gather of which every rank keeps the root's part
        std::vector<uint8_t> hs(bytes), hr(bytes * (size_t)c->size);
        BSR_HIP_OR_HOST_COPY_FROM(hs.data(), buf, bytes);
        if (c->host_fn(hs.data(), hr.data(), bytes, c->host_user) != 0)
            return set_error(BSR_E_RCCL, "host all-gather callback failed");
        BSR_HIP_OR_HOST_COPY(buf, hr.data() + (size_t)root * bytes, bytes);
        return BSR_OK;
    }
    if (c->loopback) return BSR_OK;  // (one process: this rank's buffer stands for the root's)
    BSR_HIP(hipSetDevice(c->device));
    void* d = buf;
    DevBuf tmp;
    const bool dev = is_device_ptr(buf);
    if (!dev) {
        BSR_TRY(tmp.ensure(bytes));
        BSR_HIP(hipMemcpyAsync(tmp.p, buf, bytes, hipMemcpyHostToDevice, c->stream));
        d = tmp.p;
    }
    BSR_NCCL(ncclBroadcast(d, d, bytes, ncclUint8, root, c->comm, c->stream));
    if (!dev) BSR_HIP(hipMemcpyAsync(buf, d, bytes, hipMemcpyDeviceToHost, c->stream));
    BSR_HIP(hipStreamSynchronize(c->stream));
    return BSR_OK;
}

int bsr_broadcast(bsr_comm* comm, void* buf, uint64_t bytes, int32_t root) {
    BSR_GUARD(broadcast_impl(comm, buf, bytes, root));
}

int bsr_index_last_stats(const bsr_index* ix, bsr_search_stats* out) {
    if (!ix || !out) return set_error(BSR_E_INVALID, "null argument");
    *out = ix->stats;
    return BSR_OK;
}

int bsr_index_set_profile(bsr_index* ix, int level) {
    if (!ix) return set_error(BSR_E_INVALID, "null index");
    if (level < 0 || level > 2) return set_error(BSR_E_INVALID, "profile level %d outside [0, 2]", level);
    ix->prof_level = level;
    return BSR_OK;
}

int bsr_index_profile(bsr_index* ix, bsr_profile* out, int reset) {
    if (!ix) return set_error(BSR_E_INVALID, "null index");
    if (out) *out = ix->prof;
    if (reset) ix->prof = bsr_profile{};
    return BSR_OK;
}

static int synth_impl(float* dev_out, uint64_t row0, uint64_t n_rows, uint32_t dim, uint64_t seed) {
    if (!dev_out || !dim) return set_error(BSR_E_INVALID, "bad argument");
    if (!is_device_ptr(dev_out)) return set_error(BSR_E_INVALID, "bsr_synth_uniform writes device memory only");
    BSR_HIP(launch_synth_uniform(dev_out, row0, n_rows, dim, dim, seed, nullptr));
    BSR_HIP(hipStreamSynchronize(nullptr));
    return BSR_OK;
}

int bsr_synth_uniform(float* dev_out, uint64_t row0, uint64_t n_rows, uint32_t dim, uint64_t seed) {
    BSR_GUARD(synth_impl(dev_out, row0, n_rows, dim, seed));
}

}  // extern "C"
