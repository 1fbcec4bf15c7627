// capi.cpp -- the C ABI (include/bsr.h): argument checks, exception firewall, the RCCL
// communicator, gather (src/mpi_helpers/metrics.rs:56-138), the host merge
// (:141-171) and the composed parallel search (:174-206).
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "internal.hpp"
#include "kernels.hpp"

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

struct bsr_comm {
    ncclComm_t comm = nullptr;
    int32_t rank = 0, size = 1, device = 0;
    hipStream_t stream = nullptr;
    DevBuf send_idx, send_dist, send_cnt, recv_idx, recv_dist, recv_cnt;
    std::vector<uint64_t> h_idx;
    std::vector<float> h_dist;
    std::vector<uint32_t> h_cnt;
};

#define BSR_NCCL(call)                                                                          \
    do {                                                                                        \
        ncclResult_t r_ = (call);                                                               \
        if (r_ != ncclSuccess)                                                                  \
            return set_error(BSR_E_RCCL, "%s failed: %s", #call, ncclGetErrorString(r_));       \
    } while (0)

// ---------------------------------------------------------------------------------------
// host merge
// ---------------------------------------------------------------------------------------
namespace {

struct Entry {
    uint64_t idx;
    float dist;
};

// src/mpi_helpers/metrics.rs:141-171 literally: concatenate (in list order), stable sort by
// distance, dedupe by index, keep top_k.
uint32_t global_top_k_one(const Entry* in, size_t n, uint32_t k, uint64_t* out_idx, float* out_dist,
                          std::vector<Entry>& scratch, bool* nan) {
    scratch.assign(in, in + n);
    for (const Entry& e : scratch)
        if (e.dist != e.dist) { *nan = true; return 0; }
    std::stable_sort(scratch.begin(), scratch.end(), [](const Entry& a, const Entry& b) { return a.dist < b.dist; });
    uint32_t out = 0;
    for (const Entry& e : scratch) {
        if (out >= k) break;
        bool seen = false;
        for (uint32_t j = 0; j < out; ++j)
            if (out_idx[j] == e.idx) { seen = true; break; }
        if (seen) continue;
        out_idx[out] = e.idx;
        out_dist[out] = e.dist;
        ++out;
    }
    return out;
}

// Same result for per-rank lists already in (distance, index) order over disjoint,
// rank-ordered index blocks (what bsr_local_top_k returns): a P-way merge.
uint32_t merge_sorted_lists(const uint64_t* idx, const float* dist, const uint32_t* cnt, uint32_t n_lists,
                            uint32_t n_queries, uint32_t k_in, uint32_t q, uint32_t k, uint64_t* out_idx,
                            float* out_dist) {
    uint32_t pos[64] = {0};
    uint32_t out = 0;
    while (out < k) {
        int best = -1;
        float bd = 0.0f;
        uint64_t bi = 0;
        for (uint32_t l = 0; l < n_lists; ++l) {
            const size_t base = ((size_t)l * n_queries + q) * k_in;
            if (pos[l] >= cnt[(size_t)l * n_queries + q]) continue;
            const float d = dist[base + pos[l]];
            const uint64_t i = idx[base + pos[l]];
            if (best < 0 || d < bd || (d == bd && i < bi)) { best = (int)l; bd = d; bi = i; }
        }
        if (best < 0) break;
        ++pos[best];
        if (out && out_idx[out - 1] == bi) continue;  // dedupe (a no-op for disjoint blocks)
        out_idx[out] = bi;
        out_dist[out] = bd;
        ++out;
    }
    return out;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------
extern "C" {

const char* bsr_last_error(void) { return last_error_cstr(); }

const char* bsr_status_string(int s) {
    switch (s) {
        case BSR_OK: return "BSR_OK";
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

static int global_top_k_impl(const uint64_t* idx, const float* dist, const uint32_t* count, uint32_t n_lists,
                             uint32_t n_queries, uint32_t k_in, uint32_t k, uint64_t* out_idx, float* out_dist,
                             uint32_t* out_count) {
    if (!n_queries) return BSR_OK;
    if (!count || !out_idx || !out_dist || !out_count || (n_lists && k_in && (!idx || !dist)))
        return set_error(BSR_E_INVALID, "null argument");
    if (k == 0) return set_error(BSR_E_INVALID, "k must be >= 1");
    std::vector<Entry> concat, scratch;
    for (uint32_t q = 0; q < n_queries; ++q) {
        concat.clear();
        for (uint32_t l = 0; l < n_lists; ++l) {
            const uint32_t c = std::min(count[(size_t)l * n_queries + q], k_in);
            const size_t base = ((size_t)l * n_queries + q) * k_in;
            for (uint32_t i = 0; i < c; ++i) concat.push_back({idx[base + i], dist[base + i]});
        }
        bool nan = false;
        out_count[q] = global_top_k_one(concat.data(), concat.size(), k, out_idx + (size_t)q * k,
                                        out_dist + (size_t)q * k, scratch, &nan);
        if (nan) return set_error(BSR_E_NONFINITE, "NaN distance in query %u (the reference panics)", q);
        for (uint32_t i = out_count[q]; i < k; ++i) {
            out_idx[(size_t)q * k + i] = ~0ull;
            out_dist[(size_t)q * k + i] = __builtin_inff();
        }
    }
    return BSR_OK;
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
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        ncclCommDestroy(c->comm);
        delete c;
        return set_error(BSR_E_HIP, "hipStreamCreate failed");
    }
    *out = c;
    return BSR_OK;
}

int bsr_comm_init(const uint8_t id[BSR_UNIQUE_ID_BYTES], int32_t rank, int32_t size, int32_t device,
                  bsr_comm** out) {
    BSR_GUARD(comm_init_impl(id, rank, size, device, out));
}

void bsr_comm_destroy(bsr_comm* c) {
    if (!c) return;
    try {
        (void)hipSetDevice(c->device);
        if (c->stream) { (void)hipStreamSynchronize(c->stream); (void)hipStreamDestroy(c->stream); }
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

// All-gather the [nq][k] partial lists of every rank (device buffers) on `stream`.
static int allgather_lists(bsr_comm* c, const uint64_t* d_idx, const float* d_dist, const uint32_t* d_cnt,
                           uint32_t nq, uint32_t k, hipStream_t stream) {
    const size_t nk = (size_t)nq * k;
    BSR_TRY(c->recv_idx.ensure(nk * c->size * sizeof(uint64_t)));
    BSR_TRY(c->recv_dist.ensure(nk * c->size * sizeof(float)));
    BSR_TRY(c->recv_cnt.ensure((size_t)nq * c->size * sizeof(uint32_t)));
    BSR_NCCL(ncclGroupStart());
    BSR_NCCL(ncclAllGather(d_idx, c->recv_idx.p, nk * sizeof(uint64_t), ncclUint8, c->comm, stream));
    BSR_NCCL(ncclAllGather(d_dist, c->recv_dist.p, nk * sizeof(float), ncclUint8, c->comm, stream));
    BSR_NCCL(ncclAllGather(d_cnt, c->recv_cnt.p, (size_t)nq * sizeof(uint32_t), ncclUint8, c->comm, stream));
    BSR_NCCL(ncclGroupEnd());
    return BSR_OK;
}

static int gather_impl(bsr_comm* c, const uint64_t* local_idx, const float* local_dist, const uint32_t* local_count,
                       uint32_t nq, uint32_t k, uint64_t* root_idx, float* root_dist, uint32_t* root_count) {
    if (!c) return set_error(BSR_E_INVALID, "null communicator");
    if (!nq) return BSR_OK;
    if (!local_idx || !local_dist || !local_count || k == 0) return set_error(BSR_E_INVALID, "bad argument");
    if (c->rank == 0 && (!root_idx || !root_dist || !root_count)) return set_error(BSR_E_INVALID, "null root output");
    BSR_HIP(hipSetDevice(c->device));
    const size_t nk = (size_t)nq * k;
    BSR_TRY(c->send_idx.ensure(nk * sizeof(uint64_t)));
    BSR_TRY(c->send_dist.ensure(nk * sizeof(float)));
    BSR_TRY(c->send_cnt.ensure((size_t)nq * sizeof(uint32_t)));
    BSR_HIP(hipMemcpyAsync(c->send_idx.p, local_idx, nk * sizeof(uint64_t), hipMemcpyDefault, c->stream));
    BSR_HIP(hipMemcpyAsync(c->send_dist.p, local_dist, nk * sizeof(float), hipMemcpyDefault, c->stream));
    BSR_HIP(hipMemcpyAsync(c->send_cnt.p, local_count, (size_t)nq * sizeof(uint32_t), hipMemcpyDefault, c->stream));
    BSR_TRY(allgather_lists(c, c->send_idx.as<uint64_t>(), c->send_dist.as<float>(), c->send_cnt.as<uint32_t>(), nq,
                            k, c->stream));
    if (c->rank == 0) {
        BSR_HIP(hipMemcpyAsync(root_idx, c->recv_idx.p, nk * c->size * sizeof(uint64_t), hipMemcpyDefault, c->stream));
        BSR_HIP(hipMemcpyAsync(root_dist, c->recv_dist.p, nk * c->size * sizeof(float), hipMemcpyDefault, c->stream));
        BSR_HIP(hipMemcpyAsync(root_count, c->recv_cnt.p, (size_t)nq * c->size * sizeof(uint32_t), hipMemcpyDefault,
                               c->stream));
    }
    BSR_HIP(hipStreamSynchronize(c->stream));
    return BSR_OK;
}

int bsr_gather_top_k(bsr_comm* c, const uint64_t* local_idx, const float* local_dist, const uint32_t* local_count,
                     uint32_t n_queries, uint32_t k, uint64_t* root_idx, float* root_dist, uint32_t* root_count) {
    BSR_GUARD(gather_impl(c, local_idx, local_dist, local_count, n_queries, k, root_idx, root_dist, root_count));
}

static int parallel_impl(bsr_comm* c, bsr_index* ix, const float* queries, uint32_t nq, uint32_t k,
                         uint64_t* out_idx, float* out_dist, uint32_t* out_count) {
    if (!ix) return set_error(BSR_E_INVALID, "null index");
    const bool single = !c || c->size == 1;
    const bool root = !c || c->rank == 0;
    if (nq && root && (!out_idx || !out_dist || !out_count)) return set_error(BSR_E_INVALID, "null output");
    if (c && c->device != ix->device) return set_error(BSR_E_INVALID, "communicator and index on different devices");
    // compute_local_top_k (:185-191; an error there is an error here, not an empty list)
    BSR_TRY(ix->search_device(queries, nq, k));
    if (!nq) return BSR_OK;
    const size_t nk = (size_t)nq * k;
    if (single) {
        BSR_TRY(bsr_copy_out_impl(ix, nq, k, out_idx, out_dist, out_count));
        bsr_index_collect_profile_impl(ix);
        return BSR_OK;
    }
    // gather_top_k_results (:194) as an RCCL all-gather on the index's stream, then the
    // root's merge (:200-202).
    BSR_TRY(allgather_lists(c, ix->d_idx, ix->d_dist, ix->d_cnt, nq, k, ix->stream));
    if (root) {
        c->h_idx.resize(nk * c->size);
        c->h_dist.resize(nk * c->size);
        c->h_cnt.resize((size_t)nq * c->size);
        BSR_HIP(hipMemcpyAsync(c->h_idx.data(), c->recv_idx.p, nk * c->size * sizeof(uint64_t), hipMemcpyDeviceToHost,
                               ix->stream));
        BSR_HIP(hipMemcpyAsync(c->h_dist.data(), c->recv_dist.p, nk * c->size * sizeof(float), hipMemcpyDeviceToHost,
                               ix->stream));
        BSR_HIP(hipMemcpyAsync(c->h_cnt.data(), c->recv_cnt.p, (size_t)nq * c->size * sizeof(uint32_t),
                               hipMemcpyDeviceToHost, ix->stream));
    }
    BSR_HIP(hipStreamSynchronize(ix->stream));
    bsr_index_collect_profile_impl(ix);
    if (!root) {
        if (out_count)
            for (uint32_t q = 0; q < nq; ++q) out_count[q] = 0;  // the reference's None
        return BSR_OK;
    }
    const bool host_out = !is_device_ptr(out_idx);
    std::vector<uint64_t> tmp_idx;
    std::vector<float> tmp_dist;
    std::vector<uint32_t> tmp_cnt;
    uint64_t* oi = out_idx;
    float* od = out_dist;
    uint32_t* oc = out_count;
    if (!host_out) {
        tmp_idx.resize(nk);
        tmp_dist.resize(nk);
        tmp_cnt.resize(nq);
        oi = tmp_idx.data();
        od = tmp_dist.data();
        oc = tmp_cnt.data();
    }
    if (c->size > 64) return set_error(BSR_E_INVALID, "at most 64 ranks");
    for (uint32_t q = 0; q < nq; ++q) {
        const uint32_t got = merge_sorted_lists(c->h_idx.data(), c->h_dist.data(), c->h_cnt.data(), (uint32_t)c->size,
                                                nq, k, q, k, oi + (size_t)q * k, od + (size_t)q * k);
        oc[q] = got;
        for (uint32_t i = got; i < k; ++i) {
            oi[(size_t)q * k + i] = ~0ull;
            od[(size_t)q * k + i] = __builtin_inff();
        }
    }
    if (!host_out) {
        BSR_HIP(hipMemcpy(out_idx, oi, nk * sizeof(uint64_t), hipMemcpyHostToDevice));
        BSR_HIP(hipMemcpy(out_dist, od, nk * sizeof(float), hipMemcpyHostToDevice));
        BSR_HIP(hipMemcpy(out_count, oc, (size_t)nq * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    return BSR_OK;
}

int bsr_parallel_top_k_similarity_search(bsr_comm* comm, bsr_index* ix, const float* queries, uint32_t n_queries,
                                         uint32_t k, uint64_t* out_idx, float* out_dist, uint32_t* out_count) {
    BSR_GUARD(parallel_impl(comm, ix, queries, n_queries, k, out_idx, out_dist, out_count));
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
