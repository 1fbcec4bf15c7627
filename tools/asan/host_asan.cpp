// host_asan.cpp -- the library's host code under AddressSanitizer + UBSan (VERDICT r04
// item 6).  No GPU: everything here is host-side -- the host merge (merge.cpp, behind
// bsr_global_top_k), the exchange over a host transport (capi.cpp: bsr_gather_top_k,
// bsr_gather_global_top_k, the parallel search's header + standard path with empty contributions,
// bsr_allgather_bytes, bsr_broadcast), interval_by_rank and the parquet vector store
// (vstore.cpp).  P ranks are P threads of this process; the host transport is a barrier-based
// in-process all-gather.  Every result is checked against a plain restatement here.
// Build + run: make -C tools/asan run
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <barrier>
#include <cmath>
#include <functional>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "bsr.h"
#include "bsr_vstore.h"

static int g_fail = 0;
#define EXPECT(c, ...)                                   \
    do {                                                 \
        if (!(c)) {                                      \
            printf("FAIL %s:%d: ", __FILE__, __LINE__);  \
            printf(__VA_ARGS__);                         \
            printf("\n");                                \
            ++g_fail;                                    \
        }                                                \
    } while (0)

// compute_global_top_k (src/mpi_helpers/metrics.rs:141-171): rank-order concatenation, stable
// sort by distance, first k distinct indices
static void ref_merge(const std::vector<std::pair<uint64_t, float>>& cat, uint32_t k, std::vector<uint64_t>& oi,
                      std::vector<float>& od) {
    std::vector<std::pair<uint64_t, float>> v = cat;
    std::stable_sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.second < b.second; });
    oi.clear();
    od.clear();
    for (auto& e : v) {
        if (oi.size() == k) break;
        if (std::find(oi.begin(), oi.end(), e.first) != oi.end()) continue;
        oi.push_back(e.first);
        od.push_back(e.second);
    }
}

static void test_merge(std::mt19937_64& rng) {
    for (int it = 0; it < 300; ++it) {
        const uint32_t L = 1 + rng() % 9, Q = 1 + rng() % 7, kin = 1 + rng() % 20, k = 1 + rng() % 25;
        std::vector<uint64_t> idx((size_t)L * Q * kin);
        std::vector<float> dist(idx.size());
        std::vector<uint32_t> cnt((size_t)L * Q);
        for (auto& c : cnt) c = rng() % (kin + 1);
        for (size_t i = 0; i < idx.size(); ++i) {
            idx[i] = rng() % 40;  // duplicates across lists on purpose
            dist[i] = (float)(rng() % 16) / 8.0f;  // ties on purpose
        }
        std::vector<uint64_t> oi((size_t)Q * k);
        std::vector<float> od((size_t)Q * k);
        std::vector<uint32_t> oc(Q);
        const int st = bsr_global_top_k(idx.data(), dist.data(), cnt.data(), L, Q, kin, k, oi.data(), od.data(),
                                        oc.data());
        EXPECT(st == BSR_OK, "merge status %d: %s", st, bsr_last_error());
        for (uint32_t q = 0; q < Q; ++q) {
            std::vector<std::pair<uint64_t, float>> cat;
            for (uint32_t l = 0; l < L; ++l)
                for (uint32_t j = 0; j < cnt[(size_t)l * Q + q]; ++j)
                    cat.push_back({idx[((size_t)l * Q + q) * kin + j], dist[((size_t)l * Q + q) * kin + j]});
            std::vector<uint64_t> wi;
            std::vector<float> wd;
            ref_merge(cat, k, wi, wd);
            EXPECT(oc[q] == wi.size(), "count q%u %u vs %zu", q, oc[q], wi.size());
            for (uint32_t j = 0; j < oc[q] && j < wi.size(); ++j)
                EXPECT(oi[(size_t)q * k + j] == wi[j] && od[(size_t)q * k + j] == wd[j], "entry q%u j%u", q, j);
        }
    }
    // a NaN distance is reported, not merged (the reference panics)
    uint64_t i1[2] = {1, 2};
    float d1[2] = {0.5f, NAN};
    uint32_t c1 = 2, oc = 0;
    uint64_t oi[2];
    float od[2];
    EXPECT(bsr_global_top_k(i1, d1, &c1, 1, 1, 2, 2, oi, od, &oc) == BSR_E_NONFINITE, "NaN not reported");
}

static void test_interval(std::mt19937_64& rng) {
    for (int it = 0; it < 2000; ++it) {
        const int32_t size = 1 + rng() % 70;
        const uint64_t n = rng() % 1000;
        uint64_t covered = 0;
        for (int32_t r = 0; r < size; ++r) {
            bsr_rank_interval iv;
            EXPECT(bsr_interval_by_rank(r, size, n, &iv) == BSR_OK, "interval");
            if (iv.end_index > iv.start_index) covered += iv.end_index - iv.start_index;
        }
        EXPECT(covered >= std::min<uint64_t>(n, n), "coverage");
    }
    bsr_rank_interval iv;
    EXPECT(bsr_interval_by_rank(4, 4, 10, &iv) == BSR_E_INVALID, "rank out of range accepted");
}

// ---- P ranks as P threads over an in-process host all-gather ---------------------------------
struct Hub {
    int P;
    std::barrier<> bar;
    std::vector<const void*> send;
    explicit Hub(int p) : P(p), bar(p), send(p) {}
};
struct RankCtx {
    Hub* hub;
    int rank;
};
static int hub_allgather(const void* s, void* r, uint64_t bytes, void* user) {
    RankCtx* c = static_cast<RankCtx*>(user);
    c->hub->send[c->rank] = s;
    c->hub->bar.arrive_and_wait();
    for (int i = 0; i < c->hub->P; ++i) memcpy(static_cast<uint8_t*>(r) + (size_t)i * bytes, c->hub->send[i], bytes);
    c->hub->bar.arrive_and_wait();  // (every rank has read every send buffer)
    return 0;
}

static void run_ranks(int P, const std::function<void(bsr_comm*, int)>& body) {
    Hub hub(P);
    std::vector<RankCtx> ctx(P);
    std::vector<std::thread> th;
    for (int r = 0; r < P; ++r) {
        ctx[r] = {&hub, r};
        th.emplace_back([&, r] {
            bsr_comm* c = nullptr;
            if (bsr_comm_init_host(r, P, hub_allgather, &ctx[r], &c) != BSR_OK) {
                printf("FAIL comm init: %s\n", bsr_last_error());
                ++g_fail;
                return;
            }
            body(c, r);
            bsr_comm_destroy(c);
        });
    }
    for (auto& t : th) t.join();
}

static void test_exchange(std::mt19937_64& rng0) {
    for (int P : {1, 2, 3, 5, 8}) {
        const uint32_t Q = 6, k = 7;
        // every rank's lists, drawn up front (the threads read them)
        std::vector<std::vector<uint64_t>> li(P, std::vector<uint64_t>(Q * k));
        std::vector<std::vector<float>> ld(P, std::vector<float>(Q * k));
        std::vector<std::vector<uint32_t>> lc(P, std::vector<uint32_t>(Q));
        for (int r = 0; r < P; ++r)
            for (uint32_t q = 0; q < Q; ++q) {
                lc[r][q] = rng0() % (k + 1);
                std::vector<float> d(k);
                for (auto& x : d) x = (float)(rng0() % 32) / 16.0f;
                std::sort(d.begin(), d.end());
                for (uint32_t j = 0; j < k; ++j) {
                    li[r][q * k + j] = 100 * r + rng0() % 50;
                    ld[r][q * k + j] = d[j];
                }
            }
        std::vector<uint64_t> gi(Q * k);
        std::vector<float> gd(Q * k);
        std::vector<uint32_t> gc(Q);
        std::vector<uint64_t> ri((size_t)P * Q * k);
        std::vector<float> rd(ri.size());
        std::vector<uint32_t> rc((size_t)P * Q);
        run_ranks(P, [&](bsr_comm* c, int r) {
            std::vector<uint64_t> oi(Q * k);
            std::vector<float> od(Q * k);
            std::vector<uint32_t> oc(Q);
            int st = bsr_gather_global_top_k(c, li[r].data(), ld[r].data(), lc[r].data(), Q, k, oi.data(), od.data(),
                                             oc.data());
            EXPECT(st == BSR_OK, "gather_global P%d r%d: %d %s", P, r, st, bsr_last_error());
            if (r == 0) gi = oi, gd = od, gc = oc;
            else
                for (uint32_t q = 0; q < Q; ++q) EXPECT(oc[q] == 0, "non-root count");
            st = bsr_gather_top_k(c, li[r].data(), ld[r].data(), lc[r].data(), Q, k, r == 0 ? ri.data() : nullptr,
                                  r == 0 ? rd.data() : nullptr, r == 0 ? rc.data() : nullptr);
            EXPECT(st == BSR_OK, "gather_top_k: %d %s", st, bsr_last_error());
            // the timing all-gather and the query broadcast (src/main.rs:123-125)
            double mine = r + 0.5, all[8];
            EXPECT(bsr_allgather_bytes(c, &mine, all, sizeof mine) == BSR_OK, "allgather_bytes");
            for (int i = 0; i < P; ++i) EXPECT(all[i] == i + 0.5, "allgather_bytes value");
            float qv[5] = {(float)r, 1, 2, 3, 4};
            EXPECT(bsr_broadcast(c, qv, sizeof qv, 0) == BSR_OK, "broadcast");
            EXPECT(qv[0] == 0.0f, "broadcast value");
            // the parallel search without a GPU: no index on any rank -- every rank still takes
            // part in every collective (empty contributions); non-roots report their error, the
            // root BSR_PARTIAL; mismatched batch shapes are rejected on every rank
            std::vector<float> qs(4 * 16, 0.0f);
            st = bsr_parallel_top_k_similarity_search(c, nullptr, qs.data(), 4, k, oi.data(), od.data(), oc.data());
            if (P == 1) EXPECT(st == BSR_E_INVALID || st == BSR_PARTIAL, "P1 status %d", st);
            else EXPECT(r == 0 ? st == BSR_PARTIAL : st == BSR_E_INVALID, "parallel st %d rank %d", st, r);
            if (P > 1) {
                st = bsr_parallel_top_k_similarity_search(c, nullptr, qs.data(), r == P - 1 ? 3 : 4, k, oi.data(),
                                                          od.data(), oc.data());
                EXPECT(st == BSR_E_INVALID && strstr(bsr_last_error(), "disagree"), "shape mismatch st %d", st);
            }
        });
        for (uint32_t q = 0; q < Q; ++q) {
            std::vector<std::pair<uint64_t, float>> cat;
            for (int r = 0; r < P; ++r) {
                for (uint32_t j = 0; j < lc[r][q]; ++j) cat.push_back({li[r][q * k + j], ld[r][q * k + j]});
                EXPECT(rc[(size_t)r * Q + q] == lc[r][q], "gathered count");
            }
            std::vector<uint64_t> wi;
            std::vector<float> wd;
            ref_merge(cat, k, wi, wd);
            EXPECT(gc[q] == wi.size(), "P%d q%u count %u vs %zu", P, q, gc[q], wi.size());
            for (uint32_t j = 0; j < gc[q] && j < wi.size(); ++j)
                EXPECT(gi[q * k + j] == wi[j] && gd[q * k + j] == wd[j], "P%d q%u j%u", P, q, j);
        }
    }
}

static void test_vstore(std::mt19937_64& rng) {
    char tmpl[] = "/tmp/bsr_asan_XXXXXX";
    const char* dir = mkdtemp(tmpl);
    EXPECT(dir != nullptr, "mkdtemp");
    char path[4096];
    EXPECT(bsr_vstore_global_path(dir, path, sizeof path) == BSR_OK, "global path");
    char small[8];
    EXPECT(bsr_vstore_local_path(dir, 3, small, sizeof small) == BSR_E_INVALID, "short buffer accepted");
    bsr_vstore* vs = nullptr;
    EXPECT(bsr_vstore_open(path, 1, &vs) == BSR_OK, "open empty: %s", bsr_last_error());
    const uint32_t dim = 24, n = 777;
    std::vector<float> rows((size_t)n * dim);
    for (auto& x : rows) x = (float)(rng() % 2001) / 1000.0f - 1.0f;
    EXPECT(bsr_vstore_append_many(vs, rows.data(), 500, dim) == BSR_OK, "append");
    EXPECT(bsr_vstore_append_many(vs, rows.data() + 500 * dim, n - 500, dim) == BSR_OK, "append 2");
    EXPECT(bsr_vstore_persist(vs) == BSR_OK, "persist: %s", bsr_last_error());
    bsr_vstore_close(vs);
    vs = nullptr;
    EXPECT(bsr_vstore_open(path, 0, &vs) == BSR_OK, "reopen: %s", bsr_last_error());
    uint64_t cnt = 0;
    EXPECT(bsr_vstore_get_count(vs, &cnt) == BSR_OK && cnt == n, "count %llu", (unsigned long long)cnt);
    std::vector<float> slab((size_t)n * dim);
    uint64_t got = 0;
    EXPECT(bsr_vstore_read_slab(vs, 0, n, dim, slab.data(), n, &got) == BSR_OK && got == n, "read_slab");
    EXPECT(memcmp(slab.data(), rows.data(), slab.size() * 4) == 0, "slab content");
    uint64_t r_rows = 0, r_floats = 0;
    EXPECT(bsr_vstore_get_many(vs, 100, 50, nullptr, 0, nullptr, 0, &r_rows, &r_floats) == BSR_OK &&
               r_rows == 50 && r_floats == 50 * dim, "get_many sizes");
    std::vector<float> part(r_floats);
    std::vector<uint32_t> lens(r_rows);
    EXPECT(bsr_vstore_get_many(vs, 100, 50, part.data(), part.size(), lens.data(), lens.size(), &r_rows,
                               &r_floats) == BSR_OK, "get_many");
    EXPECT(memcmp(part.data(), rows.data() + 100 * dim, part.size() * 4) == 0, "get_many content");
    EXPECT(bsr_vstore_get_many(vs, 100, 50, part.data(), part.size() - 1, lens.data(), lens.size(), &r_rows,
                               &r_floats) == BSR_E_INVALID, "short capacity accepted");
    float one[dim];
    uint32_t len = 0;
    EXPECT(bsr_vstore_get(vs, n - 1, one, dim, &len) == BSR_OK && len == dim, "get");
    EXPECT(memcmp(one, rows.data() + (size_t)(n - 1) * dim, sizeof one) == 0, "get content");
    EXPECT(bsr_vstore_get(vs, n, one, dim, &len) == BSR_E_INVALID, "get past the end accepted");
    EXPECT(bsr_vstore_read_slab(vs, 0, 10, dim + 1, slab.data(), n, &got) == BSR_E_DIM, "wrong dim accepted");
    EXPECT(bsr_vstore_reset(vs) == BSR_OK, "reset");
    EXPECT(bsr_vstore_get_count(vs, &cnt) == BSR_OK && cnt == 0, "reset count");
    EXPECT(bsr_vstore_reload(vs, 0) == BSR_OK, "reload: %s", bsr_last_error());
    EXPECT(bsr_vstore_get_count(vs, &cnt) == BSR_OK && cnt == n, "reload count");
    bsr_vstore_close(vs);
    std::string cmd = std::string("rm -rf ") + dir;
    EXPECT(system(cmd.c_str()) == 0, "cleanup");
}

int main() {
    std::mt19937_64 rng(20251018);
    test_merge(rng);
    test_interval(rng);
    test_exchange(rng);
    test_vstore(rng);
    printf("%s: host code under ASan + UBSan, %d failure(s)\n", g_fail ? "FAILED" : "OK", g_fail);
    return g_fail ? 1 : 0;
}
