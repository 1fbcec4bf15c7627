// Lab harness (round 5): the small-shard bisection.  The product emit filter k_filter_qs16<true,12>
// against the same kernel at earlier commits of this repository (tools/microbench/extract_old.sh:
// round 2's final kernel, the static DMA schedule, the dynamic tail, round 3's final kernel, the
// XCD-local tail pools, the row-stream gangs), interleaved in one process (same clocks) on a
// synthetic int8 shard; every variant must emit the same candidate set per query before it is
// timed.  Build: make -C tools/microbench filter_hist   Run: ./filter_hist [rows] [queries] [rounds] [tau]
#include "k_filter.hip"
#include "old/r02/k_filter.hip"
#include "old/static/k_filter.hip"
#include "old/dyntail/k_filter.hip"
#include "old/r03/k_filter.hip"
#include "old/xpools/k_filter.hip"
#include "old/gangs/k_filter.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <vector>

#define CHECK(x)                                                       \
    do {                                                               \
        hipError_t e_ = (x);                                           \
        if (e_ != hipSuccess) {                                        \
            printf("%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                   \
        }                                                              \
    } while (0)

__global__ void fill_i8(int8_t* p, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t h = bsr::splitmix64(seed + i);
        p[i] = (int8_t)((int)(h % 255) - 127);
    }
}
__global__ void fill_f32(float* p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

// Each commit's GemmArgs is a prefix of today's (fields were only appended): copy that prefix.
template <class GA>
static GA as_old(const bsr::GemmArgs& g) {
    static_assert(sizeof(GA) <= sizeof(bsr::GemmArgs), "old GemmArgs is a prefix");
    GA o;
    memcpy(&o, &g, sizeof(GA));
    return o;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 1000000, nq = argc > 2 ? atoi(argv[2]) : 1000;
    const int rounds = argc > 3 ? atoi(argv[3]) : 15;
    const float tau_emit = argc > 4 ? atof(argv[4]) : 0.1284f;
    const uint32_t ld = 768, qpad = (nq + 255) / 256 * 256, npad = (n + 255) / 256 * 256, cap = 1024;
    const uint32_t n_cnt = qpad + 8 * bsr::kTailCounters + bsr::kGangWords;
    uint8_t *A8, *B8;
    float *tau, *as, *bs;
    uint64_t* cand;
    uint32_t* cnt;
    CHECK(hipMalloc(&A8, (size_t)npad * ld));
    CHECK(hipMalloc(&B8, (size_t)qpad * ld));
    CHECK(hipMalloc(&as, npad / 32 * 4));
    CHECK(hipMalloc(&bs, qpad * 4));
    CHECK(hipMalloc(&tau, qpad * 4));
    CHECK(hipMalloc(&cand, (size_t)qpad * cap * 8));
    CHECK(hipMalloc(&cnt, n_cnt * 4));
    hipLaunchKernelGGL(fill_i8, dim3(4096), dim3(256), 0, 0, (int8_t*)A8, (size_t)npad * ld, 3);
    hipLaunchKernelGGL(fill_i8, dim3(1024), dim3(256), 0, 0, (int8_t*)B8, (size_t)qpad * ld, 4);
    hipLaunchKernelGGL(fill_f32, dim3(256), dim3(256), 0, 0, as, (size_t)npad / 32, 1.0f / (127.0f * 16.0f));
    hipLaunchKernelGGL(fill_f32, dim3(16), dim3(256), 0, 0, bs, (size_t)qpad, 1.0f / (127.0f * 16.0f));
    CHECK(hipDeviceSynchronize());
    bsr::GemmArgs g{};
    g.A = A8; g.B = B8; g.row_bytes = ld; g.a_stride = ld;
    g.n_rows = n; g.a_scale_rows = 32; g.n_qt = qpad / 256; g.n_rt = (n + 127) / 128;
    g.a_scale = as; g.b_scale = bs; g.tau = tau; g.cand = cand; g.cnt = cnt; g.cap = cap;
    g.tail = cnt + qpad;
    const uint32_t per_xcd = g.n_qt >= 32 ? g.n_qt : (32 / g.n_qt) * g.n_qt, grid = 8 * per_xcd;
    const double ops = 2.0 * nq * (double)n * ld;

    struct V { const char* name; std::function<void()> launch; std::vector<float> t; };
    const auto g_r02 = as_old<bsr_r02::GemmArgs>(g);
    const auto g_static = as_old<bsr_static::GemmArgs>(g);
    const auto g_dyn = as_old<bsr_dyntail::GemmArgs>(g);
    const auto g_r03 = as_old<bsr_r03::GemmArgs>(g);
    const auto g_xp = as_old<bsr_xpools::GemmArgs>(g);
    const auto g_gang = as_old<bsr_gangs::GemmArgs>(g);
    const dim3 G(grid), B(512);
    // FOCUS=1 (default): the product against its round-5 candidates and the two fastest earlier
    // kernels; FOCUS=0: every commit of the history as well
    const bool focus = getenv("FOCUS") == nullptr || atoi(getenv("FOCUS")) != 0;
    std::vector<V> vs = {
        {"product", [&] { hipLaunchKernelGGL((bsr::k_filter_qs16<true, 12>), G, B, 0, 0, g); }, {}},
        {"static", [&] { hipLaunchKernelGGL((bsr_static::k_filter_qs16<true, 12>), G, B, 0, 0, g_static); }, {}},
        {"dyntail", [&] { hipLaunchKernelGGL((bsr_dyntail::k_filter_qs16<true, 12>), G, B, 0, 0, g_dyn); }, {}},
        // round-5 variants of the product: GANG = 0 (no gang code compiled), TAILX = 0 (one tail
        // counter per query tile), L2 = 1 (level 2's bool-array form), FW = 0 (no explicit wait
        // in the flush)
        {"g0_l2b_fw0", [&] { hipLaunchKernelGGL((bsr::k_filter_qs16<true, 12, 0, 8, 0, 0, 1, 0>), G, B, 0, 0, g); }, {}},
        {"g0_t0_l2b_fw0", [&] { hipLaunchKernelGGL((bsr::k_filter_qs16<true, 12, 0, 0, 0, 0, 1, 0>), G, B, 0, 0, g); }, {}},
        {"g2_l2b_fw0", [&] { hipLaunchKernelGGL((bsr::k_filter_qs16<true, 12, 0, 8, 2, 0, 1, 0>), G, B, 0, 0, g); }, {}},
    };
    if (!focus) {
        std::vector<V> more = {
            {"r02", [&] { hipLaunchKernelGGL((bsr_r02::k_filter_qs16<true, 12>), G, B, 0, 0, g_r02); }, {}},
            {"r03", [&] { hipLaunchKernelGGL((bsr_r03::k_filter_qs16<true, 12>), G, B, 0, 0, g_r03); }, {}},
            {"xpools", [&] { hipLaunchKernelGGL((bsr_xpools::k_filter_qs16<true, 12>), G, B, 0, 0, g_xp); }, {}},
            {"gangs", [&] { hipLaunchKernelGGL((bsr_gangs::k_filter_qs16<true, 12>), G, B, 0, 0, g_gang); }, {}},
            {"g0", [&] { hipLaunchKernelGGL((bsr::k_filter_qs16<true, 12, 0, 8, 0>), G, B, 0, 0, g); }, {}},
            {"g0_l2b", [&] { hipLaunchKernelGGL((bsr::k_filter_qs16<true, 12, 0, 8, 0, 0, 1>), G, B, 0, 0, g); }, {}},
            {"g0_fw0", [&] { hipLaunchKernelGGL((bsr::k_filter_qs16<true, 12, 0, 8, 0, 0, 0, 0>), G, B, 0, 0, g); }, {}},
            {"g0_t0", [&] { hipLaunchKernelGGL((bsr::k_filter_qs16<true, 12, 0, 0, 0>), G, B, 0, 0, g); }, {}},
        };
        vs.insert(vs.end(), more.begin(), more.end());
    }

    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto run = [&](V& v, float tv) -> float {
        std::vector<float> ht(qpad, tv);
        for (uint32_t q = nq; q < qpad; ++q) ht[q] = INFINITY;  // padding queries never emit
        CHECK(hipMemcpy(tau, ht.data(), qpad * 4, hipMemcpyHostToDevice));
        CHECK(hipMemset(cnt, 0, n_cnt * 4));
        CHECK(hipEventRecord(e0));
        v.launch();
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        return ms;
    };
    std::vector<std::vector<uint64_t>> sets(vs.size());
    for (size_t i = 0; i < vs.size(); ++i) {
        run(vs[i], tau_emit);
        std::vector<uint32_t> hc(qpad);
        CHECK(hipMemcpy(hc.data(), cnt, qpad * 4, hipMemcpyDeviceToHost));
        std::vector<uint64_t> hk((size_t)qpad * cap);
        CHECK(hipMemcpy(hk.data(), cand, hk.size() * 8, hipMemcpyDeviceToHost));
        double tot = 0;
        uint32_t over = 0;
        for (uint32_t q = 0; q < nq; ++q) {
            const uint32_t c = hc[q] <= cap ? hc[q] : 0;
            over += hc[q] > cap;
            tot += hc[q];
            std::vector<uint64_t> v(hk.begin() + (size_t)q * cap, hk.begin() + (size_t)q * cap + c);
            std::sort(v.begin(), v.end());
            v.push_back(0xFFFFFFFFFFFFFFFFull - q);
            sets[i].insert(sets[i].end(), v.begin(), v.end());
        }
        printf("[%s] emitted per query %.1f (overflowed lists %u)\n", vs[i].name, tot / nq, over);
    }
    bool same = true;
    for (size_t i = 1; i < vs.size(); ++i) {
        printf("emitted sets %s vs %s: %s\n", vs[i].name, vs[0].name, sets[0] == sets[i] ? "IDENTICAL" : "DIFFER");
        same &= sets[0] == sets[i];
    }
    fflush(stdout);
    if (!same) return 2;
    for (int i = 0; i < 60; ++i) run(vs[i % vs.size()], tau_emit);  // settle the clock
    for (float tv : {INFINITY, tau_emit}) {
        for (auto& v : vs) v.t.clear();
        for (int r = 0; r < rounds; ++r)
            for (size_t j = 0; j < vs.size(); ++j) {  // rotate the order every round
                V& v = vs[(j + r) % vs.size()];
                v.t.push_back(run(v, tv));
            }
        for (auto& v : vs) {
            std::sort(v.t.begin(), v.t.end());
            const float med = v.t[v.t.size() / 2];
            printf("%-12s rows %9u tau=%-8g median %7.4f ms  min %7.4f ms  %7.1f TOP/s = %.4f of the int8 peak\n",
                   v.name, n, tv, med, v.t[0], ops / (med * 1e-3) / 1e12, ops / (med * 1e-3) / 5.0e15);
        }
        fflush(stdout);
    }
    return 0;
}
