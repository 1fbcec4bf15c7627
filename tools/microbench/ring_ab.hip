// Microbenchmark + cross-check (tooling): the product filter kernel (k_filter.hip, namespace
// bsr: k_filter_qs16) against the lab variants (k_qs16_lab.hip) and the round-1 kernel
// (k_filter_lab.hip) on a
// synthetic int8 shard, interleaved in one process (same clocks), after a clock settle.
// Checks that both kernels emit the same candidate set per query (sorted keys equal) and the
// same sample scores, then times them.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../include
//        -I../../better-search-rag-rust_amd/csrc ring_ab.hip -o ring_ab
// Run:   ./ring_ab [rows] [queries] [rounds] [tau]
#include "k_filter.hip"
#include "k_filter_lab.hip"
#include "k_ring_lab.hip"
#include "k_qs16_lab.hip"

#include <stdio.h>
#include <string.h>


#include <algorithm>
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

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 1000000, nq = argc > 2 ? atoi(argv[2]) : 1000;
    const int rounds = argc > 3 ? atoi(argv[3]) : 20;
    const float tau_emit = argc > 4 ? atof(argv[4]) : 0.125f;
    const uint32_t ld = 768, qpad = (nq + 255) / 256 * 256, npad = (n + 255) / 256 * 256, cap = 1024;
    uint8_t *A8, *B8;
    float *tau, *as, *bs, *S;
    uint64_t* cand;
    uint32_t* cnt;
    CHECK(hipMalloc(&A8, (size_t)npad * ld));
    CHECK(hipMalloc(&B8, (size_t)qpad * ld));
    CHECK(hipMalloc(&as, npad / 32 * 4));
    CHECK(hipMalloc(&bs, qpad * 4));
    CHECK(hipMalloc(&tau, qpad * 4));
    CHECK(hipMalloc(&cand, (size_t)qpad * cap * 8));
    CHECK(hipMalloc(&cnt, qpad * 4));
    const uint32_t n_s = (n + 31) / 32, s_ld = (n_s + 127) / 128 * 128;
    CHECK(hipMalloc(&S, (size_t)qpad * s_ld * 4 + 4096 * 16));
    hipLaunchKernelGGL(fill_i8, dim3(4096), dim3(256), 0, 0, (int8_t*)A8, (size_t)npad * ld, 3);
    hipLaunchKernelGGL(fill_i8, dim3(1024), dim3(256), 0, 0, (int8_t*)B8, (size_t)qpad * ld, 4);
    hipLaunchKernelGGL(fill_f32, dim3(256), dim3(256), 0, 0, as, (size_t)npad / 32, 1.0f / (127.0f * 16.0f));
    hipLaunchKernelGGL(fill_f32, dim3(16), dim3(256), 0, 0, bs, (size_t)qpad, 1.0f / (127.0f * 16.0f));
    CHECK(hipDeviceSynchronize());
    bsr::GemmArgs g{};
    g.A = A8; g.B = B8; g.row_bytes = ld; g.a_stride = ld;
    g.n_rows = n; g.a_scale_rows = 32; g.n_qt = qpad / 256; g.n_rt = (n + 255) / 256;
    g.a_scale = as; g.b_scale = bs; g.tau = tau; g.cand = cand; g.cnt = cnt; g.cap = cap;
    const uint32_t per_xcd = g.n_qt >= 32 ? g.n_qt : (32 / g.n_qt) * g.n_qt, grid = 8 * per_xcd;
    const double ops = 2.0 * nq * (double)n * ld;

    struct V { const char* name; void (*k)(bsr::GemmArgs); std::vector<float> t; int nw; };
    std::vector<V> vs = {
        {"qs16 (product)", bsr::k_filter_qs16<true, 12>, {}, 8},
        {"qs16 staged (lab)", bsrlab::k_filter_qs16s<12, 0>, {}, 8},
        {"skewed groups (lab)", bsrlab::k_filter_qs16k<12>, {}, 8},
        {"level-1 only", bsrlab::k_filter_qs16s<12, 1>, {}, 8},
        {"qs8 (round 1)", bsrlab::k_filter_qs8<true, 12, false, 72>, {}, 8},
    };
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto run = [&](void (*k)(bsr::GemmArgs), const bsr::GemmArgs& a0, float tv, int nw = 8) -> float {
        // nw = 4: 128-query workgroups, two per CU
        bsr::GemmArgs a = a0;
        uint32_t gr = grid;
        if (nw == 4) {
            a.n_qt = qpad / 128;
            gr = 8 * ((64 / a.n_qt) * a.n_qt);
        }
        std::vector<float> ht(qpad, tv);
        CHECK(hipMemcpy(tau, ht.data(), qpad * 4, hipMemcpyHostToDevice));
        CHECK(hipMemset(cnt, 0, qpad * 4));
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k, dim3(gr), dim3(64 * nw), 0, 0, a);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        return ms;
    };
    // ---- cross-check: emitted candidate sets and sample scores
    const int n_check = 3;  // product + the staged variants (emitting)
    std::vector<std::vector<uint64_t>> sets(n_check);
    for (int i = 0; i < n_check; ++i) {
        run(vs[i].k, g, tau_emit, vs[i].nw);
        std::vector<uint32_t> hc(qpad);
        CHECK(hipMemcpy(hc.data(), cnt, qpad * 4, hipMemcpyDeviceToHost));
        std::vector<uint64_t> hk((size_t)qpad * cap);
        CHECK(hipMemcpy(hk.data(), cand, hk.size() * 8, hipMemcpyDeviceToHost));
        double tot = 0;
        for (uint32_t q = 0; q < nq; ++q) {
            const uint32_t c = std::min(hc[q], cap);
            tot += hc[q];
            std::vector<uint64_t> v(hk.begin() + (size_t)q * cap, hk.begin() + (size_t)q * cap + c);
            std::sort(v.begin(), v.end());
            v.push_back(0xFFFFFFFFFFFFFFFFull - q);  // separator
            sets[i].insert(sets[i].end(), v.begin(), v.end());
        }
        printf("[%s] emitted per query %.1f\n", vs[i].name, tot / nq);
    }
    for (int i = 1; i < n_check; ++i)
        printf("emitted sets %s vs %s: %s\n", vs[i].name, vs[0].name, sets[0] == sets[i] ? "IDENTICAL" : "DIFFER");
    {
        bsr::GemmArgs gs = g;
        gs.a_stride = (uint64_t)ld * 32; gs.a_scale_rows = 128; gs.n_rows = n_s; gs.n_rt = (n_s + 255) / 256;
        gs.S = S; gs.s_ld = s_ld; gs.s_compact = 0;
        std::vector<std::vector<float>> sv(2);
        void (*ks[2])(bsr::GemmArgs) = {bsrlab::k_filter_qs8<false, 12, false, 72>, bsr::k_filter_qs16<false, 12>};
        for (int i = 0; i < 2; ++i) {
            CHECK(hipMemset(S, 0, (size_t)qpad * s_ld * 4));
            run(ks[i], gs, 0.0f);
            sv[i].resize((size_t)nq * s_ld);
            CHECK(hipMemcpy(sv[i].data(), S, sv[i].size() * 4, hipMemcpyDeviceToHost));
        }
        size_t bad = 0;
        for (uint32_t q = 0; q < nq; ++q)
            for (uint32_t r = 0; r < n_s; ++r) bad += sv[0][(size_t)q * s_ld + r] != sv[1][(size_t)q * s_ld + r];
        printf("sample scores %s (%zu differ)\n", bad ? "DIFFER" : "IDENTICAL", bad);
    }
    // ---- timing: settle ~2 s, then interleaved rounds
    for (int i = 0; i < 200; ++i) run(vs[i & 1].k, g, tau_emit, vs[i & 1].nw);
    if (argc > 5 && strcmp(argv[5], "sample") == 0) {  // the sample pass vs the emit pass on n/32 rows
        bsr::GemmArgs gs = g;
        gs.n_rows = n_s; gs.n_rt = (n_s + 255) / 256;
        const uint32_t n_vals = (n_s + 31) / 32;
        gs.S = S; gs.s_ld = (n_s + 255) / 256 * 8; gs.s_compact = 1;
        struct W { const char* name; void (*k)(bsr::GemmArgs); bsr::GemmArgs a; float tau; std::vector<float> t; };
        std::vector<W> ws = {{"sample compact", bsr::k_filter_qs16<false, 12>, gs, 0.0f, {}},
                             {"sample full", bsr::k_filter_qs16<false, 12>, gs, 0.0f, {}},
                             {"emit tau=inf", bsr::k_filter_qs16<true, 12>, gs, 1e9f, {}}};
        ws[1].a.s_compact = 0; ws[1].a.s_ld = (n_s + 255) / 256 * 256;
        for (int r = 0; r < rounds; ++r)
            for (auto& w : ws) w.t.push_back(run(w.k, w.a, w.tau));
        for (auto& w : ws) {
            std::sort(w.t.begin(), w.t.end());
            printf("%-16s rows %u (vals %u)  median %7.4f ms  min %7.4f ms\n", w.name, n_s, n_vals, w.t[w.t.size() / 2], w.t[0]);
        }
        return 0;
    }
    if (argc > 5 && strcmp(argv[5], "sweep") == 0) {  // cost of emission: time vs tau (first two variants)
        for (float tv : {1e9f, 0.145f, 0.14f, 0.135f, 0.13f, 0.125f, 0.12f}) {
            for (int i = 0; i < 2; ++i) {
                std::vector<float> t;
                for (int r = 0; r < rounds; ++r) t.push_back(run(vs[i].k, g, tv, vs[i].nw));
                std::sort(t.begin(), t.end());
                std::vector<uint32_t> hc(qpad);
                CHECK(hipMemcpy(hc.data(), cnt, qpad * 4, hipMemcpyDeviceToHost));
                double tot = 0;
                for (uint32_t q = 0; q < nq; ++q) tot += hc[q];
                printf("%-18s tau=%-8g emitted/query %7.1f  median %7.4f ms\n", vs[i].name, tv, tot / nq, t[t.size() / 2]);
            }
        }
        return 0;
    }
    for (float tv : {1e9f, tau_emit}) {
        for (auto& v : vs) v.t.clear();
        for (int r = 0; r < rounds; ++r)
            for (auto& v : vs) v.t.push_back(run(v.k, g, tv, v.nw));
        for (auto& v : vs) {
            std::sort(v.t.begin(), v.t.end());
            const float med = v.t[v.t.size() / 2];
            printf("%-18s tau=%-8g median %7.4f ms  min %7.4f ms  %7.1f TOP/s = %.3f of the 5.0 POP/s int8 peak\n",
                   v.name, tv, med, v.t[0], ops / (med * 1e-3) / 1e12, ops / (med * 1e-3) / 5.0e15);
        }
    }
    return 0;
}
