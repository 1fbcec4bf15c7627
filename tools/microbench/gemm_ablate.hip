// Microbenchmark (tooling): the MFMA filter kernel and its ablations on a synthetic shard.
// Includes the product kernels directly.  Build:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../include -I../../better-search-rag-rust_amd/csrc gemm_ablate.hip -o gemm_ablate
#include "kernels.hip"
#include <stdio.h>
#include <vector>
#include <algorithm>

using namespace bsr;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void fill_bf16(uint16_t* p, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t h = splitmix64(seed + i);
        float v = ((float)(h >> 40) * (1.0f / 8388608.0f) - 1.0f) * 0.036f;
        p[i] = f32_to_bf16_rne(v);
    }
}

template <class F>
float timeit(F f, int reps = 5) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    f(); CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a)); f(); CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
        float ms; CHECK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best;
    }
    return best;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 1000000, nq = argc > 2 ? atoi(argv[2]) : 1000, ld = 768;
    const uint32_t qpad = (nq + 255) / 256 * 256, npad = (n + 255) / 256 * 256;
    uint16_t *A, *B; float* tau; uint64_t* cand; uint32_t* cnt;
    const uint32_t cap = 1024;
    CHECK(hipMalloc(&A, (size_t)npad * ld * 2)); CHECK(hipMalloc(&B, (size_t)qpad * ld * 2));
    CHECK(hipMalloc(&tau, qpad * 4)); CHECK(hipMalloc(&cand, (size_t)qpad * cap * 8)); CHECK(hipMalloc(&cnt, qpad * 4));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, A, (size_t)npad * ld, 1);
    hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, B, (size_t)qpad * ld, 2);
    const float tauv = argc > 3 ? atof(argv[3]) : 1e9f;
    std::vector<float> ht(qpad, tauv);
    CHECK(hipMemcpy(tau, ht.data(), qpad * 4, hipMemcpyHostToDevice));
    GemmArgs g{};
    g.A = A; g.a_row_stride = ld; g.n_rows = n; g.B = B; g.ld = ld; g.n_qt = qpad / 256;
    g.tau = tau; g.cand = cand; g.cnt = cnt; g.cap = cap;
    const uint32_t per_xcd = (32 / g.n_qt) * g.n_qt, grid = 8 * per_xcd;
    const double flops = 2.0 * nq * (double)n * ld;
    struct V { const char* name; void (*k)(GemmArgs); float tau; std::vector<float> t; };
    std::vector<V> vs = {
        {"v2 tau=inf", k_gemm_filter2<true, 0>, 1e9f, {}},
        {"v4 tau=inf", k_gemm_filter4<true, 0>, 1e9f, {}},
        {"v2 tau=0.05", k_gemm_filter2<true, 0>, 0.05f, {}},
        {"v4 tau=0.05", k_gemm_filter4<true, 0>, 0.05f, {}},
        {"v4 tau=0.0415", k_gemm_filter4<true, 0>, 0.0415f, {}},
        {"v4 no-DMA", k_gemm_filter4<true, 1>, 1e9f, {}},
        {"v4 DMA-only", k_gemm_filter4<true, 3>, 1e9f, {}},
    };
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    for (int r = 0; r < rounds; ++r) {
        for (auto& v : vs) {
            std::vector<float> ht(qpad, v.tau);
            CHECK(hipMemcpy(tau, ht.data(), qpad * 4, hipMemcpyHostToDevice));
            CHECK(hipMemset(cnt, 0, qpad * 4));
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(v.k, dim3(grid), dim3(512), 0, 0, g);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0) v.t.push_back(ms);
            if (r == rounds - 1 && v.tau < 1e8f) {
                std::vector<uint32_t> hc(qpad);
                CHECK(hipMemcpy(hc.data(), cnt, qpad * 4, hipMemcpyDeviceToHost));
                double tot = 0; for (uint32_t i = 0; i < nq; ++i) tot += hc[i];
                printf("  [%s] emitted per query %.1f\n", v.name, tot / nq);
            }
        }
    }
    for (auto& v : vs) {
        std::sort(v.t.begin(), v.t.end());
        float med = v.t[v.t.size() / 2], mn = v.t[0];
        printf("%-18s median %7.3f ms  min %7.3f ms  (%6.1f TF/s at median)\n", v.name, med, mn, flops / (med * 1e-3) / 1e12);
    }
    return 0;
}
