// Microbenchmark (tooling): the MFMA filter kernel (int8 and bf16 operands) and its
// ablations on a synthetic shard.  Includes the product kernel source directly.  Build:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../include -I../../better-search-rag-rust_amd/csrc gemm_ablate.hip -o gemm_ablate
// Run: ./gemm_ablate [rows] [queries] [rounds] [variant-substring]
#include "k_filter_lab.hip"
#include <stdio.h>
#include <vector>
#include <algorithm>
#include <string.h>

using namespace bsr;
using namespace bsrlab;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// bf16: U(-0.036, 0.036) per element; int8: U{-127..127} (scores = I * s_a * s_b)
__global__ void fill_bf16(uint16_t* p, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t h = splitmix64(seed + i);
        float v = ((float)(h >> 40) * (1.0f / 8388608.0f) - 1.0f) * 0.036f;
        p[i] = f32_to_bf16_rne(v);
    }
}
__global__ void fill_i8(int8_t* p, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t h = splitmix64(seed + i);
        p[i] = (int8_t)((int)(h % 255) - 127);
    }
}
__global__ void fill_f32(float* p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 1000000, nq = argc > 2 ? atoi(argv[2]) : 1000, ld = 768;
    const int rounds = argc > 3 ? atoi(argv[3]) : 6;
    const char* only = argc > 4 ? argv[4] : nullptr;
    const uint32_t qpad = (nq + 255) / 256 * 256, npad = (n + 255) / 256 * 256;
    uint8_t *A16, *B16, *A8, *B8; float *tau, *as, *bs; uint64_t* cand; uint32_t* cnt;
    const uint32_t cap = 1024;
    CHECK(hipMalloc(&A16, (size_t)npad * ld * 2)); CHECK(hipMalloc(&B16, (size_t)qpad * ld * 2));
    CHECK(hipMalloc(&A8, (size_t)npad * ld)); CHECK(hipMalloc(&B8, (size_t)qpad * ld));
    CHECK(hipMalloc(&as, npad / 32 * 4)); CHECK(hipMalloc(&bs, qpad * 4));
    CHECK(hipMalloc(&tau, qpad * 4));
    uint64_t* stamp;
    CHECK(hipMalloc(&stamp, 4096 * 16)); CHECK(hipMalloc(&cand, (size_t)qpad * cap * 8)); CHECK(hipMalloc(&cnt, qpad * 4));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, (uint16_t*)A16, (size_t)npad * ld, 1);
    hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, (uint16_t*)B16, (size_t)qpad * ld, 2);
    hipLaunchKernelGGL(fill_i8, dim3(4096), dim3(256), 0, 0, (int8_t*)A8, (size_t)npad * ld, 3);
    hipLaunchKernelGGL(fill_i8, dim3(1024), dim3(256), 0, 0, (int8_t*)B8, (size_t)qpad * ld, 4);
    hipLaunchKernelGGL(fill_f32, dim3(256), dim3(256), 0, 0, as, (size_t)npad / 32, 1.0f / (127.0f * 16.0f));
    hipLaunchKernelGGL(fill_f32, dim3(16), dim3(256), 0, 0, bs, (size_t)qpad, 1.0f / (127.0f * 16.0f));
    CHECK(hipDeviceSynchronize());
    GemmArgs g{};
    g.n_rows = n; g.a_scale_rows = 32; g.n_qt = qpad / 256; g.n_rt = (n + 255) / 256;
    g.S = reinterpret_cast<float*>(stamp);
    g.a_scale = as; g.b_scale = bs; g.tau = tau; g.cand = cand; g.cnt = cnt; g.cap = cap;
    const uint32_t per_xcd = (32 / g.n_qt) * g.n_qt, grid = 8 * per_xcd;
    const double flops = 2.0 * nq * (double)n * ld;
    struct V { const char* name; void (*k)(GemmArgs); bool i8; float tau; std::vector<float> t; std::vector<double> clk; int threads = 512; };
    // every variant stamps its in-kernel clock (STAMP): the same instantiation is not the
    // product build, whose kernels execute no stamp
    std::vector<V> vs = {
        {"i8 tau=0.125", k_filter<OpI8, true, 0, false, false, 2, true>, true, 0.125f, {}, {}},
        {"qs2 tau=inf", k_filter_qs8<true, 12, true>, true, 1e9f, {}, {}, 512},
        {"Qs2 tau=inf", k_filter_qs8<true, 12, false>, true, 1e9f, {}, {}, 512},
        {"Qs2 tau=0.125", k_filter_qs8<true, 12, false>, true, 0.125f, {}, {}, 512},
        {"Qs2 stag tau=inf", k_filter_qs8<true, 12, false, 0, true>, true, 1e9f, {}, {}, 512},
        {"Qs2 stag tau=0.125", k_filter_qs8<true, 12, false, 0, true>, true, 0.125f, {}, {}, 512},
        {"qs2 tau=0.125", k_filter_qs8<true, 12, true>, true, 0.125f, {}, {}, 512},
        {"Qs2 no-DMA", k_filter_qs8<true, 12, false, 1>, true, 1e9f, {}, {}, 512},
        {"Qs2 no-epi", k_filter_qs8<true, 12, false, 5>, true, 1e9f, {}, {}, 512},
        {"Qs2 no-DMA no-epi", k_filter_qs8<true, 12, false, 6>, true, 1e9f, {}, {}, 512},
        {"B2 tau=inf", k_filter_qs8<true, 12, false, 8>, true, 1e9f, {}, {}, 512},
        {"B2 tau=0.125", k_filter_qs8<true, 12, false, 8>, true, 0.125f, {}, {}, 512},
        {"b2 tau=0.125", k_filter_qs8<true, 12, true, 8>, true, 0.125f, {}, {}, 512},
        {"B2 no-epi", k_filter_qs8<true, 12, false, 13>, true, 1e9f, {}, {}, 512},
        {"B2 no-DMA no-epi", k_filter_qs8<true, 12, false, 14>, true, 1e9f, {}, {}, 512},
        {"S2 tau=inf", k_filter_qs8<true, 12, false, 72>, true, 1e9f, {}, {}, 512},
        {"S2 tau=0.125", k_filter_qs8<true, 12, false, 72>, true, 0.125f, {}, {}, 512},
        {"S2 no-epi", k_filter_qs8<true, 12, false, 77>, true, 1e9f, {}, {}, 512},
        {"P2 tau=inf", k_filter_qs8<true, 12, false, 328>, true, 1e9f, {}, {}, 512},
        {"P2 tau=0.125", k_filter_qs8<true, 12, false, 328>, true, 0.125f, {}, {}, 512},
        {"D2 tau=inf", k_filter_qs8<true, 12, false, 200>, true, 1e9f, {}, {}, 512},
        {"D2 tau=0.125", k_filter_qs8<true, 12, false, 200>, true, 0.125f, {}, {}, 512},
        {"B3 tau=inf", k_filter_qs8<true, 12, false, 16>, true, 1e9f, {}, {}, 512},
        {"B3 tau=0.125", k_filter_qs8<true, 12, false, 16>, true, 0.125f, {}, {}, 512},
        {"B3 no-epi", k_filter_qs8<true, 12, false, 21>, true, 1e9f, {}, {}, 512},
    };
    if (only) {
        std::vector<V> keep;
        for (auto& v : vs)
            if (strstr(v.name, only)) keep.push_back(v);
        vs.swap(keep);
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
        for (auto& v : vs) {
            g.A = v.i8 ? A8 : A16; g.B = v.i8 ? B8 : B16;
            g.row_bytes = v.i8 ? ld : 2 * ld; g.a_stride = g.row_bytes;
            std::vector<float> ht(qpad, v.tau);
            CHECK(hipMemcpy(tau, ht.data(), qpad * 4, hipMemcpyHostToDevice));
            CHECK(hipMemset(cnt, 0, qpad * 4));
            CHECK(hipMemset(stamp, 0, 4096 * 16));
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(v.k, dim3(grid), dim3(v.threads), 0, 0, g);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0) {
                v.t.push_back(ms);
                std::vector<uint64_t> hs(2 * grid);
                CHECK(hipMemcpy(hs.data(), stamp, hs.size() * 8, hipMemcpyDeviceToHost));
                std::vector<double> c;
                for (uint32_t i = 0; i < grid; ++i)
                    if (hs[2 * i + 1]) c.push_back((double)hs[2 * i] / hs[2 * i + 1] * 0.1);  // GHz (100 MHz ref)
                std::sort(c.begin(), c.end());
                if (!c.empty()) v.clk.push_back(c[c.size() / 2]);
                if (r == rounds - 1 && strncmp(v.name, "qs", 2) == 0) {  // qs: per-segment cycles of wave 0
                    std::vector<uint64_t> sg(4 * grid);
                    CHECK(hipMemcpy(sg.data(), stamp + 2 * grid, sg.size() * 8, hipMemcpyDeviceToHost));
                    double tb = 0, td = 0, te = 0, tj = 0, tt = 0;
                    for (uint32_t i = 0; i < grid; ++i) {
                        tb += sg[4 * i]; td += sg[4 * i + 1]; te += sg[4 * i + 2]; tj += sg[4 * i + 3]; tt += hs[2 * i];
                    }
                    printf("  [%s] per slice: total %.0f cyc, barrier %.0f, dma issue %.0f, epilogue %.0f (slices/WG %.0f)\n",
                           v.name, tt / tj, tb / tj, td / tj, te / tj, tj / grid);
                }
            }
            if (r == rounds - 1 && v.tau < 1e8f) {
                std::vector<uint32_t> hc(qpad);
                CHECK(hipMemcpy(hc.data(), cnt, qpad * 4, hipMemcpyDeviceToHost));
                double tot = 0; for (uint32_t i = 0; i < nq; ++i) tot += hc[i];
                printf("  [%s] emitted per query %.1f\n", v.name, tot / nq);
            }
        }
    }
    // skinny int8 filter (1 query, HBM-bound): GB/s of the int8 rows
    if (!only || strstr("skinny", only)) {
        GemmArgs gs = g;
        gs.A = A8; gs.B = B8; gs.row_bytes = ld; gs.a_stride = ld;
        std::vector<float> ht(qpad, 0.125f);
        CHECK(hipMemcpy(tau, ht.data(), qpad * 4, hipMemcpyHostToDevice));
        std::vector<float> ts, ts1;
        for (int r = 0; r < 2 * rounds + 2; ++r) {
            CHECK(hipMemset(cnt, 0, qpad * 4));
            CHECK(hipEventRecord(e0));
            if (r & 1) hipLaunchKernelGGL(k_filter_skinny<true>, dim3(768), dim3(256), 0, 0, gs);
            else hipLaunchKernelGGL((k_filter_skinny2<true, 12>), dim3(512), dim3(256), 0, 0, gs);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 1) (r & 1 ? ts1 : ts).push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        std::sort(ts1.begin(), ts1.end());
        printf("%-18s median %7.3f ms  min %7.3f ms  (%7.1f GB/s of int8 rows at median)\n", "skinny v1",
               ts1[ts1.size() / 2], ts1[0], (double)n * ld / (ts1[ts1.size() / 2] * 1e-3) / 1e9);
        printf("%-18s median %7.3f ms  min %7.3f ms  (%7.1f GB/s of int8 rows at median)\n", "skinny v2",
               ts[ts.size() / 2], ts[0], (double)n * ld / (ts[ts.size() / 2] * 1e-3) / 1e9);
    }
    for (auto& v : vs) {
        std::sort(v.t.begin(), v.t.end());
        float med = v.t[v.t.size() / 2], mn = v.t[0];
        std::sort(v.clk.begin(), v.clk.end());
        const double clk = v.clk.empty() ? 0.0 : v.clk[v.clk.size() / 2];
        printf("%-20s median %7.3f ms  min %7.3f ms  (%7.1f T(FL)OP/s at median)  clock %.2f GHz  (%4.0f%% of peak at that clock)\n",
               v.name, med, mn, flops / (med * 1e-3) / 1e12, clk,
               clk > 0 ? 100.0 * flops / (med * 1e-3) / (256.0 * 4 * (v.i8 ? 2048 : 1024) * clk * 1e9) : 0.0);
    }
    return 0;
}
