// Lab (tooling): the tau selection kernels timed alone at the 8-GPU rank shape (1000 queries,
// 1221 compact sample maxima per query = the 1.25M-row shard, ks = 8) and at the 10M shape
// (9766 maxima), HIP events around 200 launches each.
#include "k_filter.hip"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

using namespace bsr;

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; }   \
    } while (0)

int main() {
    const uint32_t ks = 8;
    for (uint32_t n_s : {1221u, 9766u}) {
        for (uint32_t nq : {1000u, 1u}) {
            const uint32_t qpad = nq == 1 ? 16u : 1024u, s_ld = (n_s + 127) / 128 * 128;
            std::vector<float> h((size_t)qpad * s_ld);
            srand(n_s + nq);
            for (auto& x : h) x = (float)rand() / RAND_MAX * 2.0f - 1.0f;
            float *S, *tau;
            uint32_t *cnt, *status, *qflags;
            uint64_t* smax;
            CK(hipMalloc(&S, h.size() * 4));
            CK(hipMemcpy(S, h.data(), h.size() * 4, hipMemcpyHostToDevice));
            CK(hipMalloc(&tau, qpad * 4));
            CK(hipMalloc(&cnt, (qpad + 8 * kTailCounters + kGangWords) * 4));
            CK(hipMalloc(&status, 64 * 4));
            CK(hipMalloc(&qflags, qpad * 4));
            CK(hipMemset(qflags, 0, qpad * 4));
            CK(hipMalloc(&smax, (size_t)qpad * ks * 8));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            auto timeit = [&](const char* name, auto launch) -> int {
                for (int i = 0; i < 20; ++i) launch();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < 200; ++i) launch();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                printf("n_s %5u nq %4u %-22s %8.2f us per launch\n", n_s, nq, name, ms * 1e3 / 200);
                return 0;
            };
            timeit("k_select_tau<1>", [&] {
                hipLaunchKernelGGL(k_select_tau<1>, dim3(qpad), dim3(256), 0, 0, S, s_ld, n_s, nq, qpad, qflags, ks,
                                   tau, cnt, status, smax);
            });
            if (n_s <= 32 * 64)
                timeit("k_select_tau_w<32>", [&] {
                    hipLaunchKernelGGL(k_select_tau_w<32>, dim3(qpad / 4), dim3(256), 0, 0, S, s_ld, n_s, nq, qpad,
                                       qflags, ks, tau, cnt, status, smax);
                });
            if (qpad <= 16)
                timeit("k_select_tau_m<16>", [&] {
                    hipLaunchKernelGGL(k_select_tau_m<16>, dim3(qpad), dim3(1024), 0, 0, S, s_ld, n_s, nq, qpad,
                                       qflags, ks, tau, cnt, status, smax);
                });
            hipFree(S); hipFree(tau); hipFree(cnt); hipFree(status); hipFree(qflags); hipFree(smax);
        }
    }
    return 0;
}
