// Lab (tooling): k_select_tau_m<16> against k_select_tau<1> on the same random sample rows --
// tau and the ks best keys must be equal, bit for bit.
#include "k_filter.hip"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

using namespace bsr;

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } \
    } while (0)

int main() {
    const uint32_t qpad = 16, ks = 8;
    int bad = 0;
    for (uint32_t n_s : {1100u, 2048u, 4000u, 9766u, 16384u}) {
        for (uint32_t nq : {1u, 3u, 16u}) {
            const uint32_t s_ld = (n_s + 127) / 128 * 128;
            std::vector<float> h((size_t)qpad * s_ld);
            srand(n_s * 7 + nq);
            for (auto& x : h) x = (float)rand() / RAND_MAX * 2.0f - 1.0f;
            float *S, *tau;
            uint32_t *cnt, *status, *qflags;
            uint64_t* smax;
            CK(hipMalloc(&S, h.size() * 4));
            CK(hipMemcpy(S, h.data(), h.size() * 4, hipMemcpyHostToDevice));
            CK(hipMalloc(&tau, 2 * qpad * 4));
            CK(hipMalloc(&cnt, (qpad + 8 * kTailCounters + kGangWords) * 4));
            CK(hipMalloc(&status, 64 * 4));
            CK(hipMalloc(&qflags, qpad * 4));
            CK(hipMemset(qflags, 0, qpad * 4));
            CK(hipMalloc(&smax, 2 * qpad * ks * 8));
            CK(hipMemset(tau, 0x55, 2 * qpad * 4));
            hipLaunchKernelGGL(k_select_tau<1>, dim3(qpad), dim3(256), 0, 0, S, s_ld, n_s, nq, qpad, qflags, ks, tau,
                               cnt, status, smax);
            hipLaunchKernelGGL(k_select_tau_m<16>, dim3(qpad), dim3(1024), 0, 0, S, s_ld, n_s, nq, qpad, qflags, ks,
                               tau + qpad, cnt, status, smax + qpad * ks);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            std::vector<float> t(2 * qpad);
            std::vector<uint64_t> m(2 * qpad * ks);
            CK(hipMemcpy(t.data(), tau, t.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(m.data(), smax, m.size() * 8, hipMemcpyDeviceToHost));
            for (uint32_t q = 0; q < nq; ++q) {
                bool ok = t[q] == t[qpad + q];
                for (uint32_t i = 0; i < ks; ++i) ok = ok && m[q * ks + i] == m[(qpad + q) * ks + i];
                if (!ok) {
                    ++bad;
                    if (bad < 20)
                        printf("n_s %u nq %u q %u: tau %a vs %a, key0 %016llx vs %016llx\n", n_s, nq, q, t[q],
                               t[qpad + q], (unsigned long long)m[q * ks], (unsigned long long)m[(qpad + q) * ks]);
                }
            }
            hipFree(S); hipFree(tau); hipFree(cnt); hipFree(status); hipFree(qflags); hipFree(smax);
        }
    }
    printf("seltau_ab: %d mismatching queries\n", bad);
    return bad ? 2 : 0;
}
