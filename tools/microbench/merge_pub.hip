// Microbenchmark (tooling, round 4): the global-threshold path's merge kernel k_merge_lists at the
// 8-GPU exchange shape (P = 8 gathered result buffers x 1000 queries x k = 10, certification on),
// without publishing, publishing as a non-root rank (status words + fail list) and as the root
// (its merged rows written through to the pinned host mirror).  Kernel time from HIP events on
// the stream around the launch; publish latency = launch -> the host sees the flag.
// Build: make -C tools/microbench merge_pub      Run: ./merge_pub [rounds]
#include "k_exact.hip"

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CHECK(x)                                                       \
    do {                                                               \
        hipError_t e_ = (x);                                           \
        if (e_ != hipSuccess) {                                        \
            printf("%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                   \
        }                                                              \
    } while (0)

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 200;
    const uint32_t P = 8, Q = 1000, K = 10;
    const size_t nk = (size_t)Q * K;
    // gathered lists [P][Q][K], counts [P][Q], bounds [P][Q], status words [P][kStWords]
    std::vector<uint64_t> hi(P * nk);
    std::vector<float> hd(P * nk), hx(P * Q, 1.0f);
    std::vector<uint32_t> hc(P * Q, K), hs(P * bsr::kStWords, 0);
    uint64_t s = 7;
    for (uint32_t r = 0; r < P; ++r)
        for (uint32_t q = 0; q < Q; ++q) {
            float d = 0.0f;
            for (uint32_t i = 0; i < K; ++i) {
                s = s * 6364136223846793005ull + 1442695040888963407ull;
                d += (float)((s >> 40) & 0xFFFF) * 1e-7f;
                hd[(r * Q + q) * K + i] = d;
                hi[(r * Q + q) * K + i] = (uint64_t)r * 1250000 + ((s >> 20) % 1250000);
            }
        }
    uint64_t* di;
    float *dd, *dx;
    uint32_t *dc, *dst;
    CHECK(hipMalloc(&di, hi.size() * 8));
    CHECK(hipMalloc(&dd, hd.size() * 4));
    CHECK(hipMalloc(&dx, hx.size() * 4));
    CHECK(hipMalloc(&dc, hc.size() * 4));
    CHECK(hipMalloc(&dst, hs.size() * 4));
    CHECK(hipMemcpy(di, hi.data(), hi.size() * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dd, hd.data(), hd.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dx, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dst, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    // merged buffer (capi.cpp mres_layout): [fail count, first nan | st | fail list | cnt | dist | idx]
    const size_t o_st = 16, o_fail = (o_st + P * bsr::kStWords * 4 + 15) / 16 * 16,
                 o_cnt = (o_fail + Q * 4 + 15) / 16 * 16, o_dist = (o_cnt + Q * 4 + 15) / 16 * 16,
                 o_idx = (o_dist + nk * 4 + 15) / 16 * 16, bytes = (o_idx + nk * 8 + 15) / 16 * 16;
    uint8_t *md, *hm, *hm_dev;
    uint32_t *flag, *flag_dev, *ticket;
    CHECK(hipMalloc(&md, bytes));
    CHECK(hipMalloc(&ticket, bsr::kTicketWords * 4));
    CHECK(hipMemset(ticket, 0, bsr::kTicketWords * 4));
    CHECK(hipHostMalloc((void**)&hm, bytes, hipHostMallocCoherent));
    CHECK(hipHostGetDevicePointer((void**)&hm_dev, hm, 0));
    CHECK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent));
    CHECK(hipHostGetDevicePointer((void**)&flag_dev, flag, 0));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));

    auto args = [&](int mode) {  // 0 no publish, 1 non-root publish, 2 root publish
        bsr::MergeArgs a{};
        a.idx = di;
        a.dist = dd;
        a.cnt = dc;
        a.idx_stride = nk;
        a.dist_stride = nk;
        a.cnt_stride = Q;
        a.P = P;
        a.nq = Q;
        a.k_in = K;
        a.k = K;
        a.out_idx = reinterpret_cast<uint64_t*>(md + o_idx);
        a.out_dist = reinterpret_cast<float*>(md + o_dist);
        a.out_count = reinterpret_cast<uint32_t*>(md + o_cnt);
        a.first_nan = reinterpret_cast<uint32_t*>(md) + 1;
        a.excl = dx;
        a.excl_stride = Q;
        a.need = K;
        a.fail_cnt = reinterpret_cast<uint32_t*>(md);
        a.fail_list = reinterpret_cast<uint32_t*>(md + o_fail);
        a.st = dst;
        a.st_stride = bsr::kStWords;
        a.st_all = reinterpret_cast<uint32_t*>(md + o_st);
        if (mode) {
            a.pub_src = md;
            a.pub_dst = hm_dev;
            a.pub_bytes = o_cnt;
            a.pub_flag = flag_dev;
            a.pub_ticket = ticket;
            if (mode == 2) {
                a.hout_idx = reinterpret_cast<uint64_t*>(hm_dev + o_idx);
                a.hout_dist = reinterpret_cast<float*>(hm_dev + o_dist);
                a.hout_count = reinterpret_cast<uint32_t*>(hm_dev + o_cnt);
            }
        }
        return a;
    };
    struct R { std::vector<float> k, pub; };
    R res[3];
    auto run = [&](int mode) {
        CHECK(hipMemsetAsync(md, 0, 4, st));
        CHECK(hipMemsetAsync(md + 4, 0xff, 4, st));
        CHECK(hipStreamSynchronize(st));
        __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
        const bsr::MergeArgs a = args(mode);
        const auto t0 = std::chrono::steady_clock::now();
        CHECK(hipEventRecord(e0, st));
        CHECK(bsr::launch_merge(a, st));
        CHECK(hipEventRecord(e1, st));
        if (mode) {
            while (!__atomic_load_n(flag, __ATOMIC_ACQUIRE)) {}
            res[mode].pub.push_back(std::chrono::duration<float, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        res[mode].k.push_back(ms * 1e3f);
    };
    for (int i = 0; i < 30; ++i) run(i % 3);
    for (auto& r : res) { r.k.clear(); r.pub.clear(); }
    for (int i = 0; i < rounds; ++i)
        for (int m = 0; m < 3; ++m) run(m);
    // the root's host rows equal the device rows
    std::vector<uint8_t> dev(bytes);
    CHECK(hipMemcpy(dev.data(), md, bytes, hipMemcpyDeviceToHost));
    const bool same = memcmp(dev.data(), hm, bytes) == 0;
    const uint32_t fails = *reinterpret_cast<uint32_t*>(hm);
    const char* names[3] = {"no publish", "publish (non-root)", "publish (root, rows written through)"};
    for (int m = 0; m < 3; ++m) {
        auto med = [](std::vector<float> v) { if (v.empty()) return 0.0f; std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
        printf("%-40s kernel %7.2f us (median of %d)", names[m], med(res[m].k), rounds);
        if (m) printf("   launch -> flag seen %7.2f us", med(res[m].pub));
        printf("\n");
    }
    printf("root host buffer == device buffer: %s; uncertified queries %u\n", same ? "yes" : "NO", fails);
    return same ? 0 : 2;
}
