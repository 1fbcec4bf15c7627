// k_qs16x_lab.hip -- TOOLING: ablation copies of the product emit filter
// bsr::k_filter_qs16<true, 12> (k_filter.hip), to attribute its non-MFMA time.
// Included after k_filter.hip (uses its types and helpers).
//
// FLAGS:
//   kStaticDma   the DMA schedule resolved at compile time: the slice a DMA fills is
//                (kt + A) % NK of this tile or the next, its descriptor one of two computed
//                once per tile -- no per-DMA counters and branches (product: a running
//                counter and a branch per DMA)
//   kNoEpi       no epilogue at all (results discarded: the MFMA stream's floor)
//   kNoBar       no s_barrier (vmcnt waits only: reads may race the DMA; timing only)
//   kNoDma       no LDS-DMA (the ring holds whatever it held: timing only)
//   kNoLdsRead   no fragment reads (the MFMAs reuse the fragments in registers: timing only)
//   kSameTile    every row tile's DMA reads the workgroup's FIRST tile (always L2-resident: the
//                upside of perfect L2 sharing among the workgroups of a row-tile stream)
//   kSliceMajor  (with kStaticDma) the operand stored slice-major inside each 128-row tile:
//                tile rt = NK slices of 128 rows x 64 B, each slice one contiguous 8 KiB
//                (product: row-major, a slice = 128 half-lines 768 B apart)
namespace bsrlab {
using namespace bsr;

enum : int { kStaticDma = 1, kNoEpi = 2, kNoBar = 4, kNoDma = 8, kNoLdsRead = 16, kSameTile = 32, kSliceMajor = 64 };
// PACE > 0: the n_qt workgroups that stream the same row tiles (same g0) keep within PACE
// tiles of each other: after each tile wave 0 publishes its count (relaxed agent-scope store,
// progress words in p.S, zeroed before the launch); before each tile it reads the group's
// words through the scalar path (glc) and sleeps while it leads the slowest by more than
// PACE.  Bounded spin: stale words only slow it down.  Lab only (n_qt <= 4).

template <int N>
__device__ __forceinline__ void wait_vm_only() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void qs_wait_n_nobar(int n) {
    if (n == 3) wait_vm_only<3>();
    else wait_vm_only<2>();
}

// BP: slices per barrier (product 2).  Ring slots S = AHEAD + BP; at the barrier of slice jj
// (jj % BP == BP - 1, mid-slice) slices <= jj + BP + 1 must have landed, so AHEAD - BP - 2
// younger slices stay in flight.
template <int FLAGS, int PACE = 0, int AHEAD = 6, int BP = 2>
__global__ __launch_bounds__(512, 1) void k_qs16x(GemmArgs p) {
    constexpr int NK = 12;
    constexpr bool EMIT = true;
    constexpr int A = AHEAD, S = AHEAD + BP;  // slices in flight, ring slots
    static_assert(A >= BP + 2 && A < NK && NK % BP == 0, "lookahead");
    constexpr int BM = 128, BN = kFilterTile, NT = 512, SLOT = BM * kSliceB;
    constexpr int CAP = 10;
    constexpr int EM_BYTES = NT * 2 * CAP * 8;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[S * SLOT + EM_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint64_t* const lkeys = reinterpret_cast<uint64_t*>(lds + S * SLOT) + tid;
    uint32_t ecnt[2] = {0, 0};

    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * NK;

    uint32_t qq[2];
    i32x4v_t fb[2][NK];
    float tau[2], sbq[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
        qq[nb] = qt * BN + w * 32 + nb * 16 + (lane & 15);
        const uint8_t* src = p.B + (uint64_t)qq[nb] * p.row_bytes + 16 * (lane >> 4);
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) fb[nb][kt] = *reinterpret_cast<const i32x4v_t*>(src + 64 * kt);
        tau[nb] = p.tau[qq[nb]];
        sbq[nb] = p.b_scale[qq[nb]];
    }
    auto flush_ring = [&](int nb) {
        const uint32_t nn = ecnt[nb];
        if (nn) {
            const uint32_t gp = atomicAdd(p.cnt + qq[nb], nn);
            for (uint32_t i = 0; i < nn; ++i)
                if (gp + i < p.cap) p.cand[(uint64_t)qq[nb] * p.cap + gp + i] = lkeys[(nb * CAP + i) * NT];
        }
        ecnt[nb] = 0;
    };

    const uint32_t lrow = w * 16 + (lane >> 2);
    const uint32_t lchunk = ((lane & 3) ^ qs16_swz(lrow)) * 16;
    constexpr bool SM = (FLAGS & kSliceMajor) != 0;
    constexpr uint32_t kSliceSrc = SM ? BM * kSliceB : kSliceB;  // source bytes between slices
    const uint32_t aoff_dma = lrow * (SM ? (uint32_t)kSliceB : (uint32_t)p.a_stride) + lchunk;
    auto rsrc_for = [&](uint32_t ti) {
        const uint32_t rt = g0 + ((FLAGS & kSameTile) ? 0 : ti) * RG;
        return __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (uint64_t)rt * BM * p.a_stride), 0,
                                                 BM * (uint32_t)p.a_stride, 0x00020000);
    };
    // dynamic schedule (product)
    uint32_t iss_ti = 0, iss_kt = 0;
    __amdgpu_buffer_rsrc_t rsrc_a;
    auto issue_dma = [&](uint32_t jj) {
        if (FLAGS & kNoDma) return;
        uint8_t* la = lds + (jj % S) * SLOT + wu * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)la, 16, aoff_dma, iss_kt * kSliceB, 0, 0);
        if (++iss_kt == NK) {
            iss_kt = 0;
            ++iss_ti;
            if (iss_ti < my_rt) rsrc_a = rsrc_for(iss_ti);
        }
    };
    // static schedule: descriptors of this tile and the next (the last tile re-read at the end)
    __amdgpu_buffer_rsrc_t rs_cur, rs_nxt;
    auto issue_dma_static = [&](uint32_t jj, int kt) {
        if (FLAGS & kNoDma) return;
        uint8_t* la = lds + (jj % S) * SLOT + wu * 1024;
        if (kt + A < NK)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_cur, (lds_void_t*)la, 16, aoff_dma, (kt + A) * kSliceSrc, 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_nxt, (lds_void_t*)la, 16, aoff_dma, (kt + A - NK) * kSliceSrc, 0, 0);
    };
    const uint32_t aoff0 = (lane & 15) * kSliceB + (((lane >> 4) ^ qs16_swz(lane & 15)) * 16);
    i32x4v_t fa[4];
    auto read_frag = [&](uint32_t jj, int rb) {
        if ((FLAGS & kNoLdsRead) && jj >= 1) return;
        fa[rb & 3] = *reinterpret_cast<const i32x4v_t*>(lds + (jj % S) * SLOT + rb * 1024 + aoff0);
    };

    i32x4v_t acc[8][2];
    if (my_rt) {
        rsrc_a = rsrc_for(0);
        rs_cur = rsrc_a;
        rs_nxt = rsrc_for(my_rt > 1 ? 1 : 0);
    }
    const uint32_t pre = J ? (uint32_t)A : 0u;
    if (FLAGS & kStaticDma) {
        if (!(FLAGS & kNoDma))
            for (uint32_t jj = 0; jj < pre; ++jj) {
                uint8_t* la = lds + (jj % S) * SLOT + wu * 1024;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_cur, (lds_void_t*)la, 16, aoff_dma, jj * kSliceSrc, 0, 0);
            }
    } else {
        for (uint32_t jj = 0; jj < pre; ++jj) issue_dma(jj);
    }
    qs_barrier((FLAGS & kNoDma) ? 0 : (pre >= (uint32_t)BP + 1 ? pre - (BP + 1) : 0));  // slices 0..BP landed
    if (J)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) fa[rb] = *reinterpret_cast<const i32x4v_t*>(lds + rb * 1024 + aoff0);

    uint32_t* const prog = reinterpret_cast<uint32_t*>(p.S) + g0 * 4;
    for (uint32_t t = 0; t < my_rt; ++t) {
        const uint32_t rt = g0 + t * RG;
        if (PACE > 0 && w == 0 && t > (uint32_t)PACE && active) {
            typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
            for (int spin = 0; spin < 20000; ++spin) {
                u32x4_t v;
                asm volatile("s_load_dwordx4 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(prog) : "memory");
                uint32_t mn = v[0];
                for (uint32_t i = 1; i < p.n_qt; ++i) mn = min(mn, (uint32_t)v[i]);
                if (t <= mn + (uint32_t)PACE) break;
                __builtin_amdgcn_s_sleep(2);
            }
        }
        if (FLAGS & kStaticDma) {
            if (t) {
                rs_cur = rs_nxt;
                rs_nxt = rsrc_for(t + 1 < my_rt ? t + 1 : t);
            }
        }
        float4 scv = *reinterpret_cast<const float4*>(p.a_scale + (uint64_t)rt * (BM / kQuantBlock));
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) {
            const uint32_t jj = t * NK + kt;
            const bool bar_slice = (kt % BP) == BP - 1;
#pragma unroll
            for (int rb = 0; rb < 8; ++rb) {
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    if (kt == 0) {
                        const i32x4v_t z = {};
                        acc[rb][nb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[rb & 3], fb[nb][kt], z, 0, 0, 0);
                    } else {
                        acc[rb][nb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[rb & 3], fb[nb][kt], acc[rb][nb], 0, 0, 0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                if (rb < 4) read_frag(jj, rb + 4);
                else read_frag(jj + 1, rb - 4);
                if (bar_slice ? rb == 6 : rb == 1) {
                    if (FLAGS & kStaticDma) issue_dma_static(jj + A, kt);
                    else issue_dma(jj + A);
                }
                if (bar_slice && rb == 5 && ((FLAGS & kStaticDma) || jj + 1 < J)) {
                    if (FLAGS & kNoBar) {
                        if (!(FLAGS & kNoDma)) qs_wait_n_nobar(2 + (kt <= 2 ? 1 : 0));
                    } else {
                        // slices <= jj + 3 landed: the A - 4 younger slices' DMAs (and the tile's
                        // scale load while it is younger than slice jj + 3's, kt <= A - 4) in flight
                        qs_wait_n((FLAGS & kNoDma) ? (kt <= A - BP - 2 ? 1 : 0)
                                                   : (A - BP - 2) + (kt <= A - BP - 2 ? 1 : 0));
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (FLAGS & kNoEpi) {
            // keep the accumulators live: fold one value into a never-taken store
            int m = 0;
#pragma unroll
            for (int rb = 0; rb < 8; ++rb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) m ^= acc[rb][nb][0] ^ acc[rb][nb][3];
            if (m == 0x7e3a91c5 && tau[0] == 12345.0f) p.cnt[0] = (uint32_t)m;
            continue;
        }
        const float sc[4] = {scv.x, scv.y, scv.z, scv.w};
        bool stored = false;
        const float sc_hi = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
        const float sc_lo = fminf(fminf(sc[0], sc[1]), fminf(sc[2], sc[3]));
        bool any = false;
        int mrb[2];
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            int m = acc[0][nb][0];
#pragma unroll
            for (int rb = 0; rb < 8; ++rb)
#pragma unroll
                for (int r = 0; r < 4; ++r) m = (rb | r) ? max(m, acc[rb][nb][r]) : m;
            mrb[nb] = m;
            any |= ((float)m * (m >= 0 ? sc_hi : sc_lo)) * sbq[nb] >= tau[nb];
        }
        if (__ballot(any)) {
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                if (!__ballot(((float)mrb[nb] * (mrb[nb] >= 0 ? sc_hi : sc_lo)) * sbq[nb] >= tau[nb])) continue;
                bool pass_rb[8];
#pragma unroll
                for (int rb = 0; rb < 8; ++rb) {
                    const i32x4v_t& x = acc[rb][nb];
                    const int bm = max(max(x[0], x[1]), max(x[2], x[3]));
                    pass_rb[rb] = ((float)bm * sc[rb >> 1]) * sbq[nb] >= tau[nb];
                }
#pragma unroll
                for (int rb = 0; rb < 8; ++rb) {
                    if (!__ballot(pass_rb[rb])) continue;
                    if (__ballot(ecnt[nb] > (uint32_t)(CAP - 4))) {
                        flush_ring(nb);
                        stored = true;
                    }
                    const i32x4v_t& x = acc[rb][nb];
                    const float scr = sc[rb >> 1];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float v = ((float)x[r] * scr) * sbq[nb];
                        const uint32_t row = rt * BM + rb * 16 + 4 * (lane >> 4) + r;
                        lkeys[(nb * CAP + ecnt[nb]) * NT] = score_key(v, row);
                        ecnt[nb] += (v >= tau[nb] && row < p.n_rows) ? 1u : 0u;
                    }
                }
            }
        }
        if (stored) wait_vm0();
        if (PACE > 0 && tid == 0) __hip_atomic_store(prog + qt, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    wait_vm0();
    if (!(FLAGS & kNoEpi)) {
        flush_ring(0);
        flush_ring(1);
    }
}

}  // namespace bsrlab
