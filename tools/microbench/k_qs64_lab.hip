// k_qs64_lab.hip -- TOOLING: the one-wave-per-SIMD emit filter (64 queries per wave, B
// fragments pinned in AGPRs), measured against the product k_filter_qs16 in round 3
// (profiles/r03d_*): half the LDS fragment reads, but slower -- the single wave per SIMD
// exposes the epilogue, the emission work and every issue bubble.  Build the harness with
// -mllvm -amdgpu-mfma-vgpr-form (accumulators in arch VGPRs).  Included after k_filter.hip.
namespace bsrlab {
using namespace bsr;

// ------------------------------------------------------------------------------------
// Query-stationary int8 emit filter, one wave per SIMD: k_filter_qs64.
//
// k_filter_qs16 runs two waves per SIMD with 32 queries each, so every A fragment read from
// LDS feeds two MFMAs and each 16-row block of a slice is read by all 8 waves of the CU
// (64 KiB of ds_read_b128 per 8 KiB slice).  Here one 256-thread workgroup per CU holds the
// same 256-query tile in FOUR waves of 64 queries: the wave's B fragments for all of K take
// 4 x 12 x 4 = 192 registers and its accumulators 8 x 4 x 4 = 128 (the 512-entry register
// file of a one-wave-per-SIMD kernel), every A fragment feeds FOUR MFMAs and the CU reads
// each slice from LDS four times instead of eight: half the LDS read bytes and half the
// fragment-read instructions per MFMA, and four waves at each barrier instead of eight.
// Ring, swizzle, LDS-DMA stream, barriers and the two-level emission are k_filter_qs16's;
// each wave fills 32 rows of every slice (two 1 KiB LDS-DMA instructions).
// ------------------------------------------------------------------------------------
template <int NK>
__global__ __launch_bounds__(256, 1) void k_filter_qs64(GemmArgs p) {
    constexpr int S = 8, A = 6;          // ring slots, slices issued ahead
    constexpr int BM = 128, BN = kFilterTile, NT = 256, SLOT = BM * kSliceB;
    constexpr int NB = 4;                // 16-query blocks per wave
    constexpr int CAP = 10;              // candidate ring entries per (lane, query block)
    static_assert(NK % 2 == 0 && NK >= 2 && NK <= 12, "even slice counts up to 768 bytes");
    static_assert(BN == 4 * NB * 16, "four waves of NB query blocks cover the query tile");
    constexpr int EM_BYTES = NT * NB * CAP * 8;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[S * SLOT + EM_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint64_t* const lkeys = reinterpret_cast<uint64_t*>(lds + S * SLOT) + tid;
    uint32_t ecnt[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) ecnt[nb] = 0;

    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * NK;

    // B fragments of the wave's four 16-query blocks, all K: fb[nb][kt] = query
    // qt*256 + 64w + 16nb + (lane & 15), bytes 64kt + 16(lane >> 4) .. +15.
    uint32_t qq[NB];
    i32x4v_t fb[NB][NK];
    float tau[NB], sbq[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
        qq[nb] = qt * BN + w * 64 + nb * 16 + (lane & 15);
        const uint8_t* src = p.B + (uint64_t)qq[nb] * p.row_bytes + 16 * (lane >> 4);
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) fb[nb][kt] = *reinterpret_cast<const i32x4v_t*>(src + 64 * kt);
        tau[nb] = p.tau[qq[nb]];
        sbq[nb] = p.b_scale[qq[nb]];
    }
    // The B fragments live in the AGPR half of the register file (MFMA A/B operands may be
    // AGPRs; the library builds this kernel with -amdgpu-mfma-vgpr-form, so accumulators and
    // A fragments take the arch VGPRs): 192 + ~250 registers, no copies, no spills.
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) asm volatile("" : "+a"(fb[nb][kt]));
    auto flush_ring = [&](int nb) {
        const uint32_t nn = ecnt[nb];
        if (nn) {
            const uint32_t gp = atomicAdd(p.cnt + qq[nb], nn);
            for (uint32_t i = 0; i < nn; ++i)
                if (gp + i < p.cap) p.cand[(uint64_t)qq[nb] * p.cap + gp + i] = lkeys[(nb * CAP + i) * NT];
        }
        ecnt[nb] = 0;
    };

    // LDS-DMA: wave w fills rows 32w .. 32w+31 of each slice, two 1 KiB instructions (rows
    // 32w + 16i + lane/4); the source chunk XOR-swizzled as in k_filter_qs16.
    uint32_t aoff_dma[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint32_t lrow = w * 32 + i * 16 + (lane >> 2);
        aoff_dma[i] = lrow * (uint32_t)p.a_stride + ((lane & 3) ^ qs16_swz(lrow)) * 16;
    }
    uint32_t iss_ti = 0, iss_kt = 0;
    __amdgpu_buffer_rsrc_t rsrc_a;
    auto set_issue_tile = [&]() {
        const uint32_t rt = g0 + iss_ti * RG;
        rsrc_a = __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (uint64_t)rt * BM * p.a_stride), 0,
                                                   BM * (uint32_t)p.a_stride, 0x00020000);
    };
    auto issue_dma = [&](uint32_t jj, int i) {
        uint8_t* la = lds + (jj % S) * SLOT + (wu * 2 + i) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)la, 16, aoff_dma[i], iss_kt * kSliceB, 0, 0);
        if (i == 1 && ++iss_kt == NK) {
            iss_kt = 0;
            ++iss_ti;
            if (iss_ti < my_rt) set_issue_tile();
        }
    };
    const uint32_t aoff0 = (lane & 15) * kSliceB + (((lane >> 4) ^ qs16_swz(lane & 15)) * 16);
    i32x4v_t fa[4];
    auto read_frag = [&](uint32_t jj, int rb) {
        fa[rb & 3] = *reinterpret_cast<const i32x4v_t*>(lds + (jj % S) * SLOT + rb * 1024 + aoff0);
    };

    i32x4v_t acc[8][NB];
    if (my_rt) set_issue_tile();
    const uint32_t pre = J ? (uint32_t)A : 0u;
    for (uint32_t jj = 0; jj < pre; ++jj) {
        issue_dma(jj, 0);
        issue_dma(jj, 1);
    }
    qs_barrier(pre >= 3 ? 2 * (pre - 3) : 0);  // slices 0, 1, 2 landed everywhere
    if (J)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) read_frag(0, rb);

    for (uint32_t t = 0; t < my_rt; ++t) {
        const uint32_t rt = g0 + t * RG;
        const float4 scv = *reinterpret_cast<const float4*>(p.a_scale + (uint64_t)rt * (BM / kQuantBlock));
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) {
            const uint32_t jj = t * NK + kt;
            const bool bar_slice = (kt & 1) == 1;
#pragma unroll
            for (int rb = 0; rb < 8; ++rb) {
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) {
                    if (kt == 0) {
                        const i32x4v_t z = {};
                        acc[rb][nb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[rb & 3], fb[nb][kt], z, 0, 0, 0);
                    } else {
                        acc[rb][nb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[rb & 3], fb[nb][kt], acc[rb][nb], 0, 0, 0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                if (rb < 4) read_frag(jj, rb + 4);
                else read_frag(jj + 1, rb - 4);  // (past the stream's end: unused)
                // DMAs of slice jj + A: groups 1, 3 on even slices; after the barrier (groups 6,
                // 7) on odd slices (the slot they refill, slice jj - 2's, is then free everywhere)
                if (bar_slice ? rb == 6 : rb == 1) issue_dma(jj + A, 0);
                if (bar_slice ? rb == 7 : rb == 3) issue_dma(jj + A, 1);
                // barrier (odd slices, after group 5): slices <= jj + 3 landed everywhere; in
                // flight: the DMAs of slices jj + 4, jj + 5 (2 each) and, while younger than
                // slice jj + 3's (kt <= 2), the tile's scale load
                if (bar_slice && rb == 5 && jj + 1 < J) qs_wait_n(4 + (kt <= 2 ? 1 : 0));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // ---- epilogue: block (rb, nb) holds rows 16rb + 4(lane >> 4) + r, query qq[nb]
        const float sc[4] = {scv.x, scv.y, scv.z, scv.w};
        bool stored = false;
        // level 1, one ballot per tile: the lane's integer maximum over its 32 values of each
        // query block, scored with the tile's largest (or, for a negative maximum, smallest)
        // block scale -- never below any of its values' scores
        const float sc_hi = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
        const float sc_lo = fminf(fminf(sc[0], sc[1]), fminf(sc[2], sc[3]));
        bool any = false;
        int mrb[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            int m = acc[0][nb][0];
#pragma unroll
            for (int rb = 0; rb < 8; ++rb)
#pragma unroll
                for (int r = 0; r < 4; ++r) m = (rb | r) ? max(m, acc[rb][nb][r]) : m;
            mrb[nb] = m;
            any |= ((float)m * (m >= 0 ? sc_hi : sc_lo)) * sbq[nb] >= tau[nb];
        }
        if (__ballot(any)) {
            // level 2: per (query block, 16-row block) its maximum against tau, then the
            // passing blocks' 4 rows appended without branches
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
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
                    if (__ballot(ecnt[nb] > (uint32_t)(CAP - 4))) {  // room for 4 rows (rarely not)
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
        if (stored) wait_vm0();  // global stores / atomics count in vmcnt: keep the waits exact
    }
    wait_vm0();  // the stream's trailing DMAs land before the workgroup ends
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) flush_ring(nb);
}


}  // namespace bsrlab
