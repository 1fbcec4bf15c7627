// k_rs_lab.hip -- TOOLING (round 4 lab): a ROW-STREAMING emit filter, the structural alternative
// to the product's query-stationary k_filter_qs16.  Included by filter_ab.hip after
// k_filter.hip.
//
// The product keeps each wave's 32 queries in registers and streams 128-row tiles through an LDS
// ring that all 8 waves read, so the waves meet at a barrier every two K slices and one wave's
// emission work (level 2) holds the other seven there.  Here the roles swap:
//  * a workgroup owns a 128-query tile whose int8 B fragments live in LDS for the kernel's life
//    (96 KiB, [K slice][query block][lane] -- every ds_read_b128 one contiguous KiB);
//  * each wave streams its OWN 32-row tiles straight into VGPRs (buffer loads, R - 1 K slices
//    ahead) from a fragment-native corpus layout (per 16-row block and 64-byte K slice, the
//    1 KiB an A operand of v_mfma_i32_16x16x64_i8 takes, in lane order: a fully coalesced load);
//  * per K slice a wave issues 16 MFMAs (2 row blocks x 8 query blocks) on 8 LDS B reads and 2
//    VMEM loads -- the product's 0.5 LDS reads per MFMA;
//  * nothing in the loop is shared between waves: no barrier, no ring hand-off.  A wave in its
//    emission epilogue delays itself only; its SIMD partner keeps the matrix pipe busy.
// Emission: per 32-row tile one scale (the corpus's 32-row quantisation block), so level 1 (the
// lane's maximum per query block) is exact; passing values are compacted into a wave-private LDS
// list (ballot + mbcnt, no atomics) and flushed to the per-query global lists when it fills.
// Row streams: the workgroups of the n_qt query tiles that read a stream sit on one XCD
// (blockIdx % 8) and read the same tiles in the same order, sharing them through its L2.
namespace bsr {
namespace lab {

template <int NW, int R, int NB = 4, int HOT = 0, int ECAP = 256>
__global__ __launch_bounds__(NW * 64, 1) void k_filter_rs(GemmArgs p) {
    constexpr int NK = 12, NQB = 8, D = R - 1, TB = 2 * NK * 1024;  // tile bytes (32 rows)
    static_assert(NK % R == 0, "ring depth divides the slice count");
    __shared__ __attribute__((aligned(1024))) uint8_t lds[NK * NQB * 1024 + NW * ECAP * 12 + 128 * 8];
    float* const qpar = reinterpret_cast<float*>(lds + NK * NQB * 1024 + NW * ECAP * 12);  // [128] tau, [128] scale
    const int tid = threadIdx.x, lane = tid & 63;
    const uint32_t wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint64_t* const ekeys = reinterpret_cast<uint64_t*>(lds + NK * NQB * 1024) + wu * ECAP;
    uint32_t* const eq = reinterpret_cast<uint32_t*>(lds + NK * NQB * 1024 + NW * ECAP * 8) + wu * ECAP;

    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t spx = (gridDim.x >> 3) / p.n_qt, S = 8 * spx;
    const bool active = slot < spx * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0, sid = xcd * spx + (active ? slot / p.n_qt : 0);
    const uint32_t T = (p.n_rows + 31) / 32;
    const uint32_t t0 = active ? (uint32_t)((uint64_t)T * sid / S) : 0;
    const uint32_t t1 = active ? (uint32_t)((uint64_t)T * (sid + 1) / S) : 0;
    const uint32_t my_n = t1 > t0 + wu ? (t1 - t0 - wu + NW - 1) / NW : 0;

    // B fragments of the query tile: fragment (kt, qb) lane l = query qt*128 + 16qb + (l & 15),
    // bytes 64kt + 16(l >> 4) .. +15
    for (uint32_t i = tid; i < NK * NQB * 64; i += NW * 64) {
        const uint32_t f = i >> 6, l = i & 63, kt = f / NQB, qb = f % NQB;
        const uint32_t q = qt * 128 + 16 * qb + (l & 15);
        *reinterpret_cast<i32x4v_t*>(lds + f * 1024 + l * 16) =
            *reinterpret_cast<const i32x4v_t*>(p.B + (uint64_t)q * p.row_bytes + 64 * kt + 16 * (l >> 4));
    }
    if (tid < 128) {
        qpar[tid] = p.tau[qt * 128 + tid];
        qpar[128 + tid] = p.b_scale[qt * 128 + tid];
    }
    __syncthreads();

    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (uint64_t)t0 * TB), 0, (t1 - t0) * TB, 0x00020000);
    const uint32_t voff = lane * 16;
    // slice g of the wave's sequence: tile j = g / NK, slice kt = g % NK
    i32x4v_t fa[R][2];
    auto load = [&](uint32_t j, int kt, int s) {
        const uint32_t base = (wu + NW * (HOT ? j % 4 : j)) * TB + kt * 1024;  // (HOT, lab: L2-resident)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
            fa[s][rb] = (i32x4v_t)__builtin_amdgcn_raw_buffer_load_b128(rs, voff, base + rb * NK * 1024, 0);
    };
    uint32_t ecount = 0;  // (wave-uniform) entries in the wave's list
    auto flush = [&]() {
        for (uint32_t e = lane; e < ecount; e += 64) {
            const uint32_t q = eq[e];
            const uint32_t gp = atomicAdd(p.cnt + q, 1u);
            if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = ekeys[e];
        }
        ecount = 0;
    };
    if (my_n)
#pragma unroll
        for (int s = 0; s < D; ++s) load(0, s, s);

    // B fragments through a ring of NB registers, read NB - 1 ahead: fragment f = kt * NQB + qb of
    // the tile's 96 (the same 96 every tile: the queries are stationary in LDS)
    constexpr int NF = NK * NQB;
    static_assert(NF % NB == 0, "B ring divides the fragment count");
    i32x4v_t bq[NB];
    auto read_b = [&](int f) { bq[f % NB] = *reinterpret_cast<const i32x4v_t*>(lds + (f % NF) * 1024 + voff); };
#pragma unroll
    for (int f = 0; f < NB - 1; ++f) read_b(f);
    i32x4v_t acc[2][NQB];
    for (uint32_t j = 0; j < my_n; ++j) {
        static_for(std::make_integer_sequence<int, NK>{}, [&](auto KT) {
            constexpr int kt = decltype(KT)::value;
#pragma unroll
            for (int qb = 0; qb < NQB; ++qb) {
                const int f = kt * NQB + qb;
#pragma unroll
                for (int rb = 0; rb < 2; ++rb) {
                    if (kt == 0) {
                        const i32x4v_t z = {};
                        acc[rb][qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[kt % R][rb], bq[f % NB], z, 0, 0, 0);
                    } else {
                        acc[rb][qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[kt % R][rb], bq[f % NB], acc[rb][qb], 0, 0, 0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                read_b(f + NB - 1);
                // slice g + D into the slot slice g - 1 used (its MFMAs are issued), after query block 1
                if (qb == 1) {
                    if (kt + D < NK) load(j, kt + D, (kt + D) % R);
                    else load(j + 1, kt + D - NK, (kt + D) % R);  // (past the wave's last tile: out of range, reads 0)
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        });
        // ---- epilogue: acc[rb][qb] holds rows 16rb + 4(lane >> 4) + i of the tile, query 16qb + (lane & 15)
        const uint32_t tile = t0 + wu + NW * j;
        const float sc = p.a_scale[tile];  // (32-row quantisation block = the tile)
        bool any = false;
        int mq[NQB];
        float tau[NQB], sbq[NQB];
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            tau[qb] = qpar[16 * qb + (lane & 15)];
            sbq[qb] = qpar[128 + 16 * qb + (lane & 15)];
        }
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            int m = acc[0][qb][0];
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                for (int i = 0; i < 4; ++i) m = (rb | i) ? max(m, acc[rb][qb][i]) : m;
            mq[qb] = m;
            any |= ((float)m * sc) * sbq[qb] >= tau[qb];
        }
        if (__ballot(any)) {
#pragma unroll
            for (int qb = 0; qb < NQB; ++qb) {
                if (!__ballot(((float)mq[qb] * sc) * sbq[qb] >= tau[qb])) continue;
                const uint32_t q = qt * 128 + 16 * qb + (lane & 15);
#pragma unroll
                for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float v = ((float)acc[rb][qb][i] * sc) * sbq[qb];
                        const uint32_t row = tile * 32 + 16 * rb + 4 * (lane >> 4) + i;
                        const bool ok = v >= tau[qb] && row < p.n_rows;
                        if (ecount > (uint32_t)(ECAP - 64)) flush();
                        const uint64_t mask = __ballot(ok);
                        if (ok) {
                            const uint32_t pos = ecount + __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
                            ekeys[pos] = score_key(v, row);
                            eq[pos] = q;
                        }
                        ecount += (uint32_t)__builtin_popcountll(mask);
                    }
            }
        }
    }
    flush();
    __builtin_amdgcn_s_waitcnt(0x0F70);  // (trailing loads land before the wave ends)
}

// row-major int8 rows [npad][768] -> fragment-native [npad / 16][12][64 lanes][16 B]
__global__ void k_to_native(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint32_t npad) {
    const uint64_t n16 = (uint64_t)npad * 48;  // 16-byte chunks
    for (uint64_t o = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; o < n16; o += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r16 = o / (12 * 64);
        const uint32_t rem = (uint32_t)(o % (12 * 64)), kt = rem / 64, l = rem % 64;
        const uint64_t row = r16 * 16 + (l & 15);
        *reinterpret_cast<uint4*>(dst + o * 16) =
            *reinterpret_cast<const uint4*>(src + row * 768 + 64 * kt + 16 * (l >> 4));
    }
}

}  // namespace lab
}  // namespace bsr
