// k_qs16_lab.hip -- TOOLING (candidate for the product): the product's query-stationary
// int8 emit filter (k_filter.hip, bsr::k_filter_qs16<true, NK>) with a STAGED emission
// epilogue instead of the two-level per-row one.
//
// Product epilogue: level 1 = the lane's integer maximum over its 32 values per query
// block against tau, one ballot per tile; level 2 (when any lane passes) = per 16-row block
// maxima, then per passing block its 4 rows into a private per-lane LDS ring.  Level 2 runs
// on most wave-tiles at the product's emission rate (~1 emitted row per 32 queries x 128
// rows) and all 8 waves wait for the slowest at the next barrier.
// Staged: a lane that passes level 1 writes its 32 raw int32 values (8 x ds_write_b128) and
// one meta record (first row, query, tau, query scale) into a per-wave staging area (slot =
// count + mbcnt of the pass mask); the wave then scores two staged entries per iteration,
// one value per lane, and compacts passing (key, query) pairs into a per-wave key ring
// (ballot + mbcnt).  The key ring goes to the global per-query lists at the end (or when
// full) with one global atomic per (wave, query).  Emitted SETS equal the product's.
// VAR bits: 1 = no level-2 work at all (level 1 only, results discarded: cost floor);
// 2 = level-1 maxima folded into the last slice's MFMA stream (row block rb - 2 after group rb);
// 4 = staged entries scored later, one step (2 entries) per slice inside the next tile's
// MFMA stream (the two waves of a SIMD at different groups) instead of in the epilogue;
// 8 = one barrier per FOUR slices (12-slot ring, 8 slices ahead; NK % 4 == 0);
// 16 = timing probe: the final key-ring flush (global atomics + stores) skipped;
// 32 = fragment reads as inline asm with hand-counted lgkmcnt waits.
// Included after the product k_filter.hip (uses its types and helpers).
namespace bsrlab {
using namespace bsr;

// A wave-uniform 16-byte load through the scalar data cache (a LOAD: counted in lgkmcnt,
// so it leaves the LDS-DMA stream's vmcnt accounting alone); the wait is part of it.
__device__ __forceinline__ float4 smem_load_f32x4(const float* p) {
    typedef __attribute__((ext_vector_type(4))) float f4_t;
    f4_t v;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return make_float4(v[0], v[1], v[2], v[3]);
}

// compiler-only ordering of this wave's LDS accesses across lanes (the LDS executes a wave's
// operations in order, so no wait is needed)
__device__ __forceinline__ void wave_lds_order() { asm volatile("" ::: "memory"); }
// LDS accesses of the emission path as inline asm: the compiler cannot prove them disjoint
// from the in-flight LDS-DMA slots and would drain the whole DMA stream (vmcnt(0)) first
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)p; }
__device__ __forceinline__ void ds_st128(uint32_t a, i32x4v_t v) {
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void ds_st64(uint32_t a, uint64_t v) {
    asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void ds_st32(uint32_t a, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ int ds_ld32_wait(uint32_t a) {
    int r;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
    return r;
}
__device__ __forceinline__ i32x4v_t ds_ld128_wait(uint32_t a) {
    i32x4v_t r;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
    return r;
}

template <int NK, int VAR = 0, int NW = 8>
__global__ __launch_bounds__(512, 1) void k_filter_qs16s(GemmArgs p) {
    // BAR slices per barrier: 2 (product: 8 slots, 6 ahead) or 4 (VAR & 8: 12 slots, 8 ahead).
    // Slot reuse needs A <= S - BAR; at a barrier (slice jj, after group 5) slices <= jj + BAR + 1
    // must have landed, leaving A - 1 - (BAR + 1) younger DMAs in flight.
    constexpr int BAR = (VAR & 8) ? 4 : 2;
    constexpr int S = (VAR & 8) ? 12 : 8, A = (VAR & 8) ? 8 : 6;
    constexpr int WAITN = A - 2 - BAR;
    static_assert(A <= S - BAR && NK % BAR == 0, "ring geometry");
    // NW waves of 32 queries per workgroup: 8 (one workgroup per CU) or 4 (two per CU, each
    // with its own ring and barriers: one computes while the other is in its epilogue)
    static_assert(NW == 8 || NW == 4, "4 or 8 waves");
    constexpr int BM = 128, BN = 32 * NW, NT = 64 * NW, SLOT = BM * kSliceB;
    constexpr int ND = 8 / NW;           // 1-KiB DMA instructions per wave per slice
    constexpr int STG = NW == 8 ? 16 : 8;   // staged (lane, query block) entries per wave
    constexpr int KR = NW == 8 ? 256 : 128; // key-ring entries per wave
    static_assert(NK % 2 == 0 && NK >= 2 && NK <= 12, "even slice counts up to 768 bytes");
    // ONE LDS object (separate __shared__ variables get alias scopes, and the compiler then
    // waits for the LDS-DMA stream before every fragment read): ring | staging | key ring
    constexpr int STG_V = S * SLOT, STG_M = STG_V + NW * STG * 32 * 4, KR_KEY = STG_M + NW * STG * 16;
    constexpr int KR_Q = KR_KEY + NW * KR * 8, KR_CNT = KR_Q + NW * KR * 4, LDS_BYTES = KR_CNT + NW * 32 * 4;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[LDS_BYTES];
    // staging: [wave][entry][32 int32 values], meta [wave][entry] = {row0, q, tau, sbq}
    auto stg_v = reinterpret_cast<int32_t (*)[STG][32]>(lds + STG_V);
    auto stg_m = reinterpret_cast<uint32_t (*)[STG][4]>(lds + STG_M);
    auto kr_key = reinterpret_cast<uint64_t (*)[KR]>(lds + KR_KEY);
    auto kr_q = reinterpret_cast<uint32_t (*)[KR]>(lds + KR_Q);      // local query | position << 8
    auto kr_cnt = reinterpret_cast<uint32_t (*)[32]>(lds + KR_CNT);  // per-query counts, then bases
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t wu = __builtin_amdgcn_readfirstlane(tid >> 6);

    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * NK;
    const uint32_t qw0 = qt * BN + w * 32;  // the wave's first query

    uint32_t qq[2];
    i32x4v_t fb[2][NK];
    float tau[2], sbq[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
        qq[nb] = qw0 + nb * 16 + (lane & 15);
        const uint8_t* src = p.B + (uint64_t)qq[nb] * p.row_bytes + 16 * (lane >> 4);
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) fb[nb][kt] = *reinterpret_cast<const i32x4v_t*>(src + 64 * kt);
        tau[nb] = p.tau[qq[nb]];
        sbq[nb] = p.b_scale[qq[nb]];
    }
    uint32_t scnt = 0, kcnt = 0;  // wave-uniform
    // key ring -> global lists: per-query counts in LDS, one global atomic per query, scatter
    auto flush_keys = [&]() {
        if (lane < 32) kr_cnt[w][lane] = 0;
        wave_lds_order();
        for (uint32_t i = lane; i < kcnt; i += 64) {
            const uint32_t ql = kr_q[w][i] & 31u;
            const uint32_t pos = atomicAdd(&kr_cnt[w][ql], 1u);
            kr_q[w][i] = ql | (pos << 8);
        }
        wave_lds_order();
        if (lane < 32) {
            const uint32_t c = kr_cnt[w][lane];
            kr_cnt[w][lane] = c ? atomicAdd(p.cnt + qw0 + lane, c) : 0u;
        }
        wave_lds_order();
        for (uint32_t i = lane; i < kcnt; i += 64) {
            const uint32_t ql = kr_q[w][i] & 31u, gp = kr_cnt[w][ql] + (kr_q[w][i] >> 8);
            if (gp < p.cap) p.cand[(uint64_t)(qw0 + ql) * p.cap + gp] = kr_key[w][i];
        }
        kcnt = 0;
    };

    // wave w fills rows 16 * ND * w .. + 16 * ND - 1 of every slice (ND instructions)
    auto dma_off = [&](int i) {
        const uint32_t lrow = (w * ND + i) * 16 + (lane >> 2);
        return lrow * (uint32_t)p.a_stride + ((lane & 3) ^ qs16_swz(lrow)) * 16;
    };
    const uint32_t aoff_dma0 = dma_off(0), aoff_dma1 = ND > 1 ? dma_off(1) : 0u;
    uint32_t iss_ti = 0, iss_kt = 0;
    __amdgpu_buffer_rsrc_t rsrc_a;
    auto set_issue_tile = [&]() {
        const uint32_t rt = g0 + iss_ti * RG;
        rsrc_a = __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (uint64_t)rt * BM * p.a_stride), 0,
                                                   BM * (uint32_t)p.a_stride, 0x00020000);
    };
    auto issue_dma = [&](uint32_t jj) {
        uint8_t* la = lds + (jj % S) * SLOT + wu * ND * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)la, 16, aoff_dma0, iss_kt * kSliceB, 0, 0);
        if (ND > 1)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)(la + 1024), 16, aoff_dma1, iss_kt * kSliceB, 0, 0);
        if (++iss_kt == NK) {
            iss_kt = 0;
            ++iss_ti;
            if (iss_ti < my_rt) set_issue_tile();
        }
    };
    const uint32_t aoff0 = (lane & 15) * kSliceB + (((lane >> 4) ^ qs16_swz(lane & 15)) * 16);
    i32x4v_t fa[4];
    // VAR & 32: fragment reads as inline asm with hand-counted waits (the compiler does not
    // track them, so a branch in the loop does not make it wait for every read at the join)
    auto read_frag = [&](uint32_t jj, int rb) {
        if constexpr ((VAR & 32) != 0) {
            const uint32_t addr = lds_addr(lds + (jj % S) * SLOT + rb * 1024 + aoff0);
            asm volatile("ds_read_b128 %0, %1" : "=v"(fa[rb & 3]) : "v"(addr) : "memory");
        } else {
            fa[rb & 3] = *reinterpret_cast<const i32x4v_t*>(lds + (jj % S) * SLOT + rb * 1024 + aoff0);
        }
    };
    // before the MFMAs of row block rb: its read (issued four blocks earlier) has returned
    // (LDS returns in order; at most the three younger reads still in flight)
    auto frag_wait = [&](int rb) {
        if constexpr ((VAR & 32) != 0) asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(fa[rb & 3]));
    };

    i32x4v_t acc[8][2];
    if (my_rt) set_issue_tile();
    const uint32_t pre = J ? (uint32_t)A : 0u;
    for (uint32_t jj = 0; jj < pre; ++jj) issue_dma(jj);
    qs_barrier(pre >= (uint32_t)(BAR + 1) ? (pre - (BAR + 1)) * ND : 0);  // slices 0 .. BAR landed everywhere
    if (J)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) read_frag(0, rb);

    // staged entries [dr, scnt) wait to be scored with the block scales psc of their tile
    uint32_t dr = 0;
    float psc[4] = {1.0f, 1.0f, 1.0f, 1.0f};
    // score staged entries e0, e0 + 1 (lane -> entry e0 + lane/32, value lane%32)
    auto drain_step = [&](uint32_t e0) {
        const uint32_t vi = lane & 31, rb = vi >> 2;
        const float scr = rb < 4 ? (rb < 2 ? psc[0] : psc[1]) : (rb < 6 ? psc[2] : psc[3]);
        const uint32_t e = e0 + (lane >> 5);
        const bool valid = e < scnt;
        const uint32_t ec = valid ? e : e0;
        const int v = ds_ld32_wait(lds_addr(&stg_v[w][ec][vi]));
        const i32x4v_t m4 = ds_ld128_wait(lds_addr(&stg_m[w][ec][0]));
        const uint32_t row = (uint32_t)m4[0] + (rb << 4) + (vi & 3);
        const float sv = ((float)v * scr) * __int_as_float(m4[3]);
        const bool ok = valid && sv >= __int_as_float(m4[2]) && row < p.n_rows;
        const uint64_t bm = __ballot(ok);
        if (ok) {
            const uint32_t ks = kcnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
            ds_st64(lds_addr(&kr_key[w][ks]), score_key(sv, row));
            ds_st32(lds_addr(&kr_q[w][ks]), (uint32_t)m4[1]);
        }
        kcnt += (uint32_t)__builtin_popcountll(bm);
    };
    // every staged entry scored (flushing the key ring when it could overflow)
    auto drain_all = [&]() -> bool {
        bool st = false;
        wave_lds_order();
        for (; dr < scnt; dr += 2) {
            if (kcnt > (uint32_t)(KR - 64)) {
                flush_keys();
                st = true;
            }
            drain_step(dr);
        }
        scnt = dr = 0;
        return st;
    };
    // the wave pair on one SIMD (w, w + 4) drains at different groups of a slice
    const int drain_rb = (wu >> 2) ? 2 : 6;

    for (uint32_t t = 0; t < my_rt; ++t) {
        const uint32_t rt = g0 + t * RG;
        const float4 scv = *reinterpret_cast<const float4*>(p.a_scale + (uint64_t)rt * (BM / kQuantBlock));
        int mx[2] = {INT32_MIN, INT32_MIN};  // level-1 maxima, folded into the last slice
        auto fold = [&](int rb) {
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                const i32x4v_t& x = acc[rb][nb];
                mx[nb] = max(mx[nb], max(max(x[0], x[1]), max(x[2], x[3])));
            }
        };
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) {
            const uint32_t jj = t * NK + kt;
            const bool bar_slice = (kt % BAR) == BAR - 1;
#pragma unroll
            for (int rb = 0; rb < 8; ++rb) {
                frag_wait(rb);
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
                if (bar_slice ? rb == 6 : rb == 1) issue_dma(jj + A);
                if (bar_slice && rb == 5 && jj + 1 < J) qs_wait_n(WAITN * ND + (kt <= A - 2 - BAR ? 1 : 0));
                if ((VAR & 2) && kt == NK - 1 && rb >= 2) fold(rb - 2);
                if ((VAR & 4) && kt >= 1 && kt <= NK - 2 && rb == drain_rb) {
                    // deferred scoring of the previous tile's staged entries, in the MFMA stream
                    if (dr < scnt && kcnt <= (uint32_t)(KR - 64)) {
                        wave_lds_order();
                        drain_step(dr);
                        dr += 2;
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // ---- epilogue, level 1: the lane's maximum over its 32 values per query block
        const float sc[4] = {scv.x, scv.y, scv.z, scv.w};
        const float sc_hi = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
        const float sc_lo = fminf(fminf(sc[0], sc[1]), fminf(sc[2], sc[3]));
        if (VAR & 2) {
            fold(6);
            fold(7);
        } else {
#pragma unroll
            for (int rb = 0; rb < 8; ++rb) fold(rb);
        }
        bool pass[2];
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) pass[nb] = ((float)mx[nb] * (mx[nb] >= 0 ? sc_hi : sc_lo)) * sbq[nb] >= tau[nb];
        if constexpr (VAR & 1) {
            asm volatile("" ::"v"(pass[0]), "v"(pass[1]));
            continue;
        }
        bool stored = false;
        if (dr < scnt) stored |= drain_all();  // the previous tile's entries, not yet scored
        scnt = dr = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) psc[i] = sc[i];
        // stage the passing lanes' 32 values (slot = count + rank in the pass mask)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            uint64_t m = __ballot(pass[nb]);
            while (m) {
                const uint32_t room = STG - scnt;
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                const bool mine = ((m >> lane) & 1ull) && rank < room;
                if (mine) {
                    const uint32_t e = scnt + rank;
#pragma unroll
                    for (int rb = 0; rb < 8; ++rb) ds_st128(lds_addr(&stg_v[w][e][rb * 4]), acc[rb][nb]);
                    const i32x4v_t mt = {(int)(rt * BM + 4 * (lane >> 4)), nb * 16 + (lane & 15),
                                         __float_as_int(tau[nb]), __float_as_int(sbq[nb])};
                    ds_st128(lds_addr(&stg_m[w][e][0]), mt);
                }
                const uint64_t took = __ballot(mine);
                m &= ~took;
                scnt += (uint32_t)__builtin_popcountll(took);
                if (scnt == STG) stored |= drain_all();
            }
        }
        if (!(VAR & 4) && scnt) stored |= drain_all();
        if (stored) wait_vm0();  // global stores / atomics count in vmcnt: keep the waits exact
    }
    if (scnt) (void)drain_all();
    wait_vm0();
    wave_lds_order();
    if (VAR & 16) {  // timing probe: no global candidate writes at the end (results incomplete)
        if (kcnt == 12345) p.cnt[0] = kcnt;
        return;
    }
    flush_keys();
}


// ------------------------------------------------------------------------------------
// SKEWED wave groups (candidate for the product).  The two waves on each SIMD (w, w + 4)
// belong to groups A (waves 0-3) and B (waves 4-7); group B consumes the shared slice
// stream L = NK/2 slices behind group A (its query fragments loaded in rotated K order, so
// the register index of slice kt stays static), so the groups' tile epilogues alternate:
// while one group scores its tile, the other keeps the SIMD's MFMA pipe busy.  The ring
// holds S = 14 slots (A + L + 1 <= S: after the barrier of slice jj every wave is done with
// slices <= jj - L).  Emission as k_filter_qs16s (staged per-wave entries, key ring).
// Accumulators are zeroed explicitly after each epilogue (no C = 0 first MFMA).
// ------------------------------------------------------------------------------------
template <int NK>
__global__ __launch_bounds__(512, 1) void k_filter_qs16k(GemmArgs args) {
    // the arguments the lambdas below use, as locals (a reference to the by-value kernel
    // argument would put a copy of it in scratch memory, and scratch loads count in vmcnt)
    const uint8_t* const pA = args.A;
    const uint8_t* const pB = args.B;
    const uint64_t a_stride = args.a_stride, row_bytes = args.row_bytes;
    const uint32_t n_rows = args.n_rows, n_qt = args.n_qt, cap = args.cap;
    const float* const a_scale = args.a_scale;
    const float* const b_scale = args.b_scale;
    const float* const tau_in = args.tau;
    uint64_t* const cand = args.cand;
    uint32_t* const cntp = args.cnt;
    constexpr int S = 14, A = 6, L = NK / 2;
    static_assert(NK % 4 == 0 && NK >= 4 && NK <= 12, "NK in {4, 8, 12}: L even");
    static_assert(A + L + 1 <= S, "slot reuse");
    constexpr int BM = 128, BN = kFilterTile, SLOT = BM * kSliceB;
    constexpr int STG = 16, KR = 192;
    constexpr int STG_V = S * SLOT, STG_M = STG_V + 8 * STG * 32 * 4, KR_KEY = STG_M + 8 * STG * 16;
    constexpr int KR_Q = KR_KEY + 8 * KR * 8, KR_CNT = KR_Q + 8 * KR * 4, LDS_BYTES = KR_CNT + 8 * 32 * 4;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(1024))) uint8_t lds[LDS_BYTES];
    auto stg_v = reinterpret_cast<int32_t (*)[STG][32]>(lds + STG_V);
    auto stg_m = reinterpret_cast<uint32_t (*)[STG][4]>(lds + STG_M);
    auto kr_key = reinterpret_cast<uint64_t (*)[KR]>(lds + KR_KEY);
    auto kr_q = reinterpret_cast<uint32_t (*)[KR]>(lds + KR_Q);
    auto kr_cnt = reinterpret_cast<uint32_t (*)[32]>(lds + KR_CNT);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t grp = wu >> 2;            // 0: group A, 1: group B (L slices behind)
    const uint32_t lag = grp * L;

    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / n_qt;
    const uint32_t n_rt = (n_rows + BM - 1) / BM;
    const bool active = slot < G * n_qt;
    const uint32_t qt = active ? slot % n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t JA = my_rt * NK;          // slices of group A's stream
    const uint32_t X = my_rt ? JA + L : 0;   // loop positions (group B finishes L later)
    const uint32_t qw0 = qt * BN + w * 32;

    // query fragments; group B's in rotated K order: fb[nb][kt] = K slice (kt + lag) % NK
    uint32_t qq[2];
    i32x4v_t fb[2][NK];
    float tau[2], sbq[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
        qq[nb] = qw0 + nb * 16 + (lane & 15);
        const uint8_t* src = pB + (uint64_t)qq[nb] * row_bytes + 16 * (lane >> 4);
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) {
            const uint32_t ks = (kt + lag) % NK;
            fb[nb][kt] = *reinterpret_cast<const i32x4v_t*>(src + 64 * ks);
        }
        tau[nb] = tau_in[qq[nb]];
        sbq[nb] = b_scale[qq[nb]];
    }
    // these loads complete here, visibly to the compiler (s_waitcnt vmcnt(0), as a builtin):
    // otherwise its first use in an epilogue, far into the DMA stream, gets a vmcnt(0)
    __builtin_amdgcn_s_waitcnt(0xF70);
    uint32_t scnt = 0, kcnt = 0;
    auto flush_keys = [&]() __attribute__((always_inline)) {
        if (lane < 32) kr_cnt[w][lane] = 0;
        wave_lds_order();
        for (uint32_t i = lane; i < kcnt; i += 64) {
            const uint32_t ql = kr_q[w][i] & 31u;
            const uint32_t pos = atomicAdd(&kr_cnt[w][ql], 1u);
            kr_q[w][i] = ql | (pos << 8);
        }
        wave_lds_order();
        if (lane < 32) {
            const uint32_t c = kr_cnt[w][lane];
            kr_cnt[w][lane] = c ? atomicAdd(cntp + qw0 + lane, c) : 0u;
        }
        wave_lds_order();
        for (uint32_t i = lane; i < kcnt; i += 64) {
            const uint32_t ql = kr_q[w][i] & 31u, gp = kr_cnt[w][ql] + (kr_q[w][i] >> 8);
            if (gp < cap) cand[(uint64_t)(qw0 + ql) * cap + gp] = kr_key[w][i];
        }
        kcnt = 0;
    };

    const uint32_t lrow = w * 16 + (lane >> 2);
    const uint32_t aoff_dma = lrow * (uint32_t)a_stride + ((lane & 3) ^ qs16_swz(lrow)) * 16;
    uint32_t iss_ti = 0, iss_kt = 0;
    __amdgpu_buffer_rsrc_t rsrc_a;
    auto set_issue_tile = [&]() __attribute__((always_inline)) {
        const uint32_t rt = g0 + iss_ti * RG;
        rsrc_a = __builtin_amdgcn_make_buffer_rsrc((void*)(pA + (uint64_t)rt * BM * a_stride), 0,
                                                   BM * (uint32_t)a_stride, 0x00020000);
    };
    auto issue_dma = [&](uint32_t jj) __attribute__((always_inline)) {
        uint8_t* la = lds + (jj % S) * SLOT + wu * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)la, 16, aoff_dma, iss_kt * kSliceB, 0, 0);
        if (++iss_kt == NK) {
            iss_kt = 0;
            ++iss_ti;
            if (iss_ti < my_rt) set_issue_tile();
        }
    };
    const uint32_t aoff0 = (lane & 15) * kSliceB + (((lane >> 4) ^ qs16_swz(lane & 15)) * 16);
    i32x4v_t fa[4];
    // this wave's slice at loop position x is x - lag (slot (x + S - lag) % S)
    auto read_frag = [&](uint32_t x, int rb) __attribute__((always_inline)) {
        fa[rb & 3] = *reinterpret_cast<const i32x4v_t*>(lds + ((x + S - lag) % S) * SLOT + rb * 1024 + aoff0);
    };

    i32x4v_t acc[8][2];
#define mask_acc(M)                                                                               \
    do {                                                                                          \
        const int m_ = __builtin_amdgcn_readfirstlane(M);                                         \
        _Pragma("unroll") for (int rb = 0; rb < 8; ++rb)                                          \
            _Pragma("unroll") for (int nb = 0; nb < 2; ++nb) acc[rb][nb] &= m_;                   \
    } while (0)
#define zero_acc()                                                                                \
    do {                                                                                          \
        _Pragma("unroll") for (int rb = 0; rb < 8; ++rb)                                          \
            _Pragma("unroll") for (int nb = 0; nb < 2; ++nb) acc[rb][nb] = i32x4v_t{0, 0, 0, 0};  \
    } while (0)
    zero_acc();
    if (my_rt) set_issue_tile();
    const uint32_t pre = X ? (uint32_t)A : 0u;
    for (uint32_t jj = 0; jj < pre; ++jj) issue_dma(jj);
    qs_barrier(pre >= 3 ? pre - 3 : 0);  // slices 0, 1, 2 landed everywhere
    if (X)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) read_frag(0, rb);

    // the tile's 32-row block scales (uniform; read through the constant address space, i.e.
    // scalar loads counted in lgkmcnt, outside the DMA stream's vmcnt)
    float sc0 = 1.0f, sc1 = 1.0f, sc2 = 1.0f, sc3 = 1.0f;
#define load_scales(U)                                                                            \
    do {                                                                                          \
        const uint32_t rt_s = __builtin_amdgcn_readfirstlane(g0 + (U) * RG);                      \
        const float4 v_s = smem_load_f32x4(a_scale + (uint64_t)rt_s * (BM / kQuantBlock));       \
        sc0 = v_s.x; sc1 = v_s.y; sc2 = v_s.z; sc3 = v_s.w;                                       \
    } while (0)
    // tile U's epilogue: level 1 (lane maxima), staging of passing lanes, scoring; sets
    // STORED when global stores / atomics were issued (a macro: no closures in the loop)
#define BSR_QS16K_DRAIN(STORED)                                                                   \
    do {                                                                                          \
        wave_lds_order();                                                                         \
        const uint32_t vi = lane & 31, rbv = vi >> 2;                                             \
        const float scr = rbv < 4 ? (rbv < 2 ? sc0 : sc1) : (rbv < 6 ? sc2 : sc3);               \
        for (uint32_t e0 = 0; e0 < scnt; e0 += 2) {                                               \
            if (kcnt > (uint32_t)(KR - 64)) {                                                     \
                flush_keys();                                                                     \
                STORED = true;                                                                    \
            }                                                                                     \
            const uint32_t e = e0 + (lane >> 5);                                                  \
            const bool valid = e < scnt;                                                          \
            const uint32_t ec = valid ? e : e0;                                                   \
            const int v = ds_ld32_wait(lds_addr(&stg_v[w][ec][vi]));                              \
            const i32x4v_t m4 = ds_ld128_wait(lds_addr(&stg_m[w][ec][0]));                        \
            const uint32_t row = (uint32_t)m4[0] + (rbv << 4) + (vi & 3);                         \
            const float sv = ((float)v * scr) * __int_as_float(m4[3]);                            \
            const bool ok = valid && sv >= __int_as_float(m4[2]) && row < n_rows;                 \
            const uint64_t bm = __ballot(ok);                                                     \
            if (ok) {                                                                             \
                const uint32_t ks = kcnt + __builtin_amdgcn_mbcnt_hi(                             \
                                               (uint32_t)(bm >> 32),                              \
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));      \
                ds_st64(lds_addr(&kr_key[w][ks]), score_key(sv, row));                            \
                ds_st32(lds_addr(&kr_q[w][ks]), (uint32_t)m4[1]);                                 \
            }                                                                                     \
            kcnt += (uint32_t)__builtin_popcountll(bm);                                           \
        }                                                                                         \
        scnt = 0;                                                                                 \
    } while (0)
#define BSR_QS16K_EPILOGUE(U, STORED)                                                             \
    do {                                                                                          \
        const uint32_t rt_e = g0 + (U) * RG;                                                      \
        const float sc_hi = fmaxf(fmaxf(sc0, sc1), fmaxf(sc2, sc3));                              \
        const float sc_lo = fminf(fminf(sc0, sc1), fminf(sc2, sc3));                              \
        bool pass[2];                                                                             \
        _Pragma("unroll") for (int nb = 0; nb < 2; ++nb) {                                        \
            int m = acc[0][nb][0];                                                                \
            _Pragma("unroll") for (int rb = 0; rb < 8; ++rb)                                      \
                _Pragma("unroll") for (int r = 0; r < 4; ++r) m = (rb | r) ? max(m, acc[rb][nb][r]) : m; \
            pass[nb] = ((float)m * (m >= 0 ? sc_hi : sc_lo)) * sbq[nb] >= tau[nb];                \
        }                                                                                         \
        _Pragma("unroll") for (int nb = 0; nb < 2; ++nb) {                                        \
            uint64_t m = __ballot(pass[nb]);                                                      \
            while (m) {                                                                           \
                const uint32_t room = STG - scnt;                                                 \
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),              \
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)); \
                const bool sel = ((m >> lane) & 1ull) && rank < room;                             \
                if (sel) {                                                                        \
                    const uint32_t e = scnt + rank;                                               \
                    _Pragma("unroll") for (int rb = 0; rb < 8; ++rb)                              \
                        ds_st128(lds_addr(&stg_v[w][e][rb * 4]), acc[rb][nb]);                    \
                    const i32x4v_t mt = {(int)(rt_e * BM + 4 * (lane >> 4)), nb * 16 + (lane & 15), \
                                         __float_as_int(tau[nb]), __float_as_int(sbq[nb])};       \
                    ds_st128(lds_addr(&stg_m[w][e][0]), mt);                                      \
                }                                                                                 \
                const uint64_t took = __ballot(sel);                                              \
                m &= ~took;                                                                       \
                scnt += (uint32_t)__builtin_popcountll(took);                                     \
                if (scnt == STG) BSR_QS16K_DRAIN(STORED);                                         \
            }                                                                                     \
        }                                                                                         \
        if (scnt) BSR_QS16K_DRAIN(STORED);                                                        \
    } while (0)

    // loop positions x = t * NK + kt; group A works on slices x < JA, group B on x - L for
    // L <= x < X.  A's tile epilogue at kt == 0 (t > 0), B's at kt == L (t > 0).
    uint32_t uA = 0, uB = 0;  // the tile each group is on
    if (grp == 0 && my_rt) load_scales(0);
    // one slice at loop position x = t * NK + kt (kt a constant once unrolled; a macro, not a
    // lambda: the fragment arrays must not escape into memory before unrolling)
#define BSR_QS16K_SLICE(T, KT)                                                                   \
    do {                                                                                         \
        const uint32_t x = (T) * NK + (KT);                                                      \
        _Pragma("unroll") for (int rb = 0; rb < 8; ++rb) {                                        \
            _Pragma("unroll") for (int nb = 0; nb < 2; ++nb) acc[rb][nb] =                        \
                __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[rb & 3], fb[nb][KT], acc[rb][nb], 0, 0, 0); \
            __builtin_amdgcn_sched_barrier(0);                                                   \
            if (rb < 4) read_frag(x, rb + 4);                                                    \
            else read_frag(x + 1, rb - 4);                                                       \
            if (((KT) & 1) ? rb == 6 : rb == 1) issue_dma(x + A);                                \
            if (((KT) & 1) && rb == 5) qs_wait<2>();                                             \
            __builtin_amdgcn_sched_barrier(0);                                                   \
        }                                                                                        \
    } while (0)
    // Branch-free slices (a branch around the MFMAs or reads would make the compiler wait for
    // every LDS read at each join): a group's MFMAs outside its own tiles run on stale
    // fragments into accumulators that are zeroed (B before its first tile) or no longer
    // read (A after its last epilogue).
    for (uint32_t t = 0; t < my_rt; ++t) {
        // group A's tile epilogue at kt == 0, group B's at kt == L (outside the unrolled
        // slice loops)
        if (grp == 0 && t > 0) {
            bool stored = false;
            BSR_QS16K_EPILOGUE(uA, stored);
            ++uA;
            load_scales(uA);
            if (stored) wait_vm0();  // global stores / atomics count in vmcnt
        }
        // accumulators zeroed without a branch (AND with a wave-uniform mask): a conditional
        // assignment would split their live ranges and cost register copies in the loop
        mask_acc((grp == 0 && t > 0) ? 0 : -1);
#pragma unroll
        for (int kt = 0; kt < L; ++kt) BSR_QS16K_SLICE(t, kt);
        if (grp == 1) {
            bool stored = false;
            if (t > 0) {
                BSR_QS16K_EPILOGUE(uB, stored);
                ++uB;
            }
            load_scales(uB);
            if (stored) wait_vm0();
        }
        mask_acc(grp == 1 ? 0 : -1);
#pragma unroll
        for (int kt = L; kt < NK; ++kt) BSR_QS16K_SLICE(t, kt);
    }
    if (my_rt) {
        // the last half period: group A's last epilogue, group B's last L slices
        if (grp == 0) {
            bool stored = false;
            BSR_QS16K_EPILOGUE(uA, stored);
            if (stored) wait_vm0();
        }
#pragma unroll
        for (int kt = 0; kt < L; ++kt) BSR_QS16K_SLICE(my_rt, kt);
    }
#undef BSR_QS16K_SLICE
    bool stored = false;
    if (grp == 1 && my_rt) BSR_QS16K_EPILOGUE(uB, stored);  // group B's last tile
    (void)stored;
#undef BSR_QS16K_EPILOGUE
#undef zero_acc
#undef mask_acc
#undef load_scales
#undef BSR_QS16K_DRAIN
    wait_vm0();
    wave_lds_order();
    flush_keys();
}

}  // namespace bsrlab
