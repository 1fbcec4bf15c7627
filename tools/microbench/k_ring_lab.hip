// k_ring_lab.hip -- TOOLING: the barrier-free LDS-ring filter (k_filter_ring, measured slower
// than the barrier kernels: profiles/r02c_*) and its ablation variant k_lab_ring (knobs and
// ring geometry), for tools/microbench/ring_ab.  Included after the product k_filter.hip.
namespace bsrlab {
using namespace bsr;

constexpr int kRgRows = 128;                // corpus rows per tile
constexpr int kRgSlots = 12;                // S: ring slots (8 KiB each)
constexpr int kRgAhead = 8;                 // A: slices a wave's DMA runs ahead of its reads
constexpr int kRgConfirm = 4;               // C: a DMA's landing is confirmed C slices after issue
constexpr int kRgSlot = kRgRows * kSliceB;  // 8 KiB
constexpr int kRgLaneCap = 12;              // candidate ring entries per lane
static_assert(kRgSlots >= kRgAhead + 2 && kRgAhead > kRgConfirm && kRgConfirm >= 1, "ring geometry");

// the ring's flag words: volatile LDS (ds_read / ds_write, counted in lgkmcnt only)
typedef __attribute__((address_space(3))) volatile uint32_t lds_flag_t;

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <bool EMIT, int NK, int S = 12, int A = 8, int C = 4, int VAR = 0>
__global__ __launch_bounds__(512, 1) void k_lab_ring(GemmArgs p) {
    constexpr int BM = kRgRows, BN = kFilterTile, NT = 512;
    static_assert(S >= A + 2 && A > C && C >= 1, "ring");
    static_assert(NK >= 1 && NK <= 12, "rows of 1..12 slices of 64 bytes");
    constexpr int EM_BYTES = EMIT ? NT * kRgLaneCap * 8 : 0;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[S * kRgSlot + EM_BYTES + 64];
    lds_flag_t* flg = (lds_flag_t*)(lds + S * kRgSlot + EM_BYTES);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint64_t* lkeys = reinterpret_cast<uint64_t*>(lds + S * kRgSlot) + tid;
    uint32_t ecnt = 0;

    // Grid: per XCD, G row groups x n_qt query tiles; a row tile's readers share the XCD's L2.
    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * NK;
    if (!J) return;  // uniform over the workgroup

    // The wave's query fragments, all K: fb[s] = query qt*256 + 32w + (lane & 31), bytes
    // 32s + 16(lane >> 5) .. +15 (the MFMA B layout); its threshold and scale.
    const uint32_t q = qt * BN + w * 32 + (lane & 31);
    i32x4_t fb[2 * NK];
    {
        const uint8_t* src = p.B + (uint64_t)q * p.row_bytes + 16 * (lane >> 5);
#pragma unroll
        for (int s2 = 0; s2 < 2 * NK; ++s2) fb[s2] = *reinterpret_cast<const i32x4_t*>(src + 32 * s2);
    }
    const float tau = EMIT ? p.tau[q] : 0.0f;
    const float sbq = p.b_scale[q];
    // the lane's candidate ring to its query's global list (a count past cap marks the list
    // overflowed: not certified from it)
    auto flush_ring = [&]() {
        if (ecnt) {
            const uint32_t gp = atomicAdd(p.cnt + q, ecnt);
            for (uint32_t i = 0; i < ecnt; ++i)
                if (gp + i < p.cap) p.cand[(uint64_t)q * p.cap + gp + i] = lkeys[i * NT];
        }
        ecnt = 0;
    };

    // LDS-DMA: wave w fills rows 16w .. 16w+15 of each slice (1 KiB per instruction).
    const uint32_t lrow = w * 16 + (lane >> 2);
    const uint32_t lchunk = ((lane & 3) ^ ((lrow >> 2) & 3)) * 16;
    uint32_t aoff_dma = lrow * (uint32_t)p.a_stride + lchunk;
    uint32_t iss_ti = 0, iss_kt = 0;
    __amdgpu_buffer_rsrc_t rsrc_a;
    auto set_issue_tile = [&]() {
        const uint32_t rt = g0 + iss_ti * RG;
        rsrc_a = __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (uint64_t)rt * BM * p.a_stride), 0,
                                                   BM * (uint32_t)p.a_stride, 0x00020000);
        if (!EMIT) {  // sample pass: tail rows read the last valid row
            const uint32_t r = rt * BM + lrow < p.n_rows ? lrow : p.n_rows - 1 - rt * BM;
            aoff_dma = r * (uint32_t)p.a_stride + lchunk;
        }
    };
    // this wave's part of the next slice of the stream (past the end: the last tile again)
    uint32_t iss = 0;
    auto issue_dma = [&]() {
        uint8_t* la = lds + (iss % S) * kRgSlot + wu * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)la, 16, aoff_dma, iss_kt * kSliceB, 0, 0);
        ++iss;
        if (++iss_kt == NK) {
            iss_kt = 0;
            ++iss_ti;
            if (iss_ti < my_rt) set_issue_tile();
        }
    };

    int aoff[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int row = m * 32 + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int lc = 2 * kk + (lane >> 5);
            aoff[m][kk] = row * kSliceB + ((lc ^ ((row >> 2) & 3)) * 16);
        }
    }
    i32x4_t fa[4][2];
    auto read_frag = [&](uint32_t jj, int m, int kk) {
        fa[m][kk] = *reinterpret_cast<const i32x4_t*>(lds + ((VAR & 4) ? 0 : jj % S) * kRgSlot + aoff[m][kk]);
    };

    // Prologue: flags zeroed; slices 0..A-1 issued; slices 0..A-C-1 of this wave landed
    // (published); the barrier makes every wave's slice 0 visible; slice 0's fragments read.
    if (tid < 16) flg[tid] = 0;
    set_issue_tile();
    __syncthreads();
#pragma unroll
    for (int i = 0; i < A; ++i) issue_dma();
    vm_wait<C>();
    if (lane == 0) flg[w] = A - C;
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 4; ++m) { read_frag(0, m, 0); read_frag(0, m, 1); }
    asm volatile("" ::: "memory");
    if (lane == 0) flg[8 + w] = 1;

    if ((VAR & 16) && w >= 4) __builtin_amdgcn_s_setprio(1);
    i32x16_t acc[4];
    for (uint32_t t = 0; t < my_rt; ++t) {
        const uint32_t rt = g0 + t * RG;
        float4 scv = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) {
            const uint32_t jj = t * NK + kt;
            __builtin_amdgcn_sched_barrier(0);
            // (1) publish the landing of this wave's DMA issued C slices ago (slice jj-C+A).
            // Younger VMEM ops: the C-1 DMAs since, and the tile's scale load when it was
            // issued in between (counted only when certain: more younger ops than counted
            // only make the wait stricter).
            if constexpr (!(VAR & 1)) {
                if constexpr (EMIT) {
                    if (kt >= 1 && kt <= C - 1) vm_wait<C>();
                    else vm_wait<C - 1>();
                } else {
                    vm_wait<C - 1>();
                }
            }
            if (!(VAR & 32) && lane == 0) flg[w] = jj - C + A + 1;
            // (2) ring check, read now, tested after the first MFMAs: every wave's part of
            // slice jj+1 landed; every wave done reading the slot of slice jj+A-S.
            const uint32_t t_land = jj + 2, t_prog = jj + A + 1 > S ? jj + A + 1 - S : 0u;
            const uint32_t thr = t_land + ((uint32_t)(lane >> 3) & 1u) * (t_prog - t_land);
            uint32_t fv = flg[lane & 15];
            // (3) the tile's block scales (a plain load, consumed in the epilogue)
            if (EMIT && kt == 0) scv = *reinterpret_cast<const float4*>(p.a_scale + (uint64_t)rt * (BM / kQuantBlock));
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    if (kt == 0 && kk == 0) {
                        const i32x16_t z = {};
                        acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[m][kk], fb[2 * kt + kk], z, 0, 0, 0);
                    } else {
                        acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[m][kk], fb[2 * kt + kk], acc[m], 0, 0, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (kk == 0 && m == 1) {
                        // the check: spin while any wave lags (rare), then the DMA of slice jj+A
                        while (!(VAR & 2) && __ballot(fv < thr)) {
                            __builtin_amdgcn_s_sleep(1);
                            fv = flg[lane & 15];
                        }
                        asm volatile("" ::: "memory");
                        if constexpr (!(VAR & 4)) issue_dma();
                        // the fragments of slice jj+1 for m = 0, 1 (their MFMAs have issued)
                        read_frag(jj + 1, 0, 0);
                        read_frag(jj + 1, 1, 0);
                    } else if (!(kk == 0 && m == 0)) {
                        read_frag(jj + 1, m, kk);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            // (4) every fragment of slice jj+1 read: publish the progress
            asm volatile("" ::: "memory");
            if (!(VAR & 32) && lane == 0) flg[8 + w] = jj + 2;
        }
        if constexpr ((VAR & 8) != 0) {
#pragma unroll
            for (int m = 0; m < 4; ++m) asm volatile("" ::"v"(acc[m][0]));
            continue;
        }
        // ---- epilogue of tile t
        const float sc[4] = {scv.x, scv.y, scv.z, scv.w};
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint32_t rbase = rt * BM + m * 32 + 4 * (lane >> 5);
            if constexpr (!EMIT) {
                float v[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    uint32_t tr = rbase + (r & 3) + 8 * (r >> 2);
                    tr = tr < p.n_rows ? tr : p.n_rows - 1;
                    v[r] = ((float)acc[m][r] * p.a_scale[tr / p.a_scale_rows]) * sbq;
                }
                float* srow = p.S + (uint64_t)q * p.s_ld;
                if (!p.s_compact) {
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        *reinterpret_cast<float4*>(srow + rbase + 8 * g) =
                            make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
                } else {
                    float mx = v[0];
#pragma unroll
                    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, v[r]);
                    mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
                    if (lane < 32) srow[(rt * BM + m * 32) / 32] = mx;
                }
            } else {
                auto score = [&](int v) -> float { return ((float)v * sc[m]) * sbq; };
                int gm[4];
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    gm[g] = max(max(acc[m][4 * g], acc[m][4 * g + 1]), max(acc[m][4 * g + 2], acc[m][4 * g + 3]));
                const int mxv = max(max(gm[0], gm[1]), max(gm[2], gm[3]));
                if (__ballot(score(mxv) >= tau)) {
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        if (!__ballot(score(gm[g]) >= tau)) continue;
                        // room for this group's 4 rows in every lane's ring (rarely not)
                        if (__ballot(ecnt > (uint32_t)(kRgLaneCap - 4))) {
                            flush_ring();
                            vm_wait<0>();  // (keeps the counted waits exact)
                        }
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const float v = score(acc[m][4 * g + i]);
                            const uint32_t row = rbase + 8 * g + i;
                            if (v >= tau && row < p.n_rows) {
                                lkeys[ecnt * NT] = score_key(v, row);
                                ++ecnt;
                            }
                        }
                    }
                }
            }
        }
        if constexpr (!EMIT) vm_wait<0>();  // the sample stores / scale loads (keeps the waits exact)
    }
    vm_wait<0>();  // the stream's trailing DMAs land before the workgroup ends
    if constexpr (EMIT) flush_ring();
}


// ------------------------------------------------------------------------------------
// Query-stationary int8 filter on a barrier-free LDS ring (the int8 default for rows of
// NK <= 12 slices of 64 bytes, i.e. dims up to 768).
//
// One 512-thread workgroup per CU, 8 waves (two per SIMD).  Wave w keeps the int8 fragments
// of its 32 queries (qt*256 + 32w ..) for ALL of K in registers for the workgroup's life, so
// only corpus rows move: 128-row tiles stream through a ring of kRgSlots LDS slots, one
// 64-byte K slice (8 KiB) per slot, filled by LDS-DMA (buffer_load ... lds, 1 KiB per
// wave per slice, XOR-swizzled on the source chunk so every ds_read_b128 fragment read is
// conflict-free).  Per slice a wave reads 8 KiB of A fragments and issues 8
// v_mfma_i32_32x32x32_i8 (128 rows x 32 queries x 64 bytes).
//
// No s_barrier in the loop: the waves synchronise through 16 LDS words instead,
//   land[w]  slices whose wave-w part has landed (wave w publishes slice jj-C+A at its
//            slice jj, after a counted s_waitcnt on its own DMA issued C slices earlier),
//   prog[w]  slices whose fragments wave w has read (published right after the reads; a
//            wave's LDS ops execute in order, so the slot's bytes have been read by then).
// Before reading the fragments of slice jj+1 a wave needs every land[] >= jj+2; before its
// DMA of slice jj+A refills the slot of slice jj+A-S it needs every prog[] >= jj+A-S+1.
// One ds_read per lane (lanes 0-7 land, 8-15 prog), issued before the slice's first MFMAs
// and tested after them, so the check costs no latency unless a wave runs ahead.  Waves
// therefore drift up to min(A-1-C, S-A-1) slices apart instead of meeting at a barrier:
// a wave in its epilogue, its DMA issue or a landing wait leaves its SIMD partner issuing
// MFMAs.  The slowest wave never waits (every flag it needs was published by a wave at or
// ahead of it), so the ring cannot deadlock.
// The DMA stream is steady: exactly one DMA per wave per slice (past the shard's last
// slice the last tile is re-read into slots nobody reads again, subject to the same free
// check), so every counted wait is a compile-time constant; it drains before exit.
// Epilogue (EMIT) per 32x32 block: the block maximum against the query's threshold (one
// ballot), then only the groups of 4 rows whose maximum passes are expanded; passing
// (score, row) keys go to a private per-lane LDS ring (entry e of thread t at [e][t]),
// flushed to the per-query global lists at the end or when a group could overfill it.
// SAMPLE: every tile row is one sampled corpus row; scores (or one maximum per 32 sampled
// rows) go to S.
// ------------------------------------------------------------------------------------
template <bool EMIT, int NK>
__global__ __launch_bounds__(512, 1) void k_filter_ring(GemmArgs p) {
    constexpr int S = kRgSlots, A = kRgAhead, C = kRgConfirm;
    constexpr int BM = kRgRows, BN = kFilterTile, NT = 512;
    static_assert(NK >= 1 && NK <= 12, "rows of 1..12 slices of 64 bytes");
    constexpr int EM_BYTES = EMIT ? NT * kRgLaneCap * 8 : 0;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[S * kRgSlot + EM_BYTES + 64];
    lds_flag_t* flg = (lds_flag_t*)(lds + S * kRgSlot + EM_BYTES);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint64_t* lkeys = reinterpret_cast<uint64_t*>(lds + S * kRgSlot) + tid;
    uint32_t ecnt = 0;

    // Grid: per XCD, G row groups x n_qt query tiles; a row tile's readers share the XCD's L2.
    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * NK;
    if (!J) return;  // uniform over the workgroup

    // The wave's query fragments, all K: fb[s] = query qt*256 + 32w + (lane & 31), bytes
    // 32s + 16(lane >> 5) .. +15 (the MFMA B layout); its threshold and scale.
    const uint32_t q = qt * BN + w * 32 + (lane & 31);
    i32x4_t fb[2 * NK];
    {
        const uint8_t* src = p.B + (uint64_t)q * p.row_bytes + 16 * (lane >> 5);
#pragma unroll
        for (int s2 = 0; s2 < 2 * NK; ++s2) fb[s2] = *reinterpret_cast<const i32x4_t*>(src + 32 * s2);
    }
    const float tau = EMIT ? p.tau[q] : 0.0f;
    const float sbq = p.b_scale[q];
    // the lane's candidate ring to its query's global list (a count past cap marks the list
    // overflowed: not certified from it)
    auto flush_ring = [&]() {
        if (ecnt) {
            const uint32_t gp = atomicAdd(p.cnt + q, ecnt);
            for (uint32_t i = 0; i < ecnt; ++i)
                if (gp + i < p.cap) p.cand[(uint64_t)q * p.cap + gp + i] = lkeys[i * NT];
        }
        ecnt = 0;
    };

    // LDS-DMA: wave w fills rows 16w .. 16w+15 of each slice (1 KiB per instruction).
    const uint32_t lrow = w * 16 + (lane >> 2);
    const uint32_t lchunk = ((lane & 3) ^ ((lrow >> 2) & 3)) * 16;
    uint32_t aoff_dma = lrow * (uint32_t)p.a_stride + lchunk;
    uint32_t iss_ti = 0, iss_kt = 0;
    __amdgpu_buffer_rsrc_t rsrc_a;
    auto set_issue_tile = [&]() {
        const uint32_t rt = g0 + iss_ti * RG;
        rsrc_a = __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (uint64_t)rt * BM * p.a_stride), 0,
                                                   BM * (uint32_t)p.a_stride, 0x00020000);
        if (!EMIT) {  // sample pass: tail rows read the last valid row
            const uint32_t r = rt * BM + lrow < p.n_rows ? lrow : p.n_rows - 1 - rt * BM;
            aoff_dma = r * (uint32_t)p.a_stride + lchunk;
        }
    };
    // this wave's part of the next slice of the stream (past the end: the last tile again)
    uint32_t iss = 0;
    auto issue_dma = [&]() {
        uint8_t* la = lds + (iss % S) * kRgSlot + wu * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)la, 16, aoff_dma, iss_kt * kSliceB, 0, 0);
        ++iss;
        if (++iss_kt == NK) {
            iss_kt = 0;
            ++iss_ti;
            if (iss_ti < my_rt) set_issue_tile();
        }
    };

    int aoff[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int row = m * 32 + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int lc = 2 * kk + (lane >> 5);
            aoff[m][kk] = row * kSliceB + ((lc ^ ((row >> 2) & 3)) * 16);
        }
    }
    i32x4_t fa[4][2];
    auto read_frag = [&](uint32_t jj, int m, int kk) {
        fa[m][kk] = *reinterpret_cast<const i32x4_t*>(lds + (jj % S) * kRgSlot + aoff[m][kk]);
    };

    // Prologue: flags zeroed; slices 0..A-1 issued; slices 0..A-C-1 of this wave landed
    // (published); the barrier makes every wave's slice 0 visible; slice 0's fragments read.
    if (tid < 16) flg[tid] = 0;
    set_issue_tile();
    __syncthreads();
#pragma unroll
    for (int i = 0; i < A; ++i) issue_dma();
    vm_wait<C>();
    if (lane == 0) flg[w] = A - C;
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 4; ++m) { read_frag(0, m, 0); read_frag(0, m, 1); }
    asm volatile("" ::: "memory");
    if (lane == 0) flg[8 + w] = 1;

    i32x16_t acc[4];
    for (uint32_t t = 0; t < my_rt; ++t) {
        const uint32_t rt = g0 + t * RG;
        float4 scv = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) {
            const uint32_t jj = t * NK + kt;
            __builtin_amdgcn_sched_barrier(0);
            // (1) publish the landing of this wave's DMA issued C slices ago (slice jj-C+A).
            // Younger VMEM ops: the C-1 DMAs since, and the tile's scale load when it was
            // issued in between (counted only when certain: more younger ops than counted
            // only make the wait stricter).
            if constexpr (EMIT) {
                if (kt >= 1 && kt <= C - 1) vm_wait<C>();
                else vm_wait<C - 1>();
            } else {
                vm_wait<C - 1>();
            }
            if (lane == 0) flg[w] = jj - C + A + 1;
            // (2) ring check, read now, tested after the first MFMAs: every wave's part of
            // slice jj+1 landed; every wave done reading the slot of slice jj+A-S.
            const uint32_t t_land = jj + 2, t_prog = jj + A + 1 > S ? jj + A + 1 - S : 0u;
            const uint32_t thr = t_land + ((uint32_t)(lane >> 3) & 1u) * (t_prog - t_land);
            uint32_t fv = flg[lane & 15];
            // (3) the tile's block scales (a plain load, consumed in the epilogue)
            if (EMIT && kt == 0) scv = *reinterpret_cast<const float4*>(p.a_scale + (uint64_t)rt * (BM / kQuantBlock));
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    if (kt == 0 && kk == 0) {
                        const i32x16_t z = {};
                        acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[m][kk], fb[2 * kt + kk], z, 0, 0, 0);
                    } else {
                        acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[m][kk], fb[2 * kt + kk], acc[m], 0, 0, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (kk == 0 && m == 1) {
                        // the check: spin while any wave lags (rare), then the DMA of slice jj+A
                        while (__ballot(fv < thr)) {
                            __builtin_amdgcn_s_sleep(1);
                            fv = flg[lane & 15];
                        }
                        asm volatile("" ::: "memory");
                        issue_dma();
                        // the fragments of slice jj+1 for m = 0, 1 (their MFMAs have issued)
                        read_frag(jj + 1, 0, 0);
                        read_frag(jj + 1, 1, 0);
                    } else if (!(kk == 0 && m == 0)) {
                        read_frag(jj + 1, m, kk);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            // (4) every fragment of slice jj+1 read: publish the progress
            asm volatile("" ::: "memory");
            if (lane == 0) flg[8 + w] = jj + 2;
        }
        // ---- epilogue of tile t
        const float sc[4] = {scv.x, scv.y, scv.z, scv.w};
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint32_t rbase = rt * BM + m * 32 + 4 * (lane >> 5);
            if constexpr (!EMIT) {
                float v[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    uint32_t tr = rbase + (r & 3) + 8 * (r >> 2);
                    tr = tr < p.n_rows ? tr : p.n_rows - 1;
                    v[r] = ((float)acc[m][r] * p.a_scale[tr / p.a_scale_rows]) * sbq;
                }
                float* srow = p.S + (uint64_t)q * p.s_ld;
                if (!p.s_compact) {
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        *reinterpret_cast<float4*>(srow + rbase + 8 * g) =
                            make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
                } else {
                    float mx = v[0];
#pragma unroll
                    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, v[r]);
                    mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
                    if (lane < 32) srow[(rt * BM + m * 32) / 32] = mx;
                }
            } else {
                auto score = [&](int v) -> float { return ((float)v * sc[m]) * sbq; };
                int gm[4];
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    gm[g] = max(max(acc[m][4 * g], acc[m][4 * g + 1]), max(acc[m][4 * g + 2], acc[m][4 * g + 3]));
                const int mxv = max(max(gm[0], gm[1]), max(gm[2], gm[3]));
                if (__ballot(score(mxv) >= tau)) {
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        if (!__ballot(score(gm[g]) >= tau)) continue;
                        // room for this group's 4 rows in every lane's ring (rarely not)
                        if (__ballot(ecnt > (uint32_t)(kRgLaneCap - 4))) {
                            flush_ring();
                            vm_wait<0>();  // (keeps the counted waits exact)
                        }
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const float v = score(acc[m][4 * g + i]);
                            const uint32_t row = rbase + 8 * g + i;
                            if (v >= tau && row < p.n_rows) {
                                lkeys[ecnt * NT] = score_key(v, row);
                                ++ecnt;
                            }
                        }
                    }
                }
            }
        }
        if constexpr (!EMIT) vm_wait<0>();  // the sample stores / scale loads (keeps the waits exact)
    }
    vm_wait<0>();  // the stream's trailing DMAs land before the workgroup ends
    if constexpr (EMIT) flush_ring();
}

}  // namespace bsrlab
