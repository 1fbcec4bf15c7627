// k_filter_lab.hip -- TOOLING: the MFMA filter with its ablation knobs (VAR / STAG / PRIO /
// EPI / STAMP), included by tools/microbench/ring_ab; the product kernel is
// better-search-rag-rust_amd/csrc/k_filter.hip (no knobs).  Round-1 snapshot.
//
// The filter scores every (corpus row, query) pair approximately on the matrix cores and
// keeps the pairs that can belong to a query's top k.  It never produces a returned
// distance: the candidates are rescored with the reference's exact arithmetic
// (k_exact.hip) and the final list is certified against the filter's error bound.
//
// Two operand types share one kernel (template Op):
//   OpI8   int8 rows (per 32-row block scale) x int8 queries (per query scale) on
//          v_mfma_i32_32x32x32_i8; the integer dot product is exact, the score is
//          ((float)I * s_row_block) * s_query.
//   OpBF16 bf16(a/|a|) x bf16(b/|b|) on v_mfma_f32_32x32x16_bf16.
// Both move 64 bytes of K per row per slice, so the tiling, the LDS ring and the issue
// schedule are identical; an int8 slice carries twice the K of a bf16 slice.
#include "bsr_device.hpp"
#include "kernels.hpp"

#include <hip/hip_ext.h>

#include <math.h>

#include <algorithm>
#include <type_traits>

namespace bsrlab {
using namespace bsr;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;
typedef __attribute__((ext_vector_type(16))) int i32x16_t;
typedef __attribute__((address_space(3))) void lds_void_t;

struct OpBF16 {
    using frag_t = bf16x8_t;
    using acc_t = f32x16_t;
    static constexpr bool kInt = false;
    __device__ __forceinline__ static acc_t mfma(const frag_t& a, const frag_t& b, const acc_t& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};
struct OpI8 {
    using frag_t = i32x4_t;
    using acc_t = i32x16_t;
    static constexpr bool kInt = true;
    __device__ __forceinline__ static acc_t mfma(const frag_t& a, const frag_t& b, const acc_t& c) {
        return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    }
};

constexpr int kSlots = 4;     // LDS ring slots (3 slices in flight + the one being read)
constexpr int kSliceB = 64;   // bytes of K per row per slice
constexpr int kWCap = 256;    // candidate buffer entries per wave (one is the counter)
constexpr int kThreads = 512; // 8 waves: 2 (rows) x 4 (queries)

__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Mid-slice barrier: the slice the next fragment reads come from has landed for every
// wave (counted vmcnt: the N youngest LDS-DMA stay in flight), and this wave's fragment
// reads are complete (the slot they read may be refilled after the barrier).
template <int N>
__device__ __forceinline__ void mid_barrier() {
    if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ------------------------------------------------------------------------------------
// The filter.  Persistent workgroups (512 threads, waves 2 x 4, each wave 128 rows x 64
// queries = 4 x 2 blocks of 32 x 32), each owning one 256-query tile for its life
// (thresholds and query scales in registers) and walking 256-row corpus tiles g, g+RG, ...;
// the n_qt workgroups that share a row tile share an XCD (blockIdx % 8), so each row tile
// leaves HBM once per XCD.  Operands arrive by global_load_lds_dwordx4 into a 4-slot ring
// of 64-byte K slices (32 KiB per slot, 3 slices in flight), XOR-swizzled on the source
// address so that every ds_read_b128 fragment read is conflict-free.  Issue order per
// slice j (F0/F1 = fragment register sets of the two K sub-steps):
//   [F1 <- ds_read(j, kk=1)] 4 MFMA(F0) dma(j+3,A0) 4 MFMA(F0) dma(j+3,A1)
//   s_waitcnt lgkmcnt(0) vmcnt(N) ; s_barrier          <- slice j+1 landed everywhere
//   [F0 <- ds_read(j+1, kk=0)] 4 MFMA(F1) dma(j+3,B0) 4 MFMA(F1) dma(j+3,B1)
// The barrier sits mid-slice: the slot a DMA overwrites (slice j-1) was last read before
// the previous barrier.  sched_barrier(0) pins the placement against the scheduler.
//
// Epilogue per 32x32 block (EMIT): the block maximum (over four group maxima of 4 rows)
// against the query's threshold tau (one ballot); in a block that passes, only the groups
// whose maximum passes are expanded, and their passing (lane, register) pairs append
// (score, row) keys to a per-wave LDS buffer (inline-asm ds_add_rtn; hipcc would drain
// vmcnt before a plain LDS atomic), flushed to the per-query global lists at the end.
// All eight waves reach the epilogue together (the barriers keep them in step), so its
// vector work is not hidden behind MFMAs: ~29% of the blocks pass at a realistic tau.  int8: the block scales of
// the current tile are fetched into this wave's LDS words by a 4-lane LDS-DMA issued with
// the tile's first slice and covered by the counted waits two slices later.
// SAMPLE (!EMIT): every tile row is one sampled corpus row; the scores go to S, either
// all of them (s_compact == 0) or one maximum per 32 sampled rows (s_compact == 1).
//
// The first MFMA group of every tile takes a zero C operand, so the accumulators are never
// cleared by vector moves (all eight waves reach the epilogue together, so anything done
// there is not hidden behind another wave's MFMAs).
//
// VAR (tooling, tools/microbench): 1 = no LDS-DMA in the loop (compute ceiling),
// 3 = LDS-DMA, waits and barriers only (operand-feed ceiling), 4 = A always the same tile,
// 5 = no epilogue (accumulators kept live), 6 = neither LDS-DMA nor epilogue.
// STAMP (tooling): thread 0 of each workgroup writes its s_memtime / s_memrealtime deltas
// to S (in-kernel clock, MI355X_MICROARCH.md 'DVFS give-back' item 6).
// EPI (tooling): 0 = the previous epilogue (per-lane mask over all 16 registers of a block
// whose maximum passes, explicit clears), 1 = that epilogue with zero-C first MFMAs.
// ------------------------------------------------------------------------------------
template <class Op, bool EMIT, int VAR = 0, bool STAG = false, bool PRIO = false, int EPI = 2, bool STAMP = false>
__global__ __launch_bounds__(kThreads, 2) void k_filter(GemmArgs p) {
    constexpr bool kNoDMA = VAR == 1 || VAR == 6, kNoMath = VAR == 3 || VAR == 4, kNoEpi = VAR == 5 || VAR == 6;
    uint64_t t0 = 0, r0 = 0;
    if (STAMP) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    using frag_t = typename Op::frag_t;
    using acc_t = typename Op::acc_t;
    constexpr int BM = kFilterTile, BN = kFilterTile;
    constexpr int A_BYTES = BM * kSliceB, B_BYTES = BN * kSliceB;
    constexpr int SLOT = A_BYTES + B_BYTES;
    constexpr int EM_BYTES = EMIT ? 8 * kWCap * 12 : 0;
    constexpr bool kScaleDMA = EMIT && Op::kInt;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[kSlots * SLOT + EM_BYTES + (kScaleDMA ? 8 * 16 : 0)];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 2, wc = w & 3;
    uint64_t* ekeys = reinterpret_cast<uint64_t*>(lds + kSlots * SLOT) + w * kWCap;
    uint32_t* eq = reinterpret_cast<uint32_t*>(lds + kSlots * SLOT + 8 * kWCap * 8) + w * kWCap;
    float* lsc = reinterpret_cast<float*>(lds + kSlots * SLOT + EM_BYTES) + w * 4;
    // per-wave append counter: the last q slot of the wave's region (capacity kWCap-1)
    const uint32_t ecnt_addr = (uint32_t)(uintptr_t)(eq + kWCap - 1);
    if (EMIT && lane == 0) eq[kWCap - 1] = 0;

    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const uint32_t nk = p.row_bytes / kSliceB;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * nk;

    // LDS-DMA by buffer loads: per-lane byte offsets (VGPR) fixed for the kernel, the K
    // slice in the scalar soffset, the row tile in the descriptor base, the LDS slot in M0
    // (from a provably wave-uniform wave id), so one DMA costs ~2 instructions.
    const uint32_t wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint32_t lrow[2], lchunk[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        lrow[i] = (w * 2 + i) * 16 + (lane >> 2);
        lchunk[i] = (lane & 3) ^ ((lrow[i] >> 2) & 3);
    }
    const __amdgpu_buffer_rsrc_t rsrc_b =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.B, 0, p.n_qt * BN * p.row_bytes, 0x00020000);
    uint32_t boff_dma[2], aoff_dma[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        boff_dma[i] = (qt * BN + lrow[i]) * p.row_bytes + lchunk[i] * 16;
        aoff_dma[i] = lrow[i] * (uint32_t)p.a_stride + lchunk[i] * 16;
    }
    // DMA state of the slice being issued (slice jj+3), advanced incrementally.
    uint32_t iss_ti = 0, iss_kt = 0;
    __amdgpu_buffer_rsrc_t rsrc_a = rsrc_b;
    auto set_issue_tile = [&]() {
        const uint32_t rt = VAR == 4 ? g0 : g0 + iss_ti * RG;
        rsrc_a = __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (uint64_t)rt * BM * p.a_stride), 0,
                                                   BM * (uint32_t)p.a_stride, 0x00020000);
        if (!EMIT) {  // sample pass: tail rows read the last valid row
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint32_t r = rt * BM + lrow[i] < p.n_rows ? lrow[i] : p.n_rows - 1 - rt * BM;
                aoff_dma[i] = r * (uint32_t)p.a_stride + lchunk[i] * 16;
            }
        }
    };
    auto dma_a = [&](uint32_t jj, int i) {
        uint8_t* la = lds + (jj % kSlots) * SLOT + (wu * 2 + i) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)la, 16, aoff_dma[i], iss_kt * kSliceB, 0, 0);
    };
    auto dma_b = [&](uint32_t jj, int i) {
        uint8_t* lb = lds + (jj % kSlots) * SLOT + A_BYTES + (wu * 2 + i) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_b, (lds_void_t*)lb, 16, boff_dma[i], iss_kt * kSliceB, 0, 0);
    };
    auto issue_advance = [&]() {
        if (++iss_kt == nk) { iss_kt = 0; ++iss_ti; set_issue_tile(); }
    };

    int aoff[4][2], boff[2][2];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int row = wr * 128 + m * 32 + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int lc = 2 * kk + (lane >> 5);
            aoff[m][kk] = row * kSliceB + ((lc ^ ((row >> 2) & 3)) * 16);
        }
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int row = wc * 64 + n * 32 + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int lc = 2 * kk + (lane >> 5);
            boff[n][kk] = A_BYTES + row * kSliceB + ((lc ^ ((row >> 2) & 3)) * 16);
        }
    }
    float tau[2] = {0.0f, 0.0f}, sbq[2] = {1.0f, 1.0f};
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const uint32_t q = qt * BN + wc * 64 + n * 32 + (lane & 31);
        if (EMIT) tau[n] = p.tau[q];
        if (Op::kInt) sbq[n] = p.b_scale[q];
    }

    acc_t acc[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0;

    frag_t fa0[4], fb0[2], fa1[4], fb1[2];
    auto read_frags = [&](uint32_t jj, int kk, frag_t (&fa)[4], frag_t (&fb)[2]) {
        if constexpr (kNoMath) return;
        const uint8_t* base = lds + (kNoDMA ? 0 : jj % kSlots) * SLOT;
#pragma unroll
        for (int m = 0; m < 4; ++m) fa[m] = *reinterpret_cast<const frag_t*>(base + aoff[m][kk]);
#pragma unroll
        for (int n = 0; n < 2; ++n) fb[n] = *reinterpret_cast<const frag_t*>(base + boff[n][kk]);
    };
    auto mfma4 = [&](const frag_t (&fa)[4], const frag_t (&fb)[2], int half, bool first) {
        if constexpr (kNoMath) return;
        if (EPI >= 1 && first) {  // first K step of a tile: C = 0
            const acc_t z = {};
#pragma unroll
            for (int m = half * 2; m < half * 2 + 2; ++m)
#pragma unroll
                for (int n = 0; n < 2; ++n) acc[m][n] = Op::mfma(fa[m], fb[n], z);
        } else {
#pragma unroll
            for (int m = half * 2; m < half * 2 + 2; ++m)
#pragma unroll
                for (int n = 0; n < 2; ++n) acc[m][n] = Op::mfma(fa[m], fb[n], acc[m][n]);
        }
    };
    // The score of accumulator element v of block m (int8: exact integer dot, then the two
    // scale multiplies in this fixed order; the candidate keys use the same expression).
    auto score = [&](auto v, float sc_m, int n) -> float {
        if constexpr (Op::kInt) return ((float)v * sc_m) * sbq[n];
        else return v;
    };

    // PRIO: static priority for the second-dispatched half (waves 4-7, the arbitration
    // losers of every segment; MI355X_MICROARCH.md "Two waves per SIMD", item 4).
    if (PRIO && w >= 4) __builtin_amdgcn_s_setprio(1);
    // Prologue: slices 0..min(J,3)-1 issued; wait for slice 0; F0 <- (0, kk=0).
    set_issue_tile();
    const uint32_t pre = J < 3 ? J : 3;
    for (uint32_t jj = 0; jj < pre; ++jj) {
        dma_a(jj, 0); dma_a(jj, 1); dma_b(jj, 0); dma_b(jj, 1);
        issue_advance();
    }
    if (pre == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (pre == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (J) read_frags(0, 0, fa0, fb0);

    uint32_t ti = 0, kt = 0;
    for (uint32_t jj = 0; jj < J; ++jj) {
        const bool iss = !kNoDMA && jj + 3 < J;
        // ---- first half: kk = 0 MFMAs, kk = 1 reads, A-half DMA of slice jj+3.  The
        // reads go after the first MFMA group: hipcc puts a conservative lgkmcnt(0) in
        // front of an MFMA whose operands came from ds_read (it cannot see the barrier's
        // inline wait), which must not cover reads issued just before it.
        // STAG: the wr=1 waves (the SIMD partners of the wr=0 waves) issue each DMA before
        // the MFMA group instead of after it, so one partner's DMA issue overlaps the other
        // partner's MFMAs (the per-wave DMA count before each barrier is unchanged).
        const bool stag = STAG && wr == 1;
        if (stag && iss) dma_a(jj + 3, 0);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa0, fb0, 0, kt == 0);
        __builtin_amdgcn_sched_barrier(0);
        read_frags(jj, 1, fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        if (iss) { if (stag) dma_a(jj + 3, 1); else dma_a(jj + 3, 0); }
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa0, fb0, 1, kt == 0);
        __builtin_amdgcn_sched_barrier(0);
        if (!stag && iss) dma_a(jj + 3, 1);
        if constexpr (kScaleDMA) {
            // this wave's 4 block scales of the current tile (rows rt*256 + wr*128 + 32m);
            // younger than every slice DMA in flight, so covered two mid-barriers later
            if (kt == 0 && lane < 4) {
                const uint32_t blk = ((g0 + ti * RG) * BM + wr * 128) / kQuantBlock + lane;
                __builtin_amdgcn_global_load_lds((const void*)(p.a_scale + blk), (lds_void_t*)lsc, 4, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- mid-slice barrier: slice jj+1 has landed for every wave
        if (kNoDMA) {
            mid_barrier<8>();
        } else if (jj + 3 < J) {
            mid_barrier<6>();
        } else if (jj + 2 < J) {
            mid_barrier<4>();
        } else {
            mid_barrier<0>();
        }
        // ---- second half: kk = 1 MFMAs, next slice's kk = 0 reads, B-half DMA
        if (stag && iss) dma_b(jj + 3, 0);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa1, fb1, 0, false);
        __builtin_amdgcn_sched_barrier(0);
        if (jj + 1 < J) read_frags(jj + 1, 0, fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        if (iss) { if (stag) dma_b(jj + 3, 1); else dma_b(jj + 3, 0); }
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa1, fb1, 1, false);
        __builtin_amdgcn_sched_barrier(0);
        if (!stag && iss) dma_b(jj + 3, 1);
        if (iss) issue_advance();
        __builtin_amdgcn_sched_barrier(0);

        if (kNoEpi && kt == nk - 1) {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int n = 0; n < 2; ++n) asm volatile("" ::"v"(acc[m][n][0]));
            kt = 0;
            ++ti;
        } else if (kt == nk - 1) {
            const uint32_t rt = g0 + ti * RG;
            bool stored = false;
            float sc[4] = {1.0f, 1.0f, 1.0f, 1.0f};
            if constexpr (kScaleDMA) {
                if (nk < 3) wait_vm0();  // fewer than two barriers since the scale DMA
#pragma unroll
                for (int m = 0; m < 4; ++m) sc[m] = lsc[m];
            }
#pragma unroll
            for (int m = 0; m < 4; ++m) {
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    const uint32_t ql = wc * 64 + n * 32 + (lane & 31);
                    const uint32_t rbase = rt * BM + wr * 128 + m * 32 + 4 * (lane >> 5);
                    if constexpr (!EMIT) {
                        // sample scores: tile row r is corpus row r * a_row_mult
                        float v[16];
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            float s_r = 1.0f;
                            if constexpr (Op::kInt) {
                                uint32_t tr = rbase + (r & 3) + 8 * (r >> 2);
                                tr = tr < p.n_rows ? tr : p.n_rows - 1;
                                s_r = p.a_scale[tr / p.a_scale_rows];
                            }
                            v[r] = score(acc[m][n][r], s_r, n);
                        }
                        float* srow = p.S + (uint64_t)(qt * BN + ql) * p.s_ld;
                        if (!p.s_compact) {  // full: every sampled row
#pragma unroll
                            for (int g = 0; g < 4; ++g)
                                *reinterpret_cast<float4*>(srow + rbase + 8 * g) =
                                    make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
                        } else {  // compact: one maximum per 32 sampled rows
                            float mx = v[0];
#pragma unroll
                            for (int r = 1; r < 16; ++r) mx = fmaxf(mx, v[r]);
                            mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
                            if (lane < 32) srow[(rt * BM + wr * 128 + m * 32) / 32] = mx;
                        }
                        stored = true;
                    } else {
                        // append (score, row) to the wave's LDS buffer (inline-asm ds_add_rtn:
                        // hipcc would drain vmcnt before a plain LDS atomic)
                        auto emit = [&](float v, uint32_t row) {
                            uint32_t pos;
                            asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
                                         : "=v"(pos) : "v"(ecnt_addr), "v"(1u) : "memory");
                            if (pos < (uint32_t)(kWCap - 1)) {
                                ekeys[pos] = score_key(v, row);
                                eq[pos] = ql;
                            } else {  // wave buffer full: straight to the global list
                                const uint32_t q = qt * BN + ql;
                                const uint32_t gp = atomicAdd(p.cnt + q, 1u);
                                if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = score_key(v, row);
                                stored = true;
                            }
                        };
                        // group maxima: group g = registers 4g..4g+3 = rows rbase + 8g + 0..3
                        std::remove_reference_t<decltype(acc[m][n][0])> gm[4];
#pragma unroll
                        for (int g = 0; g < 4; ++g) {
                            auto x = acc[m][n][4 * g], y = acc[m][n][4 * g + 2];
                            x = x > acc[m][n][4 * g + 1] ? x : acc[m][n][4 * g + 1];
                            y = y > acc[m][n][4 * g + 3] ? y : acc[m][n][4 * g + 3];
                            gm[g] = x > y ? x : y;
                        }
                        auto mxv = gm[0] > gm[1] ? gm[0] : gm[1];
                        mxv = mxv > gm[2] ? mxv : gm[2];
                        mxv = mxv > gm[3] ? mxv : gm[3];
                        if (EPI == 0) {
                            // (the previous epilogue: per-lane mask over 16 registers)
                            if (__ballot(score(mxv, sc[m], n) >= tau[n])) {
                                uint32_t mask = 0;
#pragma unroll
                                for (int r = 0; r < 16; ++r)
                                    mask |= (score(acc[m][n][r], sc[m], n) >= tau[n]) ? (1u << r) : 0u;
                                while (mask) {
                                    const int r = __builtin_ctz(mask);
                                    mask &= mask - 1;
                                    const uint32_t row = rbase + (r & 3) + 8 * (r >> 2);
                                    if (row >= p.n_rows) continue;
                                    auto av = acc[m][n][0];
#pragma unroll
                                    for (int rr = 1; rr < 16; ++rr) av = (rr == r) ? acc[m][n][rr] : av;
                                    emit(score(av, sc[m], n), row);
                                }
                                stored = __ballot(stored) != 0;
                            }
                        } else if (__ballot(score(mxv, sc[m], n) >= tau[n])) {
                            // hierarchical: only groups whose maximum passes are expanded
#pragma unroll
                            for (int g = 0; g < 4; ++g) {
                                if (!__ballot(score(gm[g], sc[m], n) >= tau[n])) continue;
#pragma unroll
                                for (int i = 0; i < 4; ++i) {
                                    const float v = score(acc[m][n][4 * g + i], sc[m], n);
                                    const uint32_t row = rbase + 8 * g + i;
                                    if (v >= tau[n] && row < p.n_rows) emit(v, row);
                                }
                            }
                            stored = __ballot(stored) != 0;
                        }
                    }
                    if (EPI == 0 || kNoMath) {  // (EPI >= 1: the next tile's first MFMAs take C = 0)
#pragma unroll
                        for (int r = 0; r < 16; ++r) acc[m][n][r] = 0;
                    }
                }
            }
            // global stores / atomics count in vmcnt: drain them so the counted waits stay exact
            if (stored) wait_vm0();
            kt = 0;
            ++ti;
        } else {
            ++kt;
        }
    }
    if constexpr (EMIT) {
        const uint32_t ecount = eq[kWCap - 1];
        const uint32_t ne = ecount < (uint32_t)(kWCap - 1) ? ecount : (uint32_t)(kWCap - 1);
        for (uint32_t i = lane; i < ne; i += kWave) {
            const uint32_t q = qt * BN + eq[i];
            const uint32_t gp = atomicAdd(p.cnt + q, 1u);
            if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = ekeys[i];
        }
    }
    if (STAMP && tid == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        reinterpret_cast<uint64_t*>(p.S)[2 * blockIdx.x] = t1 - t0;
        reinterpret_cast<uint64_t*>(p.S)[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// ------------------------------------------------------------------------------------
// Query-stationary int8 filter (the int8 default when a row is NK = 2..12 slices of 64
// bytes, i.e. dims up to 768): one workgroup per CU, four waves (one per SIMD, ~420
// VGPRs each).  Wave w keeps the int8 fragments of its 64 queries (qt*256 + 64w ..) for ALL
// of K in registers for the workgroup's life, so only corpus rows stream through LDS:
// 128-row tiles, one 64-byte K slice (8 KiB) per ring slot, 8 slots, 6 slices in flight,
// one barrier per slice.  Per slice a wave reads 8 KiB of A fragments and issues 16 MFMAs
// (128 rows x 64 queries x 64 bytes).  Per unit of work that is half the LDS-DMA bytes and
// two thirds of the LDS-read bytes of k_filter (which re-stages its 256-query B tile for
// every row tile and reads 192 B of fragments per k per 128x64 wave tile).
// The K loop is unrolled per tile (the query registers need static indices), so the first
// MFMAs of a tile take C = 0 without a branch.  Barrier wait: the slice read next has
// landed for every wave (counted vmcnt: the DMAs of younger slices, and the tile's scale
// load while it is younger, stay in flight) and this wave's fragment reads are complete.
// Epilogue as k_filter (EMIT: group-maximum expansion; SAMPLE: scores or maxima to S).
// ------------------------------------------------------------------------------------
constexpr int kQsRows = 128;               // corpus rows per tile
constexpr int kQsSlots = 8;                // LDS ring slots
constexpr int kQsAhead = 6;                // slices issued ahead of the one being consumed
constexpr int kQsSlot = kQsRows * kSliceB;  // 8 KiB
constexpr int kQsLaneCap = 20;             // candidate ring entries per (lane, query block)

// s_waitcnt vmcnt(N) lgkmcnt(0) + s_barrier for a runtime N in [0, 15] (immediate operand).
__device__ __forceinline__ void qs_barrier(uint32_t n) {
#define BSR_QS_WAIT(N) \
    case N: asm volatile("s_waitcnt vmcnt(" #N ") lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    switch (n) {
        BSR_QS_WAIT(15) BSR_QS_WAIT(14) BSR_QS_WAIT(13) BSR_QS_WAIT(12) BSR_QS_WAIT(11) BSR_QS_WAIT(10)
        BSR_QS_WAIT(9) BSR_QS_WAIT(8) BSR_QS_WAIT(7) BSR_QS_WAIT(6) BSR_QS_WAIT(5) BSR_QS_WAIT(4)
        BSR_QS_WAIT(3) BSR_QS_WAIT(2) BSR_QS_WAIT(1)
        default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    }
#undef BSR_QS_WAIT
}

template <int N>
__device__ __forceinline__ void qs_wait() {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}
// qs_wait<n> for an n that folds to a constant once the K loop is unrolled
__device__ __forceinline__ void qs_wait_n(int n) {
#define BSR_QS_N(N) \
    case N: qs_wait<N>(); break;
    switch (n) {
        BSR_QS_N(1) BSR_QS_N(2) BSR_QS_N(3) BSR_QS_N(4) BSR_QS_N(5) BSR_QS_N(6) BSR_QS_N(7) BSR_QS_N(8)
        BSR_QS_N(9) BSR_QS_N(10) BSR_QS_N(11) BSR_QS_N(12) BSR_QS_N(13) BSR_QS_N(14) BSR_QS_N(15)
        default: qs_wait<0>(); break;
    }
#undef BSR_QS_N
}

// VAR (tooling): 1 = no LDS-DMA in the loop, 5 = no epilogue, 6 = neither.  STAG (tooling):
// waves 4-7 take each slice's barrier half a slice earlier than their SIMD partners (waves
// 0-3).
template <bool EMIT, int NK, int NB, bool STAMP, int VAR = 0, bool STAG = false>
__device__ __forceinline__ void filter_qs_body(const GemmArgs& p) {
    // VAR + 8 (P - 1): one barrier per P slices (P = 2: 8-slot ring, 6 slices ahead; P = 3:
    // 10 slots, 7 ahead; P = 3 falls back to 2 when it does not divide NK).  See the loop.
    constexpr int kV = VAR & 7, kPr = ((VAR >> 3) & 7) + 1, kP = (NK % kPr == 0) ? kPr : 2;
    // VAR + 64 (P > 1 only): steady DMA stream -- the DMAs never stop early (slices past the
    // end re-read the last tile into slots nobody reads again), so every wait is the
    // steady-state count and hipcc sees the same number of VMEM ops on every path (its own
    // wait for the tile's scale load is then not a full drain).  Drained before exit.
    constexpr bool kSteady = (VAR & 64) != 0 && kPr >= 2;
    constexpr bool kNoDMA = kV == 1 || kV == 6, kNoEpi = kV == 5 || kV == 6, kB2 = kPr >= 2;
    // VAR + 128 (P = 2, tooling): a 9-slot ring with 7 slices ahead (one more DMA in flight)
    constexpr bool kDeep = (VAR & 128) != 0 && kP == 2;
    constexpr int kS = kP == 3 ? 10 : (kDeep ? 9 : kQsSlots), kA = kP == 3 ? 7 : (kDeep ? 7 : kQsAhead);
    static_assert(!kB2 || (kS >= kA + kP && kA >= kP + 2), "ring: slot reuse and landing margins");
    // NB query blocks of 32 per wave: NB = 2 -> 4 waves x 64 queries (one wave per SIMD);
    // NB = 1 -> 8 waves x 32 queries (two per SIMD, 96 query registers each)
    constexpr int NT = 64 * (8 / NB), QW = 32 * NB;
    uint64_t t0 = 0, r0 = 0, c_bar = 0, c_dma = 0, c_epi = 0;
    if (STAMP) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    // (STAMP: per-segment cycle counters of wave 0 -- barrier waits, DMA issue, epilogue)
    auto stamp = [&]() -> uint64_t {
        uint64_t t;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
        __builtin_amdgcn_sched_barrier(0);
        return t;
    };
    static_assert(NK % 2 == 0 && NK >= 2 && NK <= 12, "even slice counts up to 768 bytes");
    constexpr int BM = kQsRows, BN = kFilterTile;
    // LDS: the ring; then (EMIT) a private candidate ring of kQsLaneCap keys per (lane, query
    // block), entry e of thread t at [e][t] (conflict-free), its count in a register: no
    // atomics and no waits in the epilogue, the rings go to the per-query global lists once,
    // at the end (earlier if a block's rows could overfill it).
    constexpr int EM_BYTES = EMIT ? NT * NB * kQsLaneCap * 8 : 0;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[kS * kQsSlot + EM_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint64_t* lkeys = reinterpret_cast<uint64_t*>(lds + kS * kQsSlot) + tid;
    uint32_t ecnt[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) ecnt[n] = 0;

    // Grid as k_filter: per XCD, G row groups x n_qt query tiles; a row tile's readers share
    // the XCD's L2.
    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * NK;

    // The wave's query fragments, all K: fb[n][s] = queries .. + n*32 + (lane & 31),
    // bytes 32s + 16(lane >> 5) .. +15 (the MFMA B layout).
    i32x4_t fb[NB][2 * NK];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
        const uint8_t* src = p.B + (uint64_t)(qt * BN + w * QW + n * 32 + (lane & 31)) * p.row_bytes + 16 * (lane >> 5);
#pragma unroll
        for (int s2 = 0; s2 < 2 * NK; ++s2) fb[n][s2] = *reinterpret_cast<const i32x4_t*>(src + 32 * s2);
    }
    float tau[NB], sbq[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
        const uint32_t q = qt * BN + w * QW + n * 32 + (lane & 31);
        tau[n] = 0.0f;
        if (EMIT) tau[n] = p.tau[q];
        sbq[n] = p.b_scale[q];
    }
    // the lane's ring of query block n to the query's global list (a count past cap marks the
    // list overflowed: not certified from it)
    auto flush_ring = [&](int n) {
        const uint32_t q = qt * BN + w * QW + n * 32 + (lane & 31), nn = ecnt[n];
        if (nn) {
            const uint32_t gp = atomicAdd(p.cnt + q, nn);
            for (uint32_t i = 0; i < nn; ++i)
                if (gp + i < p.cap) p.cand[(uint64_t)q * p.cap + gp + i] = lkeys[(n * kQsLaneCap + i) * NT];
        }
        ecnt[n] = 0;
    };

    // LDS-DMA: wave w fills rows (NB*w+i)*16 .. +15 of each slice (1 KiB per instruction),
    // XOR-swizzled on the source chunk as k_filter.
    uint32_t lrow[NB], aoff_dma[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        lrow[i] = (w * NB + i) * 16 + (lane >> 2);
        aoff_dma[i] = lrow[i] * (uint32_t)p.a_stride + (((lane & 3) ^ ((lrow[i] >> 2) & 3)) * 16);
    }
    uint32_t iss_ti = 0, iss_kt = 0;
    __amdgpu_buffer_rsrc_t rsrc_a;
    auto set_issue_tile = [&]() {
        const uint32_t rt = g0 + iss_ti * RG;
        rsrc_a = __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (uint64_t)rt * BM * p.a_stride), 0,
                                                   BM * (uint32_t)p.a_stride, 0x00020000);
        if (!EMIT) {  // sample pass: tail rows read the last valid row
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const uint32_t r = rt * BM + lrow[i] < p.n_rows ? lrow[i] : p.n_rows - 1 - rt * BM;
                aoff_dma[i] = r * (uint32_t)p.a_stride + (((lane & 3) ^ ((lrow[i] >> 2) & 3)) * 16);
            }
        }
    };
    // DMA i (< NB) of slice jj = (iss_ti, iss_kt); the last advances the issue state
    auto issue_dma = [&](uint32_t jj, int i) {
        uint8_t* la = lds + (jj % kS) * kQsSlot + wu * (NB * 1024) + i * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)la, 16, aoff_dma[i], iss_kt * kSliceB, 0, 0);
        if (i == NB - 1 && ++iss_kt == NK) {
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
    // A fragments [m][kk]; fa[.][kk] of the next slice are read as soon as this slice's kk
    // MFMAs have issued (one register set: the query fragments fill most of the file)
    i32x4_t fa[4][2];
    auto read_frag = [&](uint32_t jj, int m, int kk) {
        fa[m][kk] = *reinterpret_cast<const i32x4_t*>(lds + (jj % kS) * kQsSlot + aoff[m][kk]);
    };

    i32x16_t acc[4][NB];
    // Prologue: slices 0..min(J, kQsAhead)-1 issued; slice 0 landed everywhere; its
    // fragments read.
    if (my_rt) set_issue_tile();
    const uint32_t pre = kSteady ? (J ? (uint32_t)kA : 0u) : (J < (uint32_t)kA ? J : (uint32_t)kA);
    for (uint32_t jj = 0; jj < pre; ++jj)
#pragma unroll
        for (int i = 0; i < NB; ++i) issue_dma(jj, i);
    // slices 0 and 1 (B2: 0, 1 and 2) landed everywhere
    if (kB2) qs_barrier(pre >= kP + 1 ? NB * (pre - kP - 1) : 0);
    else qs_barrier(pre >= 2 ? NB * (pre - 2) : 0);
    if (J)
#pragma unroll
        for (int m = 0; m < 4; ++m) { read_frag(0, m, 0); read_frag(0, m, 1); }

    for (uint32_t t = 0; t < my_rt; ++t) {
        const uint32_t rt = g0 + t * RG;
        // the tile's block scales: a plain load (hipcc drains vmcnt(0) at its use in the
        // epilogue; an LDS-DMA of the scales, which avoids that drain, measured 5% slower)
        float4 scv = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
        if (EMIT) scv = *reinterpret_cast<const float4*>(p.a_scale + (uint64_t)rt * (BM / kQuantBlock));
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) {
            const uint32_t jj = t * NK + kt;
            // Per K half, per m: the two MFMAs of A block m, then the next slice's fragment
            // of block m (landed: previous barrier; the register is free once both MFMAs
            // issued).  The DMAs of slice jj + kQsAhead and the barrier sit between MFMA
            // pairs, so one wave per SIMD keeps its MFMA pipe fed while they issue.
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
#pragma unroll
                    for (int n = 0; n < NB; ++n) {
                        if (kt == 0 && kk == 0) {
                            const i32x16_t z = {};
                            acc[m][n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[m][kk], fb[n][2 * kt + kk], z, 0, 0, 0);
                        } else {
                            acc[m][n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[m][kk], fb[n][2 * kt + kk], acc[m][n], 0, 0, 0);
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    read_frag(jj + 1, m, kk);  // (past the stream's end: unused; unconditional
                                               // so hipcc can count the LDS reads exactly)
                    // B2, odd slices: the DMAs follow the slice's barrier (the slot they refill,
                    // slice jj - 2's, is free once every wave is past it)
                    const bool kBarSlice = kB2 && (kt % kP) == kP - 1;
                    const bool dma_here = kBarSlice ? (kk == 1 && m >= 2 && m - 2 < NB)
                                                             : (kk == 0 && (m & 1) && (m >> 1) < NB);
                    if (!kNoDMA && dma_here && (kSteady || jj + kA < J)) {
                        uint64_t ts = 0;
                        if (STAMP) ts = stamp();
                        issue_dma(jj + kA, kBarSlice ? m - 2 : m >> 1);
                        if (STAMP) c_dma += stamp() - ts;
                    }
                    // Barrier: the slice after next has landed everywhere.  Younger VMEM ops
                    // stay in flight: the DMAs of slices jj+3 .. jj+kQsAhead (NB each) and,
                    // while it is younger than slice jj+2 (kt <= 3), the tile's scale load.
                    // No lgkmcnt: the slot a DMA refills next step was read two steps ago
                    // (hipcc waited for those reads before their MFMAs).
                    // P > 1: a barrier on every P-th slice only, once slices up to jj + P + 1
                    // have landed everywhere (the reads before the next barrier, P slices on,
                    // reach slice jj + P + 1); in flight: the DMAs of slices jj + P + 2 ..
                    // jj + A - 1 (this slice's DMA follows the barrier) and, while younger than
                    // slice jj + P + 1 (kt <= A - P - 2), the tile's scale load.  A DMA refills
                    // slice jj + A - S's slot: every wave is past it (S >= A + P).
                    if (kBarSlice && m == 1 && kk == 1) {
                        uint64_t tb = 0;
                        if (STAMP) tb = stamp();
                        const int kSc = (EMIT && kt <= kA - kP - 2) ? 1 : 0;
                        if (kSteady ? jj + 1 < J : jj + kA < J) {
                            qs_wait_n(NB * (kA - kP - 2) + kSc);
                        } else if (jj + 1 < J) {
                            const uint32_t last = J - 1;  // every DMA issued
                            qs_barrier((last > jj + kP + 1 ? NB * (last - jj - kP - 1) : 0) + kSc);
                        }
                        if (STAMP) c_bar += stamp() - tb;
                    }
                    if (!kB2 && m == 1 && kk == ((STAG && wu >= 4) ? 0 : 1)) {
                        uint64_t tb = 0;
                        if (STAMP) tb = stamp();
                        if (jj + kA < J) {
                            qs_wait_n(NB * (kA - 2) + ((EMIT && kt <= 3) ? 1 : 0));  // (folds: kt unrolled)
                        } else if (jj + 1 < J) {  // the stream's last slices, counted at run time
                            qs_barrier((J - 1 > jj + 2 ? NB * (J - 1 - jj - 2) : 0) + ((EMIT && kt <= 3) ? 1 : 0));
                        }
                        if (STAMP) c_bar += stamp() - tb;
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        if constexpr (kNoEpi) {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int n = 0; n < NB; ++n) asm volatile("" ::"v"(acc[m][n][0]));
            continue;
        }
        // ---- epilogue (VAR + 256, tooling: at raised wave priority)
        if constexpr ((VAR & 256) != 0) __builtin_amdgcn_s_setprio(2);
        uint64_t te = 0;
        if (STAMP) te = stamp();
        bool stored = false;
        const float sc[4] = {scv.x, scv.y, scv.z, scv.w};
#pragma unroll
        for (int m = 0; m < 4; ++m) {
#pragma unroll
            for (int n = 0; n < NB; ++n) {
                const uint32_t ql = w * QW + n * 32 + (lane & 31);
                const uint32_t rbase = rt * BM + m * 32 + 4 * (lane >> 5);
                auto score = [&](int v, float s_r) -> float { return ((float)v * s_r) * sbq[n]; };
                if constexpr (!EMIT) {
                    float v[16];
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        uint32_t tr = rbase + (r & 3) + 8 * (r >> 2);
                        tr = tr < p.n_rows ? tr : p.n_rows - 1;
                        v[r] = score(acc[m][n][r], p.a_scale[tr / p.a_scale_rows]);
                    }
                    float* srow = p.S + (uint64_t)(qt * BN + ql) * p.s_ld;
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
                    stored = true;
                } else {
                    auto emit = [&](float v, uint32_t row) {
                        lkeys[(n * kQsLaneCap + ecnt[n]) * NT] = score_key(v, row);
                        ++ecnt[n];
                    };
                    int gm[4];
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int x = max(acc[m][n][4 * g], acc[m][n][4 * g + 1]);
                        const int y = max(acc[m][n][4 * g + 2], acc[m][n][4 * g + 3]);
                        gm[g] = max(x, y);
                    }
                    const int mxv = max(max(gm[0], gm[1]), max(gm[2], gm[3]));
                    if (__ballot(score(mxv, sc[m]) >= tau[n])) {
                        // room for this block's up to 16 rows in every lane's ring (rarely
                        // not: dense emission, e.g. large k)
                        if (__ballot(ecnt[n] > (uint32_t)(kQsLaneCap - 16))) flush_ring(n);
                        // only the groups whose maximum passes are expanded; each register
                        // appends under its own lane mask
#pragma unroll
                        for (int g = 0; g < 4; ++g) {
                            if (!__ballot(score(gm[g], sc[m]) >= tau[n])) continue;
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const float v = score(acc[m][n][4 * g + i], sc[m]);
                                const uint32_t row = rbase + 8 * g + i;
                                if (v >= tau[n] && row < p.n_rows) emit(v, row);
                            }
                        }
                    }
                }
            }
        }
        // global stores / atomics count in vmcnt: drain them so the counted waits stay exact
        if (stored) wait_vm0();
        if constexpr ((VAR & 256) != 0) __builtin_amdgcn_s_setprio(0);
        if (STAMP) c_epi += stamp() - te;
    }
    if (kSteady) wait_vm0();  // the stream's trailing DMAs land before the workgroup ends
    if constexpr (EMIT) {
#pragma unroll
        for (int n = 0; n < NB; ++n) flush_ring(n);
    }
    if (STAMP && tid == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        reinterpret_cast<uint64_t*>(p.S)[2 * blockIdx.x] = t1 - t0;
        reinterpret_cast<uint64_t*>(p.S)[2 * blockIdx.x + 1] = r1 - r0;
        uint64_t* seg = reinterpret_cast<uint64_t*>(p.S) + 2 * gridDim.x + 4 * blockIdx.x;
        seg[0] = c_bar;
        seg[1] = c_dma;
        seg[2] = c_epi;
        seg[3] = J;
    }
}

// One wave per SIMD (NB = 2) and two per SIMD (NB = 1): separate kernels, so each gets
// its register budget from a plain __launch_bounds__.
template <bool EMIT, int NK, int NB = 2, bool STAMP = false>
__global__ __launch_bounds__(256, 1) void k_filter_qs(GemmArgs p) {
    static_assert(NB == 2, "k_filter_qs: 4 waves x 64 queries");
    filter_qs_body<EMIT, NK, 2, STAMP>(p);
}
template <bool EMIT, int NK, bool STAMP = false, int VAR = 0, bool STAG = false>
__global__ __launch_bounds__(512, 1) void k_filter_qs8(GemmArgs p) {
    filter_qs_body<EMIT, NK, 1, STAMP, VAR, STAG>(p);
}

// ------------------------------------------------------------------------------------
// Skinny int8 filter for batches of at most 16 queries (single-query latency path): the
// work is HBM-bound (1 byte per element), so there is no LDS staging.  Each wave walks
// groups of 32 tile rows; per 64-byte K step a lane loads its 16-byte A fragments straight
// from HBM (16 rows x 64 B per v_mfma_i32_16x16x64_i8 operand; lane l: row l&15, bytes
// 16(l>>4)..+15) and the matching query fragment (L1-resident), 8 K steps of loads in
// flight before their MFMAs.  The 16x16 accumulator has query l&15 on the lane and rows
// 4(l>>4)+i in its registers.  Epilogue as k_filter: SAMPLE stores every score or the
// maximum over the 32 rows of the group; EMIT appends (score, row) keys of rows reaching
// tau straight to the per-query global lists (emission is rare).
// ------------------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(4))) int i32x4_acc_t;

template <bool EMIT>
__global__ __launch_bounds__(256) void k_filter_skinny(GemmArgs p) {
    constexpr int KC = 8;  // K steps of loads in flight
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t q = lane & 15, h = lane >> 4;
    const uint32_t nk = p.row_bytes / kSliceB;
    const uint32_t n_groups = (p.n_rows + 31) / 32;
    const uint32_t nwaves = gridDim.x * 4;
    const float sbq = p.b_scale[q];
    const float tauq = EMIT ? p.tau[q] : 0.0f;
    const uint8_t* bq = p.B + (uint64_t)q * p.row_bytes + h * 16;
    for (uint32_t g = blockIdx.x * 4 + w; g < n_groups; g += nwaves) {
        uint32_t r0 = g * 32 + q, r1 = g * 32 + 16 + q;
        r0 = r0 < p.n_rows ? r0 : p.n_rows - 1;  // tail rows: clamped, never emitted
        r1 = r1 < p.n_rows ? r1 : p.n_rows - 1;
        const uint8_t* a0 = p.A + (uint64_t)r0 * p.a_stride + h * 16;
        const uint8_t* a1 = p.A + (uint64_t)r1 * p.a_stride + h * 16;
        i32x4_acc_t acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
        for (uint32_t s0 = 0; s0 < nk; s0 += KC) {
            i32x4_t fa0[KC], fa1[KC], fb[KC];
#pragma unroll
            for (int s = 0; s < KC; ++s) {
                if (s0 + s < nk) {
                    fa0[s] = *reinterpret_cast<const i32x4_t*>(a0 + (s0 + s) * kSliceB);
                    fa1[s] = *reinterpret_cast<const i32x4_t*>(a1 + (s0 + s) * kSliceB);
                    fb[s] = *reinterpret_cast<const i32x4_t*>(bq + (s0 + s) * kSliceB);
                }
            }
#pragma unroll
            for (int s = 0; s < KC; ++s) {
                if (s0 + s < nk) {
                    acc0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa0[s], fb[s], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa1[s], fb[s], acc1, 0, 0, 0);
                }
            }
        }
        // rows of register i: tile 0 -> g*32 + 4h + i, tile 1 -> g*32 + 16 + 4h + i
        if constexpr (EMIT) {
            const float sc = p.a_scale[g];  // emit: tile row == corpus row, one 32-row block
            float v[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                v[i] = ((float)acc0[i] * sc) * sbq;
                v[4 + i] = ((float)acc1[i] * sc) * sbq;
            }
            float mx = v[0];
#pragma unroll
            for (int i = 1; i < 8; ++i) mx = fmaxf(mx, v[i]);
            if (__ballot(mx >= tauq)) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint32_t row = g * 32 + (i >> 2) * 16 + 4 * h + (i & 3);
                    if (v[i] >= tauq && row < p.n_rows) {
                        const uint32_t gp = atomicAdd(p.cnt + q, 1u);
                        if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = score_key(v[i], row);
                    }
                }
            }
        } else {
            // sample: tile row r is corpus row r * a_row_mult, scale block r * mult / 32
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t tr = g * 32 + (i >> 2) * 16 + 4 * h + (i & 3);
                tr = tr < p.n_rows ? tr : p.n_rows - 1;
                const float sc = p.a_scale[tr / p.a_scale_rows];
                v[i] = ((float)(i < 4 ? acc0[i] : acc1[i - 4]) * sc) * sbq;
            }
            float* srow = p.S + (uint64_t)q * p.s_ld;
            if (!p.s_compact) {
                *reinterpret_cast<float4*>(srow + g * 32 + 4 * h) = make_float4(v[0], v[1], v[2], v[3]);
                *reinterpret_cast<float4*>(srow + g * 32 + 16 + 4 * h) = make_float4(v[4], v[5], v[6], v[7]);
            } else {
                float mx = v[0];
#pragma unroll
                for (int i = 1; i < 8; ++i) mx = fmaxf(mx, v[i]);
                mx = fmaxf(mx, __shfl_xor(mx, 16, kWave));
                mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
                if (h == 0) srow[g] = mx;
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// Skinny filter v2 (dims <= 16 K steps = 1024 int8 per row): the query fragments of all K
// steps stay in registers, and each wave walks 16-row units with the NEXT unit's A
// fragments (one 16-byte load per K step per lane) in flight while the current unit's
// MFMAs and epilogue run.  EMIT: units dealt round-robin over all waves (small tail).
// SAMPLE: a wave takes the two units of one 32-sampled-row block back to back, so the
// compact maximum over 32 sampled rows stays in a register.
// ------------------------------------------------------------------------------------
template <bool EMIT, int NK>
__global__ __launch_bounds__(256) void k_filter_skinny2(GemmArgs p) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t q = lane & 15, h = lane >> 4;
    const uint32_t nk = p.row_bytes / kSliceB;
    const uint32_t n_units = (p.n_rows + 15) / 16;
    const uint32_t nwaves = gridDim.x * 4, wid = blockIdx.x * 4 + w;
    const float sbq = p.b_scale[q];
    const float tauq = EMIT ? p.tau[q] : 0.0f;
    i32x4_t fb[NK];
#pragma unroll
    for (int s = 0; s < NK; ++s)
        fb[s] = s < (int)nk ? *reinterpret_cast<const i32x4_t*>(p.B + (uint64_t)q * p.row_bytes + h * 16 + s * kSliceB)
                            : i32x4_t{0, 0, 0, 0};
    // unit sequence of this wave: EMIT u = wid + i*nwaves; SAMPLE u = 2(wid + j*nwaves) + (i&1)
    auto unit_of = [&](uint32_t i) -> uint32_t {
        return EMIT ? wid + i * nwaves : 2 * (wid + (i >> 1) * nwaves) + (i & 1);
    };
    auto load = [&](i32x4_t (&fa)[NK], uint32_t u) {
        uint32_t r = u * 16 + q;
        r = r < p.n_rows ? r : p.n_rows - 1;  // tail rows: clamped, never emitted
        const uint8_t* a = p.A + (uint64_t)r * p.a_stride + h * 16;
#pragma unroll
        for (int s = 0; s < NK; ++s)
            if (s < (int)nk) fa[s] = *reinterpret_cast<const i32x4_t*>(a + s * kSliceB);
    };
    float smax = -INFINITY;  // SAMPLE compact: running maximum of the 32-row block
    auto process = [&](const i32x4_t (&fa)[NK], uint32_t u) {
        i32x4_acc_t acc = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < NK; ++s)
            if (s < (int)nk) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[s], fb[s], acc, 0, 0, 0);
        // register i: tile row u*16 + 4h + i, query q
        if constexpr (EMIT) {
            const float sc = p.a_scale[(u * 16) / kQuantBlock];
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = ((float)acc[i] * sc) * sbq;
            const float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
            if (__ballot(mx >= tauq)) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t row = u * 16 + 4 * h + i;
                    if (v[i] >= tauq && row < p.n_rows) {
                        const uint32_t gp = atomicAdd(p.cnt + q, 1u);
                        if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = score_key(v[i], row);
                    }
                }
            }
        } else {
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t tr = u * 16 + 4 * h + i;
                tr = tr < p.n_rows ? tr : p.n_rows - 1;
                const float sc = p.a_scale[tr / p.a_scale_rows];
                v[i] = ((float)acc[i] * sc) * sbq;
            }
            float* srow = p.S + (uint64_t)q * p.s_ld;
            if (!p.s_compact) {
                *reinterpret_cast<float4*>(srow + u * 16 + 4 * h) = make_float4(v[0], v[1], v[2], v[3]);
            } else {
                float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
                mx = fmaxf(mx, __shfl_xor(mx, 16, kWave));
                mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
                smax = fmaxf(smax, mx);
                if ((u & 1) && h == 0) srow[u >> 1] = smax;  // second half of the block
                if (u & 1) smax = -INFINITY;
            }
        }
    };
    // this wave's unit count
    uint32_t n_my;
    if (EMIT) {
        n_my = wid < n_units ? (n_units - 1 - wid) / nwaves + 1 : 0;
    } else {
        const uint32_t n_blk = (n_units + 1) / 2;
        n_my = wid < n_blk ? 2 * ((n_blk - 1 - wid) / nwaves + 1) : 0;
    }
    if (!n_my) return;
    i32x4_t fa0[NK], fa1[NK];
    load(fa0, unit_of(0));
    for (uint32_t i = 0; i < n_my; i += 2) {
        if (i + 1 < n_my) load(fa1, unit_of(i + 1));
        process(fa0, unit_of(i));
        if (i + 1 >= n_my) break;
        if (i + 2 < n_my) load(fa0, unit_of(i + 2));
        process(fa1, unit_of(i + 1));
    }
}

// ------------------------------------------------------------------------------------
// Threshold per query from the sample scores: tau0 = the ks-th largest value of S (sample
// scores, or their maxima over 32 sampled rows -- never above the ks-th largest sample),
// so that about ks * stride rows of the shard or more reach it.  4 waves per query.  Also
// zeroes the query's candidate counter and (block 0) the emit status words.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_select_tau(const float* __restrict__ S, uint32_t s_ld,
                                                    uint32_t n_s, uint32_t nq, uint32_t qpad,
                                                    const uint32_t* __restrict__ qflags,
                                                    uint32_t ks, float* __restrict__ tau,
                                                    uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ status) {
    __shared__ uint64_t part[4][64];
    const uint32_t q = blockIdx.x;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (q == 0 && t == 0) { status[kStFail] = 0; status[kStEmitted] = 0; status[kStFail2] = 0; }
    if (q >= qpad) return;
    if (t == 0) cnt[q] = 0;
    if (q >= nq || (qflags[q] & kQueryNoApprox)) {
        if (t == 0) tau[q] = INFINITY;  // never emits: answered by the exact scan
        return;
    }
    if (n_s < ks) {
        if (t == 0) tau[q] = -INFINITY;
        return;
    }
    // wave w streams a quarter of the values, keeping its ks best
    WaveTopK<1> L;
    L.init();
    uint64_t thr = kKeyNone;
    const float* s = S + (uint64_t)q * s_ld;
    const uint32_t per = (n_s + 3) / 4, lo = w * per, hi = lo + per < n_s ? lo + per : n_s;
    for (uint32_t base = lo; base < hi; base += kWave) {
        const uint32_t i = base + lane;
        L.offer(i < hi ? score_key(s[i], i) : kKeyNone, (int)ks, thr);
    }
    part[w][lane] = L.v[0];
    __syncthreads();
    if (w == 0) {
        WaveTopK<1> M;
        M.init();
        uint64_t mt = kKeyNone;
        for (int src = 0; src < 4; ++src) M.offer(part[src][lane], (int)ks, mt);
        if (lane == 0) tau[q] = score_key_score(mt);
    }
}

// Top-(kp+1) of the emitted candidates by (score desc, row asc); the first kp go to the
// exact rescore, the (kp+1)-th score bounds every row left out.  One wave per query.
template <int E>
__global__ __launch_bounds__(64) void k_select_cand(const uint64_t* __restrict__ cand,
                                                    const uint32_t* __restrict__ cnt, uint32_t cap,
                                                    uint32_t nq, const float* __restrict__ tau,
                                                    uint32_t kp, uint32_t* __restrict__ cand_rows,
                                                    uint32_t* __restrict__ ncand,
                                                    float* __restrict__ tau_excl,
                                                    uint32_t* __restrict__ status) {
    const uint32_t q = blockIdx.x;
    if (q >= nq) return;
    const uint32_t c = cnt[q];
    if (threadIdx.x == 0) atomicAdd(status + kStEmitted, c);
    if (c > cap) {  // overflow: rows were dropped, nothing can be certified
        if (threadIdx.x == 0) { ncand[q] = 0; tau_excl[q] = INFINITY; }
        return;
    }
    WaveTopK<E> L;
    L.init();
    uint64_t thr = kKeyNone;
    const uint64_t* src = cand + (uint64_t)q * cap;
    for (uint32_t base = 0; base < c; base += 4 * kWave) {
        uint64_t x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = base + u * kWave + threadIdx.x;
            x[u] = i < c ? src[i] : kKeyNone;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) L.offer(x[u], (int)kp + 1, thr);
    }
    const uint32_t nc = c < kp ? c : kp;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t pidx = e * kWave + threadIdx.x;
        if (pidx < nc) cand_rows[(uint64_t)q * kp + pidx] = key_row(L.v[e]);
    }
    if (threadIdx.x == 0) {
        ncand[q] = nc;
        tau_excl[q] = c > kp ? score_key_score(thr) : tau[q];
    }
}

}  // namespace bsrlab
