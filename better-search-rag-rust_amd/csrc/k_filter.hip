// k_filter.hip -- the MFMA candidate filter of the search (gfx950) and its selection steps.
//
// The filter scores every (corpus row, query) pair approximately on the matrix cores and
// keeps the pairs that can belong to a query's top k.  It never produces a returned
// distance: the candidates are rescored with the reference's exact arithmetic
// (k_exact.hip) and the final list is certified against the filter's error bound.
//
// Operands: int8 rows (per 32-row block scale) x int8 queries (per query scale); the integer
// dot product is exact, the score is ((float)I * s_row_block) * s_query.  The product kernel
// is k_filter_qs16 (v_mfma_i32_16x16x64_i8, rows of an even number of 64-byte K slices up to
// 768 bytes); k_filter (v_mfma_i32_32x32x32_i8) serves the other row widths.  (The bf16
// operand of rounds 1-3 is retired: half the int8 MFMA rate at an equal bound.)
#include <cstdlib>
#include "bsr_device.hpp"
#include "kernels.hpp"

#include <hip/hip_ext.h>

#include <math.h>

#include <algorithm>
#include <type_traits>
#include <utility>

namespace bsr {

typedef __attribute__((ext_vector_type(4))) int i32x4_t;
typedef __attribute__((ext_vector_type(16))) int i32x16_t;
typedef __attribute__((address_space(3))) void lds_void_t;

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
// (Ablation variants of this kernel live in tools/microbench/k_filter_lab.hip.)
// ------------------------------------------------------------------------------------
template <class Op, bool EMIT>
__global__ __launch_bounds__(kThreads, 2) void k_filter(GemmArgs p) {
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
        const uint32_t rt = g0 + iss_ti * RG;
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
        const uint8_t* base = lds + (jj % kSlots) * SLOT;
#pragma unroll
        for (int m = 0; m < 4; ++m) fa[m] = *reinterpret_cast<const frag_t*>(base + aoff[m][kk]);
#pragma unroll
        for (int n = 0; n < 2; ++n) fb[n] = *reinterpret_cast<const frag_t*>(base + boff[n][kk]);
    };
    auto mfma4 = [&](const frag_t (&fa)[4], const frag_t (&fb)[2], int half, bool first) {
        if (first) {  // first K step of a tile: C = 0
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
        const bool iss = jj + 3 < J;
        // ---- first half: kk = 0 MFMAs, kk = 1 reads, A-half DMA of slice jj+3.  The
        // reads go after the first MFMA group: hipcc puts a conservative lgkmcnt(0) in
        // front of an MFMA whose operands came from ds_read (it cannot see the barrier's
        // inline wait), which must not cover reads issued just before it.
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa0, fb0, 0, kt == 0);
        __builtin_amdgcn_sched_barrier(0);
        read_frags(jj, 1, fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        if (iss) dma_a(jj + 3, 0);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa0, fb0, 1, kt == 0);
        __builtin_amdgcn_sched_barrier(0);
        if (iss) dma_a(jj + 3, 1);
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
        if (jj + 3 < J) {
            mid_barrier<6>();
        } else if (jj + 2 < J) {
            mid_barrier<4>();
        } else {
            mid_barrier<0>();
        }
        // ---- second half: kk = 1 MFMAs, next slice's kk = 0 reads, B-half DMA
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa1, fb1, 0, false);
        __builtin_amdgcn_sched_barrier(0);
        if (jj + 1 < J) read_frags(jj + 1, 0, fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        if (iss) dma_b(jj + 3, 0);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa1, fb1, 1, false);
        __builtin_amdgcn_sched_barrier(0);
        if (iss) dma_b(jj + 3, 1);
        if (iss) issue_advance();
        __builtin_amdgcn_sched_barrier(0);

        if (kt == nk - 1) {
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
                        // sample scores (int8: a_scale per a_scale_rows tile rows)
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
                            mx = fmaxf(mx, __uint_as_float(xor_lane32<32>(__float_as_uint(mx))));
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
                        if (__ballot(score(mxv, sc[m], n) >= tau[n])) {
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
}

// ------------------------------------------------------------------------------------
// Query-stationary int8 filter (the int8 default for rows of an even number of 64-byte
// slices up to 12, i.e. dims up to 768).
//
// One 512-thread workgroup per CU, 8 waves (two per SIMD).  Wave w keeps the int8 B
// fragments of its 32 queries (qt*256 + 32w ..) for ALL of K in registers for the
// workgroup's life (96 VGPRs), so only corpus rows move: 128-row tiles stream through an
// 8-slot LDS ring (one 64-byte K slice = 8 KiB per slot, 6 slices in flight), filled by
// LDS-DMA (buffer_load ... lds, 1 KiB per wave per slice; the source chunk XOR-swizzled --
// rows 8..15 of every 16-row group exchange chunks 0<->2, 1<->3 -- so that every
// ds_read_b128 fragment read below is conflict-free).
// MFMA shape v_mfma_i32_16x16x64_i8: per slice a wave reads 8 A fragments (16 rows x 64 bytes,
// one ds_read_b128 each, four row blocks ahead in a 4-register ring) and issues 16 MFMAs
// (8 row blocks x 2 query blocks of 16).  At the same cycles per op as the 32x32x32 shape it
// holds a higher clock under load (MI355X_MICROARCH.md, DVFS item 7): measured -12% kernel
// time at equal work (profiles/r02c_qs16_ab*.txt).
// Synchronisation: one s_waitcnt vmcnt(N) + s_barrier per two slices, mid-slice (after row
// block 5 of odd slices): slices <= jj+3 have landed everywhere, with the DMAs of jj+4, jj+5
// (and the tile's scale load while younger) in flight; the odd slice's DMA follows the
// barrier, so the slot it refills (slice jj-2's) is free on every wave.  The DMA stream is
// steady: past the shard's last slice it re-reads the last tile into slots nobody reads
// again, so every wait is the steady-state count; it drains before the workgroup ends.
// The first MFMAs of a tile take C = 0 (no accumulator clears).
// Epilogue (EMIT), in two levels: (1) per query block, the lane's integer maximum over its 32
// values scored with the tile's largest (for a negative maximum: smallest) 32-row block
// scale -- never below any of its values' scores -- and one ballot for the whole tile;
// (2) only if some lane reaches tau: per 16-row block its maximum, then its rows.  Passing
// (score, row) keys go to a private per-lane LDS ring (CAP entries per query block, entry e
// of thread t at [e][t], count in a register): no atomics and no waits in the loop; flushed
// to the per-query global lists at the end or when a block could overfill it.
// SAMPLE: every tile row is one sampled corpus row; the scores (or one maximum per 32
// sampled rows) go to S.
// ------------------------------------------------------------------------------------
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
// s_waitcnt vmcnt(N) + s_barrier for an N that folds to a constant once the loop is unrolled
template <int N>
__device__ __forceinline__ void qs_wait() {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}
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

#ifdef BSR_FILTER_STAMPS
__device__ __forceinline__ void qs_vm_n(int n) {  // (stamp build) s_waitcnt vmcnt(n) alone
#define BSR_QS_V(N) \
    case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    switch (n) {
        BSR_QS_V(1) BSR_QS_V(2) BSR_QS_V(3) BSR_QS_V(4) BSR_QS_V(5) BSR_QS_V(6) BSR_QS_V(7) BSR_QS_V(8)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef BSR_QS_V
}
#endif
typedef __attribute__((ext_vector_type(4))) int i32x4v_t;

// f(std::integral_constant<int, I>) for I = 0, 1, ...: a loop the compiler must unroll (the
// emit filter's slice loop -- each slice's DMA, barrier and epilogue placement is a constant).
template <class F, int... I>
__device__ __forceinline__ void static_for(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>{}), ...);
}

constexpr int kSampleTilesPerWG = 8;  // sample pass (compact): tiles of maxima staged in LDS

__device__ __forceinline__ uint32_t qs16_swz(uint32_t row) { return ((row >> 3) & 1u) * 2u; }

#ifdef BSR_FILTER_COUNTERS
// (lab build only: emission-epilogue event counts of k_filter_qs16<true>, summed per wave)
__device__ unsigned long long g_filter_counters[8];
extern "C" int bsr_lab_filter_counters(unsigned long long* out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_filter_counters), sizeof(g_filter_counters));
    if (e == hipSuccess && reset) {
        static const unsigned long long z[8] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_filter_counters), z, sizeof(z));
    }
    return (int)e;
}
// per-workgroup timestamps (100 MHz): [block][0] start (wave 0), [block][1 + w] wave w's end
__device__ unsigned long long g_filter_wg_stamps[4096 * 9];
__device__ uint32_t g_lab_xcd_xor;  // the row streams of XCD x go to XCD x ^ this
extern "C" int bsr_lab_set_xcd_xor(uint32_t v) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_lab_xcd_xor), &v, sizeof v);
}
__device__ unsigned int g_filter_wg_tiles[4096 * 2];  // [block]: tiles processed, static tiles
extern "C" int bsr_lab_filter_wg_tiles(unsigned int* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_filter_wg_tiles), sizeof(g_filter_wg_tiles));
}
extern "C" int bsr_lab_filter_wg_stamps(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_filter_wg_stamps), sizeof(g_filter_wg_stamps));
}
#define BSR_FCNT(I_) ++fcnt[I_]
#else
#define BSR_FCNT(I_) \
    do {             \
    } while (0)
#endif
#ifdef BSR_FILTER_STAMPS
// (lab build only: s_memtime phase sums of k_filter_qs16<true>, summed over all waves:
// [0] level-1 epilogue, [1] level-2 epilogue, [2] level-2 entries, [3] the first barrier after
// the epilogue (kt = 1), [4] the other barriers, [5] loop total, [6] the DMA (vmcnt) waits
// before the barriers, [7] tiles)
__device__ unsigned long long g_filter_stamps[8];
extern "C" int bsr_lab_filter_stamps(unsigned long long* out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_filter_stamps), sizeof(g_filter_stamps));
    if (e == hipSuccess && reset) {
        static const unsigned long long z[8] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_filter_stamps), z, sizeof(z));
    }
    return (int)e;
}
#define BSR_FST(V_)                                                                     \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(V_)::"memory");       \
        __builtin_amdgcn_sched_barrier(0);                                              \
    } while (0)
#endif
// DEFER (lab): the emission epilogue in front of the next tile's first MFMAs -- 1.9% faster at
// the 1.25M-row shard, 4% slower at tau = inf, even at 10M (profiles/r04b_fab_*.txt): not kept.
// TAILX: the dynamic tail in 8 XCD-local pools (the product, tail = 1/8); 0 = one counter per
// query tile (round 3); 1 or 2 = half or all of the tiles dynamic (no gain: r04c_fab_*.txt).
// L2, FW (lab, round 5): level 2's passing row blocks as a bool array (1) instead of a bit mask
// (0); FW = 0: no explicit vmcnt(0) in the flush path.
// KSB (lab, round 6, timing only at tau = inf): a bound on the K-split wave pair (each wave of a
// pair holding 64 queries for half of K, the partial sums exchanged through LDS): 1 = every other
// fragment read skipped (the pair's halved LDS fragment bytes per MFMA); 2 = that plus the
// exchange's cost per wave and tile (16 KiB of accumulators written to LDS, read back and added).
template <bool EMIT, int NK, int EPI = 0, int TAILX = 8, int GANG = 2, int RING = 0, int L2 = 0, int FW = 1,
          int KSB = 0>
__global__ __launch_bounds__(512, 1) void k_filter_qs16(GemmArgs p) {
    constexpr bool DEFER = EPI == 1, STAGE = EPI == 2 && EMIT;
    // EPI = 3 (lab, stagger): only waves 4-7 -- the SIMD partners of waves 0-3 -- defer their
    // epilogue, so one wave of each SIMD runs its tile-end VALU work beside the other's MFMAs
    constexpr bool SPLIT = EPI == 3 && EMIT;
    // ring slots, slices issued ahead (RING, lab: 12 slots -- slot = slice index within the tile
    // for NK = 12 -- with A = 9 / 10 / 6 and a smaller emission ring to fit the LDS)
    constexpr int S = RING ? 12 : 8, A = RING == 1 ? 9 : RING == 2 ? 10 : 6;
    // the barrier wait's DMA count (slices <= jj + 3 landed: A - 4 younger ones in flight), the
    // last odd slice at which the tile's scale load / claim is younger than the slice waited
    // for, and the slice after the first barrier that has them complete
    constexpr int kWaitN = A - 4, kYoung = A - 4, kClaimUse = ((A - 4) % 2 == 0 ? A - 3 : A - 2) + 1;
    constexpr int BM = 128, BN = kFilterTile, NT = 512, SLOT = BM * kSliceB;
    constexpr int CAP = RING ? 7 : 10;  // candidate ring entries per (lane, query block)
    static_assert(NK % 2 == 0 && NK >= 2 && NK <= 12, "even slice counts up to 768 bytes");
    // STAGE: per-query LDS lists [BN][QCAP] keys + counts, the stage of raw blocks [NSTG][1 KiB]
    // + their records [NSTG][4 words], the queries' {scale, tau} [BN][2], the stage count
    constexpr int QCAP = 32, NSTG = 16;
    constexpr int ST_QL = 0, ST_STG = ST_QL + BN * QCAP * 8, ST_META = ST_STG + NSTG * 1024,
                  ST_QPAR = ST_META + NSTG * 16, ST_QCNT = ST_QPAR + BN * 8, ST_CNT = ST_QCNT + BN * 4,
                  ST_BYTES = ST_CNT + 16;
    constexpr int EM_BYTES = !EMIT ? 0 : STAGE ? ST_BYTES : NT * 2 * CAP * 8;
    // SAMPLE, compact: the workgroup's maxima [tile][4][256 queries], written to S at the end
    constexpr int SB_BYTES = EMIT ? 0 : kSampleTilesPerWG * 4 * BN * 4;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[S * SLOT + EM_BYTES + SB_BYTES + 16];
    float* const sbuf = reinterpret_cast<float*>(lds + S * SLOT + EM_BYTES);
    // tail tile ids claimed by wave 0, shared with the other waves: [0..1] in the loop, [2..3] prologue
    uint32_t* const lds_ids = reinterpret_cast<uint32_t*>(lds + S * SLOT + EM_BYTES + SB_BYTES);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t wu = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool dfr = DEFER || (SPLIT && wu >= 4);  // (wave-uniform) this wave defers its epilogue
    uint64_t* const lkeys = reinterpret_cast<uint64_t*>(lds + S * SLOT) + tid;
    uint32_t ecnt[2] = {0, 0};

    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
#ifdef BSR_FILTER_COUNTERS
    const uint32_t g0 = (xcd ^ g_lab_xcd_xor) * G + (active ? slot / p.n_qt : 0);  // (lab: remapped streams)
#else
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
#endif
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * NK;
    // Tile sequence: the row stream's static tiles g0, g0 + RG, ... below n_st, then (dyn) tail
    // tiles claimed from this query tile's counter one at a time -- workgroups on faster XCDs
    // take more of them (the kernel ends with its slowest workgroup; XCD speeds differ by
    // 4-10%, profiles/r03bb_*).  Tail tiles are read by the n_qt workgroups of different
    // streams, so they are not shared through one XCD's L2 -- hence a small tail.
    constexpr uint32_t kEnd = 0xFFFFFFFFu;
    constexpr bool kStaticSched = NK > A;
    const bool dyn = EMIT && kStaticSched && p.tail != nullptr && active;
    const uint32_t n_st = dyn ? n_rt - n_rt / (TAILX ? TAILX : kTailDiv) : n_rt;
    const uint32_t my_static = (active && g0 < n_st) ? (n_st - 1 - g0) / RG + 1 : 0;
    // (one lane) claim the next tail tile of this query tile: the counter's old value, turned
    // into a tile id by tail_id() where it is consumed -- not at once, which would wait for the
    // atomic and, in order, for every DMA in flight.  The address is one the compiler cannot
    // prove uniform: the atomic optimizer would otherwise aggregate the atomic across the wave
    // and consume its result immediately.
    // TAILX: the tail is split into 8 pools of consecutive tiles, pool x claimed first by the
    // workgroups on XCD x (counter tail[x * n_qt + qt]), so that the n_qt workgroups reading a
    // tail tile sit on one XCD and share it through its L2; a workgroup whose own pool is empty
    // steals from the next XCD's pools (the balancing the tail exists for).  Without TAILX one
    // counter per query tile hands every tail tile to workgroups of different XCDs.
    const uint32_t n_tail = n_rt - n_st, pool_sz = (n_tail + 7) / 8;
    uint32_t cpool = xcd, pools_tried = 1;  // (lane 0 of wave 0) the pool claimed from
    auto pool_n = [&](uint32_t x) -> uint32_t {
        const uint32_t lo = x * pool_sz;
        return lo >= n_tail ? 0u : min(pool_sz, n_tail - lo);
    };
    auto claim_raw = [&]() -> uint32_t {
        uint32_t z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        return atomicAdd(p.tail + (TAILX ? cpool * p.n_qt : 0u) + qt + z, 1u);
    };
    auto tail_id = [&](uint32_t v) -> uint32_t {
        if constexpr (!TAILX) {
            return n_st + v < n_rt ? n_st + v : kEnd;
        } else {
            for (;;) {  // (own pool empty: claim from the next XCD's, synchronously -- rare)
                if (v < pool_n(cpool)) return n_st + cpool * pool_sz + v;
                if (pools_tried == 8) return kEnd;
                ++pools_tried;
                cpool = (cpool + 1) & 7;
                v = atomicAdd(p.tail + cpool * p.n_qt + qt, 1u);
            }
        }
    };
    auto claim = [&]() -> uint32_t { return tail_id(claim_raw()); };
    // GANG: the n_qt workgroups of a row stream read the same tiles, on one XCD, and share them
    // through its L2 only while they stay within a few tiles of each other.  Each static tile,
    // wave 0 adds 1 to its 16-bit field of the stream's progress word (one 64-bit atomic, its
    // old value = every member's count); a workgroup more than GANG tiles ahead of the slowest
    // member sleeps a bounded while (never waits for a condition: no member can hang another).
    // The drift grows with the stream's length: 2.02x the corpus bytes fetched at 10M rows
    // without gangs, 1.09x with GANG = 2 (and 1.4% faster); 1.03x either way at 1.25M rows, where
    // the atomic only costs (profiles/r04i_fab*) -- hence streams of >= kGangMinTiles tiles only.
    const bool gang = GANG && EMIT && kStaticSched && active && p.tail != nullptr && p.n_qt >= 2 && p.n_qt <= 4 &&
                      my_static >= kGangMinTiles;
    unsigned long long* const gprog =
        reinterpret_cast<unsigned long long*>(p.tail + 8 * kTailCounters) + (gang ? g0 : 0u);
    auto gang_raw = [&]() -> unsigned long long {
        uint32_t z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        return atomicAdd(gprog + z, 1ull << (16 * qt));
    };
    auto gang_throttle = [&](unsigned long long old) {
        const uint32_t me = (uint32_t)(old >> (16 * qt)) & 0xFFFFu;
        int lag = 0;
        for (uint32_t j = 0; j < p.n_qt; ++j)
            if (j != qt) lag = max(lag, (int)(int16_t)(uint16_t)(me - ((uint32_t)(old >> (16 * j)) & 0xFFFFu)));
        for (int i = GANG; i < lag && i < GANG + 4; ++i) __builtin_amdgcn_s_sleep(32);
    };

    // B fragments of the wave's two 16-query blocks, all K: fb[nb][kt] = query
    // qt*256 + 32w + 16nb + (lane & 15), bytes 64kt + 16(lane >> 4) .. +15.
    uint32_t qq[2];
    i32x4v_t fb[2][NK];
    float tau[2], sbq[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
        qq[nb] = qt * BN + w * 32 + nb * 16 + (lane & 15);
        const uint8_t* src = p.B + (uint64_t)qq[nb] * p.row_bytes + 16 * (lane >> 4);
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) fb[nb][kt] = *reinterpret_cast<const i32x4v_t*>(src + 64 * kt);
        tau[nb] = EMIT ? p.tau[qq[nb]] : 0.0f;
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
        // vmcnt(0) as the builtin (not asm), so that the compiler's wait counting sees the
        // atomic's return complete on this path: otherwise every join after a flush branch
        // (each level-2 append) carries a vmcnt(0) that drains the whole DMA stream
        if constexpr (FW) __builtin_amdgcn_s_waitcnt(0x0F70);
    };

    // STAGE: emission balanced over the workgroup's waves.  A wave whose tile passes level 1
    // copies each passing 16-row x 16-query block's raw accumulators (1 KiB) to the stage with
    // a record {first row, first query, block scale}; after the next tile's first barrier EVERY
    // wave scores a 1/8 share of the staged values (one per thread) and appends the passing
    // (score, row) keys to per-query LDS lists (an LDS atomic per key), flushed to the global
    // lists at the end.  The emitting wave no longer holds the workgroup at the next barrier
    // while it appends (the level-2 skew of the per-lane rings: DESIGN.md §5).
    uint8_t* const est = lds + S * SLOT;
    uint64_t* const st_ql = reinterpret_cast<uint64_t*>(est + ST_QL);
    int* const st_blk = reinterpret_cast<int*>(est + ST_STG);
    uint32_t* const st_meta = reinterpret_cast<uint32_t*>(est + ST_META);
    float* const st_qpar = reinterpret_cast<float*>(est + ST_QPAR);
    uint32_t* const st_qcnt = reinterpret_cast<uint32_t*>(est + ST_QCNT);
    uint32_t* const st_cnt = reinterpret_cast<uint32_t*>(est + ST_CNT);
    // one value of a staged or inline block: query ql of the tile (local), corpus row `row`
    auto st_append = [&](int iv, float scb, uint32_t row, uint32_t ql) {
        const float v = ((float)iv * scb) * st_qpar[2 * ql];
        if (v >= st_qpar[2 * ql + 1] && row < p.n_rows) {
            uint32_t pos;
            const uint32_t addr = (uint32_t)(uintptr_t)(st_qcnt + ql);
            asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(pos) : "v"(addr), "v"(1u) : "memory");
            if (pos < (uint32_t)QCAP) {
                st_ql[ql * QCAP + pos] = score_key(v, row);
            } else {  // (list full: straight to the global list)
                const uint32_t q = qt * BN + ql;
                const uint32_t gp = atomicAdd(p.cnt + q, 1u);
                if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = score_key(v, row);
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): keep the DMA stream's counted waits exact
            }
        }
    };
    // every thread: the staged values v = tid, tid + 512, ... of n staged blocks
    auto st_process = [&](uint32_t n) {
        for (uint32_t v = tid; v < n * 256; v += NT) {
            const uint32_t e = v >> 8, i = v & 255, l = i >> 2;
            const int iv = st_blk[v];
            const uint32_t* m = st_meta + 4 * e;
            st_append(iv, __uint_as_float(m[2]), m[0] + 4 * (l >> 4) + (i & 3), m[1] + (l & 15));
        }
    };
    if constexpr (STAGE) {
        if (lane < 16)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                const uint32_t ql = w * 32 + nb * 16 + lane;
                st_qpar[2 * ql] = sbq[nb];
                st_qpar[2 * ql + 1] = tau[nb];
            }
        if (tid < BN) st_qcnt[tid] = 0;
        if (tid == 0) *st_cnt = 0;
    }

    // LDS-DMA: wave w fills rows 16w .. 16w+15 of each slice (1 KiB per instruction); the
    // source chunk is XOR-swizzled so that LDS chunk position p holds global chunk p ^ swz.
    const uint32_t lrow = w * 16 + (lane >> 2);
    const uint32_t lchunk = ((lane & 3) ^ qs16_swz(lrow)) * 16;
    // Tile ti's descriptor (base = its first row) and this lane's byte offset in it (SAMPLE:
    // tail rows read the last valid row).
    auto tile_src_rt = [&](uint32_t rt, __amdgpu_buffer_rsrc_t& rs, uint32_t& off) {
        rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (uint64_t)rt * BM * p.a_stride), 0,
                                               BM * (uint32_t)p.a_stride, 0x00020000);
        const uint32_t r = (EMIT || rt * BM + lrow < p.n_rows) ? lrow : p.n_rows - 1 - rt * BM;
        off = r * (uint32_t)p.a_stride + lchunk;
    };
    auto tile_src = [&](uint32_t ti, __amdgpu_buffer_rsrc_t& rs, uint32_t& off) { tile_src_rt(g0 + ti * RG, rs, off); };
    // Static schedule (NK > A, every dim of the product): the DMA issued during slice kt of
    // tile t fills slice (kt + A) % NK of tile t (kt + A < NK) or of tile t + 1 -- both
    // descriptors computed once per tile, so a DMA is two instructions and no branch.  Past
    // the last tile the stream re-reads it (steady counted waits; nobody reads those slots).
    constexpr bool kStatic = kStaticSched;
    __amdgpu_buffer_rsrc_t rs_cur, rs_nxt;
    uint32_t off_cur = 0, off_nxt = 0;
    auto dma_static = [&](uint32_t jj, int kt) {
        uint8_t* la = lds + (jj % S) * SLOT + wu * 1024;
        if (kt + A < NK)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_cur, (lds_void_t*)la, 16, off_cur, (kt + A) * kSliceB, 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_nxt, (lds_void_t*)la, 16, off_nxt, (kt + A - NK) * kSliceB, 0, 0);
    };
    // dynamic schedule (NK <= A: a DMA may run more than one tile ahead)
    uint32_t iss_ti = 0, iss_kt = 0, aoff_dma = 0;
    __amdgpu_buffer_rsrc_t rsrc_a;
    auto issue_dma = [&](uint32_t jj) {
        uint8_t* la = lds + (jj % S) * SLOT + wu * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)la, 16, aoff_dma, iss_kt * kSliceB, 0, 0);
        if (++iss_kt == NK) {
            iss_kt = 0;
            ++iss_ti;
            if (iss_ti < my_rt) tile_src(iss_ti, rsrc_a, aoff_dma);
        }
    };
    // A fragment of row block rb (rows 16rb .. +15): lane -> row 16rb + (lane & 15), chunk
    // lane >> 4; the swizzle depends on row & 15 only, so block rb is at a constant 1 KiB step
    const uint32_t aoff0 = (lane & 15) * kSliceB + (((lane >> 4) ^ qs16_swz(lane & 15)) * 16);
    // four fragment registers, read four row blocks ahead: block rb of slice jj lands in
    // fa[rb & 3] while the MFMAs of block rb - 4 (the same slice, or the previous one) run
    i32x4v_t fa[4];
    auto read_frag = [&](uint32_t jj, int rb) {
        fa[rb & 3] = *reinterpret_cast<const i32x4v_t*>(lds + (jj % S) * SLOT + rb * 1024 + aoff0);
    };

    i32x4v_t acc[8][2];
    // (DEFER) the emission epilogue of the PREVIOUS tile, one 32-row pair at a time (row blocks
    // 2s, 2s+1: one block scale), placed in front of the next tile's first MFMAs on those row
    // blocks, whose C = 0 operand overwrites them: the lane's maximum per query block, scored
    // once, one ballot per pair; a pair that passes appends its passing rows as level 2 does.
    // Its VALU work runs beside the partner wave's MFMAs instead of in a tile-end phase that
    // every wave of the workgroup reaches together.
    auto epi_pair = [&](int s, float scs, uint32_t rte) {
        int bm[2][2];
        bool pass = false;
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const i32x4v_t& x = acc[2 * s + h][nb];
                bm[h][nb] = max(max(x[0], x[1]), max(x[2], x[3]));
            }
            const int m = max(bm[0][nb], bm[1][nb]);
            pass |= ((float)m * scs) * sbq[nb] >= tau[nb];
        }
        if (!__ballot(pass)) return;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                if (!__ballot(((float)bm[h][nb] * scs) * sbq[nb] >= tau[nb])) continue;
                if (__ballot(ecnt[nb] > (uint32_t)(CAP - 4))) flush_ring(nb);  // room for 4 rows
                const i32x4v_t& x = acc[2 * s + h][nb];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = ((float)x[r] * scs) * sbq[nb];
                    const uint32_t row = rte * BM + (2 * s + h) * 16 + 4 * (lane >> 4) + r;
                    lkeys[(nb * CAP + ecnt[nb]) * NT] = score_key(v, row);
                    ecnt[nb] += (v >= tau[nb] && row < p.n_rows) ? 1u : 0u;
                }
            }
        }
    };
    float sc_prev[4] = {1.0f, 1.0f, 1.0f, 1.0f};
    uint32_t rt_prev = 0;
    uint32_t n_stg = 0;  // (STAGE) the previous tile's staged block count
    // the first two tiles of the sequence
    uint32_t cur_id = my_rt ? g0 : kEnd, nxt_id = my_rt > 1 ? g0 + RG : kEnd;
    if (dyn && my_static < 2) {
        if (tid == 0) {
            const uint32_t a0 = my_static ? g0 : claim();
            lds_ids[2] = a0;
            lds_ids[3] = a0 == kEnd ? kEnd : claim();
        }
        __syncthreads();
        cur_id = __builtin_amdgcn_readfirstlane(lds_ids[2]);
        nxt_id = __builtin_amdgcn_readfirstlane(lds_ids[3]);
    } else if (dyn) {
        cur_id = g0;
        nxt_id = g0 + RG;
    }
    const bool any_tile = cur_id != kEnd;
    const uint32_t pre = (dyn ? any_tile : J != 0) ? (uint32_t)A : 0u;
    if (any_tile) {
        tile_src_rt(cur_id, rsrc_a, aoff_dma);
        rs_cur = rsrc_a;
        off_cur = aoff_dma;
        tile_src_rt(nxt_id != kEnd ? nxt_id : cur_id, rs_nxt, off_nxt);
    }
    if (kStatic) {
        for (uint32_t jj = 0; jj < pre; ++jj) {
            uint8_t* la = lds + (jj % S) * SLOT + wu * 1024;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_cur, (lds_void_t*)la, 16, off_cur, jj * kSliceB, 0, 0);
        }
    } else {
        for (uint32_t jj = 0; jj < pre; ++jj) issue_dma(jj);
    }
    qs_barrier(pre >= 3 ? pre - 3 : 0);  // slices 0, 1, 2 landed everywhere
    if (any_tile)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) read_frag(0, rb);

#ifdef BSR_FILTER_COUNTERS
    unsigned long long fcnt[5] = {0, 0, 0, 0, 0};
    if (EMIT && tid == 0 && blockIdx.x < 4096) g_filter_wg_stamps[blockIdx.x * 9] = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef BSR_FILTER_STAMPS
    unsigned long long fst[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_a, st_b, st_loop0;
    BSR_FST(st_loop0);
#endif
    uint32_t t = 0;
    for (; cur_id != kEnd; ++t) {
        const uint32_t rt = cur_id;
        BSR_FCNT(4);
        if (kStatic && t) {
            rs_cur = rs_nxt;
            off_cur = off_nxt;
            tile_src_rt(nxt_id != kEnd ? nxt_id : cur_id, rs_nxt, off_nxt);
        }
        float4 scv = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
        if (EMIT) scv = *reinterpret_cast<const float4*>(p.a_scale + (uint64_t)rt * (BM / kQuantBlock));
        // the tile after next: static, or (dyn) claimed now by wave 0 -- its atomic is one more
        // VMEM op in wave 0's count at the first barrier (kt = 1), complete by the second --
        // and shared through LDS at kt = 4, read by every wave after the tile
        uint32_t n2 = (t + 2 < my_static) ? g0 + (t + 2) * RG : kEnd;
        const bool req = dyn && t + 2 >= my_static && nxt_id != kEnd;
        uint32_t claimed = 0;
        if (req && tid == 0) claimed = claim_raw();
        // (GANG, static tiles only: the progress atomic takes the claim's place in the count)
        const bool thr = gang && t + 2 < my_static;
        unsigned long long gold = 0;
        if (thr && tid == 0) gold = gang_raw();
        const int w0_req = ((req || thr) && w == 0) ? 1 : 0;
        // SAMPLE: one scale for the tile's 128 sampled rows (a scalar load: counted in lgkmcnt,
        // it leaves the DMA stream's vmcnt waits alone)
        float sc_tile = 1.0f;
        if constexpr (!EMIT) sc_tile = p.a_scale[rt * BM / kSampleScaleRows];
        static_for(std::make_integer_sequence<int, NK>{}, [&](auto KT) {
            constexpr int kt = decltype(KT)::value;
            const uint32_t jj = t * NK + kt;
            const bool bar_slice = (kt & 1) == 1;
#pragma unroll
            for (int rb = 0; rb < 8; ++rb) {
                if constexpr ((DEFER || SPLIT) && EMIT && kt == 0) {
                    if (dfr && (rb & 1) == 0 && t > 0) epi_pair(rb >> 1, sc_prev[rb >> 1], rt_prev);
                    // pin the first MFMAs on these row blocks below the epilogue (their C = 0
                    // operand does not read the accumulators, so nothing else orders them, and
                    // hoisted above it they would need a second set of accumulators)
                    asm volatile("" : "+v"(fa[rb & 3]));
                    __builtin_amdgcn_sched_barrier(0);
                }
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
                if (KSB && (rb & 1)) {
                    // (lab KSB: this fragment read skipped; the register keeps an older fragment)
                } else if (rb < 4) {
                    read_frag(jj, rb + 4);
                } else {
                    read_frag(jj + 1, rb - 4);  // (past the stream's end: unused)
                }
                // (the atomic completed at the kt = 3 barrier; the LDS write completes, in order,
                // before wave 0's next fragment reads are waited for -- well before kt = 5's barrier)
                if (kt == kClaimUse && rb == 0 && req && tid == 0) lds_ids[t & 1] = tail_id(claimed);
                if (GANG && kt == kClaimUse && rb == 0 && thr && tid == 0) gang_throttle(gold);
                // DMA of slice jj + A: after group 1 on even slices; after the barrier (group 6)
                // on odd slices (the slot it refills, slice jj - 2's, is then free everywhere)
                if (bar_slice ? rb == 6 : rb == 1) {
                    if (kStatic) dma_static(jj + A, kt);
                    else issue_dma(jj + A);
                }
                // barrier (odd slices, after group 5): slices <= jj + 3 landed everywhere (the
                // reads before the next barrier reach rows 0-1 of slice jj + 3); in flight: the
                // DMAs of slices jj + 4, jj + 5 and, while younger than slice jj + 3 (kt <= 2),
                // the tile's scale load.  (Static schedule: also at the last slice -- the
                // trailing DMAs keep the count steady -- so no branch.)
                if (bar_slice && rb == 5 && (kStatic || jj + 1 < J)) {
#ifdef BSR_FILTER_STAMPS
                    // (stamp build: the vmcnt wait and the barrier timed apart, [3]/[4] the
                    // barrier alone, [6] the DMA wait)
                    if (EMIT) {
                        BSR_FST(st_a);
                        qs_vm_n(kWaitN + ((EMIT && kt <= kYoung) ? 1 + w0_req : 0));
                        BSR_FST(st_b);
                        fst[6] += st_b - st_a;
                        st_a = st_b;
                        asm volatile("s_barrier" ::: "memory");
                        BSR_FST(st_b);
                        fst[kt == 1 ? 3 : 4] += st_b - st_a;
                    } else
#endif
                    qs_wait_n(kWaitN + ((EMIT && kt <= kYoung) ? 1 + w0_req : 0));
                }
                if constexpr (STAGE) {
                    // the previous tile's stage: its count read after the kt = 1 barrier (every
                    // wave's stage writes landed before it), the values scored at kt = 2 (the
                    // count's read long complete), the count reset after the kt = 3 barrier (every
                    // wave has read it); the next stage writes follow the kt = 11 barrier
                    if (kt == 1 && rb == 5) n_stg = min(*st_cnt, (uint32_t)NSTG);
                    if (kt == 2 && rb == 0 && n_stg) st_process(n_stg);
                    if (kt == 3 && rb == 5 && tid == 0) {
                        *st_cnt = 0;
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        });
        if constexpr (KSB == 2 && EMIT) {
            // (lab KSB = 2, timing only) the pair's exchange: 16 KiB of this wave's accumulators to
            // LDS (the emission rings' space: unused at tau = inf), read back and added
            i32x4v_t* xs = reinterpret_cast<i32x4v_t*>(lds + S * SLOT + (w % 5) * 16384) + lane;
#pragma unroll
            for (int i = 0; i < 16; ++i) xs[i * 64] = acc[i >> 1][i & 1];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i >> 1][i & 1] += xs[(15 - i) * 64];
        }
        // ---- epilogue: block (rb, nb) holds rows 16rb + 4(lane >> 4) + r, query qq[nb]
        const float sc[4] = {scv.x, scv.y, scv.z, scv.w};
        bool stored = false;
        if constexpr (!EMIT) {
            // sample pass, one scale per tile: compact = the integer maximum over each 32-row
            // group (row blocks 2g, 2g+1: the lane's 8 values, then across the four lanes of its
            // query by two VALU lane swaps), scored once; full = every row's score
            if (p.s_compact) {
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int nb = 0; nb < 2; ++nb) {
                        const i32x4v_t& x = acc[2 * g][nb];
                        const i32x4v_t& y = acc[2 * g + 1][nb];
                        int m = max(max(max(x[0], x[1]), max(x[2], x[3])), max(max(y[0], y[1]), max(y[2], y[3])));
                        const auto p16 = __builtin_amdgcn_permlane16_swap(m, m, false, false);
                        m = max((int)p16[0], (int)p16[1]);
                        const auto p32 = __builtin_amdgcn_permlane32_swap(m, m, false, false);
                        m = max((int)p32[0], (int)p32[1]);
                        const float v = ((float)m * sc_tile) * sbq[nb];
                        if (lane < 16) sbuf[((t % kSampleTilesPerWG) * 4 + g) * BN + (qq[nb] - qt * BN)] = v;
                    }
                if (t % kSampleTilesPerWG == kSampleTilesPerWG - 1 || t + 1 == my_rt) {
                    // every kSampleTilesPerWG tiles: the staged maxima to S, 4 consecutive columns
                    // per (query, tile) (global stores inside the DMA stream only this often)
                    __syncthreads();
                    const uint32_t t0 = t - t % kSampleTilesPerWG, nt = t + 1 - t0;
                    for (uint32_t i = tid; i < nt * BN; i += NT) {
                        const uint32_t tt = i / BN, ql = i % BN;
                        const float4 v = make_float4(sbuf[(tt * 4 + 0) * BN + ql], sbuf[(tt * 4 + 1) * BN + ql],
                                                     sbuf[(tt * 4 + 2) * BN + ql], sbuf[(tt * 4 + 3) * BN + ql]);
                        *reinterpret_cast<float4*>(p.S + (uint64_t)(qt * BN + ql) * p.s_ld + (g0 + (t0 + tt) * RG) * 4) = v;
                    }
                    stored = true;
                }
            } else {
#pragma unroll
                for (int rb = 0; rb < 8; ++rb) {
                    const uint32_t rbase = rt * BM + rb * 16 + 4 * (lane >> 4);
#pragma unroll
                    for (int nb = 0; nb < 2; ++nb) {
                        const i32x4v_t& x = acc[rb][nb];
                        const float v0 = ((float)x[0] * sc_tile) * sbq[nb], v1 = ((float)x[1] * sc_tile) * sbq[nb];
                        const float v2 = ((float)x[2] * sc_tile) * sbq[nb], v3 = ((float)x[3] * sc_tile) * sbq[nb];
                        *reinterpret_cast<float4*>(p.S + (uint64_t)qq[nb] * p.s_ld + rbase) = make_float4(v0, v1, v2, v3);
                    }
                }
                stored = true;
            }
        } else if constexpr (STAGE) {
            // level 1 as below; the passing blocks go to the stage (or, when it is full, are
            // appended by this wave at once)
            const float sc_hi = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
            const float sc_lo = fminf(fminf(sc[0], sc[1]), fminf(sc[2], sc[3]));
            int mrb[2];
            bool any = false;
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
                uint32_t M = 0;  // (uniform) passing blocks, bit 8 nb + rb
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    if (!__ballot(((float)mrb[nb] * (mrb[nb] >= 0 ? sc_hi : sc_lo)) * sbq[nb] >= tau[nb])) continue;
#pragma unroll
                    for (int rb = 0; rb < 8; ++rb) {
                        const i32x4v_t& x = acc[rb][nb];
                        const int bm = max(max(x[0], x[1]), max(x[2], x[3]));
                        if (__ballot(((float)bm * sc[rb >> 1]) * sbq[nb] >= tau[nb])) M |= 1u << (8 * nb + rb);
                    }
                }
                if (M) {
                    uint32_t base = 0;
                    if (lane == 0) {
                        const uint32_t addr = (uint32_t)(uintptr_t)st_cnt;
                        asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
                                     : "=v"(base) : "v"(addr), "v"((uint32_t)__builtin_popcount(M)) : "memory");
                    }
                    base = __builtin_amdgcn_readfirstlane(__shfl(base, 0, kWave));
#pragma unroll
                    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                        for (int rb = 0; rb < 8; ++rb) {
                            if (!((M >> (8 * nb + rb)) & 1u)) continue;
                            const uint32_t slot = base + (uint32_t)__builtin_popcount(M & ((1u << (8 * nb + rb)) - 1u));
                            const uint32_t row0 = rt * BM + rb * 16, q0 = w * 32 + nb * 16;
                            if (slot < (uint32_t)NSTG) {
                                *reinterpret_cast<i32x4v_t*>(st_blk + slot * 256 + lane * 4) = acc[rb][nb];
                                if (lane == 0)
                                    *reinterpret_cast<uint4*>(st_meta + 4 * slot) =
                                        make_uint4(row0, q0, __float_as_uint(sc[rb >> 1]), 0u);
                            } else {
#pragma unroll
                                for (int r = 0; r < 4; ++r)
                                    st_append(acc[rb][nb][r], sc[rb >> 1], row0 + 4 * (lane >> 4) + r, q0 + (lane & 15));
                            }
                        }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the stage is read after a barrier)
                }
            }
        } else if constexpr (DEFER) {
            // (the epilogue runs in front of the next tile's first MFMAs, or after the loop)
            // (held in VGPRs: the loop's scalar registers are spoken for)
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("v_mov_b32 %0, %1" : "=v"(sc_prev[i]) : "s"(sc[i]));
            asm volatile("v_mov_b32 %0, %1" : "=v"(rt_prev) : "s"(rt));
        } else if (SPLIT && dfr) {
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("v_mov_b32 %0, %1" : "=v"(sc_prev[i]) : "s"(sc[i]));
            asm volatile("v_mov_b32 %0, %1" : "=v"(rt_prev) : "s"(rt));
        } else {
            // level 1, one ballot per tile: the lane's integer maximum over all its 32 values of
            // each query block, scored with the tile's largest (or, for a negative maximum,
            // smallest) block scale -- never below any of its values' scores
            const float sc_hi = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
            const float sc_lo = fminf(fminf(sc[0], sc[1]), fminf(sc[2], sc[3]));
            bool any = false;
            BSR_FCNT(0);
#ifdef BSR_FILTER_STAMPS
            BSR_FST(st_a);
            fst[7] += 1;
#endif
            int mrb[2];  // (unused lanes' values are never read)
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
            const bool l2 = __ballot(any) != 0;
#ifdef BSR_FILTER_STAMPS
            BSR_FST(st_b);
            fst[0] += st_b - st_a;
            st_a = st_b;
#endif
            if (l2) {
                BSR_FCNT(1);
                // level 2: per (query block, 16-row block) its maximum against tau -- eight
                // independent scores, then one uniform branch per passing row block -- and that
                // block's 4 rows appended without branches (every key is written to the next
                // ring slot, the count advances only for passing rows)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    if (!__ballot(((float)mrb[nb] * (mrb[nb] >= 0 ? sc_hi : sc_lo)) * sbq[nb] >= tau[nb])) continue;
                    BSR_FCNT(2);
                    uint32_t pm = 0;  // the lane's passing row blocks
                    bool pass_rb[8];
#pragma unroll
                    for (int rb = 0; rb < 8; ++rb) {
                        const i32x4v_t& x = acc[rb][nb];
                        const int bm = max(max(x[0], x[1]), max(x[2], x[3]));
                        if constexpr (L2) pass_rb[rb] = ((float)bm * sc[rb >> 1]) * sbq[nb] >= tau[nb];
                        else pm |= (((float)bm * sc[rb >> 1]) * sbq[nb] >= tau[nb]) ? 1u << rb : 0u;
                    }
#pragma unroll
                    for (int rb = 0; rb < 8; ++rb) {
                        if (!__ballot(L2 ? pass_rb[rb] : ((pm >> rb) & 1u))) continue;
                        BSR_FCNT(3);
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
#ifdef BSR_FILTER_STAMPS
                BSR_FST(st_b);
                fst[1] += st_b - st_a;
                fst[2] += 1;
#endif
            }
        }
        if (stored) wait_vm0();  // global stores / atomics count in vmcnt: keep the waits exact
        cur_id = nxt_id;
        nxt_id = req ? __builtin_amdgcn_readfirstlane(lds_ids[t & 1]) : n2;
    }
    if constexpr (STAGE) {
        // the last tile's stage, then the per-query lists to the global lists
        __syncthreads();
        const uint32_t n = min(*st_cnt, (uint32_t)NSTG);
        __syncthreads();  // (everyone has read the count before it can change)
        st_process(n);
        __syncthreads();
        if (tid < BN) {
            const uint32_t c = min(st_qcnt[tid], (uint32_t)QCAP);
            if (c) {
                const uint32_t q = qt * BN + tid;
                const uint32_t gp = atomicAdd(p.cnt + q, c);
                for (uint32_t i = 0; i < c; ++i)
                    if (gp + i < p.cap) p.cand[(uint64_t)q * p.cap + gp + i] = st_ql[tid * QCAP + i];
            }
        }
    }
    if constexpr ((DEFER || SPLIT) && EMIT) {  // the last tile's epilogue
        if (dfr && t > 0)
#pragma unroll
            for (int s = 0; s < 4; ++s) epi_pair(s, sc_prev[s], rt_prev);
    }
    wait_vm0();  // the stream's trailing DMAs land before the workgroup ends
#ifdef BSR_FILTER_STAMPS
    if (EMIT) {
        BSR_FST(st_b);
        fst[5] = st_b - st_loop0;
        if (lane == 0)
            for (int i = 0; i < 8; ++i) atomicAdd(&g_filter_stamps[i], fst[i]);
    }
#endif
    if constexpr (EMIT) {
        flush_ring(0);
        flush_ring(1);
#ifdef BSR_FILTER_COUNTERS
        if (lane == 0) {
            for (int i = 0; i < 4; ++i) atomicAdd(&g_filter_counters[i], fcnt[i]);
            if (blockIdx.x < 4096) g_filter_wg_stamps[blockIdx.x * 9 + 1 + w] = __builtin_amdgcn_s_memrealtime();
            if (blockIdx.x < 4096 && w == 0) {
                g_filter_wg_tiles[blockIdx.x * 2] = (unsigned int)fcnt[4];
                g_filter_wg_tiles[blockIdx.x * 2 + 1] = my_static;
            }
        }
#endif
    }
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
            // sample: int8 scales per a_scale_rows tile rows
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
                mx = fmaxf(mx, __uint_as_float(xor_lane32<16>(__float_as_uint(mx))));
                mx = fmaxf(mx, __uint_as_float(xor_lane32<32>(__float_as_uint(mx))));
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
// TOP (round 6, the self-thresholded single-query path): units dealt as EMIT, no threshold;
// each lane keeps the 4 best (score, row) keys of its rows, the four lanes of a query and then
// the workgroup's four waves merge them at the end, and the workgroup writes its 4 best keys per
// query to cand[q][workgroup][4] -- every row of the workgroup not among them scores at most its
// 4th (tiny batches).
// ------------------------------------------------------------------------------------
#ifndef BSR_SKINNY_NT
#define BSR_SKINNY_NT 0
#endif
constexpr int kSkSample = 0, kSkEmit = 1, kSkTop = 2;
// insert key x into the ascending 4-list t (smaller key = better score), keeping the best 4
__device__ __forceinline__ void top4_insert(uint64_t (&t)[4], uint64_t x) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool lt = x < t[j];
        const uint64_t lo = lt ? x : t[j];
        x = lt ? t[j] : x;
        t[j] = lo;
    }
}
template <int MODE, int NK>
__global__ __launch_bounds__(256) void k_filter_skinny2(GemmArgs p) {
    constexpr bool EMIT = MODE == kSkEmit, TOP = MODE == kSkTop, ROWS = EMIT || TOP;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t q = lane & 15, h = lane >> 4;
    const uint32_t nk = p.row_bytes / kSliceB;
    const uint32_t n_units = (p.n_rows + 15) / 16;
    // (TOP: the workgroup's waves take units gridDim.x apart, so that the rows of a run of
    // consecutive units -- a cluster of similar rows, below -- fall into different workgroups)
    const uint32_t nwaves = gridDim.x * 4, wid = TOP ? w * gridDim.x + blockIdx.x : blockIdx.x * 4 + w;
    const float sbq = p.b_scale[q];
    const float tauq = EMIT ? p.tau[q] : 0.0f;
    i32x4_t fb[NK];
#pragma unroll
    for (int s = 0; s < NK; ++s)
        fb[s] = s < (int)nk ? *reinterpret_cast<const i32x4_t*>(p.B + (uint64_t)q * p.row_bytes + h * 16 + s * kSliceB)
                            : i32x4_t{0, 0, 0, 0};
    // unit sequence of this wave: EMIT / TOP u = wid + i*nwaves; SAMPLE u = 2(wid + j*nwaves) + (i&1)
    auto unit_of = [&](uint32_t i) -> uint32_t {
        return ROWS ? wid + i * nwaves : 2 * (wid + (i >> 1) * nwaves) + (i & 1);
    };
    // TOP: the lane's 4 best keys (ascending) and the score of the 4th (-inf until it has 4)
    uint64_t tk[4] = {kKeyNone, kKeyNone, kKeyNone, kKeyNone};
    float tk3 = -INFINITY;
    const bool live = !TOP || q < p.n_q;  // (TOP: padding queries keep no list)
    if (TOP && blockIdx.x == 0 && threadIdx.x < 16) {
        // (the bookkeeping k_select_tau does on the thresholded path: every query's list is
        // its 4 * gridDim.x slots, the status words of the rescores that follow start at 0)
        p.cnt[threadIdx.x] = 4 * gridDim.x;
        if (threadIdx.x == 0) { p.status[kStFail] = 0; p.status[kStEmitted] = 0; p.status[kStFail2] = 0; }
    }
    // TOP: unit u holds eight strided pairs of rows, 2u, 2u + 1 of each eighth of the corpus
    // (A-row m = row (m >> 1) 2 n_units + 2u + (m & 1)), so a run of consecutive similar rows is
    // spread over consecutive units two at a time, i.e. over different workgroups: no workgroup's 4
    // best come from one cluster of up to ~2 gridDim rows.  The spread costs HBM efficiency: the
    // rows of one load instruction sit in 8 places instead of one 12 KB stretch.  p50 over 10M rows,
    // one process, interleaved (profiles/r06e_p50_top_layouts.txt, r06j_p50_top_layouts.txt):
    // contiguous units as EMIT (lab, p.top_layout = 0) 1.2925 / 1.2944 ms, sixteen strided rows
    // 1.3092, strided pairs 1.3010 / 1.3328, 128-row blocks in 8-row stripes 1.3702, against the
    // thresholded path's 1.3243 / 1.3415.  Contiguous units are fastest, but a run of >= 4 of a
    // query's top rows in one 16-row unit (consecutive chunks of one document) fills a list and
    // sends the batch to the thresholded path: the pairs are kept.
    const bool contig = !TOP || p.top_layout == 0;
    auto row_of = [&](uint32_t u, uint32_t m) -> uint32_t {
        return contig ? u * 16 + m : (m >> 1) * (2 * n_units) + 2 * u + (m & 1);
    };
    // TOP: a lane's output rows 4h + i are two pairs, each in one 32-row scale block: their two
    // scales are loaded with the unit's fragments (prefetched, as the fragments are)
    auto load = [&](i32x4_t (&fa)[NK], float (&fs)[2], uint32_t u) {
        if constexpr (TOP) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint32_t rj = row_of(u, 4 * h + 2 * j);
                fs[j] = p.a_scale[(rj < p.n_rows ? rj : p.n_rows - 1) / kQuantBlock];
            }
        }
        uint32_t r = row_of(u, q);
        r = r < p.n_rows ? r : p.n_rows - 1;  // tail rows: clamped, never emitted
        const uint8_t* a = p.A + (uint64_t)r * p.a_stride + h * 16;
#pragma unroll
        for (int s = 0; s < NK; ++s)
            if (s < (int)nk) {
                if constexpr (EMIT && BSR_SKINNY_NT)  // (lab: the streamed rows marked non-temporal)
                    fa[s] = __builtin_nontemporal_load(reinterpret_cast<const i32x4_t*>(a + s * kSliceB));
                else
                    fa[s] = *reinterpret_cast<const i32x4_t*>(a + s * kSliceB);
            }
    };
    float smax = -INFINITY;  // SAMPLE compact: running maximum of the 32-row block
    auto process = [&](const i32x4_t (&fa)[NK], const float (&fs)[2], uint32_t u) {
        i32x4_acc_t acc = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < NK; ++s)
            if (s < (int)nk) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[s], fb[s], acc, 0, 0, 0);
        // register i: tile row u*16 + 4h + i, query q
        if constexpr (TOP) {
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = ((float)acc[i] * fs[i >> 1]) * sbq;
            const float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
            // (strictly above the lane's 4th: a row at most its 4th stays within the bound; rare
            // once the lane holds 4 keys, ~4 ln(rows / 4) insertions)
            if (live && mx > tk3) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t rw = row_of(u, 4 * h + i);
                    if (v[i] > tk3 && rw < p.n_rows) {
                        top4_insert(tk, score_key(v[i], rw));
                        tk3 = tk[3] == kKeyNone ? -INFINITY : score_key_score(tk[3]);
                    }
                }
            }
        } else if constexpr (EMIT) {
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
                mx = fmaxf(mx, __uint_as_float(xor_lane32<16>(__float_as_uint(mx))));
                mx = fmaxf(mx, __uint_as_float(xor_lane32<32>(__float_as_uint(mx))));
                smax = fmaxf(smax, mx);
                if ((u & 1) && h == 0) srow[u >> 1] = smax;  // second half of the block
                if (u & 1) smax = -INFINITY;
            }
        }
    };
    // this wave's unit count
    uint32_t n_my;
    if (ROWS) {
        n_my = wid < n_units ? (n_units - 1 - wid) / nwaves + 1 : 0;
    } else {
        const uint32_t n_blk = (n_units + 1) / 2;
        n_my = wid < n_blk ? 2 * ((n_blk - 1 - wid) / nwaves + 1) : 0;
    }
    if (n_my) {
        i32x4_t fa0[NK], fa1[NK];
        float fs0[2] = {1.0f, 1.0f}, fs1[2] = {1.0f, 1.0f};
        load(fa0, fs0, unit_of(0));
        for (uint32_t i = 0; i < n_my; i += 2) {
            if (i + 1 < n_my) load(fa1, fs1, unit_of(i + 1));
            process(fa0, fs0, unit_of(i));
            if (i + 1 >= n_my) break;
            if (i + 2 < n_my) load(fa0, fs0, unit_of(i + 2));
            process(fa1, fs1, unit_of(i + 1));
        }
    }
    if constexpr (TOP) {
        // the query's four lanes (h = 0..3: lanes q, q + 16, q + 32, q + 48) merge their lists:
        // partners 16 apart, then 32 -- every lane then holds the wave's 4 best keys of query q
#pragma unroll
        for (int off = 16; off <= 32; off <<= 1) {
            uint64_t o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)tk[j], off, kWave);
                const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(tk[j] >> 32), off, kWave);
                o[j] = ((uint64_t)hi << 32) | lo;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) top4_insert(tk, o[j]);
        }
        // the workgroup's four waves: wave 0 merges the others' lists (LDS) and writes the
        // workgroup's 4 best keys of each query
        __shared__ uint64_t wl[4][16][4];
        if (h == 0)
#pragma unroll
            for (int j = 0; j < 4; ++j) wl[w][q][j] = tk[j];
        __syncthreads();
        if (w == 0 && h == 0) {
#pragma unroll
            for (int o = 1; o < 4; ++o)
#pragma unroll
                for (int j = 0; j < 4; ++j) top4_insert(tk, wl[o][q][j]);
            uint64_t* dst = p.cand + ((uint64_t)q * gridDim.x + blockIdx.x) * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) dst[j] = tk[j];
        }
    }
}

// ------------------------------------------------------------------------------------
// Skinny filter, row modes, with the rows streamed into LDS by LDS-DMA (round 6; the product for
// 768-byte rows).  The same rows, scores and keys as k_filter_skinny2 (EMIT / TOP): each wave keeps a
// ring of SL units in LDS -- a unit's NK K slices (16 rows x 64 B each: lane (row q, piece h) fetches
// exactly the 16 bytes its MFMA fragment needs, so a slice is read back with one ds_read_b128 per
// lane) and the two block scales of the lane's rows -- and refills a unit's slot as soon as its
// fragments are in registers, so SL units stay in flight through the MFMAs and the epilogue.  Two
// waves per workgroup, so the workgroup count -- TOP's list count -- is k_filter_skinny2's, at two
// workgroups per CU (LDS).  Only the B fragments are ordinary loads, consumed before the stream
// starts (an ordinary load's use while LDS-DMA is outstanding makes the compiler drain every DMA).
// One query over 10M rows, one process, interleaved against k_filter_skinny2 (BSR_SKINNY_GLDS=0;
// profiles/r06q_p50glds_*.txt, r06r_*): the self-thresholded path 1.3125 / 1.3143 vs 1.3318 / 1.3310
// ms p50 (filter 1.260 / 1.263 vs 1.279 / 1.280), the thresholded path 1.318 vs 1.340, and 0.2342
// vs 0.2385 ms at the 1.25M-row rank shard.  Two units in flight instead of three: the same.  The
// non-temporal policy (MI355X_MICROARCH.md 'nt-weights', aux = 2) made the filter 16% slower here
// (r06o_*): these rows are not a once-read weight stream the guide measured, each 16-row load
// touching sixteen half lines.
// ------------------------------------------------------------------------------------
#ifndef BSR_SKINNY_GLDS_AUX
#define BSR_SKINNY_GLDS_AUX 0  // (the default policy; 2 = nt: +16% filter time, profiles/r06o_*)
#endif
template <int MODE, int NK>
__global__ __launch_bounds__(128) void k_filter_skinny_glds(GemmArgs p) {
    constexpr bool EMIT = MODE == kSkEmit, TOP = MODE == kSkTop;
    static_assert(EMIT || TOP, "row modes only");
    constexpr int NW = 2, SL = 3, SCB = 512, SLOT = NK * 1024 + SCB, PER = NK + 2;
    __shared__ __attribute__((aligned(1024))) uint8_t ring[NW * SL * SLOT];
    const int lane = threadIdx.x & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t q = lane & 15, h = lane >> 4;
    const uint32_t n_units = (p.n_rows + 15) / 16;
    const uint32_t nwaves = gridDim.x * NW, wid = TOP ? w * gridDim.x + blockIdx.x : blockIdx.x * NW + w;
    const float sbq = p.b_scale[q];
    const float tauq = EMIT ? p.tau[q] : 0.0f;
    i32x4_t fb[NK];
#pragma unroll
    for (int s = 0; s < NK; ++s)
        fb[s] = *reinterpret_cast<const i32x4_t*>(p.B + (uint64_t)q * p.row_bytes + h * 16 + s * kSliceB);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    uint64_t tk[4] = {kKeyNone, kKeyNone, kKeyNone, kKeyNone};
    float tk3 = -INFINITY;
    const bool live = !TOP || q < p.n_q;
    if (TOP && blockIdx.x == 0 && threadIdx.x < 16) {
        p.cnt[threadIdx.x] = 4 * gridDim.x;
        if (threadIdx.x == 0) { p.status[kStFail] = 0; p.status[kStEmitted] = 0; p.status[kStFail2] = 0; }
    }
    const bool contig = !TOP || p.top_layout == 0;
    auto row_of = [&](uint32_t u, uint32_t m) -> uint32_t {
        return contig ? u * 16 + m : (m >> 1) * (2 * n_units) + 2 * u + (m & 1);
    };
    const uint32_t n_rows = p.n_rows;
    uint8_t* const wr = ring + w * (SL * SLOT);
    const uint32_t n_my = wid < n_units ? (n_units - 1 - wid) / nwaves + 1 : 0;
    auto issue = [&](uint32_t i) {
        const uint32_t u = wid + i * nwaves;
        uint8_t* const dst = wr + (i % SL) * SLOT;
        uint32_t r = row_of(u, q);
        r = r < n_rows ? r : n_rows - 1;  // tail rows: clamped, never emitted
        const uint8_t* const src = p.A + (uint64_t)r * p.a_stride + h * 16;
#pragma unroll
        for (int s = 0; s < NK; ++s)
            __builtin_amdgcn_global_load_lds((const void*)(src + s * kSliceB), (lds_void_t*)(dst + s * 1024), 16, 0,
                                             BSR_SKINNY_GLDS_AUX);
        // the block scales of the lane's output rows 4h .. 4h + 3 (TOP: two pairs; EMIT: the unit's)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            uint32_t rj = TOP ? row_of(u, 4 * h + 2 * j) : u * 16;
            rj = rj < n_rows ? rj : n_rows - 1;
            __builtin_amdgcn_global_load_lds((const void*)(p.a_scale + rj / kQuantBlock),
                                             (lds_void_t*)(dst + NK * 1024 + j * 256), 4, 0, BSR_SKINNY_GLDS_AUX);
        }
    };
    // SL units in flight: unit i + SL is issued into unit i's slot as soon as unit i's fragments
    // and scales are in registers, so the stream keeps SL units in flight through the MFMAs and
    // the epilogue
#pragma unroll
    for (uint32_t j = 0; j < (uint32_t)SL; ++j)
        if (j < n_my) issue(j);
    for (uint32_t i = 0; i < n_my; ++i) {
        const uint32_t u = wid + i * nwaves;
        // unit i landed: the units issued after it (at most SL - 1) stay in flight, PER DMAs each
        // (the builtin, not asm: the compiler's own wait counting sees it; vmcnt N: bits 3:0 and
        // 15:14, expcnt and lgkmcnt left at their maxima)
        constexpr int kW2 = ((2 * PER) & 15) | (((2 * PER) >> 4) << 14) | 0x0F70;
        constexpr int kW1 = (PER & 15) | ((PER >> 4) << 14) | 0x0F70;
        static_assert(SL == 3, "the waits below count two younger units");
        if (i + 2 < n_my) __builtin_amdgcn_s_waitcnt(kW2);
        else if (i + 1 < n_my) __builtin_amdgcn_s_waitcnt(kW1);
        else __builtin_amdgcn_s_waitcnt(0x0F70);
        const uint8_t* const src = wr + (i % SL) * SLOT;
        i32x4_t fa[NK];
#pragma unroll
        for (int s = 0; s < NK; ++s) fa[s] = *reinterpret_cast<const i32x4_t*>(src + s * 1024 + lane * 16);
        const float fs0 = reinterpret_cast<const float*>(src + NK * 1024)[lane];
        const float fs1 = reinterpret_cast<const float*>(src + NK * 1024 + 256)[lane];
        // (every read of the slot complete -- lgkmcnt(0), vmcnt and expcnt at their maxima --
        // before the DMA that refills it)
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (i + SL < n_my) issue(i + SL);
        i32x4_acc_t acc = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < NK; ++s) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[s], fb[s], acc, 0, 0, 0);
        // register i: row row_of(u, 4h + i), query q
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = ((float)acc[k] * (k < 2 ? fs0 : fs1)) * sbq;
        const float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
        if constexpr (TOP) {
            if (live && mx > tk3) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t rw = row_of(u, 4 * h + k);
                    if (v[k] > tk3 && rw < n_rows) {
                        top4_insert(tk, score_key(v[k], rw));
                        tk3 = tk[3] == kKeyNone ? -INFINITY : score_key_score(tk[3]);
                    }
                }
            }
        } else {
            if (__ballot(mx >= tauq)) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t row = u * 16 + 4 * h + k;
                    if (v[k] >= tauq && row < n_rows) {
                        const uint32_t gp = atomicAdd(p.cnt + q, 1u);
                        if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = score_key(v[k], row);
                    }
                }
            }
        }
    }
    if constexpr (TOP) {
        // as k_filter_skinny2: the query's four lanes merge, then wave 0 the workgroup's waves
#pragma unroll
        for (int off = 16; off <= 32; off <<= 1) {
            uint64_t o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)tk[j], off, kWave);
                const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(tk[j] >> 32), off, kWave);
                o[j] = ((uint64_t)hi << 32) | lo;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) top4_insert(tk, o[j]);
        }
        __shared__ uint64_t wl[NW][16][4];
        if (h == 0)
#pragma unroll
            for (int j = 0; j < 4; ++j) wl[w][q][j] = tk[j];
        __syncthreads();
        if (w == 0 && h == 0) {
#pragma unroll
            for (int o = 1; o < NW; ++o)
#pragma unroll
                for (int j = 0; j < 4; ++j) top4_insert(tk, wl[o][q][j]);
            uint64_t* dst = p.cand + ((uint64_t)q * gridDim.x + blockIdx.x) * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) dst[j] = tk[j];
        }
    }
}

// ------------------------------------------------------------------------------------
// Threshold per query from the sample scores: tau0 = the ks-th largest value of S (sample
// scores, or their maxima over 32 sampled rows -- never above the ks-th largest sample),
// so that about ks * stride rows of the shard or more reach it.  4 waves per query.  Also
// zeroes the query's candidate counter and (block 0) the emit status words.
// ------------------------------------------------------------------------------------
template <int E>  // ks <= 64 E
__global__ __launch_bounds__(256) void k_select_tau(const float* __restrict__ S, uint32_t s_ld,
                                                    uint32_t n_s, uint32_t nq, uint32_t qpad,
                                                    const uint32_t* __restrict__ qflags,
                                                    uint32_t ks, float* __restrict__ tau,
                                                    uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ status,
                                                    uint64_t* __restrict__ smax) {
    __shared__ uint64_t part[4][64 * E];
    const uint32_t q = blockIdx.x;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (q == 0 && t == 0) { status[kStFail] = 0; status[kStEmitted] = 0; status[kStFail2] = 0; }
    if (q == 0)  // the emit filter's tail counters
        for (uint32_t i = t; i < 8 * kTailCounters + kGangWords; i += blockDim.x) cnt[qpad + i] = 0;
    if (q >= qpad) return;
    if (t == 0) cnt[q] = 0;
    // (smax, the global threshold's input: the query's ks best sample keys, or none)
    if (smax && (q >= nq || (qflags[q] & kQueryNoApprox) || n_s < ks))
        for (uint32_t i = t; i < ks; i += blockDim.x) smax[(uint64_t)q * ks + i] = kKeyNone;
    if (q >= nq || (qflags[q] & kQueryNoApprox)) {
        if (t == 0) tau[q] = INFINITY;  // never emits: answered by the exact scan
        return;
    }
    if (n_s < ks) {
        if (t == 0) tau[q] = -INFINITY;
        return;
    }
    // wave w takes a quarter of the values.  Pass 1: each lane's maximum; the wave's ks-th
    // largest lane maximum is a lower bound lb_w of the query's ks-th largest value (those ks
    // maxima are ks distinct values), and lb = max_w lb_w.  Pass 2 (L2-hot re-read): only
    // values >= lb are offered to the wave's ks best -- a few per wave instead of streaming
    // every batch through the sorted list.
    __shared__ float lbw[4];
    const float* s = S + (uint64_t)q * s_ld;
    const uint32_t per = (n_s + 3) / 4, lo = w * per, hi = lo + per < n_s ? lo + per : n_s;
    constexpr int B = 16;  // loads per lane in flight
    float m = -INFINITY;
    for (uint32_t base = lo; base < hi; base += B * kWave) {
        float v[B];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const uint32_t i = base + j * kWave + lane;
            v[j] = i < hi ? s[i] : -INFINITY;
        }
#pragma unroll
        for (int j = 0; j < B; ++j) m = fmaxf(m, v[j]);
    }
    if (ks <= (uint32_t)kWave) {
        const uint64_t sorted = wave_sort64(score_key(m, (uint32_t)lane));  // ascending key = descending score
        const uint64_t kth = shfl64(sorted, (int)ks - 1);
        if (lane == 0) lbw[w] = score_key_score(kth);
    } else if (lane == 0) {
        lbw[w] = -INFINITY;  // (more than 64 needed: no lower bound from 64 lane maxima)
    }
    __syncthreads();
    const float lb = fmaxf(fmaxf(lbw[0], lbw[1]), fmaxf(lbw[2], lbw[3]));
    WaveTopK<E> L;
    L.init();
    uint64_t thr = kKeyNone;
    for (uint32_t base = lo; base < hi; base += B * kWave) {
        float v[B];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const uint32_t i = base + j * kWave + lane;
            v[j] = i < hi ? s[i] : -INFINITY;
        }
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const uint32_t i = base + j * kWave + lane;
            L.offer(v[j] >= lb ? score_key(v[j], i) : kKeyNone, (int)ks, thr);
        }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) part[w][e * 64 + lane] = L.v[e];
    __syncthreads();
    if (w == 0) {
        WaveTopK<E> M;
        M.init();
        uint64_t mt = kKeyNone;
        for (int src = 0; src < 4; ++src)
#pragma unroll
            for (int e = 0; e < E; ++e) M.offer(part[src][e * 64 + lane], (int)ks, mt);
        if (lane == 0) tau[q] = score_key_score(mt);
        if (smax) M.store(smax + (uint64_t)q * ks, (int)ks);
    }
}

// The same selection for short sample rows (n_s <= 64 NV values, ks <= 64: every shard of up to
// ~2M rows at k <= 10, the shards of an 8-GPU split): ONE wave per query, four per workgroup, the
// whole row in registers -- its lane maxima's ks-th largest as the lower bound, then the offers
// from the same registers (no second read, no workgroup merge, no barrier).  The selection is
// exact either way, so tau and the ks best keys are k_select_tau's, bit for bit.
template <int NV>
__global__ __launch_bounds__(256) void k_select_tau_w(const float* __restrict__ S, uint32_t s_ld, uint32_t n_s,
                                                      uint32_t nq, uint32_t qpad, const uint32_t* __restrict__ qflags,
                                                      uint32_t ks, float* __restrict__ tau, uint32_t* __restrict__ cnt,
                                                      uint32_t* __restrict__ status, uint64_t* __restrict__ smax) {
    const uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int t = threadIdx.x, lane = t & 63;
    if (blockIdx.x == 0 && t == 0) { status[kStFail] = 0; status[kStEmitted] = 0; status[kStFail2] = 0; }
    if (blockIdx.x == 0)  // the emit filter's tail counters
        for (uint32_t i = t; i < 8 * kTailCounters + kGangWords; i += blockDim.x) cnt[qpad + i] = 0;
    if (q >= qpad) return;
    if (lane == 0) cnt[q] = 0;
    const bool none = q >= nq || (qflags[q] & kQueryNoApprox);
    if (smax && (none || n_s < ks))
        for (uint32_t i = lane; i < ks; i += kWave) smax[(uint64_t)q * ks + i] = kKeyNone;
    if (none) {
        if (lane == 0) tau[q] = INFINITY;  // never emits: answered by the exact scan
        return;
    }
    if (n_s < ks) {
        if (lane == 0) tau[q] = -INFINITY;
        return;
    }
    const float* s = S + (uint64_t)q * s_ld;
    float v[NV];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const uint32_t i = j * kWave + lane;
        v[j] = i < n_s ? s[i] : -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) m = fmaxf(m, v[j]);
    // the ks-th largest lane maximum: ks distinct values reach it, so it bounds the ks-th value
    const uint64_t sorted = wave_sort64(score_key(m, (uint32_t)lane));
    const float lb = score_key_score(shfl64(sorted, (int)ks - 1));
    WaveTopK<1> L;
    L.init();
    uint64_t thr = kKeyNone;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const uint32_t i = j * kWave + lane;
        if (j * kWave < (int)n_s) L.offer((i < n_s && v[j] >= lb) ? score_key(v[j], i) : kKeyNone, (int)ks, thr);
    }
    if (lane == 0) tau[q] = score_key_score(thr);
    if (smax) L.store(smax + (uint64_t)q * ks, (int)ks);
}

// The same selection for tiny batches (<= 16 queries: the single-query p50 path) over long sample
// rows (2048 < n_s <= 16 x 64 NV; shorter rows take k_select_tau_w): SIXTEEN waves per query,
// each holding a sixteenth of the row in registers.  The lower bound lb is the largest of the
// waves' ks-th lane maxima (each a lower bound of the query's ks-th value, as above); each wave
// keeps its own ks best among the values >= lb (usually a few), and wave 0 merges the waves' ks
// best.  Exact, so tau and the ks best keys are k_select_tau's, bit for bit
// (tools/microbench/seltau_ab); timed alone at one query over 9766 values, 13.8 us for one 4-wave
// workgroup (tools/microbench/seltau_time).
template <int NV>
__global__ __launch_bounds__(1024) void k_select_tau_m(const float* __restrict__ S, uint32_t s_ld, uint32_t n_s,
                                                       uint32_t nq, uint32_t qpad, const uint32_t* __restrict__ qflags,
                                                       uint32_t ks, float* __restrict__ tau, uint32_t* __restrict__ cnt,
                                                       uint32_t* __restrict__ status, uint64_t* __restrict__ smax) {
    constexpr int NW = 16;
    const uint32_t q = blockIdx.x;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (q == 0 && t == 0) { status[kStFail] = 0; status[kStEmitted] = 0; status[kStFail2] = 0; }
    if (q == 0)  // the emit filter's tail counters
        for (uint32_t i = t; i < 8 * kTailCounters + kGangWords; i += blockDim.x) cnt[qpad + i] = 0;
    if (q >= qpad) return;
    if (t == 0) cnt[q] = 0;
    const bool none = q >= nq || (qflags[q] & kQueryNoApprox);
    if (smax && (none || n_s < ks))
        for (uint32_t i = t; i < ks; i += blockDim.x) smax[(uint64_t)q * ks + i] = kKeyNone;
    if (none) {
        if (t == 0) tau[q] = INFINITY;  // never emits: answered by the exact scan
        return;
    }
    if (n_s < ks) {
        if (t == 0) tau[q] = -INFINITY;
        return;
    }
    __shared__ float lbw[NW];
    __shared__ uint64_t part[NW][kWave];
    const float* s = S + (uint64_t)q * s_ld;
    const uint32_t per = (n_s + NW - 1) / NW, lo = w * per, hi = lo + per < n_s ? lo + per : n_s;
    float v[NV];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const uint32_t i = lo + j * kWave + lane;
        v[j] = i < hi ? s[i] : -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) m = fmaxf(m, v[j]);
    const uint64_t sorted = wave_sort64(score_key(m, (uint32_t)lane));
    const uint64_t kth = shfl64(sorted, (int)ks - 1);  // (every lane: a shuffle reads active lanes only)
    if (lane == 0) lbw[w] = score_key_score(kth);
    __syncthreads();
    float lb = lbw[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) lb = fmaxf(lb, lbw[i]);
    WaveTopK<1> L;
    L.init();
    uint64_t thr = kKeyNone;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const uint32_t i = lo + j * kWave + lane;
        if (lo + j * kWave < hi) L.offer((i < hi && v[j] >= lb) ? score_key(v[j], i) : kKeyNone, (int)ks, thr);
    }
    // each wave's ks best (the query's ks best are among them), packed [w][ks]: wave 0 merges
    // 16 ks keys in batches of 64 (two for ks = 8), not sixteen 64-key lists
    uint64_t* const packed = &part[0][0];
    if (lane < (int)ks) packed[w * ks + lane] = L.v[0];
    __syncthreads();
    if (w != 0) return;
    WaveTopK<1> M;
    M.init();
    uint64_t mt = kKeyNone;
    for (uint32_t b = 0; b < NW * ks; b += kWave) M.offer(b + lane < NW * ks ? packed[b + lane] : kKeyNone, (int)ks, mt);
    if (lane == 0) tau[q] = score_key_score(mt);
    if (smax) M.store(smax + (uint64_t)q * ks, (int)ks);
}

// The global emission threshold of a parallel search: tau[q] = the ks-th best
// of the P ranks' ks best sample keys, all-gathered as g[P][qpad][ks] -- the threshold one
// shard holding every rank's rows would select.  One wave per query, four per workgroup.
template <int E>
__global__ __launch_bounds__(256) void k_global_tau(const uint64_t* __restrict__ g, uint32_t P, uint32_t qpad,
                                                    uint32_t nq, uint32_t ks, const uint32_t* __restrict__ qflags,
                                                    float* __restrict__ tau) {
    const uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (q >= qpad) return;
    if (q >= nq || (qflags[q] & kQueryNoApprox)) {
        if (lane == 0) tau[q] = INFINITY;
        return;
    }
    WaveTopK<E> L;
    L.init();
    uint64_t thr = kKeyNone;
    // the P * ks keys as one flat sequence, 64 per offer (P = 8, ks = 8: one offer, not eight);
    // all of a lane's loads are issued before the first offer
    const uint32_t tot = P * ks;
    constexpr int NB = 8;
    for (uint32_t b = 0; b < tot; b += NB * kWave) {
        uint64_t x[NB];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const uint32_t f = b + u * kWave + lane, r = f / ks, i = f - r * ks;
            x[u] = f < tot ? g[((uint64_t)r * qpad + q) * ks + i] : kKeyNone;
        }
#pragma unroll
        for (int u = 0; u < NB; ++u)
            if (b + u * kWave < tot) L.offer(x[u], (int)ks, thr);
    }
    // (fewer than ks sample keys in the whole corpus: every row is emitted)
    if (lane == 0) tau[q] = thr == kKeyNone ? -INFINITY : score_key_score(thr);
}

// Top-(kp+1) of the emitted candidates by (score desc, row asc); the first kp go to the
// exact rescore, the (kp+1)-th score bounds every row left out.  One wave per query.
template <int E>
__global__ __launch_bounds__(64) void k_select_cand(const uint64_t* __restrict__ cand,
                                                    const uint32_t* __restrict__ cnt, uint32_t cap,
                                                    uint32_t nq, const float* __restrict__ tau,
                                                    uint32_t kp, uint32_t* __restrict__ cand_rows,
                                                    uint32_t* __restrict__ ncand,
                                                    float* __restrict__ tau_excl) {
    const uint32_t q = blockIdx.x;
    if (q >= nq) return;
    const uint32_t c = cnt[q];
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

// ------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------
// Workgroups for the persistent filter: 8 XCDs x (32 CUs rounded down to a multiple of n_qt).
static uint32_t filter_grid(uint32_t n_qt) {
    const uint32_t per_xcd = n_qt >= 32 ? n_qt : (32 / n_qt) * n_qt;
    return 8 * per_xcd;
}

// Filter launches: with timing events, hipExtLaunchKernel records them at the kernel's own
// dispatch and completion; without, a plain launch (also inside stream capture).
#define BSR_KLAUNCH(K, G, B, S, E0, E1, A)                               \
    do {                                                                 \
        if (E0) hipExtLaunchKernelGGL(K, G, B, 0, S, E0, E1, 0u, A);     \
        else hipLaunchKernelGGL(K, G, B, 0, S, A);                       \
    } while (0)

static uint32_t skinny_grid(uint32_t n_rows) {
    const uint32_t groups = (n_rows + 31) / 32, wgs = (groups + 3) / 4;
    return wgs < 768 ? (wgs ? wgs : 1) : 768;  // 3 workgroups per CU (VGPR-limited occupancy)
}
// v2 for rows of <= 16 K steps (1024 int8), v1 beyond.
// v2's grid: 4 waves per workgroup, at most 512 workgroups (~170 VGPRs: 2 waves per SIMD)
static uint32_t skinny2_grid(uint32_t n_rows) {
    const uint32_t units = (n_rows + 15) / 16;
    return std::min<uint32_t>(512, std::max<uint32_t>(1, (units + 3) / 4));
}
uint32_t skinny_top_lists(uint32_t n_rows) { return skinny2_grid(n_rows); }
// The row modes over 768-byte rows take k_filter_skinny_glds (BSR_SKINNY_GLDS=0, read per launch:
// k_filter_skinny2 instead, for A/B runs)
bool skinny_glds_on() {
    const char* v = getenv("BSR_SKINNY_GLDS");
    return !(v && v[0] == '0');
}
template <int MODE>
static void launch_skinny(const GemmArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const uint32_t nk = a.row_bytes / kSliceB;
    if constexpr (MODE != kSkSample) {
        if (nk == 12 && skinny_glds_on()) {
            BSR_KLAUNCH((k_filter_skinny_glds<MODE, 12>), dim3(skinny2_grid(a.n_rows)), dim3(128), s, e0, e1, a);
            return;
        }
    }
    const dim3 g(nk <= 16 ? skinny2_grid(a.n_rows) : skinny_grid(a.n_rows)), b(256);
    if (nk <= 4) BSR_KLAUNCH((k_filter_skinny2<MODE, 4>), g, b, s, e0, e1, a);
    else if (nk <= 8) BSR_KLAUNCH((k_filter_skinny2<MODE, 8>), g, b, s, e0, e1, a);
    else if (nk <= 12) BSR_KLAUNCH((k_filter_skinny2<MODE, 12>), g, b, s, e0, e1, a);
    else if (nk <= 16) BSR_KLAUNCH((k_filter_skinny2<MODE, 16>), g, b, s, e0, e1, a);
    else if constexpr (MODE != kSkTop) BSR_KLAUNCH(k_filter_skinny<MODE == kSkEmit>, g, b, s, e0, e1, a);
}
hipError_t launch_filter_skinny_sample(const GemmArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    launch_skinny<kSkSample>(a, s, e0, e1);
    return hipGetLastError();
}
hipError_t launch_filter_skinny_emit(const GemmArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    launch_skinny<kSkEmit>(a, s, e0, e1);
    return hipGetLastError();
}
hipError_t launch_filter_skinny_top(const GemmArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if (a.row_bytes / kSliceB > 16) return hipErrorInvalidValue;  // (v2 widths only: the caller checks)
    launch_skinny<kSkTop>(a, s, e0, e1);
    return hipGetLastError();
}

// int8 rows of an even number of 64-byte slices up to 12 (dims <= 768): the query-stationary
// kernel; other widths: k_filter.  (A one-wave-per-SIMD variant
// with 64 queries per wave, tools/microbench/k_qs64_lab.hip, measured slower: DESIGN.md §5.)
// Whether any workgroup of the emit filter can run in a row-stream gang (k_filter_qs16's `gang`
// condition with its longest static stream).  Otherwise -- every shard of up to ~5.6M rows at 1000
// queries, and configs[4]'s 16 query tiles -- the launch takes the small-shard build: no gang code
// (GANG = 0), level 2's bool-array form (L2 = 1) and no explicit wait in the flush (FW = 0): 3-4%
// faster than the gang build at 1M and 1.25M rows with emission, the same at tau = inf
// (tools/microbench/filter_hist, profiles/r05c_hist_*, r05e_hist_*).  Round 6: its dynamic tail in
// the XCD-local pools (TAILX = 8, as the gang build) instead of one counter per query tile -- HBM
// fetch at the 1.25M-row shard 1.25x -> 1.005x the int8 rows, time within 0.4%
// (profiles/r06b_fab_125.txt, r06b_fabpmc_1250000.txt: variants "small" / "smallx").  At 10M the
// gang build stays: its HBM traffic is 1.1x the rows instead of 2x.
static bool gang_possible(const GemmArgs& a, uint32_t grid) {
    if (!a.tail || a.n_qt < 2 || a.n_qt > 4) return false;
    const uint32_t G = (grid / 8) / a.n_qt, RG = 8 * G;
    const uint32_t n_rt = (a.n_rows + 127) / 128, n_st = n_rt - n_rt / 8;  // (TAILX = 8)
    return RG && n_st && (n_st - 1) / RG + 1 >= kGangMinTiles;
}

template <bool EMIT>
static void launch_filter(const GemmArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const uint32_t nk = a.row_bytes / kSliceB, grid = filter_grid(a.n_qt);
    if (nk % 2 == 0 && nk <= 12) {
        const dim3 g(grid), b(512);
        if (EMIT && nk == 12 && !gang_possible(a, grid)) {
            BSR_KLAUNCH((k_filter_qs16<EMIT, 12, 0, 8, 0, 0, 1, 0>), g, b, s, e0, e1, a);
            return;
        }
        switch (nk) {
            case 2: BSR_KLAUNCH((k_filter_qs16<EMIT, 2>), g, b, s, e0, e1, a); return;
            case 4: BSR_KLAUNCH((k_filter_qs16<EMIT, 4>), g, b, s, e0, e1, a); return;
            case 6: BSR_KLAUNCH((k_filter_qs16<EMIT, 6>), g, b, s, e0, e1, a); return;
            case 8: BSR_KLAUNCH((k_filter_qs16<EMIT, 8>), g, b, s, e0, e1, a); return;
            case 10: BSR_KLAUNCH((k_filter_qs16<EMIT, 10>), g, b, s, e0, e1, a); return;
            default: BSR_KLAUNCH((k_filter_qs16<EMIT, 12>), g, b, s, e0, e1, a); return;
        }
    }
    BSR_KLAUNCH((k_filter<OpI8, EMIT>), dim3(grid), dim3(kThreads), s, e0, e1, a);
}
hipError_t launch_filter_sample(const GemmArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    launch_filter<false>(a, s, e0, e1);
    return hipGetLastError();
}
hipError_t launch_filter_emit(const GemmArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    launch_filter<true>(a, s, e0, e1);
    return hipGetLastError();
}
hipError_t launch_select_tau(const float* S, uint32_t s_ld, uint32_t n_s, uint32_t nq, uint32_t qpad,
                             const uint32_t* qflags, uint32_t ks, float* tau, uint32_t* cnt, uint32_t* status,
                             hipStream_t s, uint64_t* smax) {
    if (ks > 2 * kWave) return hipErrorInvalidValue;
    // (BSR_SELECT_TAU_M=0: the 4-wave kernel instead; =2 (lab): the 16-wave kernel for every batch
    // size, for A/B runs)
    static const int m_on = [] {
        const char* v = getenv("BSR_SELECT_TAU_M");
        return v && v[0] == '0' ? 0 : v && v[0] == '2' ? 2 : 1;
    }();
    if (m_on && ks <= kWave && (qpad <= 16 || m_on == 2) && n_s > 32 * kWave && n_s <= 16 * 16 * kWave)
        hipLaunchKernelGGL(k_select_tau_m<16>, dim3(qpad), dim3(1024), 0, s, S, s_ld, n_s, nq, qpad, qflags, ks,
                           tau, cnt, status, smax);
    else if (ks <= kWave && n_s <= 32 * kWave && qpad % 4 == 0)
        hipLaunchKernelGGL(k_select_tau_w<32>, dim3(qpad / 4), dim3(256), 0, s, S, s_ld, n_s, nq, qpad, qflags, ks,
                           tau, cnt, status, smax);
    else if (ks > kWave)
        hipLaunchKernelGGL(k_select_tau<2>, dim3(qpad), dim3(256), 0, s, S, s_ld, n_s, nq, qpad, qflags, ks, tau,
                           cnt, status, smax);
    else
        hipLaunchKernelGGL(k_select_tau<1>, dim3(qpad), dim3(256), 0, s, S, s_ld, n_s, nq, qpad, qflags, ks, tau,
                           cnt, status, smax);
    return hipGetLastError();
}
hipError_t launch_global_tau(const uint64_t* g, uint32_t P, uint32_t qpad, uint32_t nq, uint32_t ks,
                             const uint32_t* qflags, float* tau, hipStream_t s) {
    if (ks > 2 * kWave || P == 0) return hipErrorInvalidValue;
    if (ks > kWave)
        hipLaunchKernelGGL(k_global_tau<2>, dim3(qpad / 4), dim3(256), 0, s, g, P, qpad, nq, ks, qflags, tau);
    else
        hipLaunchKernelGGL(k_global_tau<1>, dim3(qpad / 4), dim3(256), 0, s, g, P, qpad, nq, ks, qflags, tau);
    return hipGetLastError();
}
hipError_t launch_select_cand(const uint64_t* cand, const uint32_t* cnt, uint32_t cap, uint32_t nq,
                              const float* tau, uint32_t kp, uint32_t* cand_rows, uint32_t* ncand,
                              float* tau_excl, hipStream_t s) {
    const uint32_t e = (kp + 1 + 63) / 64;
#define BSR_SELECT(E)                                                                                   \
    hipLaunchKernelGGL(k_select_cand<E>, dim3(nq), dim3(64), 0, s, cand, cnt, cap, nq, tau, kp, cand_rows, \
                       ncand, tau_excl)
    switch (e) {
        case 1: BSR_SELECT(1); break;
        case 2: BSR_SELECT(2); break;
        case 3: BSR_SELECT(3); break;
        case 4: BSR_SELECT(4); break;
        case 5: BSR_SELECT(5); break;
        case 6: BSR_SELECT(6); break;
        case 7: BSR_SELECT(7); break;
        case 8: BSR_SELECT(8); break;
        case 9: BSR_SELECT(9); break;
        case 10: BSR_SELECT(10); break;
        default: return hipErrorInvalidValue;
    }
#undef BSR_SELECT
    return hipGetLastError();
}

}  // namespace bsr
