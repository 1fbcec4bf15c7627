// kernels.hip -- gfx950 (MI355X, CDNA4) kernels for the exact cosine top-k search path.
//
// Compiled with -ffp-contract=off: in every kernel that reproduces the reference's
// arithmetic (norms, exact scan, rescore, pair distance) each f32 multiply and add rounds
// separately, in index order, exactly as src/metrics.rs:153-155 does.  The MFMA filter is
// the only reordered arithmetic and it never produces a returned distance: it only selects
// candidates, whose exact distances are then recomputed sequentially.
#include "bsr_device.hpp"
#include "kernels.hpp"

#include <math.h>
#include <stdlib.h>

namespace bsr {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((address_space(3))) void lds_void_t;

// ------------------------------------------------------------------------------------
// Synthetic data: value(row, col) = U[-1,1) from splitmix64(seed, row*dim + col), 24 bits.
// ------------------------------------------------------------------------------------
__global__ void k_synth_uniform(float* __restrict__ out, uint64_t row0, uint64_t n_rows,
                                uint32_t dim, uint32_t ld, uint64_t seed) {
    const uint64_t total = n_rows * (uint64_t)ld;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = e / ld;
        const uint32_t c = (uint32_t)(e - r * ld);
        float v = 0.0f;
        if (c < dim) {
            const uint64_t g = (row0 + r) * (uint64_t)dim + c;
            const uint64_t h = splitmix64(seed * 0xD1B54A32D192ED03ull + g);
            v = (float)(h >> 40) * (1.0f / 8388608.0f) - 1.0f;  // 24-bit grid on [-1, 1)
        }
        out[e] = v;
    }
}

// Dense copy into the padded [n][ld] layout (zeros in the pad columns).
__global__ void k_copy_rows_f32(const float* __restrict__ src, uint64_t n, uint32_t dim,
                                uint32_t ld, float* __restrict__ dst) {
    const uint64_t total = n * (uint64_t)ld;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = e / ld;
        const uint32_t c = (uint32_t)(e - r * ld);
        dst[e] = c < dim ? src[r * dim + c] : 0.0f;
    }
}

__global__ void k_widen_bf16_rows(const uint16_t* __restrict__ src, uint64_t n, uint32_t dim,
                                  uint32_t ld, float* __restrict__ dst) {
    const uint64_t total = n * (uint64_t)ld;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = e / ld;
        const uint32_t c = (uint32_t)(e - r * ld);
        dst[e] = c < dim ? bf16_to_f32(src[r * dim + c]) : 0.0f;
    }
}

__global__ void k_check_finite(const float* __restrict__ x, uint64_t count, uint32_t* flag) {
    bool bad = false;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < count;
         e += (uint64_t)gridDim.x * blockDim.x)
        bad |= !isfinite(x[e]);
    if (__ballot(bad) && lane_id() == 0) atomicOr(flag, 1u);
}

// ------------------------------------------------------------------------------------
// Row magnitudes exactly as src/metrics.rs:154: sqrt of the sequential f32 sum of a_i*a_i.
// One lane per row; the per-row dependency chain is inherently serial.
// ------------------------------------------------------------------------------------
__global__ void k_row_norms(const float* __restrict__ rows, uint64_t n, uint32_t dim,
                            uint32_t ld, float* __restrict__ na, uint32_t* flags) {
    const uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint32_t f = 0;
    if (r < n) {
        const float* a = rows + r * ld;
        float acc = -0.0f;
        bool bad = false;
        uint32_t i = 0;
        for (; i + 4 <= dim; i += 4) {
            const float4 x = *reinterpret_cast<const float4*>(a + i);
            bad = bad || !isfinite(x.x) || !isfinite(x.y) || !isfinite(x.z) || !isfinite(x.w);
            acc = acc + x.x * x.x;
            acc = acc + x.y * x.y;
            acc = acc + x.z * x.z;
            acc = acc + x.w * x.w;
        }
        for (; i < dim; ++i) {
            const float x = a[i];
            bad |= !isfinite(x);
            acc = acc + x * x;
        }
        const float m = __builtin_sqrtf(acc);
        na[r] = m;
        if (bad) f |= kRowNonFinite;
        if (!isfinite(m)) f |= kRowNormOvf;
        if (m != 0.0f && (m < 1e-18f || m > 1e18f)) f |= kRowNormRange;
    }
    const uint32_t any = __reduce_or_sync(~0ull, f);
    if (any && lane_id() == 0) atomicOr(flags, any);
}

// Normalised bf16 copy for the MFMA filter: bf16_rne(a_i / |a|), zero rows / pad -> 0.
// Each thread writes 8 consecutive elements (16 B).
__global__ void k_rows_to_bf16n(const float* __restrict__ rows, const float* __restrict__ na,
                                uint64_t n, uint64_t n_pad, uint32_t dim, uint32_t ld,
                                uint16_t* __restrict__ out) {
    const uint64_t groups = n_pad * (uint64_t)(ld / 8);
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = g / (ld / 8);
        const uint32_t c0 = (uint32_t)(g - r * (ld / 8)) * 8;
        uint16_t h[8];
        const float m = r < n ? na[r] : 0.0f;
        const bool ok = r < n && m != 0.0f && isfinite(m);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t c = c0 + j;
            h[j] = (ok && c < dim) ? f32_to_bf16_rne(rows[r * ld + c] / m) : (uint16_t)0;
        }
        uint4 v;
        v.x = h[0] | ((uint32_t)h[1] << 16);
        v.y = h[2] | ((uint32_t)h[3] << 16);
        v.z = h[4] | ((uint32_t)h[5] << 16);
        v.w = h[6] | ((uint32_t)h[7] << 16);
        *reinterpret_cast<uint4*>(out + r * ld + c0) = v;
    }
}

// Query magnitudes exactly as src/metrics.rs:155 (lane per query, sequential f32 sum of
// squares from the caller's rows), finiteness, and eligibility for the MFMA filter.
__global__ __launch_bounds__(64) void k_query_norms(const float* __restrict__ q, uint32_t nq, uint32_t qpad,
                                                    uint32_t dim, float* __restrict__ nb,
                                                    uint32_t* __restrict__ qflags) {
    const uint32_t qi = blockIdx.x * 64 + threadIdx.x;
    if (qi >= qpad) return;
    if (qi >= nq) {
        nb[qi] = 0.0f;
        qflags[qi] = kQueryNoApprox;
        return;
    }
    const float* b = q + (uint64_t)qi * dim;
    float acc = -0.0f;
    bool bad = false;
    for (uint32_t i = 0; i < dim; ++i) {
        const float x = b[i];
        bad = bad || !isfinite(x);
        acc = acc + x * x;
    }
    const float m = __builtin_sqrtf(acc);
    nb[qi] = m;
    const bool approx_ok = !bad && isfinite(m) && m >= 1e-18f && m <= 1e18f;
    qflags[qi] = (bad ? kQueryNonFinite : 0u) | (approx_ok ? 0u : kQueryNoApprox);
}

// Padded f32 copy [qpad][ld] and normalised bf16 copy (zeros where not eligible / pad).
__global__ void k_query_convert(const float* __restrict__ q, uint32_t nq, uint32_t qpad, uint32_t dim,
                                uint32_t ld, const float* __restrict__ nb,
                                const uint32_t* __restrict__ qflags, float* __restrict__ qf32,
                                uint16_t* __restrict__ qbf) {
    const uint64_t total = (uint64_t)qpad * ld;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t qi = (uint32_t)(e / ld), c = (uint32_t)(e - (uint64_t)qi * ld);
        const float v = (qi < nq && c < dim) ? q[(uint64_t)qi * dim + c] : 0.0f;
        qf32[e] = v;
        const bool ok = qi < nq && c < dim && !(qflags[qi] & kQueryNoApprox);
        qbf[e] = ok ? f32_to_bf16_rne(v / nb[qi]) : (uint16_t)0;
    }
}

// ------------------------------------------------------------------------------------
// MFMA filter: S~[r][q] = sum_k bf16(a_rk/|a_r|) * bf16(b_qk/|b_q|) on
// v_mfma_f32_32x32x16_bf16.  Tile 128 rows x 128 queries x 64-deep K steps; 4 waves, each
// 64x64 = 2x2 MFMA blocks.  Operands staged global->LDS with global_load_lds_dwordx4 into
// two LDS buffers; the 16-B chunk of each 128-B LDS row is XOR-swizzled by (row>>1)&7 on
// the SOURCE address (LDS-DMA writes lane-linearly), which makes every ds_read_b128 of the
// fragments conflict-free.  Lane l of an MFMA holds A[row l&31][k 8(l>>5)..+7] and
// B[k..][query l&31]; the accumulator holds query l&31 and rows (r&3)+8(r>>2)+4(l>>5).
// Epilogue: SAMPLE stores the scores densely; EMIT appends (score, row) keys whose score
// reaches the query's threshold tau to a per-query candidate list.
// ------------------------------------------------------------------------------------
template <bool EMIT>
__global__ __launch_bounds__(256, 2) void k_gemm_filter(GemmArgs p) {
    constexpr int BM = kGemmBM, BN = kGemmBN, BK = 64;
    constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB (BM == BN)
    __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * 2 * TILE_BYTES];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;

    // XCD-aware bijective remap: the blocks that share an XCD (b % 8) take consecutive
    // tiles, so the n_qt query tiles of one corpus row tile run on one L2.
    const uint32_t nwg = gridDim.x, b = blockIdx.x;
    const uint32_t xcd = b & 7, loc = b >> 3, q8 = nwg >> 3, r8 = nwg & 7;
    const uint32_t tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const uint32_t rt = tile / p.n_qt, qt = tile - rt * p.n_qt;

    // Per-lane LDS-DMA sources: instruction i of wave w fills LDS rows (4w+i)*8 + lane/8,
    // physical chunk lane&7, with logical chunk (lane&7) ^ ((row>>1)&7).
    const uint16_t* asrc[4];
    const uint16_t* bsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = (w * 4 + i) * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ ((row >> 1) & 7);
        uint32_t arow = rt * BM + row;
        if (!EMIT && arow >= p.n_rows) arow = p.n_rows - 1;  // sample tail: clamp, ignored later
        asrc[i] = p.A + (uint64_t)arow * p.a_row_stride + lc * 8;
        bsrc[i] = p.B + (uint64_t)(qt * BN + row) * p.ld + lc * 8;
    }
    auto stage = [&](int s, int kt) {
        uint8_t* la = lds + (s * 2 + 0) * TILE_BYTES;
        uint8_t* lb = lds + (s * 2 + 1) * TILE_BYTES;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + kt * BK),
                                             (lds_void_t*)(la + (w * 4 + i) * 1024), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + kt * BK),
                                             (lds_void_t*)(lb + (w * 4 + i) * 1024), 16, 0, 0);
    };

    // Fragment read offsets (bytes within a tile) for k-substep kk: row*128 + pc*16.
    int aoff[2][4], boff[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int arow = wr * 64 + m * 32 + (lane & 31);
        const int brow = wc * 64 + m * 32 + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int lc = 2 * kk + (lane >> 5);
            aoff[m][kk] = arow * 128 + ((lc ^ ((arow >> 1) & 7)) * 16);
            boff[m][kk] = brow * 128 + ((lc ^ ((brow >> 1) & 7)) * 16);
        }
    }

    f32x16_t acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.0f;

    const int nk = (int)(p.ld / BK);
    stage(0, 0);
    __syncthreads();  // emits vmcnt(0): the LDS-DMA of stage 0 has landed
    for (int kt = 0; kt < nk; ++kt) {
        const int s = kt & 1;
        if (kt + 1 < nk) stage(s ^ 1, kt + 1);
        const uint8_t* la = lds + (s * 2 + 0) * TILE_BYTES;
        const uint8_t* lb = lds + (s * 2 + 1) * TILE_BYTES;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            bf16x8_t af[2], bfr[2];
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                af[m] = *reinterpret_cast<const bf16x8_t*>(la + aoff[m][kk]);
                bfr[m] = *reinterpret_cast<const bf16x8_t*>(lb + boff[m][kk]);
            }
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int n = 0; n < 2; ++n)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
        }
        __syncthreads();  // next stage landed (vmcnt(0)) and this stage fully read
    }

#pragma unroll
    for (int m = 0; m < 2; ++m) {
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            const uint32_t q = qt * BN + wc * 64 + n * 32 + (lane & 31);
            const uint32_t rbase = rt * BM + wr * 64 + m * 32 + 4 * (lane >> 5);
            if constexpr (!EMIT) {
                float* dst = p.S + (uint64_t)q * p.s_ld + rbase;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    float4 v = make_float4(acc[m][n][4 * g], acc[m][n][4 * g + 1],
                                           acc[m][n][4 * g + 2], acc[m][n][4 * g + 3]);
                    *reinterpret_cast<float4*>(dst + 8 * g) = v;
                }
            } else {
                const float tau = p.tau[q];
                float mx = acc[m][n][0];
#pragma unroll
                for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[m][n][r]);
                if (__ballot(mx >= tau)) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float v = acc[m][n][r];
                        const uint32_t row = rbase + (r & 3) + 8 * (r >> 2);
                        if (v >= tau && row < p.n_rows) {
                            const uint32_t pos = atomicAdd(p.cnt + q, 1u);
                            if (pos < p.cap) p.cand[(uint64_t)q * p.cap + pos] = score_key(v, row);
                        }
                    }
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// MFMA filter v2 (persistent): 256 corpus rows x 256 queries per tile, 8 waves (2 x 4),
// each wave 128 x 64 = 4 x 2 blocks of v_mfma_f32_32x32x16_bf16 (128 accumulator VGPRs).
// Operand feed per 64-deep K step: 64 KiB by global_load_lds_dwordx4 into the other half
// of a 2 x (32 + 32) KiB LDS ring, overlapping the 32 MFMAs per wave on the current half;
// one barrier per K step.  The (row tile, K step) loop is flattened so the next tile's
// first K step is staged during the current tile's last one.  A workgroup keeps ONE query
// tile for its whole life (thresholds stay in registers, no global load in the loop) and
// walks row tiles g, g+G, ...; the n_qt workgroups that share a row tile share an XCD
// (blockIdx % 8), so the tile comes from HBM once per XCD.  Candidates go to an LDS buffer
// (ds_add_rtn; no vmcnt in the loop) and are flushed to global lists once at the end.
// ------------------------------------------------------------------------------------
constexpr int kG2BM = 256, kG2BN = 256, kG2BK = 64;
constexpr int kG2Threads = 512;
constexpr int kG2Cap = 2048;  // LDS candidate buffer entries per workgroup

// VAR (tooling ablations, tools/microbench/gemm_ablate.hip): 0 = product; 1 = no LDS-DMA in
// the loop (compute ceiling); 2 = no MFMA (operand-feed ceiling).
template <bool EMIT, int VAR = 0>
__global__ __launch_bounds__(512, 2) void k_gemm_filter2(GemmArgs p) {
    constexpr int BM = kG2BM, BN = kG2BN, BK = kG2BK;
    constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;  // 32 KiB each
    constexpr int STAGE = A_BYTES + B_BYTES;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * STAGE + (EMIT ? kG2Cap * 10 + 16 : 0)];
    uint64_t* ekeys = reinterpret_cast<uint64_t*>(lds + 2 * STAGE);
    uint16_t* eq = reinterpret_cast<uint16_t*>(lds + 2 * STAGE + kG2Cap * 8);
    uint32_t* ecnt = reinterpret_cast<uint32_t*>(lds + 2 * STAGE + kG2Cap * 10);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 2, wc = w & 3;

    // Work assignment (see above).  G row groups per XCD, n_qt workgroups per group.
    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const uint32_t nk = p.ld / BK;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * nk;

    if (EMIT && tid == 0) *ecnt = 0;

    // LDS-DMA sources: instruction i (0..3) of wave w fills LDS rows (4w+i)*8 + lane/8 of
    // the A and of the B half, physical 16-B chunk lane&7 <- logical chunk ^ ((row>>1)&7).
    uint32_t lrow[4], lchunk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        lrow[i] = (w * 4 + i) * 8 + (lane >> 3);
        lchunk[i] = (lane & 7) ^ ((lrow[i] >> 1) & 7);
    }
    const uint16_t* bsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bsrc[i] = p.B + (uint64_t)(qt * BN + lrow[i]) * p.ld + lchunk[i] * 8;
    auto stage = [&](uint32_t jj) {
        const uint32_t ti = jj / nk, kt = jj - ti * nk;
        const uint32_t rt = g0 + ti * RG;
        uint8_t* la = lds + (jj & 1) * STAGE;
        uint8_t* lb = la + A_BYTES;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t arow = rt * BM + lrow[i];
            if (!EMIT && arow >= p.n_rows) arow = p.n_rows - 1;  // sample tail (ignored later)
            const uint16_t* src = p.A + (uint64_t)arow * p.a_row_stride + lchunk[i] * 8 + kt * BK;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(la + (w * 4 + i) * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + kt * BK),
                                             (lds_void_t*)(lb + (w * 4 + i) * 1024), 16, 0, 0);
    };

    int aoff[4][4], boff[2][4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int row = wr * 128 + m * 32 + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int lc = 2 * kk + (lane >> 5);
            aoff[m][kk] = row * 128 + ((lc ^ ((row >> 1) & 7)) * 16);
        }
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int row = wc * 64 + n * 32 + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int lc = 2 * kk + (lane >> 5);
            boff[n][kk] = A_BYTES + row * 128 + ((lc ^ ((row >> 1) & 7)) * 16);
        }
    }
    float tau[2] = {0.0f, 0.0f};
    if (EMIT) {
#pragma unroll
        for (int n = 0; n < 2; ++n) tau[n] = p.tau[qt * BN + wc * 64 + n * 32 + (lane & 31)];
    }

    f32x16_t acc[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.0f;

    if (J) stage(0);
    __syncthreads();  // stage 0 landed (vmcnt(0)); ecnt visible
    uint32_t ti = 0, kt = 0;
    for (uint32_t jj = 0; jj < J; ++jj) {
        if (VAR != 1 && jj + 1 < J) stage(jj + 1);
        const uint8_t* base = lds + (VAR == 1 ? 0 : (jj & 1)) * STAGE;
#pragma unroll
        for (int kk = 0; kk < (VAR == 3 ? 0 : 4); ++kk) {
            bf16x8_t af[4], bfr[2];
#pragma unroll
            for (int m = 0; m < 4; ++m) af[m] = *reinterpret_cast<const bf16x8_t*>(base + aoff[m][kk]);
#pragma unroll
            for (int n = 0; n < 2; ++n) bfr[n] = *reinterpret_cast<const bf16x8_t*>(base + boff[n][kk]);
            if constexpr (VAR == 2) {
#pragma unroll
                for (int m = 0; m < 4; ++m) acc[m][0][0] += (float)af[m][0] + (float)bfr[m & 1][0];
            } else {
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int n = 0; n < 2; ++n)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
            }
        }
        if (kt == nk - 1) {
            const uint32_t rt = g0 + ti * RG;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    const uint32_t ql = wc * 64 + n * 32 + (lane & 31);
                    const uint32_t rbase = rt * BM + wr * 128 + m * 32 + 4 * (lane >> 5);
                    if constexpr (!EMIT) {
                        float* dst = p.S + (uint64_t)(qt * BN + ql) * p.s_ld + rbase;
#pragma unroll
                        for (int g = 0; g < 4; ++g)
                            *reinterpret_cast<float4*>(dst + 8 * g) =
                                make_float4(acc[m][n][4 * g], acc[m][n][4 * g + 1], acc[m][n][4 * g + 2],
                                            acc[m][n][4 * g + 3]);
                    } else {
                        float mx = acc[m][n][0];
#pragma unroll
                        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[m][n][r]);
                        if (__ballot(mx >= tau[n])) {
#pragma unroll
                            for (int r = 0; r < 16; ++r) {
                                const float v = acc[m][n][r];
                                const uint32_t row = rbase + (r & 3) + 8 * (r >> 2);
                                if (v >= tau[n] && row < p.n_rows) {
                                    const uint32_t pos = atomicAdd(ecnt, 1u);
                                    if (pos < (uint32_t)kG2Cap) {
                                        ekeys[pos] = score_key(v, row);
                                        eq[pos] = (uint16_t)ql;
                                    } else {  // LDS buffer full: straight to the global list
                                        const uint32_t q = qt * BN + ql;
                                        const uint32_t gp = atomicAdd(p.cnt + q, 1u);
                                        if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = score_key(v, row);
                                    }
                                }
                            }
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.0f;
                }
            }
            kt = 0;
            ++ti;
        } else {
            ++kt;
        }
        __syncthreads();  // next stage landed (vmcnt(0)); this stage fully read
    }
    if constexpr (EMIT) {
        const uint32_t ne = *ecnt < (uint32_t)kG2Cap ? *ecnt : (uint32_t)kG2Cap;
        for (uint32_t i = tid; i < ne; i += kG2Threads) {
            const uint32_t q = qt * BN + eq[i];
            const uint32_t gp = atomicAdd(p.cnt + q, 1u);
            if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = ekeys[i];
        }
    }
}

// ------------------------------------------------------------------------------------
// MFMA filter v3: v2's persistent 256 x 256 tile and work assignment, but the operand feed
// is a 4-slot LDS ring of 32-deep K slices (A 256x32 + B 256x32 bf16 = 32 KiB per slot)
// with THREE slices in flight: slice j+3 is issued while slice j is multiplied, and the
// end-of-slice wait is a counted `s_waitcnt vmcnt(8)` (the 8 younger LDS-DMA of slices
// j+2, j+3 stay in flight) followed by a raw s_barrier -- __syncthreads() would drain
// vmcnt to 0.  64-B LDS rows: physical 16-B chunk = logical ^ ((row >> 2) & 3), which
// makes the ds_read_b128 fragment reads conflict-free.
// ------------------------------------------------------------------------------------
constexpr int kG3Slots = 4, kG3BK = 32;

__device__ __forceinline__ void wait_vm8_barrier() {
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

constexpr int kG3WCap = 256;  // candidate buffer entries per wave

template <bool EMIT, int VAR = 0>
__global__ __launch_bounds__(512, 2) void k_gemm_filter3(GemmArgs p) {
    constexpr int BM = kG2BM, BN = kG2BN, BK = kG3BK;
    constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;  // 16 KiB each
    constexpr int SLOT = A_BYTES + B_BYTES;                       // 32 KiB
    // Candidate buffer: a private region per wave (kG3WCap entries), positions from
    // ballot + mbcnt -- no LDS atomics (the compiler would drain vmcnt before them).
    __shared__ __attribute__((aligned(1024))) uint8_t lds[kG3Slots * SLOT + (EMIT ? 8 * kG3WCap * 12 : 0)];
    const int w_ = threadIdx.x >> 6;
    uint64_t* ekeys = reinterpret_cast<uint64_t*>(lds + kG3Slots * SLOT) + w_ * kG3WCap;
    uint32_t* eq = reinterpret_cast<uint32_t*>(lds + kG3Slots * SLOT + 8 * kG3WCap * 8) + w_ * kG3WCap;
    uint32_t ecount = 0;  // wave-uniform

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 2, wc = w & 3;

    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const uint32_t nk = p.ld / BK;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * nk;

    // LDS-DMA: per slot each wave issues 2 instructions for A and 2 for B; instruction i
    // fills 16 rows x 64 B: rows (2w+i)*16 + lane/4, physical chunk lane&3.
    uint32_t lrow[2], lchunk[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        lrow[i] = (w * 2 + i) * 16 + (lane >> 2);
        lchunk[i] = (lane & 3) ^ ((lrow[i] >> 2) & 3);
    }
    const uint16_t* bsrc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) bsrc[i] = p.B + (uint64_t)(qt * BN + lrow[i]) * p.ld + lchunk[i] * 8;
    // Slice jj -> (row tile, k slice) tracked incrementally for the issue pointer.
    uint32_t iss_ti = 0, iss_kt = 0;
    auto issue = [&](uint32_t jj) {
        const uint32_t rt = g0 + iss_ti * RG;
        uint8_t* la = lds + (jj % kG3Slots) * SLOT;
        uint8_t* lb = la + A_BYTES;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            uint32_t arow = rt * BM + lrow[i];
            if (!EMIT && arow >= p.n_rows) arow = p.n_rows - 1;
            const uint16_t* src = p.A + (uint64_t)arow * p.a_row_stride + lchunk[i] * 8 + iss_kt * BK;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(la + (w * 2 + i) * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + iss_kt * BK),
                                             (lds_void_t*)(lb + (w * 2 + i) * 1024), 16, 0, 0);
        if (++iss_kt == nk) { iss_kt = 0; ++iss_ti; }
    };

    int aoff[4][2], boff[2][2];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int row = wr * 128 + m * 32 + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int lc = 2 * kk + (lane >> 5);
            aoff[m][kk] = row * 64 + ((lc ^ ((row >> 2) & 3)) * 16);
        }
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int row = wc * 64 + n * 32 + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int lc = 2 * kk + (lane >> 5);
            boff[n][kk] = A_BYTES + row * 64 + ((lc ^ ((row >> 2) & 3)) * 16);
        }
    }
    float tau[2] = {0.0f, 0.0f};
    if (EMIT) {
#pragma unroll
        for (int n = 0; n < 2; ++n) tau[n] = p.tau[qt * BN + wc * 64 + n * 32 + (lane & 31)];
    }

    f32x16_t acc[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.0f;

    // Prologue: slices 0..2 in flight (issue() for slices past J re-loads slice J-1's
    // addresses harmlessly is NOT done: the counts below only assume what was issued, so
    // pad with real issues clamped to valid slices).
    const uint32_t pre = J < 3 ? J : 3;
    for (uint32_t jj = 0; jj < pre; ++jj) issue(jj);
    // wait until slice 0 has landed: (pre-1) slices x 4 instructions may stay in flight
    if (pre == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    uint32_t ti = 0, kt = 0;
    for (uint32_t jj = 0; jj < J; ++jj) {
        const bool more = jj + 3 < J;
        if (VAR != 1 && more) issue(jj + 3);
        const uint8_t* base = lds + (VAR == 1 ? 0 : (jj % kG3Slots)) * SLOT;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            bf16x8_t af[4], bfr[2];
#pragma unroll
            for (int m = 0; m < 4; ++m) af[m] = *reinterpret_cast<const bf16x8_t*>(base + aoff[m][kk]);
#pragma unroll
            for (int n = 0; n < 2; ++n) bfr[n] = *reinterpret_cast<const bf16x8_t*>(base + boff[n][kk]);
            if constexpr (VAR == 2) {
#pragma unroll
                for (int m = 0; m < 4; ++m) acc[m][0][0] += (float)af[m][0] + (float)bfr[m & 1][0];
            } else {
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int n = 0; n < 2; ++n)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
            }
        }
        bool stored = false;
        if (kt == nk - 1) {
            const uint32_t rt = g0 + ti * RG;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    const uint32_t ql = wc * 64 + n * 32 + (lane & 31);
                    const uint32_t rbase = rt * BM + wr * 128 + m * 32 + 4 * (lane >> 5);
                    if constexpr (!EMIT) {
                        float* dst = p.S + (uint64_t)(qt * BN + ql) * p.s_ld + rbase;
#pragma unroll
                        for (int g = 0; g < 4; ++g)
                            *reinterpret_cast<float4*>(dst + 8 * g) =
                                make_float4(acc[m][n][4 * g], acc[m][n][4 * g + 1], acc[m][n][4 * g + 2],
                                            acc[m][n][4 * g + 3]);
                        stored = true;
                    } else {
                        float mx = acc[m][n][0];
#pragma unroll
                        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[m][n][r]);
                        if (__ballot(mx >= tau[n])) {
#pragma unroll
                            for (int r = 0; r < 16; ++r) {
                                const float v = acc[m][n][r];
                                const uint32_t row = rbase + (r & 3) + 8 * (r >> 2);
                                const bool pass = v >= tau[n] && row < p.n_rows;
                                const uint64_t bm = __ballot(pass);
                                if (bm) {
                                    const uint32_t pos = ecount + __builtin_amdgcn_mbcnt_hi(
                                        (uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
                                    if (pass) {
                                        if (pos < (uint32_t)kG3WCap) {
                                            ekeys[pos] = score_key(v, row);
                                            eq[pos] = ql;
                                        } else {  // wave buffer full: straight to the global list
                                            const uint32_t q = qt * BN + ql;
                                            const uint32_t gp = atomicAdd(p.cnt + q, 1u);
                                            if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = score_key(v, row);
                                        }
                                    }
                                    if (ecount + (uint32_t)__popcll(bm) > (uint32_t)kG3WCap) stored = true;
                                    ecount += (uint32_t)__popcll(bm);
                                }
                            }
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.0f;
                }
            }
            kt = 0;
            ++ti;
        } else {
            ++kt;
        }
        // Slice jj+1 must have landed for every wave.  Global stores / atomics of the
        // epilogue also count in vmcnt: after any of them, drain fully (rare: once a tile).
        if (stored || !more) wait_vm0();
        if (more) wait_vm8_barrier();
        else asm volatile("s_barrier" ::: "memory");
    }
    if constexpr (EMIT) {
        // flush this wave's buffer (its own LDS region: no barrier needed)
        const uint32_t ne = ecount < (uint32_t)kG3WCap ? ecount : (uint32_t)kG3WCap;
        for (uint32_t i = lane; i < ne; i += kWave) {
            const uint32_t q = qt * BN + eq[i];
            const uint32_t gp = atomicAdd(p.cnt + q, 1u);
            if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = ekeys[i];
        }
    }
}

// ------------------------------------------------------------------------------------
// MFMA filter v4: v3's ring (4 slots x 32-deep K slices, 3 in flight) with the issue stream
// arranged so that neither the LDS-DMA issue (60-185 cycles per instruction) nor the
// fragment reads sit in front of a wave's MFMAs:
//   [F1 <- ds_read(j, kk=1)] 4 MFMA(F0) dma(j+3,A0) 4 MFMA(F0) dma(j+3,A1)
//   s_waitcnt lgkmcnt(0) vmcnt(N) ; s_barrier          <- slice j+1 landed everywhere
//   [F0 <- ds_read(j+1, kk=0)] 4 MFMA(F1) dma(j+3,B0) 4 MFMA(F1) dma(j+3,B1)
// F0/F1 are two register sets of fragments (kk = 0 / 1).  The barrier sits mid-slice: the
// slot a DMA overwrites (slice j-1) was last read before the previous barrier, and each
// wave's reads are complete (lgkmcnt(0)) before it arrives there.  N counts this wave's
// younger DMAs still allowed in flight: slice j+2 (4) and slice j+3's A half (2).
// sched_barrier(0) pins the placement against the scheduler.
// ------------------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void mid_barrier() {
    if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// VAR 3 (tooling): LDS-DMA, waits and barriers only (raw operand-feed rate).
template <bool EMIT, int VAR = 0>
__global__ __launch_bounds__(512, 2) void k_gemm_filter4(GemmArgs p) {
    constexpr int BM = kG2BM, BN = kG2BN, BK = kG3BK;
    constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
    constexpr int SLOT = A_BYTES + B_BYTES;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[kG3Slots * SLOT + (EMIT ? 8 * kG3WCap * 12 : 0)];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 2, wc = w & 3;
    uint64_t* ekeys = reinterpret_cast<uint64_t*>(lds + kG3Slots * SLOT) + w * kG3WCap;
    uint32_t* eq = reinterpret_cast<uint32_t*>(lds + kG3Slots * SLOT + 8 * kG3WCap * 8) + w * kG3WCap;
    // per-wave append counter (LDS word; the last q slot of the wave's region is never a
    // real entry: capacity kG3WCap-1)
    const uint32_t ecnt_addr = (uint32_t)(uintptr_t)(eq + kG3WCap - 1);
    if (EMIT && lane == 0) eq[kG3WCap - 1] = 0;

    const uint32_t b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const uint32_t G = (gridDim.x >> 3) / p.n_qt;
    const uint32_t n_rt = (p.n_rows + BM - 1) / BM;
    const uint32_t nk = p.ld / BK;
    const bool active = slot < G * p.n_qt;
    const uint32_t qt = active ? slot % p.n_qt : 0;
    const uint32_t g0 = xcd * G + (active ? slot / p.n_qt : 0);
    const uint32_t RG = 8 * G;
    const uint32_t my_rt = (active && g0 < n_rt) ? (n_rt - 1 - g0) / RG + 1 : 0;
    const uint32_t J = my_rt * nk;

    uint32_t lrow[2], lchunk[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        lrow[i] = (w * 2 + i) * 16 + (lane >> 2);
        lchunk[i] = (lane & 3) ^ ((lrow[i] >> 2) & 3);
    }
    const uint16_t* bsrc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) bsrc[i] = p.B + (uint64_t)(qt * BN + lrow[i]) * p.ld + lchunk[i] * 8;
    const uint64_t a_lane_off[2] = {(uint64_t)lrow[0] * p.a_row_stride + lchunk[0] * 8,
                                    (uint64_t)lrow[1] * p.a_row_stride + lchunk[1] * 8};
    // DMA pointers of the slice being issued (slice jj+3), advanced incrementally.
    uint32_t iss_ti = 0, iss_kt = 0;
    const uint16_t* a_tile = p.A;  // row tile base of the issue slice
    auto set_issue_tile = [&]() {
        const uint32_t rt = VAR == 4 ? g0 : g0 + iss_ti * RG;  // VAR 4: A always from L2
        a_tile = p.A + (uint64_t)rt * BM * p.a_row_stride;
    };
    auto dma_a = [&](uint32_t jj, int i) {
        uint8_t* la = lds + (jj % kG3Slots) * SLOT;
        const uint16_t* src = a_tile + a_lane_off[i] + iss_kt * BK;
        if (!EMIT) {  // sample pass: clamp tail rows to the last valid one
            const uint32_t rt = g0 + iss_ti * RG;
            if (rt * BM + lrow[i] >= p.n_rows)
                src = p.A + (uint64_t)(p.n_rows - 1) * p.a_row_stride + lchunk[i] * 8 + iss_kt * BK;
        }
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(la + (w * 2 + i) * 1024), 16, 0, 0);
    };
    auto dma_b = [&](uint32_t jj, int i) {
        uint8_t* lb = lds + (jj % kG3Slots) * SLOT + A_BYTES;
        __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + iss_kt * BK),
                                         (lds_void_t*)(lb + (w * 2 + i) * 1024), 16, 0, 0);
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
            aoff[m][kk] = row * 64 + ((lc ^ ((row >> 2) & 3)) * 16);
        }
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int row = wc * 64 + n * 32 + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int lc = 2 * kk + (lane >> 5);
            boff[n][kk] = A_BYTES + row * 64 + ((lc ^ ((row >> 2) & 3)) * 16);
        }
    }
    float tau[2] = {0.0f, 0.0f};
    if (EMIT) {
#pragma unroll
        for (int n = 0; n < 2; ++n) tau[n] = p.tau[qt * BN + wc * 64 + n * 32 + (lane & 31)];
    }

    f32x16_t acc[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.0f;

    bf16x8_t fa0[4], fb0[2], fa1[4], fb1[2];
    auto read_frags = [&](uint32_t jj, int kk, bf16x8_t (&fa)[4], bf16x8_t (&fb)[2]) {
        if constexpr (VAR >= 3) return;
        const uint8_t* base = lds + (VAR == 1 ? 0 : jj % kG3Slots) * SLOT;
#pragma unroll
        for (int m = 0; m < 4; ++m) fa[m] = *reinterpret_cast<const bf16x8_t*>(base + aoff[m][kk]);
#pragma unroll
        for (int n = 0; n < 2; ++n) fb[n] = *reinterpret_cast<const bf16x8_t*>(base + boff[n][kk]);
    };
    auto mfma4 = [&](const bf16x8_t (&fa)[4], const bf16x8_t (&fb)[2], int half) {
        if constexpr (VAR >= 3) return;
#pragma unroll
        for (int m = half * 2; m < half * 2 + 2; ++m)
#pragma unroll
            for (int n = 0; n < 2; ++n)
                acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);
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
        const bool iss = VAR != 1 && jj + 3 < J;
        // ---- first half: kk = 0 MFMAs, kk = 1 reads, A-half DMA of slice jj+3
        read_frags(jj, 1, fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa0, fb0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (iss) dma_a(jj + 3, 0);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa0, fb0, 1);
        __builtin_amdgcn_sched_barrier(0);
        if (iss) dma_a(jj + 3, 1);
        __builtin_amdgcn_sched_barrier(0);
        // ---- mid-slice barrier: slice jj+1 has landed for every wave
        if (VAR == 1) {
            mid_barrier<8>();
        } else if (jj + 3 < J) {
            mid_barrier<6>();
        } else if (jj + 2 < J) {
            mid_barrier<4>();
        } else {
            mid_barrier<0>();
        }
        const bool next = jj + 1 < J;
        if (next) read_frags(jj + 1, 0, fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa1, fb1, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (iss) dma_b(jj + 3, 0);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa1, fb1, 1);
        __builtin_amdgcn_sched_barrier(0);
        if (iss) { dma_b(jj + 3, 1); issue_advance(); }
        __builtin_amdgcn_sched_barrier(0);

        if (kt == nk - 1) {
            const uint32_t rt = g0 + ti * RG;
            bool stored = false;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    const uint32_t ql = wc * 64 + n * 32 + (lane & 31);
                    const uint32_t rbase = rt * BM + wr * 128 + m * 32 + 4 * (lane >> 5);
                    if constexpr (!EMIT) {
                        float* dst = p.S + (uint64_t)(qt * BN + ql) * p.s_ld + rbase;
#pragma unroll
                        for (int g = 0; g < 4; ++g)
                            *reinterpret_cast<float4*>(dst + 8 * g) =
                                make_float4(acc[m][n][4 * g], acc[m][n][4 * g + 1], acc[m][n][4 * g + 2],
                                            acc[m][n][4 * g + 3]);
                        stored = true;
                    } else {
                        float mx = acc[m][n][0];
#pragma unroll
                        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[m][n][r]);
                        if (__ballot(mx >= tau[n])) {
                            // per-lane pass mask, then only the passing (lane, register)
                            // pairs append: an LDS counter bumped with an inline-asm
                            // ds_add_rtn (hipcc would drain vmcnt before a plain LDS atomic)
                            uint32_t mask = 0;
#pragma unroll
                            for (int r = 0; r < 16; ++r) mask |= (acc[m][n][r] >= tau[n]) ? (1u << r) : 0u;
                            while (mask) {
                                const int r = __builtin_ctz(mask);
                                mask &= mask - 1;
                                const uint32_t row = rbase + (r & 3) + 8 * (r >> 2);
                                if (row >= p.n_rows) continue;
                                float v = acc[m][n][0];
#pragma unroll
                                for (int rr = 1; rr < 16; ++rr) v = (rr == r) ? acc[m][n][rr] : v;
                                uint32_t pos;
                                asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
                                             : "=v"(pos) : "v"(ecnt_addr), "v"(1u) : "memory");
                                if (pos < (uint32_t)(kG3WCap - 1)) {
                                    ekeys[pos] = score_key(v, row);
                                    eq[pos] = ql;
                                } else {  // wave buffer full: straight to the global list
                                    const uint32_t q = qt * BN + ql;
                                    const uint32_t gp = atomicAdd(p.cnt + q, 1u);
                                    if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = score_key(v, row);
                                    stored = true;
                                }
                            }
                            stored = __ballot(stored) != 0;
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.0f;
                }
            }
            // global stores / atomics count in vmcnt: drain them so the counted waits stay exact
            if (stored) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            kt = 0;
            ++ti;
        } else {
            ++kt;
        }
    }
    if constexpr (EMIT) {
        const uint32_t ecount = eq[kG3WCap - 1];
        const uint32_t ne = ecount < (uint32_t)(kG3WCap - 1) ? ecount : (uint32_t)(kG3WCap - 1);
        for (uint32_t i = lane; i < ne; i += kWave) {
            const uint32_t q = qt * BN + eq[i];
            const uint32_t gp = atomicAdd(p.cnt + q, 1u);
            if (gp < p.cap) p.cand[(uint64_t)q * p.cap + gp] = ekeys[i];
        }
    }
}

// ------------------------------------------------------------------------------------
// Threshold per query from the sample scores: tau0 = ks-th largest sampled score (so at
// least ~ks*stride rows of the whole shard reach it).  One wave per query.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_select_tau(const float* __restrict__ S, uint32_t s_ld,
                                                    uint32_t n_s, uint32_t nq, uint32_t qpad,
                                                    const uint32_t* __restrict__ qflags,
                                                    uint32_t ks, float* __restrict__ tau) {
    __shared__ uint64_t part[4][64];
    const uint32_t q = blockIdx.x;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (q >= qpad) return;
    if (q >= nq || (qflags[q] & kQueryNoApprox)) {
        if (t == 0) tau[q] = INFINITY;  // never emits: answered by the exact scan
        return;
    }
    if (n_s < ks) {
        if (t == 0) tau[q] = -INFINITY;
        return;
    }
    // wave w streams a quarter of the sampled scores, keeping its ks best
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
    for (uint32_t base = 0; base < c; base += kWave) {
        const uint32_t i = base + threadIdx.x;
        L.offer(i < c ? src[i] : kKeyNone, (int)kp + 1, thr);
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
// Exact rescoring of the candidates (one wave per query, lane = candidate): the row and the
// query are walked in index order with separate f32 multiply/add, chunks of 64 elements
// staged through LDS (rows padded to 68 floats: conflict-free ds_read_b128).  The final
// top-k list is certified against the MFMA filter's error bound.
// ------------------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

// Loads of one 64-element chunk of 64 candidate rows (16 x 16 B per lane; each
// wave-instruction covers 4 rows x 256 B).
__device__ __forceinline__ void load_cand_chunk(f32x4_t (&pre)[16], const float* __restrict__ rows,
                                                uint32_t ld, const uint32_t (&lrow)[16], uint32_t ch,
                                                int lane) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
        pre[i] = *reinterpret_cast<const f32x4_t*>(rows + (uint64_t)lrow[i] * ld + ch * 64 + (lane & 15) * 4);
}

// One 64-element chunk of 64 rows held in LDS (stride 68 floats), walked in index order by
// the lane that owns the row: sequential dot (separate f32 mul and add) and max|a_i - b_i|.
template <int QF>
__device__ __forceinline__ void seq_chunk(const float* __restrict__ my, const float* const (&bq)[QF],
                                          uint32_t nvalid, float (&acc)[QF], float (&mx)[QF]) {
    if (nvalid == 64) {
#pragma unroll
        for (int i = 0; i < 64; i += 4) {
            const f32x4_t a = *reinterpret_cast<const f32x4_t*>(my + i);
#pragma unroll
            for (int j = 0; j < QF; ++j) {
                const float* bb = bq[j] + i;
                acc[j] = acc[j] + a.x * bb[0]; mx[j] = fmaxf(mx[j], fabsf(a.x - bb[0]));
                acc[j] = acc[j] + a.y * bb[1]; mx[j] = fmaxf(mx[j], fabsf(a.y - bb[1]));
                acc[j] = acc[j] + a.z * bb[2]; mx[j] = fmaxf(mx[j], fabsf(a.z - bb[2]));
                acc[j] = acc[j] + a.w * bb[3]; mx[j] = fmaxf(mx[j], fabsf(a.w - bb[3]));
            }
        }
    } else {
        for (uint32_t i = 0; i < nvalid; ++i) {
            const float a = my[i];
#pragma unroll
            for (int j = 0; j < QF; ++j) {
                const float bv = bq[j][i];
                acc[j] = acc[j] + a * bv;
                mx[j] = fmaxf(mx[j], fabsf(a - bv));
            }
        }
    }
}

template <int E>
__global__ __launch_bounds__(64) void k_rescore(const float* __restrict__ rows, uint32_t ld, uint32_t dim,
                                                const float* __restrict__ na, const float* __restrict__ qf32,
                                                const float* __restrict__ nb, uint32_t nq,
                                                const uint32_t* __restrict__ cand_rows,
                                                const uint32_t* __restrict__ ncand, uint32_t kp,
                                                const float* __restrict__ tau_excl, uint32_t k,
                                                double ebound, uint64_t* __restrict__ out_keys,
                                                uint32_t* __restrict__ fail_cnt,
                                                uint32_t* __restrict__ fail_list) {
    __shared__ __attribute__((aligned(16))) float lds[64 * 68];
    const uint32_t q = blockIdx.x;
    if (q >= nq) return;
    const int lane = threadIdx.x;
    const uint32_t c = ncand[q];
    const float* bq = qf32 + (uint64_t)q * ld;
    const float mag_b = nb[q];
    const uint32_t nch = ld / 64;

    WaveTopK<E> L;
    L.init();
    uint64_t thr = kKeyNone;
    for (uint32_t base = 0; base < c; base += kWave) {
        const uint32_t ci = base + lane;
        const uint32_t myrow = cand_rows[(uint64_t)q * kp + (ci < c ? ci : 0)];
        float acc[1] = {-0.0f}, mx[1] = {0.0f};
        uint32_t lrow[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) lrow[i] = (uint32_t)__shfl((int)myrow, (i * 64 + lane) >> 4, kWave);
        f32x4_t pre[16];
        load_cand_chunk(pre, rows, ld, lrow, 0, lane);
        for (uint32_t ch = 0; ch < nch; ++ch) {
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int L16 = i * 64 + lane;
                *reinterpret_cast<f32x4_t*>(lds + (L16 >> 4) * 68 + (L16 & 15) * 4) = pre[i];
            }
            __syncthreads();
            load_cand_chunk(pre, rows, ld, lrow, ch + 1 < nch ? ch + 1 : ch, lane);  // clamped prefetch
            const float* const bb[1] = {bq + ch * 64};
            const uint32_t nvalid = dim - ch * 64 < 64 ? dim - ch * 64 : 64;
            seq_chunk<1>(lds + lane * 68, bb, nvalid, acc, mx);
        }
        const float d = finish_distance(acc[0], mx[0], na[myrow], mag_b);
        L.offer(ci < c ? dist_key(d, myrow) : kKeyNone, (int)k, thr);
    }
    L.store(out_keys + (uint64_t)q * k, (int)k);

    if (lane == 0) {
        // Certification: every row outside the candidate set has approximate
        // cosine <= tau_x, hence reference cosine <= tau_x + ebound and reference distance
        // >= 1 - tau_x - ebound - 2^-23; the k-th exact distance must lie strictly below
        // that, and no excluded row can be element-wise identical to the query.
        const float tx = tau_excl[q];
        bool ok;
        if (tx == -INFINITY) {
            ok = true;  // every row of the shard was a candidate
        } else if (!(tx < INFINITY) || thr == kKeyNone) {
            ok = false;
        } else {
            const double dk = (double)key_dist(thr);
            ok = dk < 1.0 - (double)tx - ebound - 2.5e-7 &&
                 (double)tx < 1.0 - ebound - 1e-4 - 6e-9 / (double)mag_b;
        }
        if (!ok) {
            const uint32_t pos = atomicAdd(fail_cnt, 1u);
            fail_list[pos] = q;
        }
    }
}

// ------------------------------------------------------------------------------------
// Exact full scan (src/mpi_helpers/metrics.rs:36-50 for up to QF queries at once): 256
// rows per tile (lane = row), 64-element chunks of the row-major slab staged through LDS
// (padded to 68 floats: conflict-free ds_read_b128), next chunk prefetched into registers.
// Each lane walks its row in index order per query: sequential dot, max|a_i-b_i|.  Per
// wave a sorted top-k per query; the 4 waves merge through LDS into one list per block.
// ------------------------------------------------------------------------------------
template <int QF, int E>
__global__ __launch_bounds__(256, 2) void k_scan_exact(const float* __restrict__ rows, uint32_t ld,
                                                       uint32_t dim, uint64_t n,
                                                       const float* __restrict__ na,
                                                       const float* __restrict__ qf32,
                                                       const int32_t* __restrict__ qids,
                                                       const float* __restrict__ nb, uint32_t k,
                                                       uint64_t* __restrict__ part) {
    // rows [256][68] + (QF > 1) query chunk [QF][64]; QF == 1 reads the query through the
    // scalar cache instead (64 SGPRs per chunk), QF > 1 would spill SGPRs.
    __shared__ __attribute__((aligned(16))) float lds[256 * 68 + (QF > 1 ? QF * 64 : 0)];
    float* ldq = lds + 256 * 68;
    const int t = threadIdx.x, w = t >> 6;
    const uint64_t n_tiles = (n + 255) / 256;
    const uint32_t nch = ld / 64;

    const float* qp[QF];
    float mag_b[QF];
#pragma unroll
    for (int j = 0; j < QF; ++j) {
        const int32_t id = qids[j];
        qp[j] = qf32 + (uint64_t)id * ld;
        mag_b[j] = nb[id];
    }
    WaveTopK<E> L[QF];
    uint64_t thr[QF];
#pragma unroll
    for (int j = 0; j < QF; ++j) { L[j].init(); thr[j] = kKeyNone; }

    // This lane's 16 load addresses within a tile chunk: row (i*256+t)>>4, float4 (t&15).
    const uint32_t lrow0 = (uint32_t)t >> 4;   // + 16*i
    const uint32_t lcol = ((uint32_t)t & 15) * 4;
    uint64_t tile = blockIdx.x;
    uint32_t ch = 0;
    f32x4_t pre[16];
    f32x4_t qpre = {0.0f, 0.0f, 0.0f, 0.0f};
    // thread t < QF*16 also stages float4 (t&15) of query t>>4's chunk
    const float* qsrc = (QF > 1 && t < QF * 16) ? qp[QF > 1 ? (t >> 4) % QF : 0] + lcol : nullptr;
    auto issue = [&](uint64_t tl, uint32_t c) {
        const float* base = rows + (tl * 256 + lrow0) * ld + c * 64 + lcol;
#pragma unroll
        for (int i = 0; i < 16; ++i) pre[i] = *reinterpret_cast<const f32x4_t*>(base + (uint64_t)i * 16 * ld);
        if constexpr (QF > 1) {
            if (qsrc) qpre = *reinterpret_cast<const f32x4_t*>(qsrc + c * 64);
        }
    };
    if (tile < n_tiles) issue(tile, 0);
    float acc[QF], mx[QF];
#pragma unroll
    for (int j = 0; j < QF; ++j) { acc[j] = -0.0f; mx[j] = 0.0f; }

    while (tile < n_tiles) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i)
            *reinterpret_cast<f32x4_t*>(lds + (lrow0 + 16 * i) * 68 + lcol) = pre[i];
        if constexpr (QF > 1) {
            if (qsrc) *reinterpret_cast<f32x4_t*>(ldq + (t >> 4) * 64 + lcol) = qpre;
        }
        __syncthreads();
        // next (tile, chunk); past the end: reload the current chunk (branch-free prefetch)
        uint64_t ntile = tile;
        uint32_t nch_ = ch + 1;
        if (nch_ == nch) { nch_ = 0; ntile = tile + gridDim.x; }
        if (ntile >= n_tiles) { ntile = tile; nch_ = ch; }
        issue(ntile, nch_);

        const uint32_t nvalid = dim - ch * 64 < 64 ? dim - ch * 64 : 64;
        const float* bq[QF];
#pragma unroll
        for (int j = 0; j < QF; ++j) bq[j] = (QF > 1) ? ldq + j * 64 : qp[j] + ch * 64;
        seq_chunk<QF>(lds + t * 68, bq, nvalid, acc, mx);

        if (ch == nch - 1) {
            const uint64_t row = tile * 256 + t;
            const bool valid = row < n;
            const float mag_a = valid ? na[row] : 0.0f;
#pragma unroll
            for (int j = 0; j < QF; ++j) {
                const float d = finish_distance(acc[j], mx[j], mag_a, mag_b[j]);
                L[j].offer(valid ? dist_key(d, (uint32_t)row) : kKeyNone, (int)k, thr[j]);
                acc[j] = -0.0f;
                mx[j] = 0.0f;
            }
            ch = 0;
            tile += gridDim.x;
        } else {
            ++ch;
        }
    }

    // Block merge: 4 wave lists per query -> one list per query.
    __syncthreads();
    uint64_t* lk = reinterpret_cast<uint64_t*>(lds);  // [4][QF][64E] keys (<= 64 KiB)
#pragma unroll
    for (int j = 0; j < QF; ++j) L[j].store(lk + ((uint64_t)w * QF + j) * 64 * E, (int)k);
    __syncthreads();
    for (int j = w; j < QF; j += 4) {
        WaveTopK<E> M;
        M.init();
        uint64_t mt = kKeyNone;
        for (int s = 0; s < 4; ++s) {
            const uint64_t* src = lk + ((uint64_t)s * QF + j) * 64 * E;
            for (uint32_t base = 0; base < k; base += kWave) {
                const uint32_t i = base + (t & 63);
                M.offer(i < k ? src[i] : kKeyNone, (int)k, mt);
            }
        }
        M.store(part + ((uint64_t)blockIdx.x * QF + j) * k, (int)k);
    }
}

// Per scanned query: merge the per-block lists of k_scan_exact into out_keys[qid].
template <int E>
__global__ __launch_bounds__(64) void k_merge_parts(const uint64_t* __restrict__ part, uint32_t grid,
                                                    const int32_t* __restrict__ qids, uint32_t qf,
                                                    uint32_t nqf, uint32_t k,
                                                    uint64_t* __restrict__ out_keys) {
    const uint32_t j = blockIdx.x;
    if (j >= nqf) return;
    WaveTopK<E> L;
    L.init();
    uint64_t thr = kKeyNone;
    const uint64_t total = (uint64_t)grid * k;
    for (uint64_t base = 0; base < total; base += kWave) {
        const uint64_t i = base + threadIdx.x;
        uint64_t key = kKeyNone;
        if (i < total) {
            const uint64_t g = i / k, e = i - g * k;
            key = part[(g * qf + j) * k + e];
        }
        L.offer(key, (int)k, thr);
    }
    L.store(out_keys + (uint64_t)qids[j] * k, (int)k);
}

__global__ void k_finalize(const uint64_t* __restrict__ keys, uint32_t nq, uint32_t k, uint64_t n,
                           uint64_t offset, uint64_t* __restrict__ out_idx, float* __restrict__ out_dist,
                           uint32_t* __restrict__ out_count) {
    const uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (e >= (uint64_t)nq * k) return;
    const uint32_t q = (uint32_t)(e / k), i = (uint32_t)(e - (uint64_t)q * k);
    const uint32_t cnt = (uint64_t)k < n ? k : (uint32_t)n;
    const uint64_t key = keys[e];
    if (i < cnt && key != kKeyNone) {
        out_idx[e] = offset + key_row(key);
        out_dist[e] = key_dist(key);
    } else {
        out_idx[e] = ~0ull;
        out_dist[e] = INFINITY;
    }
    if (i == 0) out_count[q] = cnt;
}

// src/metrics.rs:143-165 for one pair (single lane, fully sequential, from global memory).
__global__ void k_cosine_pair(const float* __restrict__ a, uint32_t la, const float* __restrict__ b,
                              uint32_t lb, float* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (la != lb || la == 0) { *out = 1.0f; return; }
    float dot = -0.0f, aa = -0.0f, bb = -0.0f, mx = 0.0f;
    for (uint32_t i = 0; i < la; ++i) {
        const float x = a[i], y = b[i];
        mx = fmaxf(mx, fabsf(x - y));
        dot = dot + x * y;
        aa = aa + x * x;
        bb = bb + y * y;
    }
    *out = finish_distance(dot, mx, __builtin_sqrtf(aa), __builtin_sqrtf(bb));
}

// ------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------
static inline uint32_t grid_for(uint64_t work, uint32_t block, uint32_t cap = 65536) {
    uint64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    return (uint32_t)(g > cap ? cap : g);
}

hipError_t launch_synth_uniform(float* out, uint64_t row0, uint64_t n_rows, uint32_t dim,
                                uint32_t ld, uint64_t seed, hipStream_t s) {
    hipLaunchKernelGGL(k_synth_uniform, dim3(grid_for(n_rows * ld, 256)), dim3(256), 0, s, out, row0,
                       n_rows, dim, ld, seed);
    return hipGetLastError();
}
hipError_t launch_copy_rows_f32(const float* src, uint64_t n, uint32_t dim, uint32_t ld, float* dst,
                                hipStream_t s) {
    hipLaunchKernelGGL(k_copy_rows_f32, dim3(grid_for(n * ld, 256)), dim3(256), 0, s, src, n, dim, ld, dst);
    return hipGetLastError();
}
hipError_t launch_widen_bf16_rows(const uint16_t* src, uint64_t n, uint32_t dim, uint32_t ld,
                                  float* dst, hipStream_t s) {
    hipLaunchKernelGGL(k_widen_bf16_rows, dim3(grid_for(n * ld, 256)), dim3(256), 0, s, src, n, dim, ld, dst);
    return hipGetLastError();
}
hipError_t launch_check_finite(const float* x, uint64_t count, uint32_t* flag, hipStream_t s) {
    hipLaunchKernelGGL(k_check_finite, dim3(grid_for(count, 256, 4096)), dim3(256), 0, s, x, count, flag);
    return hipGetLastError();
}
hipError_t launch_row_norms(const float* rows, uint64_t n, uint32_t dim, uint32_t ld, float* na,
                            uint32_t* flags, hipStream_t s) {
    hipLaunchKernelGGL(k_row_norms, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, rows, n, dim, ld,
                       na, flags);
    return hipGetLastError();
}
hipError_t launch_rows_to_bf16n(const float* rows, const float* na, uint64_t n, uint64_t n_pad,
                                uint32_t dim, uint32_t ld, uint16_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_rows_to_bf16n, dim3(grid_for(n_pad * (ld / 8), 256)), dim3(256), 0, s, rows, na, n,
                       n_pad, dim, ld, out);
    return hipGetLastError();
}
hipError_t launch_query_prep(const float* q, uint32_t nq, uint32_t qpad, uint32_t dim, uint32_t ld,
                             float* qf32, float* nb, uint16_t* qbf, uint32_t* qflags, hipStream_t s) {
    hipLaunchKernelGGL(k_query_norms, dim3((qpad + 63) / 64), dim3(64), 0, s, q, nq, qpad, dim, nb, qflags);
    hipLaunchKernelGGL(k_query_convert, dim3(grid_for((uint64_t)qpad * ld, 256)), dim3(256), 0, s, q, nq, qpad,
                       dim, ld, nb, qflags, qf32, qbf);
    return hipGetLastError();
}
static int gemm_variant() {
    static int v = [] {
        const char* e = getenv("BSR_GEMM_VARIANT");
        return e ? atoi(e) : 4;
    }();
    return v;
}
// Workgroups for the persistent filter: 8 XCDs x (32 CUs rounded down to a multiple of n_qt).
static uint32_t gemm2_grid(uint32_t n_qt) {
    const uint32_t per_xcd = n_qt >= 32 ? n_qt : (32 / n_qt) * n_qt;
    return 8 * per_xcd;
}
uint32_t gemm_query_pad() { return gemm_variant() == 1 ? kGemmBN : (uint32_t)kG2BN; }
uint32_t gemm_row_tile() { return gemm_variant() == 1 ? kGemmBM : (uint32_t)kG2BM; }

hipError_t launch_gemm_sample(const GemmArgs& a, hipStream_t s) {
    if (gemm_variant() == 1) {
        hipLaunchKernelGGL(k_gemm_filter<false>, dim3(a.n_rt * a.n_qt), dim3(256), 0, s, a);
    } else if (gemm_variant() == 2) {
        hipLaunchKernelGGL(k_gemm_filter2<false>, dim3(gemm2_grid(a.n_qt)), dim3(kG2Threads), 0, s, a);
    } else if (gemm_variant() == 3) {
        hipLaunchKernelGGL(k_gemm_filter3<false>, dim3(gemm2_grid(a.n_qt)), dim3(kG2Threads), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_gemm_filter4<false>, dim3(gemm2_grid(a.n_qt)), dim3(kG2Threads), 0, s, a);
    }
    return hipGetLastError();
}
hipError_t launch_gemm_emit(const GemmArgs& a, hipStream_t s) {
    if (gemm_variant() == 1) {
        hipLaunchKernelGGL(k_gemm_filter<true>, dim3(a.n_rt * a.n_qt), dim3(256), 0, s, a);
    } else if (gemm_variant() == 2) {
        hipLaunchKernelGGL(k_gemm_filter2<true>, dim3(gemm2_grid(a.n_qt)), dim3(kG2Threads), 0, s, a);
    } else if (gemm_variant() == 3) {
        hipLaunchKernelGGL(k_gemm_filter3<true>, dim3(gemm2_grid(a.n_qt)), dim3(kG2Threads), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_gemm_filter4<true>, dim3(gemm2_grid(a.n_qt)), dim3(kG2Threads), 0, s, a);
    }
    return hipGetLastError();
}
hipError_t launch_select_tau(const float* S, uint32_t s_ld, uint32_t n_s, uint32_t nq, uint32_t qpad,
                             const uint32_t* qflags, uint32_t ks, float* tau, hipStream_t s) {
    hipLaunchKernelGGL(k_select_tau, dim3(qpad), dim3(256), 0, s, S, s_ld, n_s, nq, qpad, qflags, ks, tau);
    return hipGetLastError();
}
hipError_t launch_select_cand(const uint64_t* cand, const uint32_t* cnt, uint32_t cap, uint32_t nq,
                              const float* tau, uint32_t kp, uint32_t* cand_rows, uint32_t* ncand,
                              float* tau_excl, hipStream_t s) {
    const uint32_t e = (kp + 1 + 63) / 64;
    switch (e) {
        case 1: hipLaunchKernelGGL(k_select_cand<1>, dim3(nq), dim3(64), 0, s, cand, cnt, cap, nq, tau, kp, cand_rows, ncand, tau_excl); break;
        case 2: hipLaunchKernelGGL(k_select_cand<2>, dim3(nq), dim3(64), 0, s, cand, cnt, cap, nq, tau, kp, cand_rows, ncand, tau_excl); break;
        case 3: hipLaunchKernelGGL(k_select_cand<3>, dim3(nq), dim3(64), 0, s, cand, cnt, cap, nq, tau, kp, cand_rows, ncand, tau_excl); break;
        case 4: hipLaunchKernelGGL(k_select_cand<4>, dim3(nq), dim3(64), 0, s, cand, cnt, cap, nq, tau, kp, cand_rows, ncand, tau_excl); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_rescore(const float* rows, uint32_t ld, uint32_t dim, const float* na, const float* qf32,
                          const float* nb, uint32_t nq, const uint32_t* cand_rows, const uint32_t* ncand,
                          uint32_t kp, const float* tau_excl, uint32_t k, double ebound, uint64_t* out_keys,
                          uint32_t* fail_cnt, uint32_t* fail_list, hipStream_t s) {
    const uint32_t e = (k + 63) / 64;
#define BSR_RESCORE(E)                                                                              \
    hipLaunchKernelGGL(k_rescore<E>, dim3(nq), dim3(64), 0, s, rows, ld, dim, na, qf32, nb, nq,   \
                       cand_rows, ncand, kp, tau_excl, k, ebound, out_keys, fail_cnt, fail_list)
    switch (e) {
        case 1: BSR_RESCORE(1); break;
        case 2: BSR_RESCORE(2); break;
        case 3: BSR_RESCORE(3); break;
        case 4: BSR_RESCORE(4); break;
        default: return hipErrorInvalidValue;
    }
#undef BSR_RESCORE
    return hipGetLastError();
}

uint32_t scan_grid_for(uint64_t n) {
    const uint64_t tiles = (n + 255) / 256;
    const uint64_t g = tiles < 512 ? tiles : 512;  // 2 blocks per CU x 256 CUs
    return (uint32_t)(g < 1 ? 1 : g);
}

template <int QF>
static void launch_scan_qf(const float* rows, uint32_t ld, uint32_t dim, uint64_t n, const float* na,
                           const float* qf32, const int32_t* qids, const float* nb, uint32_t k,
                           uint32_t grid, uint64_t* part, hipStream_t s) {
    const uint32_t e = (k + 63) / 64;
#define BSR_SCAN(E)                                                                                  \
    hipLaunchKernelGGL((k_scan_exact<QF, E>), dim3(grid), dim3(256), 0, s, rows, ld, dim, n, na,  \
                       qf32, qids, nb, k, part)
    switch (e) {
        case 1: BSR_SCAN(1); break;
        case 2: BSR_SCAN(2); break;
        case 3: BSR_SCAN(3); break;
        default: BSR_SCAN(4); break;
    }
#undef BSR_SCAN
}

hipError_t launch_scan_exact(const float* rows, uint32_t ld, uint32_t dim, uint64_t n, const float* na,
                             const float* qf32, const int32_t* qids, uint32_t nqf, const float* nb,
                             uint32_t k, uint32_t grid, uint64_t* part, hipStream_t s) {
    // Query ids beyond nqf must be valid (the caller repeats the last id); results for them
    // are computed and ignored.
    if (nqf <= 1) launch_scan_qf<1>(rows, ld, dim, n, na, qf32, qids, nb, k, grid, part, s);
    else if (nqf <= 2) launch_scan_qf<2>(rows, ld, dim, n, na, qf32, qids, nb, k, grid, part, s);
    else if (nqf <= 4) launch_scan_qf<4>(rows, ld, dim, n, na, qf32, qids, nb, k, grid, part, s);
    else launch_scan_qf<8>(rows, ld, dim, n, na, qf32, qids, nb, k, grid, part, s);
    return hipGetLastError();
}

hipError_t launch_merge_parts(const uint64_t* part, uint32_t grid, const int32_t* qids, uint32_t nqf,
                              uint32_t k, uint64_t* out_keys, hipStream_t s) {
    const uint32_t qf = nqf <= 1 ? 1 : nqf <= 2 ? 2 : nqf <= 4 ? 4 : 8;
    const uint32_t e = (k + 63) / 64;
#define BSR_MERGE(E)                                                                              \
    hipLaunchKernelGGL(k_merge_parts<E>, dim3(nqf), dim3(64), 0, s, part, grid, qids, qf, nqf, k, \
                       out_keys)
    switch (e) {
        case 1: BSR_MERGE(1); break;
        case 2: BSR_MERGE(2); break;
        case 3: BSR_MERGE(3); break;
        default: BSR_MERGE(4); break;
    }
#undef BSR_MERGE
    return hipGetLastError();
}

hipError_t launch_finalize(const uint64_t* keys, uint32_t nq, uint32_t k, uint64_t n, uint64_t offset,
                           uint64_t* out_idx, float* out_dist, uint32_t* out_count, hipStream_t s) {
    const uint64_t total = (uint64_t)nq * k;
    hipLaunchKernelGGL(k_finalize, dim3(grid_for(total, 256)), dim3(256), 0, s, keys, nq, k, n, offset,
                       out_idx, out_dist, out_count);
    return hipGetLastError();
}

hipError_t launch_cosine_pair(const float* a, uint32_t la, const float* b, uint32_t lb, float* out,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_cosine_pair, dim3(1), dim3(64), 0, s, a, la, b, lb, out);
    return hipGetLastError();
}

}  // namespace bsr
