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

// Per query (one wave): padded f32 copy, exact magnitude |b| (src/metrics.rs:155, lane 0,
// sequential), normalised bf16 copy, flags.  Queries q >= nq (padding) become zeros.
__global__ void k_query_prep(const float* __restrict__ q, uint32_t nq, uint32_t qpad, uint32_t dim,
                             uint32_t ld, float* __restrict__ qf32, float* __restrict__ nb,
                             uint16_t* __restrict__ qbf, uint32_t* __restrict__ qflags) {
    const uint32_t qi = blockIdx.x;
    const int lane = threadIdx.x;
    if (qi >= qpad) return;
    bool bad = false;
    for (uint32_t c = lane; c < ld; c += kWave) {
        float v = (qi < nq && c < dim) ? q[(uint64_t)qi * dim + c] : 0.0f;
        bad |= !isfinite(v);
        qf32[(uint64_t)qi * ld + c] = v;
    }
    __syncthreads();
    float m = 0.0f;
    if (lane == 0) {
        const float* b = qf32 + (uint64_t)qi * ld;
        float acc = -0.0f;
        for (uint32_t i = 0; i < dim; ++i) acc = acc + b[i] * b[i];
        m = __builtin_sqrtf(acc);
        if (qi < nq) nb[qi] = m;
    }
    m = __shfl(m, 0, kWave);
    const bool anybad = __ballot(bad) != 0;
    const bool approx_ok = qi < nq && !anybad && isfinite(m) && m >= 1e-18f && m <= 1e18f;
    for (uint32_t c = lane; c < ld; c += kWave) {
        const float v = qf32[(uint64_t)qi * ld + c];
        qbf[(uint64_t)qi * ld + c] = (approx_ok && c < dim) ? f32_to_bf16_rne(v / m) : (uint16_t)0;
    }
    if (lane == 0)
        qflags[qi] = (anybad ? kQueryNonFinite : 0u) | (approx_ok ? 0u : kQueryNoApprox);
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
// Threshold per query from the sample scores: tau0 = ks-th largest sampled score (so at
// least ~ks*stride rows of the whole shard reach it).  One wave per query.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_select_tau(const float* __restrict__ S, uint32_t s_ld,
                                                   uint32_t n_s, uint32_t nq, uint32_t qpad,
                                                   const uint32_t* __restrict__ qflags,
                                                   uint32_t ks, float* __restrict__ tau) {
    const uint32_t q = blockIdx.x;
    if (q >= qpad) return;
    if (q >= nq || (qflags[q] & kQueryNoApprox)) {
        if (threadIdx.x == 0) tau[q] = INFINITY;  // never emits: answered by the exact scan
        return;
    }
    if (n_s < ks) {
        if (threadIdx.x == 0) tau[q] = -INFINITY;
        return;
    }
    WaveTopK<1> L;
    L.init();
    uint64_t thr = kKeyNone;
    const float* s = S + (uint64_t)q * s_ld;
    for (uint32_t base = 0; base < n_s; base += kWave) {
        const uint32_t i = base + threadIdx.x;
        const uint64_t key = i < n_s ? score_key(s[i], i) : kKeyNone;
        L.offer(key, (int)ks, thr);
    }
    if (threadIdx.x == 0) tau[q] = score_key_score(thr);
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
// Loads of one 64-element chunk of 64 candidate rows (16 x 16 B per lane, rows 4 per
// wave-instruction: 256-B coalesced segments).
__device__ __forceinline__ void load_cand_chunk(float4 (&pre)[16], const float* __restrict__ rows,
                                                uint32_t ld, const uint32_t (&lrow)[16], uint32_t ch,
                                                int lane) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
        pre[i] = *reinterpret_cast<const float4*>(rows + (uint64_t)lrow[i] * ld + ch * 64 + ((i * 64 + lane) & 15) * 4);
}

// Loads of one 64-element chunk of a 256-row scan tile (iteration `it` of this block).
__device__ __forceinline__ void load_tile_chunk(float4 (&pre)[16], const float* __restrict__ rows,
                                                uint32_t ld, uint32_t nch, uint64_t it, int t) {
    const uint64_t ti = it / nch;
    const uint32_t ch = (uint32_t)(it - ti * nch);
    const uint64_t row0 = (blockIdx.x + ti * gridDim.x) * 256;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int L16 = i * 256 + t;
        pre[i] = *reinterpret_cast<const float4*>(rows + (row0 + (L16 >> 4)) * ld + ch * 64 + (L16 & 15) * 4);
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
        const uint32_t myrow = ci < c ? cand_rows[(uint64_t)q * kp + ci] : cand_rows[(uint64_t)q * kp];
        float acc = -0.0f, mx = 0.0f;
        float4 pre[16];
        // row of candidate r (lanes 16r'..) for each of the 16 loads, fixed per round
        uint32_t lrow[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) lrow[i] = (uint32_t)__shfl((int)myrow, (i * 64 + lane) >> 4, kWave);
        load_cand_chunk(pre, rows, ld, lrow, 0, lane);
        for (uint32_t ch = 0; ch < nch; ++ch) {
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int L16 = i * 64 + lane;
                *reinterpret_cast<float4*>(lds + (L16 >> 4) * 68 + (L16 & 15) * 4) = pre[i];
            }
            __syncthreads();
            if (ch + 1 < nch) load_cand_chunk(pre, rows, ld, lrow, ch + 1, lane);
            const float* my = lds + lane * 68;
            const float* bb = bq + ch * 64;
            const uint32_t nvalid = dim - ch * 64 < 64 ? dim - ch * 64 : 64;
            if (nvalid == 64) {
#pragma unroll
                for (int i = 0; i < 64; i += 4) {
                    const float4 a = *reinterpret_cast<const float4*>(my + i);
                    acc = acc + a.x * bb[i + 0]; mx = fmaxf(mx, fabsf(a.x - bb[i + 0]));
                    acc = acc + a.y * bb[i + 1]; mx = fmaxf(mx, fabsf(a.y - bb[i + 1]));
                    acc = acc + a.z * bb[i + 2]; mx = fmaxf(mx, fabsf(a.z - bb[i + 2]));
                    acc = acc + a.w * bb[i + 3]; mx = fmaxf(mx, fabsf(a.w - bb[i + 3]));
                }
            } else {
                for (uint32_t i = 0; i < nvalid; ++i) {
                    const float a = my[i];
                    acc = acc + a * bb[i];
                    mx = fmaxf(mx, fabsf(a - bb[i]));
                }
            }
        }
        const float d = finish_distance(acc, mx, na[myrow], mag_b);
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
    __shared__ __attribute__((aligned(16))) float lds[256 * 68];
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

    const uint64_t my_tiles = blockIdx.x < n_tiles ? (n_tiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
    const uint64_t total_it = my_tiles * nch;
    float4 pre[16];
    if (total_it) load_tile_chunk(pre, rows, ld, nch, 0, t);
    float acc[QF], mx[QF];
#pragma unroll
    for (int j = 0; j < QF; ++j) { acc[j] = -0.0f; mx[j] = 0.0f; }

    for (uint64_t it = 0; it < total_it; ++it) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int L16 = i * 256 + t;
            *reinterpret_cast<float4*>(lds + (L16 >> 4) * 68 + (L16 & 15) * 4) = pre[i];
        }
        __syncthreads();
        if (it + 1 < total_it) load_tile_chunk(pre, rows, ld, nch, it + 1, t);
        const uint64_t ti = it / nch;
        const uint32_t ch = (uint32_t)(it - ti * nch);
        if (ch == 0) {
#pragma unroll
            for (int j = 0; j < QF; ++j) { acc[j] = -0.0f; mx[j] = 0.0f; }
        }
        const float* my = lds + t * 68;
        const uint32_t nvalid = dim - ch * 64 < 64 ? dim - ch * 64 : 64;
        if (nvalid == 64) {
#pragma unroll
            for (int i = 0; i < 64; i += 4) {
                const float4 a = *reinterpret_cast<const float4*>(my + i);
#pragma unroll
                for (int j = 0; j < QF; ++j) {
                    const float* bb = qp[j] + ch * 64 + i;
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
                    const float bv = qp[j][ch * 64 + i];
                    acc[j] = acc[j] + a * bv;
                    mx[j] = fmaxf(mx[j], fabsf(a - bv));
                }
            }
        }
        if (ch == nch - 1) {
            const uint64_t row = (blockIdx.x + ti * gridDim.x) * 256 + t;
            const bool valid = row < n;
            const float mag_a = valid ? na[row] : 0.0f;
#pragma unroll
            for (int j = 0; j < QF; ++j) {
                const float d = finish_distance(acc[j], mx[j], mag_a, mag_b[j]);
                L[j].offer(valid ? dist_key(d, (uint32_t)row) : kKeyNone, (int)k, thr[j]);
            }
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
    hipLaunchKernelGGL(k_query_prep, dim3(qpad), dim3(64), 0, s, q, nq, qpad, dim, ld, qf32, nb, qbf, qflags);
    return hipGetLastError();
}
hipError_t launch_gemm_sample(const GemmArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_gemm_filter<false>, dim3(a.n_rt * a.n_qt), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_gemm_emit(const GemmArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_gemm_filter<true>, dim3(a.n_rt * a.n_qt), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_select_tau(const float* S, uint32_t s_ld, uint32_t n_s, uint32_t nq, uint32_t qpad,
                             const uint32_t* qflags, uint32_t ks, float* tau, hipStream_t s) {
    hipLaunchKernelGGL(k_select_tau, dim3(qpad), dim3(64), 0, s, S, s_ld, n_s, nq, qpad, qflags, ks, tau);
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
