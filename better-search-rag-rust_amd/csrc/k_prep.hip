// k_prep.hip -- data movement and preparation kernels (gfx950): synthetic data, the padded
// f32 slab, the reference's exact magnitudes, and the MFMA filter operands (int8)
// of corpus rows and queries together with their certification error bounds.
//
// Compiled with -ffp-contract=off: the magnitudes reproduce src/metrics.rs:154-155 (a
// sequential f32 sum of squares in index order, then a correctly rounded sqrt).  The
// filter operands are approximations whose error is measured here, in double precision,
// and carried to the certification step.
#include "bsr_device.hpp"
#include "kernels.hpp"

#include <math.h>

#include <algorithm>

namespace bsr {

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

// ------------------------------------------------------------------------------------
// Row magnitudes exactly as src/metrics.rs:154: sqrt of the sequential f32 sum of a_i*a_i.
// One lane per row (the per-row dependency chain is inherently serial), but the rows reach
// the lanes through LDS: each wave owns 64 consecutive rows and stages them 64 columns at a
// time with coalesced 16-byte loads (16 lanes per 256-byte row segment), then every lane
// walks its own row's staged segment in index order.  (Round 2's lane-per-row float4 loads
// touched 64 rows per wave-instruction and fetched 3.6x the slab.)  Requires ld % 64 == 0
// (rows zero-padded to ld, kLdAlign).
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_row_norms(const float* __restrict__ rows, uint64_t n, uint32_t dim,
                                                   uint32_t ld, float* __restrict__ na, uint32_t* flags) {
    constexpr int kCols = 64, kPitch = kCols + 1;  // odd pitch: lane l reads bank (l + j) % 32
    __shared__ float tile[4][64 * kPitch];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t r0 = ((uint64_t)blockIdx.x * 4 + w) * 64;
    float* t = tile[w];
    float acc = -0.0f;
    bool bad = false;
    for (uint32_t c0 = 0; c0 < dim; c0 += kCols) {
        const uint32_t cw = dim - c0 < (uint32_t)kCols ? dim - c0 : (uint32_t)kCols;
        const uint32_t col = (lane & 15) * 4;
#pragma unroll 4
        for (int i = 0; i < 16; ++i) {
            const uint32_t rr = i * 4 + (lane >> 4);
            float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (r0 + rr < n) v = *reinterpret_cast<const float4*>(rows + (r0 + rr) * ld + c0 + col);
            float* d = t + rr * kPitch + col;
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
        __syncthreads();
        const float* a = t + lane * kPitch;
        for (uint32_t j = 0; j < cw; ++j) {
            const float x = a[j];
            bad |= !isfinite(x);
            acc = acc + x * x;
        }
        __syncthreads();
    }
    const uint64_t r = r0 + lane;
    uint32_t f = 0;
    if (r < n) {
        const float m = __builtin_sqrtf(acc);
        na[r] = m;
        if (bad) f |= kRowNonFinite;
        if (!isfinite(m)) f |= kRowNormOvf;
        if (m != 0.0f && (m < 1e-18f || m > 1e18f)) f |= kRowNormRange;
    }
    const uint32_t any = __reduce_or_sync(~0ull, f);
    if (any && lane_id() == 0) atomicOr(flags, any);
}

// ------------------------------------------------------------------------------------
// int8 filter operand.  One workgroup (4 waves) per block of 32 rows, the rows of one
// 32x32 MFMA accumulator block:
//   x = a / |a|                      (double; |a| = sqrt of the double sum of squares)
//   s = the smallest f32 >= max_block |x_i| / 127
//   q_i = rint(x_i / s) in [-127, 127]
//   e_row = || x - s q ||_2          (double), ea_max = max_row e_row rounded up to f32.
// By Cauchy-Schwarz |x.y - (s q).(t p)| <= e_row + e_q + e_row e_q for unit x, y, which is
// the row-side half of the certification bound.  Zero rows give q = 0 and e = 0 (the
// reference scores them 1.0 = cosine 0, which is exactly the filter's value).
// ------------------------------------------------------------------------------------
// (butterflies in the VALU: the partner's value by DPP / permlane moves, bsr_device.hpp)
__device__ __forceinline__ double xor_lane_f64(double v, int o) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = xor_lane32((uint32_t)u, o), hi = xor_lane32((uint32_t)(u >> 32), o);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += xor_lane_f64(v, o);
    return v;
}
__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmax(v, xor_lane_f64(v, o));
    return v;
}
// Smallest f32 >= x (x >= 0, finite).
__device__ __forceinline__ float f32_round_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = __uint_as_float(__float_as_uint(f) + 1u);
    return f;
}
__device__ __forceinline__ int8_t quant_i8(double x, double s) {
    double qd = rint(x / s);
    qd = fmin(127.0, fmax(-127.0, qd));
    return (int8_t)(int)qd;
}

__global__ __launch_bounds__(256) void k_rows_to_i8(const float* __restrict__ rows, uint64_t n,
                                                    uint32_t dim, uint32_t ld,
                                                    int8_t* __restrict__ out,
                                                    float* __restrict__ scales,
                                                    uint32_t* __restrict__ ea_max) {
    __shared__ double s_inv[kQuantBlock];
    __shared__ double s_wmax[4];
    const uint64_t blk = blockIdx.x;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    constexpr int kRowsPerWave = kQuantBlock / 4;
    double wmax = 0.0;
    for (int i = 0; i < kRowsPerWave; ++i) {
        const int rl = w * kRowsPerWave + i;
        const uint64_t r = blk * kQuantBlock + rl;
        double ss = 0.0, mx = 0.0;
        if (r < n) {
            const float* a = rows + r * ld;
            for (uint32_t c = lane; c < dim; c += kWave) {
                const double x = a[c];
                ss += x * x;
                mx = fmax(mx, fabs(x));
            }
        }
        ss = wave_sum_f64(ss);
        mx = wave_max_f64(mx);
        const double inv = (ss > 0.0 && ss < 1e300) ? 1.0 / sqrt(ss) : 0.0;
        if (lane == 0) s_inv[rl] = inv;
        wmax = fmax(wmax, mx * inv);
    }
    if (lane == 0) s_wmax[w] = wmax;
    __syncthreads();
    const double bmax = fmax(fmax(s_wmax[0], s_wmax[1]), fmax(s_wmax[2], s_wmax[3]));
    const float sc = bmax > 0.0 ? f32_round_up(bmax / 127.0) : 1.0f;
    if (t == 0) scales[blk] = sc;
    const double s = sc;
    double ew = 0.0;
    for (int i = 0; i < kRowsPerWave; ++i) {
        const int rl = w * kRowsPerWave + i;
        const uint64_t r = blk * kQuantBlock + rl;
        const double inv = s_inv[rl];
        const float* a = rows + r * ld;
        double e2 = 0.0;
        for (uint32_t c0 = lane * 4; c0 < ld; c0 += 4 * kWave) {
            char4 v = make_char4(0, 0, 0, 0);
            int8_t qv[4] = {0, 0, 0, 0};
            if (r < n && inv > 0.0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t c = c0 + j;
                    if (c < dim) {
                        const double x = (double)a[c] * inv;
                        qv[j] = quant_i8(x, s);
                        const double d = x - s * (double)qv[j];
                        e2 += d * d;
                    }
                }
            }
            v.x = qv[0]; v.y = qv[1]; v.z = qv[2]; v.w = qv[3];
            *reinterpret_cast<char4*>(out + r * ld + c0) = v;
        }
        e2 = wave_sum_f64(e2);
        ew = fmax(ew, sqrt(e2));
    }
    if (lane == 0) atomicMax(ea_max, __float_as_uint(f32_round_up(ew * (1.0 + 1e-9) + 1e-12)));
}

// The sample operand: kSampleScaleRows sampled rows (corpus rows kSampleStride apart) per
// workgroup, one scale for all of them; rows past the corpus are zero.
__global__ __launch_bounds__(256) void k_rows_to_i8_sample(const float* __restrict__ rows, uint64_t n,
                                                           uint32_t dim, uint32_t ld, int8_t* __restrict__ out,
                                                           float* __restrict__ scales) {
    __shared__ double s_inv[kSampleScaleRows];
    __shared__ double s_wmax[4];
    const uint64_t blk = blockIdx.x;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    constexpr int kRowsPerWave = kSampleScaleRows / 4;
    double wmax = 0.0;
    for (int i = 0; i < kRowsPerWave; ++i) {
        const int rl = w * kRowsPerWave + i;
        const uint64_t r = (blk * kSampleScaleRows + rl) * kSampleStride;  // corpus row
        double ss = 0.0, mx = 0.0;
        if (r < n) {
            const float* a = rows + r * ld;
            for (uint32_t c = lane; c < dim; c += kWave) {
                const double x = a[c];
                ss += x * x;
                mx = fmax(mx, fabs(x));
            }
        }
        ss = wave_sum_f64(ss);
        mx = wave_max_f64(mx);
        const double inv = (ss > 0.0 && ss < 1e300) ? 1.0 / sqrt(ss) : 0.0;
        if (lane == 0) s_inv[rl] = inv;
        wmax = fmax(wmax, mx * inv);
    }
    if (lane == 0) s_wmax[w] = wmax;
    __syncthreads();
    const double bmax = fmax(fmax(s_wmax[0], s_wmax[1]), fmax(s_wmax[2], s_wmax[3]));
    const float sc = bmax > 0.0 ? f32_round_up(bmax / 127.0) : 1.0f;
    if (t == 0) scales[blk] = sc;
    const double s = sc;
    for (int i = 0; i < kRowsPerWave; ++i) {
        const int rl = w * kRowsPerWave + i;
        const uint64_t rs = blk * kSampleScaleRows + rl;  // sample row
        const uint64_t r = rs * kSampleStride;
        const double inv = s_inv[rl];
        const float* a = rows + r * ld;
        for (uint32_t c0 = lane * 4; c0 < ld; c0 += 4 * kWave) {
            int8_t qv[4] = {0, 0, 0, 0};
            if (r < n && inv > 0.0) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (c0 + j < dim) qv[j] = quant_i8((double)a[c0 + j] * inv, s);
            }
            *reinterpret_cast<char4*>(out + rs * ld + c0) = make_char4(qv[0], qv[1], qv[2], qv[3]);
        }
    }
}

// ------------------------------------------------------------------------------------
// Queries: one workgroup of two waves per (padded) query, the whole preparation in one kernel.
//   1. the caller's row -> LDS (coalesced) and the padded f32 copy qf32[q] (zeros past dim)
//   2. wave 0's lane 0 walks the row in index order: |b| exactly as src/metrics.rs:155 (sequential
//      f32 sum of squares from -0.0, correctly rounded sqrt), finiteness
//   3. flags, the identity query-id list of the exact scan (min(q, nq-1))
//   4. the int8 filter operand from the LDS copy: x = b/|b| (double), s = smallest f32 >=
//      max|x_i|/127, q_i = rint(x_i/s), eb = ||x - s q||_2, E_q = ea + eb + ea*eb + 1.5e-4 (ea:
//      the row side; 1.5e-4 covers the reference's own f32 rounding, <= 9.3e-5, and the two f32
//      roundings of the filter's score)
//      queries the filter cannot serve (pad, zero/tiny/huge |b|) get a zero operand and
//      E_q = inf.
// ------------------------------------------------------------------------------------
constexpr uint32_t kQueryLdsFloats = 8192;  // rows up to 8192 floats are staged in LDS

// Steps 2 and 4 (int8) overlap: while wave 0's lane 0 walks the exact |b| (the reference's
// dependent chain of f32 adds), wave 1 quantises the row to int8 (double precision) into
// registers; the result is kept only if |b| admits the filter (else zeros, E_q = inf).
__global__ __launch_bounds__(128) void k_query_prep(const float* __restrict__ q, uint32_t nq, uint32_t dim,
                                                    uint32_t ld, bool with_op,
                                                    const uint32_t* __restrict__ ea_max,
                                                    float* __restrict__ qf32, float* __restrict__ nb,
                                                    void* __restrict__ qop, float* __restrict__ qscale,
                                                    float* __restrict__ ebound, uint32_t* __restrict__ qflags,
                                                    int32_t* __restrict__ qids, uint32_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) float row[kQueryLdsFloats];
    __shared__ uint32_t s_flags;
    __shared__ uint32_t s_bad;
    const uint32_t qi = blockIdx.x;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const bool real = qi < nq;
    const bool staged = ld <= kQueryLdsFloats;
    const float* src = q + (uint64_t)qi * dim;
    float* dst = qf32 + (uint64_t)qi * ld;
    if (t == 0) s_bad = 0;
    __syncthreads();
    bool bad = false;
    // 8 loads per thread in flight, then their stores (rows up to 1024 floats: one round)
    constexpr int B = 8;
    for (uint32_t c0 = 0; c0 < ld; c0 += B * 128) {
        float v[B];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const uint32_t c = c0 + j * 128 + t;
            v[j] = (real && c < dim) ? src[c] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const uint32_t c = c0 + j * 128 + t;
            if (c < ld) {
                bad |= !isfinite(v[j]);
                dst[c] = v[j];
                if (staged) row[c] = v[j];
            }
        }
    }
    if (__ballot(bad) != 0 && lane == 0) s_bad = 1;
    __syncthreads();
    bad = s_bad != 0;
    auto val = [&](uint32_t c) -> float { return staged ? row[c] : dst[c]; };
    const bool i8 = with_op;
    // wave 1 (int8 operand): the quantisation, speculatively, into registers
    constexpr int QV = 4;  // char4 groups per lane held (rows up to 1024 int8); longer rows: second pass
    char4 qv[QV];
    double e2 = 0.0;
    float sc = 1.0f;
    if (w == 1 && i8) {
        double ss = 0.0, mx = 0.0;
        if (real && !bad) {
            for (uint32_t c = lane; c < dim; c += kWave) {
                const double x = val(c);
                ss += x * x;
                mx = fmax(mx, fabs(x));
            }
        }
        ss = wave_sum_f64(ss);
        mx = wave_max_f64(mx);
        const double inv = ss > 0.0 ? 1.0 / sqrt(ss) : 0.0;
        sc = (mx > 0.0 && inv > 0.0) ? f32_round_up(mx * inv / 127.0) : 1.0f;
        const double sd = sc;
        for (uint32_t g = 0, c0 = lane * 4; c0 < ld; ++g, c0 += 4 * kWave) {
            int8_t qq[4] = {0, 0, 0, 0};
            if (inv > 0.0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t c = c0 + j;
                    if (c < dim) {
                        const double x = (double)val(c) * inv;
                        qq[j] = quant_i8(x, sd);
                        const double d = x - sd * (double)qq[j];
                        e2 += d * d;
                    }
                }
            }
            const char4 v4 = make_char4(qq[0], qq[1], qq[2], qq[3]);
            if (g < (uint32_t)QV) qv[g] = v4;
            else *reinterpret_cast<char4*>(static_cast<int8_t*>(qop) + (uint64_t)qi * ld + c0) = v4;
        }
        e2 = wave_sum_f64(e2);
    }
    if (t == 0) {
        // the reference's sequential sum, 16 elements per step from 4 ds_read_b128
        float acc = -0.0f;
        uint32_t i = 0;
        if (real && staged) {
            const float4* r4 = reinterpret_cast<const float4*>(row);
            for (; i + 16 <= dim; i += 16) {
                const float4 x0 = r4[i / 4], x1 = r4[i / 4 + 1], x2 = r4[i / 4 + 2], x3 = r4[i / 4 + 3];
                acc = acc + x0.x * x0.x; acc = acc + x0.y * x0.y; acc = acc + x0.z * x0.z; acc = acc + x0.w * x0.w;
                acc = acc + x1.x * x1.x; acc = acc + x1.y * x1.y; acc = acc + x1.z * x1.z; acc = acc + x1.w * x1.w;
                acc = acc + x2.x * x2.x; acc = acc + x2.y * x2.y; acc = acc + x2.z * x2.z; acc = acc + x2.w * x2.w;
                acc = acc + x3.x * x3.x; acc = acc + x3.y * x3.y; acc = acc + x3.z * x3.z; acc = acc + x3.w * x3.w;
            }
        }
        if (real)
            for (; i < dim; ++i) {
                const float x = staged ? row[i] : src[i];
                acc = acc + x * x;
            }
        const float m = __builtin_sqrtf(acc);
        const bool approx_ok = real && !bad && isfinite(m) && m >= 1e-18f && m <= 1e18f;
        const uint32_t f = real ? ((bad ? kQueryNonFinite : 0u) | (approx_ok ? 0u : kQueryNoApprox)) : kQueryNoApprox;
        nb[qi] = real ? m : 0.0f;
        qflags[qi] = f;
        qids[qi] = (int32_t)(real ? qi : (nq ? nq - 1 : 0));
        if (f & kQueryNonFinite) atomicOr(status + kStQueryFlags, kQueryNonFinite);
        s_flags = f;
    }
    __syncthreads();
    const bool ok = !(s_flags & kQueryNoApprox);
    if (!with_op || w != 1) return;
    // wave 1: keep the speculative operand (the filter serves this query) or zero it
    int8_t* o = static_cast<int8_t*>(qop) + (uint64_t)qi * ld;
    for (uint32_t g = 0, c0 = lane * 4; c0 < ld; ++g, c0 += 4 * kWave) {
        if (g < (uint32_t)QV) *reinterpret_cast<char4*>(o + c0) = ok ? qv[g] : make_char4(0, 0, 0, 0);
        else if (!ok) *reinterpret_cast<char4*>(o + c0) = make_char4(0, 0, 0, 0);
    }
    if (lane == 0) {
        qscale[qi] = ok ? sc : 0.0f;
        if (ok) {
            const double ea = (double)__uint_as_float(*ea_max);
            const double eb = sqrt(e2) * (1.0 + 1e-9) + 1e-12;
            ebound[qi] = f32_round_up(ea + eb + ea * eb + 1.5e-4);
        } else {
            ebound[qi] = INFINITY;
        }
    }
}

// ------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------
static inline uint32_t grid_for(uint64_t work, uint32_t block, uint32_t cap = 65536) {
    uint64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    return (uint32_t)(g > cap ? cap : g);
}

// ------------------------------------------------------------------------------------
// The loopback communicator's all-gather (bsr_comm_init_loopback): slot r of
// recv [P][bytes] receives this rank's `send` (r == rank, or every slot when there is no
// script) or the recorded contribution script[r] of a real P-rank run -- one launch on the
// stream where ncclAllGather would sit, no host wait.  bytes % 4 == 0.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gather_emulate(const uint32_t* __restrict__ send,
                                                        const uint32_t* __restrict__ script,
                                                        uint32_t* __restrict__ recv, uint64_t words,
                                                        uint32_t P, uint32_t rank) {
    const uint64_t total = words * P;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = (uint32_t)(e / words);
        const uint64_t i = e - (uint64_t)r * words;
        recv[e] = (script && r != rank) ? script[e] : send[i];
    }
}

// ------------------------------------------------------------------------------------
// The parallel search's header exchange without host copies (round 5): k_header_put writes this
// rank's 8 words (kernel arguments) into the device send buffer; after the all-gather,
// k_header_publish copies the P received headers into fine-grained pinned host memory with
// system-scope stores, releases them at system scope and then stores the search's sequence
// number into the host flag the host polls.  (Small hipMemcpyAsync copies to and from pinned
// memory return only when they are done: the header's two copies held the host's enqueue of
// phase A / phase B for their round trip.)
// ------------------------------------------------------------------------------------
struct HeaderWords { int32_t w[8]; };
__global__ void k_header_put(HeaderWords h, int32_t* __restrict__ dst) {
    if (threadIdx.x < 8) dst[threadIdx.x] = h.w[threadIdx.x];
}
__global__ __launch_bounds__(256) void k_header_publish(const int32_t* __restrict__ src, uint32_t words,
                                                        int32_t* host, uint32_t* host_flag, uint32_t seq) {
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
        __hip_atomic_store(host + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(host_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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
hipError_t launch_row_norms(const float* rows, uint64_t n, uint32_t dim, uint32_t ld, float* na,
                            uint32_t* flags, hipStream_t s) {
    hipLaunchKernelGGL(k_row_norms, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, rows, n, dim, ld,
                       na, flags);
    return hipGetLastError();
}
hipError_t launch_rows_to_i8(const float* rows, uint64_t n, uint64_t n_pad, uint32_t dim, uint32_t ld,
                             int8_t* out, float* scales, uint32_t* ea_max, hipStream_t s) {
    const uint64_t blocks = n_pad / kQuantBlock;
    hipLaunchKernelGGL(k_rows_to_i8, dim3((uint32_t)blocks), dim3(256), 0, s, rows, n, dim, ld, out, scales,
                       ea_max);
    return hipGetLastError();
}
hipError_t launch_rows_to_i8_sample(const float* rows, uint64_t n, uint32_t dim, uint32_t ld, int8_t* out,
                                    float* scales, hipStream_t s) {
    const uint64_t n_s = (n + kSampleStride - 1) / kSampleStride;
    const uint64_t blocks = (n_s + kSampleScaleRows - 1) / kSampleScaleRows;
    if (blocks)
        hipLaunchKernelGGL(k_rows_to_i8_sample, dim3((uint32_t)blocks), dim3(256), 0, s, rows, n, dim, ld, out,
                           scales);
    return hipGetLastError();
}
hipError_t launch_query_prep(const QueryPrepArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_query_prep, dim3(a.qpad), dim3(128), 0, s, a.q, a.nq, a.dim, a.ld, a.with_op,
                       a.ea_max, a.qf32, a.nb, a.qop, a.qscale, a.ebound, a.qflags, a.qids, a.status);
    return hipGetLastError();
}

hipError_t launch_gather_emulate(const void* send, const void* script, void* recv, uint64_t bytes, uint32_t P,
                                 uint32_t rank, hipStream_t s) {
    if (bytes % 4) return hipErrorInvalidValue;
    const uint64_t words = bytes / 4, total = words * P;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, std::max<uint64_t>(1, (total + 255) / 256));
    hipLaunchKernelGGL(k_gather_emulate, dim3(grid), dim3(256), 0, s, static_cast<const uint32_t*>(send),
                       static_cast<const uint32_t*>(script), static_cast<uint32_t*>(recv), words, P, rank);
    return hipGetLastError();
}

hipError_t launch_header_put(const int32_t w[8], int32_t* dst, hipStream_t s) {
    HeaderWords h;
    for (int i = 0; i < 8; ++i) h.w[i] = w[i];
    hipLaunchKernelGGL(k_header_put, dim3(1), dim3(64), 0, s, h, dst);
    return hipGetLastError();
}
hipError_t launch_header_publish(const int32_t* src, uint32_t words, int32_t* host, uint32_t* host_flag, uint32_t seq,
                                 hipStream_t s) {
    hipLaunchKernelGGL(k_header_publish, dim3(1), dim3(256), 0, s, src, words, host, host_flag, seq);
    return hipGetLastError();
}

}  // namespace bsr
