// bsr_device.hpp -- device-side building blocks shared by the kernels (gfx950, wave64).
//
// * Exact distance: the reference's cosine_distance (src/metrics.rs:143-165) finished from
//   per-lane sequential partial sums.  This translation unit is compiled with
//   -ffp-contract=off, so `a * b` and `acc + p` round separately exactly like Rust's f32
//   ops; sqrt uses __builtin_sqrtf (correctly rounded; NB: HIP's __fsqrt_rn lowers to the
//   approximate native sqrt on ROCm 7.2) and `/` is the correctly rounded division.
// * Keys: a result (distance d >= 0, local row r) is the u64 (bits(d) << 32) | r, so the
//   reference's order (distance asc, index asc -- SURVEY.md §8a-5) is plain u64 order.
// * WaveTopK<E>: a sorted list of the 64*E smallest keys held by one wavefront, position
//   p = e*64 + lane.  Insertion is wave-parallel (ballot + popcount + one shuffle).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bsr {

constexpr int kWave = 64;
constexpr uint64_t kKeyNone = ~0ull;

__device__ __forceinline__ uint64_t dist_key(float d, uint32_t row) {
    return ((uint64_t)__float_as_uint(d) << 32) | (uint64_t)row;
}
__device__ __forceinline__ float key_dist(uint64_t k) { return __uint_as_float((uint32_t)(k >> 32)); }
__device__ __forceinline__ uint32_t key_row(uint64_t k) { return (uint32_t)k; }

// Score keys order LARGER approximate scores first (then smaller row): the candidate
// stage keeps the smallest score keys.
__device__ __forceinline__ uint32_t ord_f32(float s) {
    uint32_t u = __float_as_uint(s);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
__device__ __forceinline__ uint64_t score_key(float s, uint32_t row) {
    return ((uint64_t)(~ord_f32(s)) << 32) | (uint64_t)row;
}
__device__ __forceinline__ float score_key_score(uint64_t k) { return unord_f32(~(uint32_t)(k >> 32)); }

// Round-to-nearest-even f32 -> bf16 bits (inputs are finite here).
__device__ __forceinline__ uint16_t f32_to_bf16_rne(float x) {
    uint32_t u = __float_as_uint(x);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

// src/metrics.rs:144-164 given the sequential dot product, the max |a_i - b_i| (the
// identical test `all |a_i-b_i| <= 1e-10` is `max <= 1e-10` for finite inputs) and the two
// magnitudes (each sqrt of a sequential sum of squares).
__device__ __forceinline__ float finish_distance(float dot, float maxdiff, float mag_a, float mag_b) {
    if (maxdiff <= 1e-10f) return 0.0f;                 // :149-151
    if (mag_a == 0.0f || mag_b == 0.0f) return 1.0f;    // :157-159
    float denom = mag_a * mag_b;
    float s = dot / denom;                              // :161
    s = fmaxf(s, -1.0f);                                // :162 .max(-1.0) (maxNum: NaN -> -1)
    s = fminf(s, 1.0f);                                 //      .min(1.0)
    return 1.0f - s;                                    // :164
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)x, l);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
// Cross-lane moves inside the VALU (no LDS round trip: __shfl* lower to ds_bpermute):
// DPP quad_perm / row rotations / row_mirror / wave_shr and v_permlane16/32_swap.
template <int CTRL>
__device__ __forceinline__ uint32_t dppc(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}
// The value lane (lane ^ M) holds, for a constant M in {1, 2, 4, 8, 16, 32}.
template <int M>
__device__ __forceinline__ uint32_t xor_lane32(uint32_t x) {
    if constexpr (M == 1) return dppc<0xB1>(x);        // quad_perm [1,0,3,2]
    else if constexpr (M == 2) return dppc<0x4E>(x);   // quad_perm [2,3,0,1]
    else if constexpr (M == 4) {
        const uint32_t up = dppc<0x12C>(x);  // row_ror:12 -> lane + 4 (within its row of 16)
        const uint32_t dn = dppc<0x124>(x);  // row_ror:4  -> lane - 4
        return (lane_id() & 4) ? dn : up;
    } else if constexpr (M == 8) return dppc<0x128>(x);  // row_ror:8 -> lane ^ 8
    else if constexpr (M == 16) {
        // odd rows of the first operand swap with even rows of the second: with both = x,
        // r[1] holds row r+1 in even rows, r[0] holds row r-1 in odd rows
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane_id() & 16) ? (uint32_t)r[0] : (uint32_t)r[1];
    } else {
        static_assert(M == 32, "xor 1..32");
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane_id() & 32) ? (uint32_t)r[0] : (uint32_t)r[1];
    }
}
__device__ __forceinline__ uint32_t xor_lane32(uint32_t x, int m) {  // m a constant after unrolling
    switch (m) {
        case 1: return xor_lane32<1>(x);
        case 2: return xor_lane32<2>(x);
        case 4: return xor_lane32<4>(x);
        case 8: return xor_lane32<8>(x);
        case 16: return xor_lane32<16>(x);
        default: return xor_lane32<32>(x);
    }
}
// Butterfly reductions over the wave (xor 32, 16, ..., 1), every lane gets the result.
template <class F>
__device__ __forceinline__ uint32_t wave_reduce_u32(uint32_t v, F op) {
    v = op(v, xor_lane32<32>(v));
    v = op(v, xor_lane32<16>(v));
    v = op(v, xor_lane32<8>(v));
    v = op(v, xor_lane32<4>(v));
    v = op(v, xor_lane32<2>(v));
    return op(v, xor_lane32<1>(v));
}
__device__ __forceinline__ uint64_t shfl_up1_64(uint64_t x) {  // lane - 1 (lane 0: its own)
    const uint32_t lo = dppc<0x138>((uint32_t)x);          // wave_shr:1
    const uint32_t hi = dppc<0x138>((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t x, int src) {
    int lo = __shfl((int)(uint32_t)x, src, kWave);
    int hi = __shfl((int)(uint32_t)(x >> 32), src, kWave);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int m) {
    const uint32_t lo = xor_lane32((uint32_t)x, m);
    const uint32_t hi = xor_lane32((uint32_t)(x >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}
// The value lane 63 - lane holds: row_mirror (lane ^ 15 within its row), then ^ 16, ^ 32.
__device__ __forceinline__ uint64_t reverse64(uint64_t x) {
    uint32_t lo = dppc<0x140>((uint32_t)x), hi = dppc<0x140>((uint32_t)(x >> 32));
    lo = xor_lane32<32>(xor_lane32<16>(lo));
    hi = xor_lane32<32>(xor_lane32<16>(hi));
    return ((uint64_t)hi << 32) | lo;
}
// Ascending bitonic sort of one key per lane across the wave (21 compare-exchange steps).
__device__ __forceinline__ uint64_t wave_sort64(uint64_t x) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t y = shfl_xor64(x, j);
            const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
            x = keep_min ? (x < y ? x : y) : (x < y ? y : x);
        }
    }
    return x;
}
// A bitonic sequence of 64 keys (one per lane) -> ascending.
__device__ __forceinline__ uint64_t bitonic_clean64(uint64_t x) {
    const int lane = lane_id();
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) {
        const uint64_t y = shfl_xor64(x, j);
        x = (lane & j) ? (x < y ? y : x) : (x < y ? x : y);
    }
    return x;
}

template <int E>
struct WaveTopK {
    uint64_t v[E];

    __device__ __forceinline__ void init() {
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = kKeyNone;
    }
    // Key at (wave-uniform) position pos.
    // (Each entry is read out as a wave-uniform scalar and selected afterwards: selecting
    // v[e] first lets LLVM fold the chain into a dynamically indexed stack array.)
    __device__ __forceinline__ uint64_t at(int pos) const {
        const int e = pos >> 6, l = pos & 63;
        uint64_t x = readlane64(v[0], l);
#pragma unroll
        for (int i = 1; i < E; ++i) {
            const uint64_t y = readlane64(v[i], l);
            x = (i == e) ? y : x;
        }
        return x;
    }
    // Insert a wave-uniform key (duplicates allowed; the largest entry falls off).
    __device__ __forceinline__ void insert(uint64_t x) {
        const int lane = lane_id();
        int pos = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) pos += __popcll(__ballot(v[e] < x));
#pragma unroll
        for (int e = E - 1; e >= 0; --e) {
            const uint64_t up = shfl_up1_64(v[e]);
            const uint64_t carry = (e > 0) ? readlane64(v[e > 0 ? e - 1 : 0], 63) : kKeyNone;
            const uint64_t prev = (lane == 0) ? carry : up;
            const int p = e * kWave + lane;
            v[e] = (p > pos) ? prev : ((p == pos) ? x : v[e]);
        }
    }
    // Merge a batch of up to 64 keys (one per lane, kKeyNone = nothing) into the list:
    // bitonic sort of the batch across the wave, then a merge cascade down the E registers
    // (min/max against the reversed batch leaves two bitonic halves, each sorted by a
    // 6-step half-cleaner; the larger half moves on to the next register).
    __device__ __forceinline__ void merge_batch(uint64_t x) {
        x = wave_sort64(x);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint64_t xr = reverse64(x);
            const uint64_t lo = v[e] < xr ? v[e] : xr;
            const uint64_t hi = v[e] < xr ? xr : v[e];
            v[e] = bitonic_clean64(lo);
            if (e + 1 < E) x = bitonic_clean64(hi);
        }
    }
    // Offer one key per lane (kKeyNone = nothing); keeps the smallest `k` keys seen
    // (k <= 64*E).  `thr` is the current k-th smallest key, updated.  A few passing keys
    // are inserted one by one; a larger batch is merged.
    __device__ __forceinline__ void offer(uint64_t x, int k, uint64_t& thr) {
        uint64_t m = __ballot(x < thr);
        if (!m) return;
        if (__popcll(m) > 3) {
            merge_batch(x < thr ? x : kKeyNone);
            thr = at(k - 1);
            return;
        }
        while (m) {
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            const uint64_t y = readlane64(x, l);
            if (y < thr) {
                insert(y);
                thr = at(k - 1);
            }
        }
    }
    // Store the first n positions (n <= 64*E) to out[0..n).
    __device__ __forceinline__ void store(uint64_t* out, int n) const {
        const int lane = lane_id();
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int p = e * kWave + lane;
            if (p < n) out[p] = v[e];
        }
    }
};

// splitmix64 finaliser: the counter-based generator behind bsr_synth_uniform.
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

}  // namespace bsr
