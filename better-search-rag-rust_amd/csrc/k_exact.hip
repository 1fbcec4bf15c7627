// k_exact.hip -- the reference's exact arithmetic on the GPU (gfx950): candidate rescoring
// with certification, the exact full scan, per-block list merges and output finalisation.
//
// Compiled with -ffp-contract=off: every f32 multiply and add rounds separately, in index
// order, exactly as src/metrics.rs:153-155 does; sqrt is __builtin_sqrtf (correctly
// rounded) and `/` is the correctly rounded division (see bsr_device.hpp).
#include <cstdlib>
#include "bsr_device.hpp"
#include "kernels.hpp"

#include <math.h>

#include <algorithm>
#include <type_traits>

// Workgroups that write result rows straight into the pinned host mirror (host_put) release them
// at system scope before they end or arrive at the publish ticket (round 5, VERDICT r04: the
// memory model's form for a host consumer; 0 = the round-4 form, vmcnt(0) alone -- lab A/B only).
#ifndef BSR_PUB_SYSREL
#define BSR_PUB_SYSREL 1
#endif


namespace {
// A system-scope release of this wave's prior stores (buffer_wbl2 sc0 sc1 + the wait), then the
// explicit vmcnt(0) the guide's compiler-hazard note asks for between a release and a flag.
__device__ __forceinline__ void release_system() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// The publish copy (device result -> fine-grained host memory) by the threads t of n of one
// workgroup: 8 loads in flight per thread before their stores (a load-store pair per trip would
// wait out one load latency per 16 bytes x n)
__device__ __forceinline__ void publish_copy(const uint8_t* src8, uint8_t* dst8, size_t bytes, uint32_t t, uint32_t n) {
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(src8);
    uint4* __restrict__ dst = reinterpret_cast<uint4*>(dst8);
    const size_t n16 = bytes / 16;
    size_t i = t;
    for (; i + 7 * (size_t)n < n16; i += 8 * (size_t)n) {
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = src[i + j * (size_t)n];
#pragma unroll
        for (int j = 0; j < 8; ++j) dst[i + j * (size_t)n] = v[j];
    }
    for (; i < n16; i += n) dst[i] = src[i];
}
// A result value into the pinned host mirror: a system-scope store (written through, never left
// in an L2), so that the writing wave's s_waitcnt vmcnt(0) is all the host needs before the flag
__device__ __forceinline__ void host_put(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void host_put(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void host_put(float* p, float v) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The publishing kernels' "who arrived last" (one thread per workgroup, after the workgroup's
// release): an add to the workgroup's leaf counter (blockIdx % 8), and for the last of a leaf an
// add to the root -- the workgroups of a launch split over 9 lines instead of queueing on one
// (1000 adds to one word are the larger part of a 1000-workgroup publish).  The last workgroup
// to arrive zeroes the counters for the next launch (the stream orders it before that launch).
__device__ bool last_arrival(uint32_t* ticket) {
    constexpr uint32_t L = bsr::kTicketLeaves, S = bsr::kTicketStride;
    const uint32_t nb = gridDim.x, leaf = blockIdx.x % L;
    const uint32_t in_leaf = (nb - leaf + L - 1) / L;  // workgroups b < nb with b % L == leaf
    if (atomicAdd(ticket + leaf * S, 1u) != in_leaf - 1) return false;
    const uint32_t leaves = nb < L ? nb : L;
    if (atomicAdd(ticket + L * S, 1u) != leaves - 1) return false;
    for (uint32_t i = 0; i <= L; ++i) ticket[i * S] = 0u;
    return true;
}
}  // namespace

namespace bsr {
typedef __attribute__((address_space(3))) void lds_void_t;

static inline uint32_t grid_for(uint64_t work, uint32_t block, uint32_t cap = 65536) {
    uint64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    return (uint32_t)(g > cap ? cap : g);
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

// This wave's LDS stage for the candidate rows is private to it (W > 1 waves per workgroup
// each walk their own 64 candidates): ordering inside the wave is enough.
// The LDS executes one wave's operations in order, so only the compiler must not move LDS
// accesses across this point.  (A fence or __syncthreads would also wait for every global
// load in flight -- vmcnt(0) -- and serialise the two-chunk prefetch below.)
__device__ __forceinline__ void wave_sync() { asm volatile("" ::: "memory"); }

// Mode S's candidate selection, one wave: the (kp+1)-th smallest of the c emitted keys xk (cap <=
// 1024: 16 registers, kp <= 63) by radix select -- the high words first (score bits: only the bits
// below the highest one in which the emitted keys differ are searched), then, only when several
// keys share the K-th high word, the low words (rows) among those -- and the kp keys below it
// compacted through lsel (LDS, 64 words): lane l's row in sel_row (l < c on return).  tx_sel: the
// (kp+1)-th score (every row left out is at most that), or tau0 when every emitted row is a
// candidate; INFINITY for an overflowed list.
// kth_key<NR>: the K-th smallest of the valid keys (kKeyNone = no key; at least K valid) held NR
// per lane -- the radix search above; only slots j * 64 + lane < dense_c can hold keys (~0u: any).
template <int NR>
__device__ __forceinline__ uint64_t kth_key(const uint64_t (&x)[NR], uint32_t K, uint32_t dense_c) {
    uint32_t hmin = ~0u, hmax = 0;
#pragma unroll
    for (int j = 0; j < NR; ++j)
        if (x[j] != kKeyNone) {
            hmin = min(hmin, (uint32_t)(x[j] >> 32));
            hmax = max(hmax, (uint32_t)(x[j] >> 32));
        }
    hmin = wave_reduce_u32(hmin, [](uint32_t a, uint32_t b) { return min(a, b); });
    hmax = wave_reduce_u32(hmax, [](uint32_t a, uint32_t b) { return max(a, b); });
    const uint32_t diff = hmin ^ hmax;
    const int top = diff ? 31 - __builtin_clz(diff) : -1;
    // (top < 0: every key has the same high word)
    uint32_t Th = top < 0 ? hmin : top >= 31 ? 0u : (hmin & ~((2u << top) - 1u));
    for (int b = top; b >= 0; --b) {
        const uint32_t t = Th | (1u << b);
        uint32_t below = 0;
#pragma unroll
        for (int j = 0; j < NR; ++j)
            if ((uint32_t)(j * kWave) < dense_c) below += (uint32_t)__popcll(__ballot((uint32_t)(x[j] >> 32) < t));
        if (below < K) Th = t;
    }
    uint32_t lt = 0, eq = 0;
#pragma unroll
    for (int j = 0; j < NR; ++j)
        if ((uint32_t)(j * kWave) < dense_c) {
            const uint32_t h = (uint32_t)(x[j] >> 32);
            lt += (uint32_t)__popcll(__ballot(x[j] != kKeyNone && h < Th));
            eq += (uint32_t)__popcll(__ballot(x[j] != kKeyNone && h == Th));
        }
    const uint32_t K2 = K - lt;  // 1 <= K2 <= eq
    uint32_t Tl = 0;
    if (eq > 1)
        for (int b = 31; b >= 0; --b) {
            const uint32_t t = Tl | (1u << b);
            uint32_t below = 0;
#pragma unroll
            for (int j = 0; j < NR; ++j)
                if ((uint32_t)(j * kWave) < dense_c)
                    below += (uint32_t)__popcll(__ballot((uint32_t)(x[j] >> 32) == Th && (uint32_t)x[j] < t));
            if (below < K2) Tl = t;
        }
    else
#pragma unroll
        for (int j = 0; j < NR; ++j) {  // the one key with high word Th
            const uint64_t m = __ballot(x[j] != kKeyNone && (uint32_t)(x[j] >> 32) == Th);
            if (m) Tl = (uint32_t)__shfl((int)(uint32_t)x[j], __builtin_ctzll(m), kWave);
        }
    return ((uint64_t)Th << 32) | Tl;
}
// (select_kp_n<NR>: NR keys per lane; sparse = true: the kKeyNone slots may lie anywhere among
// the first slots -- c counts the valid keys, each slot is masked by its own key, not its index)
template <int NR>
__device__ __forceinline__ void select_kp_n(const uint64_t (&xk)[NR], uint32_t& c, bool overflow, uint32_t kp,
                                            float tau0, float& tx_sel, uint32_t* lsel, uint32_t& sel_row, int lane,
                                            bool sparse = false) {
    uint64_t x[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        const uint32_t i = j * kWave + lane;
        x[j] = (sparse || i < c) ? xk[j] : kKeyNone;
    }
    uint64_t T = kKeyNone;
    if (!overflow && c > kp) {
        T = kth_key<NR>(x, kp + 1, sparse ? ~0u : c);
        tx_sel = score_key_score(T);
        c = kp;
    } else if (!overflow) {
        tx_sel = tau0;  // every emitted row is a candidate; tau0 bounds the rest
    }
    uint32_t base = 0;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        const bool pick = x[j] < T;
        const uint64_t m = __ballot(pick);
        if (pick) {
            const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            lsel[pos] = key_row(x[j]);
        }
        base += (uint32_t)__popcll(m);
    }
    wave_sync();
    sel_row = lane < (int)c ? lsel[lane] : 0u;
    wave_sync();
}

__device__ __forceinline__ void select_kp(const uint64_t (&xk)[16], uint32_t& c, bool overflow, uint32_t kp,
                                          float tau0, float& tx_sel, uint32_t* lsel, uint32_t& sel_row, int lane) {
    select_kp_n<16>(xk, c, overflow, kp, tau0, tx_sel, lsel, sel_row, lane);
}

// Certification: every row outside the candidate set has approximate cosine
// <= tau_x, hence reference cosine <= tau_x + E_q and reference distance >= 1 - tau_x - E_q -
// 2^-23; the k-th exact distance (key thr) must lie strictly below that, and no excluded row can
// be element-wise identical to the query.  tau_x = -inf: every row of the shard was a candidate.
__device__ __forceinline__ bool certify(float tx, uint64_t thr, float ebound_q, float mag_b) {
    const double ebound = (double)ebound_q;
    if (tx == -INFINITY) return true;
    if (!(tx < INFINITY) || thr == kKeyNone) return false;
    const double dk = (double)key_dist(thr);
    return ebound < 1.0 && dk < 1.0 - (double)tx - ebound - 2.5e-7 &&
           (double)tx < 1.0 - ebound - 1e-4 - 6e-9 / (double)mag_b;
}
// The global threshold's exclusion bound of one rank's list: the distance below
// which no row it left out can lie, 1 - tau0 - E_q - 2.5e-7 rounded down; +inf when every row of
// the shard was a candidate, -inf when nothing can be certified.
__device__ __forceinline__ float exclusion_bound(float tx, float ebound_q, float mag_b) {
    const double eb = (double)ebound_q;
    double x;
    if (tx == -INFINITY) x = INFINITY;
    else if (!(tx < INFINITY) || !(eb < 1.0) || !((double)tx < 1.0 - eb - 1e-4 - 6e-9 / (double)mag_b))
        x = -INFINITY;
    else x = 1.0 - (double)tx - eb - 2.5e-7;
    float xf = (float)x;
    if ((double)xf > x) xf = nextafterf(xf, -INFINITY);  // (rounded down)
    return xf;
}
// A query's list (one wave, WaveTopK order) as its first `cnt` result rows (global index,
// distance), the rest (~0, +inf), and its count -- in device memory and, when the launch has one,
// the pinned host mirror too.  Returns whether host-mirror rows were written (to be released).
template <int E>
__device__ __forceinline__ bool put_result_rows(const RescoreArgs& a, uint32_t q, const WaveTopK<E>& L, uint32_t cnt,
                                                int lane) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t i = e * kWave + lane;
        if (i < a.k) {
            const uint64_t key = L.v[e];
            const bool has = i < cnt && key != kKeyNone;
            const uint64_t gi = has ? a.offset + key_row(key) : ~0ull;
            const float gd = has ? key_dist(key) : INFINITY;
            a.res_idx[(uint64_t)q * a.k + i] = gi;
            a.res_dist[(uint64_t)q * a.k + i] = gd;
            if (a.hres_idx) {
                host_put(a.hres_idx + (uint64_t)q * a.k + i, gi);
                host_put(a.hres_dist + (uint64_t)q * a.k + i, gd);
            }
        }
    }
    if (lane == 0) {
        a.res_cnt[q] = cnt;
        if (a.hres_cnt) host_put(a.hres_cnt + q, cnt);
    }
    return a.hres_idx != nullptr || a.hres_cnt != nullptr;
}

// W waves per workgroup, one query per workgroup at a time: wave w takes candidates
// w*64 + lane, + 64W, ...; the W per-wave lists merge through LDS.  W = 1: one wave per
// query (the k' selected candidates, every query).  W = 8: the queries that failed
// certification, every emitted row (~4k'), their count read on the device
// (a.n_items_dev), so the launch needs no host round trip.  P chunks of candidate rows are
// loaded ahead (rows of 768 floats; other widths: 2).
#ifdef BSR_RESCORE_STAMPS
// (lab build only: per-wave phase timestamps of the one-wave-per-query rescore, 100 MHz clock,
// indexed by the item)
__device__ uint64_t g_rescore_stamps[4096 * 8];
#define BSR_STAMP(W_, I_)                                                                          \
    do {                                                                                           \
        if ((W_) == 1 && (threadIdx.x & 63) == 0 && item < 2048)                                   \
            g_rescore_stamps[item * 8 + (I_)] = __builtin_amdgcn_s_memrealtime();                  \
        if ((W_) > 1 && threadIdx.x == 0 && item < 2048) /* (the second chance: slots 2048 +) */   \
            g_rescore_stamps[(2048 + item) * 8 + (I_)] = __builtin_amdgcn_s_memrealtime();         \
    } while (0)
#else
#define BSR_STAMP(W_, I_) \
    do {                  \
    } while (0)
#endif

// QPW > 1 (W = 1): QPW independent waves per workgroup, each its own item with its own LDS stage
// and query copy (round 5).  One-wave workgroups let the dispatcher put two waves of a 1000-item
// launch on one SIMD while others stay empty: those waves ran ~1.5x long and set the kernel's
// time (median wave 27 us, kernel 42 us at the 1.25M shard, profiles/r05e_rstamps_gtau.txt); a
// 4-wave workgroup with 86 KB of LDS is alone on its CU, one wave per SIMD.
template <int E, int W, int P, int QPW = 1>
__global__ __launch_bounds__(64 * W * QPW) void k_rescore(RescoreArgs a) {
    static_assert(QPW == 1 || W == 1, "independent waves per workgroup: one wave per item");
    constexpr int STAGE = 64 * 68;  // 64 rows (stride 68) per wave
    constexpr int QMAX = 1024;      // the whole query in LDS (rows up to 1024 floats)
    __shared__ __attribute__((aligned(16))) float lds_all[QPW > 1 ? QPW * (STAGE + QMAX) : W * STAGE + QMAX];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float* const lds = lds_all + (QPW > 1 ? w * (STAGE + QMAX) : w * STAGE);
    float* const ldq_all = QPW > 1 ? lds + STAGE : lds_all + W * STAGE;
    const uint32_t n_items = a.n_items_dev ? *a.n_items_dev : a.n_items;
    // (publish) this workgroup wrote state the publishing workgroup reads: the status words
    // (block 0) or a failure list entry
    __shared__ uint32_t s_wrote;
    if (threadIdx.x == 0) s_wrote = blockIdx.x == 0 ? 1u : 0u;
    if constexpr (QPW > 1) __syncthreads();  // (before any wave's failure entry sets it)
    bool host_rows = false;  // (wave 0) this workgroup wrote result rows into the host mirror
    if ((W > 1 || a.excl_out) && a.next_status && blockIdx.x == 0 && threadIdx.x < kWave) {
        // (k_finalize's bookkeeping, fused: this is the batch's last kernel)
        if (threadIdx.x < kStWords) a.next_status[threadIdx.x] = 0;
        if (a.merge_words && threadIdx.x < 2) a.merge_words[threadIdx.x] = threadIdx.x ? ~0u : 0u;
        uint32_t sum = 0;
        for (uint32_t q = threadIdx.x; q < a.n_queries; q += kWave) sum += a.emit_cnt[q];
        sum = wave_reduce_u32(sum, [](uint32_t x, uint32_t y) { return x + y; });
        if (threadIdx.x == 0) a.cur_status[kStEmitted] = sum;
    }
    for (uint32_t item = blockIdx.x * QPW + (QPW > 1 ? w : 0); item < n_items; item += gridDim.x * QPW) {
        BSR_STAMP(W, 0);
        const uint32_t q = a.qlist ? a.qlist[item] : item;
        // mode S (a.sel: select the k' candidates here, from the emitted keys), mode B (every
        // emitted candidate) or mode A (the k' selected ones, from k_select_cand)
        const bool sel = W == 1 && a.sel;
        const bool all = !sel && a.cand_keys != nullptr;
        // The item's independent loads are all issued before any is consumed -- the candidate
        // count, the emitted keys (mode S: every one of the cap <= 1024 slots, masked by the
        // count afterwards, so they do not wait for it) and the query row in one batch.  (Phase
        // stamps, tools/diag/rescore_stamps.py: query + keys 7.2 -> 5.5 us of a 46-48 us wave;
        // the rows' scan that follows is HBM-bound, ~31 us for 63k rows at 1000 queries.)
        const uint32_t cnt = (sel || all) ? a.cnt[q] : a.ncand[q];
        constexpr int NR = 16;
        uint64_t xk[W == 1 ? NR : 1];
        if constexpr (W == 1) {
            if (sel) {
                const uint64_t* src = a.cand_keys + (uint64_t)q * a.cap;
#pragma unroll
                for (int j = 0; j < NR; ++j) {
                    const uint32_t i = j * kWave + lane;
                    xk[j] = i < a.cap ? src[i] : kKeyNone;
                }
            }
        }
        // the query, once per item (its loads are not behind the candidate prefetch); rows
        // longer than QMAX read it from global memory instead
        const bool qlds = a.ld <= (uint32_t)QMAX;
        if (qlds) {
            constexpr int QN = QMAX / (64 * W);
            const float* qsrc = a.qf32 + (uint64_t)q * a.ld;
            float qv[QN];
            const uint32_t tq = QPW > 1 ? (uint32_t)lane : threadIdx.x;  // (this item's threads)
#pragma unroll
            for (int j = 0; j < QN; ++j) {
                const uint32_t cc = j * 64 * W + tq;
                qv[j] = cc < a.ld ? qsrc[cc] : 0.0f;
            }
#pragma unroll
            for (int j = 0; j < QN; ++j) {
                const uint32_t cc = j * 64 * W + tq;
                if (cc < a.ld) ldq_all[cc] = qv[j];
            }
        }
        if constexpr (W > 1) __syncthreads();
        else wave_sync();
        BSR_STAMP(W, 1);
        const bool overflow = (sel || all) && cnt > a.cap;  // rows were dropped: nothing can be certified
        uint32_t c = overflow ? 0u : cnt;
        float tx_sel = INFINITY;
        uint32_t sel_row = 0;
        if constexpr (W == 1) {
            if (sel) select_kp(xk, c, overflow, a.kp, a.tau0[q], tx_sel, reinterpret_cast<uint32_t*>(lds), sel_row, lane);
        }
        BSR_STAMP(W, 2);
        const float mag_b = a.nb[q];
        const uint32_t ld = a.ld, dim = a.dim, nch = ld / 64;
        const float* rows = a.rows;

        WaveTopK<E> L;
        L.init();
        uint64_t thr = kKeyNone;
        // QL: the query chunk from the LDS copy (typed as LDS after inlining: ds_read), else
        // from global memory (rows longer than QMAX)
        // NC > 0: the chunk count as a constant (ld = 64 NC; the loop below fully unrolls, so
        // the prefetch's vmcnt waits are exact); NC = 0: any ld
        auto scan = [&](auto ql_tag, auto nc_tag) {
            constexpr bool QL = decltype(ql_tag)::value;
            constexpr uint32_t NC = decltype(nc_tag)::value;
            const uint32_t nchk = NC ? NC : nch;
            for (uint32_t base = QPW > 1 ? 0u : 64u * w; base < c; base += 64 * W) {
                const uint32_t ci = base + lane, cc = ci < c ? ci : 0;
                const uint64_t ck = all ? a.cand_keys[(uint64_t)q * a.cap + cc] : 0ull;
                const bool valid = ci < c && ck != kKeyNone;  // (an empty slot of a list: no row)
                const uint32_t myrow = sel ? sel_row
                                     : all ? (ck != kKeyNone ? key_row(ck) : 0u)
                                           : a.cand_rows[(uint64_t)q * a.kp + cc];
                float acc[1] = {-0.0f}, mx[1] = {0.0f};
                uint32_t lrow[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) lrow[i] = (uint32_t)__shfl((int)myrow, (i * 64 + lane) >> 4, kWave);
                // one chunk: this wave's 64 rows x 64 elements through its LDS stage, then each
                // lane walks its row in index order
                auto step = [&](f32x4_t (&pre)[16], uint32_t ch, uint32_t ahead) {
                    wave_sync();
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int L16 = i * 64 + lane;
                        *reinterpret_cast<f32x4_t*>(lds + (L16 >> 4) * 68 + (L16 & 15) * 4) = pre[i];
                    }
                    wave_sync();
                    if (ch + ahead < nchk) load_cand_chunk(pre, rows, ld, lrow, ch + ahead, lane);
                    const float* const bb[1] = {QL ? ldq_all + ch * 64 : a.qf32 + (uint64_t)q * ld + ch * 64};
                    const uint32_t nvalid = dim - ch * 64 < 64 ? dim - ch * 64 : 64;
                    seq_chunk<1>(lds + lane * 68, bb, nvalid, acc, mx);
                };
                if constexpr (NC > 0) {
                    // P chunks of loads in flight (a register ring; the loop unrolls fully, so
                    // the vmcnt waits are counted)
                    constexpr uint32_t PP = (uint32_t)P < NC ? (uint32_t)P : NC;
                    f32x4_t pre[PP][16];
#pragma unroll
                    for (uint32_t ch = 0; ch < PP; ++ch) load_cand_chunk(pre[ch], rows, ld, lrow, ch, lane);
#pragma unroll
                    for (uint32_t ch = 0; ch < NC; ++ch) step(pre[ch % PP], ch, PP);
                } else {
                    // any ld: two chunks in flight (register sets A / B)
                    f32x4_t preA[16], preB[16];
                    load_cand_chunk(preA, rows, ld, lrow, 0, lane);
                    if (nchk > 1) load_cand_chunk(preB, rows, ld, lrow, 1, lane);
                    for (uint32_t ch = 0; ch < nchk; ch += 2) {
                        step(preA, ch, 2);
                        if (ch + 1 < nchk) step(preB, ch + 1, 2);
                    }
                }
                const float d = finish_distance(acc[0], mx[0], a.na[myrow], mag_b);
                L.offer(valid ? dist_key(d, myrow) : kKeyNone, (int)a.k, thr);
            }
        };
        if (qlds && nch == 12) scan(std::true_type{}, std::integral_constant<uint32_t, 12>{});
        else if (qlds) scan(std::true_type{}, std::integral_constant<uint32_t, 0>{});
        else scan(std::false_type{}, std::integral_constant<uint32_t, 0>{});
        BSR_STAMP(W, 3);
        if constexpr (W > 1) {
            // the W lists (k <= 64E keys each) through LDS, merged by wave 0
            static_assert(W * 64 * E * 8 <= (int)sizeof(lds_all), "merge area");
            uint64_t* part = reinterpret_cast<uint64_t*>(lds_all);
            __syncthreads();
#pragma unroll
            for (int e = 0; e < E; ++e) part[(w * E + e) * 64 + lane] = L.v[e];
            __syncthreads();
            if (w == 0) {
                WaveTopK<E> M;
                M.init();
                uint64_t mt = kKeyNone;
                for (int src = 0; src < W; ++src)
#pragma unroll
                    for (int e = 0; e < E; ++e) M.offer(part[(src * E + e) * 64 + lane], (int)a.k, mt);
                L = M;
                thr = mt;
            }
            __syncthreads();  // part is the next item's LDS stage
        }
        if (QPW > 1 || w == 0) {
            L.store(a.out_keys + (uint64_t)q * a.k, (int)a.k);
            bool certified = false;
            if (a.excl_out) {
                // (global threshold: the root certifies; this rank reports its exclusion bound)
                if (lane == 0) a.excl_out[q] = exclusion_bound(overflow ? INFINITY : a.tau0[q], a.ebound[q], mag_b);
            } else if (lane == 0) {
                // (mode B: every emitted row is a candidate, so tau_x is the emission threshold tau0)
                const float tx = overflow ? INFINITY : sel ? tx_sel : (all ? a.tau0[q] : a.tau_excl[q]);
                const bool ok = certify(tx, thr, a.ebound[q], mag_b);
                if (!ok) {
                    const uint32_t pos = atomicAdd(a.fail_cnt, 1u);
                    a.fail_list[pos] = q;
                    s_wrote = 1u;
                }
                certified = ok;
            }
            // fused finalize: certified lists (modes S / A) and every second-chance item (mode
            // B) become result rows now; the first pass's uncertified ones are left to mode B
            if (a.res_idx && (W > 1 || a.excl_out || __shfl((int)certified, 0, kWave))) {
                const uint32_t cnt = a.excl_out ? min(a.k, c) : (uint64_t)a.k < a.n_rows ? a.k : (uint32_t)a.n_rows;
                host_rows = put_result_rows(a, q, L, cnt, lane) || host_rows;
            }
        }
        BSR_STAMP(W, 4);
    }
    // (a kernel that does not publish -- the first pass -- releases its host rows here: the host
    // reads them once the batch's last kernel has raised the flag)
    if (BSR_PUB_SYSREL && !a.pub_flag && __ballot(host_rows)) release_system();
    if (a.pub_flag) {
        // publish: every workgroup's writes released (system scope when it wrote result rows
        // to the host mirror itself, else agent scope) before its ticket; the last one acquires
        // them, copies pub_bytes of the packed result (with a host mirror: the status words
        // alone) to host memory, releases it at system scope and raises the flag the host polls
        // Only a workgroup that wrote what the last one reads releases it to the agent (an agent
        // fence writes back its XCD's L2): block 0's status words, a failure entry -- and, without
        // a host mirror, the result rows it wrote.  A workgroup that wrote result rows into the host
        // mirror releases them at system scope (BSR_PUB_SYSREL) before its ticket: the host reads
        // them once it sees the flag.
        // (a one-workgroup grid -- a tiny batch's second chance -- is its own last arrival: no
        // agent fences, no ticket)
        const bool solo = a.solo != 0;
        __shared__ uint32_t s_last;
        __syncthreads();  // (s_wrote final)
        if (!solo && (s_wrote || (!a.hres_idx && blockIdx.x * QPW < n_items))) __threadfence();
        if (BSR_PUB_SYSREL && __ballot(host_rows)) release_system();  // (wave 0 wrote them)
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) s_last = solo || last_arrival(a.pub_ticket) ? 1u : 0u;
        __syncthreads();
        if (s_last) {
#ifdef BSR_RESCORE_STAMPS
            if (W > 1 && threadIdx.x == 0) g_rescore_stamps[4095 * 8 + 0] = __builtin_amdgcn_s_memrealtime();
#endif
            if (!solo) __threadfence();
            publish_copy(a.pub_src, a.pub_dst, a.pub_bytes, threadIdx.x, blockDim.x);
            __threadfence_system();
            __syncthreads();
            if (threadIdx.x == 0) {
                __hip_atomic_store(a.pub_flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
#ifdef BSR_RESCORE_STAMPS
            if (W > 1 && threadIdx.x == 0) g_rescore_stamps[4095 * 8 + 1] = __builtin_amdgcn_s_memrealtime();
#endif
        }
    }
}


// ------------------------------------------------------------------------------------
// The global threshold's rescore (mode B with exclusion bounds; round 5): four
// queries per workgroup, their emitted rows DEALT over the workgroup's 256 lanes -- lane t of a
// round scores row t of the four lists laid end to end -- instead of one query per wave.  A rank
// emits ~32 rows per query on average, so one query per wave left half its lanes idle while a
// query with more than 64 rows on this rank ran a second batch of chunks alone and set the
// kernel's time (median wave 24.6 us, slowest 38.7 us, profiles/r05k_rstamps_gtau.txt); dealt, a
// workgroup takes one round unless its four queries hold more than 256 rows.  Each lane walks its
// row against its own query's LDS copy in index order, exactly as k_rescore; the keys of a round go
// through LDS, and wave w keeps query w's list.  Then wave w finishes query w as k_rescore's
// global-threshold branch does (the list, the exclusion bound, the result rows).
// ------------------------------------------------------------------------------------
#ifndef BSR_GT_FLAT_P
#define BSR_GT_FLAT_P 2
#endif
template <int E, int NC>
__global__ __launch_bounds__(256) void k_rescore_flat(RescoreArgs a) {
    constexpr int QW = 4, STAGE = 64 * 68, QMAX = 1024, T = 64 * QW;
    __shared__ __attribute__((aligned(16))) float stage_all[QW * STAGE];
    __shared__ __attribute__((aligned(16))) float ldq[QW][QMAX];
    __shared__ uint64_t kbuf[T];
    __shared__ uint32_t s_c[QW], s_ov[QW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
    float* const lds = stage_all + w * STAGE;
    if (a.next_status && blockIdx.x == 0 && tid < kWave) {
        // (k_finalize's bookkeeping, fused, as k_rescore)
        if (tid < kStWords) a.next_status[tid] = 0;
        if (a.merge_words && tid < 2) a.merge_words[tid] = tid ? ~0u : 0u;
        uint32_t sum = 0;
        for (uint32_t q = tid; q < a.n_queries; q += kWave) sum += a.emit_cnt[q];
        sum = wave_reduce_u32(sum, [](uint32_t x, uint32_t y) { return x + y; });
        if (tid == 0) a.cur_status[kStEmitted] = sum;
    }
    const uint32_t q0 = blockIdx.x * QW, qw = q0 + w, ld = a.ld, dim = a.dim;
    const bool has_q = qw < a.n_items;
    if (lane == 0) {
        const uint32_t cn = has_q ? a.cnt[qw] : 0u;
        s_ov[w] = cn > a.cap ? 1u : 0u;  // rows were dropped: nothing can be certified
        s_c[w] = cn > a.cap ? 0u : cn;
    }
    if (has_q) {
        constexpr int QN = QMAX / 64;
        const float* qsrc = a.qf32 + (uint64_t)qw * ld;
        float qv[QN];
#pragma unroll
        for (int j = 0; j < QN; ++j) qv[j] = (uint32_t)(j * 64 + lane) < ld ? qsrc[j * 64 + lane] : 0.0f;
#pragma unroll
        for (int j = 0; j < QN; ++j)
            if ((uint32_t)(j * 64 + lane) < ld) ldq[w][j * 64 + lane] = qv[j];
    }
    __syncthreads();
    const uint32_t o1 = s_c[0], o2 = o1 + s_c[1], o3 = o2 + s_c[2], total = o3 + s_c[3];
    const uint32_t my_lo = w == 0 ? 0u : w == 1 ? o1 : w == 2 ? o2 : o3, my_hi = my_lo + s_c[w];
    WaveTopK<E> L;
    L.init();
    uint64_t thr = kKeyNone;
    const uint32_t nch = NC ? (uint32_t)NC : ld / 64;
    for (uint32_t base = 0; base < total; base += T) {
        if (base + (uint32_t)w * 64 < total) {  // (wave-uniform) this wave has rows this round
            const uint32_t f = base + tid;
            const bool live = f < total;
            const uint32_t j = live ? (f >= o1) + (f >= o2) + (f >= o3) : 0u;
            const uint32_t qj = q0 + j;
            const uint32_t lo = j == 0 ? 0u : j == 1 ? o1 : j == 2 ? o2 : o3;
            const uint32_t myrow = live ? key_row(a.cand_keys[(uint64_t)qj * a.cap + (f - lo)]) : 0u;
            const float* const qrow = &ldq[j][0];
            float acc[1] = {-0.0f}, mx[1] = {0.0f};
            uint32_t lrow[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) lrow[i] = (uint32_t)__shfl((int)myrow, (i * 64 + lane) >> 4, kWave);
            auto step = [&](f32x4_t (&pre)[16], uint32_t ch, uint32_t ahead) {
                wave_sync();
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int L16 = i * 64 + lane;
                    *reinterpret_cast<f32x4_t*>(lds + (L16 >> 4) * 68 + (L16 & 15) * 4) = pre[i];
                }
                wave_sync();
                if (ch + ahead < nch) load_cand_chunk(pre, a.rows, ld, lrow, ch + ahead, lane);
                const float* const bb[1] = {qrow + ch * 64};
                const uint32_t nvalid = dim - ch * 64 < 64 ? dim - ch * 64 : 64;
                seq_chunk<1>(lds + lane * 68, bb, nvalid, acc, mx);
            };
            if constexpr (NC > 0) {
                // BSR_GT_FLAT_P chunks of loads in flight (a register ring)
                constexpr uint32_t PP = (uint32_t)BSR_GT_FLAT_P < (uint32_t)NC ? (uint32_t)BSR_GT_FLAT_P : (uint32_t)NC;
                f32x4_t pre[PP][16];
#pragma unroll
                for (uint32_t ch = 0; ch < PP; ++ch) load_cand_chunk(pre[ch], a.rows, ld, lrow, ch, lane);
#pragma unroll
                for (uint32_t ch = 0; ch < (uint32_t)NC; ++ch) step(pre[ch % PP], ch, PP);
            } else {
                f32x4_t preA[16], preB[16];
                load_cand_chunk(preA, a.rows, ld, lrow, 0, lane);
                if (nch > 1) load_cand_chunk(preB, a.rows, ld, lrow, 1, lane);
                for (uint32_t ch = 0; ch < nch; ch += 2) {
                    step(preA, ch, 2);
                    if (ch + 1 < nch) step(preB, ch + 1, 2);
                }
            }
            const float d = finish_distance(acc[0], mx[0], a.na[myrow], a.nb[qj]);
            kbuf[tid] = live ? dist_key(d, myrow) : kKeyNone;
        }
        __syncthreads();
        // wave w: the keys of query w scored this round
        const uint32_t lo = my_lo > base ? my_lo : base, hi = my_hi < base + T ? my_hi : base + T;
        for (uint32_t x = lo; x < hi; x += kWave) {
            const uint32_t idx = x + lane;
            L.offer(idx < hi ? kbuf[idx - base] : kKeyNone, (int)a.k, thr);
        }
        __syncthreads();  // (kbuf and the stages are the next round's)
    }
    if (!has_q) return;
    const uint32_t q = qw, c = s_c[w];
    L.store(a.out_keys + (uint64_t)q * a.k, (int)a.k);
    if (lane == 0) a.excl_out[q] = exclusion_bound(s_ov[w] ? INFINITY : a.tau0[q], a.ebound[q], a.nb[q]);
    if (a.res_idx) put_result_rows(a, q, L, min(a.k, c), lane);  // (no host mirror on this path)
}

// ------------------------------------------------------------------------------------
// The first rescore pass of a tiny batch (<= 16 queries: the single-query p50 path), mode S
// (round 5): ONE workgroup per query with one wave per 64-float chunk of the rows (ld / 64 <= 16
// waves).  Wave 0 selects the k' candidates (select_kp); then every wave loads ITS chunk of every
// candidate row at once, coalesced -- all of a row's loads in flight together, one memory latency
// instead of one per chunk -- and the reference's sequential sum runs through the waves in chunk
// order, each transposing its chunk through an LDS stage and continuing the running dot /
// max|a-b| it reads from LDS (a workgroup barrier per chunk).  (A first version loaded each
// lane's own row, 64 cache lines per instruction: the one CU's address path made it slower than
// the one-wave kernel.)  The
// arithmetic and its order are k_rescore's, so the distances are its bits; wave 0 finishes
// (top-k, certification, result rows) as k_rescore mode S does.  One-wave k_rescore spent ~30 us
// on one query's 63 rows: 12 chunks, each behind its own load latency.
// The self-thresholded path's selection (RescoreArgs::top_w), wave 0 of k_rescore_kp: the query's
// 4 * top_w keys (ascending 4-lists, one per workgroup of the skinny filter) in registers; the
// bound X of the rows outside the lists -- the smallest 4th key: every row a workgroup left out
// scores at most its 4th --; select_kp's radix select of the (kp+1)-th smallest key, the kp keys
// below it compacted into lsel.  tau_x = max(that score, score(X)): every row outside the
// candidates scores at most that.  Then the keys below X go to the front of the query's list,
// their count to top_cnt and score(X) to top_tau: the second chance's input.
__device__ __forceinline__ void top_select(const RescoreArgs& a, uint32_t q, uint32_t* lsel, uint32_t& s_c,
                                           float& s_tx, uint32_t& s_ov, int lane, uint64_t* scratch) {
    constexpr int NR = (int)kTopKeysPerLane;
    const uint32_t U = 4 * a.top_w;
    const bool served = !(a.qflags[q] & kQueryNoApprox);
    uint64_t* const list = const_cast<uint64_t*>(a.cand_keys) + (uint64_t)q * a.cap;
    uint64_t xk[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        const uint32_t i = j * kWave + lane;
        xk[j] = (served && i < U) ? list[i] : kKeyNone;
    }
    // X: the smallest of the lists' 4th keys (slot 3 of each list: lanes with lane % 4 == 3)
    uint64_t mx = kKeyNone;
    uint32_t V = 0;  // valid keys
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        if ((lane & 3) == 3) mx = xk[j] < mx ? xk[j] : mx;
        V += (uint32_t)__popcll(__ballot(xk[j] != kKeyNone));
    }
    {
        uint32_t lo = (uint32_t)mx, hi = (uint32_t)(mx >> 32);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t lo2 = (uint32_t)__shfl_xor((int)lo, off, kWave), hi2 = (uint32_t)__shfl_xor((int)hi, off, kWave);
            const bool lt = hi2 < hi || (hi2 == hi && lo2 < lo);
            lo = lt ? lo2 : lo;
            hi = lt ? hi2 : hi;
        }
        mx = ((uint64_t)hi << 32) | lo;
    }
    const uint64_t X = mx;
#ifdef BSR_RESCORE_STAMPS
    if (lane == 0 && q < 2048) g_rescore_stamps[q * 8 + 6] = __builtin_amdgcn_s_memrealtime();  // (keys in, X)
#endif
    const float tx_trunc = X == kKeyNone ? -INFINITY : score_key_score(X);
    // the second chance's input first (select_kp compacts in place): the keys below X, in order
    uint32_t base = 0;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        const bool pick = xk[j] < X;  // (kKeyNone never: it is no smaller than X)
        const uint64_t m = __ballot(pick);
        if (pick) list[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = xk[j];
        base += (uint32_t)__popcll(m);
    }
    // The k' candidates.  The kp + 1 smallest keys lie among the keys <= H, H the (kp+1)-th smallest
    // list head (at least kp + 1 keys -- those heads -- are <= H), and only the kp + 1 lists whose
    // head is <= H hold such keys: at most 4 (kp + 1) of them.  So the radix selects run over the
    // 512 heads (8 per lane, gathered through LDS) and then those <= 256 keys (4 per lane), not over
    // all 2048 keys (keys are unique: the row is the low word).
    uint32_t c = V;
    float tx = tx_trunc;
    uint32_t sel_row = 0;
    const uint32_t K = a.kp + 1, nl = a.top_w;
    uint32_t nh = 0;
    uint64_t hv[8];
    if (nl <= 8 * kWave) {
#pragma unroll
        for (int j = 0; j < NR; ++j)
            if ((lane & 3) == 0) scratch[j * 16 + (lane >> 2)] = xk[j];
        wave_sync();
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const uint32_t i = t * kWave + lane;
            hv[t] = i < nl ? scratch[i] : kKeyNone;
            nh += (uint32_t)__popcll(__ballot(hv[t] != kKeyNone));
        }
        wave_sync();
    }
    if (nl <= 8 * kWave && nh >= K) {
        const uint64_t H = kth_key<8>(hv, K, ~0u);
#ifdef BSR_RESCORE_STAMPS
        if (lane == 0 && q < 2048) g_rescore_stamps[q * 8 + 7] = __builtin_amdgcn_s_memrealtime();  // (H)
#endif
        uint64_t* const cb = scratch + 8 * kWave;
        uint32_t C = 0;
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const bool pick = xk[j] <= H && xk[j] != kKeyNone;
            const uint64_t m = __ballot(pick);
            if (pick) cb[C + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = xk[j];
            C += (uint32_t)__popcll(m);
        }
        wave_sync();
        uint64_t cv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint32_t i = t * kWave + lane;
            cv[t] = i < C ? cb[i] : kKeyNone;
        }
        wave_sync();
        c = C;  // (K <= C <= 4 K)
        select_kp_n<4>(cv, c, false, a.kp, tx_trunc, tx, lsel, sel_row, lane);
    } else {  // (fewer than kp + 1 lists hold a key: every slot searched)
        select_kp_n<NR>(xk, c, false, a.kp, tx_trunc, tx, lsel, sel_row, lane, true);
    }
    if (lane == 0) {
        s_c = c;
        s_tx = served ? fmaxf(tx, tx_trunc) : INFINITY;
        s_ov = served ? 0u : 1u;
        a.top_cnt[q] = base;
        a.top_tau[q] = served ? tx_trunc : INFINITY;
    }
}

// ------------------------------------------------------------------------------------
constexpr int kKpStage = 64 * 68;  // 64 rows x one chunk (stride 68)
template <int E>
__global__ __launch_bounds__(1024) void k_rescore_kp(RescoreArgs a) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __shared__ __attribute__((aligned(16))) float ldq[1024];
    __shared__ __attribute__((aligned(16))) float stage[2 * kKpStage];
    __shared__ float s_acc[64], s_mxw[16][64];
    __shared__ uint32_t lsel[64];
    __shared__ uint32_t s_c, s_ov;
    __shared__ float s_tx;
    const uint32_t item = blockIdx.x;
    if (item >= a.n_items) return;  // (grid = n_items: uniform per workgroup)
    if (w == 0) BSR_STAMP(1, 0);
    const uint32_t q = a.qlist ? a.qlist[item] : item;
    const uint32_t ld = a.ld, dim = a.dim;
    // the query's chunk of this wave, staged in LDS (read as broadcasts)
    if ((uint32_t)(w * 64 + lane) < ld) ldq[w * 64 + lane] = a.qf32[(uint64_t)q * ld + w * 64 + lane];
    if (a.top_w) {
        // (LDS scratch for the heads and candidates: the product stage, first written after this)
        if (w == 0) {
            BSR_STAMP(1, 5);  // (lab: no separate key arrival on this path)
            top_select(a, q, lsel, s_c, s_tx, s_ov, lane, reinterpret_cast<uint64_t*>(stage));
            BSR_STAMP(1, 1);
        }
    } else if (w == 0) {
        constexpr int NR = 16;
        uint64_t xk[NR];
        const uint64_t* src = a.cand_keys + (uint64_t)q * a.cap;
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const uint32_t i = j * kWave + lane;
            xk[j] = i < a.cap ? src[i] : kKeyNone;
        }
        const uint32_t cnt = a.cnt[q];
#ifdef BSR_RESCORE_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (lab: the keys' arrival, stamp 5)
        BSR_STAMP(1, 5);
#endif
        const bool overflow = cnt > a.cap;
        uint32_t c = overflow ? 0u : cnt;
        float tx = INFINITY;
        uint32_t sel_row = 0;
        select_kp(xk, c, overflow, a.kp, a.tau0[q], tx, lsel, sel_row, lane);
        if (lane == 0) {
            s_c = c;
            s_tx = tx;
            s_ov = overflow ? 1u : 0u;
        }
        BSR_STAMP(1, 1);
    }
    __syncthreads();
    const uint32_t c = s_c;
    const uint32_t myrow = lane < (int)c ? lsel[lane] : (c ? lsel[0] : 0u);
    // this wave's chunk of the 64 rows, coalesced (a quarter wave per row, 16 loads in flight)
    uint32_t lrow[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) lrow[i] = (uint32_t)__shfl((int)myrow, (i * 64 + lane) >> 4, kWave);
    f32x4_t pre[16];
    load_cand_chunk(pre, a.rows, ld, lrow, (uint32_t)w, lane);
    // The products x_i * b_i (rounded, as the reference's separate multiply rounds them) and
    // max |x_i - b_i| (order-free, no NaN reaches here) need no order: every wave forms them for
    // its chunk in place, at once.  Only the running sum is sequential.
    const uint32_t nvalid = dim > (uint32_t)w * 64 ? min(64u, dim - (uint32_t)w * 64) : 0u;
    {
        const uint32_t c0 = (lane & 15) * 4;
        const f32x4_t bq = *reinterpret_cast<const f32x4_t*>(ldq + w * 64 + c0);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            f32x4_t x = pre[i];
            float m = 0.0f;
            if (c0 + 0 < nvalid) m = fmaxf(m, fabsf(x.x - bq.x));
            if (c0 + 1 < nvalid) m = fmaxf(m, fabsf(x.y - bq.y));
            if (c0 + 2 < nvalid) m = fmaxf(m, fabsf(x.z - bq.z));
            if (c0 + 3 < nvalid) m = fmaxf(m, fabsf(x.w - bq.w));
            x.x = x.x * bq.x;
            x.y = x.y * bq.y;
            x.z = x.z * bq.z;
            x.w = x.w * bq.w;
            pre[i] = x;
            // the row's maximum over this chunk: its 16 lanes
            m = fmaxf(m, __shfl_xor(m, 1, kWave));
            m = fmaxf(m, __shfl_xor(m, 2, kWave));
            m = fmaxf(m, __shfl_xor(m, 4, kWave));
            m = fmaxf(m, __shfl_xor(m, 8, kWave));
            if ((lane & 15) == 0) s_mxw[w][4 * i + (lane >> 4)] = m;
        }
    }
    // Two LDS stages of products: while wave s sums its rows' from stage s & 1, wave s + 1
    // transposes its chunk into the other (last read by wave s - 1, before the previous barrier)
    auto put = [&](float* st) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int L16 = i * 64 + lane;
            *reinterpret_cast<f32x4_t*>(st + (L16 >> 4) * 68 + (L16 & 15) * 4) = pre[i];
        }
    };
    if (w == 0) put(stage);
    __syncthreads();
    if (w == 0) BSR_STAMP(1, 2);
    float acc = -0.0f;
    for (int step = 0; step < nw; ++step) {
        if (w == step) {
            if (step) acc = s_acc[lane];
            const float* my = stage + (step & 1) * kKpStage + lane * 68;
            if (nvalid == 64) {
#pragma unroll
                for (int i = 0; i < 64; i += 4) {
                    const f32x4_t x = *reinterpret_cast<const f32x4_t*>(my + i);
                    acc = acc + x.x;
                    acc = acc + x.y;
                    acc = acc + x.z;
                    acc = acc + x.w;
                }
            } else {
                for (uint32_t i = 0; i < nvalid; ++i) acc = acc + my[i];
            }
            s_acc[lane] = acc;
        } else if (w == step + 1) {
            put(stage + (w & 1) * kKpStage);
        }
        __syncthreads();
    }
    if (w != 0) return;
    BSR_STAMP(1, 3);
    const float mag_b = a.nb[q];
    WaveTopK<E> L;
    L.init();
    uint64_t thr = kKeyNone;
    {
        float mx = 0.0f;
        for (int v = 0; v < nw; ++v) mx = fmaxf(mx, s_mxw[v][lane]);
        const float d = finish_distance(s_acc[lane], mx, a.na[myrow], mag_b);  // (the last wave's sum)
        L.offer(lane < (int)c ? dist_key(d, myrow) : kKeyNone, (int)a.k, thr);
    }
    L.store(a.out_keys + (uint64_t)q * a.k, (int)a.k);
    bool certified = false;
    if (lane == 0) {
        // certification, as k_rescore mode S
        const bool ok = certify(s_ov ? INFINITY : s_tx, thr, a.ebound[q], mag_b);
        if (!ok) a.fail_list[atomicAdd(a.fail_cnt, 1u)] = q;
        certified = ok;
    }
    bool host_rows = false;
    if (a.res_idx && __shfl((int)certified, 0, kWave))
        host_rows = put_result_rows(a, q, L, (uint64_t)a.k < a.n_rows ? a.k : (uint32_t)a.n_rows, lane);
    // (the first pass: the host reads these rows once the batch's last kernel raises its flag)
    if (BSR_PUB_SYSREL && __ballot(host_rows)) release_system();
    BSR_STAMP(1, 4);
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

// Per scanned query: merge the per-block lists of k_scan_exact into out_keys[qid].  Four
// waves each take a quarter of the grid's lists (loads issued 4 deep), then wave 0 merges
// the four wave lists through LDS.
template <int E>
__global__ __launch_bounds__(256) void k_merge_parts(const uint64_t* __restrict__ part, uint32_t grid,
                                                     const int32_t* __restrict__ qids, uint32_t qf,
                                                     uint32_t nqf, uint32_t k,
                                                     uint64_t* __restrict__ out_keys) {
    __shared__ uint64_t lk[4][64 * E];
    const uint32_t j = blockIdx.x;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (j >= nqf) return;
    WaveTopK<E> L;
    L.init();
    uint64_t thr = kKeyNone;
    const uint64_t total = (uint64_t)grid * k;
    const uint64_t per = (total + 3) / 4, lo = w * per, hi = lo + per < total ? lo + per : total;
    auto key_at = [&](uint64_t i) -> uint64_t {
        if (i >= hi) return kKeyNone;
        const uint64_t g = i / k, e = i - g * k;
        return part[(g * qf + j) * k + e];
    };
    for (uint64_t base = lo; base < hi; base += 4 * kWave) {
        uint64_t x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = key_at(base + u * kWave + lane);
#pragma unroll
        for (int u = 0; u < 4; ++u) L.offer(x[u], (int)k, thr);
    }
    L.store(&lk[w][0], (int)k);
    __syncthreads();
    if (w == 0) {
        WaveTopK<E> M;
        M.init();
        uint64_t mt = kKeyNone;
        for (int src = 0; src < 4; ++src)
            for (uint32_t b = 0; b < k; b += kWave) {
                const uint32_t i = b + lane;
                M.offer(i < k ? lk[src][i] : kKeyNone, (int)k, mt);
            }
        M.store(out_keys + (uint64_t)qids[j] * k, (int)k);
    }
}

__global__ void k_finalize(const uint64_t* __restrict__ keys, uint32_t nq, uint32_t k, uint64_t n,
                           uint64_t offset, uint64_t* __restrict__ out_idx, float* __restrict__ out_dist,
                           uint32_t* __restrict__ out_count, uint32_t* __restrict__ status,
                           const uint32_t* __restrict__ emit_cnt, uint32_t* __restrict__ cur_status) {
    const uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (e < kStWords) status[e] = 0;  // the status words of the NEXT search's result buffer
    if (emit_cnt && blockIdx.x == 0 && threadIdx.x < kWave) {
        // rows emitted by the filter over the batch (a statistic; one wave, no atomics)
        uint32_t sum = 0;
        for (uint32_t q = threadIdx.x; q < nq; q += kWave) sum += emit_cnt[q];
        sum = wave_reduce_u32(sum, [](uint32_t a, uint32_t b) { return a + b; });
        if (threadIdx.x == 0) cur_status[kStEmitted] = sum;
    }
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

// The root's merge (compute_global_top_k, src/mpi_helpers/metrics.rs:141-171) of gathered
// lists laid out [P][nq][k_in] (counts [P][nq]) on the device, one wave per query: the
// rank-order concatenation is staged in LDS with its order key (distance, position in the
// concatenation) -- the stable sort by distance is the ascending order of that key; -0.0
// and +0.0 compare equal as partial_cmp has them -- every entry whose index occurs at a
// smaller key is dropped (the HashSet keeps first occurrences), and the k smallest keys left
// are the result.  Rows past out_count[q] are (~0, +inf), as merge_top_k_lists writes them.
// A NaN distance: out_count[q] = 0 and the lowest such q in *first_nan (the reference panics).
// (MergeArgs: list l of query q at idx + l * idx_stride + q * k_in, dist likewise, its count
// at cnt[l * cnt_stride + q]; with excl, the certification of a parallel search with a global
// threshold, and the lists' status words copied out -- kernels.hpp.)
template <int E>
__global__ __launch_bounds__(64) void k_merge_lists(MergeArgs a) {
    const uint64_t* __restrict__ idx = a.idx;
    const float* __restrict__ dist = a.dist;
    const uint32_t P = a.P, nq = a.nq, k_in = a.k_in, k = a.k;
    uint64_t* __restrict__ out_idx = a.out_idx;
    float* __restrict__ out_dist = a.out_dist;
    uint32_t* __restrict__ out_count = a.out_count;
    __shared__ uint64_t s_idx[kMergeMaxEntries];
    __shared__ uint64_t s_key[kMergeMaxEntries];
    __shared__ float s_dist[kMergeMaxEntries];
    __shared__ uint64_t h_idx[kMergeMaxEntries], h_min[kMergeMaxEntries];
    const uint32_t q = blockIdx.x;
    const int lane = threadIdx.x;
    // (the lambdas below read the kernel argument's fields through these locals: capturing the
    // by-value argument itself makes it addressable, i.e. a copy in scratch -- 144 B per lane)
    const auto m_cnt = a.cnt;
    const auto m_force_hash = a.force_hash;
    const auto m_lists_unique = a.lists_unique;
    const auto m_cnt_stride = a.cnt_stride;
    const auto m_dist_stride = a.dist_stride;
    const auto m_excl = a.excl;
    const auto m_excl_stride = a.excl_stride;
    const auto m_fail_cnt = a.fail_cnt;
    const auto m_fail_list = a.fail_list;
    const auto m_first_nan = a.first_nan;
    const auto m_hout_count = a.hout_count;
    const auto m_hout_dist = a.hout_dist;
    const auto m_hout_idx = a.hout_idx;
    const auto m_idx_stride = a.idx_stride;
    const auto m_need = a.need;
    const auto m_st = a.st;
    const auto m_st_all = a.st_all;
    const auto m_st_stride = a.st_stride;
    float x_l = INFINITY;  // (certification) list `lane`'s exclusion bound for q
    auto merge_query = [&]() -> bool {
        if (m_st_all && q == 0)  // every list's status words, compact
            for (uint32_t i = lane; i < P * kStWords; i += kWave)
                m_st_all[i] = m_st[(uint64_t)(i / kStWords) * m_st_stride + i % kStWords];
        if (q >= nq) return false;
        // ONE batch of loads for the whole query (round 5: they were three dependent rounds --
        // counts, then each list's entries, then the certification bounds): every slot of every
        // list (l, i < k_in), list l's count and exclusion bound on lane l; the slots past a
        // list's count are loaded and dropped.
        constexpr int U = kMergeMaxEntries / kWave;
        const uint32_t slots = P * k_in;  // (<= kMergeMaxEntries)
        float dv[U];
        uint64_t iv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t f = u * kWave + lane;
            dv[u] = 0.0f;
            iv[u] = 0;
            if (u * kWave < (int)slots && f < slots) {
                const uint32_t l = f / k_in, i = f - l * k_in;
                dv[u] = dist[(uint64_t)l * m_dist_stride + (uint64_t)q * k_in + i];
                iv[u] = idx[(uint64_t)l * m_idx_stride + (uint64_t)q * k_in + i];
            }
        }
        const uint32_t c_l = lane < (int)P ? min(m_cnt[(uint64_t)lane * m_cnt_stride + q], k_in) : 0u;
        x_l = (m_excl && lane < (int)P) ? m_excl[(uint64_t)lane * m_excl_stride + q] : INFINITY;
        // list l's offset in the concatenation (exclusive prefix sum of the counts)
        uint32_t incl = c_l;
    #pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)incl, off, kWave);
            if (lane >= off) incl += t;
        }
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t off_l = incl - c_l;
        bool nan = false;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t f = u * kWave + lane;
            const uint32_t l = f / (k_in ? k_in : 1u), i = f - l * k_in;
            // (every lane takes part in the shuffles; l < P for the slots that exist)
            const uint32_t cl = (uint32_t)__shfl((int)c_l, (int)(l < 64 ? l : 0), kWave);
            const uint32_t ol = (uint32_t)__shfl((int)off_l, (int)(l < 64 ? l : 0), kWave);
            if (u * kWave < (int)slots && f < slots && i < cl) {
                const uint32_t j = ol + i;
                const float d = dv[u];
                nan |= d != d;
                s_idx[j] = iv[u];
                s_dist[j] = d;
                s_key[j] = ((uint64_t)ord_f32(d + 0.0f) << 32) | j;  // (-0.0 + 0.0 = +0.0)
            }
        }
        __syncthreads();
        // (the merged rows also go to the host mirror when the kernel publishes through one)
        auto put = [&](uint32_t p, uint64_t vi, float vd) {
            out_idx[(uint64_t)q * k + p] = vi;
            out_dist[(uint64_t)q * k + p] = vd;
            if (m_hout_idx) {
                host_put(m_hout_idx + (uint64_t)q * k + p, vi);
                host_put(m_hout_dist + (uint64_t)q * k + p, vd);
            }
        };
        auto put_count = [&](uint32_t c) {
            out_count[q] = c;
            if (m_hout_count) host_put(m_hout_count + q, c);
        };
        if (__ballot(nan)) {
            if (lane == 0) {
                put_count(0);
                atomicMin(m_first_nan, q);
            }
            for (uint32_t p = lane; p < k; p += kWave) put(p, ~0ull, INFINITY);
            return true;
        }
        // Lists without repeats (lists_unique: each one rank's own top-k) whose index ranges are
        // pairwise disjoint -- the rank shards of a parallel search -- hold no index twice: no
        // first-occurrence filter (round 6; the hash below is a chain of LDS atomics and two
        // barriers).  Lane l < P: list l's [min, max] index.
        uint64_t lo = ~0ull, hi = 0;
        if (lane < (int)P)
            for (uint32_t i = 0; i < c_l; ++i) {
                const uint64_t x = s_idx[off_l + i];
                lo = x < lo ? x : lo;
                hi = x > hi ? x : hi;
            }
        bool ovl = false;
        for (uint32_t m = 0; m < P; ++m) {
            const uint64_t lo_m = shfl64(lo, (int)m), hi_m = shfl64(hi, (int)m);
            const uint32_t c_m = (uint32_t)__shfl((int)c_l, (int)m, kWave);
            ovl |= lane < (int)P && (uint32_t)lane != m && c_l && c_m && !(hi < lo_m || hi_m < lo);
        }
        const bool disjoint = m_lists_unique && !m_force_hash && __ballot(ovl) == 0;
        // First occurrences: an LDS hash of index -> smallest key (open addressing, 64-bit CAS
        // and min); an entry is kept iff its key is its index's minimum.  (An index of ~0, the
        // hash's empty mark, takes the pairwise check instead.)
        bool has_empty_mark = false;
        if (!disjoint)
            for (uint32_t j = lane; j < total; j += kWave) has_empty_mark |= s_idx[j] == ~0ull;
        const bool pairwise = __ballot(has_empty_mark) != 0;
        uint32_t hmask = 127;
        while (hmask + 1 < 2 * total && hmask + 1 < kMergeMaxEntries) hmask = 2 * hmask + 1;  // load <= 1
        auto slot0 = [&](uint64_t x) -> uint32_t {
            uint64_t h = x * 0x9E3779B97F4A7C15ull;
            return (uint32_t)(h >> 40) & hmask;
        };
        if (!disjoint && !pairwise) {
            for (uint32_t i = lane; i <= hmask; i += kWave) {
                h_idx[i] = ~0ull;
                h_min[i] = ~0ull;
            }
            __syncthreads();
            for (uint32_t j = lane; j < total; j += kWave) {
                const uint64_t x = s_idx[j];
                for (uint32_t sl = slot0(x);; sl = (sl + 1) & hmask) {
                    const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&h_idx[sl]), ~0ull,
                                                    (unsigned long long)x);
                    if (prev == ~0ull || prev == x) {
                        atomicMin(reinterpret_cast<unsigned long long*>(&h_min[sl]), (unsigned long long)s_key[j]);
                        break;
                    }
                }
            }
            __syncthreads();
        }
        WaveTopK<E> L;
        L.init();
        uint64_t thr = kKeyNone;
        for (uint32_t b = 0; b < total; b += kWave) {
            const uint32_t j = b + lane;
            uint64_t key = kKeyNone;
            if (j < total) {
                key = s_key[j];
                const uint64_t x = s_idx[j];
                if (disjoint) {
                    // (every entry is its index's only one)
                } else if (!pairwise) {
                    uint32_t sl = slot0(x);
                    while (h_idx[sl] != x) sl = (sl + 1) & hmask;
                    if (h_min[sl] != key) key = kKeyNone;
                } else {
                    for (uint32_t i = 0; i < total; ++i)  // an earlier-sorting copy of the same index
                        if (s_idx[i] == x && s_key[i] < key) { key = kKeyNone; break; }
                }
            }
            L.offer(key, (int)k, thr);
        }
        uint32_t got = 0;
    #pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t p = e * kWave + lane;
            const uint64_t key = L.v[e];
            got += (uint32_t)__popcll(__ballot(p < k && key != kKeyNone));
            if (p < k) {
                const uint32_t j = (uint32_t)key;
                put(p, key != kKeyNone ? s_idx[j] : ~0ull, key != kKeyNone ? s_dist[j] : INFINITY);
            }
        }
        if (lane == 0) put_count(got);
        const uint64_t kth = (m_excl && got == k) ? L.at((int)k - 1) : kKeyNone;  // (wave-uniform)
        // the smallest bound over the lists (NaN: nothing certifiable), loaded with the lists
        float xmin = x_l == x_l ? x_l : -INFINITY;
    #pragma unroll
        for (int off = 32; off >= 1; off >>= 1) xmin = fminf(xmin, __shfl_xor(xmin, off, kWave));
        bool shared = false;
        if (m_excl && lane == 0) {
            // Certification of a global-threshold parallel search: every row left
            // out on rank l lies at a distance >= excl_l[q] (its kernel's bound, rounded down), so
            // the merged list is the reference's iff it holds need = min(k, corpus rows) entries and
            // its k-th distance lies strictly below every rank's bound (a shorter list only when
            // every row of the corpus was a candidate: every bound +inf).
            bool ok = got >= m_need;
            if (ok && got == k) {
                ok = (double)s_dist[(uint32_t)kth] < (double)xmin;
            } else if (ok) {
                ok = xmin == INFINITY;
            }
            if (!ok) m_fail_list[atomicAdd(m_fail_cnt, 1u)] = q;
            shared = !ok;
        }
        return __shfl((int)shared, 0, kWave) != 0 || (m_st_all && q == 0);
    };
    // (publish) whether this wave wrote state the publishing workgroup reads: the status words
    // (q = 0), a failure entry, the lowest NaN query
    const bool wrote = merge_query();
    if (a.pub_flag) {
        // publish (as k_rescore's): the last workgroup copies the merged result (with a host
        // mirror of the rows: the part before them) to host memory and raises the host's flag
        // Only a wave that wrote what the last one copies releases it (an agent fence writes back
        // its XCD's L2); the rows count when no host mirror takes them and the copy covers them.
        // A wave whose merged rows went into the host mirror releases them at system scope
        // (BSR_PUB_SYSREL) before its ticket.
        __shared__ uint32_t s_last;
        const bool rows_copied = !a.hout_idx && a.pub_src + a.pub_bytes > reinterpret_cast<const uint8_t*>(out_count);
        if (wrote || rows_copied) __threadfence();
        if (BSR_PUB_SYSREL && a.hout_idx && q < nq) release_system();  // (its merged rows, in the host mirror)
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (lane == 0) s_last = last_arrival(a.pub_ticket) ? 1u : 0u;
        __syncthreads();
        if (s_last) {
            __threadfence();
            publish_copy(a.pub_src, a.pub_dst, a.pub_bytes, lane, kWave);
            __threadfence_system();
            __syncthreads();
            if (lane == 0) {
                __hip_atomic_store(a.pub_flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
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
#ifdef BSR_RESCORE_STAMPS
extern "C" int bsr_lab_rescore_stamps(uint64_t* out, int n) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rescore_stamps), (size_t)n * 8 * sizeof(uint64_t));
}
#endif
// Chunks of candidate rows in flight in the global-threshold search's rescore of every emitted
// row (one wave per query, ~32 rows per query per rank at N = 8: latency-bound, not HBM-bound).
#ifndef BSR_GT_RESCORE_W  // (lab) 2: the global threshold's rescore with two waves per query
#define BSR_GT_RESCORE_W 1
#endif
#ifndef BSR_GT_RESCORE_P
#define BSR_GT_RESCORE_P 2
#endif
bool rescore_kp_enabled() {
    const char* v = getenv("BSR_RESCORE_KP");
    return !(v && v[0] == '0');
}

hipError_t launch_rescore(const RescoreArgs& a_in, hipStream_t s) {
    if (!a_in.n_items) return hipSuccess;
    RescoreArgs a = a_in;
    a.solo = 0;
    const uint32_t e = (a.k + 63) / 64;
    // the first pass (mode S) of a tiny batch: one workgroup per query, one wave per chunk
    // (BSR_RESCORE_KP=0: the one-wave kernel instead, for A/B runs)
    static const bool kp_on = rescore_kp_enabled();
    if (a.top_w && !(kp_on && a.n_items <= 16 && a.ld % 64 == 0 && a.ld <= 1024 && a.k <= 64 && a.kp <= 63 &&
                     4 * a.top_w <= 64u * kTopKeysPerLane))
        return hipErrorInvalidValue;  // (the self-thresholded path needs k_rescore_kp: the caller checks)
    // (lab, BSR_RESCORE_KP=2: the tiny-batch kernel for every batch size, for A/B runs)
    static const bool kp_any = [] {
        const char* v = getenv("BSR_RESCORE_KP");
        return v && v[0] == '2';
    }();
    if (kp_on && a.sel && !a.n_items_dev && !a.pub_flag && !a.excl_out && (a.n_items <= 16 || kp_any) &&
        a.ld % 64 == 0 &&
        a.ld <= 1024 && a.k <= 64 && a.kp <= 64 && (a.cap <= 1024 || a.top_w)) {
        hipLaunchKernelGGL(k_rescore_kp<1>, dim3(a.n_items), dim3(a.ld), 0, s, a);
        return hipGetLastError();
    }
    // the global threshold's rescore: four queries' rows dealt over a workgroup (BSR_GT_FLAT=0:
    // one wave per query instead, for A/B runs)
    static const bool flat_on = [] {
        const char* v = getenv("BSR_GT_FLAT");
        return !(v && v[0] == '0');
    }();
    if (flat_on && a.excl_out && a.cand_keys && !a.sel && !a.n_items_dev && !a.pub_flag && !a.hres_idx &&
        !a.qlist && a.ld % 64 == 0 && a.ld <= 1024 && BSR_GT_RESCORE_W == 1) {
        const dim3 gf((a.n_items + 3) / 4), bf(256);
#define BSR_FLAT(E)                                                                           \
    do {                                                                                      \
        if (a.ld == 768) hipLaunchKernelGGL((k_rescore_flat<E, 12>), gf, bf, 0, s, a);        \
        else hipLaunchKernelGGL((k_rescore_flat<E, 0>), gf, bf, 0, s, a);                     \
    } while (0)
        switch (e) {
            case 1: BSR_FLAT(1); break;
            case 2: BSR_FLAT(2); break;
            case 3: BSR_FLAT(3); break;
            case 4: BSR_FLAT(4); break;
            default: return hipErrorInvalidValue;
        }
#undef BSR_FLAT
        return hipGetLastError();
    }
    // items counted on the device: a persistent grid of 8-wave workgroups; else one wave per item
    const bool dev = a.n_items_dev != nullptr;
    // (one item per wave: four independent waves per workgroup, one workgroup per CU)
    // (a tiny batch's second chance: one workgroup, its own last arrival -- rarely any item)
    // (BSR_SOLO_PUB=0: the grid as before, for A/B runs)
    static const bool solo_on = [] {
        const char* v = getenv("BSR_SOLO_PUB");
        return !(v && v[0] == '0');
    }();
    const uint32_t gdev = solo_on && a.n_items <= 16 ? 1u : std::min<uint32_t>(a.n_items, kRescoreAllGrid);
    const dim3 g(dev ? gdev : (a.n_items + 3) / 4), b(dev ? 512 : 256);
    a.solo = dev && solo_on && a.n_items <= 16 ? 1u : 0u;
#define BSR_RESCORE(E)                                                                        \
    do {                                                                                      \
        if (dev) hipLaunchKernelGGL((k_rescore<E, 8, 2>), g, b, 0, s, a);                     \
        else if (a.excl_out && BSR_GT_RESCORE_W == 2)                                        \
            hipLaunchKernelGGL((k_rescore<E, 2, BSR_GT_RESCORE_P, 1>), dim3(a.n_items), dim3(128), 0, s, a); \
        else if (a.excl_out) hipLaunchKernelGGL((k_rescore<E, 1, BSR_GT_RESCORE_P, 4>), g, b, 0, s, a); \
        else hipLaunchKernelGGL((k_rescore<E, 1, 2, 4>), g, b, 0, s, a);                      \
    } while (0)
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
    hipLaunchKernelGGL(k_merge_parts<E>, dim3(nqf), dim3(256), 0, s, part, grid, qids, qf, nqf, k, \
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
                           uint64_t* out_idx, float* out_dist, uint32_t* out_count, uint32_t* status,
                           const uint32_t* emit_cnt, uint32_t* cur_status, hipStream_t s) {
    const uint64_t total = (uint64_t)nq * k;
    hipLaunchKernelGGL(k_finalize, dim3(grid_for(total, 256)), dim3(256), 0, s, keys, nq, k, n, offset,
                       out_idx, out_dist, out_count, status, emit_cnt, cur_status);
    return hipGetLastError();
}

hipError_t launch_merge_lists(const uint64_t* idx, const float* dist, const uint32_t* cnt, uint32_t P, uint32_t nq,
                              uint32_t k_in, uint32_t k, uint64_t* out_idx, float* out_dist, uint32_t* out_count,
                              uint32_t* first_nan, hipStream_t s) {
    MergeArgs a{};
    a.idx = idx;
    a.dist = dist;
    a.cnt = cnt;
    a.idx_stride = a.dist_stride = (uint64_t)nq * k_in;
    a.cnt_stride = nq;
    a.P = P;
    a.nq = nq;
    a.k_in = k_in;
    a.k = k;
    a.out_idx = out_idx;
    a.out_dist = out_dist;
    a.out_count = out_count;
    a.first_nan = first_nan;
    return launch_merge(a, s);
}
hipError_t launch_merge(const MergeArgs& a_in, hipStream_t s) {
    MergeArgs a = a_in;
    {  // (lab A/B: BSR_MERGE_HASH=1 keeps the first-occurrence filter for disjoint lists too)
        const char* v = getenv("BSR_MERGE_HASH");
        a.force_hash = v && v[0] == '1' ? 1u : 0u;
    }
    const uint32_t P = a.P, nq = a.nq, k_in = a.k_in, k = a.k;
    if (P > (uint32_t)kWave || (uint64_t)P * k_in > kMergeMaxEntries || k > 4 * kWave) return hipErrorInvalidValue;
    const uint32_t e = (k + 63) / 64;
#define BSR_MLISTS(E)                                                                                \
    hipLaunchKernelGGL(k_merge_lists<E>, dim3(nq), dim3(64), 0, s, a)
    switch (e) {
        case 1: BSR_MLISTS(1); break;
        case 2: BSR_MLISTS(2); break;
        case 3: BSR_MLISTS(3); break;
        default: BSR_MLISTS(4); break;
    }
#undef BSR_MLISTS
    return hipGetLastError();
}

hipError_t launch_cosine_pair(const float* a, uint32_t la, const float* b, uint32_t lb, float* out,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_cosine_pair, dim3(1), dim3(64), 0, s, a, la, b, lb, out);
    return hipGetLastError();
}

}  // namespace bsr
