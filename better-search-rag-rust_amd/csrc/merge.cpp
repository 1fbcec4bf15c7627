// merge.cpp -- compute_global_top_k (src/mpi_helpers/metrics.rs:141-171) on the host: the
// root's merge of the rank-ordered partial lists, for a batch of queries.
//
// The reference concatenates the lists in rank order (:86-126), stable-sorts the pairs by
// distance (:153; partial_cmp, a NaN panics) and keeps the first top_k distinct indices
// (HashSet, :156-168).  When every list of a query is already ordered by distance -- what
// bsr_local_top_k returns -- the stable sort of the concatenation is exactly a P-way merge
// that breaks distance ties by list number and then by position in the list (both are the
// concatenation order), so that case is merged without sorting; any other input takes the
// literal stable sort.  Either way the dedupe keeps an index's first
// occurrence, so overlapping shards (caller-chosen global offsets) behave as the reference.
// Large batches are split over host threads by query.
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "internal.hpp"
#include "merge.hpp"

namespace bsr {

namespace {

struct Entry {
    uint64_t idx;
    float dist;
};

// Open-addressing set of indices already emitted for one query (the reference's HashSet).
struct SeenSet {
    std::vector<uint64_t> slot;
    std::vector<uint8_t> used;
    uint64_t mask = 0;
    void reset(size_t expect) {
        size_t cap = 16;
        while (cap < 2 * expect) cap <<= 1;
        if (slot.size() < cap) {
            slot.resize(cap);
            used.resize(cap);
        }
        mask = cap - 1;
        memset(used.data(), 0, cap);
    }
    // true if x was newly inserted
    bool insert(uint64_t x) {
        uint64_t h = x * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        for (uint64_t i = h & mask;; i = (i + 1) & mask) {
            if (!used[i]) {
                used[i] = 1;
                slot[i] = x;
                return true;
            }
            if (slot[i] == x) return false;
        }
    }
};

struct Scratch {
    std::vector<Entry> concat;
    SeenSet seen;
    std::vector<uint32_t> pos, cnt;
    std::vector<float> head;
};

// One query.  Returns the output count, or UINT32_MAX on a NaN distance.
uint32_t merge_one(const ListsView& in, uint32_t q, uint32_t k, uint64_t* out_idx, float* out_dist,
                   Scratch& s) {
    const uint32_t L = in.n_lists;
    size_t total = 0;
    bool sorted = true;
    s.cnt.resize(L);
    s.head.resize(L);
    for (uint32_t l = 0; l < L; ++l) {
        const uint32_t c = in.count_of(l, q);
        const float* d = in.dist_of(l, q);
        for (uint32_t i = 0; i < c; ++i) {
            if (d[i] != d[i]) return UINT32_MAX;  // partial_cmp().unwrap() panics
            if (i && d[i] < d[i - 1]) sorted = false;
        }
        s.cnt[l] = c;
        s.head[l] = c ? d[0] : __builtin_inff();
        total += c;
    }
    // seen indices: a linear scan of the output for short lists, the hash set beyond
    const bool small = k <= 32;
    if (!small) s.seen.reset(std::min<size_t>(total, k));
    uint32_t out = 0;
    auto take = [&](uint64_t idx, float dist) {
        if (small) {
            for (uint32_t i = 0; i < out; ++i)
                if (out_idx[i] == idx) return;
        } else if (!s.seen.insert(idx)) {
            return;
        }
        out_idx[out] = idx;
        out_dist[out] = dist;
        ++out;
    };
    if (sorted) {
        // P-way merge; ties -> lower list number, then list position (= concatenation order).
        // Exhausted lists hold +inf heads and are skipped by their count.
        s.pos.assign(L, 0);
        for (size_t taken = 0; out < k && taken < total; ++taken) {
            uint32_t best = UINT32_MAX;
            float bd = 0.0f;
            for (uint32_t l = 0; l < L; ++l)
                if (s.pos[l] < s.cnt[l] && (best == UINT32_MAX || s.head[l] < bd)) {
                    best = l;
                    bd = s.head[l];
                }
            const uint32_t p = s.pos[best]++;
            take(in.idx_of(best, q)[p], bd);
            if (p + 1 < s.cnt[best]) s.head[best] = in.dist_of(best, q)[p + 1];
        }
        return out;
    }
    s.concat.clear();
    for (uint32_t l = 0; l < L; ++l) {
        const uint32_t c = s.cnt[l];
        const uint64_t* ix = in.idx_of(l, q);
        const float* d = in.dist_of(l, q);
        for (uint32_t i = 0; i < c; ++i) s.concat.push_back({ix[i], d[i]});
    }
    std::stable_sort(s.concat.begin(), s.concat.end(), [](const Entry& a, const Entry& b) { return a.dist < b.dist; });
    for (const Entry& e : s.concat) {
        if (out >= k) break;
        take(e.idx, e.dist);
    }
    return out;
}

}  // namespace

int merge_top_k_lists(const ListsView& in, uint32_t n_queries, uint32_t k, uint64_t* out_idx, float* out_dist,
                      uint32_t* out_count) {
    if (!n_queries) return BSR_OK;
    if (k == 0) return set_error(BSR_E_INVALID, "k must be >= 1");
    // threads: one per 1M list entries of work (starting a thread costs tens of us), at most 8
    const size_t work = (size_t)n_queries * in.n_lists * std::max<uint32_t>(in.k_in, 1);
    unsigned hw = std::thread::hardware_concurrency();
    unsigned nt = (unsigned)std::min<size_t>({(size_t)8, (size_t)(hw ? hw : 1), work / 1048576 + 1, (size_t)n_queries});
    std::vector<uint32_t> bad(nt, UINT32_MAX);
    auto run = [&](unsigned t) {
        Scratch s;
        const uint32_t q0 = (uint32_t)((uint64_t)n_queries * t / nt), q1 = (uint32_t)((uint64_t)n_queries * (t + 1) / nt);
        for (uint32_t q = q0; q < q1; ++q) {
            uint64_t* oi = out_idx + (size_t)q * k;
            float* od = out_dist + (size_t)q * k;
            const uint32_t got = merge_one(in, q, k, oi, od, s);
            if (got == UINT32_MAX) {
                if (bad[t] == UINT32_MAX) bad[t] = q;
                out_count[q] = 0;
                continue;
            }
            out_count[q] = got;
            for (uint32_t i = got; i < k; ++i) {
                oi[i] = ~0ull;
                od[i] = __builtin_inff();
            }
        }
    };
    if (nt <= 1) {
        run(0);
    } else {
        std::vector<std::thread> th;
        th.reserve(nt);
        for (unsigned t = 0; t < nt; ++t) th.emplace_back(run, t);
        for (std::thread& x : th) x.join();
    }
    for (unsigned t = 0; t < nt; ++t)
        if (bad[t] != UINT32_MAX)
            return set_error(BSR_E_NONFINITE, "NaN distance in query %u (the reference panics)", bad[t]);
    return BSR_OK;
}

}  // namespace bsr
