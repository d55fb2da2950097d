// Candidate-pair generation (replaces blocking.py:95-318, Spark's per-rule equi-join + UNION ALL).
//
// Per rule: rows with a non-NULL key are radix-sorted by (key, rank); runs of equal keys are
// blocks.  Every block contributes a contiguous range of candidate ordinals (n(n-1)/2 for a
// symmetric self-join, nL*nR for a bipartite join), so the whole job is one int64 ordinal space
// that is cut into equal chunks regardless of block skew, and sharded evenly across GPUs.
// Each ordinal decodes to one (l, r) row pair; the earlier-rule exclusion and the link-type
// predicate are applied per pair.  Two passes (count, emit) keep the output in ordinal order,
// so pair order is deterministic and independent of the grid.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cmath>

#include "spk_internal.h"

namespace spk {

static constexpr int EN_THREADS = 256;
static constexpr int EN_PER_THREAD = 8;
static constexpr int64_t EN_CHUNK = (int64_t)EN_THREADS * EN_PER_THREAD;
static constexpr int MAX_RULES = 32;

struct RuleKeys {
    const int64_t *keyL[MAX_RULES];  // key of rule j at each l-view position (position-ordered copy)
    const int64_t *keyR[MAX_RULES];  // key of rule j at each r-view position
};

// dst[i] = src[rows[i]]: a table array in a rule's view order, so k_enum reads it by view position
// (contiguous within a block) instead of gathering it by row for every candidate pair.
__global__ void k_by_position(int64_t n, const int32_t *__restrict__ rows, const int64_t *__restrict__ src,
                              int64_t *__restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[rows[i]];
}

// Grid-stride, valid keys counted per workgroup (ballots, then LDS): one atomic per workgroup -- an atomic
// per wave on the one counter serialised at L2 (187 us per million rows at cfg2).
__global__ void k_make_sort_keys(int64_t n, const int64_t *__restrict__ key, const int64_t *__restrict__ rank,
                                 uint64_t *__restrict__ out_keys, int32_t *__restrict__ out_rows,
                                 unsigned long long *__restrict__ n_valid) {
    __shared__ unsigned long long s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    unsigned long long cnt = 0;  // wave-uniform
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = i0 + threadIdx.x;
        bool v = false;
        if (i < n) {
            const int64_t k = key[i];
            const uint64_t r = rank ? (uint64_t)rank[i] : 0ull;
            out_keys[i] = k < 0 ? ~0ull : (((uint64_t)k << 32) | r);
            out_rows[i] = (int32_t)i;
            v = k >= 0;
        }
        cnt += (unsigned long long)__popcll(__ballot(v));
    }
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (threadIdx.x == 0 && s_cnt) atomicAdd(n_valid, s_cnt);
}

__global__ void k_heads(int64_t n, const uint64_t *__restrict__ keys, int64_t *__restrict__ flag) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    flag[i] = (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32)) ? 1 : 0;
}

__global__ void k_starts(int64_t n, const int64_t *__restrict__ flag, const int64_t *__restrict__ pos,
                         int64_t *__restrict__ bstart) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (flag[i]) bstart[pos[i]] = i;
}

__device__ inline int64_t lower_bound_hi(const uint64_t *keys, int64_t n, uint64_t k) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if ((keys[mid] >> 32) < k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// candidate count per block; bipartite blocks locate their r-side range by binary search.
__global__ void k_cand(int64_t B, const int64_t *__restrict__ bstart, int tri, const uint64_t *__restrict__ keysL,
                       const uint64_t *__restrict__ keysR, int64_t nR, int64_t *__restrict__ bstartR,
                       int64_t *__restrict__ bnR, int64_t *__restrict__ cand) {
    int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    int64_t n = bstart[b + 1] - bstart[b];
    if (tri) {
        cand[b] = n * (n - 1) / 2;
        return;
    }
    uint64_t k = keysL[bstart[b]] >> 32;
    int64_t lo = lower_bound_hi(keysR, nR, k);
    int64_t hi = lower_bound_hi(keysR, nR, k + 1);
    bstartR[b] = lo;
    bnR[b] = hi - lo;
    cand[b] = n * (hi - lo);
}

struct EnumArgs {
    int64_t q0, q1;             // rule-local ordinal range of this shard
    int64_t B;
    const int64_t *cand_off;    // [B] exclusive prefix of candidates
    const int64_t *bstart;      // [B+1] l-view block starts
    const int64_t *bstartR;     // [B] r-view starts (bipartite)
    const int64_t *bnR;         // [B] r-view sizes (bipartite)
    const int32_t *rowsL, *rowsR;
    const int64_t *rankL, *rankR;  // rank at each l- / r-view position (position-ordered copies)
    int tri;
    int rank_filter;            // 1: keep rank(l) < rank(r) (dedupe / link_and_dedupe)
    int64_t null_div;           // > 0: rank = src * null_div + r, r == null_div - 1 for a NULL unique id
    int rule;                   // index of this rule; rules [0, rule) exclude their pairs
    RuleKeys keys;
    int64_t *chunk_count;       // count pass output
    const int64_t *chunk_off;   // emit pass input
    int32_t *out_l, *out_r;
    int32_t *out_vl, *out_vr;   // emit pass: view positions (rules with a view), or null
};

__device__ inline int64_t tri_s(int64_t a, int64_t n) { return a * (2 * n - a - 1) / 2; }

template <bool EMIT>
__global__ __launch_bounds__(EN_THREADS) void k_enum(EnumArgs A) {
    __shared__ int64_t s_scan[EN_THREADS];
    const int64_t chunk = blockIdx.x;
    const int64_t base = A.q0 + chunk * EN_CHUNK + (int64_t)threadIdx.x * EN_PER_THREAD;
    int32_t xs[EN_PER_THREAD], ys[EN_PER_THREAD], vx[EN_PER_THREAD], vy[EN_PER_THREAD];
    unsigned keep = 0;
    if (base < A.q1) {
        // block containing `base`: last b with cand_off[b] <= base
        int64_t lo = 0, hi = A.B;
        while (hi - lo > 1) {
            int64_t mid = (lo + hi) >> 1;
            if (A.cand_off[mid] <= base) lo = mid;
            else hi = mid;
        }
        int64_t b = lo;
        int64_t w = base - A.cand_off[b];
        int64_t n = A.bstart[b + 1] - A.bstart[b];
        int64_t nr = A.tri ? n : A.bnR[b];
        int64_t cand_b = A.tri ? n * (n - 1) / 2 : n * nr;
        while (w >= cand_b) {  // skip empty blocks
            w -= cand_b;
            ++b;
            n = A.bstart[b + 1] - A.bstart[b];
            nr = A.tri ? n : A.bnR[b];
            cand_b = A.tri ? n * (n - 1) / 2 : n * nr;
        }
        int64_t a, c;
        if (A.tri) {
            double tn = 2.0 * (double)n - 1.0;
            double disc = tn * tn - 8.0 * (double)w;
            a = (int64_t)((tn - sqrt(disc > 0 ? disc : 0.0)) * 0.5);
            if (a < 0) a = 0;
            while (a > 0 && tri_s(a, n) > w) --a;
            while (a + 1 < n && tri_s(a + 1, n) <= w) ++a;
            c = a + 1 + (w - tri_s(a, n));
        } else {
            a = w / nr;
            c = w - a * nr;
        }
        for (int i = 0; i < EN_PER_THREAD; ++i) {
            int64_t q = base + i;
            if (q >= A.q1) break;
            if (i > 0) {  // advance to the next ordinal
                ++c;
                if (c >= nr) {
                    ++a;
                    c = A.tri ? a + 1 : 0;
                    if (a >= (A.tri ? n - 1 : n)) {
                        do {
                            ++b;
                            n = A.bstart[b + 1] - A.bstart[b];
                            nr = A.tri ? n : A.bnR[b];
                        } while ((A.tri ? n * (n - 1) / 2 : n * nr) == 0);
                        a = 0;
                        c = A.tri ? 1 : 0;
                    }
                }
            }
            const int64_t pa = A.bstart[b] + a, pc = A.tri ? A.bstart[b] + c : A.bstartR[b] + c;
            int32_t x = A.rowsL[pa];
            int32_t y = A.tri ? A.rowsL[pc] : A.rowsR[pc];
            vx[i] = (int32_t)pa;
            vy[i] = (int32_t)pc;
            bool ok = true;
            if (A.rank_filter) {
                int64_t rx = A.rankL[pa], ry = A.rankR[pc];
                if (A.tri) {
                    ok = rx != ry;  // sorted by rank inside the block: rx <= ry
                } else {
                    ok = rx < ry;
                }
                // `l.uid < r.uid` is NULL (the pair is dropped) when either unique id is NULL; pairs
                // across the two sources of link_and_dedupe are kept by `l.src < r.src` alone
                if (ok && A.null_div > 0 && rx / A.null_div == ry / A.null_div &&
                    (rx % A.null_div == A.null_div - 1 || ry % A.null_div == A.null_div - 1))
                    ok = false;
            }
            for (int j = 0; ok && j < A.rule; ++j) {
                int64_t kl = A.keys.keyL[j][pa];
                if (kl >= 0 && kl == A.keys.keyR[j][pc]) ok = false;
            }
            xs[i] = x;
            ys[i] = y;
            if (ok) keep |= 1u << i;
        }
    }
    int cnt = __popc(keep);
    // block-wide exclusive scan of the per-thread counts (Hillis-Steele in LDS)
    s_scan[threadIdx.x] = cnt;
    __syncthreads();
    for (int off = 1; off < EN_THREADS; off <<= 1) {
        int64_t v = threadIdx.x >= off ? s_scan[threadIdx.x - off] : 0;
        __syncthreads();
        s_scan[threadIdx.x] += v;
        __syncthreads();
    }
    int64_t incl = s_scan[threadIdx.x];
    if (!EMIT) {
        if (threadIdx.x == EN_THREADS - 1) A.chunk_count[chunk] = incl;
        return;
    }
    // the block's kept pairs are compacted in LDS, then written out with consecutive lanes on
    // consecutive positions (a thread's own run of EN_PER_THREAD would give strided lane writes)
    __shared__ int32_t s_out[4][EN_CHUNK];
    const bool views = A.out_vl != nullptr;
    int loc = (int)(incl - cnt);
    for (int i = 0; i < EN_PER_THREAD; ++i) {
        if (keep & (1u << i)) {
            s_out[0][loc] = xs[i];
            s_out[1][loc] = ys[i];
            if (views) {
                s_out[2][loc] = vx[i];
                s_out[3][loc] = vy[i];
            }
            ++loc;
        }
    }
    __syncthreads();
    const int total = (int)s_scan[EN_THREADS - 1];
    const int64_t out0 = A.chunk_off[chunk];
    for (int k = threadIdx.x; k < total; k += EN_THREADS) {
        A.out_l[out0 + k] = s_out[0][k];
        A.out_r[out0 + k] = s_out[1][k];
        if (views) {
            A.out_vl[out0 + k] = s_out[2][k];
            A.out_vr[out0 + k] = s_out[3][k];
        }
    }
}

struct SortedView {
    DevBuf<uint64_t> keys;
    DevBuf<int32_t> rows;
    int64_t n_valid = 0;
};

static int sort_view(spk_ctx *ctx, int64_t n, const int64_t *d_key, const int64_t *d_rank, SortedView &v,
                     DevBuf<uint8_t> &tmp) {
    DevBuf<uint64_t> k_in;
    DevBuf<int32_t> r_in;
    DevBuf<unsigned long long> cnt;
    SPK_TRY(k_in.alloc((size_t)n + 1));
    SPK_TRY(r_in.alloc((size_t)n + 1));
    SPK_TRY(v.keys.alloc((size_t)n + 1));
    SPK_TRY(v.rows.alloc((size_t)n + 1));
    SPK_TRY(cnt.alloc(1));
    SPK_HIP(hipMemsetAsync(cnt.p, 0, sizeof(unsigned long long), ctx->stream));
    if (n == 0) {
        v.n_valid = 0;
        return SPK_OK;
    }
    k_make_sort_keys<<<(unsigned)std::min<int64_t>((n + 255) / 256, 4 * (int64_t)ctx->n_cu), 256, 0, ctx->stream>>>(
        n, d_key, d_rank, k_in.p, r_in.p, cnt.p);
    SPK_HIP(hipGetLastError());
    size_t bytes = 0;
    SPK_HIP(rocprim::radix_sort_pairs(nullptr, bytes, k_in.p, v.keys.p, r_in.p, v.rows.p, (size_t)n, 0, 64,
                                      ctx->stream));
    SPK_TRY(tmp.alloc(bytes + 1));
    SPK_HIP(rocprim::radix_sort_pairs(tmp.p, bytes, k_in.p, v.keys.p, r_in.p, v.rows.p, (size_t)n, 0, 64,
                                      ctx->stream));
    unsigned long long h = 0;
    SPK_HIP(hipMemcpyAsync(&h, cnt.p, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    v.n_valid = (int64_t)h;
    return SPK_OK;
}

template <typename T>
static int exclusive_scan(spk_ctx *ctx, const T *in, T *out, int64_t n, DevBuf<uint8_t> &tmp) {
    if (n == 0) return SPK_OK;
    size_t bytes = 0;
    SPK_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, (T)0, (size_t)n, rocprim::plus<T>(), ctx->stream));
    SPK_TRY(tmp.alloc(bytes + 1));
    SPK_HIP(rocprim::exclusive_scan(tmp.p, bytes, in, out, (T)0, (size_t)n, rocprim::plus<T>(), ctx->stream));
    return SPK_OK;
}

struct RulePlan {
    SortedView L, R;
    DevBuf<int64_t> bstart, bstartR, bnR, cand, cand_off;
    // by view position: rank (l, r), then the keys of the earlier rules (l then r per rule)
    DevBuf<int64_t> bypos;
    const int64_t *rankL = nullptr, *rankR = nullptr;
    const int64_t *keyL[MAX_RULES] = {}, *keyR[MAX_RULES] = {};
    int64_t B = 0, T = 0;
    int tri = 1;
};

static int plan_rule(spk_ctx *ctx, int rule, bool symmetric, RulePlan &P, DevBuf<uint8_t> &tmp) {
    Table &tl = ctx->table[0];
    Table &tr = ctx->side_table(1);
    bool link_only = ctx->link_type == SPK_LINK_ONLY;
    P.tri = (symmetric && !link_only) ? 1 : 0;
    const int64_t *rankL = tl.rank.p;
    SPK_TRY(sort_view(ctx, tl.n, tl.key[0][rule]->p, link_only ? nullptr : rankL, P.L, tmp));
    if (!P.tri) SPK_TRY(sort_view(ctx, tr.n, tr.key[1][rule]->p, nullptr, P.R, tmp));
    int64_t n = P.L.n_valid;
    P.B = 0;
    P.T = 0;
    if (n == 0) return SPK_OK;
    DevBuf<int64_t> flag, pos;
    SPK_TRY(flag.alloc((size_t)n));
    SPK_TRY(pos.alloc((size_t)n));
    unsigned g = (unsigned)((n + 255) / 256);
    k_heads<<<g, 256, 0, ctx->stream>>>(n, P.L.keys.p, flag.p);
    SPK_TRY(exclusive_scan<int64_t>(ctx, flag.p, pos.p, n, tmp));
    int64_t last[2];
    SPK_HIP(hipMemcpyAsync(&last[0], pos.p + n - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipMemcpyAsync(&last[1], flag.p + n - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    int64_t B = last[0] + last[1];
    P.B = B;
    SPK_TRY(P.bstart.alloc((size_t)B + 1));
    SPK_TRY(P.bstartR.alloc((size_t)B + 1));
    SPK_TRY(P.bnR.alloc((size_t)B + 1));
    SPK_TRY(P.cand.alloc((size_t)B + 1));
    SPK_TRY(P.cand_off.alloc((size_t)B + 1));
    k_starts<<<g, 256, 0, ctx->stream>>>(n, flag.p, pos.p, P.bstart.p);
    SPK_HIP(hipMemcpyAsync(P.bstart.p + B, &n, 8, hipMemcpyHostToDevice, ctx->stream));
    k_cand<<<(unsigned)((B + 255) / 256), 256, 0, ctx->stream>>>(B, P.bstart.p, P.tri, P.L.keys.p,
                                                                 P.tri ? nullptr : P.R.keys.p, P.R.n_valid,
                                                                 P.bstartR.p, P.bnR.p, P.cand.p);
    SPK_HIP(hipGetLastError());
    SPK_TRY(exclusive_scan<int64_t>(ctx, P.cand.p, P.cand_off.p, B, tmp));
    int64_t lc[2];
    SPK_HIP(hipMemcpyAsync(&lc[0], P.cand_off.p + B - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipMemcpyAsync(&lc[1], P.cand.p + B - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    P.T = lc[0] + lc[1];
    return SPK_OK;
}

// Position-ordered copies of what k_enum reads per candidate pair: ranks (dedupe / link_and_dedupe) and
// the keys of rules 0 .. rule-1 (earlier-rule exclusion).  Built just before a pass over the rule and
// released after it (release_by_position), so at most one rule's copies exist at a time; a symmetric
// self-join (tri) reads the l-side rank copy for both sides.
static int build_by_position(spk_ctx *ctx, int rule, RulePlan &P) {
    Table &tl = ctx->table[0];
    Table &tr = ctx->side_table(1);
    const bool ranks = ctx->link_type != SPK_LINK_ONLY;
    const int64_t nL = P.L.n_valid, nR = P.tri ? nL : P.R.n_valid;
    const int32_t *rowsR = P.tri ? P.L.rows.p : P.R.rows.p;
    const int64_t n_rank = ranks ? (P.tri ? nL : nL + nR) : 0;
    SPK_TRY(P.bypos.alloc((size_t)(n_rank + (int64_t)rule * (nL + nR)) + 1));
    int64_t *at = P.bypos.p;
    auto by_pos = [&](int64_t m, const int32_t *rows, const int64_t *src) -> const int64_t * {
        int64_t *dst = at;
        at += m;
        if (m > 0) k_by_position<<<(unsigned)((m + 255) / 256), 256, 0, ctx->stream>>>(m, rows, src, dst);
        return dst;
    };
    if (ranks) {
        P.rankL = by_pos(nL, P.L.rows.p, tl.rank.p);
        P.rankR = P.tri ? P.rankL : by_pos(nR, rowsR, tr.rank.p);
    }
    for (int j = 0; j < rule; ++j) {
        P.keyL[j] = by_pos(nL, P.L.rows.p, tl.key[0][j]->p);
        P.keyR[j] = by_pos(nR, rowsR, tr.key[1][j]->p);
    }
    SPK_HIP(hipGetLastError());
    return SPK_OK;
}

static void release_by_position(RulePlan &P) {
    P.bypos.release();
    P.rankL = P.rankR = nullptr;
    for (int j = 0; j < MAX_RULES; ++j) P.keyL[j] = P.keyR[j] = nullptr;
}

}  // namespace spk

using namespace spk;

extern "C" int spk_ctx_set_link_type(spk_ctx *ctx, int link_type) {
    SPK_REQUIRE(ctx && link_type >= 0 && link_type <= 2, SPK_E_INVALID, "bad link_type");
    ctx->link_type = link_type;
    return SPK_OK;
}

extern "C" int spk_block(spk_ctx *ctx, int link_type, int n_rules, const int32_t *rule_symmetric, int shard,
                         int n_shards, int64_t *out_n_pairs, int64_t *out_n_candidates_total) {
    SPK_REQUIRE(ctx && n_rules >= 1 && n_rules <= MAX_RULES && rule_symmetric, SPK_E_INVALID,
                "spk_block: need 1..32 rules");
    SPK_REQUIRE(link_type >= 0 && link_type <= 2, SPK_E_INVALID, "spk_block: bad link_type");
    SPK_REQUIRE(n_shards >= 1 && shard >= 0 && shard < n_shards, SPK_E_INVALID, "spk_block: bad shard");
    SPK_HIP(hipSetDevice(ctx->device));
    ctx->link_type = link_type;
    Table &tl = ctx->table[0];
    Table &tr = ctx->side_table(1);
    SPK_REQUIRE(tl.n >= 0 && tr.n >= 0, SPK_E_STATE, "spk_block: tables not loaded");
    bool link_only = link_type == SPK_LINK_ONLY;
    SPK_REQUIRE(link_only || tl.rank.p || tl.n == 0, SPK_E_STATE, "spk_block: rank not set");
    for (int r = 0; r < n_rules; ++r) {
        SPK_REQUIRE((int)tl.key[0].size() > r && tl.key[0][r]->p && (int)tr.key[1].size() > r && tr.key[1][r]->p,
                    SPK_E_STATE, "spk_block: keys not set for every rule");
    }
    SPK_TRY(ctx->begin(K_BLOCK));
    DevBuf<uint8_t> tmp;
    std::vector<RulePlan *> plans;
    struct Guard {
        std::vector<RulePlan *> &v;
        ~Guard() {
            for (RulePlan *p : v) delete p;
        }
    } guard{plans};
    int64_t total = 0;
    for (int r = 0; r < n_rules; ++r) {
        plans.push_back(new RulePlan());
        SPK_TRY(plan_rule(ctx, r, rule_symmetric[r] != 0, *plans.back(), tmp));
        total += plans.back()->T;
    }
    int64_t g_lo = (int64_t)((__int128)total * shard / n_shards);
    int64_t g_hi = (int64_t)((__int128)total * (shard + 1) / n_shards);

    EnumArgs base{};
    // count pass
    std::vector<DevBuf<int64_t> *> counts(n_rules, nullptr), offs(n_rules, nullptr);
    struct G2 {
        std::vector<DevBuf<int64_t> *> &a, &b;
        ~G2() {
            for (auto *x : a) delete x;
            for (auto *x : b) delete x;
        }
    } g2{counts, offs};
    std::vector<int64_t> rule_lo(n_rules), rule_hi(n_rules), rule_base(n_rules), n_chunks(n_rules);
    int64_t acc = 0, n_out = 0;
    for (int r = 0; r < n_rules; ++r) {
        RulePlan &P = *plans[r];
        int64_t lo = std::max<int64_t>(g_lo - acc, 0), hi = std::min<int64_t>(g_hi - acc, P.T);
        acc += P.T;
        rule_lo[r] = lo;
        rule_hi[r] = hi;
        n_chunks[r] = hi > lo ? (hi - lo + EN_CHUNK - 1) / EN_CHUNK : 0;
        rule_base[r] = n_out;
        if (!n_chunks[r]) continue;
        counts[r] = new DevBuf<int64_t>();
        offs[r] = new DevBuf<int64_t>();
        SPK_TRY(build_by_position(ctx, r, P));
        SPK_TRY(counts[r]->alloc((size_t)n_chunks[r]));
        SPK_TRY(offs[r]->alloc((size_t)n_chunks[r]));
        EnumArgs A = base;
        A.q0 = lo;
        A.q1 = hi;
        A.B = P.B;
        A.cand_off = P.cand_off.p;
        A.bstart = P.bstart.p;
        A.bstartR = P.bstartR.p;
        A.bnR = P.bnR.p;
        A.rowsL = P.L.rows.p;
        A.rowsR = P.tri ? P.L.rows.p : P.R.rows.p;
        A.rankL = P.rankL;
        A.rankR = P.rankR;
        for (int j = 0; j < r; ++j) {
            A.keys.keyL[j] = P.keyL[j];
            A.keys.keyR[j] = P.keyR[j];
        }
        A.tri = P.tri;
        A.rank_filter = link_only ? 0 : 1;
        A.null_div = tl.null_div;
        A.rule = r;
        A.chunk_count = counts[r]->p;
        k_enum<false><<<(unsigned)n_chunks[r], EN_THREADS, 0, ctx->stream>>>(A);
        SPK_HIP(hipGetLastError());
        SPK_TRY(exclusive_scan<int64_t>(ctx, counts[r]->p, offs[r]->p, n_chunks[r], tmp));
        SPK_HIP(hipStreamSynchronize(ctx->stream));  // the copies are freed next: the pass must be done
        release_by_position(P);
        int64_t lc[2];
        SPK_HIP(hipMemcpyAsync(&lc[0], offs[r]->p + n_chunks[r] - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
        SPK_HIP(hipMemcpyAsync(&lc[1], counts[r]->p + n_chunks[r] - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
        SPK_HIP(hipStreamSynchronize(ctx->stream));
        n_out += lc[0] + lc[1];
    }
    SPK_REQUIRE(n_out < (int64_t)1 << 40, SPK_E_LIMIT, "spk_block: pair count too large");
    SPK_TRY(ctx->pl.alloc((size_t)n_out + 1));
    SPK_TRY(ctx->pr.alloc((size_t)n_out + 1));
    // rules 1 .. MAX_VIEWS-1 keep their row order (view) and emit their pairs' view positions
    const int n_views = std::min(n_rules, MAX_VIEWS) - 1;
    const int64_t pv_base = n_views > 0 ? rule_base[1] : n_out;
    ctx->n_views = 0;
    ctx->pv_base = pv_base;
    if (n_views > 0 && n_out > pv_base) {
        SPK_TRY(ctx->pvl.alloc((size_t)(n_out - pv_base) + 1));
        SPK_TRY(ctx->pvr.alloc((size_t)(n_out - pv_base) + 1));
    }
    for (int r = 0; r < n_rules; ++r) {
        if (!n_chunks[r]) continue;
        RulePlan &P = *plans[r];
        SPK_TRY(build_by_position(ctx, r, P));
        EnumArgs A = base;
        A.q0 = rule_lo[r];
        A.q1 = rule_hi[r];
        A.B = P.B;
        A.cand_off = P.cand_off.p;
        A.bstart = P.bstart.p;
        A.bstartR = P.bstartR.p;
        A.bnR = P.bnR.p;
        A.rowsL = P.L.rows.p;
        A.rowsR = P.tri ? P.L.rows.p : P.R.rows.p;
        A.rankL = P.rankL;
        A.rankR = P.rankR;
        for (int j = 0; j < r; ++j) {
            A.keys.keyL[j] = P.keyL[j];
            A.keys.keyR[j] = P.keyR[j];
        }
        A.tri = P.tri;
        A.rank_filter = link_only ? 0 : 1;
        A.null_div = tl.null_div;
        A.rule = r;
        A.chunk_off = offs[r]->p;
        A.out_l = ctx->pl.p + rule_base[r];
        A.out_r = ctx->pr.p + rule_base[r];
        const bool view = r >= 1 && r <= n_views;
        A.out_vl = view ? ctx->pvl.p + (rule_base[r] - pv_base) : nullptr;
        A.out_vr = view ? ctx->pvr.p + (rule_base[r] - pv_base) : nullptr;
        k_enum<true><<<(unsigned)n_chunks[r], EN_THREADS, 0, ctx->stream>>>(A);
        SPK_HIP(hipGetLastError());
        SPK_HIP(hipStreamSynchronize(ctx->stream));
        release_by_position(P);
    }
    SPK_TRY(ctx->end(K_BLOCK));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    for (int r = 1; r <= n_views; ++r) {
        RuleView &v = ctx->views[r];
        RulePlan &P = *plans[r];
        take_buf(v.rowsL, P.L.rows);
        v.nL = P.L.n_valid;
        v.tri = P.tri != 0;
        if (!v.tri) take_buf(v.rowsR, P.R.rows);
        else v.rowsR.release();
        v.nR = v.tri ? v.nL : P.R.n_valid;
        v.pair_lo = rule_base[r];
        v.pair_hi = r + 1 < n_rules ? rule_base[r + 1] : n_out;
    }
    ctx->n_views = n_views;
    ctx->pair_terms.assign(ctx->rule_terms, ctx->rule_terms + n_rules);
    ctx->pair_rule_lo.assign(rule_base.begin(), rule_base.end());
    ctx->pair_rule_hi.resize(n_rules);
    for (int r = 0; r < n_rules; ++r) ctx->pair_rule_hi[r] = r + 1 < n_rules ? rule_base[r + 1] : n_out;
    ctx->n_pairs = n_out;
    ctx->pairs_valid = true;
    ctx->pairs_epoch++;
    ctx->tf_mp.release();  // a kept tf result describes the old pair set (spk_tf_copy refuses it)
    ctx->tf_count = -1;
    ctx->codes_valid = false;
    if (out_n_pairs) *out_n_pairs = n_out;
    if (out_n_candidates_total) *out_n_candidates_total = total;
    return SPK_OK;
}
