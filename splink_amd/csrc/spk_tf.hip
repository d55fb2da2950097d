// Term-frequency adjustment (replaces term_frequencies.py:49-117: the per-value GROUP BY of the match
// probability over pairs with equal values, the broadcast join of the adjustments and the Bayes
// combination).
//
// The per-value sums are exact and order-free, so they are bit-identical for any grid, any run and any
// number of ranks: mp depends only on the comparison pattern, so Σ_{pairs with value v} mp =
// Σ_p count(v, p) · mp(p).  The qualifying pairs' keys (v, pattern) are radix-sorted and run-length
// encoded (integer counts).  Each value v has a scale E_v = max over its terms of ilogb(mp) + 1 (a first
// pass, spk_tf_scales: ranks holding shards of the pairs all-reduce it with MAX), and each run adds
// count · mp(p) · 2^-E_v to v's accumulator in fixed point: SPK_TF_LIMBS int64 limbs of 20 bits (limb 0
// the integer part, limb j the bits 2^-20j .. 2^-20(j-1)+1), truncated below 2^-260.  The window follows
// the value's largest term, so a value whose pairs all score tiny (mp ~ 1e-300, subnormals included)
// keeps its relative precision (2^-200 or better); integer adds are exact, so the device atomics' order,
// the shard of pairs and the ranks' all-reduce (int64 sum) do not change the result, and one conversion
// to double at the end (spk_tf_limbs_to_sum, scaled back by 2^E_v) gives every caller the same value.
#include <algorithm>
#include <cmath>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_run_length_encode.hpp>

#include "spk_internal.h"

namespace spk {

constexpr int TF_LIMBS = SPK_TF_LIMBS;
constexpr int TF_BITS = 20;
constexpr unsigned long long TF_NONE = ~0ull;  // key of a pair that does not qualify

// key = value * n_patterns + code for pairs with equal, non-NULL values and a non-NULL mp, else `none` (all ones in
// the key's bits: the keys are sorted over bit_length(n_values * n_patterns) bits only, in 32-bit words when that
// fits -- cfg3 on one GPU: 31 bits instead of 64, half the bytes and half the radix passes)
template <typename KeyT, typename CodeT>
__global__ void k_tf_keys(int64_t P, const int32_t *__restrict__ pl, const int32_t *__restrict__ pr,
                          const int64_t *__restrict__ ids0, const int64_t *__restrict__ ids1, const CodeT *__restrict__ codes,
                          const double *__restrict__ mpat, int64_t n_values, int64_t npat, KeyT none,
                          KeyT *__restrict__ keys) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const int64_t a = ids0[pl[p]], b = ids1[pr[p]];
    const uint32_t c = (uint32_t)codes[p];
    const bool ok = a >= 0 && a == b && a < n_values && !isnan(mpat[c]);
    keys[p] = ok ? (KeyT)(a * npat + (int64_t)c) : none;
}

// The fixed-point limbs of y = x 2^-E (x > 0, y < 1 for E >= ilogb(x) + 1): y = Σ_j limb_j 2^(-20 j),
// truncated below 2^-260.
__device__ inline void tf_limbs(double x, int E, uint32_t (&limb)[TF_LIMBS]) {
#pragma unroll
    for (int j = 0; j < TF_LIMBS; ++j) limb[j] = 0;
    if (!(x > 0.0)) return;
    const uint64_t bits = (uint64_t)__double_as_longlong(x);
    const int ex = (int)((bits >> 52) & 0x7FF);
    const uint64_t M = (bits & ((1ull << 52) - 1)) | (ex ? (1ull << 52) : 0ull);
    // x = M 2^(e - 1075) (subnormals: e = 1); bit b of F = y 2^260 is bit b - s of M
    const int s = (ex ? ex : 1) - 1075 - E + TF_BITS * (TF_LIMBS - 1);
#pragma unroll
    for (int j = 0; j < TF_LIMBS; ++j) {
        const int lo = TF_BITS * (TF_LIMBS - 1 - j);  // F's bit of limb j's lowest bit
        const int sh = lo - s;
        uint64_t v;
        if (sh >= 0) v = sh >= 64 ? 0ull : (M >> sh);
        else v = -sh >= 64 ? 0ull : (M << (-sh));
        limb[j] = (uint32_t)(v & ((1u << TF_BITS) - 1));
    }
}

// ilogb(x) + 1 for x > 0 (subnormals included): the smallest E with x < 2^E
__device__ inline int tf_exponent(double x) {
    const uint64_t bits = (uint64_t)__double_as_longlong(x);
    const int ex = (int)((bits >> 52) & 0x7FF);
    if (ex) return ex - 1022;
    const uint64_t M = bits & ((1ull << 52) - 1);
    return (63 - __clzll((long long)M)) - 1073;  // x = M 2^-1074
}

constexpr int TF_NO_SCALE = INT32_MIN;  // a value with no (positive) term

// One run of equal keys: the value's scale (max of its terms' exponents).
template <typename KeyT>
__global__ void k_tf_scale(const KeyT *__restrict__ keys, const unsigned int *__restrict__ n_runs,
                           const double *__restrict__ mpat, int64_t npat, KeyT none, int *__restrict__ scale) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)*n_runs) return;
    const KeyT k = keys[i];
    if (k == none) return;
    const int64_t v = (int64_t)k / npat;
    const double x = mpat[(int64_t)k - v * npat];
    if (x > 0.0) atomicMax(&scale[v], tf_exponent(x));
}

// One run of equal keys: its count times the pattern's mp, scaled by the value's 2^-E, limb by limb, into
// the value's accumulator.
template <typename KeyT>
__global__ void k_tf_runs(const KeyT *__restrict__ keys, const unsigned int *__restrict__ counts,
                          const unsigned int *__restrict__ n_runs, const double *__restrict__ mpat, int64_t npat, KeyT none,
                          const int *__restrict__ scale, unsigned long long *__restrict__ acc,
                          unsigned long long *__restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)*n_runs) return;
    const KeyT k = keys[i];
    if (k == none) return;
    const int64_t v = (int64_t)k / npat;
    const double x = mpat[(int64_t)k - v * npat];
    const unsigned long long n = counts[i];
    atomicAdd(&cnt[v], n);
    const int E = scale[v];
    if (!(x > 0.0) || E == TF_NO_SCALE) return;
    uint32_t limb[TF_LIMBS];
    tf_limbs(x, E, limb);
#pragma unroll
    for (int j = 0; j < TF_LIMBS; ++j)
        if (limb[j]) atomicAdd(&acc[v * TF_LIMBS + j], n * (unsigned long long)limb[j]);
}

// The (value, pattern) counts directly: one counter per value x pattern (64-bit), lanes of a wave with equal
// keys add once (the pairs of a block share a value and mostly a pattern, so a wave adds a few times, not 64).
// Replaces the keys + radix sort + run-length encode of tf_pass when n_values x n_patterns <= TF_HIST_MAX: the
// whole cfg3 job on one GPU (3.08e9 pairs, 300k values x 576 patterns) sorted 6 x 2^30 keys, ~0.35 s of device
// time (profiles/r6_tf_sort_kernel_stats.csv).  The counts are the runs' counts, so the sums are identical.
// Up to 2^30 counters (8 GB) and no more than ~4 per pair: beyond that the sort's keys (4-8 B per pair) are smaller.
constexpr int64_t TF_HIST_MAX = (int64_t)1 << 30;
template <typename CodeT>
__global__ void k_tf_hist(int64_t P, const int32_t *__restrict__ pl, const int32_t *__restrict__ pr,
                          const int64_t *__restrict__ ids0, const int64_t *__restrict__ ids1,
                          const CodeT *__restrict__ codes, const double *__restrict__ mpat, int64_t n_values,
                          int64_t npat, unsigned long long *__restrict__ hist) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < P; base += stride) {  // wave-uniform
        const int64_t p = base + threadIdx.x;
        int64_t key = -1;
        if (p < P) {
            const int64_t a = ids0[pl[p]], b = ids1[pr[p]];
            const uint32_t c = (uint32_t)codes[p];
            if (a >= 0 && a == b && a < n_values && !isnan(mpat[c])) key = a * npat + (int64_t)c;
        }
        bool todo = key >= 0;
        while (__any(todo)) {  // one add per distinct key of the wave
            const unsigned long long m = __ballot(todo);
            const int lead = __ffsll((unsigned long long)m) - 1;
            const int64_t k = __shfl(key, lead);
            const unsigned long long same = __ballot(todo && key == k);
            if ((int)(threadIdx.x & 63) == lead) atomicAdd(&hist[k], (unsigned long long)__popcll(same));
            todo = todo && key != k;
        }
    }
}

// The scale / sum passes over the histogram's non-zero counters (as k_tf_scale / k_tf_runs over the runs).
__global__ void k_tf_hist_apply(int64_t M, int64_t npat, const unsigned long long *__restrict__ hist,
                                const double *__restrict__ mpat, int *__restrict__ scale, unsigned long long *__restrict__ acc,
                                unsigned long long *__restrict__ cnt) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += stride) {
        const unsigned long long n = hist[i];
        if (!n) continue;
        const int64_t v = i / npat;
        const double x = mpat[i - v * npat];
        if (!acc) {
            if (x > 0.0) atomicMax(&scale[v], tf_exponent(x));
            continue;
        }
        atomicAdd(&cnt[v], n);
        const int E = scale[v];
        if (!(x > 0.0) || E == TF_NO_SCALE) continue;
        uint32_t limb[TF_LIMBS];
        tf_limbs(x, E, limb);
#pragma unroll
        for (int j = 0; j < TF_LIMBS; ++j)
            if (limb[j]) atomicAdd(&acc[v * TF_LIMBS + j], n * (unsigned long long)limb[j]);
    }
}

// The sort form of tf_pass: (value, pattern) keys of `bits` bits, radix-sorted and run-length encoded, chunk by
// chunk.  The keys, the sorted keys and the sort's scratch live in one context buffer (tf_sort) from the scale
// pass to the sum pass, instead of five hipMalloc / hipFree pairs per pass: at cfg3's 3.08e9 pairs those were
// ~36 GB per pass, and the same kernels' tf stage took 0.49 s on one box and 1.8 s on another
// (profiles/r6_fulljob_cfg3_1gpu_tfsort*.json).
template <typename KeyT>
static int tf_pass_sort(spk_ctx *ctx, int64_t n_values, int64_t npat, int bits, const int64_t *d0, const int64_t *d1,
                        int *d_scale, unsigned long long *acc, unsigned long long *cnt, const std::vector<int64_t> *key) {
    const int64_t P = ctx->n_pairs;
    const KeyT none = (KeyT)(bits >= 64 ? ~0ull : ((1ull << bits) - 1));
    // the sort and the run counts work on uint32 lengths: chunks of at most 2^30 pairs
    const int64_t CH = (int64_t)1 << 30;
    const bool cache = key != nullptr && P <= CH;
    const int64_t cap = std::min<int64_t>(std::max<int64_t>(P, 1), CH);
    const size_t kb = ((size_t)cap * sizeof(KeyT) + 255) & ~(size_t)255;
    auto finish = [&]() {  // the sum pass ends the column's use of the sort buffers
        if (acc) {
            ctx->tf_sort.release();
            ctx->tf_uniq.release();
            ctx->tf_runs.release();
            ctx->tf_key.clear();
        }
    };
    if (cache && ctx->tf_key == *key && ctx->tf_uniq.p) {  // the runs of the scale pass
        const unsigned g = (unsigned)((cap + 255) / 256);
        const KeyT *uk = reinterpret_cast<const KeyT *>(ctx->tf_uniq.p);
        if (acc) k_tf_runs<KeyT><<<g, 256, 0, ctx->stream>>>(uk, ctx->tf_runs.p, ctx->tf_nruns.p, ctx->mpat_score.p, npat, none,
                                                             d_scale, acc, cnt);
        else k_tf_scale<KeyT><<<g, 256, 0, ctx->stream>>>(uk, ctx->tf_nruns.p, ctx->mpat_score.p, npat, none, d_scale);
        SPK_HIP(hipGetLastError());
        SPK_HIP(hipStreamSynchronize(ctx->stream));
        finish();
        return SPK_OK;
    }
    ctx->tf_key.clear();
    SPK_TRY(ctx->tf_uniq.alloc((size_t)cap));  // 8-byte slots: room for either key width
    SPK_TRY(ctx->tf_runs.alloc((size_t)cap));
    SPK_TRY(ctx->tf_nruns.alloc(1));
    KeyT *uniq = reinterpret_cast<KeyT *>(ctx->tf_uniq.p);
    size_t bytes = 0, b2 = 0;
    SPK_HIP(rocprim::radix_sort_keys(nullptr, bytes, (KeyT *)nullptr, (KeyT *)nullptr, (size_t)cap, 0, bits, ctx->stream));
    SPK_HIP(rocprim::run_length_encode(nullptr, b2, (KeyT *)nullptr, (size_t)cap, uniq, ctx->tf_runs.p, ctx->tf_nruns.p,
                                       ctx->stream));
    const size_t tb = std::max(bytes, b2) + 256;
    SPK_TRY(ctx->tf_sort.alloc(2 * kb + tb));
    KeyT *k_in = reinterpret_cast<KeyT *>(ctx->tf_sort.p), *k_out = reinterpret_cast<KeyT *>(ctx->tf_sort.p + kb);
    uint8_t *tmp = ctx->tf_sort.p + 2 * kb;
    for (int64_t c0 = 0; c0 < P; c0 += CH) {
        const int64_t n = std::min<int64_t>(CH, P - c0);
        const unsigned g = (unsigned)((n + 255) / 256);
        if (ctx->code_bytes == 2)
            k_tf_keys<KeyT, uint16_t><<<g, 256, 0, ctx->stream>>>(n, ctx->pl.p + c0, ctx->pr.p + c0, d0, d1,
                                                                 reinterpret_cast<const uint16_t *>(ctx->codes.p) + c0,
                                                                 ctx->mpat_score.p, n_values, npat, none, k_in);
        else
            k_tf_keys<KeyT, uint32_t><<<g, 256, 0, ctx->stream>>>(n, ctx->pl.p + c0, ctx->pr.p + c0, d0, d1,
                                                                 reinterpret_cast<const uint32_t *>(ctx->codes.p) + c0,
                                                                 ctx->mpat_score.p, n_values, npat, none, k_in);
        SPK_HIP(hipGetLastError());
        size_t tb1 = tb, tb2 = tb;
        SPK_HIP(rocprim::radix_sort_keys(tmp, tb1, k_in, k_out, (size_t)n, 0, bits, ctx->stream));
        SPK_HIP(rocprim::run_length_encode(tmp, tb2, k_out, (size_t)n, uniq, ctx->tf_runs.p, ctx->tf_nruns.p, ctx->stream));
        if (acc) k_tf_runs<KeyT><<<g, 256, 0, ctx->stream>>>(uniq, ctx->tf_runs.p, ctx->tf_nruns.p, ctx->mpat_score.p, npat,
                                                             none, d_scale, acc, cnt);
        else k_tf_scale<KeyT><<<g, 256, 0, ctx->stream>>>(uniq, ctx->tf_nruns.p, ctx->mpat_score.p, npat, none, d_scale);
        SPK_HIP(hipGetLastError());
    }
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    if (cache && !acc) ctx->tf_key = *key;  // the sum pass reuses these runs
    finish();
    return SPK_OK;
}

// The runs of (value, pattern) keys of the current pairs, value ids per row on the device (d0 side 0, d1
// side 1), chunk by chunk: scale pass (acc null: each value's scale into d_scale) or sum pass (the counts
// and the scaled fixed-point sums at the given d_scale).
// key (optional): what the runs depend on (pair set, codes, scores, value ids).  With a key and one chunk,
// the runs stay in the context after the scale pass, and a sum pass with the same key reuses them instead of
// building and sorting the keys again (the tf adjustment's two passes then cost one sort); the sum pass
// releases them.
static int tf_pass(spk_ctx *ctx, int64_t n_values, const int64_t *d0, const int64_t *d1, int *d_scale,
                   unsigned long long *acc, unsigned long long *cnt, const std::vector<int64_t> *key = nullptr) {
    SPK_REQUIRE(ctx->mpat_valid && ctx->mpat_score.p, SPK_E_STATE, "tf: run spk_score first (mp per pattern)");
    SPK_REQUIRE(n_values < ((int64_t)1 << 31), SPK_E_LIMIT, "tf: more than 2^31 distinct values");
    const int64_t P = ctx->n_pairs;
    const int64_t npat = std::max<int64_t>(ctx->n_patterns, 1);
    if (ctx->tf_mode == 0 && n_values <= TF_HIST_MAX / npat &&
        n_values * npat <= std::max<int64_t>(4 * P, (int64_t)1 << 24)) {  // the counts directly, no sort
        const int64_t M = std::max<int64_t>(n_values * npat, 1);
        const bool hit = key != nullptr && ctx->tf_key == *key && ctx->tf_hist.p && ctx->tf_hist.n >= (size_t)M;
        if (!hit) {
            ctx->tf_key.clear();
            ctx->tf_uniq.release();
            ctx->tf_runs.release();
            SPK_TRY(ctx->tf_hist.alloc((size_t)M));
            SPK_HIP(hipMemsetAsync(ctx->tf_hist.p, 0, (size_t)M * 8, ctx->stream));
            const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((P + 255) / 256, 64 * (int64_t)ctx->n_cu));
            if (P > 0) {
                if (ctx->code_bytes == 2)
                    k_tf_hist<uint16_t><<<g, 256, 0, ctx->stream>>>(P, ctx->pl.p, ctx->pr.p, d0, d1,
                                                                   reinterpret_cast<const uint16_t *>(ctx->codes.p),
                                                                   ctx->mpat_score.p, n_values, npat, ctx->tf_hist.p);
                else
                    k_tf_hist<uint32_t><<<g, 256, 0, ctx->stream>>>(P, ctx->pl.p, ctx->pr.p, d0, d1,
                                                                   reinterpret_cast<const uint32_t *>(ctx->codes.p),
                                                                   ctx->mpat_score.p, n_values, npat, ctx->tf_hist.p);
                SPK_HIP(hipGetLastError());
            }
        }
        const unsigned g2 = (unsigned)std::max<int64_t>(1, std::min<int64_t>((M + 255) / 256, 16 * (int64_t)ctx->n_cu));
        k_tf_hist_apply<<<g2, 256, 0, ctx->stream>>>(M, npat, ctx->tf_hist.p, ctx->mpat_score.p, d_scale, acc, cnt);
        SPK_HIP(hipGetLastError());
        SPK_HIP(hipStreamSynchronize(ctx->stream));
        if (key != nullptr && !acc) {
            ctx->tf_key = *key;  // the sum pass with the same key reuses the counts
        } else {
            ctx->tf_key.clear();
            ctx->tf_hist.release();
        }
        return SPK_OK;
    }
    const int bits = 64 - __builtin_clzll((unsigned long long)std::max<int64_t>(n_values * npat, 1));
    if (bits <= 32 && ctx->tf_mode != 2) return tf_pass_sort<uint32_t>(ctx, n_values, npat, bits, d0, d1, d_scale, acc, cnt, key);
    return tf_pass_sort<unsigned long long>(ctx, n_values, npat, bits, d0, d1, d_scale, acc, cnt, key);
}

__global__ void k_fill_i32(int64_t n, int v, int *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = v;
}

// Per-value scales of this context's pairs (TF_NO_SCALE: no positive term).
static int tf_scales(spk_ctx *ctx, int64_t n_values, const int64_t *d0, const int64_t *d1, int32_t *out_scale,
                     const std::vector<int64_t> *key = nullptr) {
    DevBuf<int> sc;
    SPK_TRY(sc.alloc((size_t)n_values + 1));
    k_fill_i32<<<(unsigned)((n_values + 256) / 256), 256, 0, ctx->stream>>>(n_values + 1, TF_NO_SCALE, sc.p);
    SPK_TRY(tf_pass(ctx, n_values, d0, d1, sc.p, nullptr, nullptr, key));
    if (n_values) SPK_HIP(hipMemcpyAsync(out_scale, sc.p, (size_t)n_values * 4, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    return SPK_OK;
}

// Exact per-value sums at the given scales (every rank's scales all-reduced with MAX).
static int tf_exact(spk_ctx *ctx, int64_t n_values, const int64_t *d0, const int64_t *d1, const int32_t *scale,
                    int64_t *out_limbs, int64_t *out_count, const std::vector<int64_t> *key = nullptr) {
    DevBuf<unsigned long long> acc, cnt;
    DevBuf<int> sc;
    SPK_TRY(acc.alloc((size_t)n_values * TF_LIMBS + 1));
    SPK_TRY(cnt.alloc((size_t)n_values + 1));
    SPK_TRY(sc.alloc((size_t)n_values + 1));
    SPK_HIP(hipMemsetAsync(acc.p, 0, ((size_t)n_values * TF_LIMBS + 1) * 8, ctx->stream));
    SPK_HIP(hipMemsetAsync(cnt.p, 0, ((size_t)n_values + 1) * 8, ctx->stream));
    if (n_values) SPK_HIP(hipMemcpyAsync(sc.p, scale, (size_t)n_values * 4, hipMemcpyHostToDevice, ctx->stream));
    SPK_TRY(tf_pass(ctx, n_values, d0, d1, sc.p, acc.p, cnt.p, key));
    if (n_values) {
        SPK_HIP(hipMemcpyAsync(out_limbs, acc.p, (size_t)n_values * TF_LIMBS * 8, hipMemcpyDeviceToHost, ctx->stream));
        SPK_HIP(hipMemcpyAsync(out_count, cnt.p, (size_t)n_values * 8, hipMemcpyDeviceToHost, ctx->stream));
    }
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    return SPK_OK;
}

struct TfApply {
    int n;
    const int64_t *ids0[8];
    const int64_t *ids1[8];
    const double *tab[8];
    int64_t tab_n[8];
};

// bayes(mp, adj...) = Πp / (Πp + Π(1-p)) (term_frequencies.py:21-46, :98-117)
__global__ void k_tf_apply(TfApply T, int64_t start, int64_t n, const int32_t *__restrict__ pl,
                           const int32_t *__restrict__ pr, const double *__restrict__ mp, double *__restrict__ out,
                           double *__restrict__ out_adj) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t p = start + i;
    double m = mp[p];
    double adj[8];
    for (int c = 0; c < T.n; ++c) {
        int64_t a = T.ids0[c][pl[p]], b = T.ids1[c][pr[p]];
        double v = 0.5;
        if (a >= 0 && a == b && a < T.tab_n[c]) {
            double x = T.tab[c][a];
            if (!isnan(x)) v = x;
        }
        adj[c] = v;
        if (out_adj) out_adj[i * T.n + c] = v;
    }
    if (isnan(m)) {
        out[i] = NAN;
        return;
    }
    double a = m, b = 1.0 - m;
    for (int c = 0; c < T.n; ++c) a = a * adj[c];
    for (int c = 0; c < T.n; ++c) b = b * (1.0 - adj[c]);
    double d = a + b;
    out[i] = d == 0.0 ? NAN : a / d;
}


__global__ void k_ids_from_meta(int64_t n, const RecMeta *__restrict__ meta, int64_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = meta[i].len16 < 0 ? -1 : (int64_t)meta[i].key;
}

static int column_ids(spk_ctx *ctx, Table &t, int col, DevBuf<int64_t> &out, int64_t *n_ids) {
    SPK_REQUIRE(col >= 0 && col < (int)t.cols.size() && t.cols[col] && t.cols[col]->kind == COL_STR &&
                    t.cols[col]->n_ids >= 0,
                SPK_E_STATE, "tf: the column carries no device dictionary ids (spk_table_add_raw_utf8)");
    *n_ids = t.cols[col]->n_ids;
    SPK_TRY(out.alloc((size_t)t.n + 1));
    if (t.n) k_ids_from_meta<<<(unsigned)((t.n + 255) / 256), 256, 0, ctx->stream>>>(t.n, t.cols[col]->meta.p, out.p);
    SPK_HIP(hipGetLastError());
    return SPK_OK;
}


}  // namespace spk

using namespace spk;

extern "C" int spk_tf_limbs_to_sum(int64_t n_values, const int64_t *limbs, const int32_t *scale, double *out_sum) {
    SPK_REQUIRE(n_values >= 0 && (n_values == 0 || (limbs && scale && out_sum)), SPK_E_INVALID,
                "spk_tf_limbs_to_sum: bad args");
    for (int64_t v = 0; v < n_values; ++v) {
        int64_t l[TF_LIMBS];
        for (int j = 0; j < TF_LIMBS; ++j) l[j] = limbs[v * TF_LIMBS + j];
        for (int j = TF_LIMBS - 1; j > 0; --j) {  // carries: every fraction limb back below 2^20
            l[j - 1] += l[j] >> TF_BITS;
            l[j] &= (1 << TF_BITS) - 1;
        }
        double acc = 0.0;
        for (int j = TF_LIMBS - 1; j > 0; --j) acc = (acc + (double)l[j]) * std::ldexp(1.0, -TF_BITS);
        acc += (double)l[0];
        out_sum[v] = scale[v] == TF_NO_SCALE ? 0.0 : std::ldexp(acc, scale[v]);
    }
    return SPK_OK;
}

// Value ids per row of both sides on the device: host arrays (ids_side0 / 1) or the column's dictionary ids.
struct TfIds {
    DevBuf<int64_t> d0, d1;
    const int64_t *p0 = nullptr, *p1 = nullptr;
};
static int tf_host_ids(spk_ctx *ctx, const int64_t *ids_side0, const int64_t *ids_side1, TfIds &I) {
    Table &t0 = ctx->table[0], &t1 = ctx->side_table(1);
    SPK_TRY(I.d0.alloc((size_t)t0.n + 1));
    SPK_TRY(I.d1.alloc((size_t)t1.n + 1));
    if (t0.n) SPK_HIP(hipMemcpyAsync(I.d0.p, ids_side0, (size_t)t0.n * 8, hipMemcpyHostToDevice, ctx->stream));
    if (t1.n) SPK_HIP(hipMemcpyAsync(I.d1.p, ids_side1, (size_t)t1.n * 8, hipMemcpyHostToDevice, ctx->stream));
    I.p0 = I.d0.p;
    I.p1 = I.d1.p;
    return SPK_OK;
}
static int tf_column_ids(spk_ctx *ctx, int col, int64_t n_values, TfIds &I) {
    Table &t0 = ctx->table[0], &t1 = ctx->side_table(1);
    int64_t n0 = 0, n1 = 0;
    SPK_TRY(column_ids(ctx, t0, col, I.d0, &n0));
    if (&t1 != &t0) SPK_TRY(column_ids(ctx, t1, col, I.d1, &n1));
    SPK_REQUIRE(n_values == n0, SPK_E_INVALID, "tf: n_values is not the column's value count");
    I.p0 = I.d0.p;
    I.p1 = &t1 != &t0 ? I.d1.p : I.d0.p;
    return SPK_OK;
}
// What the runs of a device-id tf column depend on (tf_pass's cache key).
static std::vector<int64_t> tf_column_key(spk_ctx *ctx, int col, int64_t n_values) {
    return {(int64_t)ctx->pairs_epoch, (int64_t)ctx->gamma_seq, (int64_t)ctx->score_seq,
            (int64_t)ctx->table[0].version, (int64_t)ctx->side_table(1).version, col, n_values};
}
static int tf_ready(spk_ctx *ctx, const char *what) {
    SPK_REQUIRE(ctx->pairs_valid && ctx->codes_valid, SPK_E_STATE, std::string(what) + ": run spk_score first");
    SPK_HIP(hipSetDevice(ctx->device));
    return settle_gammas(ctx, nullptr);
}

extern "C" int spk_tf_scales(spk_ctx *ctx, int64_t n_values, const int64_t *ids_side0, const int64_t *ids_side1,
                             int32_t *out_scale) {
    SPK_REQUIRE(ctx && ids_side0 && ids_side1 && n_values >= 0 && (n_values == 0 || out_scale), SPK_E_INVALID,
                "spk_tf_scales: bad args");
    SPK_TRY(tf_ready(ctx, "spk_tf_scales"));
    TfIds I;
    SPK_TRY(tf_host_ids(ctx, ids_side0, ids_side1, I));
    return tf_scales(ctx, n_values, I.p0, I.p1, out_scale);
}

extern "C" int spk_tf_scales_column(spk_ctx *ctx, int col, int64_t n_values, int32_t *out_scale) {
    SPK_REQUIRE(ctx && n_values >= 0 && (n_values == 0 || out_scale), SPK_E_INVALID, "spk_tf_scales_column: bad args");
    SPK_TRY(tf_ready(ctx, "spk_tf_scales_column"));
    TfIds I;
    SPK_TRY(tf_column_ids(ctx, col, n_values, I));
    const std::vector<int64_t> key = tf_column_key(ctx, col, n_values);
    return tf_scales(ctx, n_values, I.p0, I.p1, out_scale, &key);
}

extern "C" int spk_tf_accumulate_exact(spk_ctx *ctx, int64_t n_values, const int64_t *ids_side0, const int64_t *ids_side1,
                                       const int32_t *scale, int64_t *out_limbs, int64_t *out_count) {
    SPK_REQUIRE(ctx && ids_side0 && ids_side1 && (n_values == 0 || (scale && out_limbs && out_count)) && n_values >= 0,
                SPK_E_INVALID, "spk_tf_accumulate_exact: bad args");
    SPK_TRY(tf_ready(ctx, "spk_tf_accumulate_exact"));
    TfIds I;
    SPK_TRY(tf_host_ids(ctx, ids_side0, ids_side1, I));
    return tf_exact(ctx, n_values, I.p0, I.p1, scale, out_limbs, out_count);
}

extern "C" int spk_tf_accumulate_column_exact(spk_ctx *ctx, int col, int64_t n_values, const int32_t *scale,
                                              int64_t *out_limbs, int64_t *out_count) {
    SPK_REQUIRE(ctx && n_values >= 0 && (n_values == 0 || (scale && out_limbs && out_count)), SPK_E_INVALID,
                "spk_tf_accumulate_column_exact: bad args");
    SPK_TRY(tf_ready(ctx, "spk_tf_accumulate_column_exact"));
    TfIds I;
    SPK_TRY(tf_column_ids(ctx, col, n_values, I));
    const std::vector<int64_t> key = tf_column_key(ctx, col, n_values);
    return tf_exact(ctx, n_values, I.p0, I.p1, scale, out_limbs, out_count, &key);
}

// The double forms: the exact sums of this context's pairs at its own scales, converted (the values the
// exact forms give after a one-rank all-reduce).
extern "C" int spk_tf_accumulate(spk_ctx *ctx, int64_t n_values, const int64_t *ids_side0, const int64_t *ids_side1,
                                 double *out_sum, int64_t *out_count) {
    SPK_REQUIRE(n_values >= 0 && (n_values == 0 || (out_sum && out_count)), SPK_E_INVALID, "spk_tf_accumulate: bad args");
    std::vector<int32_t> scale((size_t)n_values + 1);
    std::vector<int64_t> limbs((size_t)n_values * TF_LIMBS + 1);
    SPK_TRY(spk_tf_scales(ctx, n_values, ids_side0, ids_side1, scale.data()));
    SPK_TRY(spk_tf_accumulate_exact(ctx, n_values, ids_side0, ids_side1, scale.data(), limbs.data(), out_count));
    return spk_tf_limbs_to_sum(n_values, limbs.data(), scale.data(), out_sum);
}

extern "C" int spk_tf_accumulate_column(spk_ctx *ctx, int col, int64_t n_values, double *out_sum, int64_t *out_count) {
    SPK_REQUIRE(n_values >= 0 && (n_values == 0 || (out_sum && out_count)), SPK_E_INVALID,
                "spk_tf_accumulate_column: bad args");
    std::vector<int32_t> scale((size_t)n_values + 1);
    std::vector<int64_t> limbs((size_t)n_values * TF_LIMBS + 1);
    SPK_TRY(spk_tf_scales_column(ctx, col, n_values, scale.data()));
    SPK_TRY(spk_tf_accumulate_column_exact(ctx, col, n_values, scale.data(), limbs.data(), out_count));
    return spk_tf_limbs_to_sum(n_values, limbs.data(), scale.data(), out_sum);
}

extern "C" int spk_tf_column_values(spk_ctx *ctx, int col, int64_t *out_n_values) {
    SPK_REQUIRE(ctx && out_n_values, SPK_E_INVALID, "spk_tf_column_values: null arg");
    Table &t = ctx->table[0];
    SPK_REQUIRE(col >= 0 && col < (int)t.cols.size() && t.cols[col] && t.cols[col]->kind == COL_STR &&
                    t.cols[col]->n_ids >= 0,
                SPK_E_STATE, "spk_tf_column_values: the column carries no device dictionary ids");
    *out_n_values = t.cols[col]->n_ids;
    return SPK_OK;
}

static int tf_apply_dev(spk_ctx *ctx, TfApply &T, const double *const *adj_tables, const int64_t *table_sizes,
                        int64_t start, int64_t count, double *out_tf_mp, double *out_adj) {
    DevBuf<double> dt[8], dout, dadj;
    for (int c = 0; c < T.n; ++c) {
        SPK_TRY(dt[c].alloc((size_t)table_sizes[c] + 1));
        if (table_sizes[c])
            SPK_HIP(hipMemcpyAsync(dt[c].p, adj_tables[c], (size_t)table_sizes[c] * 8, hipMemcpyHostToDevice,
                                   ctx->stream));
        T.tab[c] = dt[c].p;
        T.tab_n[c] = table_sizes[c];
    }
    // out_tf_mp = NULL: the results stay on the device (ctx->tf_mp, read by range with spk_tf_copy), as spk_score
    // keeps mp there -- at cfg3's 3.08e9 pairs the host copy alone (24.6 GB into pageable memory) took ~5.8 s of
    // the 6.1 s tf stage (profiles/r6_fulljob_cfg3_10Mx10M_1gpu.json)
    const bool dev_out = out_tf_mp == nullptr;
    ctx->tf_count = -1;
    double *res = nullptr;
    if (dev_out) {
        SPK_TRY(ctx->tf_mp.alloc((size_t)count + 1));
        res = ctx->tf_mp.p;
    } else {
        SPK_TRY(dout.alloc((size_t)count + 1));
        res = dout.p;
    }
    if (out_adj) SPK_TRY(dadj.alloc((size_t)count * T.n + 1));
    if (count)
        k_tf_apply<<<(unsigned)((count + 255) / 256), 256, 0, ctx->stream>>>(T, start, count, ctx->pl.p, ctx->pr.p,
                                                                         ctx->mp.p, res, out_adj ? dadj.p : nullptr);
    SPK_HIP(hipGetLastError());
    if (count) {
        if (!dev_out) SPK_HIP(hipMemcpyAsync(out_tf_mp, dout.p, (size_t)count * 8, hipMemcpyDeviceToHost, ctx->stream));
        if (out_adj)
            SPK_HIP(hipMemcpyAsync(out_adj, dadj.p, (size_t)count * T.n * 8, hipMemcpyDeviceToHost, ctx->stream));
    }
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    if (dev_out) {
        ctx->tf_start = start;
        ctx->tf_count = count;
        ctx->tf_epoch = ctx->pairs_epoch;
    }
    return SPK_OK;
}

extern "C" int spk_tf_set_mode(spk_ctx *ctx, int mode) {
    SPK_REQUIRE(ctx && mode >= 0 && mode <= 2, SPK_E_INVALID, "spk_tf_set_mode: mode 0 (auto), 1 (sort) or 2 (sort, 64-bit keys)");
    ctx->tf_mode = mode;
    ctx->tf_key.clear();
    ctx->tf_hist.release();
    ctx->tf_uniq.release();
    ctx->tf_runs.release();
    return SPK_OK;
}

extern "C" int spk_tf_copy(spk_ctx *ctx, int64_t start, int64_t count, double *out_tf_mp) {
    SPK_REQUIRE(ctx && count >= 0 && (count == 0 || out_tf_mp), SPK_E_INVALID, "spk_tf_copy: bad args");
    SPK_REQUIRE(ctx->tf_count >= 0 && ctx->tf_epoch == ctx->pairs_epoch, SPK_E_STATE,
                "spk_tf_copy: no device-resident tf results for this pair set (spk_tf_apply* with out_tf_mp = NULL)");
    SPK_REQUIRE(start >= ctx->tf_start && start + count <= ctx->tf_start + ctx->tf_count, SPK_E_INVALID,
                "spk_tf_copy: range outside the applied pairs");
    SPK_HIP(hipSetDevice(ctx->device));
    if (count)
        SPK_HIP(hipMemcpyAsync(out_tf_mp, ctx->tf_mp.p + (start - ctx->tf_start), (size_t)count * 8,
                               hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    return SPK_OK;
}

extern "C" int spk_tf_apply_columns(spk_ctx *ctx, int n_tf_cols, const int32_t *cols, const double *const *adj_tables,
                                    const int64_t *table_sizes, int64_t start, int64_t count, double *out_tf_mp,
                                    double *out_adj) {
    SPK_REQUIRE(ctx && cols && n_tf_cols >= 1 && n_tf_cols <= 8, SPK_E_INVALID, "spk_tf_apply_columns: 1..8 columns");
    SPK_REQUIRE(ctx->pairs_valid && ctx->mp.p, SPK_E_STATE, "spk_tf_apply_columns: run spk_score first");
    SPK_REQUIRE(start >= 0 && count >= 0 && start + count <= ctx->n_pairs, SPK_E_INVALID, "spk_tf_apply_columns: range");
    SPK_HIP(hipSetDevice(ctx->device));
    SPK_TRY(settle_gammas(ctx, nullptr));
    Table &t0 = ctx->table[0], &t1 = ctx->side_table(1);
    DevBuf<int64_t> d0[8], d1[8];
    TfApply T{};
    T.n = n_tf_cols;
    for (int c = 0; c < n_tf_cols; ++c) {
        int64_t n0 = 0, n1 = 0;
        SPK_TRY(column_ids(ctx, t0, cols[c], d0[c], &n0));
        if (&t1 != &t0) SPK_TRY(column_ids(ctx, t1, cols[c], d1[c], &n1));
        T.ids0[c] = d0[c].p;
        T.ids1[c] = &t1 != &t0 ? d1[c].p : d0[c].p;
    }
    return tf_apply_dev(ctx, T, adj_tables, table_sizes, start, count, out_tf_mp, out_adj);
}

extern "C" int spk_tf_apply(spk_ctx *ctx, int n_tf_cols, const int64_t *const *ids_side0,
                            const int64_t *const *ids_side1, const double *const *adj_tables,
                            const int64_t *table_sizes, int64_t start, int64_t count, double *out_tf_mp,
                            double *out_adj) {
    SPK_REQUIRE(ctx && n_tf_cols >= 1 && n_tf_cols <= 8, SPK_E_INVALID, "spk_tf_apply: 1..8 columns");
    SPK_REQUIRE(ctx->pairs_valid && ctx->mp.p, SPK_E_STATE, "spk_tf_apply: run spk_score first");
    SPK_REQUIRE(start >= 0 && count >= 0 && start + count <= ctx->n_pairs, SPK_E_INVALID, "spk_tf_apply: range");
    SPK_HIP(hipSetDevice(ctx->device));
    SPK_TRY(settle_gammas(ctx, nullptr));
    Table &t0 = ctx->table[0], &t1 = ctx->side_table(1);
    DevBuf<int64_t> d0[8], d1[8];
    TfApply T{};
    T.n = n_tf_cols;
    for (int c = 0; c < n_tf_cols; ++c) {
        SPK_TRY(d0[c].alloc((size_t)t0.n + 1));
        SPK_TRY(d1[c].alloc((size_t)t1.n + 1));
        SPK_HIP(hipMemcpyAsync(d0[c].p, ids_side0[c], (size_t)t0.n * 8, hipMemcpyHostToDevice, ctx->stream));
        SPK_HIP(hipMemcpyAsync(d1[c].p, ids_side1[c], (size_t)t1.n * 8, hipMemcpyHostToDevice, ctx->stream));
        T.ids0[c] = d0[c].p;
        T.ids1[c] = d1[c].p;
    }
    return tf_apply_dev(ctx, T, adj_tables, table_sizes, start, count, out_tf_mp, out_adj);
}
