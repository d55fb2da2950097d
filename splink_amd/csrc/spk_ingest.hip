// Device ingest: the per-row preparation in front of the blocking joins (blocking.py:95-160) and the
// comparison columns (gammas.py:65-89), done on the GPU from the input columns' Arrow buffers.
//
// The input columns go to the device once, in input row order ("raw" columns, spk_raw_*).  Then:
//   * blocking keys (spk_key_build): a 64-bit hash of every value -- after an optional Spark
//     substr on code points -- a radix sort of (hash, row), and dense ids from the heads of equal-hash
//     runs.  Every row of a run is compared byte for byte with its predecessor, so equal ids mean
//     equal values; a hash collision (unequal values in one run) re-hashes with another seed.  The
//     l- and r-side values of a term share one id space; multi-term rules combine the terms' ids
//     (NULL if any term is NULL, `ifnull(rule, false)` of blocking.py:59-68) with a second sort.
//   * unique-id ranks for the link predicate (spk_rank_from_raw, int64 ids): sort + dense rank.
//   * the clustering of the tables by the first rule's key, then rank (spk_cluster): the keys and
//     ranks are permuted, and every comparison column is later decoded through the permutation.
//   * comparison columns (spk_table_add_raw_utf8): UTF-8 -> UTF-16 decode through the permutation,
//     with dictionary ids computed like the keys (string equality = one integer compare).
// Every kernel here is a streaming pass or a gather over the rows; the sorts are rocPRIM radix sorts.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstring>

#include "spk_internal.h"

namespace spk {

// One side of a hashed id space: a raw column with an optional substr(start, len) (Spark rules).
struct HashSeg {
    const int64_t *off;
    const uint8_t *bytes;
    const int64_t *i64;
    const uint8_t *valid;
    int64_t n;
    int32_t kind;
    int32_t substr_start;
    int32_t substr_len;    // < 0: no substr
    int32_t pad;
};

__device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// Byte range [*b, *e) of Spark's substringSQL(pos, len) of the UTF-8 value in [b, e) (code points).
__device__ inline void substr_range(const uint8_t *p, int64_t &b, int64_t &e, int pos, int len) {
    if (len < 0) return;  // no substr
    int64_t nc = 0;
    if (pos < 0)
        for (int64_t i = b; i < e; ++i) nc += (p[i] & 0xC0) != 0x80;
    int64_t start = pos > 0 ? pos - 1 : (pos < 0 ? nc + pos : 0);
    int64_t end = start + len;
    if (start < 0) start = 0;
    if (start >= end) {
        e = b;
        return;
    }
    int64_t c = -1, i = b, bs = e, be = e;
    for (; i < e; ++i) {
        if ((p[i] & 0xC0) != 0x80) {
            ++c;
            if (c == start) bs = i;
            if (c == end) {
                be = i;
                break;
            }
        }
    }
    b = bs;
    e = bs < be ? be : bs;
}

__device__ inline void seg_range(const HashSeg &s, int64_t row, int64_t &b, int64_t &e) {
    b = s.off[row];
    e = s.off[row + 1];
    substr_range(s.bytes, b, e, s.substr_start, s.substr_len);
}

__device__ inline uint64_t hash_bytes(const uint8_t *p, int64_t n, uint64_t seed) {
    uint64_t h = mix64(seed ^ ((uint64_t)n * 0x9E3779B97F4A7C15ull));
    int64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) w |= (uint64_t)p[i + k] << (8 * k);
        h = mix64(h ^ w) + 0x9E3779B97F4A7C15ull;
    }
    uint64_t w = 0;
    for (int k = 0; i + k < n; ++k) w |= (uint64_t)p[i + k] << (8 * k);
    return mix64(h ^ w ^ 0x632BE59BD9B4E019ull);
}

// keys[i] = 63-bit hash of global row i (rows [0, s0.n) of s0, then s1), ~0 for NULL; idx[i] = i.
__global__ void k_hash(HashSeg s0, HashSeg s1, uint64_t seed, uint64_t *__restrict__ keys,
                       int32_t *__restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s0.n + s1.n) return;
    const bool first = i < s0.n;
    const HashSeg &s = first ? s0 : s1;
    const int64_t row = first ? i : i - s0.n;
    uint64_t k = ~0ull;
    if (s.valid[row]) {
        if (s.kind == RAW_I64) {
            k = mix64((uint64_t)s.i64[row] ^ seed) >> 1;
        } else {
            int64_t b, e;
            seg_range(s, row, b, e);
            k = hash_bytes(s.bytes + b, e - b, seed) >> 1;
        }
    }
    keys[i] = k;
    idx[i] = (int32_t)i;
}

__device__ inline bool same_value(const HashSeg &s0, const HashSeg &s1, int64_t i, int64_t j) {
    const HashSeg &a = i < s0.n ? s0 : s1, &b = j < s0.n ? s0 : s1;
    const int64_t ri = i < s0.n ? i : i - s0.n, rj = j < s0.n ? j : j - s0.n;
    if (a.kind == RAW_I64 || b.kind == RAW_I64) return a.kind == b.kind && a.i64[ri] == b.i64[rj];
    int64_t ab, ae, bb, be;
    seg_range(a, ri, ab, ae);
    seg_range(b, rj, bb, be);
    if (ae - ab != be - bb) return false;
    for (int64_t k = 0; k < ae - ab; ++k)
        if (a.bytes[ab + k] != b.bytes[bb + k]) return false;
    return true;
}

// Run heads of the sorted keys; with `verify`, every row of a run is compared with its predecessor
// (a mismatch is a hash collision: *collision = 1).
__global__ void k_heads_verify(int64_t n, const uint64_t *__restrict__ keys, const int32_t *__restrict__ idx,
                               HashSeg s0, HashSeg s1, int verify, int64_t *__restrict__ heads,
                               unsigned int *__restrict__ collision) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool head = i == 0 || keys[i] != keys[i - 1];
    heads[i] = head ? 1 : 0;
    if (verify && !head && keys[i] != ~0ull && !same_value(s0, s1, idx[i], idx[i - 1])) atomicOr(collision, 1u);
}

// ids[idx[i]] = run number of sorted row i (0-based), -1 for NULL rows (key ~0 and, for exact keys,
// a NULL flag: an exact key may legitimately equal ~0).
__global__ void k_scatter_ids(int64_t n, const uint64_t *__restrict__ keys, const int32_t *__restrict__ idx,
                              const int64_t *__restrict__ incl, const uint8_t *__restrict__ null_flag,
                              int64_t *__restrict__ ids) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t r = idx[i];
    const bool nul = null_flag ? null_flag[r] != 0 : keys[i] == ~0ull;
    ids[r] = nul ? -1 : incl[i] - 1;
}

// Two per-row ids -> one packed exact key (NULL if either is NULL).
__global__ void k_pack_ids(int64_t n, const int64_t *__restrict__ a, const int64_t *__restrict__ b,
                           uint64_t *__restrict__ keys, int32_t *__restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = (a[i] < 0 || b[i] < 0) ? ~0ull : (((uint64_t)a[i] << 32) | (uint64_t)b[i]);
    idx[i] = (int32_t)i;
}

// Order-preserving keys of int64 values (unique-id ranks); NULL rows get ~0 and a NULL flag.
__global__ void k_i64_keys(int64_t n, const int64_t *__restrict__ v, const uint8_t *__restrict__ valid,
                           uint64_t *__restrict__ keys, int32_t *__restrict__ idx, uint8_t *__restrict__ nul) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool ok = valid[i] != 0;
    keys[i] = ok ? ((uint64_t)v[i] ^ 0x8000000000000000ull) : ~0ull;
    idx[i] = (int32_t)i;
    nul[i] = ok ? 0 : 1;
}

// rank of table row i = input row perm[i] (perm null: identity; a table reordered by spk_cluster)
__global__ void k_rank(int64_t n, const int64_t *__restrict__ ids, const int32_t *__restrict__ perm, int64_t right_from,
                       int64_t div, int64_t *__restrict__ rank) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = perm ? perm[i] : i;
    const int64_t src = r >= right_from ? 1 : 0;
    rank[i] = src * div + (ids[r] < 0 ? div - 1 : ids[r]);
}

__global__ void k_cluster_keys(int64_t n, const int64_t *__restrict__ key, const int64_t *__restrict__ rank,
                               uint64_t *__restrict__ keys, int32_t *__restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = key[i] < 0 ? 0x7FFFFFFFull : (uint64_t)key[i];
    keys[i] = (k << 32) | (rank ? (uint64_t)rank[i] : 0ull);
    idx[i] = (int32_t)i;
}

template <typename T>
__global__ void k_gather(int64_t n, const T *__restrict__ src, const int32_t *__restrict__ perm, T *__restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dst[i] = src[perm[i]];
}

__global__ void k_perm_lengths(int64_t n, const int64_t *__restrict__ off, const int32_t *__restrict__ perm,
                               int64_t *__restrict__ len) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    if (i == n) {
        len[i] = 0;
        return;
    }
    const int64_t r = perm ? perm[i] : i;
    len[i] = off[r + 1] - off[r];
}

static unsigned grid(int64_t n) { return (unsigned)((n + 255) / 256); }

// Work buffers of one dense-id computation.
struct IdWork {
    DevBuf<uint64_t> k_in, k_out;
    DevBuf<int32_t> i_in, i_out;
    DevBuf<int64_t> heads, incl;
    DevBuf<uint8_t> tmp;
    DevBuf<unsigned int> flag;
    int alloc(int64_t n) {
        SPK_TRY(k_in.alloc((size_t)n + 1));
        SPK_TRY(k_out.alloc((size_t)n + 1));
        SPK_TRY(i_in.alloc((size_t)n + 1));
        SPK_TRY(i_out.alloc((size_t)n + 1));
        SPK_TRY(heads.alloc((size_t)n + 1));
        SPK_TRY(incl.alloc((size_t)n + 1));
        SPK_TRY(flag.alloc(1));
        return SPK_OK;
    }
};

// Sort w.k_in / w.i_in (n rows), heads (verified against s0 / s1 when verify), ids[row] (int64,
// -1 NULL).  Returns the number of runs (distinct keys, a NULL run included) and the collision flag.
static int sorted_ids(spk_ctx *ctx, int64_t n, IdWork &w, const HashSeg &s0, const HashSeg &s1, bool verify,
                      const uint8_t *null_flag, int64_t *ids, int64_t *n_runs, bool *collision) {
    *n_runs = 0;
    *collision = false;
    if (n == 0) return SPK_OK;
    size_t bytes = 0;
    SPK_HIP(rocprim::radix_sort_pairs(nullptr, bytes, w.k_in.p, w.k_out.p, w.i_in.p, w.i_out.p, (size_t)n, 0, 64,
                                      ctx->stream));
    SPK_TRY(w.tmp.alloc(bytes + 1));
    SPK_HIP(rocprim::radix_sort_pairs(w.tmp.p, bytes, w.k_in.p, w.k_out.p, w.i_in.p, w.i_out.p, (size_t)n, 0, 64,
                                      ctx->stream));
    SPK_HIP(hipMemsetAsync(w.flag.p, 0, sizeof(unsigned int), ctx->stream));
    k_heads_verify<<<grid(n), 256, 0, ctx->stream>>>(n, w.k_out.p, w.i_out.p, s0, s1, verify ? 1 : 0, w.heads.p,
                                                     w.flag.p);
    SPK_HIP(hipGetLastError());
    bytes = 0;
    SPK_HIP(rocprim::inclusive_scan(nullptr, bytes, w.heads.p, w.incl.p, (size_t)n, rocprim::plus<int64_t>(),
                                    ctx->stream));
    SPK_TRY(w.tmp.alloc(bytes + 1));
    SPK_HIP(rocprim::inclusive_scan(w.tmp.p, bytes, w.heads.p, w.incl.p, (size_t)n, rocprim::plus<int64_t>(),
                                    ctx->stream));
    k_scatter_ids<<<grid(n), 256, 0, ctx->stream>>>(n, w.k_out.p, w.i_out.p, w.incl.p, null_flag, ids);
    SPK_HIP(hipGetLastError());
    int64_t runs = 0;
    unsigned int coll = 0;
    SPK_HIP(hipMemcpyAsync(&runs, w.incl.p + n - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipMemcpyAsync(&coll, w.flag.p, 4, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    *n_runs = runs;
    *collision = coll != 0;
    return SPK_OK;
}

// Dense ids of the values of s0 then s1 (one id space), by hash + sort + verified run heads.
static int hashed_ids(spk_ctx *ctx, const HashSeg &s0, const HashSeg &s1, DevBuf<int64_t> &ids, int64_t *n_ids) {
    const int64_t n = s0.n + s1.n;
    SPK_TRY(ids.alloc((size_t)n + 1));
    IdWork w;
    SPK_TRY(w.alloc(n));
    static const uint64_t seeds[4] = {0x243F6A8885A308D3ull, 0x13198A2E03707344ull, 0xA4093822299F31D0ull,
                                      0x082EFA98EC4E6C89ull};
    for (int attempt = 0; attempt < 4; ++attempt) {
        if (n > 0) {
            k_hash<<<grid(n), 256, 0, ctx->stream>>>(s0, s1, seeds[attempt], w.k_in.p, w.i_in.p);
            SPK_HIP(hipGetLastError());
        }
        bool coll = false;
        SPK_TRY(sorted_ids(ctx, n, w, s0, s1, true, nullptr, ids.p, n_ids, &coll));
        if (!coll) return SPK_OK;
    }
    set_error("device ingest: 64-bit hash collisions under four seeds");
    return SPK_E_STATE;
}

static int seg_of(spk_ctx *ctx, int raw, int64_t want_rows, int substr_start, int substr_len, HashSeg *out) {
    SPK_REQUIRE(raw >= 0 && raw < (int)ctx->raw.size() && ctx->raw[raw], SPK_E_INVALID, "unknown raw column");
    RawCol *r = ctx->raw[raw];
    SPK_REQUIRE(!r->released, SPK_E_STATE, "raw column released (spk_raw_release): upload it again");
    SPK_REQUIRE(r->n == want_rows, SPK_E_INVALID, "raw column length does not match the table");
    SPK_REQUIRE(r->kind == RAW_UTF8 || substr_len < 0, SPK_E_INVALID,
                "substr of a non-string raw column");
    HashSeg s{};
    s.off = r->off.p;
    s.bytes = r->bytes.p;
    s.i64 = r->i64.p;
    s.valid = r->valid.p;
    s.n = r->n;
    s.kind = r->kind;
    s.substr_start = substr_start;
    s.substr_len = substr_len;
    *out = s;
    return SPK_OK;
}

static int new_raw(spk_ctx *ctx, int raw, RawCol **out) {
    SPK_REQUIRE(ctx && raw >= 0 && raw < 65536, SPK_E_INVALID, "raw column index out of range");
    if (raw >= (int)ctx->raw.size()) ctx->raw.resize((size_t)raw + 1, nullptr);
    delete ctx->raw[raw];
    ctx->raw[raw] = new RawCol();
    ctx->raw[raw]->serial = ++ctx->raw_serial;
    *out = ctx->raw[raw];
    return SPK_OK;
}

// Keys come in input row order; a table already reordered by spk_cluster takes them through its
// permutation (table row i = input row perm[i]), so keys always follow the table's rows.
static int set_key(spk_ctx *ctx, Table &t, int which, int rule, const int64_t *src, int64_t n) {
    while ((int)t.key[which].size() <= rule) t.key[which].push_back(new DevBuf<int64_t>());
    SPK_TRY(t.key[which][rule]->alloc((size_t)n + 1));
    if (!n) return SPK_OK;
    if (t.perm.p) {
        k_gather<int64_t><<<grid(n), 256, 0, ctx->stream>>>(n, src, t.perm.p, t.key[which][rule]->p);
        SPK_HIP(hipGetLastError());
    } else {
        SPK_HIP(hipMemcpyAsync(t.key[which][rule]->p, src, (size_t)n * 8, hipMemcpyDeviceToDevice, ctx->stream));
    }
    return SPK_OK;
}

}  // namespace spk

using namespace spk;

// Arrow buffers as handed over: offsets rebased to 0 (sliced arrays start past 0), the validity bitmap
// (LSB first, from bit `bit0`) expanded to bytes, and the longest row / empty-string flag reduced, all on
// the device (no per-row host pass).
__global__ void k_arrow_rebase(int64_t n, int64_t *__restrict__ off, int64_t base, const uint8_t *__restrict__ bitmap,
                               int64_t bit0, uint8_t *__restrict__ valid) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) off[i] -= base;
    if (i < n) {
        const int64_t b = bit0 + i;
        valid[i] = !bitmap ? (uint8_t)1 : (bit0 < 0 ? (uint8_t)(bitmap[i] != 0) : (uint8_t)((bitmap[b >> 3] >> (b & 7)) & 1));
    }
}
__global__ void k_arrow_lengths(int64_t n, const int64_t *__restrict__ off, const uint8_t *__restrict__ valid,
                                unsigned long long *__restrict__ stats) {
    // grid-stride over the rows, then wave and workgroup reductions: one atomic per workgroup (an atomic per
    // wave on the same two words serialised at L2: 180 us per million rows)
    __shared__ unsigned long long s_len[4], s_empty[4];
    unsigned long long len = 0, empty = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long l = (unsigned long long)(off[i + 1] - off[i]);
        len = l > len ? l : len;
        empty |= (valid[i] && l == 0) ? 1ull : 0ull;
    }
    for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long a = __shfl_xor(len, o), e = __shfl_xor(empty, o);
        len = a > len ? a : len;
        empty |= e;
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_len[wv] = len;
        s_empty[wv] = empty;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < (int)(blockDim.x >> 6); ++q) {
            len = s_len[q] > len ? s_len[q] : len;
            empty |= s_empty[q];
        }
        if (len) atomicMax(&stats[0], len);
        if (empty) atomicOr(&stats[1], 1ull);
    }
}

// FNV-style 64-bit digest of a byte range, order-dependent (the replication tests compare two contexts'
// encoded tables): each thread folds its 8-byte words, then the per-thread digests are combined in
// thread order on the host.
__global__ void k_digest(const uint64_t *__restrict__ w, int64_t n_words, uint64_t *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    uint64_t h = 1469598103934665603ull ^ (uint64_t)t;
    for (int64_t i = t; i < n_words; i += T) h = (h ^ (w[i] + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1))) * 1099511628211ull;
    out[t] = h;
}

static int digest(spk_ctx *ctx, const void *p, int64_t bytes, uint64_t &acc) {
    const int64_t nw = bytes / 8;
    constexpr int G = 256, B = 256;
    DevBuf<uint64_t> d;
    SPK_TRY(d.alloc((size_t)G * B));
    k_digest<<<G, B, 0, ctx->stream>>>(reinterpret_cast<const uint64_t *>(p), nw, d.p);
    SPK_HIP(hipGetLastError());
    std::vector<uint64_t> h((size_t)G * B);
    SPK_HIP(hipMemcpyAsync(h.data(), d.p, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    std::vector<uint8_t> tail((size_t)(bytes - nw * 8));
    if (!tail.empty())
        SPK_HIP(hipMemcpyAsync(tail.data(), static_cast<const uint8_t *>(p) + nw * 8, tail.size(), hipMemcpyDeviceToHost,
                               ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    for (uint64_t x : h) acc = (acc ^ x) * 1099511628211ull;
    for (uint8_t x : tail) acc = (acc ^ x) * 1099511628211ull;
    acc = (acc ^ (uint64_t)bytes) * 1099511628211ull;
    return SPK_OK;
}

extern "C" {

int spk_raw_utf8(spk_ctx *ctx, int raw, int64_t n, const int64_t *offsets, const uint8_t *data, const uint8_t *valid) {
    SPK_REQUIRE(ctx && offsets && valid && n >= 0 && n < (int64_t)INT32_MAX, SPK_E_INVALID, "spk_raw_utf8: bad args");
    SPK_REQUIRE(offsets[0] == 0 && offsets[n] >= 0, SPK_E_INVALID, "spk_raw_utf8: offsets must start at 0");
    SPK_HIP(hipSetDevice(ctx->device));
    RawCol *r = nullptr;
    SPK_TRY(new_raw(ctx, raw, &r));
    r->kind = RAW_UTF8;
    r->n = n;
    const int64_t nbytes = offsets[n];
    int64_t mx = 0;
    bool empty = false;
    for (int64_t i = 0; i < n; ++i) {
        mx = std::max(mx, offsets[i + 1] - offsets[i]);
        empty = empty || (valid[i] && offsets[i + 1] == offsets[i]);
    }
    r->max_len = mx;
    r->has_empty = empty;
    SPK_TRY(r->off.alloc((size_t)n + 1));
    SPK_TRY(r->bytes.alloc((size_t)nbytes + 1));
    SPK_TRY(r->valid.alloc((size_t)n + 1));
    SPK_HIP(hipMemcpyAsync(r->off.p, offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    if (nbytes) SPK_HIP(hipMemcpyAsync(r->bytes.p, data, (size_t)nbytes, hipMemcpyHostToDevice, ctx->stream));
    if (n) SPK_HIP(hipMemcpyAsync(r->valid.p, valid, (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    return SPK_OK;
}

int spk_raw_utf8_arrow(spk_ctx *ctx, int raw, int64_t n, const int64_t *offsets, const uint8_t *data,
                       const uint8_t *validity, int64_t validity_bit_offset, int on_device) {
    SPK_REQUIRE(ctx && offsets && data && n >= 0 && n < (int64_t)INT32_MAX && validity_bit_offset >= -1, SPK_E_INVALID,
                "spk_raw_utf8_arrow: bad args");
    SPK_HIP(hipSetDevice(ctx->device));
    int64_t ends[2] = {0, 0};  // offsets[0], offsets[n]
    if (on_device) {
        SPK_HIP(hipMemcpyAsync(&ends[0], offsets, 8, hipMemcpyDeviceToHost, ctx->stream));
        SPK_HIP(hipMemcpyAsync(&ends[1], offsets + n, 8, hipMemcpyDeviceToHost, ctx->stream));
        SPK_HIP(hipStreamSynchronize(ctx->stream));
    } else {
        ends[0] = offsets[0];
        ends[1] = offsets[n];
    }
    SPK_REQUIRE(ends[0] >= 0 && ends[1] >= ends[0], SPK_E_INVALID, "spk_raw_utf8_arrow: offsets out of order");
    RawCol *r = nullptr;
    SPK_TRY(new_raw(ctx, raw, &r));
    r->kind = RAW_UTF8;
    r->n = n;
    const int64_t nbytes = ends[1] - ends[0];
    SPK_TRY(r->off.alloc((size_t)n + 1));
    SPK_TRY(r->bytes.alloc((size_t)nbytes + 1));
    SPK_TRY(r->valid.alloc((size_t)n + 1));
    if (on_device) {
        SPK_HIP(hipMemcpyAsync(r->off.p, offsets, (size_t)(n + 1) * 8, hipMemcpyDeviceToDevice, ctx->stream));
        if (nbytes) SPK_HIP(hipMemcpyAsync(r->bytes.p, data + ends[0], (size_t)nbytes, hipMemcpyDeviceToDevice, ctx->stream));
    } else {
        SPK_HIP(hipMemcpyAsync(r->off.p, offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        if (nbytes) SPK_HIP(hipMemcpyAsync(r->bytes.p, data + ends[0], (size_t)nbytes, hipMemcpyHostToDevice, ctx->stream));
    }
    DevBuf<uint8_t> bm;
    const uint8_t *d_bm = nullptr;
    if (validity && n) {
        const int64_t nb = validity_bit_offset < 0 ? n : (validity_bit_offset + n + 7) / 8;
        if (on_device) {
            d_bm = validity;
        } else {
            SPK_TRY(bm.alloc((size_t)nb));
            SPK_HIP(hipMemcpyAsync(bm.p, validity, (size_t)nb, hipMemcpyHostToDevice, ctx->stream));
            d_bm = bm.p;
        }
    }
    DevBuf<unsigned long long> st;
    SPK_TRY(st.alloc(2));
    SPK_HIP(hipMemsetAsync(st.p, 0, 16, ctx->stream));
    k_arrow_rebase<<<grid(n + 1), 256, 0, ctx->stream>>>(n, r->off.p, ends[0], d_bm, validity_bit_offset, r->valid.p);
    if (n)
        k_arrow_lengths<<<(unsigned)std::min<int64_t>(grid(n), 4 * (int64_t)ctx->n_cu), 256, 0, ctx->stream>>>(
            n, r->off.p, r->valid.p, st.p);
    SPK_HIP(hipGetLastError());
    unsigned long long h[2] = {0, 0};
    SPK_HIP(hipMemcpyAsync(h, st.p, 16, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    r->max_len = (int64_t)h[0];
    r->has_empty = h[1] != 0;
    return SPK_OK;
}

int spk_raw_utf8_arrow_chunks(spk_ctx *ctx, int raw, int n_chunks, const int64_t *rows, const int64_t *const *offsets,
                              const uint8_t *const *data, const uint8_t *const *validity, const int64_t *bit_offsets) {
    SPK_REQUIRE(ctx && n_chunks >= 1 && rows && offsets && data && validity && bit_offsets, SPK_E_INVALID,
                "spk_raw_utf8_arrow_chunks: bad args");
    int64_t n = 0, nbytes = 0;
    for (int c = 0; c < n_chunks; ++c) {
        SPK_REQUIRE(rows[c] >= 0 && offsets[c] && data[c] && bit_offsets[c] >= -1, SPK_E_INVALID,
                    "spk_raw_utf8_arrow_chunks: bad chunk");
        SPK_REQUIRE(offsets[c][0] >= 0 && offsets[c][rows[c]] >= offsets[c][0], SPK_E_INVALID,
                    "spk_raw_utf8_arrow_chunks: offsets out of order");
        n += rows[c];
        nbytes += offsets[c][rows[c]] - offsets[c][0];
    }
    SPK_REQUIRE(n < (int64_t)INT32_MAX, SPK_E_LIMIT, "spk_raw_utf8_arrow_chunks: more than 2^31-1 rows");
    SPK_HIP(hipSetDevice(ctx->device));
    RawCol *r = nullptr;
    SPK_TRY(new_raw(ctx, raw, &r));
    r->kind = RAW_UTF8;
    r->n = n;
    SPK_TRY(r->off.alloc((size_t)n + 1));
    SPK_TRY(r->bytes.alloc((size_t)nbytes + 1));
    SPK_TRY(r->valid.alloc((size_t)n + 1));
    // chunk c's rows go to [row0, row0 + rows[c]) and its bytes to [byte0, ...): its offsets are copied as
    // they are and rebased on the device by (first offset - byte0); the next chunk's copy overwrites the
    // shared end offset with the same value
    std::vector<DevBuf<uint8_t>> bms((size_t)n_chunks);
    int64_t row0 = 0, byte0 = 0;
    for (int c = 0; c < n_chunks; ++c) {
        const int64_t m = rows[c], first = offsets[c][0], len = offsets[c][m] - first;
        SPK_HIP(hipMemcpyAsync(r->off.p + row0, offsets[c], (size_t)(m + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        if (len) SPK_HIP(hipMemcpyAsync(r->bytes.p + byte0, data[c] + first, (size_t)len, hipMemcpyHostToDevice, ctx->stream));
        const uint8_t *d_bm = nullptr;
        if (validity[c] && m) {
            const int64_t nb = bit_offsets[c] < 0 ? m : (bit_offsets[c] + m + 7) / 8;
            SPK_TRY(bms[c].alloc((size_t)nb));
            SPK_HIP(hipMemcpyAsync(bms[c].p, validity[c], (size_t)nb, hipMemcpyHostToDevice, ctx->stream));
            d_bm = bms[c].p;
        }
        k_arrow_rebase<<<grid(m + 1), 256, 0, ctx->stream>>>(m, r->off.p + row0, first - byte0, d_bm, bit_offsets[c],
                                                            r->valid.p + row0);
        SPK_HIP(hipGetLastError());
        row0 += m;
        byte0 += len;
    }
    DevBuf<unsigned long long> st;
    SPK_TRY(st.alloc(2));
    SPK_HIP(hipMemsetAsync(st.p, 0, 16, ctx->stream));
    if (n)
        k_arrow_lengths<<<(unsigned)std::min<int64_t>(grid(n), 4 * (int64_t)ctx->n_cu), 256, 0, ctx->stream>>>(
            n, r->off.p, r->valid.p, st.p);
    SPK_HIP(hipGetLastError());
    unsigned long long h[2] = {0, 0};
    SPK_HIP(hipMemcpyAsync(h, st.p, 16, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    r->max_len = (int64_t)h[0];
    r->has_empty = h[1] != 0;
    return SPK_OK;
}

int spk_table_digest(spk_ctx *ctx, int side, uint64_t *out) {
    SPK_REQUIRE(ctx && out && (side == 0 || side == 1), SPK_E_INVALID, "spk_table_digest: bad args");
    SPK_HIP(hipSetDevice(ctx->device));
    Table &t = ctx->table[side];
    SPK_REQUIRE(t.n >= 0, SPK_E_STATE, "spk_table_digest: table not created");
    uint64_t acc = 1469598103934665603ull ^ (uint64_t)t.n;
    if (t.perm.p) SPK_TRY(digest(ctx, t.perm.p, t.n * 4, acc));
    if (t.rank.p) SPK_TRY(digest(ctx, t.rank.p, t.n * 8, acc));
    for (const Column *c : t.cols) {
        if (!c || c->kind == COL_NONE) continue;
        acc = (acc ^ (uint64_t)c->kind) * 1099511628211ull;
        if (c->kind == COL_STR) {
            // units: the zeroed extent the last decode wrote (a reused buffer's capacity past it is not part of
            // the encoding)
            SPK_TRY(digest(ctx, c->meta.p, t.n * (int64_t)sizeof(RecMeta), acc));
            SPK_TRY(digest(ctx, c->units.p, c->units_len * 2, acc));
            if (c->planes.p) SPK_TRY(digest(ctx, c->planes.p, t.n * N_PLANES * 8, acc));
            if (c->planes_hi.p) SPK_TRY(digest(ctx, c->planes_hi.p, t.n * N_PLANES * 8, acc));
            acc = (acc ^ (uint64_t)c->n_ids) * 1099511628211ull;
        } else {
            SPK_TRY(digest(ctx, c->val.p, t.n * 8, acc));
            SPK_TRY(digest(ctx, c->valid.p, t.n, acc));
        }
    }
    for (int w = 0; w < 2; ++w)
        for (size_t r = 0; r < t.key[w].size(); ++r)
            if (t.key[w][r] && t.key[w][r]->p) SPK_TRY(digest(ctx, t.key[w][r]->p, t.n * 8, acc));
    *out = acc;
    return SPK_OK;
}

// Free a raw column's device buffers once everything derived from it exists (keys, decoded comparison
// columns): its serial stays, so the blocking-key / column provenance checks still see it.
int spk_raw_release(spk_ctx *ctx, int raw) {
    SPK_REQUIRE(ctx && raw >= 0 && raw < (int)ctx->raw.size() && ctx->raw[raw], SPK_E_INVALID,
                "spk_raw_release: unknown raw column");
    SPK_HIP(hipSetDevice(ctx->device));
    SPK_HIP(hipStreamSynchronize(ctx->stream));  // no queued kernel reads it any more
    RawCol *r = ctx->raw[raw];
    r->off.release();
    r->bytes.release();
    r->i64.release();
    r->valid.release();
    r->released = true;
    return SPK_OK;
}

int spk_raw_i64(spk_ctx *ctx, int raw, int64_t n, const int64_t *values, const uint8_t *valid) {
    SPK_REQUIRE(ctx && values && valid && n >= 0 && n < (int64_t)INT32_MAX, SPK_E_INVALID, "spk_raw_i64: bad args");
    SPK_HIP(hipSetDevice(ctx->device));
    RawCol *r = nullptr;
    SPK_TRY(new_raw(ctx, raw, &r));
    r->kind = RAW_I64;
    r->n = n;
    SPK_TRY(r->i64.alloc((size_t)n + 1));
    SPK_TRY(r->valid.alloc((size_t)n + 1));
    if (n) {
        SPK_HIP(hipMemcpyAsync(r->i64.p, values, (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream));
        SPK_HIP(hipMemcpyAsync(r->valid.p, valid, (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    }
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    return SPK_OK;
}

int spk_key_build(spk_ctx *ctx, int rule, int n_terms, const spk_key_term *terms) {
    SPK_REQUIRE(ctx && terms && n_terms >= 1 && rule >= 0 && rule < 32, SPK_E_INVALID, "spk_key_build: bad args");
    SPK_HIP(hipSetDevice(ctx->device));
    Table &t0 = ctx->table[0];
    Table &tr = ctx->side_table(1);
    SPK_REQUIRE(t0.n >= 0 && tr.n >= 0, SPK_E_STATE, "spk_key_build: tables not created");
    const int64_t n0 = t0.n, n1 = tr.n;
    const bool any_r = [&] {
        for (int i = 0; i < n_terms; ++i)
            if (terms[i].raw_r >= 0) return true;
        return false;
    }();
    const int64_t N = n0 + (any_r ? n1 : 0);
    // k_hash / k_pack_ids / sorted_ids hold the global row (both sides) in an int32
    SPK_REQUIRE(N < (int64_t)INT32_MAX, SPK_E_LIMIT, "spk_key_build: more than 2^31-1 rows over both tables");
    DevBuf<int64_t> acc, cur;
    int64_t n_ids = 0;
    for (int i = 0; i < n_terms; ++i) {
        const spk_key_term &tm = terms[i];
        HashSeg s0{}, s1{};
        SPK_TRY(seg_of(ctx, tm.raw_l, n0, tm.l_substr_start, tm.l_substr_len, &s0));
        if (any_r) {
            // every term has an r side when one has: a symmetric term repeats its l-side column
            SPK_TRY(seg_of(ctx, tm.raw_r >= 0 ? tm.raw_r : tm.raw_l, n1, tm.raw_r >= 0 ? tm.r_substr_start : tm.l_substr_start,
                           tm.raw_r >= 0 ? tm.r_substr_len : tm.l_substr_len, &s1));
        }
        SPK_TRY(hashed_ids(ctx, s0, s1, i == 0 ? acc : cur, &n_ids));
        if (i > 0 && N > 0) {  // combine with the terms so far
            IdWork w;
            SPK_TRY(w.alloc(N));
            k_pack_ids<<<grid(N), 256, 0, ctx->stream>>>(N, acc.p, cur.p, w.k_in.p, w.i_in.p);
            SPK_HIP(hipGetLastError());
            bool coll = false;
            HashSeg none{};
            SPK_TRY(sorted_ids(ctx, N, w, none, none, false, nullptr, acc.p, &n_ids, &coll));
        }
    }
    SPK_REQUIRE(n_ids < (int64_t)INT32_MAX, SPK_E_LIMIT, "spk_key_build: more than 2^31 distinct keys");
    SPK_TRY(set_key(ctx, t0, 0, rule, acc.p, n0));
    SPK_TRY(set_key(ctx, tr, 1, rule, any_r ? acc.p + n0 : acc.p, n1));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    std::vector<KeyTerm> rec;
    for (int i = 0; i < n_terms; ++i) {
        const spk_key_term &tm = terms[i];
        const int rr = tm.raw_r >= 0 ? tm.raw_r : tm.raw_l;
        KeyTerm k;
        k.src_l = ctx->raw[tm.raw_l]->serial;
        k.src_r = ctx->raw[rr]->serial;
        k.plain = tm.l_substr_len < 0 && (tm.raw_r >= 0 ? tm.r_substr_len : tm.l_substr_len) < 0;
        rec.push_back(k);
    }
    ctx->rule_terms[rule] = rec;
    return SPK_OK;
}

int spk_rank_from_raw(spk_ctx *ctx, int raw_uid, int64_t right_from) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    SPK_HIP(hipSetDevice(ctx->device));
    Table &t = ctx->table[0];
    HashSeg s{};
    SPK_TRY(seg_of(ctx, raw_uid, t.n, 0, -1, &s));
    SPK_REQUIRE(s.kind == RAW_I64, SPK_E_INVALID, "spk_rank_from_raw: unique ids must be an int64 raw column");
    const int64_t n = t.n;
    SPK_TRY(t.rank.alloc((size_t)n + 1));
    if (n == 0) return SPK_OK;
    IdWork w;
    SPK_TRY(w.alloc(n));
    DevBuf<uint8_t> nul;
    DevBuf<int64_t> ids;
    SPK_TRY(nul.alloc((size_t)n + 1));
    SPK_TRY(ids.alloc((size_t)n + 1));
    k_i64_keys<<<grid(n), 256, 0, ctx->stream>>>(n, s.i64, s.valid, w.k_in.p, w.i_in.p, nul.p);
    SPK_HIP(hipGetLastError());
    int64_t runs = 0;
    bool coll = false;
    HashSeg none{};
    SPK_TRY(sorted_ids(ctx, n, w, none, none, false, nul.p, ids.p, &runs, &coll));
    // a NULL id (possibly sharing the last run's key) never undercounts: div = runs + 1 > any id + 1
    const int64_t div = runs + 1;
    SPK_REQUIRE(2 * div < (int64_t)UINT32_MAX, SPK_E_LIMIT, "rank must be in [0, 2^32)");
    k_rank<<<grid(n), 256, 0, ctx->stream>>>(n, ids.p, t.perm.p, right_from < 0 ? n : right_from, div, t.rank.p);
    SPK_HIP(hipGetLastError());
    // NULL ids present?  (the rank layout then marks them for the link predicate)
    DevBuf<unsigned long long> cnt;
    SPK_TRY(cnt.alloc(1));
    size_t bytes = 0;
    SPK_HIP(rocprim::reduce(nullptr, bytes, nul.p, cnt.p, (size_t)n, rocprim::plus<unsigned long long>(), ctx->stream));
    SPK_TRY(w.tmp.alloc(bytes + 1));
    SPK_HIP(rocprim::reduce(w.tmp.p, bytes, nul.p, cnt.p, (size_t)n, rocprim::plus<unsigned long long>(), ctx->stream));
    unsigned long long n_null = 0;
    SPK_HIP(hipMemcpyAsync(&n_null, cnt.p, 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    t.null_div = n_null ? div : 0;
    return SPK_OK;
}

int spk_cluster(spk_ctx *ctx, int32_t *out_perm0, int32_t *out_perm1) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    SPK_HIP(hipSetDevice(ctx->device));
    const bool link_only = ctx->link_type == SPK_LINK_ONLY;
    for (int side = 0; side < (link_only ? 2 : 1); ++side) {
        Table &t = ctx->table[side];
        const int which = side == 0 ? 0 : 1;
        SPK_REQUIRE(!t.key[which].empty() && t.key[which][0]->p, SPK_E_STATE, "spk_cluster: rule 0 key not set");
        const bool use_rank = side == 0 && !link_only;
        SPK_REQUIRE(!use_rank || t.rank.p || t.n == 0, SPK_E_STATE, "spk_cluster: rank not set");
        const int64_t n = t.n;
        int32_t *out = side == 0 ? out_perm0 : out_perm1;
        if (n == 0) continue;
        IdWork w;
        SPK_TRY(w.alloc(n));
        k_cluster_keys<<<grid(n), 256, 0, ctx->stream>>>(n, t.key[which][0]->p, use_rank ? t.rank.p : nullptr,
                                                         w.k_in.p, w.i_in.p);
        SPK_HIP(hipGetLastError());
        size_t bytes = 0;
        SPK_HIP(rocprim::radix_sort_pairs(nullptr, bytes, w.k_in.p, w.k_out.p, w.i_in.p, w.i_out.p, (size_t)n, 0, 64,
                                          ctx->stream));
        SPK_TRY(w.tmp.alloc(bytes + 1));
        SPK_HIP(rocprim::radix_sort_pairs(w.tmp.p, bytes, w.k_in.p, w.k_out.p, w.i_in.p, w.i_out.p, (size_t)n, 0, 64,
                                          ctx->stream));
        const int32_t *perm = w.i_out.p;
        DevBuf<int64_t> tmp64;
        SPK_TRY(tmp64.alloc((size_t)n + 1));
        auto permute64 = [&](DevBuf<int64_t> &b) -> int {
            if (!b.p) return SPK_OK;
            k_gather<int64_t><<<grid(n), 256, 0, ctx->stream>>>(n, b.p, perm, tmp64.p);
            SPK_HIP(hipGetLastError());
            SPK_HIP(hipMemcpyAsync(b.p, tmp64.p, (size_t)n * 8, hipMemcpyDeviceToDevice, ctx->stream));
            return SPK_OK;
        };
        for (int wh = 0; wh < 2; ++wh)
            for (DevBuf<int64_t> *k : t.key[wh]) SPK_TRY(permute64(*k));
        SPK_TRY(permute64(t.rank));
        // compose with an earlier permutation: table row i = input row old[perm[i]]
        DevBuf<int32_t> np;
        SPK_TRY(np.alloc((size_t)n + 1));
        if (t.perm.p) {
            k_gather<int32_t><<<grid(n), 256, 0, ctx->stream>>>(n, t.perm.p, perm, np.p);
            SPK_HIP(hipGetLastError());
        } else {
            SPK_HIP(hipMemcpyAsync(np.p, perm, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream));
        }
        SPK_TRY(t.perm.alloc((size_t)n + 1));
        SPK_HIP(hipMemcpyAsync(t.perm.p, np.p, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream));
        if (out) SPK_HIP(hipMemcpyAsync(out, t.perm.p, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
        // the rows moved: comparison columns are decoded again (through the permutation)
        for (Column *&c : t.cols) {
            delete c;
            c = nullptr;
        }
        t.desc_dirty = true;
        t.version = ++ctx->table_epoch;
        SPK_HIP(hipStreamSynchronize(ctx->stream));
    }
    ctx->pairs_valid = false;
    ctx->codes_valid = false;
    return SPK_OK;
}

int spk_table_add_raw_utf8(spk_ctx *ctx, int col, int raw0, int raw1) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    SPK_HIP(hipSetDevice(ctx->device));
    const bool two = ctx->link_type == SPK_LINK_ONLY;
    SPK_REQUIRE(!two || raw1 >= 0, SPK_E_INVALID, "spk_table_add_raw_utf8: link_only needs the side-1 raw column");
    Table &t0 = ctx->table[0];
    SPK_REQUIRE(t0.n + (two ? ctx->table[1].n : 0) < (int64_t)INT32_MAX, SPK_E_LIMIT,
                "spk_table_add_raw_utf8: more than 2^31-1 rows over both tables");
    HashSeg s0{}, s1{};
    SPK_TRY(seg_of(ctx, raw0, t0.n, 0, -1, &s0));
    SPK_REQUIRE(s0.kind == RAW_UTF8, SPK_E_INVALID, "spk_table_add_raw_utf8: not a string raw column");
    if (two) {
        SPK_TRY(seg_of(ctx, raw1, ctx->table[1].n, 0, -1, &s1));
        SPK_REQUIRE(s1.kind == RAW_UTF8, SPK_E_INVALID, "spk_table_add_raw_utf8: not a string raw column");
    }
    DevBuf<int64_t> ids;
    int64_t n_ids = 0;
    SPK_TRY(hashed_ids(ctx, s0, s1, ids, &n_ids));  // one id space for both sides
    SPK_REQUIRE(n_ids <= (int64_t)UINT32_MAX, SPK_E_LIMIT, "more than 2^32 distinct values in a column");
    for (int side = 0; side < (two ? 2 : 1); ++side) {
        Table &t = ctx->table[side];
        RawCol *r = ctx->raw[side == 0 ? raw0 : raw1];
        const int64_t n = t.n;
        const int32_t *perm = t.perm.p;
        Column *c = nullptr;
        SPK_TRY(new_column(ctx, side, col, &c));
        c->kind = COL_STR;
        c->has_ids = true;
        c->n_ids = n_ids;
        c->src[0] = ctx->raw[raw0]->serial;
        c->src[1] = ctx->raw[two ? raw1 : raw0]->serial;
        c->has_empty = ctx->raw[raw0]->has_empty || (two && ctx->raw[raw1]->has_empty);
        DevBuf<int64_t> len, off8;
        SPK_TRY(len.alloc((size_t)n + 1));
        SPK_TRY(off8.alloc((size_t)n + 1));
        k_perm_lengths<<<grid(n + 1), 256, 0, ctx->stream>>>(n, r->off.p, perm, len.p);
        SPK_HIP(hipGetLastError());
        DevBuf<uint8_t> tmp;
        size_t bytes = 0;
        SPK_HIP(rocprim::exclusive_scan(nullptr, bytes, len.p, off8.p, (int64_t)0, (size_t)n + 1,
                                        rocprim::plus<int64_t>(), ctx->stream));
        SPK_TRY(tmp.alloc(bytes + 1));
        SPK_HIP(rocprim::exclusive_scan(tmp.p, bytes, len.p, off8.p, (int64_t)0, (size_t)n + 1,
                                        rocprim::plus<int64_t>(), ctx->stream));
        int64_t nbytes = 0;
        SPK_HIP(hipMemcpyAsync(&nbytes, off8.p + n, 8, hipMemcpyDeviceToHost, ctx->stream));
        SPK_HIP(hipStreamSynchronize(ctx->stream));
        SPK_REQUIRE(nbytes + 3 * n + 16 < ((int64_t)1 << 34), SPK_E_LIMIT,
                    "a string column is limited to 2^34 UTF-16 units (16 GiB of text)");
        const bool long_rows = r->max_len > 64;
        c->max_bytes = r->max_len;
        SPK_TRY(c->units.alloc((size_t)(nbytes + 3 * n + 16)));
        SPK_TRY(c->meta.alloc((size_t)n + 1));
        SPK_TRY(c->planes.alloc((size_t)(n + 1) * N_PLANES));
        if (long_rows) SPK_TRY(c->planes_hi.alloc((size_t)(n + 1) * N_PLANES));
        else c->planes_hi.release();
        SPK_HIP(hipMemsetAsync(c->units.p, 0, (size_t)(nbytes + 3 * n + 16) * 2, ctx->stream));
        c->units_len = nbytes + 3 * n + 16;
        SPK_TRY(launch_utf8_decode(ctx, n, off8.p, r->off.p, perm, r->bytes.p, r->valid.p, c, long_rows,
                                   ids.p + (side == 0 ? 0 : s0.n)));
        SPK_HIP(hipStreamSynchronize(ctx->stream));
        SPK_TRY(launch_unit_bits(ctx, n, c));
    }
    ctx->codes_valid = false;
    return SPK_OK;
}

}  // extern "C"
