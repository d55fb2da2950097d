// Context, record-table upload (UTF-8 -> UTF-16 on the device) and pair buffers.
#include <algorithm>
#include <cstring>

#include "spk_internal.h"

namespace spk {

static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }

Table::~Table() {
    for (Column *c : cols) delete c;
    for (int w = 0; w < 2; ++w)
        for (DevBuf<int64_t> *k : key[w]) delete k;
}

int ensure_desc(spk_ctx *ctx, Table &t) {
    if (!t.desc_dirty && t.d_desc.p) return SPK_OK;
    std::vector<ColDesc> h(t.cols.size());
    for (size_t i = 0; i < t.cols.size(); ++i) {
        Column *c = t.cols[i];
        ColDesc d{};
        d.kind = c ? c->kind : COL_NONE;
        if (c && c->kind == COL_STR) {
            d.units = c->units.p;
            d.meta = c->meta.p;
            d.planes = c->planes.p;
            d.planes_hi = c->planes_hi.n ? c->planes_hi.p : nullptr;
            d.bag = c->bag.n ? c->bag.p : nullptr;
        } else if (c && c->kind == COL_NUM) {
            d.val = c->val.p;
            d.valid = c->valid.p;
        }
        h[i] = d;
    }
    SPK_TRY(t.d_desc.alloc(h.size() ? h.size() : 1));
    if (!h.empty())
        SPK_HIP(hipMemcpyAsync(t.d_desc.p, h.data(), h.size() * sizeof(ColDesc), hipMemcpyHostToDevice, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    t.desc_dirty = false;
    return SPK_OK;
}

// One thread per row: decode the row's UTF-8 into UTF-16 units at its aligned start, count code
// points, hash the units and build the bucket sketch used by the comparison filters, the head units and
// the bit-planes -- all in the one pass over the bytes.
// Surrogate-encoded (CESU / "surrogatepass") 3-byte sequences decode to lone surrogate units,
// exactly as a Java String would hold them.
//
// Four bytes at a time: a dword-aligned window of the source (two aligned dword loads and a byte shift) whose
// four bytes are all ASCII becomes four units at once -- plane bits by a multiply that gathers bit b of the
// four bytes into a nibble, the units as one 8-byte store when aligned.  Other bytes take the code-point
// path.  (The one-byte-per-iteration loop was a chain of dependent byte loads and re-read the units it had
// written to build the planes: 0.55 ms per million rows at cfg5.)

// perm (optional): row `row` of the table is row perm[row] of the source buffers (src_off / bytes /
// valid / ids); off8 is then the layout of the permuted rows (exclusive scan of their byte lengths).
__global__ void k_utf8_decode(int64_t n, const int64_t *__restrict__ off8, const int64_t *__restrict__ src_off,
                              const int32_t *__restrict__ perm, const uint8_t *__restrict__ bytes,
                              const uint8_t *__restrict__ valid, uint16_t *__restrict__ units,
                              RecMeta *__restrict__ meta, uint64_t *__restrict__ planes,
                              uint64_t *__restrict__ planes_hi, const int64_t *__restrict__ ids) {
    int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= n) return;
    const int64_t src = perm ? (int64_t)perm[row] : row;
    RecMeta m;
    const int64_t start = (off8[row] + 3 * row + 3) & ~(int64_t)3;
    m.off4 = (uint32_t)(start >> 2);
    m.head = 0;
    if (!valid[src]) {
        m.len16 = -1;
        m.cpf = 0;
        m.key = 0;
        m.sketch = 0;
        meta[row] = m;
        for (int b = 0; b < N_PLANES; ++b) planes[row * N_PLANES + b] = 0;
        if (planes_hi)
            for (int b = 0; b < N_PLANES; ++b) planes_hi[row * N_PLANES + b] = 0;
        return;
    }
    const int64_t *so = src_off ? src_off : off8;
    const int64_t b0 = so[src], e = so[src + 1];
    uint16_t *dst = units + start;
    const int cap = planes_hi ? PLANES2_MAX : 64;  // units the planes can hold
    int32_t nu = 0, nc = 0;
    uint64_t h = 1469598103934665603ull, sk = 0, head = 0;
    uint64_t pl[N_PLANES] = {0, 0, 0, 0, 0, 0, 0, 0}, ph[N_PLANES] = {0, 0, 0, 0, 0, 0, 0, 0};
    bool latin = true;  // every unit so far < 256
    auto put = [&](uint32_t u) {  // one unit, the code-point path
        if (nu < 4) head |= (uint64_t)u << (16 * nu);
        latin = latin && u < 256u;
        if (latin && nu < cap) {
#pragma unroll
            for (int b = 0; b < N_PLANES; ++b) {
                const uint64_t bit = (uint64_t)((u >> b) & 1u);
                if (nu < 64) pl[b] |= bit << nu;
                else ph[b] |= bit << (nu - 64);
            }
        }
        dst[nu++] = (uint16_t)u;
        h = (h ^ u) * 1099511628211ull;
        sketch_add(sk, u);
    };
    // dword view of the source bytes from the dword boundary at or below `bytes` (an Arrow buffer may start
    // anywhere); a dword holding a byte of the column lies inside its allocation
    const uint32_t mis = (uint32_t)((uintptr_t)bytes & 3u);
    const uint32_t *w = reinterpret_cast<const uint32_t *>(bytes - mis);
    int64_t pos = b0;
    while (pos < e) {
        if (pos + 4 <= e) {
            const int64_t ap = pos + mis;
            const uint32_t sh = (uint32_t)(ap & 3);
            const uint32_t lo = w[ap >> 2], hi = sh ? w[(ap >> 2) + 1] : 0u;  // (ap + 3 >> 2: a byte of the row)
            const uint32_t v = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
            if ((v & 0x80808080u) == 0) {  // four ASCII bytes: four units
                const uint32_t u0 = v & 0xFFu, u1 = (v >> 8) & 0xFFu, u2 = (v >> 16) & 0xFFu, u3 = v >> 24;
                if (nu < 4) {
                    const uint64_t q = (uint64_t)u0 | ((uint64_t)u1 << 16) | ((uint64_t)u2 << 32) | ((uint64_t)u3 << 48);
                    head |= q << (16 * nu);
                }
                if (latin && nu < cap) {
#pragma unroll
                    for (int b = 0; b < N_PLANES; ++b) {
                        // bit b of the four bytes (bits 0, 8, 16, 24 after the shift) into bits 28 .. 31
                        const uint64_t nib = (uint64_t)((((v >> b) & 0x01010101u) * 0x10204080u) >> 28);
                        if (nu < 64) {
                            pl[b] |= nib << nu;
                            if (nu > 60) ph[b] |= nib >> (64 - nu);
                        } else {
                            ph[b] |= nib << (nu - 64);
                        }
                    }
                }
                if ((nu & 3) == 0) {
                    *reinterpret_cast<uint2 *>(dst + nu) = make_uint2(u0 | (u1 << 16), u2 | (u3 << 16));
                } else {
                    dst[nu] = (uint16_t)u0;
                    dst[nu + 1] = (uint16_t)u1;
                    dst[nu + 2] = (uint16_t)u2;
                    dst[nu + 3] = (uint16_t)u3;
                }
                h = (h ^ u0) * 1099511628211ull;
                h = (h ^ u1) * 1099511628211ull;
                h = (h ^ u2) * 1099511628211ull;
                h = (h ^ u3) * 1099511628211ull;
                sketch_add(sk, u0);
                sketch_add(sk, u1);
                sketch_add(sk, u2);
                sketch_add(sk, u3);
                nu += 4;
                nc += 4;
                pos += 4;
                continue;
            }
        }
        uint32_t c0 = bytes[pos];
        uint32_t cp;
        int len;
        if (c0 < 0x80) { cp = c0; len = 1; }
        else if (c0 < 0xE0) { cp = c0 & 0x1F; len = 2; }
        else if (c0 < 0xF0) { cp = c0 & 0x0F; len = 3; }
        else { cp = c0 & 0x07; len = 4; }
        for (int i = 1; i < len && pos + i < e; ++i) cp = (cp << 6) | (bytes[pos + i] & 0x3F);
        pos += len;
        if (cp >= 0x10000) {
            const uint32_t v = cp - 0x10000;
            put(0xD800u + (v >> 10));
            put(0xDC00u + (v & 0x3FFu));
        } else {
            put(cp);
        }
        ++nc;
    }
    // bit-planes for Latin-1 rows of <= 64 units (one word) or, when the column has planes_hi,
    // <= PLANES2_MAX units (two words)
    latin = latin && nu <= cap;
    const bool ok = latin && nu <= 64, ok2 = latin && nu > 64;
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) planes[row * N_PLANES + b] = (ok || ok2) ? pl[b] : 0;
    if (planes_hi)
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) planes_hi[row * N_PLANES + b] = ok2 ? ph[b] : 0;
    m.head = head;
    m.len16 = nu;
    m.cpf = (uint32_t)nc | (ok ? CPF_PLANES : 0u) | (ok2 ? CPF_PLANES2 : 0u) | (ids ? CPF_ID : 0u);
    h ^= (uint64_t)nu;
    m.key = ids ? (uint32_t)ids[src] : (uint32_t)(h ^ (h >> 32));
    m.sketch = sk;
    meta[row] = m;
}

// OR / AND over the units of every plane row of a column (bits 0..7, from the planes: bit b of the
// OR is set when some unit has bit b, of the AND when every unit has it).  spk_gammas drops the top
// planes whose bit is the same for every unit of both sides (SimpleCol.np).
__global__ void k_unit_bits(int64_t n, const RecMeta *__restrict__ meta, const uint64_t *__restrict__ planes,
                            const uint64_t *__restrict__ planes_hi, unsigned int *__restrict__ out) {
    __shared__ unsigned int s_or, s_and;
    if (threadIdx.x == 0) {
        s_or = 0;
        s_and = 0xFFu;
    }
    __syncthreads();
    unsigned int o = 0, a = 0xFFu;
    for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < n; row += (int64_t)gridDim.x * blockDim.x) {
        const RecMeta m = meta[row];
        const bool two = (m.cpf & CPF_PLANES2) != 0, one = (m.cpf & CPF_PLANES) != 0;
        if (m.len16 <= 0 || !(one || two)) continue;
        const int nu = m.len16;
        const uint64_t lo_mask = nu >= 64 ? ~0ull : ((1ull << nu) - 1);
        const uint64_t hi_mask = two ? (nu - 64 >= 64 ? ~0ull : ((1ull << (nu - 64)) - 1)) : 0ull;
        for (int b = 0; b < N_PLANES; ++b) {
            const uint64_t p = planes[row * N_PLANES + b], q = two ? planes_hi[row * N_PLANES + b] : 0ull;
            if (p | q) o |= 1u << b;
            if ((p & lo_mask) != lo_mask || (q & hi_mask) != hi_mask) a &= ~(1u << b);
        }
    }
    atomicOr(&s_or, o);
    atomicAnd(&s_and, a);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicOr(&out[0], s_or);
        atomicAnd(&out[1], s_and);
    }
}

// Character-bag rows of a free-text string column that a Levenshtein comparison reads: per row 32 bytes, the counts of
// 60 buckets in 4-bit saturating nibbles ('a'-'z', 'A'-'Z', digits mod 8: words 0-6 and the low half of word
// 7), then the count of the row's other units (byte 30) and its length (byte 31; 255: no bag -- NULL, past 128
// units, or a surrogate pair, whose units are not its code points).  The Levenshtein distance of two rows is
// at least their bag distance max(la, lb) - |A ∩ B| (one edit changes one unit of either multiset), and the
// intersection is at most Σ min over the buckets plus min(other_a, other_b): k_compact_lev decides the listed
// cells whose bound already exceeds the cut (cfg5 addresses: 5.69 of 15.90 M listed cells).  Built on first
// use (spk_gammas), dropped when the column is decoded again.  One thread per row, its nibbles in LDS
// (dynamic bucket index).
constexpr int BAG_THREADS = 256;
__global__ __launch_bounds__(BAG_THREADS) void k_bag_rows(int64_t n, const RecMeta *__restrict__ meta,
                                                          const uint16_t *__restrict__ units, uint4 *__restrict__ bag) {
    __shared__ uint32_t s_w[BAG_THREADS][9];  // (stride 9: rows of consecutive threads in different banks)
    const int64_t row = (int64_t)blockIdx.x * BAG_THREADS + threadIdx.x;
    if (row >= n) return;
    uint32_t *w = s_w[threadIdx.x];
    for (int q = 0; q < 8; ++q) w[q] = 0;
    const RecMeta m = meta[row];
    const int len = m.len16;
    if (len >= 0 && len <= 128 && meta_cplen(m) == len) {
        const uint16_t *u = units + meta_off(m);
        uint32_t other = 0;
        for (int i = 0; i < len; ++i) {
            const uint32_t c = u[i];
            int b = -1;
            if (c >= 'a' && c <= 'z') b = (int)(c - 'a');
            else if (c >= 'A' && c <= 'Z') b = 26 + (int)(c - 'A');
            else if (c >= '0' && c <= '9') b = 52 + (int)((c - '0') & 7u);
            if (b < 0) {
                ++other;
                continue;
            }
            const int sh = (b & 7) * 4;
            const uint32_t x = w[b >> 3];
            if (((x >> sh) & 15u) < 15u) w[b >> 3] = x + (1u << sh);
        }
        w[7] |= (other << 16) | ((uint32_t)len << 24);
    } else {
        w[7] = 0xFF000000u;
    }
    bag[2 * row] = make_uint4(w[0], w[1], w[2], w[3]);
    bag[2 * row + 1] = make_uint4(w[4], w[5], w[6], w[7]);
}

int build_bag_rows(spk_ctx *ctx, int64_t n, Column *c) {
    SPK_TRY(c->bag.alloc((size_t)(2 * n + 2)));
    if (n > 0) {
        k_bag_rows<<<(unsigned)((n + BAG_THREADS - 1) / BAG_THREADS), BAG_THREADS, 0, ctx->stream>>>(n, c->meta.p,
                                                                                                  c->units.p, c->bag.p);
        SPK_HIP(hipGetLastError());
    }
    return SPK_OK;
}

int launch_unit_bits(spk_ctx *ctx, int64_t n, Column *c) {
    c->unit_bits = false;
    c->bag.release();  // the rows changed: built again on first use
    if (n <= 0) return SPK_OK;
    DevBuf<unsigned int> d;
    SPK_TRY(d.alloc(2));
    const unsigned int init[2] = {0u, 0xFFu};
    SPK_HIP(hipMemcpyAsync(d.p, init, sizeof(init), hipMemcpyHostToDevice, ctx->stream));
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4 * (int64_t)ctx->n_cu);
    k_unit_bits<<<(unsigned)blocks, 256, 0, ctx->stream>>>(n, c->meta.p, c->planes.p, c->planes_hi.p, d.p);
    SPK_HIP(hipGetLastError());
    unsigned int h[2];
    SPK_HIP(hipMemcpyAsync(h, d.p, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    c->unit_or = h[0];
    c->unit_and = h[1];
    c->unit_bits = true;
    return SPK_OK;
}

int launch_utf8_decode(spk_ctx *ctx, int64_t n, const int64_t *off8, const int64_t *src_off, const int32_t *perm,
                       const uint8_t *bytes, const uint8_t *valid, Column *c, bool long_rows, const int64_t *ids) {
    if (n <= 0) return SPK_OK;
    k_utf8_decode<<<(unsigned)((n + 255) / 256), 256, 0, ctx->stream>>>(n, off8, src_off, perm, bytes, valid, c->units.p,
                                                                        c->meta.p, c->planes.p,
                                                                        long_rows ? c->planes_hi.p : nullptr, ids);
    SPK_HIP(hipGetLastError());
    return SPK_OK;
}


int new_column(spk_ctx *ctx, int side, int col, Column **out) {
    SPK_REQUIRE(ctx && (side == 0 || side == 1), SPK_E_INVALID, "bad side");
    Table &t = ctx->table[side];
    SPK_REQUIRE(t.n >= 0, SPK_E_STATE, "table not created");
    SPK_REQUIRE(col >= 0 && col < 4096, SPK_E_INVALID, "column index out of range");
    if (col >= (int)t.cols.size()) t.cols.resize((size_t)col + 1, nullptr);
    delete t.cols[col];
    t.cols[col] = new Column();
    t.desc_dirty = true;
    t.version = ++ctx->table_epoch;
    *out = t.cols[col];
    return SPK_OK;
}

}  // namespace spk

using namespace spk;

int spk_ctx::begin(Kern k) {
    if (!timing) return SPK_OK;
    ev_slot[k] ^= 1;
    ev_used[ev_slot[k]][k] = false;
    SPK_HIP(hipEventRecord(ev0[ev_slot[k]][k], stream));
    return SPK_OK;
}
int spk_ctx::end(Kern k) {
    if (!timing) return SPK_OK;
    SPK_HIP(hipEventRecord(ev1[ev_slot[k]][k], stream));
    ev_used[ev_slot[k]][k] = true;
    return SPK_OK;
}

int spk_ctx::xbegin(int k) {
    if (!timing || !timing_exact) return SPK_OK;
    while ((int)xev0.size() <= k) {
        hipEvent_t a = nullptr, b = nullptr;
        SPK_HIP(hipEventCreate(&a));
        SPK_HIP(hipEventCreate(&b));
        xev0.push_back(a);
        xev1.push_back(b);
        xev_used.push_back(0);
    }
    xev_used[k] = 0;
    SPK_HIP(hipEventRecord(xev0[k], stream));
    return SPK_OK;
}
int spk_ctx::xend(int k) {
    if (!timing || !timing_exact) return SPK_OK;
    SPK_HIP(hipEventRecord(xev1[k], stream));
    xev_used[k] = 1;
    return SPK_OK;
}

extern "C" {

const char *spk_last_error(void) { return g_last_error.c_str(); }
int spk_version(void) { return 1; }

int spk_device_count(int *out) {
    SPK_REQUIRE(out, SPK_E_INVALID, "spk_device_count: null out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *out = n;
    return SPK_OK;
}

int spk_ctx_create(int device, spk_ctx **out) {
    SPK_REQUIRE(out, SPK_E_INVALID, "spk_ctx_create: null out");
    int n = 0;
    SPK_HIP(hipGetDeviceCount(&n));
    SPK_REQUIRE(device >= 0 && device < n, SPK_E_INVALID, "spk_ctx_create: no such HIP device");
    SPK_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    SPK_HIP(hipGetDeviceProperties(&prop, device));
    SPK_REQUIRE(std::strncmp(prop.gcnArchName, "gfx950", 6) == 0, SPK_E_INVALID,
                std::string("libsplink_hip is built for gfx950 (MI355X); device is ") + prop.gcnArchName);
    spk_ctx *c = new spk_ctx();
    c->device = device;
    c->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    // LDS one workgroup may allocate (the lane-private E/M histogram sizes its copies to it)
    int lds = 0, lds_optin = 0;
    (void)hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device);
    (void)hipDeviceGetAttribute(&lds_optin, hipDeviceAttributeSharedMemPerBlockOptin, device);
    c->lds_per_block = std::max(std::max(lds, lds_optin), 64 * 1024);
    hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        set_error(std::string("hipStreamCreate: ") + hipGetErrorString(e));
        return SPK_E_HIP;
    }
    c->stream = c->own_stream;
    for (int b = 0; b < 2; ++b)
        for (int k = 0; k < K_COUNT; ++k) {
            (void)hipEventCreate(&c->ev0[b][k]);
            (void)hipEventCreate(&c->ev1[b][k]);
        }
    (void)hipEventCreateWithFlags(&c->ev_info, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&c->ev_stats, hipEventDisableTiming);
    *out = c;
    return SPK_OK;
}

void spk_ctx_destroy(spk_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (int b = 0; b < 2; ++b)
        for (int k = 0; k < K_COUNT; ++k) {
            (void)hipEventDestroy(ctx->ev0[b][k]);
            (void)hipEventDestroy(ctx->ev1[b][k]);
        }
    for (size_t k = 0; k < ctx->xev0.size(); ++k) {
        (void)hipEventDestroy(ctx->xev0[k]);
        (void)hipEventDestroy(ctx->xev1[k]);
    }
    if (ctx->split_ready) {
        (void)hipStreamSynchronize(ctx->alt.stream);
        for (size_t k = 0; k < ctx->alt.xev0.size(); ++k) {
            (void)hipEventDestroy(ctx->alt.xev0[k]);
            (void)hipEventDestroy(ctx->alt.xev1[k]);
        }
        (void)hipEventDestroy(ctx->alt.ev_info);
        (void)hipEventDestroy(ctx->ev_fork);
        (void)hipEventDestroy(ctx->ev_join);
        if (ctx->alt.h_info) (void)hipHostFree(ctx->alt.h_info);
        (void)hipStreamDestroy(ctx->alt.stream);
    }
    if (ctx->gexec) (void)hipGraphExecDestroy(ctx->gexec);
    if (ctx->graph) (void)hipGraphDestroy(ctx->graph);
    if (ctx->ev_info) (void)hipEventDestroy(ctx->ev_info);
    if (ctx->ev_stats) (void)hipEventDestroy(ctx->ev_stats);
    if (ctx->h_stats) (void)hipHostFree(ctx->h_stats);
    if (ctx->h_info) (void)hipHostFree(ctx->h_info);
    hipStream_t own = ctx->own_stream;
    delete ctx;
    if (own) (void)hipStreamDestroy(own);
}

int spk_ctx_set_stream(spk_ctx *ctx, void *hip_stream) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    ctx->stream = hip_stream ? (hipStream_t)hip_stream : ctx->own_stream;
    return SPK_OK;
}

int spk_ctx_sync(spk_ctx *ctx) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    SPK_TRY(settle_gammas(ctx, nullptr));
    return SPK_OK;
}

int spk_ctx_enable_timing(spk_ctx *ctx, int on) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    ctx->timing = on != 0;
    ctx->timing_exact = on >= 2;
    return SPK_OK;
}

int spk_ctx_kernel_ms(spk_ctx *ctx, double *out5) {
    SPK_REQUIRE(ctx && out5, SPK_E_INVALID, "null arg");
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    for (int k = 0; k < K_COUNT; ++k) {
        const int b = ctx->ev_slot[k];
        float ms = 0.f;
        if (ctx->ev_used[b][k]) SPK_HIP(hipEventElapsedTime(&ms, ctx->ev0[b][k], ctx->ev1[b][k]));
        out5[k] = ctx->ev_used[b][k] ? (double)ms : -1.0;
    }
    return SPK_OK;
}

int spk_ctx_kernel_ms_done(spk_ctx *ctx, double *out5) {
    SPK_REQUIRE(ctx && out5, SPK_E_INVALID, "null arg");
    for (int k = 0; k < K_COUNT; ++k) {
        out5[k] = -1.0;
        for (int i = 0; i < 2; ++i) {  // the newest pair whose end event has completed
            const int b = i == 0 ? ctx->ev_slot[k] : ctx->ev_slot[k] ^ 1;
            if (!ctx->ev_used[b][k] || hipEventQuery(ctx->ev1[b][k]) != hipSuccess) continue;
            float ms = 0.f;
            SPK_HIP(hipEventElapsedTime(&ms, ctx->ev0[b][k], ctx->ev1[b][k]));
            out5[k] = (double)ms;
            break;
        }
    }
    return SPK_OK;
}

int spk_table_create(spk_ctx *ctx, int side, int64_t n_rows, int n_cols) {
    SPK_REQUIRE(ctx && (side == 0 || side == 1), SPK_E_INVALID, "spk_table_create: bad side");
    SPK_REQUIRE(n_rows >= 0 && n_rows < (int64_t)INT32_MAX && n_cols >= 0, SPK_E_LIMIT,
                "spk_table_create: row count must be < 2^31");
    SPK_HIP(hipSetDevice(ctx->device));
    Table &t = ctx->table[side];
    for (Column *c : t.cols) delete c;
    t.cols.assign((size_t)n_cols, nullptr);
    for (int w = 0; w < 2; ++w) {
        for (DevBuf<int64_t> *k : t.key[w]) delete k;
        t.key[w].clear();
    }
    t.rank.release();
    t.perm.release();
    t.null_div = 0;
    for (auto &v : ctx->rule_terms) v.clear();
    t.n = n_rows;
    t.desc_dirty = true;
    t.version = ++ctx->table_epoch;
    ctx->pairs_valid = false;
    ctx->codes_valid = false;
    return SPK_OK;
}


int spk_table_add_utf8(spk_ctx *ctx, int side, int col, const int64_t *offsets, const uint8_t *data,
                       const uint8_t *valid, const int64_t *value_ids) {
    SPK_REQUIRE(offsets && valid, SPK_E_INVALID, "spk_table_add_utf8: null buffer");
    Column *c = nullptr;
    SPK_TRY(new_column(ctx, side, col, &c));
    SPK_HIP(hipSetDevice(ctx->device));
    int64_t n = ctx->table[side].n;
    int64_t nbytes = offsets[n];
    SPK_REQUIRE(offsets[0] == 0 && nbytes >= 0, SPK_E_INVALID, "spk_table_add_utf8: offsets must start at 0");
    SPK_REQUIRE(nbytes + 3 * n + 16 < ((int64_t)1 << 34), SPK_E_LIMIT,
                "spk_table_add_utf8: a string column is limited to 2^34 UTF-16 units (16 GiB of text)");
    if (value_ids) {
        for (int64_t i = 0; i < n; ++i)
            SPK_REQUIRE(!valid[i] || (value_ids[i] >= 0 && value_ids[i] <= (int64_t)UINT32_MAX), SPK_E_INVALID,
                        "spk_table_add_utf8: value ids must lie in [0, 2^32) for non-NULL rows");
    }
    c->kind = COL_STR;
    c->has_ids = value_ids != nullptr;
    DevBuf<uint8_t> d_bytes, d_valid;
    SPK_TRY(d_bytes.alloc((size_t)nbytes + 1));
    SPK_TRY(d_valid.alloc((size_t)n + 1));
    SPK_TRY(c->units.alloc((size_t)(nbytes + 3 * n + 16)));
    SPK_TRY(c->meta.alloc((size_t)n + 1));
    SPK_TRY(c->planes.alloc((size_t)(n + 1) * N_PLANES));
    // two-word planes only for columns that can have rows of more than 64 units (> 64 bytes)
    int64_t max_bytes = 0;
    for (int64_t i = 0; i < n; ++i) max_bytes = std::max<int64_t>(max_bytes, offsets[i + 1] - offsets[i]);
    c->max_bytes = max_bytes;
    const bool long_rows = max_bytes > 64;
    if (long_rows) SPK_TRY(c->planes_hi.alloc((size_t)(n + 1) * N_PLANES));
    else c->planes_hi.release();
    DevBuf<int64_t> d_off8, d_ids;
    SPK_TRY(d_off8.alloc((size_t)n + 1));
    if (value_ids) {
        SPK_TRY(d_ids.alloc((size_t)n + 1));
        if (n) SPK_HIP(hipMemcpyAsync(d_ids.p, value_ids, (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream));
    }
    if (nbytes) SPK_HIP(hipMemcpyAsync(d_bytes.p, data, (size_t)nbytes, hipMemcpyHostToDevice, ctx->stream));
    if (n) SPK_HIP(hipMemcpyAsync(d_valid.p, valid, (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    SPK_HIP(hipMemsetAsync(c->units.p, 0, (size_t)(nbytes + 3 * n + 16) * 2, ctx->stream));
    c->units_len = nbytes + 3 * n + 16;
    SPK_HIP(hipMemcpyAsync(d_off8.p, offsets, (size_t)(n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
    if (n) {
        int bs = 256;
        k_utf8_decode<<<(unsigned)((n + bs - 1) / bs), bs, 0, ctx->stream>>>(n, d_off8.p, nullptr, nullptr, d_bytes.p,
                                                                          d_valid.p, c->units.p, c->meta.p, c->planes.p,
                                                                          long_rows ? c->planes_hi.p : nullptr,
                                                                          value_ids ? d_ids.p : nullptr);
        SPK_HIP(hipGetLastError());
    }
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    SPK_TRY(launch_unit_bits(ctx, n, c));
    ctx->codes_valid = false;
    return SPK_OK;
}

int spk_table_add_float64(spk_ctx *ctx, int side, int col, const double *values, const uint8_t *valid) {
    SPK_REQUIRE(values && valid, SPK_E_INVALID, "spk_table_add_float64: null buffer");
    Column *c = nullptr;
    SPK_TRY(new_column(ctx, side, col, &c));
    SPK_HIP(hipSetDevice(ctx->device));
    int64_t n = ctx->table[side].n;
    c->kind = COL_NUM;
    SPK_TRY(c->val.alloc((size_t)n + 1));
    SPK_TRY(c->valid.alloc((size_t)n + 1));
    if (n) {
        SPK_HIP(hipMemcpyAsync(c->val.p, values, (size_t)n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
        SPK_HIP(hipMemcpyAsync(c->valid.p, valid, (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    }
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    ctx->codes_valid = false;
    return SPK_OK;
}

}  // extern "C"

// Per-row host values (input row order) into a device array in table row order: a table reordered by
// spk_cluster takes them through its permutation (table row i = input row perm[i]).
__global__ void k_take_rows(int64_t n, const int64_t *__restrict__ src, const int32_t *__restrict__ perm,
                            int64_t *__restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[perm[i]];
}

static int upload_rows(spk_ctx *ctx, const Table &t, const int64_t *host, int64_t *dev) {
    if (t.n <= 0) return SPK_OK;
    if (!t.perm.p) {
        SPK_HIP(hipMemcpyAsync(dev, host, (size_t)t.n * 8, hipMemcpyHostToDevice, ctx->stream));
        SPK_HIP(hipStreamSynchronize(ctx->stream));
        return SPK_OK;
    }
    DevBuf<int64_t> tmp;
    SPK_TRY(tmp.alloc((size_t)t.n));
    SPK_HIP(hipMemcpyAsync(tmp.p, host, (size_t)t.n * 8, hipMemcpyHostToDevice, ctx->stream));
    k_take_rows<<<(unsigned)((t.n + 255) / 256), 256, 0, ctx->stream>>>(t.n, tmp.p, t.perm.p, dev);
    SPK_HIP(hipGetLastError());
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    return SPK_OK;
}

extern "C" {

int spk_table_set_rank(spk_ctx *ctx, int side, const int64_t *rank) {
    SPK_REQUIRE(ctx && (side == 0 || side == 1) && rank, SPK_E_INVALID, "spk_table_set_rank: bad args");
    Table &t = ctx->table[side];
    SPK_REQUIRE(t.n >= 0, SPK_E_STATE, "table not created");
    SPK_HIP(hipSetDevice(ctx->device));
    for (int64_t i = 0; i < t.n; ++i)
        SPK_REQUIRE(rank[i] >= 0 && rank[i] < (int64_t)UINT32_MAX, SPK_E_LIMIT, "rank must be in [0, 2^32)");
    SPK_TRY(t.rank.alloc((size_t)t.n + 1));
    SPK_TRY(upload_rows(ctx, t, rank, t.rank.p));
    // a new rank has no NULL-id layout until spk_table_set_rank_null declares one again
    t.null_div = 0;
    return SPK_OK;
}

int spk_table_set_rank_null(spk_ctx *ctx, int side, int64_t divisor) {
    SPK_REQUIRE(ctx && (side == 0 || side == 1) && divisor >= 0, SPK_E_INVALID, "spk_table_set_rank_null: bad args");
    ctx->table[side].null_div = divisor;
    return SPK_OK;
}

int spk_table_set_key(spk_ctx *ctx, int side, int rule, int which, const int64_t *keys) {
    SPK_REQUIRE(ctx && (side == 0 || side == 1) && keys && rule >= 0 && (which == 0 || which == 1), SPK_E_INVALID,
                "spk_table_set_key: bad args");
    Table &t = ctx->table[side];
    SPK_REQUIRE(t.n >= 0, SPK_E_STATE, "table not created");
    SPK_HIP(hipSetDevice(ctx->device));
    for (int64_t i = 0; i < t.n; ++i)
        SPK_REQUIRE(keys[i] >= -1 && keys[i] < (int64_t)INT32_MAX, SPK_E_LIMIT, "key ids must be in [-1, 2^31)");
    while ((int)t.key[which].size() <= rule) t.key[which].push_back(new DevBuf<int64_t>());
    SPK_TRY(t.key[which][rule]->alloc((size_t)t.n + 1));
    if (rule < 32) ctx->rule_terms[rule].clear();  // a host-computed key: no term is known
    SPK_TRY(upload_rows(ctx, t, keys, t.key[which][rule]->p));
    return SPK_OK;
}

int spk_pairs_count(spk_ctx *ctx, int64_t *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "null arg");
    SPK_REQUIRE(ctx->pairs_valid, SPK_E_STATE, "no pairs (run spk_block or spk_pairs_load)");
    *out = ctx->n_pairs;
    return SPK_OK;
}

int spk_pairs_copy(spk_ctx *ctx, int64_t start, int64_t count, int32_t *out_l, int32_t *out_r) {
    SPK_REQUIRE(ctx && ctx->pairs_valid, SPK_E_STATE, "no pairs");
    SPK_REQUIRE(start >= 0 && count >= 0 && start + count <= ctx->n_pairs, SPK_E_INVALID, "pair range out of bounds");
    SPK_HIP(hipSetDevice(ctx->device));
    if (count && out_l)
        SPK_HIP(hipMemcpyAsync(out_l, ctx->pl.p + start, (size_t)count * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (count && out_r)
        SPK_HIP(hipMemcpyAsync(out_r, ctx->pr.p + start, (size_t)count * 4, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    return SPK_OK;
}

int spk_pairs_load(spk_ctx *ctx, int64_t n, const int32_t *rows_l, const int32_t *rows_r) {
    SPK_REQUIRE(ctx && n >= 0 && (n == 0 || (rows_l && rows_r)), SPK_E_INVALID, "spk_pairs_load: bad args");
    SPK_HIP(hipSetDevice(ctx->device));
    int64_t nl = ctx->table[0].n, nr = ctx->side_table(1).n;
    for (int64_t i = 0; i < n; ++i)
        SPK_REQUIRE(rows_l[i] >= 0 && rows_l[i] < nl && rows_r[i] >= 0 && rows_r[i] < nr, SPK_E_INVALID,
                    "spk_pairs_load: row index out of range");
    SPK_TRY(ctx->pl.alloc((size_t)n + 1));
    SPK_TRY(ctx->pr.alloc((size_t)n + 1));
    if (n) {
        SPK_HIP(hipMemcpyAsync(ctx->pl.p, rows_l, (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream));
        SPK_HIP(hipMemcpyAsync(ctx->pr.p, rows_r, (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream));
    }
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    ctx->n_pairs = n;
    ctx->pairs_valid = true;
    ctx->pairs_epoch++;
    ctx->tf_mp.release();  // a kept tf result describes the old pair set (spk_tf_copy refuses it)
    ctx->tf_count = -1;
    ctx->n_views = 0;
    ctx->pv_base = n;
    ctx->pair_terms.clear();
    ctx->pair_rule_lo.clear();
    ctx->pair_rule_hi.clear();
    ctx->codes_valid = false;
    return SPK_OK;
}

}  // extern "C"
