// EM over packed comparison-vector codes (replaces expectation_step.py:25-221 and the GROUP BY
// aggregate of maximisation_step.py:41-90), final scoring and term-frequency adjustment.
//
// The E-step's match_probability is a function of the comparison vector only, so the M-step's
// sufficient statistic is the histogram of codes.  Each EM iteration streams every pair's code
// once (HBM-bound: 2 or 4 bytes per pair) into an LDS-privatised histogram (lane-private counters,
// k_hist_lanes; wave-level aggregation of equal codes for large pattern spaces, k_hist), then evaluates mp per pattern with the reference's literal
// arithmetic and reduces the per-(column, level) sums in a fixed order (deterministic, and
// identical for any sharding of pairs over GPUs since the histogram is an exact integer sum).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "spk_internal.h"

// The count rows' publication below relies on gfx950's cache behaviour (sc1 write-through stores drained
// before the ticket atomic, no release fence); build for gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "spk_em.hip targets gfx950 (MI355X) only"
#endif

namespace spk {

constexpr int H_THREADS = 512;
constexpr int H_LDS_BINS = 16384;  // LDS-privatised up to this many patterns (64 KiB)

template <typename CodeT, bool LDS>
__global__ __launch_bounds__(H_THREADS) void k_hist(const CodeT *__restrict__ codes, int64_t P, int n_pat,
                                                    unsigned long long *__restrict__ ghist) {
    extern __shared__ uint32_t sh[];
    if (LDS) {
        for (int b = threadIdx.x; b < n_pat; b += H_THREADS) sh[b] = 0;
        __syncthreads();
    }
    constexpr int VEC = 16 / sizeof(CodeT);  // codes per 16-byte load
    const int64_t n_vec = P / VEC;
    const int lane = threadIdx.x & 63;
    using V4 = uint4;
    const V4 *cv = reinterpret_cast<const V4 *>(codes);
    for (int64_t v = (int64_t)blockIdx.x * H_THREADS + threadIdx.x;; v += (int64_t)gridDim.x * H_THREADS) {
        // wave-uniform loop exit keeps every lane inside the ballots below
        const bool in = v < n_vec;
        if (!__any(in)) break;
        CodeT c[VEC];
        if (in) {
            V4 w = cv[v];
            const CodeT *e = reinterpret_cast<const CodeT *>(&w);
#pragma unroll
            for (int j = 0; j < VEC; ++j) c[j] = e[j];
        }
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            uint32_t mine = in ? (uint32_t)c[j] : 0xFFFFFFFFu;
            unsigned long long todo = __ballot(in);
            // aggregate up to 4 distinct codes per wave with ballots, the rest with plain atomics
            for (int it = 0; it < 4 && todo; ++it) {
                const int leader = __ffsll(todo) - 1;
                const uint32_t lc = __shfl(mine, leader);
                const unsigned long long same = __ballot(mine == lc) & todo;
                if (lane == leader) {
                    if (LDS) atomicAdd(&sh[lc], (uint32_t)__popcll(same));
                    else atomicAdd(&ghist[lc], (unsigned long long)__popcll(same));
                }
                todo &= ~same;
            }
            if ((todo >> lane) & 1ull) {
                if (LDS) atomicAdd(&sh[mine], 1u);
                else atomicAdd(&ghist[mine], 1ull);
            }
        }
    }
    // tail (P not a multiple of VEC): block 0 handles it
    if (blockIdx.x == 0) {
        for (int64_t p = n_vec * VEC + threadIdx.x; p < P; p += H_THREADS) {
            if (LDS) atomicAdd(&sh[codes[p]], 1u);
            else atomicAdd(&ghist[codes[p]], 1ull);
        }
    }
    if (LDS) {
        __syncthreads();
        for (int b = threadIdx.x; b < n_pat; b += H_THREADS) {
            uint32_t v = sh[b];
            if (v) atomicAdd(&ghist[b], (unsigned long long)v);
        }
    }
}

// Histogram with lane-private LDS counters.  Counter (bin, copy) lives at word bin * R + copy with copy =
// lane % R, R = 64 / 32 / 16 / 8 / 4 copies: with R = 64 every lane of a wave hits its own bank (64 x
// 4-byte banks) whatever the codes are, so one code costs one conflict-free `ds_add_u32` and a couple of
// VALU ops -- no ballots, no serialisation on the few dominant patterns.  Smaller R (larger pattern spaces)
// admits 64 / R lanes per counter, and equal codes among them serialise on it; there (R < 64) the most
// frequent pattern of the pair set (found by the launch that first counts it) is not counted at all: its
// bin is P minus every other bin, and the half or more of the codes that carry it skip the atomic.  Waves
// of a workgroup share the copies (atomics; different instructions never bank-conflict).  Codes are
// streamed as 16-byte vectors, four loads in flight per lane.
//
// Measured and not kept (round 5): two tiers for R < 64 -- the 256 most frequent patterns in 64-copy slots,
// the others in R copies, an LDS map pattern -> counters -- with and without the uncounted top pattern:
// the map read per code cost more than the conflicts it removed (cfg5 codes tiled to 368 M pairs: 0.177 ms
// against 0.142; the real 100M-record share: 0.768 against 0.598 ms per iteration; profiles/r5_ab_em_tiers.log).
constexpr int HL_THREADS = 1024;
constexpr int HL_LDS_BYTES = 160 * 1024;  // one workgroup per CU, all of its LDS (gfx950), capped by the device attribute
constexpr int HL_UNROLL = 4;
constexpr int EM_AROWS = 4;               // the one-level reduction's rows (workgroup mod EM_AROWS)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Comparison-pattern arithmetic.  The pattern space description (mixed-radix strides, levels,
// offsets into the flattened m / u) and -- for up to PA_INLINE_MU levels, every template setting --
// the m / u tables themselves travel in the kernel arguments: no per-iteration uploads.
constexpr int PA_MAXK = 64;
constexpr int PA_INLINE_MU = 96;

struct PatArgs {
    int K;
    int n_pat;  // <= 2^31 (set_pattern_space)
    int n_slots;
    int tot;    // Σ L_k
    double lambda, one_minus;
    const double *mu_dev;  // [m | u] (tot each) when tot > PA_INLINE_MU, else null
    int32_t stride[PA_MAXK];
    int16_t moff[PA_MAXK];
    uint8_t nlev[PA_MAXK];
    double mu[2 * PA_INLINE_MU];
};
static_assert(sizeof(PatArgs) <= 4096 && sizeof(PatArgs) % 4 == 0, "kernel argument size");

__device__ inline int pa_gamma(const PatArgs &A, int p, int k) { return (p / A.stride[k]) % (A.nlev[k] + 1) - 1; }
__device__ inline double pa_m(const PatArgs &A, int i) { return A.mu_dev ? A.mu_dev[i] : A.mu[i]; }
__device__ inline double pa_u(const PatArgs &A, int i) { return A.mu_dev ? A.mu_dev[A.tot + i] : A.mu[A.tot + i]; }

// mp of pattern p: (λ·m1·…·mK) / ((λ·m1·…·mK) + ((1-λ)·u1·…·uK)), left-associative products,
// γ = -1 contributes 1.0; a zero denominator is NULL (NaN) as in Spark (expectation_step.py:167-185).
// *ll = ln(λΠm + (1-λ)Πu), NULL for ln(<= 0) (expectation_step.py:224-256).
__device__ inline double pattern_mp(const PatArgs &A, int p, double *ll) {
    double num = A.lambda;
    for (int k = 0; k < A.K; ++k) {
        const int g = pa_gamma(A, p, k);
        num = num * (g < 0 ? 1.0 : pa_m(A, A.moff[k] + g));
    }
    double den = A.one_minus;
    for (int k = 0; k < A.K; ++k) {
        const int g = pa_gamma(A, p, k);
        den = den * (g < 0 ? 1.0 : pa_u(A, A.moff[k] + g));
    }
    const double d = num + den;
    *ll = d > 0.0 ? log(d) : NAN;
    return d == 0.0 ? NAN : num / d;
}

// The arguments are indexed per lane (column tables, m / u by level): stage them in LDS once per
// block instead of letting dynamic indexing of the kernel-argument struct spill it to scratch.
__device__ inline const PatArgs &stage_args(const PatArgs &A, PatArgs *sA) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(&A);
    uint32_t *dst = reinterpret_cast<uint32_t *>(sA);
    for (int i = threadIdx.x; i < (int)(sizeof(PatArgs) / 4); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    return *sA;
}

// One thread per pattern (the per-pattern chain of table lookups is latency-bound: spread it).
__global__ void k_pattern_mp(PatArgs A0, double *__restrict__ mpat, double *__restrict__ llpat) {
    __shared__ PatArgs sA;
    const PatArgs &A = stage_args(A0, &sA);
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= A.n_pat) return;
    double ll;
    mpat[p] = pattern_mp(A, p, &ll);
    if (llpat) llpat[p] = ll;
}

constexpr int N_HEAD = 5;  // [Σmp, rows, non-null rows, Σ ln(...), non-null ln rows]

// Diagnostic build only (-DSPK_EM_STAMPS): wall-clock stamps (100 MHz) of k_em_iter's stages in the
// workgroup that finishes the reduction, read with spk_debug_em_stamps (tools/ab_em_stamps.py).
#ifdef SPK_EM_STAMPS
__device__ unsigned long long g_em_stamps[16];
#define EM_STAMP(i) \
    do {            \
        if (threadIdx.x == 0) g_em_stamps[i] = wall_clock64(); \
    } while (0)
#else
#define EM_STAMP(i) \
    do {            \
    } while (0)
#endif

// ---- one EM iteration in one launch (single GPU) ----------------------------------------------------------
// The E-step per pattern and the M-step sums of the whole pattern space, by ONE workgroup of
// EF_THREADS: each thread evaluates its strided patterns (mp, ln, count) into LDS (global arrays past
// EF_LDS_PAT patterns), then each wave takes statistics slots (slot 0 = totals, slot 1 + s = (column k,
// level v)), sums its lanes' strided patterns and reduces with a fixed butterfly -- deterministic, and
// the same for any sharding of the pairs (the histogram is an exact integer sum).  count(p) supplies
// pattern p's count.  Pattern digits come from divisions by wave-uniform radices in fp64 (exact for
// p < 2^31 after one correction step) instead of integer division sequences.
constexpr int EF_THREADS = 1024;
constexpr int EF_LDS_PAT = 4096;  // 3 doubles per pattern in LDS (96 KiB)

__device__ __forceinline__ int udiv_uniform(int p, int d, double rd, int &rem) {
    int q = (int)((double)p * rd);
    int r = p - q * d;
    if (r < 0) {
        --q;
        r += d;
    } else if (r >= d) {
        ++q;
        r -= d;
    }
    rem = r;
    return q;
}

// Wave-level helpers for doubles: a DPP move within rows of 16 lanes and a lane read (both halves).
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
    const int lo = __double2loint(x), hi = __double2hiint(x);
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, CTRL, 0xF, 0xF, false),
                            __builtin_amdgcn_update_dpp(0, lo, CTRL, 0xF, 0xF, false));
}
// Sum over each row of 16 lanes, left in every lane of the row: quad_perm xor 1 (0xB1), xor 2 (0x4E),
// row_half_mirror (0x141), row_mirror (0x140).  Each step adds a lane's value and its partner's, and
// a + b == b + a exactly, so every lane of a row ends with the same bits.
__device__ __forceinline__ double row_sum16(double x) {
    x += dpp_d<0xB1>(x);
    x += dpp_d<0x4E>(x);
    x += dpp_d<0x141>(x);
    x += dpp_d<0x140>(x);
    return x;
}
__device__ __forceinline__ double readlane_d(double x, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l), __builtin_amdgcn_readlane(__double2loint(x), l));
}

template <class Count>
__device__ void em_finalize_block(const PatArgs &A, Count count, double *__restrict__ mpat, double *__restrict__ llpat,
                                  double *__restrict__ cpat, double *__restrict__ out, double *s_tab,
                                  bool pre = false) {
    const bool lds = s_tab != nullptr && A.n_pat <= EF_LDS_PAT;  // block-uniform
    double *tc = lds ? s_tab : cpat, *tm = lds ? s_tab + A.n_pat : mpat, *tl = lds ? s_tab + 2 * A.n_pat : llpat;
    __shared__ double s_rr[PA_MAXK];  // 1 / (L_k + 1): the digits' reciprocals, once per launch
    if (threadIdx.x < A.K) s_rr[threadIdx.x] = 1.0 / (double)(A.nlev[threadIdx.x] + 1);
    __syncthreads();
    for (int p = threadIdx.x; p < A.n_pat; p += blockDim.x) {
        const unsigned long long c = count(p);
        if (pre) {  // E-step per pattern already in mpat / llpat (k_em_iter's workgroup 0)
            const double mp = mpat[p], ll = llpat[p];
            if (lds) {
                tc[p] = (double)c;
                tm[p] = mp;
                tl[p] = ll;
            } else {
                cpat[p] = (double)c;
            }
            continue;
        }
        // mixed-radix digits, then the reference's left-associative products (pattern_mp)
        double num = A.lambda, den = A.one_minus;
        int q = p;
        for (int k = 0; k < A.K; ++k) {
            const int radix = A.nlev[k] + 1;
            int g;
            q = udiv_uniform(q, radix, s_rr[k], g);
            --g;
            num = num * (g < 0 ? 1.0 : pa_m(A, A.moff[k] + g));
        }
        q = p;
        for (int k = 0; k < A.K; ++k) {
            const int radix = A.nlev[k] + 1;
            int g;
            q = udiv_uniform(q, radix, s_rr[k], g);
            --g;
            den = den * (g < 0 ? 1.0 : pa_u(A, A.moff[k] + g));
        }
        const double d = num + den;
        const double ll = d > 0.0 ? log(d) : NAN;
        const double mp = d == 0.0 ? NAN : num / d;
        if (lds) {  // the global copies are written after the M-step sums, off the critical path
            tc[p] = (double)c;
            tm[p] = mp;
            tl[p] = ll;
        } else {
            mpat[p] = mp;
            llpat[p] = ll;
            cpat[p] = (double)c;
        }
    }
    if (!lds) __threadfence_block();
    __syncthreads();
    EM_STAMP(8);
    // Two slots per wave, one per half-wave (32 lanes): cfg2's 19 slots fit 16 waves in one round.  Each
    // half sums its strided patterns, then a fixed DPP tree within rows of 16 lanes and two readlanes per
    // half -- VALU latency, where a 64-lane shuffle butterfly of six doubles cost ~72 LDS-crossbar
    // round trips.  Deterministic: the same tree whatever the counts.
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, n_waves = blockDim.x >> 6;
    const int half = lane >> 5, l32 = lane & 31;
    // The totals slot (0) sums every pattern, the column slots a 1 / radix share: with spare waves (slots
    // 1 .. n_slots two per wave) the totals are split over them -- a strided share per wave, a 64-lane
    // fixed tree, the waves' partials added in wave order -- instead of 32 lanes walking the whole table.
    const int col_waves = (A.n_slots + 1) / 2, spare = n_waves - col_waves;
    const bool split = spare >= 2;  // block-uniform
    __shared__ double s_tot[16][6];
    if (split && wave >= col_waves) {
        const int sw = wave - col_waves;
        double v[6] = {0, 0, 0, 0, 0, 0};
        for (int p = sw * 64 + lane; p < A.n_pat; p += spare * 64) {
            const double c = tc[p], mp = tm[p], ll = tl[p];
            if (c == 0.0) continue;
            v[0] += c;
            if (!isnan(mp)) {
                v[1] += c;
                v[2] += c * mp;
                v[3] += c * (1.0 - mp);
            }
            if (!isnan(ll)) {
                v[5] += c;
                v[4] += c * ll;
            }
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const double r = row_sum16(v[q]);
            v[q] = (readlane_d(r, 0) + readlane_d(r, 16)) + (readlane_d(r, 32) + readlane_d(r, 48));
        }
        if (lane == 0)
#pragma unroll
            for (int q = 0; q < 6; ++q) s_tot[sw][q] = v[q];
    }
    for (int s0 = split ? 1 + 2 * wave : 2 * wave; s0 <= A.n_slots && (!split || wave < col_waves);
         s0 += split ? 2 * col_waves : 2 * n_waves) {  // wave-uniform
        const int slot = s0 + half;
        double v[6] = {0, 0, 0, 0, 0, 0};  // rows, non-null rows, Σmp, Σ(1-mp), Σ ln, non-null ln rows
        if (slot <= A.n_slots) {
            int kk = -1, vv = 0;
            if (slot > 0) {
                int r = slot - 1;
                for (kk = 0; kk < A.K && r > A.nlev[kk]; ++kk) r -= A.nlev[kk] + 1;
                vv = r - 1;
            }
            // the slot's patterns directly: digit vv + 1 of column kk, p = a·(st·radix) + (vv + 1)·st + b with
            // t = a·st + b stepping by 32 in integers (t = l32 + 32 i), two patterns' loads in flight per
            // step, added in the same order as one at a time
            const int st = kk >= 0 ? A.stride[kk] : 1, radix = kk >= 0 ? A.nlev[kk] + 1 : 1;
            const int n_sel = A.n_pat / radix, base = kk >= 0 ? (vv + 1) * st : 0;
            const int q32 = 32 / st, r32 = 32 - q32 * st, span = st * radix;
            int a = l32 / st, b = l32 - (l32 / st) * st;
            auto step = [&]() {
                a += q32;
                b += r32;
                if (b >= st) {
                    b -= st;
                    ++a;
                }
            };
            auto add = [&](double c, double mp, double ll) {
                if (c == 0.0) return;
                v[0] += c;
                if (!isnan(mp)) {
                    v[1] += c;
                    v[2] += c * mp;
                    v[3] += c * (1.0 - mp);
                }
                if (!isnan(ll)) {
                    v[5] += c;
                    v[4] += c * ll;
                }
            };
            for (int t = l32; t < n_sel; t += 64) {
                const int p1 = kk >= 0 ? a * span + base + b : t;
                step();
                const bool two = t + 32 < n_sel;
                const int p2 = kk >= 0 ? a * span + base + b : t + 32;
                step();
                const double c1 = tc[p1], m1 = tm[p1], l1 = tl[p1];
                double c2 = 0.0, m2 = 0.0, l2 = 0.0;
                if (two) {
                    c2 = tc[p2];
                    m2 = tm[p2];
                    l2 = tl[p2];
                }
                add(c1, m1, l1);
                if (two) add(c2, m2, l2);
            }
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const double r = row_sum16(v[q]);
            v[q] = half ? readlane_d(r, 32) + readlane_d(r, 48) : readlane_d(r, 0) + readlane_d(r, 16);
        }
        if (l32 == 0 && slot <= A.n_slots) {
            if (slot == 0) {
                out[0] = v[2];
                out[1] = v[0];
                out[2] = v[1];
                out[3] = v[4];
                out[4] = v[5];
            } else {
                double *o = out + N_HEAD + 4 * (slot - 1);
                o[0] = v[0];
                o[1] = v[1];
                o[2] = v[2];
                o[3] = v[3];
            }
        }
    }
    if (split) {
        __syncthreads();
        if (threadIdx.x == 0) {
            double v[6] = {0, 0, 0, 0, 0, 0};
            for (int w = 0; w < spare; ++w)
#pragma unroll
                for (int q = 0; q < 6; ++q) v[q] += s_tot[w][q];
            out[0] = v[2];
            out[1] = v[0];
            out[2] = v[1];
            out[3] = v[4];
            out[4] = v[5];
        }
    }
    if (lds) {
        for (int p = threadIdx.x; p < A.n_pat; p += blockDim.x) {
            mpat[p] = tm[p];
            llpat[p] = tl[p];
            cpat[p] = tc[p];
        }
    }
}

// E-step + M-step sums from a complete histogram (after the ranks' all-reduce): one workgroup.
__global__ __launch_bounds__(EF_THREADS) void k_em_finalize(PatArgs A0, const unsigned long long *__restrict__ hist,
                                                            double *__restrict__ mpat, double *__restrict__ llpat,
                                                            double *__restrict__ cpat, double *__restrict__ out) {
    __shared__ PatArgs sA;
    __shared__ double s_tab[3 * EF_LDS_PAT];
    const PatArgs &A = stage_args(A0, &sA);
    em_finalize_block(A, [&](int p) { return hist[p]; }, mpat, llpat, cpat, out, s_tab);
}

// One EM iteration (FIN) or one histogram (!FIN) over the codes with the lane-private counters above.  Each
// workgroup sums its counters per pattern and adds them into one of EM_AROWS global rows with agent-scope
// integer atomics (exact, so their order does not matter), drains them and takes a ticket; the last one sums
// the rows in row order, zeroes them for the next launch, and either (FIN) runs the E-step and the M-step sums
// -- one launch per EM iteration -- or writes the plain histogram to out_hist (multi-GPU: the caller
// all-reduces it).  Workgroup 0 of a FIN launch streams nothing: it evaluates mp and ln(...) per pattern from
// the parameters while the others stream (published with its ticket), so the finishing workgroup only runs
// the M-step sums.  R < 64: ghot[0] is the pattern not counted (-1: none yet); `refresh` makes the last
// workgroup write the most frequent pattern there for the next launches.
__host__ __device__ inline int64_t part_stride(int64_t n_pat) { return (n_pat + 31) / 32 * 32; }  // whole 128-B lines
template <typename CodeT, int R, bool FIN>
__global__ __launch_bounds__(HL_THREADS) void k_em_iter(const CodeT *__restrict__ codes, int64_t P, PatArgs A0,
                                                        unsigned int *__restrict__ ticket, double *__restrict__ mpat,
                                                        double *__restrict__ llpat, double *__restrict__ cpat,
                                                        double *__restrict__ out, unsigned long long *__restrict__ out_hist,
                                                        int fence, uint32_t *__restrict__ arow,
                                                        int32_t *__restrict__ ghot, int refresh, int lds_bytes) {
    extern __shared__ uint32_t sh[];
    __shared__ bool s_last;
    const int n_pat = A0.n_pat;
    const int n_cnt = n_pat * R;  // counter words
    constexpr bool HOT = R < 64;
#ifdef SPK_EM_STAMPS
    const unsigned long long t_start = wall_clock64();
    if (blockIdx.x == 0) EM_STAMP(0);
#endif
    const bool pre = FIN && gridDim.x > 1;
    if (pre && blockIdx.x == 0) {
        PatArgs *sA = reinterpret_cast<PatArgs *>(sh);
        const PatArgs &A = stage_args(A0, sA);
        for (int p = threadIdx.x; p < n_pat; p += HL_THREADS) {
            double ll;
            const double mp = pattern_mp(A, p, &ll);
            __hip_atomic_store(reinterpret_cast<unsigned long long *>(mpat) + p,
                               (unsigned long long)__double_as_longlong(mp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(reinterpret_cast<unsigned long long *>(llpat) + p,
                               (unsigned long long)__double_as_longlong(ll), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    }
    for (int b = threadIdx.x; b < n_cnt; b += HL_THREADS) sh[b] = 0;
    // HOT: the most frequent pattern (-1: none yet) is not counted at all and the last workgroup sets its bin
    // to P minus every other bin (exact: every one of the P codes is streamed once and is < n_pat; P < 2^32 on
    // this path).  With R = 64 the compare would only cost issue slots in an issue-bound loop (cfg2 0.121 ->
    // 0.147 ms at 368 M pairs when it ran there).
    const uint32_t hot0 = HOT ? (uint32_t)ghot[0] : 0xFFFFFFFFu;
    __syncthreads();
    constexpr int VEC = 16 / sizeof(CodeT);
    constexpr int BITS = 8 * sizeof(CodeT);
    const uint32_t copy = threadIdx.x & (R - 1);
    const u32x4 *cv = reinterpret_cast<const u32x4 *>(codes);
    const int64_t n_vec = P / VEC;
    const int64_t stride = (int64_t)(gridDim.x - (pre ? 1 : 0)) * HL_THREADS;
    int64_t v = (pre && blockIdx.x == 0) ? n_vec : (int64_t)(blockIdx.x - (pre ? 1 : 0)) * HL_THREADS + threadIdx.x;
    auto count_code = [&](uint32_t c) {
        if (HOT && c == hot0) return;
        atomicAdd(&sh[c * R + copy], 1u);
    };
    auto count_word = [&](uint32_t w) {
#pragma unroll
        for (int j = 0; j < 32 / BITS; ++j) count_code(BITS == 32 ? w : ((w >> (BITS * j)) & ((1u << BITS) - 1u)));
    };
    // software-pipelined 16-byte nontemporal loads, 2 x HL_UNROLL in flight per lane
    const int64_t step = HL_UNROLL * stride;
    bool have = v + (HL_UNROLL - 1) * stride < n_vec;
    u32x4 w[HL_UNROLL];
    if (have) {
#pragma unroll
        for (int u = 0; u < HL_UNROLL; ++u) w[u] = __builtin_nontemporal_load(cv + v + u * stride);
    }
    while (have) {
        const int64_t vn = v + step;
        const bool hn = vn + (HL_UNROLL - 1) * stride < n_vec;
        // unconditional loads (the last round re-reads its own vectors): under a branch the wait before the
        // counting has to cover the path without them
        const int64_t vl = hn ? vn : v;
        u32x4 x[HL_UNROLL];
#pragma unroll
        for (int u = 0; u < HL_UNROLL; ++u) x[u] = __builtin_nontemporal_load(cv + vl + u * stride);
#pragma unroll
        for (int u = 0; u < HL_UNROLL; ++u) {
            count_word(w[u].x);
            count_word(w[u].y);
            count_word(w[u].z);
            count_word(w[u].w);
        }
#pragma unroll
        for (int u = 0; u < HL_UNROLL; ++u) w[u] = x[u];
        v = vn;
        have = hn;
    }
    for (; v < n_vec; v += stride) {
        const u32x4 x = cv[v];
        count_word(x.x);
        count_word(x.y);
        count_word(x.z);
        count_word(x.w);
    }
    if (blockIdx.x == (pre ? 1u : 0u))  // tail (P not a multiple of VEC)
        for (int64_t p = n_vec * VEC + threadIdx.x; p < P; p += HL_THREADS) count_code((uint32_t)codes[p]);
    __syncthreads();
#ifdef SPK_EM_STAMPS
    const unsigned long long t_streamed = wall_clock64();
#endif
    // fence != 0 (default): an agent-scope release fence before each ticket, the ordering the HSA memory model
    // itself guarantees (after the barrier it is cumulative over the workgroup's atomics).  It cost nothing
    // measurable on MI355X (tools/ab_em_fence.py: E+M launch 121.1 vs 121.7 us at cfg2 x8, 82.2 vs 82.2 us at
    // cfg5 x4, medians of 20, identical statistics).  fence == 0 (spk_em_set_lane_histogram mode 2, A/B
    // only): the row adds are device-scope atomics performed at L2, drained (s_waitcnt) before the ticket
    // atomic, which gfx950 orders behind them (MI355X_MICROARCH.md visibility table, cdna_hip_programming.md
    // G16 R1); the A/B test checks both forms give the same statistics.
    auto arrive = [&](unsigned int *t, unsigned int last) {  // true in the last arriver (whole workgroup)
        if (threadIdx.x == 0) {
            if (fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            s_last = atomicAdd(t, 1u) == last;
        }
        __syncthreads();
        if (!s_last) return false;
        if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        return true;
    };
    const int G = (int)gridDim.x;
    const int64_t ps = part_stride(n_pat);
    uint32_t *my_row = arow + (int64_t)(blockIdx.x % EM_AROWS) * ps;
    for (int b = threadIdx.x; b < n_pat; b += HL_THREADS) {
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < R; ++k) c += sh[b * R + ((k + b) & (R - 1))];  // rotate: spread banks
        if (c) __hip_atomic_fetch_add(my_row + b, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#ifdef SPK_EM_STAMPS
    const unsigned long long t_added = wall_clock64();
#endif
    if (!arrive(ticket, (unsigned int)(G - 1))) return;
#ifdef SPK_EM_STAMPS
    if (threadIdx.x == 0) {  // the last arriver: its start, end of streaming, row adds drained, ticket
        g_em_stamps[1] = t_start;
        g_em_stamps[2] = t_streamed;
        g_em_stamps[3] = t_added;
        g_em_stamps[4] = t_added;
    }
    EM_STAMP(5);
#endif
    uint32_t *s1 = sh;  // per-pattern counts from here on
    const int nr = G < EM_AROWS ? G : EM_AROWS;
    // every row's bin first (independent loads in flight together), then the zeroing stores: a store
    // behind each load to the same address serialised the round trips
    for (int b = threadIdx.x; b < n_pat; b += HL_THREADS) {
        uint32_t vr[EM_AROWS];
#pragma unroll
        for (int r = 0; r < EM_AROWS; ++r)
            vr[r] = r < nr ? __hip_atomic_load(arow + r * ps + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        uint32_t c = 0;
#pragma unroll
        for (int r = 0; r < EM_AROWS; ++r) c += vr[r];
        s1[b] = c;
    }
    __syncthreads();
    for (int b = threadIdx.x; b < n_pat; b += HL_THREADS)
        for (int r = 0; r < nr; ++r) arow[r * ps + b] = 0u;
    if (HOT && hot0 < (uint32_t)n_pat) {  // the uncounted pattern's bin: P minus every other bin
        __shared__ uint32_t s_rest[HL_THREADS / 64];
        uint32_t t = 0;
        for (int p = threadIdx.x; p < n_pat; p += HL_THREADS) t += (uint32_t)p == hot0 ? 0u : s1[p];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
        if ((threadIdx.x & 63) == 0) s_rest[threadIdx.x >> 6] = t;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t rest = 0;
            for (int w = 0; w < HL_THREADS / 64; ++w) rest += s_rest[w];
            s1[hot0] = (uint32_t)P - rest;
        }
        __syncthreads();
    }
    EM_STAMP(6);
    // thread t owns bins p = t, t + HL_THREADS, ... (the same mapping as em_finalize_block's loop, so
    // the count it parks in cpat is read back by the thread that wrote it)
    for (int p = threadIdx.x; p < n_pat; p += HL_THREADS) {
        const unsigned long long c = s1[p];
        if (FIN) cpat[p] = (double)c;
        else out_hist[p] = c;
    }
    if (HOT && refresh) {  // the most frequent pattern (ties: the lower one) for the next launches
        __shared__ unsigned long long s_best[HL_THREADS / 64];
        unsigned long long best = 0;
        for (int p = threadIdx.x; p < n_pat; p += HL_THREADS) {
            const unsigned long long v = ((unsigned long long)s1[p] << 32) | (0xFFFFFFFFull - (uint32_t)p);
            best = v > best ? v : best;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(best, off);
            best = o > best ? o : best;
        }
        if ((threadIdx.x & 63) == 0) s_best[threadIdx.x >> 6] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long bb = 0;
            for (int w = 0; w < HL_THREADS / 64; ++w) bb = s_best[w] > bb ? s_best[w] : bb;
            ghot[0] = (bb >> 32) ? (int32_t)(0xFFFFFFFFull - (bb & 0xFFFFFFFFull)) : -1;
        }
    }
    if (FIN) {
        __syncthreads();  // the counts' LDS is reused for the staged arguments and the pattern table
        PatArgs *sA = reinterpret_cast<PatArgs *>(sh);
        const PatArgs &A = stage_args(A0, sA);
        double *tab = reinterpret_cast<double *>(sh) + (sizeof(PatArgs) + 7) / 8;
        const bool room = ((sizeof(PatArgs) + 7) / 8 + 3 * (size_t)n_pat) * 8 <= (size_t)lds_bytes;
        EM_STAMP(7);
        em_finalize_block(A, [&](int p) { return (unsigned long long)cpat[p]; }, mpat, llpat, cpat, out,
                          room ? tab : nullptr, pre);
    }
    EM_STAMP(9);
    if (threadIdx.x == 0) atomicExch(ticket, 0u);
}

// The uncounted pattern of k_em_iter's first launch on a pair set, guessed from a sample: ghot[0] = the most
// frequent code (ties: the lower one) among HS_SAMPLES 16-byte vectors spread evenly over the codes.  Without
// it that launch counted every pair of the dominant pattern into its R lane copies, a same-address LDS atomic
// chain (cfg5's 100M-record share: 2.5 ms against 0.42 for the launches after it).  Any frequent pattern is a
// good guess: the counts are exact whichever it is (P minus every other bin).  One workgroup; each equal-code
// group of a wave adds once per lane group led by the wave's first active code (the dominant one, mostly).
constexpr int HS_THREADS = 1024;
constexpr int64_t HS_SAMPLES = 8192;
template <typename CodeT>
__global__ __launch_bounds__(HS_THREADS) void k_em_hot_sample(const CodeT *__restrict__ codes, int64_t P, int n_pat,
                                                              int32_t *__restrict__ ghot) {
    extern __shared__ uint32_t bins[];  // n_pat
    __shared__ unsigned long long s_best[HS_THREADS / 64];
    for (int b = threadIdx.x; b < n_pat; b += HS_THREADS) bins[b] = 0;
    __syncthreads();
    auto count = [&](uint32_t c) {
        const uint32_t lead = __builtin_amdgcn_readfirstlane(c);
        const unsigned long long m = __ballot(c == lead);
        if (c != lead) atomicAdd(&bins[c], 1u);
        else if ((int)__lane_id() == __ffsll((long long)m) - 1) atomicAdd(&bins[lead], (uint32_t)__popcll(m));
    };
    constexpr int VEC = 16 / sizeof(CodeT);
    constexpr int BITS = 8 * sizeof(CodeT);
    const int64_t n_vec = P / VEC;
    const int64_t S = n_vec < HS_SAMPLES ? n_vec : HS_SAMPLES;
    const u32x4 *cv = reinterpret_cast<const u32x4 *>(codes);
    for (int64_t i = threadIdx.x; i < S; i += HS_THREADS) {
        const u32x4 x = cv[i * n_vec / S];
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 32 / BITS; ++k) count(BITS == 32 ? w[j] : (w[j] >> (BITS * k)) & ((1u << (BITS & 31)) - 1u));
    }
    for (int64_t p = n_vec * VEC + threadIdx.x; S == 0 && p < P; p += HS_THREADS) atomicAdd(&bins[codes[p]], 1u);
    __syncthreads();
    unsigned long long best = 0;
    for (int p = threadIdx.x; p < n_pat; p += HS_THREADS) {
        const unsigned long long v = ((unsigned long long)bins[p] << 32) | (0xFFFFFFFFull - (uint32_t)p);
        best = v > best ? v : best;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(best, off);
        best = o > best ? o : best;
    }
    if ((threadIdx.x & 63) == 0) s_best[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long bb = 0;
        for (int w = 0; w < HS_THREADS / 64; ++w) bb = s_best[w] > bb ? s_best[w] : bb;
        ghot[0] = (bb >> 32) ? (int32_t)(0xFFFFFFFFull - (bb & 0xFFFFFFFFull)) : -1;
    }
}

// Final E-step: mp[i] = mpat[code[i]] for pairs [start, start + n).  Each lane turns two codes into
// one 16-byte store of two doubles, so a wave instruction writes 1 KiB contiguous (the 8 B/pair of
// output is the dominant stream); the per-pattern table sits in LDS when it fits.  Plain stores:
// 0.704 ms against 0.757 with nontemporal ones over 368M pairs (65 % of HBM peak).  The odd pair at
// either end (when start or start + n is odd) is written by lane 0 of block 0.
constexpr int SC_THREADS = 256;
constexpr int SC_UNROLL = 4;
constexpr int SC_WG_PER_CU = 8;  // grid-stride over at most this many workgroups per CU
constexpr int SC_LDS_PAT = 4096;
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <typename CodeT, bool LDS>
__global__ __launch_bounds__(SC_THREADS) void k_score(const CodeT *__restrict__ codes, int64_t start, int64_t n,
                                                      const double *__restrict__ mpat, int n_pat,
                                                      double *__restrict__ mp) {
    extern __shared__ double tab[];  // n_pat doubles (dynamic: a 576-pattern table leaves room for 8 workgroups per CU)
    if (LDS) {
        for (int b = threadIdx.x; b < n_pat; b += SC_THREADS) tab[b] = mpat[b];
        __syncthreads();
    }
    const double *T = LDS ? tab : mpat;
    const int64_t head = start & 1;
    const int64_t n2 = (n - head) / 2;  // pairs of pairs, from the even ordinal start + head
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (head && n > 0) mp[0] = T[codes[start]];
        if (n - head > 2 * n2) mp[n - 1] = T[codes[start + n - 1]];
    }
    typedef CodeT code2 __attribute__((ext_vector_type(2)));
    const code2 *c = reinterpret_cast<const code2 *>(codes + start + head);
    f64x2 *out = reinterpret_cast<f64x2 *>(mp + head);
    const int64_t stride = (int64_t)gridDim.x * SC_THREADS;
    int64_t v = (int64_t)blockIdx.x * SC_THREADS + threadIdx.x;
    for (; v + (SC_UNROLL - 1) * stride < n2; v += SC_UNROLL * stride) {
        code2 a[SC_UNROLL];
#pragma unroll
        for (int u = 0; u < SC_UNROLL; ++u) a[u] = __builtin_nontemporal_load(c + v + u * stride);
#pragma unroll
        for (int u = 0; u < SC_UNROLL; ++u) {
            f64x2 o;
            o.x = T[a[u].x];
            o.y = T[a[u].y];
            out[v + u * stride] = o;
        }
    }
    for (; v < n2; v += stride) {
        const code2 a = c[v];
        f64x2 o;
        o.x = T[a.x];
        o.y = T[a.y];
        out[v] = o;
    }
}

// Pattern arguments for the current pattern space and m / u (one upload only for large tables).
static int pat_args(spk_ctx *ctx, double lambda, double one_minus, const double *m, const double *u, PatArgs &A) {
    const int K = ctx->K;
    SPK_REQUIRE(K <= PA_MAXK, SPK_E_LIMIT, "too many comparison columns");
    A.K = K;
    A.n_pat = (int)ctx->n_patterns;
    A.lambda = lambda;
    A.one_minus = one_minus;
    int tot = 0, slots = 0;
    for (int k = 0; k < K; ++k) {
        A.stride[k] = (int32_t)ctx->stride[k];
        A.nlev[k] = (uint8_t)ctx->n_levels[k];
        A.moff[k] = (int16_t)tot;
        tot += ctx->n_levels[k];
        slots += ctx->n_levels[k] + 1;
    }
    A.tot = tot;
    A.n_slots = slots;
    A.mu_dev = nullptr;
    if (tot <= PA_INLINE_MU) {
        for (int i = 0; i < tot; ++i) {
            A.mu[i] = m[i];
            A.mu[tot + i] = u[i];
        }
    } else {
        SPK_TRY(ctx->mu.alloc((size_t)2 * tot));
        SPK_HIP(hipMemcpyAsync(ctx->mu.p, m, (size_t)tot * 8, hipMemcpyHostToDevice, ctx->stream));
        SPK_HIP(hipMemcpyAsync(ctx->mu.p + tot, u, (size_t)tot * 8, hipMemcpyHostToDevice, ctx->stream));
        SPK_HIP(hipStreamSynchronize(ctx->stream));  // pageable source: complete before returning
        A.mu_dev = ctx->mu.p;
    }
    return SPK_OK;
}

}  // namespace spk

using namespace spk;


// The LDS plan of k_em_iter: R lane-private copies per pattern (64 .. 4).  R = 0: no lane path (the pattern
// space exceeds the LDS, or 2^32 or more pairs: k_em_iter sums its rows in uint32); those take k_hist (uint64
// counters) + k_em_finalize.
struct LanePlan {
    int R = 0;
    size_t bytes = 0;  // dynamic LDS of the launch
};

static LanePlan lane_plan(spk_ctx *ctx) {
    LanePlan L;
    const int64_t n_pat = ctx->n_patterns;
    const int64_t budget = std::min<int64_t>(HL_LDS_BYTES, ctx->lds_per_block);
    int R = 64;
    while (R >= 4 && n_pat * R * 4 > budget) R >>= 1;
    if (R < 4 || !ctx->hist_lanes || ctx->n_pairs >= (int64_t)UINT32_MAX) return L;
    L.R = R;
    L.bytes = (size_t)std::max<int64_t>(n_pat * R * 4, (int64_t)sizeof(PatArgs));
    return L;
}

// Grid of the lane-histogram launches: one 1024-thread workgroup per CU.
static int64_t lane_grid(spk_ctx *ctx) {
    const int64_t vecs = ctx->n_pairs / (16 / ctx->code_bytes);
    return std::max<int64_t>(1, std::min<int64_t>(ctx->n_cu, (vecs + HL_THREADS - 1) / HL_THREADS));
}

// The reduction rows and the ticket of k_em_iter (zero between launches: the last workgroup resets them,
// zeroed here only when allocated) and its uncounted pattern, found again (by the launch's last workgroup)
// when the pair set or the pattern space changed; repeated comparison passes over the same pairs keep it.
struct EmState {
    unsigned int *ticket = nullptr;
    uint32_t *arow = nullptr;
    int32_t *ghot = nullptr;
    int refresh = 0;
};

// (allocations and their clears: before the launch's timing events, by the callers)
static int em_state_alloc(spk_ctx *ctx) {
    if (!ctx->em_ticket.p) {
        SPK_TRY(ctx->em_ticket.alloc(1));
        SPK_HIP(hipMemsetAsync(ctx->em_ticket.p, 0, 4, ctx->stream));
    }
    const size_t ps = (size_t)part_stride(ctx->n_patterns) * EM_AROWS;
    if (!ctx->em_row.p || ctx->em_row.n < ps) {
        SPK_TRY(ctx->em_row.alloc(ps));
        SPK_HIP(hipMemsetAsync(ctx->em_row.p, 0, ps * 4, ctx->stream));
    }
    if (!ctx->em_hot.p) {
        SPK_TRY(ctx->em_hot.alloc(1));
        SPK_HIP(hipMemsetAsync(ctx->em_hot.p, 0xFF, sizeof(int32_t), ctx->stream));
    }
    return SPK_OK;
}

static int em_state(spk_ctx *ctx, EmState &S) {
    SPK_REQUIRE(ctx->em_ticket.p && ctx->em_hot.p && ctx->em_row.p &&
                    ctx->em_row.n >= (size_t)part_stride(ctx->n_patterns) * EM_AROWS,
                SPK_E_STATE, "k_em_iter state not allocated");
    S.ticket = ctx->em_ticket.p;
    S.arow = ctx->em_row.p;
    const std::vector<int64_t> key = {(int64_t)ctx->pairs_epoch, ctx->n_pairs, ctx->n_patterns, ctx->code_bytes};
    S.refresh = ctx->em_hot_key != key ? 1 : 0;
    ctx->em_hot_key = key;
    S.ghot = ctx->em_hot.p;
    return SPK_OK;
}

template <int R, bool FIN>
static void launch_em_iter(spk_ctx *ctx, const LanePlan &L, const EmState &S, int64_t g, const PatArgs &A,
                           double *mpat, double *llpat, double *cpat, double *out, unsigned long long *h) {
    const int64_t P = ctx->n_pairs;
    const int fence = ctx->em_fence ? 1 : 0;
    const unsigned grid = (unsigned)g;
    if (ctx->code_bytes == 2)
        k_em_iter<uint16_t, R, FIN><<<grid, HL_THREADS, L.bytes, ctx->stream>>>(
            reinterpret_cast<const uint16_t *>(ctx->codes.p), P, A, S.ticket, mpat, llpat, cpat, out, h, fence, S.arow,
            S.ghot, S.refresh, (int)L.bytes);
    else
        k_em_iter<uint32_t, R, FIN><<<grid, HL_THREADS, L.bytes, ctx->stream>>>(
            reinterpret_cast<const uint32_t *>(ctx->codes.p), P, A, S.ticket, mpat, llpat, cpat, out, h, fence, S.arow,
            S.ghot, S.refresh, (int)L.bytes);
}

template <bool FIN>
static int launch_em_lanes(spk_ctx *ctx, const LanePlan &L, const PatArgs &A, double *mpat, double *llpat,
                           double *cpat, double *out, unsigned long long *h) {
    EmState S;
    SPK_TRY(em_state(ctx, S));
    const int64_t g = lane_grid(ctx);
    if (S.refresh && L.R < 64) {  // a new pair set: guess the uncounted pattern before the first launch
        const size_t shm = (size_t)ctx->n_patterns * 4;
        if (ctx->code_bytes == 2)
            k_em_hot_sample<uint16_t><<<1, HS_THREADS, shm, ctx->stream>>>(
                reinterpret_cast<const uint16_t *>(ctx->codes.p), ctx->n_pairs, (int)ctx->n_patterns, S.ghot);
        else
            k_em_hot_sample<uint32_t><<<1, HS_THREADS, shm, ctx->stream>>>(
                reinterpret_cast<const uint32_t *>(ctx->codes.p), ctx->n_pairs, (int)ctx->n_patterns, S.ghot);
    }
    switch (L.R) {
        case 64: launch_em_iter<64, FIN>(ctx, L, S, g, A, mpat, llpat, cpat, out, h); break;
        case 32: launch_em_iter<32, FIN>(ctx, L, S, g, A, mpat, llpat, cpat, out, h); break;
        case 16: launch_em_iter<16, FIN>(ctx, L, S, g, A, mpat, llpat, cpat, out, h); break;
        case 8: launch_em_iter<8, FIN>(ctx, L, S, g, A, mpat, llpat, cpat, out, h); break;
        default: launch_em_iter<4, FIN>(ctx, L, S, g, A, mpat, llpat, cpat, out, h); break;
    }
    SPK_HIP(hipGetLastError());
    return SPK_OK;
}

// Each translation unit's kernels are one code object, loaded by HIP at the first launch of any of them:
// about 1.2 ms of host time that landed between the first E+M launch's timing events on MI355X (a 0.42 ms
// kernel timed at 1.67 ms; rocprofv3 kernel trace, profiles/r5_fulljob_em_trace.txt).  The first E+M call
// of a process launches an empty k_pattern_mp before its events instead.  (Loading it in spk_ctx_create
// with hipFuncGetAttributes cost 0.55 s of job setup: it loaded far more than this code object.)
static int em_load_code_object(spk_ctx *ctx) {
    static bool loaded[64] = {};  // per device (the code object is loaded per device)
    const int d = ctx->device;
    if (d < 64 && loaded[d]) return SPK_OK;
    PatArgs A{};
    k_pattern_mp<<<1, 64, 0, ctx->stream>>>(A, nullptr, nullptr);  // n_pat = 0: no thread does anything
    SPK_HIP(hipGetLastError());
    if (d < 64) loaded[d] = true;
    return SPK_OK;
}

// The pattern histogram into d_hist (NULL = the context's).
static int enqueue_histogram(spk_ctx *ctx, uint64_t *d_hist) {
    const int64_t n_pat = ctx->n_patterns;
    unsigned long long *h = reinterpret_cast<unsigned long long *>(d_hist);
    if (!h) {
        SPK_TRY(ctx->hist.alloc((size_t)n_pat));
        h = reinterpret_cast<unsigned long long *>(ctx->hist.p);
    }
    const int64_t P = ctx->n_pairs;
    const int vec = 16 / ctx->code_bytes;
    const LanePlan L = lane_plan(ctx);
    if (L.R) SPK_TRY(em_state_alloc(ctx));
    SPK_TRY(em_load_code_object(ctx));
    SPK_TRY(ctx->begin(K_EMHIST));
    if (L.R) {
        PatArgs A{};
        A.n_pat = (int)n_pat;
        SPK_TRY(launch_em_lanes<false>(ctx, L, A, nullptr, nullptr, nullptr, nullptr, h));
    } else {
        SPK_HIP(hipMemsetAsync(h, 0, (size_t)n_pat * 8, ctx->stream));
        int64_t blocks = (P / vec + H_THREADS - 1) / H_THREADS;
        if (blocks > 4 * (int64_t)ctx->n_cu) blocks = 4 * (int64_t)ctx->n_cu;
        if (blocks < 1) blocks = 1;
        const bool lds = n_pat <= H_LDS_BINS;
        const size_t shm = lds ? (size_t)n_pat * 4 : 0;
        if (ctx->code_bytes == 2) {
            if (lds) k_hist<uint16_t, true><<<(unsigned)blocks, H_THREADS, shm, ctx->stream>>>(
                reinterpret_cast<const uint16_t *>(ctx->codes.p), P, (int)n_pat, h);
            else k_hist<uint16_t, false><<<(unsigned)blocks, H_THREADS, 0, ctx->stream>>>(
                reinterpret_cast<const uint16_t *>(ctx->codes.p), P, (int)n_pat, h);
        } else {
            if (lds) k_hist<uint32_t, true><<<(unsigned)blocks, H_THREADS, shm, ctx->stream>>>(
                reinterpret_cast<const uint32_t *>(ctx->codes.p), P, (int)n_pat, h);
            else k_hist<uint32_t, false><<<(unsigned)blocks, H_THREADS, 0, ctx->stream>>>(
                reinterpret_cast<const uint32_t *>(ctx->codes.p), P, (int)n_pat, h);
        }
    }
    SPK_HIP(hipGetLastError());
    SPK_TRY(ctx->end(K_EMHIST));
    return SPK_OK;
}

static int em_buffers(spk_ctx *ctx, int n_stats) {
    SPK_TRY(ctx->stats.alloc((size_t)n_stats));
    SPK_TRY(ctx->pinned_stats(n_stats));
    SPK_TRY(ctx->mpat.alloc((size_t)ctx->n_patterns));
    SPK_TRY(ctx->llpat.alloc((size_t)ctx->n_patterns));
    SPK_TRY(ctx->cpat.alloc((size_t)ctx->n_patterns));
    return SPK_OK;
}

// E-step + M-step sums from the histogram h (one workgroup), statistics copied to out_stats.
static int finalize_from(spk_ctx *ctx, const unsigned long long *h, const PatArgs &A, double *out_stats, int n_stats) {
    SPK_REQUIRE(!ctx->em_pending, SPK_E_STATE, "spk_em_finalize: an asynchronous iteration is pending (spk_em_iteration_wait)");
    SPK_TRY(em_buffers(ctx, n_stats));
    SPK_TRY(ctx->begin(K_EMFIN));
    k_em_finalize<<<1, EF_THREADS, 0, ctx->stream>>>(A, h, ctx->mpat.p, ctx->llpat.p, ctx->cpat.p, ctx->stats.p);
    SPK_HIP(hipGetLastError());
    SPK_TRY(ctx->end(K_EMFIN));
    SPK_HIP(hipMemcpyAsync(ctx->h_stats, ctx->stats.p, (size_t)n_stats * 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    std::memcpy(out_stats, ctx->h_stats, (size_t)n_stats * 8);
    return SPK_OK;
}

extern "C" int spk_em_set_lane_histogram(spk_ctx *ctx, int on) {
    SPK_REQUIRE(ctx && on >= 0 && on <= 2, SPK_E_INVALID, "spk_em_set_lane_histogram: mode 0, 1 or 2");
    ctx->hist_lanes = on != 0;
    ctx->em_fence = on != 2;
    return SPK_OK;
}

extern "C" int spk_em_histogram(spk_ctx *ctx, uint64_t *d_hist) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    SPK_REQUIRE(ctx->codes_valid, SPK_E_STATE, "spk_em_histogram: no gammas");
    SPK_HIP(hipSetDevice(ctx->device));
    SPK_TRY(enqueue_histogram(ctx, d_hist));
    if (d_hist) {
        // a caller-owned histogram is all-reduced over ranks next: it must be final when this returns
        SPK_HIP(hipStreamSynchronize(ctx->stream));
        bool fixed = false;
        SPK_TRY(settle_gammas(ctx, &fixed));
        if (fixed) {
            SPK_TRY(enqueue_histogram(ctx, d_hist));
            SPK_HIP(hipStreamSynchronize(ctx->stream));
        }
    }
    return SPK_OK;
}

extern "C" int spk_em_finalize(spk_ctx *ctx, const uint64_t *d_hist, double lambda, double one_minus, const double *m,
                               const double *u, double *out_stats, int n_stats) {
    SPK_REQUIRE(ctx && m && u && out_stats, SPK_E_INVALID, "spk_em_finalize: null arg");
    SPK_REQUIRE(ctx->codes_valid, SPK_E_STATE, "spk_em_finalize: no gammas");
    SPK_HIP(hipSetDevice(ctx->device));
    PatArgs A;
    SPK_TRY(pat_args(ctx, lambda, one_minus, m, u, A));
    SPK_REQUIRE(n_stats == N_HEAD + 4 * A.n_slots, SPK_E_INVALID, "spk_em_finalize: n_stats mismatch");
    const unsigned long long *h = reinterpret_cast<const unsigned long long *>(d_hist ? d_hist : ctx->hist.p);
    SPK_REQUIRE(h, SPK_E_STATE, "spk_em_finalize: no histogram");
    SPK_TRY(finalize_from(ctx, h, A, out_stats, n_stats));
    bool fixed = false;
    SPK_TRY(settle_gammas(ctx, &fixed));
    if (fixed && !d_hist) {  // the codes changed after the histogram was taken: take it again
        SPK_TRY(enqueue_histogram(ctx, nullptr));
        SPK_TRY(finalize_from(ctx, h, A, out_stats, n_stats));
    }
    return SPK_OK;
}

// Enqueue one E+M iteration on the current codes with the arguments saved in ctx (em_*): the statistics
// are copied to the pinned h_stats and ev_stats is recorded behind them.  No host synchronisation on the
// lane-histogram path (one launch); pattern spaces past the lane-private counters take the histogram +
// finalize launches.
static int enqueue_em(spk_ctx *ctx) {
    PatArgs A;
    SPK_TRY(pat_args(ctx, ctx->em_lambda, ctx->em_one_minus, ctx->em_m.data(), ctx->em_u.data(), A));
    const int n_stats = ctx->em_n_stats;
    SPK_REQUIRE(n_stats == N_HEAD + 4 * A.n_slots, SPK_E_INVALID, "spk_em_iteration: n_stats mismatch");
    SPK_TRY(em_buffers(ctx, n_stats));
    SPK_TRY(em_load_code_object(ctx));
    const LanePlan L = lane_plan(ctx);
    if (!L.R) {
        SPK_TRY(enqueue_histogram(ctx, nullptr));
        SPK_TRY(ctx->begin(K_EMFIN));
        k_em_finalize<<<1, EF_THREADS, 0, ctx->stream>>>(A, reinterpret_cast<const unsigned long long *>(ctx->hist.p),
                                                         ctx->mpat.p, ctx->llpat.p, ctx->cpat.p, ctx->stats.p);
        SPK_HIP(hipGetLastError());
        SPK_TRY(ctx->end(K_EMFIN));
    } else {
        SPK_TRY(em_state_alloc(ctx));
        SPK_TRY(ctx->begin(K_EMHIST));
        SPK_TRY(launch_em_lanes<true>(ctx, L, A, ctx->mpat.p, ctx->llpat.p, ctx->cpat.p, ctx->stats.p, nullptr));
        SPK_TRY(ctx->end(K_EMHIST));
        ctx->ev_used[0][K_EMFIN] = ctx->ev_used[1][K_EMFIN] = false;  // one launch: the E-step is inside it
    }
    SPK_HIP(hipMemcpyAsync(ctx->h_stats, ctx->stats.p, (size_t)n_stats * 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipEventRecord(ctx->ev_stats, ctx->stream));
    return SPK_OK;
}

namespace spk {
int em_requeue(spk_ctx *ctx) { return enqueue_em(ctx); }

}  // namespace spk



#ifdef SPK_EM_STAMPS
extern "C" int spk_debug_em_stamps(uint64_t *out) {
    SPK_HIP(hipDeviceSynchronize());
    SPK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_em_stamps), sizeof(uint64_t) * 16));
    return SPK_OK;
}
#endif

extern "C" int spk_em_iteration_start(spk_ctx *ctx, double lambda, double one_minus, const double *m, const double *u,
                                      int n_stats) {
    SPK_REQUIRE(ctx && m && u, SPK_E_INVALID, "spk_em_iteration_start: null arg");
    SPK_REQUIRE(ctx->codes_valid, SPK_E_STATE, "spk_em_iteration_start: no gammas");
    SPK_REQUIRE(!ctx->em_pending, SPK_E_STATE, "spk_em_iteration_start: the previous iteration was not waited for");
    SPK_HIP(hipSetDevice(ctx->device));
    int tot = 0;
    for (int k = 0; k < ctx->K; ++k) tot += ctx->n_levels[k];
    ctx->em_lambda = lambda;
    ctx->em_one_minus = one_minus;
    ctx->em_m.assign(m, m + tot);
    ctx->em_u.assign(u, u + tot);
    ctx->em_n_stats = n_stats;
    ctx->em_kind = 0;
    SPK_TRY(enqueue_em(ctx));
    ctx->em_pending = true;
    ctx->em_seq = ctx->gamma_seq;
    return SPK_OK;
}

extern "C" int spk_em_histogram_async(spk_ctx *ctx, uint64_t *d_hist) {
    SPK_REQUIRE(ctx && d_hist, SPK_E_INVALID, "spk_em_histogram_async: null arg");
    SPK_REQUIRE(ctx->codes_valid, SPK_E_STATE, "spk_em_histogram_async: no gammas");
    SPK_HIP(hipSetDevice(ctx->device));
    // the codes must be final before they are counted: every rank then reduces exactly one histogram
    // per iteration (a correction after the collective could not be repeated on one rank alone)
    SPK_TRY(settle_gammas(ctx, nullptr));
    return enqueue_histogram(ctx, d_hist);
}

extern "C" int spk_em_finalize_start(spk_ctx *ctx, const uint64_t *d_hist, double lambda, double one_minus,
                                     const double *m, const double *u, int n_stats) {
    SPK_REQUIRE(ctx && d_hist && m && u, SPK_E_INVALID, "spk_em_finalize_start: null arg");
    SPK_REQUIRE(ctx->codes_valid, SPK_E_STATE, "spk_em_finalize_start: no gammas");
    SPK_REQUIRE(!ctx->em_pending, SPK_E_STATE, "spk_em_finalize_start: the previous iteration was not waited for");
    SPK_HIP(hipSetDevice(ctx->device));
    PatArgs A;
    SPK_TRY(pat_args(ctx, lambda, one_minus, m, u, A));
    SPK_REQUIRE(n_stats == N_HEAD + 4 * A.n_slots, SPK_E_INVALID, "spk_em_finalize_start: n_stats mismatch");
    SPK_TRY(em_buffers(ctx, n_stats));
    SPK_TRY(ctx->begin(K_EMFIN));
    k_em_finalize<<<1, EF_THREADS, 0, ctx->stream>>>(A, reinterpret_cast<const unsigned long long *>(d_hist),
                                                     ctx->mpat.p, ctx->llpat.p, ctx->cpat.p, ctx->stats.p);
    SPK_HIP(hipGetLastError());
    SPK_TRY(ctx->end(K_EMFIN));
    SPK_HIP(hipMemcpyAsync(ctx->h_stats, ctx->stats.p, (size_t)n_stats * 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipEventRecord(ctx->ev_stats, ctx->stream));
    ctx->em_n_stats = n_stats;
    ctx->em_kind = 1;
    ctx->em_pending = true;
    ctx->em_seq = ctx->gamma_seq;
    return SPK_OK;
}

extern "C" int spk_em_iteration_wait(spk_ctx *ctx, double *out_stats, int n_stats) {
    SPK_REQUIRE(ctx && out_stats, SPK_E_INVALID, "spk_em_iteration_wait: null arg");
    SPK_REQUIRE(ctx->em_pending, SPK_E_STATE, "spk_em_iteration_wait: no iteration started");
    SPK_REQUIRE(n_stats == ctx->em_n_stats, SPK_E_INVALID, "spk_em_iteration_wait: n_stats mismatch");
    SPK_HIP(hipSetDevice(ctx->device));
    // the codes' info block first: a correction of the codes re-enqueues this iteration (settle_gammas)
    if (ctx->em_seq == ctx->gamma_seq) SPK_TRY(settle_gammas(ctx, nullptr));
    SPK_HIP(hipEventSynchronize(ctx->ev_stats));
    std::memcpy(out_stats, ctx->h_stats, (size_t)n_stats * 8);
    ctx->em_pending = false;
    return SPK_OK;
}

extern "C" int spk_em_iteration(spk_ctx *ctx, double lambda, double one_minus, const double *m, const double *u,
                                double *out_stats, int n_stats) {
    SPK_TRY(spk_em_iteration_start(ctx, lambda, one_minus, m, u, n_stats));
    return spk_em_iteration_wait(ctx, out_stats, n_stats);
}

extern "C" int spk_score(spk_ctx *ctx, double lambda, double one_minus, const double *m, const double *u,
                         int64_t start, int64_t count, double *out_mp) {
    SPK_REQUIRE(ctx && m && u, SPK_E_INVALID, "spk_score: null arg");
    SPK_REQUIRE(ctx->codes_valid, SPK_E_STATE, "spk_score: no gammas");
    SPK_REQUIRE(start >= 0 && count >= 0 && start + count <= ctx->n_pairs, SPK_E_INVALID, "spk_score: range");
    SPK_HIP(hipSetDevice(ctx->device));
    SPK_TRY(settle_gammas(ctx, nullptr));
    PatArgs A;
    SPK_TRY(pat_args(ctx, lambda, one_minus, m, u, A));
    SPK_TRY(ctx->mpat_score.alloc((size_t)ctx->n_patterns));
    SPK_TRY(ctx->mp.alloc((size_t)ctx->n_pairs + 1));
    SPK_TRY(ctx->begin(K_SCORE));
    k_pattern_mp<<<(unsigned)((ctx->n_patterns + 255) / 256), 256, 0, ctx->stream>>>(A, ctx->mpat_score.p, nullptr);
    SPK_HIP(hipGetLastError());
    ctx->mpat_valid = true;
    ++ctx->score_seq;
    if (count) {
        int64_t g = (count / 2 + SC_THREADS - 1) / SC_THREADS;
        if (g > SC_WG_PER_CU * (int64_t)ctx->n_cu) g = SC_WG_PER_CU * (int64_t)ctx->n_cu;  // grid-stride
        if (g < 1) g = 1;
        const int np = (int)ctx->n_patterns;
        const bool lds = ctx->n_patterns <= SC_LDS_PAT;  // LDS table: 0.795 ms vs 0.828 from L1 (368M pairs)
        const auto *c16 = reinterpret_cast<const uint16_t *>(ctx->codes.p);
        const auto *c32 = reinterpret_cast<const uint32_t *>(ctx->codes.p);
        double *o = ctx->mp.p + start;
        const size_t shm = lds ? (size_t)np * 8 : 0;
        if (ctx->code_bytes == 2) {
            if (lds) k_score<uint16_t, true><<<(unsigned)g, SC_THREADS, shm, ctx->stream>>>(c16, start, count, ctx->mpat_score.p, np, o);
            else k_score<uint16_t, false><<<(unsigned)g, SC_THREADS, 0, ctx->stream>>>(c16, start, count, ctx->mpat_score.p, np, o);
        } else {
            if (lds) k_score<uint32_t, true><<<(unsigned)g, SC_THREADS, shm, ctx->stream>>>(c32, start, count, ctx->mpat_score.p, np, o);
            else k_score<uint32_t, false><<<(unsigned)g, SC_THREADS, 0, ctx->stream>>>(c32, start, count, ctx->mpat_score.p, np, o);
        }
        SPK_HIP(hipGetLastError());
    }
    SPK_TRY(ctx->end(K_SCORE));
    if (out_mp && count)
        SPK_HIP(hipMemcpyAsync(out_mp, ctx->mp.p + start, (size_t)count * 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    return SPK_OK;
}

