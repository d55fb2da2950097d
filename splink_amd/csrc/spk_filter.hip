// Filter pass over the template-shaped comparison columns (case_statements.py:62-246: the strict
// equality, Jaro-Winkler, Levenshtein and numeric templates), one lane per pair.
//
// Every such column is "WHEN x_l IS NULL OR x_r IS NULL THEN n  WHEN test_1 THEN l_1 ... ELSE e" over
// the same two operands.  On the host each column's chain of tests is folded into a few constants
// per decision case (FJw / FLev / FEq below), so the device decides a cell with a handful of compares
// and selects from the two rows' image fields:
//   equality   equal dictionary ids -> lv_same, else lv_diff;
//   JW         equal strings -> the level of 1.0, no common unit -> the level of 0.0, otherwise the
//              sketch / head-unit upper bound either proves every remaining test false (one compare
//              against the smallest threshold: lv_bound) or leaves the cell to the exact pass;
//   Levenshtein  the distance lies in [max(length gap, bag distance), max length]; the tests that can
//              still hold for unequal strings are a short chain of integer compares (threshold tables
//              of the ratio tests in LDS).
// The class loops are unrolled to a fixed maximum with wave-uniform guards, so the kernel has no
// per-column dispatch and keeps every column's parameters in scalar registers.  Cells a bound does
// not settle go to the column's work list for the exact pass (spk_gamma.hip).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "spk_gamma.h"

namespace spk {

enum LevKind : int32_t { LK_GE = 0, LK_LE = 1, LK_EXACT = 2, LK_RATIO = 3 };

struct FCommon {
    int64_t p0, p1;        // byte offset of the chunk plane holding the column's field, side 0 / side 1
    uint32_t in;           // byte offset of the field inside its 16-byte chunk (0 or 8)
    uint32_t stride;       // code stride of the column
    int32_t k;             // comparison column (work list)
    int32_t null_level;
    int64_t imp_lo, imp_hi;  // pairs whose level the blocking key implies (SimpleCol.imp_lo / imp_hi)
    uint32_t imp_add;        // (eq_level + 1) * stride
    int32_t und_same;        // equal keys without dictionary ids: the exact pass compares the units
    int ws;
};

struct FEq {
    FCommon c;
    int32_t lv_same, lv_diff;
    int32_t eq4;  // a 4-byte id field (SimpleCol.eq4): compare the ids, all ones = NULL
};

struct FJw {
    FCommon c;
    int64_t h0, h1;  // planes of the four head units (low 8 bytes of the next chunk)
    int32_t lv_one, lv_zero, lv_bound;
    float cf;        // undecided iff the fp32 upper bound >= cf (+inf: never)
    // Equality columns in the high half of the head chunk (layout_image puts EQ fields in those gaps:
    // one 8-byte field, or two 4-byte id fields): one 16-byte load per side serves them all, instead
    // of separate loads.  ge[q].c.in = 8 or 12 says which half.
    int32_t geq;  // gap equality columns (0 .. 2)
    FEq ge[2];
};

struct FLev {
    FCommon c;
    int32_t lv_same, lv_same_empty, lv_else;
    int32_t n;  // the chain of tests that can hold for unequal strings
    int32_t kind[MAX_TESTS], a[MAX_TESTS], cmp[MAX_TESTS], level[MAX_TESTS];
    double t[MAX_TESTS];
};

struct FNum {
    FCommon c;
    int32_t null_level, else_level, n_tests;
    int32_t op[MAX_TESTS], cmp[MAX_TESTS], level[MAX_TESTS];
    double t[MAX_TESTS];
};

struct FiltArgs {
    const int32_t *pl, *pr;
    const uint8_t *img0, *img1;
    uint32_t plane0, plane1;  // bytes of one chunk plane of each image (rows x 16)
    void *codes;
    int32_t *work;
    unsigned int *region_count;
    int64_t P, region_len;
    int n_regions, region_base;
    const int16_t *thr;
    int n_thr;
    int nj, nl, ne, nn;
    FJw jw[FJ_MAX];
    FLev lev[FL_MAX];
    FEq eq[FE_MAX];
    FNum num[FN_MAX];
};
static_assert(sizeof(FiltArgs) <= 4096, "kernel argument size");

// Loads of one field of FP pairs' rows (ox / oy = row x 16) from the planes of a column.
template <int FP>
__device__ __attribute__((always_inline)) inline void load16(const FiltArgs &A, int64_t p0, int64_t p1,
                                                             const uint32_t (&ox)[FP], const uint32_t (&oy)[FP],
                                                             uint4 (&a)[FP], uint4 (&b)[FP]) {
    const __amdgpu_buffer_rsrc_t r0 = image_rsrc(A.img0 + p0, A.plane0), r1 = image_rsrc(A.img1 + p1, A.plane1);
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(r0, ox[u], 0, 0);
        const u32x4_t y = __builtin_amdgcn_raw_buffer_load_b128(r1, oy[u], 0, 0);
        a[u] = make_uint4(x.x, x.y, x.z, x.w);
        b[u] = make_uint4(y.x, y.y, y.z, y.w);
    }
}

template <int FP>
__device__ __attribute__((always_inline)) inline void load8(const FiltArgs &A, int64_t p0, int64_t p1, uint32_t in,
                                                            const uint32_t (&ox)[FP], const uint32_t (&oy)[FP],
                                                            uint2 (&a)[FP], uint2 (&b)[FP]) {
    const __amdgpu_buffer_rsrc_t r0 = image_rsrc(A.img0 + p0, A.plane0), r1 = image_rsrc(A.img1 + p1, A.plane1);
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        const u32x2_t x = __builtin_amdgcn_raw_buffer_load_b64(r0, ox[u] + in, 0, 0);
        const u32x2_t y = __builtin_amdgcn_raw_buffer_load_b64(r1, oy[u] + in, 0, 0);
        a[u] = make_uint2(x.x, x.y);
        b[u] = make_uint2(y.x, y.y);
    }
}

// Append the undecided cells of one column to its region's work list (one LDS atomic per wave).
template <int FP>
__device__ __attribute__((always_inline)) inline void append(const FiltArgs &A, const FCommon &c, int64_t r0,
                                                             unsigned int *cnt, const bool (&und)[FP],
                                                             const uint32_t (&p)[FP]) {
    unsigned long long m[FP];
    unsigned int total = 0;
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        m[u] = __ballot(und[u]);
        total += (unsigned int)__popcll(m[u]);
    }
    if (!total) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    unsigned int base = 0;
    if (lane == 0) base = atomicAdd(cnt, total);
    base = __shfl(base, 0);
    int32_t *list = A.work + (int64_t)c.ws * A.P + r0;
    const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        if (und[u]) list[base + __popcll(m[u] & below)] = (int32_t)p[u];
        base += (unsigned int)__popcll(m[u]);
    }
}

// A per-column constant held in a scalar register.  The level a lane takes is a select among a column's constants
// (`nul ? null_level : same ? lv_same : lv_diff`); written on the kernel-argument fields directly, the compiler
// turned that into a select of their ADDRESSES and one per-lane vector load of the chosen field, followed by
// s_waitcnt vmcnt(0) -- a wait on every load in flight, the next pairs' rows included -- once per column, pair
// group and iteration (12 of ~38 vector-memory instructions per 192 pairs, round-6 ISA).  readfirstlane makes the
// operands values, not loads, so the select is a v_cndmask between scalar registers.
__device__ __attribute__((always_inline)) inline uint32_t sconst(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
// (level + 1) * stride: the amount a level adds to the pair's code
__device__ __attribute__((always_inline)) inline uint32_t sadd(int32_t level, uint32_t stride) {
    return sconst((uint32_t)(level + 1) * stride);
}

__device__ __attribute__((always_inline)) inline bool implied(const FCommon &c, int64_t base, int64_t span) {
    return base >= c.imp_lo && base + span <= c.imp_hi;  // wave-uniform
}

// ---- Jaro-Winkler template column ---------------------------------------------------------------------
// jaro_winkler_sim(l, r) > / >= t tests.  The upper bound (sketch intersection for the matches,
// (m - t)/m <= 1, the head units for the Winkler prefix) is evaluated in fp32 with a 1e-5 margin, far
// above its rounding; it is computed only when some lane of the wave needs it.
template <int FP>
struct JwData {
    uint4 a[FP], b[FP];
    uint4 qa[FP], qb[FP];  // head chunk: head units in .x / .y, the gap EQ field (if any) in .z / .w
};
template <int FP>
__device__ __attribute__((always_inline)) inline void ld_jw(const FiltArgs &A, const FJw &J, const uint32_t (&ox)[FP],
                                                            const uint32_t (&oy)[FP], JwData<FP> &d) {
    load16<FP>(A, J.c.p0, J.c.p1, ox, oy, d.a, d.b);
    if (J.geq) {  // kernel-argument (wave-uniform) branch
        load16<FP>(A, J.h0, J.h1, ox, oy, d.qa, d.qb);
    } else {
        uint2 ha[FP], hb[FP];
        load8<FP>(A, J.h0, J.h1, 0, ox, oy, ha, hb);
#pragma unroll
        for (int u = 0; u < FP; ++u) {
            d.qa[u] = make_uint4(ha[u].x, ha[u].y, 0u, 0u);
            d.qb[u] = make_uint4(hb[u].x, hb[u].y, 0u, 0u);
        }
    }
}
template <int FP>
__device__ __attribute__((always_inline)) inline void ev_jw(const FJw &J, const JwData<FP> &d, const bool (&act)[FP],
                                                            uint32_t (&acc)[FP], bool (&und)[FP]) {
    const uint4(&a)[FP] = d.a;
    const uint4(&b)[FP] = d.b;
    uint2 ha[FP], hb[FP];
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        ha[u] = make_uint2(d.qa[u].x, d.qa[u].y);
        hb[u] = make_uint2(d.qb[u].x, d.qb[u].y);
    }
    bool same[FP], nul[FP], zero[FP];
    int lf[FP], ls[FP];
    bool need = false;
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        same[u] = a[u].x == b[u].x && a[u].y == b[u].y;
        nul[u] = a[u].y == LENS_NULL || b[u].y == LENS_NULL;
        lf[u] = lens_u16(a[u].y);
        ls[u] = lens_u16(b[u].y);
        zero[u] = (lf[u] < ls[u] ? lf[u] : ls[u]) == 0;
        need = need || !(same[u] || zero[u] || nul[u]);
    }
    float hi[FP];
#pragma unroll
    for (int u = 0; u < FP; ++u) hi[u] = 0.f;
    if (__any(need)) {
#pragma unroll
        for (int u = 0; u < FP; ++u) {
            const int lmn = lf[u] < ls[u] ? lf[u] : ls[u], lmx = lf[u] < ls[u] ? ls[u] : lf[u];
            const int M = sketch_inter_ub_bf(img_sketch(a[u]), img_sketch(b[u]), lf[u], ls[u]);
            zero[u] = zero[u] || M == 0;
            // v_rcp_f32 (1 ulp) instead of IEEE divisions: the error (< 1e-6 on j) sits far inside the
            // 1e-5 margin, so hi stays an upper bound (the exact cases never read it)
            const float j = ((float)M * (float)(lf[u] + ls[u]) * __builtin_amdgcn_rcpf((float)lf[u] * (float)ls[u]) +
                             1.0f) * (1.0f / 3.0f);
            const uint32_t dlo = ha[u].x ^ hb[u].x, dhi = ha[u].y ^ hb[u].y;
            const int cp = dlo ? (__builtin_ctz(dlo) >> 4) : (dhi ? 2 + (__builtin_ctz(dhi) >> 4) : 4);
            const int prefix = cp < 4 ? (cp < lmn ? cp : lmn) : lmn;
            const float pw = (lmx > 10 ? __builtin_amdgcn_rcpf((float)lmx) : 0.1f) * (float)prefix;
            hi[u] = (j >= 0.7f - 1e-4f ? j + pw * (1.0f - j) : j) + 1e-5f;
        }
    }
    const uint32_t a_one = sadd(J.lv_one, J.c.stride), a_zero = sadd(J.lv_zero, J.c.stride);
    const uint32_t a_bound = sadd(J.lv_bound, J.c.stride), a_null = sadd(J.c.null_level, J.c.stride);
    const bool und_same = sconst((uint32_t)J.c.und_same) != 0;
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        const bool sat = lf[u] >= LEN_SAT || ls[u] >= LEN_SAT;
        const bool exact = same[u] || zero[u];
        const uint32_t add = same[u] ? (lf[u] > 0 ? a_one : a_zero) : (zero[u] ? a_zero : a_bound);
        const bool u0 = (same[u] && und_same) || sat || (!exact && hi[u] >= J.cf);
        und[u] = act[u] && !nul[u] && u0;
        acc[u] += und[u] ? 0u : (nul[u] ? a_null : add);
    }
}
template <int FP>
__device__ __attribute__((always_inline)) inline void f_jw(const FiltArgs &A, const FJw &J, const uint32_t (&ox)[FP],
                                                           const uint32_t (&oy)[FP], const bool (&act)[FP],
                                                           uint32_t (&acc)[FP], bool (&und)[FP]) {
    JwData<FP> d;
    ld_jw<FP>(A, J, ox, oy, d);
    ev_jw<FP>(J, d, act, acc, und);
}

// ---- Levenshtein template column ---------------------------------------------------------------------
template <int FP>
struct Data16 {
    uint4 a[FP], b[FP];
};
template <int FP>
__device__ __attribute__((always_inline)) inline void ev_lev(const FLev &L, const int16_t *s_thr, const Data16<FP> &d,
                                                             const bool (&act)[FP], uint32_t (&acc)[FP], bool (&und)[FP]) {
    const uint4(&a)[FP] = d.a;
    const uint4(&b)[FP] = d.b;
    bool same[FP], nul[FP], bmp[FP], u0[FP];
    int lo[FP], hi[FP], S[FP];
    bool need = false;
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        same[u] = a[u].x == b[u].x && a[u].y == b[u].y;
        nul[u] = a[u].y == LENS_NULL || b[u].y == LENS_NULL;
        const int la = lens_u16(a[u].y), lb = lens_u16(b[u].y), na = lens_cp(a[u].y), nb = lens_cp(b[u].y);
        u0[u] = (same[u] && L.c.und_same) || la >= LEN_SAT || lb >= LEN_SAT || na >= LEN_SAT || nb >= LEN_SAT;
        bmp[u] = na == la && nb == lb && !same[u] && !nul[u];  // BMP rows: units are code points (bag bound)
        need = need || bmp[u];
        lo[u] = na > nb ? na - nb : nb - na;
        hi[u] = na > nb ? na : nb;
        S[u] = na + nb;
    }
    if (__any(need)) {
#pragma unroll
        for (int u = 0; u < FP; ++u) {
            const int na = lens_cp(a[u].y), nb = lens_cp(b[u].y);
            const int bag = hi[u] - sketch_inter_ub_bf(img_sketch(a[u]), img_sketch(b[u]), na, nb);
            lo[u] = (bmp[u] && bag > lo[u]) ? bag : lo[u];
        }
    }
    Chain ch[FP];
#pragma unroll
    for (int u = 0; u < FP; ++u) ch[u] = Chain(L.lv_else);
    // The templates' shape (levenshtein_3 / _4: one or two ratio tests with threshold tables) with the
    // test parameters at constant indices: read once, not per test through a dynamic kernel-argument
    // index (a dependent scalar load per test and pair group).
    bool fast = (L.n == 1 || L.n == 2) && L.kind[0] == LK_RATIO && L.a[0] >= 0 &&
                (L.n == 1 || (L.kind[1] == LK_RATIO && L.a[1] >= 0));
    if (fast) {
        bool narrow = true;
#pragma unroll
        for (int u = 0; u < FP; ++u) narrow = narrow && S[u] < THR_S;
        fast = !__any(!narrow);
    }
    if (fast) {
        const int a0 = L.a[0], lv0 = L.level[0];
#pragma unroll
        for (int u = 0; u < FP; ++u) {
            const int th = s_thr[a0 + S[u]];
            ch[u].fold(hi[u] <= th ? KT : (lo[u] > th ? KF : KU), lv0);
        }
        if (L.n == 2) {
            const int a1 = L.a[1], lv1 = L.level[1];
#pragma unroll
            for (int u = 0; u < FP; ++u) {
                const int th = s_thr[a1 + S[u]];
                ch[u].fold(hi[u] <= th ? KT : (lo[u] > th ? KF : KU), lv1);
            }
        }
    }
    for (int i = 0; i < (fast ? 0 : L.n); ++i) {  // wave-uniform: the tests unequal strings can still pass
        const int kind = L.kind[i], A_ = L.a[i], lv = L.level[i];
        if (kind == LK_RATIO) {
            // integer thresholds from the table when len_l + len_r < THR_S, else the fp64 bound with one
            // part in 1e12 of margin (exact ties left to the exact pass)
            int r[FP];
            bool wide = false;
#pragma unroll
            for (int u = 0; u < FP; ++u) {
                const bool tab = A_ >= 0 && S[u] < THR_S;
                wide = wide || !tab;
                const int th = tab ? s_thr[A_ + S[u]] : 0;
                r[u] = !tab ? KU : (hi[u] <= th ? KT : (lo[u] > th ? KF : KU));
            }
            if (__any(wide)) {
                const double t = L.t[i];
                const int cmp = L.cmp[i];
#pragma unroll
                for (int u = 0; u < FP; ++u) {
                    if (A_ >= 0 && S[u] < THR_S) continue;
                    const double tl = t * ((double)S[u] * 0.5), up = tl * (1.0 + 1e-12), dn = tl * (1.0 - 1e-12);
                    const double tl_hi = up > dn ? up : dn, tl_lo = up > dn ? dn : up;
                    r[u] = cmp == SPK_CMP_LE ? ((double)hi[u] <= tl_lo ? KT : ((double)lo[u] > tl_hi ? KF : KU))
                                             : ((double)hi[u] < tl_lo ? KT : ((double)lo[u] >= tl_hi ? KF : KU));
                }
            }
#pragma unroll
            for (int u = 0; u < FP; ++u) ch[u].fold(r[u], lv);
        } else {
#pragma unroll
            for (int u = 0; u < FP; ++u) {
                int r;
                if (kind == LK_EXACT) r = lo[u] == hi[u] ? cmpd((double)lo[u], L.t[i], L.cmp[i]) : KU;
                else if (kind == LK_GE) r = lo[u] >= A_ ? KT : (hi[u] < A_ ? KF : KU);
                else r = hi[u] <= A_ ? KT : (lo[u] > A_ ? KF : KU);
                ch[u].fold(r, lv);
            }
        }
    }
    const uint32_t stride = sconst(L.c.stride);
    const int lv_same = (int)sconst((uint32_t)L.lv_same), lv_same_empty = (int)sconst((uint32_t)L.lv_same_empty);
    const int null_level = (int)sconst((uint32_t)L.c.null_level);
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        const int lv = same[u] ? (lens_u16(a[u].y) > 0 ? lv_same : lv_same_empty) : ch[u].lvl;
        und[u] = act[u] && !nul[u] && (u0[u] || (!same[u] && ch[u].und));
        const int level = nul[u] ? null_level : lv;
        acc[u] += und[u] ? 0u : (uint32_t)(level + 1) * stride;
    }
}
template <int FP>
__device__ __attribute__((always_inline)) inline void f_lev(const FiltArgs &A, const FLev &L, const int16_t *s_thr,
                                                            const uint32_t (&ox)[FP], const uint32_t (&oy)[FP],
                                                            const bool (&act)[FP], uint32_t (&acc)[FP],
                                                            bool (&und)[FP]) {
    Data16<FP> d;
    load16<FP>(A, L.c.p0, L.c.p1, ox, oy, d.a, d.b);
    ev_lev<FP>(L, s_thr, d, act, acc, und);
}

// ---- strict-equality template column -----------------------------------------------------------------
template <int FP>
struct Data8 {
    uint2 a[FP], b[FP];
};
template <int FP>
__device__ __attribute__((always_inline)) inline void ev_eq(const FEq &E, const Data8<FP> &d, const bool (&act)[FP],
                                                            uint32_t (&acc)[FP], bool (&und)[FP]) {
    const uint2(&a)[FP] = d.a;
    const uint2(&b)[FP] = d.b;
    const uint32_t a_same = sadd(E.lv_same, E.c.stride), a_diff = sadd(E.lv_diff, E.c.stride);
    const uint32_t a_null = sadd(E.c.null_level, E.c.stride);
    const bool und_same = sconst((uint32_t)E.c.und_same) != 0;
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        const bool same = a[u].x == b[u].x && a[u].y == b[u].y;
        const bool nul = a[u].y == LENS_NULL || b[u].y == LENS_NULL;
        und[u] = act[u] && !nul && same && und_same;
        acc[u] += und[u] ? 0u : (nul ? a_null : (same ? a_same : a_diff));
    }
}
// A gap equality column from the high half (z, w) of the head chunks: the 8-byte field, or the 4-byte id at
// byte 8 (z) or 12 (w) of the chunk.
template <int FP>
__device__ __attribute__((always_inline)) inline void ev_gap_eq(const FEq &E, const uint2 (&ha)[FP], const uint2 (&hb)[FP],
                                                                const bool (&act)[FP], uint32_t (&acc)[FP],
                                                                bool (&und)[FP]) {
    if (E.eq4) {  // kernel-argument (wave-uniform) branch
        const bool hi = E.c.in == 12;
        const uint32_t a_same = sadd(E.lv_same, E.c.stride), a_diff = sadd(E.lv_diff, E.c.stride);
        const uint32_t a_null = sadd(E.c.null_level, E.c.stride);
#pragma unroll
        for (int u = 0; u < FP; ++u) {
            const uint32_t a = hi ? ha[u].y : ha[u].x, b = hi ? hb[u].y : hb[u].x;
            const bool nul = a == 0xFFFFFFFFu || b == 0xFFFFFFFFu;
            und[u] = false;  // ids: equal ids are equal strings
            acc[u] += nul ? a_null : (a == b ? a_same : a_diff);
        }
        (void)act;
        return;
    }
    Data8<FP> d;
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        d.a[u] = ha[u];
        d.b[u] = hb[u];
    }
    ev_eq<FP>(E, d, act, acc, und);
}

template <int FP>
__device__ __attribute__((always_inline)) inline void f_eq(const FiltArgs &A, const FEq &E, const uint32_t (&ox)[FP],
                                                           const uint32_t (&oy)[FP], const bool (&act)[FP],
                                                           uint32_t (&acc)[FP], bool (&und)[FP]) {
    Data8<FP> d;
    load8<FP>(A, E.c.p0, E.c.p1, E.c.in, ox, oy, d.a, d.b);
    ev_eq<FP>(E, d, act, acc, und);
}

// ---- numeric template column --------------------------------------------------------------------------
template <int FP>
__device__ __attribute__((always_inline)) inline void f_num(const FiltArgs &A, const FNum &N, const uint32_t (&ox)[FP],
                                                            const uint32_t (&oy)[FP], uint32_t (&acc)[FP]) {
    uint4 a[FP], b[FP];
    load16<FP>(A, N.c.p0, N.c.p1, ox, oy, a, b);
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        const int level = simple_num(N, a[u].z != 0, bits_to_double(a[u].x, a[u].y), b[u].z != 0,
                                     bits_to_double(b[u].x, b[u].y));
        acc[u] += (uint32_t)(level + 1) * N.c.stride;
    }
}

constexpr int N_FCOLS = FJ_MAX + FL_MAX + FE_MAX + FN_MAX;

// One workgroup per region of consecutive pair ordinals; each lane takes FP pairs per iteration (the
// next iteration's pair rows are in flight meanwhile).  Per column: the FP pairs' field loads, then
// their evaluation, then one wave-aggregated append of the undecided cells.
template <int FP, int MINW, bool C32>
__global__ __launch_bounds__(F_THREADS, MINW) void k_filter(const FiltArgs A) {
    __shared__ unsigned int s_cnt[N_FCOLS + FJ_MAX];  // work-list lengths: per column slot, then JW gap EQs
    extern __shared__ int16_t s_thr[];  // A.thr (dynamic LDS: n_thr entries)
    if (threadIdx.x < N_FCOLS + FJ_MAX) s_cnt[threadIdx.x] = 0;
    for (int i = threadIdx.x; i < A.n_thr; i += F_THREADS) s_thr[i] = A.thr[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t r0 = (int64_t)(A.region_base + blockIdx.x) * A.region_len;
    const int64_t r1 = r0 + A.region_len < A.P ? r0 + A.region_len : A.P;
    constexpr int SPAN = 64 * FP;
    constexpr int STEP = (F_THREADS / 64) * SPAN;
    const uint32_t end = (uint32_t)r1;
    uint32_t base = (uint32_t)r0 + (uint32_t)(threadIdx.x >> 6) * SPAN;
    int32_t nx[FP], ny[FP];
    // pair rows of the lane's next pairs: unconditional loads at clamped ordinals (inactive lanes re-read the
    // region's last pair harmlessly), so no divergent branch sits between them and the field gathers
    const uint32_t last = end > (uint32_t)r0 ? end - 1 : (uint32_t)r0;
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        const uint32_t q = base + u * 64 + lane;
        nx[u] = A.pl[q < end ? q : last];
        ny[u] = A.pr[q < end ? q : last];
    }
    for (; base < end; base += STEP) {  // wave-uniform
        uint32_t p[FP], ox[FP], oy[FP], acc[FP];
        bool act[FP], und[FP];
#pragma unroll
        for (int u = 0; u < FP; ++u) {
            p[u] = base + u * 64 + lane;
            act[u] = p[u] < end;
            ox[u] = (uint32_t)nx[u] << 4;
            oy[u] = (uint32_t)ny[u] << 4;
            acc[u] = 0;
        }
        // The next pairs' rows are requested only after this iteration's row offsets are taken from the last
        // ones: hoisted above the shifts, the loads made the compiler wait for them right there (s_waitcnt
        // vmcnt(0) at the loop head), so every iteration paid the pair-row and the field-gather round trips one
        // after the other instead of together.
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < FP; ++u) {
            const uint32_t q = p[u] + STEP;
            nx[u] = A.pl[q < end ? q : last];
            ny[u] = A.pr[q < end ? q : last];
        }
#pragma unroll 1
        for (int j = 0; j < A.nj; ++j) {
            const FJw &J = A.jw[j];
            const bool ji = implied(J.c, base, SPAN);
            bool gi[2] = {false, false}, gneed = false;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                gi[q] = q < J.geq && implied(J.ge[q].c, base, SPAN);
                gneed = gneed || (q < J.geq && !gi[q]);
            }
            if (ji) {
#pragma unroll
                for (int u = 0; u < FP; ++u) acc[u] += act[u] ? J.c.imp_add : 0u;
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (!gi[q]) continue;
#pragma unroll
                for (int u = 0; u < FP; ++u) acc[u] += act[u] ? J.ge[q].c.imp_add : 0u;
            }
            uint2 ga[FP], gb[FP];  // the head chunks' high halves: the gap equality fields
            if (ji) {
                if (!gneed) continue;
                load8<FP>(A, J.h0, J.h1, 8, ox, oy, ga, gb);  // only the gap fields are needed
            } else {
                JwData<FP> d;
                ld_jw<FP>(A, J, ox, oy, d);
                ev_jw<FP>(J, d, act, acc, und);
                append<FP>(A, J.c, r0, &s_cnt[j], und, p);
#pragma unroll
                for (int u = 0; u < FP; ++u) {
                    ga[u] = make_uint2(d.qa[u].z, d.qa[u].w);
                    gb[u] = make_uint2(d.qb[u].z, d.qb[u].w);
                }
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (q >= J.geq || gi[q]) continue;
                ev_gap_eq<FP>(J.ge[q], ga, gb, act, acc, und);
                if (J.ge[q].c.und_same) append<FP>(A, J.ge[q].c, r0, &s_cnt[N_FCOLS + j], und, p);
            }
        }
#pragma unroll 1
        for (int j = 0; j < A.nl; ++j) {
            const FLev &L = A.lev[j];
            if (implied(L.c, base, SPAN)) {
#pragma unroll
                for (int u = 0; u < FP; ++u) acc[u] += act[u] ? L.c.imp_add : 0u;
                continue;
            }
            f_lev<FP>(A, L, s_thr, ox, oy, act, acc, und);
            append<FP>(A, L.c, r0, &s_cnt[FJ_MAX + j], und, p);
        }
#pragma unroll 1
        for (int j = 0; j < A.ne; ++j) {
            const FEq &E = A.eq[j];
            if (implied(E.c, base, SPAN)) {
#pragma unroll
                for (int u = 0; u < FP; ++u) acc[u] += act[u] ? E.c.imp_add : 0u;
                continue;
            }
            f_eq<FP>(A, E, ox, oy, act, acc, und);
            if (E.c.und_same) append<FP>(A, E.c, r0, &s_cnt[FJ_MAX + FL_MAX + j], und, p);
        }
#pragma unroll 1
        for (int j = 0; j < A.nn; ++j) {
            f_num<FP>(A, A.num[j], ox, oy, acc);
        }
#pragma unroll
        for (int u = 0; u < FP; ++u) {
            if (!act[u]) continue;
            if (C32) static_cast<uint32_t *>(A.codes)[p[u]] = acc[u];
            else static_cast<uint16_t *>(A.codes)[p[u]] = (uint16_t)acc[u];
        }
    }
    __syncthreads();
    const int64_t slot = A.region_base + blockIdx.x;
    const int t = threadIdx.x;
    if (t < A.nj) A.region_count[(int64_t)A.jw[t].c.k * A.n_regions + slot] = s_cnt[t];
    else if (t >= FJ_MAX && t < FJ_MAX + A.nl) A.region_count[(int64_t)A.lev[t - FJ_MAX].c.k * A.n_regions + slot] = s_cnt[t];
    else if (t >= FJ_MAX + FL_MAX && t < FJ_MAX + FL_MAX + A.ne)
        A.region_count[(int64_t)A.eq[t - FJ_MAX - FL_MAX].c.k * A.n_regions + slot] = s_cnt[t];
    else if (t >= FJ_MAX + FL_MAX + FE_MAX && t < FJ_MAX + FL_MAX + FE_MAX + A.nn)
        A.region_count[(int64_t)A.num[t - FJ_MAX - FL_MAX - FE_MAX].c.k * A.n_regions + slot] = 0;
    else if (t >= N_FCOLS && t < N_FCOLS + A.nj && A.jw[t - N_FCOLS].geq) {
        // a gap with two id fields appends nothing (ids); an 8-byte field is alone in its gap
        const FJw &J = A.jw[t - N_FCOLS];
        A.region_count[(int64_t)J.ge[0].c.k * A.n_regions + slot] = s_cnt[t];
        if (J.geq > 1) A.region_count[(int64_t)J.ge[1].c.k * A.n_regions + slot] = 0;
    }
}

// ---- host: the per-column decision constants --------------------------------------------------------------
static bool hcmp(double a, double b, int cmp) {
    switch (cmp) {
        case SPK_CMP_EQ: return a == b;
        case SPK_CMP_NE: return a != b;
        case SPK_CMP_LT: return a < b;
        case SPK_CMP_LE: return a <= b;
        case SPK_CMP_GT: return a > b;
        default: return a >= b;
    }
}

static void common(const SimpleCol &s, const GammaArgs &A, int off, FCommon &c) {
    c.p0 = (int64_t)(off >> 4) * A.img_rows0 * 16;
    c.p1 = (int64_t)(off >> 4) * A.img_rows1 * 16;
    c.in = (uint32_t)(off & 15);
    c.stride = (uint32_t)s.stride;
    c.k = s.k;
    c.ws = A.wslot[s.k];
    c.null_level = s.null_level;
    c.imp_lo = s.imp_lo;
    c.imp_hi = s.imp_hi;
    c.imp_add = (uint32_t)(s.eq_level + 1) * (uint32_t)s.stride;
    c.und_same = s.has_ids ? 0 : 1;
}

// The level a chain of `=` / `<>` tests gives when the equality is `eq`.
static int32_t eq_chain(const SimpleCol &s, bool eq) {
    for (int i = 0; i < s.n_tests; ++i)
        if ((s.cmp[i] == SPK_CMP_EQ) == eq) return s.level[i];
    return s.else_level;
}

static void make_jw(const SimpleCol &s, const GammaArgs &A, FJw &J) {
    common(s, A, s.off, J.c);
    J.h0 = (int64_t)(s.off2 >> 4) * A.img_rows0 * 16;
    J.h1 = (int64_t)(s.off2 >> 4) * A.img_rows1 * 16;
    auto first_pass = [&](double v) {
        for (int i = 0; i < s.n_tests; ++i)
            if (hcmp(v, s.t[i], s.cmp[i])) return s.level[i];
        return s.else_level;
    };
    J.lv_one = first_pass(1.0);
    J.lv_zero = first_pass(0.0);
    // bound cells: a test that 0.0 passes holds for every value (jw >= 0, tests are `>` / `>=`) and ends
    // the chain; each test before it is false iff hi < its float threshold (prepare_tests), so the cell
    // is decided iff hi is below the smallest of them
    J.lv_bound = s.else_level;
    J.cf = INFINITY;
    for (int i = 0; i < s.n_tests; ++i) {
        if (hcmp(0.0, s.t[i], s.cmp[i])) {
            J.lv_bound = s.level[i];
            break;
        }
        J.cf = std::min(J.cf, s.jw_cf[i]);
    }
}

static void make_lev(const SimpleCol &s, const GammaArgs &A, FLev &L) {
    common(s, A, s.off, L.c);
    // equal strings: `=` holds, the distance is 0 and its ratio 0.0 (NULL when both are empty: den = 0)
    auto same_level = [&](bool empty) {
        for (int i = 0; i < s.n_tests; ++i) {
            const int op = s.op[i];
            bool r;
            if (op == SPK_OP_STR_CMP) r = s.cmp[i] == SPK_CMP_EQ;
            else if (op == SPK_OP_LEV) r = hcmp(0.0, s.t[i], s.cmp[i]);
            else r = !empty && hcmp(0.0, s.t[i], s.cmp[i]);  // SPK_OP_LEVRATIO
            if (r) return s.level[i];
        }
        return s.else_level;
    };
    L.lv_same = same_level(false);
    L.lv_same_empty = same_level(true);
    // unequal strings: `=` is false (dropped), `<>` true (ends the chain), the distance tests remain
    L.n = 0;
    L.lv_else = s.else_level;
    for (int i = 0; i < s.n_tests; ++i) {
        const int op = s.op[i];
        if (op == SPK_OP_STR_CMP) {
            if (s.cmp[i] == SPK_CMP_EQ) continue;
            L.lv_else = s.level[i];
            break;
        }
        const int n = L.n++;
        L.level[n] = s.level[i];
        L.cmp[n] = s.cmp[i];
        L.t[n] = s.t[i];
        if (op == SPK_OP_LEVRATIO) {
            L.kind[n] = LK_RATIO;
            L.a[n] = s.thr_off[i];
        } else {
            L.kind[n] = (s.tflag[i] & TF_EXACT) ? LK_EXACT : ((s.tflag[i] & TF_GE) ? LK_GE : LK_LE);
            L.a[n] = s.lev_a[i];
        }
    }
}

static void make_eq(const SimpleCol &s, const GammaArgs &A, FEq &E) {
    common(s, A, s.off, E.c);
    E.lv_same = eq_chain(s, true);
    E.lv_diff = eq_chain(s, false);
    E.eq4 = s.eq4;
}

static void make_num(const SimpleCol &s, const GammaArgs &A, FNum &N) {
    common(s, A, s.off, N.c);
    N.null_level = s.null_level;
    N.else_level = s.else_level;
    N.n_tests = s.n_tests;
    for (int i = 0; i < MAX_TESTS; ++i) {
        N.op[i] = s.op[i];
        N.cmp[i] = s.cmp[i];
        N.level[i] = s.level[i];
        N.t[i] = s.t[i];
    }
}

int launch_template_filter(hipStream_t stream, const GammaArgs &A, const std::vector<SimpleCol> &simple,
                           int64_t region_lo, int64_t region_hi) {
    if (region_hi <= region_lo || simple.empty()) return SPK_OK;
    SPK_REQUIRE(A.img_rows0 <= IMG_MAX_ROWS && A.img_rows1 <= IMG_MAX_ROWS, SPK_E_LIMIT,
                "spk_gammas: more than 2^27 rows in one table (row-image planes are limited to 2^31 bytes)");
    FiltArgs F;
    std::memset(&F, 0, sizeof(F));
    F.pl = A.pl;
    F.pr = A.pr;
    F.img0 = A.img0;
    F.img1 = A.img1;
    F.plane0 = (uint32_t)(A.img_rows0 * 16);
    F.plane1 = (uint32_t)(A.img_rows1 * 16);
    F.codes = A.codes;
    F.work = A.work;
    F.region_count = A.region_count;
    F.P = A.P;
    F.region_len = A.region_len;
    F.n_regions = A.n_regions;
    F.region_base = (int)region_lo;
    F.thr = A.thr;
    F.n_thr = A.n_thr;
    std::vector<int> jw_off2;  // head-chunk offset of each JW slot
    for (const SimpleCol &s : simple) {
        switch (s.cls) {
            case SC_JW:
                SPK_REQUIRE(F.nj < FJ_MAX, SPK_E_INVALID, "filter: JW slots");
                jw_off2.push_back(s.off2);
                make_jw(s, A, F.jw[F.nj++]);
                break;
            case SC_LEV: SPK_REQUIRE(F.nl < FL_MAX, SPK_E_INVALID, "filter: LEV slots"); make_lev(s, A, F.lev[F.nl++]); break;
            case SC_EQ: break;  // below
            case SC_NUM: SPK_REQUIRE(F.nn < FN_MAX, SPK_E_INVALID, "filter: NUM slots"); make_num(s, A, F.num[F.nn++]); break;
            default: SPK_REQUIRE(false, SPK_E_INVALID, "filter: column without a filter class");
        }
    }
    for (const SimpleCol &s : simple) {
        if (s.cls != SC_EQ) continue;
        int host = -1;  // a JW slot whose head chunk's high half holds this column's field
        for (int j = 0; j < F.nj && host < 0; ++j)
            if (F.jw[j].geq < 2 && (jw_off2[j] & 15) == 0 && s.off >= jw_off2[j] + 8 && s.off < jw_off2[j] + 16 &&
                (s.eq4 || s.off == jw_off2[j] + 8))
                host = j;
        if (host >= 0) {
            make_eq(s, A, F.jw[host].ge[F.jw[host].geq++]);
            continue;
        }
        SPK_REQUIRE(!s.eq4, SPK_E_INVALID, "filter: a 4-byte equality field outside a JW gap");
        SPK_REQUIRE(F.ne < FE_MAX, SPK_E_INVALID, "filter: EQ slots");
        make_eq(s, A, F.eq[F.ne++]);
    }
    const unsigned g = (unsigned)(region_hi - region_lo);
    const size_t shm = (size_t)A.n_thr * sizeof(int16_t);
    // 3 pairs per lane per step at a register budget for 5 waves per SIMD (94 VGPRs): the best point of the
    // round-4 sweep (<2,6> / <4,4> slower, <3,6> / <2,8> spill: profiles/r4_ab_filter_occupancy.log)
#ifndef SPK_FILTER_FP
#define SPK_FILTER_FP 3
#endif
#ifndef SPK_FILTER_MINW
#define SPK_FILTER_MINW 5
#endif
    constexpr int FP = SPK_FILTER_FP, MINW = SPK_FILTER_MINW;
    if (A.code16) k_filter<FP, MINW, false><<<g, F_THREADS, shm, stream>>>(F);
    else k_filter<FP, MINW, true><<<g, F_THREADS, shm, stream>>>(F);
    SPK_HIP(hipGetLastError());
    return SPK_OK;
}

}  // namespace spk

