// Device string similarity: the jar's Jaro-Winkler (commons-text 1.4 JaroWinklerDistance,
// SURVEY.md §2.3) and Spark's Levenshtein, exact, plus the cheap bounds the comparison filter
// pass uses to decide most (pair, column) cells without running them.
//
// Exactness: jw_finish evaluates the reference's expression in its exact operation order; the
// library is compiled with -ffp-contract=off so no FMA contraction changes the rounding.
#pragma once

#include <cmath>
#include <type_traits>

#include "spk_internal.h"

namespace spk {

constexpr int MAXU = 64;          // LDS staging capacity per string (UTF-16 units), exact pass
constexpr int SLOW_LIMIT = 1024;  // slow pass: per-lane scratch arrays up to this many units per string;
                                  // longer strings go to the huge pass (device scratch sized to the data)

struct StrView {
    const uint16_t *p = nullptr;
    int32_t n = 0;     // UTF-16 units
    int32_t ncp = 0;   // code points
    int32_t null = 1;
    int32_t has_meta = 0;   // key / sketch valid
    int32_t exact_key = 0;  // column + 1 when `key` is that column's dictionary id, else 0
    uint32_t key = 0;
    uint64_t sketch = 0;
    const uint64_t *planes = nullptr;  // N_PLANES bit-planes of the whole row, or null
};

__device__ inline StrView plain_view(const uint16_t *p, int32_t n, int32_t ncp) {
    StrView s;
    s.p = p;
    s.n = n;
    s.ncp = ncp;
    s.null = 0;
    return s;
}

// ---- accessors ---------------------------------------------------------------------------
template <int STRIDE>
struct LdsAcc {
    const uint16_t *b;
    __device__ uint16_t operator[](int i) const { return b[i * STRIDE]; }
};
struct GlbAcc {
    const uint16_t *p;
    __device__ uint16_t operator[](int i) const { return p[i]; }
};

// Element i of one lane's array in a device scratch buffer shared by `s` lanes, interleaved so that
// lanes stepping through the same index touch consecutive words.
template <typename T>
struct Strided {
    T *p;
    int64_t s;
    __device__ T &operator[](int i) const { return p[(int64_t)i * s]; }
};

// Device scratch of the huge pass (strings longer than SLOW_LIMIT units): n_slots lanes, lane `slot`
// owns elements slot, slot + n_slots, ... of each typed view of `base`.  `units` bounds every string
// the pass can meet (the longest row of any string column, in UTF-8 bytes >= UTF-16 units, and the
// longest literal); `words` = ceil(units / 64).
struct Scratch {
    uint8_t *base = nullptr;
    int64_t n_slots = 0, slot = 0;
    int32_t units = 0, words = 0;
    template <typename T>
    __device__ Strided<T> at(int64_t elem0) const {
        return Strided<T>{reinterpret_cast<T *>(base) + elem0 * n_slots + slot, n_slots};
    }
};

template <int STRIDE>
__device__ inline void stage(uint16_t *slot, const StrView &s) {
    for (int i = 0; i < s.n; ++i) slot[i * STRIDE] = s.p[i];
}

__device__ inline bool aligned8(const uint16_t *p) { return ((uintptr_t)p & 7u) == 0; }

// Units [0, lim) compared four at a time when both rows start 8-byte aligned (column rows do;
// substr / literal views may not).  Reads stay inside the row's padded slot.
__device__ inline int common_prefix(const uint16_t *a, const uint16_t *b, int lim) {
    if (aligned8(a) && aligned8(b)) {
        for (int i = 0; i < lim; i += 4) {
            const uint64_t d = *reinterpret_cast<const uint64_t *>(a + i) ^ *reinterpret_cast<const uint64_t *>(b + i);
            if (d) {
                const int k = i + (__ffsll((unsigned long long)d) - 1) / 16;
                return k < lim ? k : lim;
            }
        }
        return lim;
    }
    int i = 0;
    while (i < lim && a[i] == b[i]) ++i;
    return i;
}

// Exact string equality: dictionary ids when both rows carry them, else hash then units.
__device__ inline bool units_equal(const StrView &a, const StrView &b) {
    if (a.n != b.n) return false;
    if (a.has_meta && b.has_meta) {
        // ids are equal iff the strings are, within one column's id space only
        if (a.exact_key && a.exact_key == b.exact_key) return a.key == b.key;
        if (!a.exact_key && !b.exact_key && a.key != b.key) return false;
    }
    return common_prefix(a.p, b.p, a.n) == a.n;
}

// Sequential reader of UTF-16 units: one aligned 8-byte load per four units.  A word is loaded
// only when one of its units is consumed, so the reader never touches memory past the aligned
// word holding the last unit read (safe for unpadded literal buffers too).
struct UnitReader {
    const uint64_t *q;
    uint64_t w;
    int pos;
    bool live;
    __device__ explicit UnitReader(const uint16_t *p) {
        const uintptr_t a = (uintptr_t)p;
        q = reinterpret_cast<const uint64_t *>(a & ~(uintptr_t)7);
        pos = (int)((a & 7u) >> 1);
        w = 0;
        live = false;
    }
    __device__ uint32_t next() {
        if (!live) {
            w = *q;
            live = true;
        }
        const uint32_t c = (uint32_t)(w >> (16 * pos)) & 0xFFFFu;
        if (++pos == 4) {
            pos = 0;
            ++q;
            live = false;
        }
        return c;
    }
};

// ---- Jaro-Winkler (exact) ----------------------------------------------------------------------
// apply(): m = matches, t = transpositions / 2 (integer), prefix not capped, max length lmx.
__device__ inline double jw_finish(int m, int t, int prefix, int lf, int ls, int lmx) {
    if (m == 0) return 0.0;
    double md = (double)m;
    double j = ((md / (double)lf + md / (double)ls) + (md - (double)(t / 2)) / md) / 3.0;
    if (j < 0.7) return j;
    double w = 1.0 / (double)lmx;
    if (w > 0.1) w = 0.1;
    return j + (w * (double)prefix) * (1.0 - j);
}

// matches(): greedy first free match inside the window, strings of <= 64 units (bit-mask flags).
template <class Acc>
__device__ double jw_small(Acc first, int lf, Acc second, int ls) {
    const bool fmax = lf > ls;
    const Acc mx = fmax ? first : second;
    const Acc mn = fmax ? second : first;
    const int lmx = fmax ? lf : ls, lmn = fmax ? ls : lf;
    const int range = lmx / 2 - 1 > 0 ? lmx / 2 - 1 : 0;
    uint64_t flags = 0, matched = 0;
    int m = 0;
    for (int mi = 0; mi < lmn; ++mi) {
        const uint16_t c = mn[mi];
        const int lo = mi - range > 0 ? mi - range : 0;
        const int hi = mi + range + 1 < lmx ? mi + range + 1 : lmx;
        for (int xi = lo; xi < hi; ++xi) {
            if (!((flags >> xi) & 1ull) && mx[xi] == c) {
                flags |= 1ull << xi;
                matched |= 1ull << mi;
                ++m;
                break;
            }
        }
    }
    if (m == 0) return 0.0;
    int t = 0;
    uint64_t fm = flags, mm = matched;
    while (mm) {
        int i = __ffsll((unsigned long long)mm) - 1;
        int x = __ffsll((unsigned long long)fm) - 1;
        t += mn[i] != mx[x];
        mm &= mm - 1;
        fm &= fm - 1;
    }
    int prefix = 0;
    for (int mi = 0; mi < lmn; ++mi) {
        if (first[mi] == second[mi]) ++prefix;
        else break;
    }
    return jw_finish(m, t, prefix, lf, ls, lmx);
}

// Same algorithm for any length: flag words in caller storage (a lane's scratch array up to
// SLOW_LIMIT units, or the huge pass's device scratch); ceil(lmx / 64) + ceil(lmn / 64) words.
template <class Words>
__device__ inline double jw_long(GlbAcc first, int lf, GlbAcc second, int ls, Words flags, Words matched) {
    const bool fmax = lf > ls;
    const GlbAcc mx = fmax ? first : second;
    const GlbAcc mn = fmax ? second : first;
    const int lmx = fmax ? lf : ls, lmn = fmax ? ls : lf;
    const int range = lmx / 2 - 1 > 0 ? lmx / 2 - 1 : 0;
    for (int i = 0; i < (lmx + 63) / 64; ++i) flags[i] = 0;
    for (int i = 0; i < (lmn + 63) / 64; ++i) matched[i] = 0;
    int m = 0;
    for (int mi = 0; mi < lmn; ++mi) {
        const uint16_t c = mn[mi];
        const int lo = mi - range > 0 ? mi - range : 0;
        const int hi = mi + range + 1 < lmx ? mi + range + 1 : lmx;
        for (int xi = lo; xi < hi; ++xi) {
            if (!((flags[xi >> 6] >> (xi & 63)) & 1ull) && mx[xi] == c) {
                flags[xi >> 6] |= 1ull << (xi & 63);
                matched[mi >> 6] |= 1ull << (mi & 63);
                ++m;
                break;
            }
        }
    }
    if (m == 0) return 0.0;
    int t = 0, xi = 0;
    for (int mi = 0; mi < lmn; ++mi) {
        if (!((matched[mi >> 6] >> (mi & 63)) & 1ull)) continue;
        while (!((flags[xi >> 6] >> (xi & 63)) & 1ull)) ++xi;
        t += mn[mi] != mx[xi];
        ++xi;
    }
    int prefix = 0;
    for (int mi = 0; mi < lmn; ++mi) {
        if (first[mi] == second[mi]) ++prefix;
        else break;
    }
    return jw_finish(m, t, prefix, lf, ls, lmx);
}

__device__ inline double jw_long(GlbAcc first, int lf, GlbAcc second, int ls) {  // <= SLOW_LIMIT units
    uint64_t flags[SLOW_LIMIT / 64], matched[SLOW_LIMIT / 64];
    return jw_long(first, lf, second, ls, flags, matched);
}

// ---- Levenshtein (exact) -----------------------------------------------------------------------
// Myers 1999 bit-parallel, pattern <= 64 symbols.
template <class Acc>
__device__ int lev_myers(Acc pat, int m, Acc txt, int n) {
    if (m == 0) return n;
    if (n == 0) return m;
    uint64_t vp = ~0ull, vn = 0;
    const uint64_t hib = 1ull << (m - 1);
    int dist = m;
    for (int j = 0; j < n; ++j) {
        const uint16_t c = txt[j];
        uint64_t eq = 0;
        for (int i = 0; i < m; ++i) eq |= (uint64_t)(pat[i] == c) << i;
        const uint64_t x = eq | vn;
        const uint64_t d0 = (((x & vp) + vp) ^ vp) | x;
        uint64_t hp = vn | ~(d0 | vp);
        uint64_t hn = d0 & vp;
        dist += (hp & hib) ? 1 : 0;
        dist -= (hn & hib) ? 1 : 0;
        hp = (hp << 1) | 1ull;
        hn = hn << 1;
        vp = hn | ~(d0 | hp);
        vn = hp & d0;
    }
    return dist;
}

// Code points, any length: two-row DP with b's code points and the row in caller storage (nb and
// nb + 1 elements).
template <class U32, class I32>
__device__ inline int lev_long(const StrView &a, const StrView &b, U32 cb, I32 row) {
    int nb = 0;
    for (int j = 0; j < b.n; ++j) {
        uint32_t w = b.p[j];
        if (w >= 0xD800 && w < 0xDC00 && j + 1 < b.n) {
            w = 0x10000 + ((w - 0xD800) << 10) + (b.p[j + 1] - 0xDC00);
            ++j;
        }
        cb[nb++] = w;
    }
    for (int j = 0; j <= nb; ++j) row[j] = j;
    int i = 0;
    for (int u = 0; u < a.n; ++u) {
        uint32_t w = a.p[u];
        if (w >= 0xD800 && w < 0xDC00 && u + 1 < a.n) {
            w = 0x10000 + ((w - 0xD800) << 10) + (a.p[u + 1] - 0xDC00);
            ++u;
        }
        ++i;
        int diag = row[0];
        row[0] = i;
        int left = i;
        for (int j = 1; j <= nb; ++j) {
            const int up = row[j];
            int best = diag + (w != cb[j - 1] ? 1 : 0);
            if (up + 1 < best) best = up + 1;
            if (left + 1 < best) best = left + 1;
            row[j] = best;
            left = best;
            diag = up;
        }
    }
    return row[nb];
}

__device__ inline int lev_long(const StrView &a, const StrView &b) {  // <= SLOW_LIMIT units
    uint32_t cb[SLOW_LIMIT];
    int32_t row[SLOW_LIMIT + 1];
    return lev_long(a, b, cb, row);
}

// ---- bounds for the filter pass ---------------------------------------------------------------
// Upper bound of the multiset intersection |a ∩ b| of two unit strings of la / lb units from
// their sketches (spk_internal.h): Σ over buckets of min(count_a, count_b), exact per bucket unless
// both counts are saturated; those buckets together hold at most what the other buckets leave of
// either length.  |a ∩ b| bounds the Jaro match count m from above, and max(la, lb) - |a ∩ b| (the
// bag distance) bounds the Levenshtein distance from below.
__device__ inline int sketch_inter_ub(uint64_t sa, uint64_t sb, int la, int lb) {
    const uint32_t aL = (uint32_t)sa, aH = (uint32_t)(sa >> 32);
    const uint32_t bL = (uint32_t)sb, bH = (uint32_t)(sb >> 32);
    const uint32_t gt = (aH & ~bH) | (~(aH ^ bH) & aL & ~bL);  // buckets where count_a > count_b
    const uint32_t mL = (aL & ~gt) | (bL & gt), mH = (aH & ~gt) | (bH & gt);
    const uint32_t both_sat = aL & aH & bL & bH, rest = ~both_sat;
    int inter = __builtin_popcount(mL & rest) + 2 * __builtin_popcount(mH & rest);
    if (both_sat) {
        const int ra = la - (__builtin_popcount(aL & rest) + 2 * __builtin_popcount(aH & rest));
        const int rb = lb - (__builtin_popcount(bL & rest) + 2 * __builtin_popcount(bH & rest));
        inter += ra < rb ? ra : rb;
    }
    const int lmn = la < lb ? la : lb;
    return inter < lmn ? inter : lmn;
}

__device__ inline uint64_t view_sketch(const StrView &s) {
    if (s.has_meta) return s.sketch;
    uint64_t sk = 0;
    for (int i = 0; i < s.n; ++i) sketch_add(sk, s.p[i]);
    return sk;
}

// Upper bound of jaro_winkler_sim(first, second) for unequal strings.  m <= M from the sketches;
// j <= ((M/lf + M/ls) + 1)/3 since (m - t)/m <= 1; jw = f(j) is non-decreasing in j for the
// actual prefix.  Returns -1 when the bound proves m == 0 (so jw is exactly 0.0).
__device__ inline double jw_upper(const StrView &first, const StrView &second) {
    const int lf = first.n, ls = second.n;
    const int lmn = lf < ls ? lf : ls, lmx = lf < ls ? ls : lf;
    if (lmn == 0) return -1.0;
    const int M = sketch_inter_ub(view_sketch(first), view_sketch(second), lf, ls);
    if (M == 0) return -1.0;
    const int prefix = common_prefix(first.p, second.p, lmn);
    const double md = (double)M;
    const double j = ((md / (double)lf + md / (double)ls) + 1.0) / 3.0;
    if (j < 0.7) return j;
    double w = 1.0 / (double)lmx;
    if (w > 0.1) w = 0.1;
    return j + (w * (double)prefix) * (1.0 - j);
}

// Lower bound of the code-point Levenshtein distance of unequal strings.
__device__ inline int lev_lower(const StrView &a, const StrView &b) {
    int lb = a.ncp > b.ncp ? a.ncp - b.ncp : b.ncp - a.ncp;
    if (a.ncp == a.n && b.ncp == b.n) {  // BMP: units are code points, so the bag bound holds
        const int bag = (a.n > b.n ? a.n : b.n) - sketch_inter_ub(view_sketch(a), view_sketch(b), a.n, b.n);
        if (bag > lb) lb = bag;
    }
    return lb;
}

// ---- bit-plane kernels (exact) -----------------------------------------------------------------
template <typename W>
__device__ inline W mask_below(int k) {  // bits [0, k)
    return k >= (int)(8 * sizeof(W)) ? ~(W)0 : (((W)1 << k) - (W)1);
}

// Positions i of a plane-encoded string with unit i == c (garbage above the string's length).
// Positions i of a plane-encoded string with unit i == c (garbage above the string's length).
template <typename W>
__device__ inline W eq_mask(const W (&pl)[N_PLANES], uint32_t c) {
    W eq = c < 256u ? ~(W)0 : (W)0;
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) eq &= pl[b] ^ ((W)((c >> b) & 1u) - (W)1);
    return eq;
}

// commons-text matches() with the longer string as bit-planes (<= 64 units).  mxp / mnp are the
// longer / shorter strings' units, first / second the original argument order.
template <typename W>
__device__ double jw_planes(const uint64_t *mx_planes, const uint16_t *mxp, int lmx, const uint16_t *mnp, int lmn,
                            const uint16_t *first, int lf, const uint16_t *second, int ls) {
    W pl[N_PLANES];
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) pl[b] = (W)mx_planes[b];
    const int range = lmx / 2 - 1 > 0 ? lmx / 2 - 1 : 0;
    W flags = 0;
    uint64_t matched = 0;
    int m = 0;
    UnitReader rd(mnp);
    for (int mi = 0; mi < lmn; ++mi) {
        const int lo = mi - range > 0 ? mi - range : 0;
        const int hi = mi + range + 1 < lmx ? mi + range + 1 : lmx;
        const W cand = eq_mask<W>(pl, rd.next()) & mask_below<W>(hi) & ~mask_below<W>(lo) & ~flags;
        if (cand) {
            flags |= cand & (~cand + (W)1);  // lowest set bit: the first free match in the window
            matched |= 1ull << mi;
            ++m;
        }
    }
    if (m == 0) return 0.0;
    int t = 0;
    uint64_t mm = matched, fm = (uint64_t)flags;
    while (mm) {
        const int i = __ffsll((unsigned long long)mm) - 1;
        const int x = __ffsll((unsigned long long)fm) - 1;
        t += mnp[i] != mxp[x];
        mm &= mm - 1;
        fm &= fm - 1;
    }
    return jw_finish(m, t, common_prefix(first, second, lmn), lf, ls, lmx);
}

// Myers 1999 with the pattern's match masks from its bit-planes, shifted by `shift` units.
// `cut`: the caller only distinguishes distances up to cut; once the score minus the text still to
// come exceeds it (each remaining text unit lowers the final distance by at most one), the scan
// stops and returns cut + 1.
template <typename W>
__device__ int lev_planes(const uint64_t *planes, int shift, int m, const uint16_t *txt, int n, int cut) {
    W pl[N_PLANES];
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) pl[b] = (W)(planes[b] >> shift);
    W vp = ~(W)0, vn = 0;
    const W hib = (W)1 << (m - 1);
    int dist = m;
    UnitReader rd(txt);
    for (int j = 0; j < n; ++j) {
        const W x = eq_mask<W>(pl, rd.next()) | vn;
        const W d0 = (((x & vp) + vp) ^ vp) | x;
        W hp = vn | ~(d0 | vp);
        W hn = d0 & vp;
        dist += (hp & hib) ? 1 : 0;
        dist -= (hn & hib) ? 1 : 0;
        if (dist - (n - 1 - j) > cut) return cut + 1;
        hp = (hp << 1) | (W)1;
        hn = hn << 1;
        vp = hn | ~(d0 | hp);
        vn = hp & d0;
    }
    return dist;
}

// Myers 1999 with both strings as bit-planes: the pattern's match mask for text unit j is
// AND_b(bit b of unit j ? plane_b : ~plane_b), and bit b of unit j is bit j of the text's plane b,
// so the scan issues no memory access at all.  Per plane and unit: one signed bit-field extract
// (0 or all ones), one bit-select between the plane and its complement, one AND.  P / T are shifted
// to the first unit after the common prefix; bits past m (pattern) and n (text) are ignored.
template <typename W>
__device__ inline W lane_mask(uint32_t m32) {  // 0 / all ones -> W
    return sizeof(W) == 4 ? (W)m32 : (W)(((uint64_t)m32 << 32) | m32);
}

// eq & XNOR(unit-bit mask, plane) as one 3-input bit op per dword (truth table 0x90 = S0 & ~(S1 ^ S2))
__device__ inline uint32_t eq_plane(uint32_t eq, uint32_t mb, uint32_t pl) {
    return __builtin_amdgcn_bitop3_b32(eq, mb, pl, 0x90);
}
__device__ inline uint64_t eq_plane(uint64_t eq, uint32_t mb, uint64_t pl) {
    return ((uint64_t)eq_plane((uint32_t)(eq >> 32), mb, (uint32_t)(pl >> 32)) << 32) |
           eq_plane((uint32_t)eq, mb, (uint32_t)pl);
}

// The score D[m][j+1] is not carried through the scan: after text unit j the vertical deltas give
// it as (j + 1) + popc(VP & M) - popc(VN & M) (row 0 is D[0][j+1] = j + 1, M the pattern's m rows),
// so it is computed only where the cut is tested (every fourth unit) and once at the end.
template <typename W>
__device__ inline int popc_w(W x) {
    return sizeof(W) == 4 ? __builtin_popcount((uint32_t)x) : __builtin_popcountll((unsigned long long)x);
}
template <typename W>
__device__ inline W low_mask(int m) {  // bits [0, m), 1 <= m <= bits of W
    return m >= (int)(8 * sizeof(W)) ? ~(W)0 : (((W)1 << m) - 1);
}

// Early-exit score of the scans (pattern m >= text n): after text unit j, the cell of the end cell's
// diagonal, D[i*][j + 1] with i* = j + 1 + (m - n) = (j + 1) + popc(VP & low i* rows) - popc(VN & ...).
// Values never decrease along a diagonal (Ukkonen), and this one ends at D[m][n], so D[i*][j + 1] > cut
// proves the distance > cut.  It dominates the score-minus-units-left test (D[m][j + 1] <= D[i*][j + 1]
// + (n - j - 1)) and cuts the scan ~18 % earlier on cfg5's dissimilar addresses (host simulation over
// 600 cells).  In the lazy scans the rows that entered late hold upper bounds that differ from the true
// values only where both are > cut, so the test reads the same there.  Used by the 128-bit scans (the
// slow pass, 141 VGPRs); in the 32 / 64-bit scans of the exact pass it pushed that kernel 4 VGPRs past
// its 96-VGPR cap (scratch spills: 67 -> 176 MB of writes per cfg2 call at the same time), so those keep
// the score-minus-units-left test.
template <typename W>
__device__ inline int diag_score(W vp, W vn, int j, int m, int n) {
    const W M = low_mask<W>(j + 1 + (m - n));
    return j + 1 + popc_w(vp & M) - popc_w(vn & M);
}

// NP: the scans read planes 0..NP-1 only.  A caller passes NP < 8 when every unit of the column
// (both sides) has the same bits NP..7 (e.g. 7 for ASCII text): those planes' terms then only touch
// mask bits above the pattern, which never reach the rows below (carries and shifts move upward).
template <typename W, int NP = N_PLANES>
__device__ inline int myers_plane_text(const uint64_t (&P)[N_PLANES], int m, const uint64_t (&T)[N_PLANES], int n,
                                       int cut) {
    W pl[N_PLANES];
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) pl[b] = (W)P[b];
    W vp = ~(W)0, vn = 0;
    const W M = low_mask<W>(m);
    for (int h = 0; h < 2 && 32 * h < n; ++h) {  // text units [32h, 32h + 32) from 32-bit plane words
        uint32_t tw[N_PLANES];
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) tw[b] = (uint32_t)(T[b] >> (32 * h));
        const int jn = n - 32 * h < 32 ? n - 32 * h : 32;
        for (int jj = 0; jj < jn; ++jj) {
            W eq = ~(W)0;
#pragma unroll
            for (int b = 0; b < NP; ++b)
                eq = eq_plane(eq, (uint32_t)__builtin_amdgcn_sbfe((int)tw[b], jj, 1), pl[b]);
            const W x = eq | vn;
            const W d0 = (((x & vp) + vp) ^ vp) | x;
            const W hp = (vn | ~(d0 | vp)) << 1 | (W)1;
            const W hn = (d0 & vp) << 1;
            vp = hn | ~(d0 | hp);
            vn = hp & d0;
            // every fourth unit: the end cell's diagonal (diag_score; it dominates the bound dist - (units
            // left)).  Clamping at the end returns cut + 1 for every cell whose distance passes the cut.
            if ((jj & 3) == 3 && diag_score<W>(vp, vn, 32 * h + jj, m, n) > cut) return cut + 1;
        }
    }
    const int dist = n + popc_w(vp & M) - popc_w(vn & M);
    return dist > cut ? cut + 1 : dist;
}

// Patterns of 33..64 units: the upper word starts late (Ukkonen's cutoff).  D[i][j] >= |i - j|, so a
// cell of a row i >= 33 at text unit j <= 31 - cut is > cut, and a path through it ends > cut.  Rows
// 1..32 never depend on the rows above them, so the scan runs one 32-bit word (pattern rows 1..32,
// the score tracked at row 32) up to text unit J0 <= 31 - cut, then takes the rows above as D[32][J0]
// + (i - 32) (vertical deltas +1, an upper bound of the true values, and > cut where they differ) and
// continues with 64-bit words.  Every distance <= cut comes out exact and every larger one > cut, as
// the callers need; the early exit is taken on the computed scores, which obey the same delta
// bounds.  J0 is the wave's minimum (one switch point for all lanes); lanes with m <= 32 run the
// same loops with their one word.  cfg2 emails: most waves hold a cell of 33+ units, cut ~ 10.
template <int NP = N_PLANES>
__device__ inline int myers_plane_text_lazy(const uint64_t (&P)[N_PLANES], int m, const uint64_t (&T)[N_PLANES], int n,
                                            int cut) {
    const bool wide = m > 32;
    const int mine = wide ? (cut < 31 ? 31 - cut : 0) : 32;
    int lo = 0, hi = 32;  // wave minimum of `mine` (active lanes) by bisection over ballots
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (__ballot(mine <= mid)) hi = mid;
        else lo = mid + 1;
    }
    const int J0 = lo;
    uint32_t pl[N_PLANES], tw[N_PLANES];
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) {
        pl[b] = (uint32_t)P[b];
        tw[b] = (uint32_t)T[b];
    }
    uint32_t vp = ~0u, vn = 0;
    const uint32_t M1 = low_mask<uint32_t>(wide ? 32 : m);  // the rows the first phase scores
    const int j1 = n < J0 ? n : J0;
    for (int j = 0; j < j1; ++j) {
        uint32_t eq = ~0u;
#pragma unroll
        for (int b = 0; b < NP; ++b) eq = eq_plane(eq, (uint32_t)__builtin_amdgcn_sbfe((int)tw[b], j, 1), pl[b]);
        const uint32_t x = eq | vn;
        const uint32_t d0 = (((x & vp) + vp) ^ vp) | x;
        const uint32_t hp = (vn | ~(d0 | vp)) << 1 | 1u;
        const uint32_t hn = (d0 & vp) << 1;
        vp = hn | ~(d0 | hp);
        vn = hp & d0;
        // the end cell's diagonal (diag_score) -- for a wide pattern too: its row i* = j + 1 + m - n <= 31
        // here (m - n <= cut, j < J0 <= 31 - cut) is one of the rows this phase tracks exactly
        if ((j & 3) == 3 && diag_score<uint32_t>(vp, vn, j, m, n) > cut) return cut + 1;
    }
    if (n <= J0) {
        const int dist = n + popc_w(vp & M1) - popc_w(vn & M1) + (wide ? m - 32 : 0);
        return dist > cut ? cut + 1 : dist;
    }
    // rows 33..m enter with vertical deltas +1 (D[32][J0] + (i - 32))
    uint64_t VP = (uint64_t)vp | 0xFFFFFFFF00000000ull, VN = vn;
    const uint64_t M2 = low_mask<uint64_t>(m);
    for (int h = J0 >> 5; h < 2 && 32 * h < n; ++h) {
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) tw[b] = (uint32_t)(T[b] >> (32 * h));
        const int jb = 32 * h < J0 ? J0 - 32 * h : 0;
        const int jn = n - 32 * h < 32 ? n - 32 * h : 32;
        for (int jj = jb; jj < jn; ++jj) {
            uint64_t eq = ~0ull;
#pragma unroll
            for (int b = 0; b < NP; ++b)
                eq = eq_plane(eq, (uint32_t)__builtin_amdgcn_sbfe((int)tw[b], jj, 1), P[b]);
            const uint64_t x = eq | VN;
            const uint64_t d0 = (((x & VP) + VP) ^ VP) | x;
            const uint64_t hp = (VN | ~(d0 | VP)) << 1 | 1ull;
            const uint64_t hn = (d0 & VP) << 1;
            VP = hn | ~(d0 | hp);
            VN = hp & d0;
            if ((jj & 3) == 3 && diag_score<uint64_t>(VP, VN, 32 * h + jj, m, n) > cut) return cut + 1;
        }
    }
    const int dist = n + popc_w(VP & M2) - popc_w(VN & M2);
    return dist > cut ? cut + 1 : dist;
}

// Code-point Levenshtein of two unequal rows that both carry bit-planes (<= 64 units, all < 256, so
// units are code points), from the planes alone: the common prefix is the lowest set bit of
// OR_b(a_b ^ b_b), the common suffix the highest of the same with both strings' ends aligned at bit
// 63; both strips are exact for unit-cost edit distance.  The longer remainder is the pattern, so
// the scan runs over the shorter one.  `cut` as in lev_planes.
template <int NP>
__device__ inline int lev_rows_planes_np(const uint64_t (&pa)[N_PLANES], int la, const uint64_t (&pb)[N_PLANES], int lb,
                                         int cut) {
    if (la == 0) return lb;
    if (lb == 0) return la;
    const int mn = la < lb ? la : lb;
    uint64_t d = 0, e = 0;
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) {
        d |= pa[b] ^ pb[b];
        e |= (pa[b] << (64 - la)) ^ (pb[b] << (64 - lb));
    }
    int pre = d ? __ffsll((unsigned long long)d) - 1 : 64;
    if (pre > mn) pre = mn;
    int suf = e ? __clzll((long long)e) : 64;
    if (suf > mn - pre) suf = mn - pre;
    const int ra = la - pre - suf, rb = lb - pre - suf;
    if (ra == 0) return rb;
    if (rb == 0) return ra;
    const bool a_pat = ra >= rb;
    const int m = a_pat ? ra : rb, n = a_pat ? rb : ra;
    if (m - n > cut) return cut + 1;  // the length gap alone (the lazy scans' diagonal tests rely on m - n <= cut)
    uint64_t P[N_PLANES], T[N_PLANES];
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) {
        P[b] = (a_pat ? pa[b] : pb[b]) >> pre;
        T[b] = (a_pat ? pb[b] : pa[b]) >> pre;
    }
    // one word width for all active lanes: a wave that mixed both would run both loops
    if (!__any(m > 32)) return myers_plane_text<uint32_t, NP>(P, m, T, n, cut);
    return myers_plane_text_lazy<NP>(P, m, T, n, cut);
}

// np: planes the scans need (wave-uniform; see myers_plane_text), 8 when unknown.
__device__ inline int lev_rows_planes(const uint64_t (&pa)[N_PLANES], int la, const uint64_t (&pb)[N_PLANES], int lb,
                                      int cut, int np = N_PLANES) {
    switch (np) {
        case 5: return lev_rows_planes_np<5>(pa, la, pb, lb, cut);
        case 6: return lev_rows_planes_np<6>(pa, la, pb, lb, cut);
        case 7: return lev_rows_planes_np<7>(pa, la, pb, lb, cut);
        default: return lev_rows_planes_np<N_PLANES>(pa, la, pb, lb, cut);
    }
}

// ---- rows of 65..128 units (CPF_PLANES2): the same scan over 128-bit plane words ----------------
// The 128-bit add of Myers' D0 carries from word 0 into word 1 exactly as the multi-block form
// (Hyyro 2003) propagates it; unsigned __int128 is two VGPR pairs and the compiler emits the
// add-with-carry, funnel shifts and per-word logic.
typedef unsigned __int128 u128;

__device__ inline int ctz128(u128 v) {
    const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
    return lo ? __ffsll((unsigned long long)lo) - 1 : (hi ? 64 + __ffsll((unsigned long long)hi) - 1 : 128);
}

__device__ inline int clz128(u128 v) {
    const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
    return hi ? __clzll((long long)hi) : (lo ? 64 + __clzll((long long)lo) : 128);
}

__device__ inline int popc128(u128 x) {
    return __builtin_popcountll((unsigned long long)x) + __builtin_popcountll((unsigned long long)(x >> 64));
}

__device__ inline int diag_score128(u128 vp, u128 vn, int j, int m, int n) {  // diag_score over 128-bit words
    const int i = j + 1 + (m - n);
    const u128 M = i >= 128 ? ~(u128)0 : (((u128)1 << i) - 1);
    return j + 1 + popc128(vp & M) - popc128(vn & M);
}

template <int NP = N_PLANES>
__device__ inline int myers_plane_text128(const u128 (&P)[N_PLANES], int m, const u128 (&T)[N_PLANES], int n,
                                          int cut) {
    u128 vp = ~(u128)0, vn = 0;

    for (int h = 0; h < 4 && 32 * h < n; ++h) {  // text units [32h, 32h + 32)
        uint32_t tw[N_PLANES];
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) tw[b] = (uint32_t)(T[b] >> (32 * h));
        const int jn = n - 32 * h < 32 ? n - 32 * h : 32;
        for (int jj = 0; jj < jn; ++jj) {
            uint64_t e0 = ~0ull, e1 = ~0ull;
#pragma unroll
            for (int b = 0; b < NP; ++b) {
                const uint32_t m32 = (uint32_t)__builtin_amdgcn_sbfe((int)tw[b], jj, 1);
                e0 = eq_plane(e0, m32, (uint64_t)P[b]);
                e1 = eq_plane(e1, m32, (uint64_t)(P[b] >> 64));
            }
            const u128 x = (((u128)e1 << 64) | e0) | vn;
            const u128 d0 = (((x & vp) + vp) ^ vp) | x;
            const u128 hp = (vn | ~(d0 | vp)) << 1 | (u128)1;
            const u128 hn = (d0 & vp) << 1;
            vp = hn | ~(d0 | hp);
            vn = hp & d0;
            if ((jj & 3) == 3 && diag_score128(vp, vn, 32 * h + jj, m, n) > cut) return cut + 1;  // as in myers_plane_text
        }
    }
    const int dist = diag_score128(vp, vn, n - 1, m, n);
    return dist > cut ? cut + 1 : dist;
}

// Patterns of 65..128 units: the upper 64 rows start late, the 64-bit analogue of
// myers_plane_text_lazy (same argument: D[i][j] >= |i - j|, so rows >= 65 cannot hold a distance
// <= cut before text unit 63 - cut).  The scan runs 64-bit words (score tracked at row 64) up to the
// wave's minimum switch point J0, takes rows 65..m as D[64][J0] + (i - 64), and continues with
// 128-bit words.  Free-text columns (cfg5 addresses, cut ~ 0.4 x length) spend about a third of
// their text in the cheaper first phase.
template <int NP = N_PLANES>
__device__ inline int myers_plane_text128_lazy(const u128 (&P)[N_PLANES], int m, const u128 (&T)[N_PLANES], int n,
                                               int cut) {
    const bool wide = m > 64;
    const int mine = wide ? (cut < 63 ? 63 - cut : 0) : 128;
    int lo = 0, hi = 128;  // wave minimum of `mine` (active lanes) by bisection over ballots
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (__ballot(mine <= mid)) hi = mid;
        else lo = mid + 1;
    }
    const int J0 = lo;
    uint64_t pl[N_PLANES];
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) pl[b] = (uint64_t)P[b];
    uint64_t vp = ~0ull, vn = 0;
    const uint64_t M1 = low_mask<uint64_t>(wide ? 64 : m);  // the rows the first phase scores
    const int j1 = n < J0 ? n : J0;
    for (int h = 0; h < 4 && 32 * h < j1; ++h) {
        uint32_t tw[N_PLANES];
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) tw[b] = (uint32_t)(T[b] >> (32 * h));
        const int jn = j1 - 32 * h < 32 ? j1 - 32 * h : 32;
        for (int jj = 0; jj < jn; ++jj) {
            uint64_t eq = ~0ull;
#pragma unroll
            for (int b = 0; b < NP; ++b) eq = eq_plane(eq, (uint32_t)__builtin_amdgcn_sbfe((int)tw[b], jj, 1), pl[b]);
            const uint64_t x = eq | vn;
            const uint64_t d0 = (((x & vp) + vp) ^ vp) | x;
            const uint64_t hp = (vn | ~(d0 | vp)) << 1 | 1ull;
            const uint64_t hn = (d0 & vp) << 1;
            vp = hn | ~(d0 | hp);
            vn = hp & d0;
            // diagonal exit for a wide pattern too: row i* = j + 1 + m - n <= 63 here (m - n <= cut, j < J0 <= 63 - cut)
            if ((jj & 3) == 3 && diag_score<uint64_t>(vp, vn, 32 * h + jj, m, n) > cut) return cut + 1;
        }
    }
    if (n <= J0) {
        const int dist = n + popc_w(vp & M1) - popc_w(vn & M1) + (wide ? m - 64 : 0);
        return dist > cut ? cut + 1 : dist;
    }
    // rows 65..m enter with vertical deltas +1 (D[64][J0] + (i - 64))
    u128 VP = (u128)vp | ((u128)~0ull << 64), VN = vn;

    for (int h = J0 >> 5; h < 4 && 32 * h < n; ++h) {
        uint32_t tw[N_PLANES];
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) tw[b] = (uint32_t)(T[b] >> (32 * h));
        const int jb = 32 * h < J0 ? J0 - 32 * h : 0;
        const int jn = n - 32 * h < 32 ? n - 32 * h : 32;
        for (int jj = jb; jj < jn; ++jj) {
            uint64_t e0 = ~0ull, e1 = ~0ull;
#pragma unroll
            for (int b = 0; b < NP; ++b) {
                const uint32_t m32 = (uint32_t)__builtin_amdgcn_sbfe((int)tw[b], jj, 1);
                e0 = eq_plane(e0, m32, (uint64_t)P[b]);
                e1 = eq_plane(e1, m32, (uint64_t)(P[b] >> 64));
            }
            const u128 x = (((u128)e1 << 64) | e0) | VN;
            const u128 d0 = (((x & VP) + VP) ^ VP) | x;
            const u128 hp = (VN | ~(d0 | VP)) << 1 | (u128)1;
            const u128 hn = (d0 & VP) << 1;
            VP = hn | ~(d0 | hp);
            VN = hp & d0;
            if ((jj & 3) == 3 && diag_score128(VP, VN, 32 * h + jj, m, n) > cut) return cut + 1;
        }
    }
    const int dist = diag_score128(VP, VN, n - 1, m, n);
    return dist > cut ? cut + 1 : dist;
}

// Patterns of 65..128 units in Ukkonen's diagonal band, held in one BW-bit word (Hyyro's banded
// bit-vector form).  With d = i - j (pattern row minus text column) and dm = m - n, a path of cost
// <= cut through a cell needs |d| + |d - dm| <= cut, so only diagonals [dlo, dhi] = [-((cut - dm) >> 1),
// (cut + dm) >> 1] matter: at most cut + 1 of them (cfg5's 65..128-unit addresses: cut <= 52).  At column
// c the word holds the vertical deltas of rows s + 1 .. s + BW with s = max(0, c + dlo - 1), the row above
// it tracked as a score.  Moving to the next column drops the top row into the score (its value becomes
// D[s][c - 1] + 1, the rows entering below take D[row - 1] + 1: both >= the true values, and a cell of an
// optimal path of cost <= cut never reads one of them), and the text unit's match mask is the pattern's
// window [s, s + BW) (a funnel shift of a per-32-column window of the planes).  Every distance <= cut
// comes out exact, every larger one > cut.  The early exit reads the end cell's diagonal as the other
// scans do: from that row the score plus the diagonal gap |d - dm| never decreases along the column (one
// row changes the score by at most 1 and the gap by exactly 1), so a score > cut there bounds every
// cell of the column.  Columns with s = 0 (j <= -dlo) run the plain scan over rows 1..BW first.
// Host emulation against a full DP (180 k random cells, BW = 32 and 64) before building.
template <int NP, int BW>
__device__ inline int myers_plane_text128_band(const u128 (&P)[N_PLANES], int m, const u128 (&T)[N_PLANES], int n,
                                               int cut, int dlo) {
    typedef typename std::conditional<BW == 64, uint64_t, uint32_t>::type W;
    constexpr int NQ = BW / 32 + 1;  // window dwords per plane
    const int dm = m - n;
    const int mine = 1 - dlo;  // columns j < mine have s = 0
    int lo = 0, hi = 128;      // wave minimum by bisection over ballots
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (__ballot(mine <= mid)) hi = mid;
        else lo = mid + 1;
    }
    const int J1 = lo;
    W vp = ~(W)0, vn = 0;
    {
        W pl[N_PLANES];
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) pl[b] = (W)P[b];
        const int j1 = n < J1 ? n : J1;
        for (int h = 0; h < 4 && 32 * h < j1; ++h) {
            uint32_t tw[N_PLANES];
#pragma unroll
            for (int b = 0; b < N_PLANES; ++b) tw[b] = (uint32_t)(T[b] >> (32 * h));
            const int jn = j1 - 32 * h < 32 ? j1 - 32 * h : 32;
            for (int jj = 0; jj < jn; ++jj) {
                W eq = ~(W)0;
#pragma unroll
                for (int b = 0; b < NP; ++b)
                    eq = eq_plane(eq, (uint32_t)__builtin_amdgcn_sbfe((int)tw[b], jj, 1), pl[b]);
                const W x = eq | vn;
                const W d0 = (((x & vp) + vp) ^ vp) | x;
                const W hp = (vn | ~(d0 | vp)) << 1 | (W)1;
                const W hn = (d0 & vp) << 1;
                vp = hn | ~(d0 | hp);
                vn = hp & d0;
                // row i* = j + 1 + dm <= 1 - dlo + dm <= the band's width: inside the word
                if ((jj & 3) == 3 && diag_score<W>(vp, vn, 32 * h + jj, m, n) > cut) return cut + 1;
            }
        }
    }
    if (n <= J1) {  // s = 0 at the end, so m <= the band's width <= BW
        const W M = low_mask<W>(m);
        const int dist = n + popc_w(vp & M) - popc_w(vn & M);
        return dist > cut ? cut + 1 : dist;
    }
    int s = 0, D = 0;  // band offset; deltas of the rows dropped above it (the score of row s is c + D)
    for (int h = J1 >> 5; h < 4 && 32 * h < n; ++h) {
        const int jb = 32 * h < J1 ? J1 - 32 * h : 0;
        const int jn = n - 32 * h < 32 ? n - 32 * h : 32;
        const int sb = 32 * h + jb + dlo > 0 ? 32 * h + jb + dlo : 0;  // s at the chunk's first column
        uint32_t tw[N_PLANES], wq[N_PLANES][NQ];
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) {
            tw[b] = (uint32_t)(T[b] >> (32 * h));
            const u128 v = P[b] >> sb;
#pragma unroll
            for (int q = 0; q < NQ; ++q) wq[b][q] = (uint32_t)(v >> (32 * q));
        }
        for (int jj = jb; jj < jn; ++jj) {
            const int j = 32 * h + jj;
            const uint32_t sh = j + dlo > 0 ? 1u : 0u;
            // the top row leaves the word (its delta into D), a +1 row enters below
            if constexpr (BW == 64) {
                const uint32_t pl0 = (uint32_t)vp, ph0 = (uint32_t)(vp >> 32);
                const uint32_t nl0 = (uint32_t)vn, nh0 = (uint32_t)(vn >> 32);
                D += (int)__builtin_amdgcn_ubfe(pl0, 0, sh) - (int)__builtin_amdgcn_ubfe(nl0, 0, sh);
                vp = ((uint64_t)__builtin_amdgcn_alignbit(~0u, ph0, sh) << 32) | __builtin_amdgcn_alignbit(ph0, pl0, sh);
                vn = ((uint64_t)__builtin_amdgcn_alignbit(0u, nh0, sh) << 32) | __builtin_amdgcn_alignbit(nh0, nl0, sh);
            } else {
                D += (int)__builtin_amdgcn_ubfe((uint32_t)vp, 0, sh) - (int)__builtin_amdgcn_ubfe((uint32_t)vn, 0, sh);
                vp = __builtin_amdgcn_alignbit(~0u, (uint32_t)vp, sh);
                vn = __builtin_amdgcn_alignbit(0u, (uint32_t)vn, sh);
            }
            s += (int)sh;
            const uint32_t k = (uint32_t)(s - sb);  // 0..31
            uint32_t e[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) e[q] = ~0u;
#pragma unroll
            for (int b = 0; b < NP; ++b) {
                const uint32_t tb = (uint32_t)__builtin_amdgcn_sbfe((int)tw[b], jj, 1);
#pragma unroll
                for (int q = 0; q < NQ; ++q) e[q] = eq_plane(e[q], tb, wq[b][q]);
            }
            W eq;
            if constexpr (BW == 64)
                eq = ((uint64_t)__builtin_amdgcn_alignbit(e[2], e[1], k) << 32) | __builtin_amdgcn_alignbit(e[1], e[0], k);
            else
                eq = __builtin_amdgcn_alignbit(e[1], e[0], k);
            const W x = eq | vn;
            const W d0 = (((x & vp) + vp) ^ vp) | x;
            const W hp = (vn | ~(d0 | vp)) << 1 | (W)1;
            const W hn = (d0 & vp) << 1;
            vp = hn | ~(d0 | hp);
            vn = hp & d0;
            if ((jj & 3) == 3) {  // the end cell's diagonal, row j + 1 + dm: bit j + dm - s of the word
                const W M = low_mask<W>(j + 1 + dm - s);
                if (j + 1 + D + popc_w(vp & M) - popc_w(vn & M) > cut) return cut + 1;
            }
        }
    }
    const W M = low_mask<W>(m - s);
    const int dist = n + D + popc_w(vp & M) - popc_w(vn & M);
    return dist > cut ? cut + 1 : dist;
}

// lev_rows_planes for rows of up to 128 units held as 128-bit planes (bits past a row's length are
// zero).  After the common prefix and suffix are stripped, a pattern of <= 64 units runs the
// one-word scan (the same word width for the whole wave), else the banded scan in 32- or 64-bit words
// when every lane's band fits one (the same width for the whole wave), else the 128-bit one.
template <int NP>
__device__ inline int lev_rows_planes128_np(const u128 (&pa)[N_PLANES], int la, const u128 (&pb)[N_PLANES], int lb,
                                            int cut) {
    if (la == 0) return lb;
    if (lb == 0) return la;
    const int mn = la < lb ? la : lb;
    u128 d = 0, e = 0;
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) {
        d |= pa[b] ^ pb[b];
        e |= (pa[b] << (128 - la)) ^ (pb[b] << (128 - lb));
    }
    int pre = ctz128(d);
    if (pre > mn) pre = mn;
    int suf = clz128(e);
    if (suf > mn - pre) suf = mn - pre;
    const int ra = la - pre - suf, rb = lb - pre - suf;
    if (ra == 0) return rb;
    if (rb == 0) return ra;
    const bool a_pat = ra >= rb;
    const int m = a_pat ? ra : rb, n = a_pat ? rb : ra;
    if (m - n > cut) return cut + 1;  // the length gap alone (the lazy scans' diagonal tests rely on m - n <= cut)
    u128 P[N_PLANES], T[N_PLANES];
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) {
        P[b] = (a_pat ? pa[b] : pb[b]) >> pre;
        T[b] = (a_pat ? pb[b] : pa[b]) >> pre;
    }
    if (!__any(m > 64)) {
        uint64_t P64[N_PLANES], T64[N_PLANES];
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) {
            P64[b] = (uint64_t)P[b];
            T64[b] = (uint64_t)T[b];
        }
        if (!__any(m > 32)) return myers_plane_text<uint32_t, NP>(P64, m, T64, n, cut);
        return myers_plane_text_lazy<NP>(P64, m, T64, n, cut);
    }
#ifndef SPK_NO_LEV_BAND
    const int dlo = -((cut - (m - n)) >> 1), width = ((cut + (m - n)) >> 1) - dlo + 1;
    if (!__any(width > 32)) return myers_plane_text128_band<NP, 32>(P, m, T, n, cut, dlo);
    if (!__any(width > 64)) return myers_plane_text128_band<NP, 64>(P, m, T, n, cut, dlo);
#endif
    return myers_plane_text128_lazy<NP>(P, m, T, n, cut);
}

// P8: the caller's column uses all 8 planes (Latin-1 beyond ASCII); a kernel instantiated for the columns that
// drop the top plane (np <= 7) holds 162 VGPRs instead of 174 (3 waves per SIMD instead of 2).
template <bool P8>
__device__ inline int lev_rows_planes128(const u128 (&pa)[N_PLANES], int la, const u128 (&pb)[N_PLANES], int lb,
                                         int cut, int np = N_PLANES) {
    if (P8) return lev_rows_planes128_np<N_PLANES>(pa, la, pb, lb, cut);
    switch (np) {
        case 5: return lev_rows_planes128_np<5>(pa, la, pb, lb, cut);
        case 6: return lev_rows_planes128_np<6>(pa, la, pb, lb, cut);
        case 7: return lev_rows_planes128_np<7>(pa, la, pb, lb, cut);
        default: return lev_rows_planes128_np<7>(pa, la, pb, lb, cut);
    }
}

// matches() with BOTH strings as bit-planes (<= 64 units each, all < 256): the greedy matching,
// the transpositions and the common prefix come from register planes, with no unit loads (the
// unit-reading form waits on a dependent load per four units and per match).  The k-th matched
// unit of the shorter string is recorded as bit k of A_b (its bit b), the k-th flagged unit of the
// longer string as bit k of B_b, so transpositions = popc(OR_b (A_b ^ B_b)).  The prefix is the
// first position where the planes differ (zero past a row's end), capped at the shorter length.
template <typename W>
__device__ double jw_planes2(const uint64_t *mxq, int lmx, const uint64_t *mnq, int lmn, int lf, int ls) {
    uint64_t px[N_PLANES], pn[N_PLANES];
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) {
        px[b] = mxq[b];
        pn[b] = mnq[b];
    }
    W pl[N_PLANES], A[N_PLANES];
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) {
        pl[b] = (W)px[b];
        A[b] = 0;
    }
    const int range = lmx / 2 - 1 > 0 ? lmx / 2 - 1 : 0;
    W flags = 0;
    int m = 0;
    for (int h = 0; h < 2 && 32 * h < lmn; ++h) {
        uint32_t tw[N_PLANES];
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) tw[b] = (uint32_t)(pn[b] >> (32 * h));
        const int jn = lmn - 32 * h < 32 ? lmn - 32 * h : 32;
        for (int jj = 0; jj < jn; ++jj) {
            const int mi = 32 * h + jj;
            const int lo = mi - range > 0 ? mi - range : 0;
            const int hi = mi + range + 1 < lmx ? mi + range + 1 : lmx;
            W eq = ~(W)0;
#pragma unroll
            for (int b = 0; b < N_PLANES; ++b) eq = eq_plane(eq, (uint32_t)__builtin_amdgcn_sbfe((int)tw[b], jj, 1), pl[b]);
            const W cand = eq & mask_below<W>(hi) & ~mask_below<W>(lo) & ~flags;
            if (cand) {
                flags |= cand & (~cand + (W)1);  // lowest set bit: the first free match in the window
#pragma unroll
                for (int b = 0; b < N_PLANES; ++b) A[b] |= (W)((tw[b] >> jj) & 1u) << m;
                ++m;
            }
        }
    }
    if (m == 0) return 0.0;
    W diff = 0, fm = flags;
    for (int k = 0; k < m; ++k) {  // the longer string's flagged units, in order
        const int x = sizeof(W) == 4 ? __builtin_ctz((uint32_t)fm) : __builtin_ctzll((unsigned long long)fm);
        fm &= fm - (W)1;
        W d = 0;
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) d |= (W)(((px[b] >> x) & 1u) ^ ((A[b] >> k) & 1u));
        diff |= d << k;
    }
    const int t = sizeof(W) == 4 ? __builtin_popcount((uint32_t)diff) : __builtin_popcountll((unsigned long long)diff);
    uint64_t d = 0;
#pragma unroll
    for (int b = 0; b < N_PLANES; ++b) d |= px[b] ^ pn[b];
    int prefix = d ? __ffsll((unsigned long long)d) - 1 : 64;
    if (prefix > lmn) prefix = lmn;
    return jw_finish(m, t, prefix, lf, ls, lmx);
}

// Exact Jaro-Winkler for unequal strings of <= 64 units, without LDS.
__device__ inline double jw_exact(const StrView &a, const StrView &b) {
    const bool fmax = a.n > b.n;  // commons-text: max = first only if strictly longer
    const StrView &mx = fmax ? a : b;
    const StrView &mn = fmax ? b : a;
    if (mx.planes && mn.planes) {
        if (mx.n <= 32) return jw_planes2<uint32_t>(mx.planes, mx.n, mn.planes, mn.n, a.n, b.n);
        return jw_planes2<uint64_t>(mx.planes, mx.n, mn.planes, mn.n, a.n, b.n);
    }
    if (mx.planes) {
        if (mx.n <= 32) return jw_planes<uint32_t>(mx.planes, mx.p, mx.n, mn.p, mn.n, a.p, a.n, b.p, b.n);
        return jw_planes<uint64_t>(mx.planes, mx.p, mx.n, mn.p, mn.n, a.p, a.n, b.p, b.n);
    }
    return jw_small(GlbAcc{a.p}, a.n, GlbAcc{b.p}, b.n);
}

// Exact code-point Levenshtein of unequal BMP strings of <= 64 units, without LDS: common prefix
// and suffix are stripped (exact for unit-cost edit distance), then bit-parallel on the rest.
__device__ inline int lev_exact(const StrView &a, const StrView &b, int cut = 1 << 30) {
    const int mn = a.n < b.n ? a.n : b.n;
    const int pre = common_prefix(a.p, b.p, mn);
    int suf = 0;
    while (suf < mn - pre && a.p[a.n - 1 - suf] == b.p[b.n - 1 - suf]) ++suf;
    const int la = a.n - pre - suf, lb = b.n - pre - suf;
    if (la == 0) return lb;
    if (lb == 0) return la;
    // pattern: the longer trimmed string if it has planes (fewer text steps), else the other
    const bool a_pat = a.planes && (la >= lb || !b.planes);
    const StrView &pat = a_pat ? a : b;
    const StrView &txt = a_pat ? b : a;
    const int m = a_pat ? la : lb, n = a_pat ? lb : la;
    if (pat.planes) {
        if (m <= 32) return lev_planes<uint32_t>(pat.planes, pre, m, txt.p + pre, n, cut);
        return lev_planes<uint64_t>(pat.planes, pre, m, txt.p + pre, n, cut);
    }
    return lev_myers(GlbAcc{a.p + pre}, la, GlbAcc{b.p + pre}, lb);
}

}  // namespace spk
