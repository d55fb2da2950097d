// Comparison vectors (replaces gammas.py:65-124 evaluating the CASE templates of
// case_statements.py:62-277 with the jar's jaro_winkler_sim and Spark's levenshtein).
//
// One pair per lane.  Every comparison column is a small program of WHEN branches; each branch
// is an RPN predicate over Kleene booleans (SQL three-valued logic, NULL = not taken).  The
// program is uniform across the wave, so instruction fetch and dispatch are scalar; only the
// string work diverges.  Strings of a JW / Levenshtein operand are staged in LDS in a
// [position][lane] layout (lane-indexed banks, conflict-free for any per-lane position).
// Pairs whose strings exceed the LDS staging capacity (or carry surrogates for Levenshtein) are
// deferred to a second, global-memory pass with no length restriction up to SLOW_LIMIT.
//
// Output: one packed code per pair, code = Σ_k (γ_k + 1) · Π_{j<k}(L_j + 1), uint16 when the
// pattern space fits, else uint32.
//
// Jaro-Winkler arithmetic follows commons-text 1.4 exactly; the library is built
// with -ffp-contract=off so no FMA contraction changes the rounding.
#include <cmath>

#include "spk_internal.h"

namespace spk {

constexpr int G_THREADS = 256;
constexpr int MAXU = 40;          // LDS staging capacity per string (UTF-16 units)
constexpr int SLOW_LIMIT = 1024;  // deferred-pass capacity per string

struct GammaArgs {
    const ColDesc *cols0, *cols1;  // tables for operand side 0 (`_l`) and 1 (`_r`)
    const int32_t *pl, *pr;
    int64_t P;
    int K;
    const spk_column_program *progs;
    const int32_t *when_first, *when_n, *when_level;
    const spk_instr *instr;
    const spk_operand *ops;
    const uint16_t *lit_units;
    const int64_t *lit_off;
    const int32_t *lit_len, *lit_cplen;
    const int64_t *stride;
    uint8_t *codes;
    int code_bytes;
    int32_t *defer_list;
    unsigned int *defer_count;
    const int32_t *work;  // slow pass: pair indices
    int64_t n_work;
    int *err;
};

struct StrView {
    const uint16_t *p;
    int32_t n;    // UTF-16 units
    int32_t ncp;  // code points
    int32_t null;
    uint64_t hash;
    int32_t has_hash;
};

enum : int { KF = 0, KT = 1, KN = 2 };

__device__ inline int k_and(int a, int b) { return (a == KF || b == KF) ? KF : ((a == KN || b == KN) ? KN : KT); }
__device__ inline int k_or(int a, int b) { return (a == KT || b == KT) ? KT : ((a == KN || b == KN) ? KN : KF); }
__device__ inline int k_not(int a) { return a == KN ? KN : (a == KT ? KF : KT); }

__device__ inline int cmpd(double a, double b, int cmp) {
    bool r;
    switch (cmp) {
        case SPK_CMP_EQ: r = a == b; break;
        case SPK_CMP_NE: r = a != b; break;
        case SPK_CMP_LT: r = a < b; break;
        case SPK_CMP_LE: r = a <= b; break;
        case SPK_CMP_GT: r = a > b; break;
        default: r = a >= b; break;
    }
    return r ? KT : KF;
}

// Spark UTF8String.substringSQL(pos, len) on a code-point range, mapped to UTF-16 units.
__device__ inline void apply_substr(StrView &s, int pos, int len) {
    int nc = s.ncp;
    int start = pos > 0 ? pos - 1 : (pos < 0 ? nc + pos : 0);
    long end = (long)start + len;
    if (start < 0) start = 0;
    if (end > nc) end = nc;
    s.has_hash = 0;
    if (start >= end) {
        s.n = 0;
        s.ncp = 0;
        return;
    }
    if (s.ncp == s.n) {  // BMP only: units == code points
        s.p += start;
        s.n = (int)(end - start);
        s.ncp = s.n;
        return;
    }
    int u = 0, c = 0, ub = 0;
    while (u < s.n && c < end) {
        if (c == start) ub = u;
        uint16_t w = s.p[u];
        u += (w >= 0xD800 && w < 0xDC00 && u + 1 < s.n) ? 2 : 1;
        ++c;
    }
    s.p += ub;
    s.n = u - ub;
    s.ncp = (int)(end - start);
}

__device__ inline StrView lit_view(const GammaArgs &A, int lit) {
    StrView s;
    s.p = A.lit_units + A.lit_off[lit];
    s.n = A.lit_len[lit];
    s.ncp = A.lit_cplen[lit];
    s.null = 0;
    s.has_hash = 0;
    s.hash = 0;
    return s;
}

__device__ inline StrView get_str(const GammaArgs &A, const spk_operand &op, int32_t x, int32_t y) {
    StrView s{nullptr, 0, 0, 1, 0, 0};
    if (op.kind == 0) {
        int32_t row = op.side ? y : x;
        const ColDesc &c = (op.side ? A.cols1 : A.cols0)[op.col];
        int32_t n = c.len16[row];
        if (n >= 0) {
            s.p = c.units + c.off[row];
            s.n = n;
            s.ncp = c.cplen[row];
            s.null = 0;
            s.hash = c.hash[row];
            s.has_hash = 1;
        } else if (op.lit >= 0) {
            s = lit_view(A, op.lit);
        }
    } else if (op.kind == 1) {
        s = lit_view(A, op.lit);
    }
    if (!s.null && op.substr_start != 0) apply_substr(s, op.substr_start, op.substr_len);
    return s;
}

__device__ inline bool get_num(const GammaArgs &A, const spk_operand &op, int32_t x, int32_t y, double &v) {
    if (op.kind == 2) {
        v = op.num;
        return true;
    }
    int32_t row = op.side ? y : x;
    const ColDesc &c = (op.side ? A.cols1 : A.cols0)[op.col];
    if (c.valid[row]) {
        v = c.val[row];
        return true;
    }
    if (op.has_num_default) {
        v = op.num;
        return true;
    }
    return false;
}

__device__ inline bool units_equal(const StrView &a, const StrView &b) {
    if (a.n != b.n) return false;
    if (a.has_hash && b.has_hash && a.hash != b.hash) return false;
    for (int i = 0; i < a.n; ++i)
        if (a.p[i] != b.p[i]) return false;
    return true;
}

// code-point order (= Spark's UTF-8 byte order) for <, <=, >, >=
__device__ inline int str_order(const StrView &a, const StrView &b) {
    int i = 0, j = 0;
    while (i < a.n && j < b.n) {
        uint32_t ca = a.p[i], cb = b.p[j];
        int la = 1, lb = 1;
        if (ca >= 0xD800 && ca < 0xDC00 && i + 1 < a.n) { ca = 0x10000 + ((ca - 0xD800) << 10) + (a.p[i + 1] - 0xDC00); la = 2; }
        if (cb >= 0xD800 && cb < 0xDC00 && j + 1 < b.n) { cb = 0x10000 + ((cb - 0xD800) << 10) + (b.p[j + 1] - 0xDC00); lb = 2; }
        if (ca != cb) return ca < cb ? -1 : 1;
        i += la;
        j += lb;
    }
    if (i < a.n) return 1;
    if (j < b.n) return -1;
    return 0;
}

// ---- accessors -------------------------------------------------------------------------
struct LdsAcc {
    const uint16_t *b;
    __device__ uint16_t operator[](int i) const { return b[i * G_THREADS]; }
};
struct GlbAcc {
    const uint16_t *p;
    __device__ uint16_t operator[](int i) const { return p[i]; }
};

__device__ inline double jw_finish(int m, int t, int prefix, int lf, int ls, int lmx) {
    if (m == 0) return 0.0;
    double md = (double)m;
    double j = ((md / (double)lf + md / (double)ls) + (md - (double)(t / 2)) / md) / 3.0;
    if (j < 0.7) return j;
    double w = 1.0 / (double)lmx;
    if (w > 0.1) w = 0.1;
    return j + (w * (double)prefix) * (1.0 - j);
}

// commons-text 1.4 JaroWinklerDistance for strings of <= 64 units (bit-mask flags).
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

// Same algorithm, any length up to SLOW_LIMIT (flag words in scratch).
__device__ double jw_long(GlbAcc first, int lf, GlbAcc second, int ls) {
    const bool fmax = lf > ls;
    const GlbAcc mx = fmax ? first : second;
    const GlbAcc mn = fmax ? second : first;
    const int lmx = fmax ? lf : ls, lmn = fmax ? ls : lf;
    const int range = lmx / 2 - 1 > 0 ? lmx / 2 - 1 : 0;
    uint64_t flags[SLOW_LIMIT / 64], matched[SLOW_LIMIT / 64];
    for (int i = 0; i < SLOW_LIMIT / 64; ++i) flags[i] = matched[i] = 0;
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

// Levenshtein (Myers 1999 bit-parallel), pattern <= 64 symbols.
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

// Levenshtein over code points, any length up to SLOW_LIMIT (two-row DP in scratch).
__device__ int lev_long(const StrView &a, const StrView &b) {
    uint32_t cb[SLOW_LIMIT];
    int32_t row[SLOW_LIMIT + 1];
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
        for (int j = 1; j <= nb; ++j) {
            int up = row[j];
            int best = diag + (w != cb[j - 1] ? 1 : 0);
            if (up + 1 < best) best = up + 1;
            if (row[j - 1] + 1 < best) best = row[j - 1] + 1;
            row[j] = best;
            diag = up;
        }
    }
    return row[nb];
}

__device__ inline void stage(uint16_t *slot, const StrView &s) {
    for (int i = 0; i < s.n; ++i) slot[i * G_THREADS] = s.p[i];
}

struct Memo {
    int jw_key, lev_key;
    double jw;
    int lev;
    int staged_a, staged_b;  // operand ids currently in LDS slots 0 / 1
};

// Evaluate one WHEN predicate.  Returns KT / KF / KN; sets *defer if the fast pass cannot.
template <bool SLOW>
__device__ int eval_pred(const GammaArgs &A, int first, int count, int32_t x, int32_t y, uint16_t *slot_a,
                         uint16_t *slot_b, Memo &mm, bool *defer) {
    uint32_t st = 0;  // Kleene stack, 2 bits per entry
    for (int k = 0; k < count; ++k) {
        const spk_instr in = A.instr[first + k];
        int r = KN;
        switch (in.op) {
            case SPK_OP_AND: {
                int b = st & 3; st >>= 2; int a = st & 3; st >>= 2;
                r = k_and(a, b);
                break;
            }
            case SPK_OP_OR: {
                int b = st & 3; st >>= 2; int a = st & 3; st >>= 2;
                r = k_or(a, b);
                break;
            }
            case SPK_OP_NOT: {
                int a = st & 3; st >>= 2;
                r = k_not(a);
                break;
            }
            case SPK_OP_CONST: r = in.i0; break;
            case SPK_OP_ISNULL:
            case SPK_OP_NOTNULL: {
                const spk_operand &o = A.ops[in.a];
                bool isnull;
                if (o.kind == 0 && ((o.side ? A.cols1 : A.cols0)[o.col].kind == COL_NUM)) {
                    double v;
                    isnull = !get_num(A, o, x, y, v);
                } else {
                    isnull = get_str(A, o, x, y).null != 0;
                }
                r = (isnull == (in.op == SPK_OP_ISNULL)) ? KT : KF;
                break;
            }
            case SPK_OP_NUM_CMP:
            case SPK_OP_ABSDIFF:
            case SPK_OP_PERCDIFF: {
                double a, b;
                if (!get_num(A, A.ops[in.a], x, y, a) || !get_num(A, A.ops[in.b], x, y, b)) { r = KN; break; }
                if (in.op == SPK_OP_NUM_CMP) {
                    r = cmpd(a, b, in.cmp);
                } else if (in.op == SPK_OP_ABSDIFF) {
                    r = cmpd(fabs(a - b), in.t, in.cmp);
                } else {
                    double mx = a > b ? a : b;
                    double d = fabs(mx);
                    r = d == 0.0 ? KN : cmpd(fabs(a - b) / d, in.t, in.cmp);
                }
                break;
            }
            case SPK_OP_STR_CMP: {
                StrView a = get_str(A, A.ops[in.a], x, y), b = get_str(A, A.ops[in.b], x, y);
                if (a.null || b.null) { r = KN; break; }
                if (in.cmp == SPK_CMP_EQ || in.cmp == SPK_CMP_NE) {
                    bool eq = units_equal(a, b);
                    r = (eq == (in.cmp == SPK_CMP_EQ)) ? KT : KF;
                } else {
                    r = cmpd((double)str_order(a, b), 0.0, in.cmp);
                }
                break;
            }
            case SPK_OP_LEN: {
                StrView a = get_str(A, A.ops[in.a], x, y);
                r = a.null ? KN : cmpd((double)a.ncp, in.t, in.cmp);
                break;
            }
            case SPK_OP_JW: {
                StrView a = get_str(A, A.ops[in.a], x, y), b = get_str(A, A.ops[in.b], x, y);
                if (a.null || b.null) { r = KN; break; }
                const int key = in.a * 4096 + in.b;
                if (mm.jw_key != key) {
                    double v;
                    if (a.n == b.n && units_equal(a, b)) {
                        v = a.n > 0 ? 1.0 : 0.0;  // identical strings: m = n, t = 0 -> exactly 1.0
                    } else if (SLOW) {
                        if (a.n > SLOW_LIMIT || b.n > SLOW_LIMIT) { atomicOr(A.err, 1); v = 0.0; }
                        else if (a.n <= 64 && b.n <= 64) v = jw_small(GlbAcc{a.p}, a.n, GlbAcc{b.p}, b.n);
                        else v = jw_long(GlbAcc{a.p}, a.n, GlbAcc{b.p}, b.n);
                    } else {
                        if (a.n > MAXU || b.n > MAXU) { *defer = true; return KN; }
                        if (mm.staged_a != in.a) { stage(slot_a, a); mm.staged_a = in.a; }
                        if (mm.staged_b != in.b) { stage(slot_b, b); mm.staged_b = in.b; }
                        v = jw_small(LdsAcc{slot_a}, a.n, LdsAcc{slot_b}, b.n);
                    }
                    mm.jw = v;
                    mm.jw_key = key;
                }
                r = cmpd(mm.jw, in.t, in.cmp);
                break;
            }
            case SPK_OP_LEV:
            case SPK_OP_LEVRATIO: {
                StrView a = get_str(A, A.ops[in.a], x, y), b = get_str(A, A.ops[in.b], x, y);
                if (a.null || b.null) { r = KN; break; }
                const int key = in.a * 4096 + in.b;
                if (mm.lev_key != key) {
                    int v;
                    if (a.n == b.n && units_equal(a, b)) {
                        v = 0;
                    } else if (SLOW) {
                        if (a.n > SLOW_LIMIT || b.n > SLOW_LIMIT) { atomicOr(A.err, 1); v = 0; }
                        else v = lev_long(a, b);
                    } else {
                        if (a.n > MAXU || b.n > MAXU || a.ncp != a.n || b.ncp != b.n) { *defer = true; return KN; }
                        if (mm.staged_a != in.a) { stage(slot_a, a); mm.staged_a = in.a; }
                        if (mm.staged_b != in.b) { stage(slot_b, b); mm.staged_b = in.b; }
                        v = lev_myers(LdsAcc{slot_a}, a.n, LdsAcc{slot_b}, b.n);
                    }
                    mm.lev = v;
                    mm.lev_key = key;
                }
                if (in.op == SPK_OP_LEV) {
                    r = cmpd((double)mm.lev, in.t, in.cmp);
                } else {
                    double den = (double)(a.ncp + b.ncp) / 2.0;
                    r = den == 0.0 ? KN : cmpd((double)mm.lev / den, in.t, in.cmp);
                }
                break;
            }
            default: atomicOr(A.err, 2); r = KN; break;
        }
        st = (st << 2) | (uint32_t)r;
    }
    return (int)(st & 3);
}

template <bool SLOW>
__device__ bool eval_pair(const GammaArgs &A, int64_t p, uint16_t *slot_a, uint16_t *slot_b, uint32_t &code) {
    const int32_t x = A.pl[p], y = A.pr[p];
    uint32_t acc = 0;
    bool defer = false;
    for (int k = 0; k < A.K; ++k) {
        const spk_column_program prog = A.progs[k];
        Memo mm{-1, -1, 0.0, 0, -1, -1};
        int level = prog.else_level;
        for (int w = 0; w < prog.n_when; ++w) {
            const int wi = prog.first_when + w;
            int r = eval_pred<SLOW>(A, A.when_first[wi], A.when_n[wi], x, y, slot_a, slot_b, mm, &defer);
            if (!SLOW && defer) return false;
            if (r == KT) {
                level = A.when_level[wi];
                break;
            }
        }
        acc += (uint32_t)(level + 1) * (uint32_t)A.stride[k];
    }
    code = acc;
    return true;
}

__device__ inline void store_code(const GammaArgs &A, int64_t p, uint32_t code) {
    if (A.code_bytes == 2) reinterpret_cast<uint16_t *>(A.codes)[p] = (uint16_t)code;
    else reinterpret_cast<uint32_t *>(A.codes)[p] = code;
}

__global__ __launch_bounds__(G_THREADS) void k_gamma_fast(GammaArgs A) {
    __shared__ uint16_t lds[2][MAXU][G_THREADS];
    uint16_t *slot_a = &lds[0][0][threadIdx.x];
    uint16_t *slot_b = &lds[1][0][threadIdx.x];
    const int64_t stride = (int64_t)gridDim.x * G_THREADS;
    for (int64_t p = (int64_t)blockIdx.x * G_THREADS + threadIdx.x; p < A.P; p += stride) {
        uint32_t code;
        if (eval_pair<false>(A, p, slot_a, slot_b, code)) {
            store_code(A, p, code);
        } else {
            unsigned int i = atomicAdd(A.defer_count, 1u);
            A.defer_list[i] = (int32_t)p;
        }
    }
}

__global__ __launch_bounds__(64) void k_gamma_slow(GammaArgs A) {
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= A.n_work) return;
    const int64_t p = A.work[i];
    uint32_t code = 0;
    eval_pair<true>(A, p, nullptr, nullptr, code);
    store_code(A, p, code);
}

__global__ void k_codes_from_gammas(int64_t n, int K, const int8_t *__restrict__ g, const int64_t *__restrict__ stride,
                                    uint8_t *codes, int code_bytes) {
    int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    uint32_t acc = 0;
    for (int k = 0; k < K; ++k) acc += (uint32_t)(g[p * K + k] + 1) * (uint32_t)stride[k];
    if (code_bytes == 2) reinterpret_cast<uint16_t *>(codes)[p] = (uint16_t)acc;
    else reinterpret_cast<uint32_t *>(codes)[p] = acc;
}

__global__ void k_gammas_from_codes(int64_t start, int64_t n, int K, const uint8_t *codes, int code_bytes,
                                    const int64_t *__restrict__ stride, const int32_t *__restrict__ nlev,
                                    int8_t *__restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t p = start + i;
    uint32_t c = code_bytes == 2 ? reinterpret_cast<const uint16_t *>(codes)[p] : reinterpret_cast<const uint32_t *>(codes)[p];
    for (int k = 0; k < K; ++k) out[i * K + k] = (int8_t)((c / (uint32_t)stride[k]) % (uint32_t)(nlev[k] + 1)) - 1;
}

static int set_pattern_space(spk_ctx *ctx, int K, const int32_t *nlev) {
    SPK_REQUIRE(K >= 1 && K <= 64, SPK_E_INVALID, "need 1..64 comparison columns");
    ctx->K = K;
    ctx->n_levels.assign(nlev, nlev + K);
    ctx->stride.assign(K, 1);
    int64_t s = 1;
    for (int k = 0; k < K; ++k) {
        SPK_REQUIRE(nlev[k] >= 1 && nlev[k] <= 126, SPK_E_INVALID, "num_levels out of range");
        ctx->stride[k] = s;
        s *= (int64_t)(nlev[k] + 1);
        SPK_REQUIRE(s <= (int64_t)1 << 31, SPK_E_LIMIT,
                    "comparison-vector pattern space exceeds 2^31 (too many columns x levels)");
    }
    ctx->n_patterns = s;
    ctx->code_bytes = s <= 65536 ? 2 : 4;
    ctx->mpat_valid = false;
    return SPK_OK;
}

}  // namespace spk

using namespace spk;

static std::vector<uint16_t> utf8_to_utf16(const uint8_t *b, int64_t n, int32_t *ncp) {
    std::vector<uint16_t> out;
    int64_t i = 0;
    int32_t c = 0;
    while (i < n) {
        uint32_t c0 = b[i], cp;
        int len;
        if (c0 < 0x80) { cp = c0; len = 1; }
        else if (c0 < 0xE0) { cp = c0 & 0x1F; len = 2; }
        else if (c0 < 0xF0) { cp = c0 & 0x0F; len = 3; }
        else { cp = c0 & 0x07; len = 4; }
        for (int k = 1; k < len && i + k < n; ++k) cp = (cp << 6) | (b[i + k] & 0x3F);
        i += len;
        if (cp >= 0x10000) {
            cp -= 0x10000;
            out.push_back((uint16_t)(0xD800 + (cp >> 10)));
            out.push_back((uint16_t)(0xDC00 + (cp & 0x3FF)));
        } else {
            out.push_back((uint16_t)cp);
        }
        ++c;
    }
    *ncp = c;
    return out;
}

extern "C" int spk_gammas(spk_ctx *ctx, int n_cols, const spk_column_program *cols, int n_when,
                          const int32_t *when_first_instr, const int32_t *when_n_instr, const int32_t *when_level,
                          int n_instr, const spk_instr *instr, int n_operands, const spk_operand *operands, int n_lits,
                          const int64_t *lit_offsets, const uint8_t *lit_utf8) {
    SPK_REQUIRE(ctx && cols && n_cols >= 1, SPK_E_INVALID, "spk_gammas: bad args");
    SPK_REQUIRE(ctx->pairs_valid, SPK_E_STATE, "spk_gammas: no pairs");
    SPK_REQUIRE(n_operands < 4096 && n_instr >= 0 && n_when >= 0, SPK_E_LIMIT, "spk_gammas: program too large");
    SPK_HIP(hipSetDevice(ctx->device));
    // ---- host-side validation of the program against the loaded tables
    Table &t0 = ctx->table[0];
    Table &t1 = ctx->side_table(1);
    for (int i = 0; i < n_operands; ++i) {
        const spk_operand &o = operands[i];
        if (o.kind == 0) {
            Table &t = o.side ? t1 : t0;
            SPK_REQUIRE(o.col >= 0 && o.col < (int)t.cols.size() && t.cols[o.col] && t.cols[o.col]->kind != COL_NONE,
                        SPK_E_INVALID, "spk_gammas: operand references a column that was not loaded");
        }
        if (o.kind == 1 || (o.kind == 0 && o.lit >= 0))
            SPK_REQUIRE(o.lit < n_lits, SPK_E_INVALID, "spk_gammas: literal index out of range");
    }
    std::vector<int32_t> nlev(n_cols);
    for (int k = 0; k < n_cols; ++k) {
        nlev[k] = cols[k].n_levels;
        SPK_REQUIRE(cols[k].first_when >= 0 && cols[k].first_when + cols[k].n_when <= n_when, SPK_E_INVALID,
                    "spk_gammas: when range");
        SPK_REQUIRE(cols[k].else_level >= -1 && cols[k].else_level < cols[k].n_levels, SPK_E_INVALID,
                    "spk_gammas: else level out of range");
        for (int w = cols[k].first_when; w < cols[k].first_when + cols[k].n_when; ++w) {
            SPK_REQUIRE(when_level[w] >= -1 && when_level[w] < cols[k].n_levels, SPK_E_INVALID,
                        "spk_gammas: THEN level out of range");
            SPK_REQUIRE(when_first_instr[w] >= 0 && when_n_instr[w] >= 1 && when_n_instr[w] <= 16 &&
                            when_first_instr[w] + when_n_instr[w] <= n_instr,
                        SPK_E_INVALID, "spk_gammas: predicate range (max 16 RPN instructions)");
        }
    }
    for (int i = 0; i < n_instr; ++i) {
        const spk_instr &in = instr[i];
        bool binop = in.op == SPK_OP_AND || in.op == SPK_OP_OR || in.op == SPK_OP_NOT || in.op == SPK_OP_CONST;
        if (!binop) {
            SPK_REQUIRE(in.a >= 0 && in.a < n_operands, SPK_E_INVALID, "spk_gammas: operand index");
            bool two = !(in.op == SPK_OP_ISNULL || in.op == SPK_OP_NOTNULL || in.op == SPK_OP_LEN);
            if (two) SPK_REQUIRE(in.b >= 0 && in.b < n_operands, SPK_E_INVALID, "spk_gammas: operand index");
        }
    }
    SPK_TRY(set_pattern_space(ctx, n_cols, nlev.data()));

    // ---- literals -> UTF-16
    std::vector<uint16_t> lu;
    std::vector<int64_t> loff;
    std::vector<int32_t> llen, lcp;
    for (int i = 0; i < n_lits; ++i) {
        int32_t ncp = 0;
        auto u = utf8_to_utf16(lit_utf8 + lit_offsets[i], lit_offsets[i + 1] - lit_offsets[i], &ncp);
        loff.push_back((int64_t)lu.size());
        llen.push_back((int32_t)u.size());
        lcp.push_back(ncp);
        lu.insert(lu.end(), u.begin(), u.end());
    }
    lu.push_back(0);
    loff.push_back((int64_t)lu.size());
    llen.push_back(0);
    lcp.push_back(0);

    SPK_TRY(ensure_desc(ctx, t0));
    SPK_TRY(ensure_desc(ctx, t1));
    DevBuf<spk_column_program> d_prog;
    DevBuf<int32_t> d_wf, d_wn, d_wl, d_defer;
    DevBuf<spk_instr> d_instr;
    DevBuf<spk_operand> d_ops;
    DevBuf<uint16_t> d_lu;
    DevBuf<int64_t> d_loff, d_stride;
    DevBuf<int32_t> d_llen, d_lcp;
    DevBuf<unsigned int> d_cnt;
    DevBuf<int> d_err;
    auto up = [&](auto &buf, const auto *src, size_t n) -> int {
        SPK_TRY(buf.alloc(n ? n : 1));
        if (n) SPK_HIP(hipMemcpyAsync(buf.p, src, n * sizeof(*src), hipMemcpyHostToDevice, ctx->stream));
        return SPK_OK;
    };
    SPK_TRY(up(d_prog, cols, (size_t)n_cols));
    SPK_TRY(up(d_wf, when_first_instr, (size_t)n_when));
    SPK_TRY(up(d_wn, when_n_instr, (size_t)n_when));
    SPK_TRY(up(d_wl, when_level, (size_t)n_when));
    SPK_TRY(up(d_instr, instr, (size_t)n_instr));
    SPK_TRY(up(d_ops, operands, (size_t)n_operands));
    SPK_TRY(up(d_lu, lu.data(), lu.size()));
    SPK_TRY(up(d_loff, loff.data(), loff.size()));
    SPK_TRY(up(d_llen, llen.data(), llen.size()));
    SPK_TRY(up(d_lcp, lcp.data(), lcp.size()));
    SPK_TRY(up(d_stride, ctx->stride.data(), ctx->stride.size()));
    SPK_TRY(d_cnt.alloc(1));
    SPK_TRY(d_err.alloc(1));
    SPK_HIP(hipMemsetAsync(d_cnt.p, 0, sizeof(unsigned int), ctx->stream));
    SPK_HIP(hipMemsetAsync(d_err.p, 0, sizeof(int), ctx->stream));
    const int64_t P = ctx->n_pairs;
    SPK_TRY(ctx->codes.alloc((size_t)(P + 1) * ctx->code_bytes));
    SPK_TRY(d_defer.alloc((size_t)P + 1));

    GammaArgs A{};
    A.cols0 = t0.d_desc.p;
    A.cols1 = t1.d_desc.p;
    A.pl = ctx->pl.p;
    A.pr = ctx->pr.p;
    A.P = P;
    A.K = n_cols;
    A.progs = d_prog.p;
    A.when_first = d_wf.p;
    A.when_n = d_wn.p;
    A.when_level = d_wl.p;
    A.instr = d_instr.p;
    A.ops = d_ops.p;
    A.lit_units = d_lu.p;
    A.lit_off = d_loff.p;
    A.lit_len = d_llen.p;
    A.lit_cplen = d_lcp.p;
    A.stride = d_stride.p;
    A.codes = ctx->codes.p;
    A.code_bytes = ctx->code_bytes;
    A.defer_list = d_defer.p;
    A.defer_count = d_cnt.p;
    A.err = d_err.p;

    SPK_TRY(ctx->begin(K_GAMMA));
    if (P > 0) {
        int64_t blocks = (P + G_THREADS - 1) / G_THREADS;
        if (blocks > 256 * 16) blocks = 256 * 16;
        k_gamma_fast<<<(unsigned)blocks, G_THREADS, 0, ctx->stream>>>(A);
        SPK_HIP(hipGetLastError());
    }
    unsigned int n_def = 0;
    SPK_HIP(hipMemcpyAsync(&n_def, d_cnt.p, sizeof(n_def), hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    if (n_def) {
        A.work = d_defer.p;
        A.n_work = n_def;
        k_gamma_slow<<<(unsigned)((n_def + 63) / 64), 64, 0, ctx->stream>>>(A);
        SPK_HIP(hipGetLastError());
    }
    SPK_TRY(ctx->end(K_GAMMA));
    int err = 0;
    SPK_HIP(hipMemcpyAsync(&err, d_err.p, sizeof(err), hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    SPK_REQUIRE(!(err & 1), SPK_E_LIMIT, "spk_gammas: a compared string exceeds 1024 UTF-16 units");
    SPK_REQUIRE(!(err & 2), SPK_E_INVALID, "spk_gammas: unknown instruction");
    ctx->codes_valid = true;
    ctx->mpat_valid = false;
    ctx->last_deferred = (int64_t)n_def;
    return SPK_OK;
}

extern "C" int spk_gammas_load(spk_ctx *ctx, int n_cols, const int32_t *n_levels, int64_t n, const int8_t *gammas) {
    SPK_REQUIRE(ctx && n_levels && n >= 0 && (n == 0 || gammas), SPK_E_INVALID, "spk_gammas_load: bad args");
    SPK_HIP(hipSetDevice(ctx->device));
    SPK_TRY(set_pattern_space(ctx, n_cols, n_levels));
    for (int64_t p = 0; p < n; ++p)
        for (int k = 0; k < n_cols; ++k)
            SPK_REQUIRE(gammas[p * n_cols + k] >= -1 && gammas[p * n_cols + k] < n_levels[k], SPK_E_INVALID,
                        "spk_gammas_load: gamma value out of range");
    DevBuf<int8_t> d_g;
    DevBuf<int64_t> d_stride;
    SPK_TRY(d_g.alloc((size_t)n * n_cols + 1));
    SPK_TRY(d_stride.alloc((size_t)n_cols));
    if (n) SPK_HIP(hipMemcpyAsync(d_g.p, gammas, (size_t)n * n_cols, hipMemcpyHostToDevice, ctx->stream));
    SPK_HIP(hipMemcpyAsync(d_stride.p, ctx->stride.data(), (size_t)n_cols * 8, hipMemcpyHostToDevice, ctx->stream));
    SPK_TRY(ctx->codes.alloc((size_t)(n + 1) * ctx->code_bytes));
    if (n) {
        k_codes_from_gammas<<<(unsigned)((n + 255) / 256), 256, 0, ctx->stream>>>(n, n_cols, d_g.p, d_stride.p,
                                                                              ctx->codes.p, ctx->code_bytes);
        SPK_HIP(hipGetLastError());
    }
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    ctx->n_pairs = n;
    ctx->codes_valid = true;
    return SPK_OK;
}

extern "C" int spk_gammas_copy(spk_ctx *ctx, int64_t start, int64_t count, int8_t *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "spk_gammas_copy: bad args");
    SPK_REQUIRE(ctx->codes_valid, SPK_E_STATE, "spk_gammas_copy: no gammas");
    SPK_REQUIRE(start >= 0 && count >= 0 && start + count <= ctx->n_pairs, SPK_E_INVALID, "range out of bounds");
    SPK_HIP(hipSetDevice(ctx->device));
    if (!count) return SPK_OK;
    DevBuf<int8_t> d_out;
    DevBuf<int64_t> d_stride;
    DevBuf<int32_t> d_nlev;
    SPK_TRY(d_out.alloc((size_t)count * ctx->K));
    SPK_TRY(d_stride.alloc((size_t)ctx->K));
    SPK_TRY(d_nlev.alloc((size_t)ctx->K));
    SPK_HIP(hipMemcpyAsync(d_stride.p, ctx->stride.data(), (size_t)ctx->K * 8, hipMemcpyHostToDevice, ctx->stream));
    SPK_HIP(hipMemcpyAsync(d_nlev.p, ctx->n_levels.data(), (size_t)ctx->K * 4, hipMemcpyHostToDevice, ctx->stream));
    k_gammas_from_codes<<<(unsigned)((count + 255) / 256), 256, 0, ctx->stream>>>(
        start, count, ctx->K, ctx->codes.p, ctx->code_bytes, d_stride.p, d_nlev.p, d_out.p);
    SPK_HIP(hipGetLastError());
    SPK_HIP(hipMemcpyAsync(out, d_out.p, (size_t)count * ctx->K, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    return SPK_OK;
}

// ---- the jar's UDFs as bulk device functions (JaroWinklerSimilarity.call, Spark levenshtein) -----
// Same device code as the comparison kernel: LDS-staged jw_small / lev_myers for short strings,
// the global-memory jw_long / lev_long for the rest.
struct UdfArgs {
    int64_t n;
    const uint16_t *u16;
    const int64_t *off;  // [2n+1]: string i of pair p is 2p (left) and 2p+1 (right)
    const int32_t *cp;   // code points per string
    int op;              // 0 JW, 1 Levenshtein
    double *out;
    int *err;
};

__global__ __launch_bounds__(G_THREADS) void k_udf(UdfArgs U) {
    __shared__ uint16_t lds[2][MAXU][G_THREADS];
    uint16_t *slot_a = &lds[0][0][threadIdx.x];
    uint16_t *slot_b = &lds[1][0][threadIdx.x];
    int64_t p = (int64_t)blockIdx.x * G_THREADS + threadIdx.x;
    if (p >= U.n) return;
    StrView a{U.u16 + U.off[2 * p], (int32_t)(U.off[2 * p + 1] - U.off[2 * p]), U.cp[2 * p], 0, 0, 0};
    StrView b{U.u16 + U.off[2 * p + 1], (int32_t)(U.off[2 * p + 2] - U.off[2 * p + 1]), U.cp[2 * p + 1], 0, 0, 0};
    if (a.n > SLOW_LIMIT || b.n > SLOW_LIMIT) {
        atomicOr(U.err, 1);
        U.out[p] = NAN;
        return;
    }
    if (U.op == 0) {
        double v;
        if (a.n <= MAXU && b.n <= MAXU) {
            stage(slot_a, a);
            stage(slot_b, b);
            v = jw_small(LdsAcc{slot_a}, a.n, LdsAcc{slot_b}, b.n);
        } else if (a.n <= 64 && b.n <= 64) {
            v = jw_small(GlbAcc{a.p}, a.n, GlbAcc{b.p}, b.n);
        } else {
            v = jw_long(GlbAcc{a.p}, a.n, GlbAcc{b.p}, b.n);
        }
        U.out[p] = v;
    } else {
        int v;
        if (a.n <= MAXU && b.n <= MAXU && a.ncp == a.n && b.ncp == b.n) {
            stage(slot_a, a);
            stage(slot_b, b);
            v = lev_myers(LdsAcc{slot_a}, a.n, LdsAcc{slot_b}, b.n);
        } else {
            v = lev_long(a, b);
        }
        U.out[p] = (double)v;
    }
}

static int run_udf(spk_ctx *ctx, int op, int64_t n, const int64_t *l_off, const uint8_t *l_utf8, const int64_t *r_off,
                   const uint8_t *r_utf8, double *out) {
    SPK_REQUIRE(ctx && n >= 0 && out && l_off && r_off, SPK_E_INVALID, "spk udf: bad args");
    SPK_HIP(hipSetDevice(ctx->device));
    std::vector<uint16_t> u;
    std::vector<int64_t> off{0};
    std::vector<int32_t> cp;
    for (int64_t i = 0; i < n; ++i) {
        for (int side = 0; side < 2; ++side) {
            const int64_t *o = side ? r_off : l_off;
            const uint8_t *d = side ? r_utf8 : l_utf8;
            int32_t ncp = 0;
            auto v = utf8_to_utf16(d + o[i], o[i + 1] - o[i], &ncp);
            u.insert(u.end(), v.begin(), v.end());
            off.push_back((int64_t)u.size());
            cp.push_back(ncp);
        }
    }
    u.push_back(0);
    DevBuf<uint16_t> d_u;
    DevBuf<int64_t> d_off;
    DevBuf<int32_t> d_cp;
    DevBuf<double> d_out;
    DevBuf<int> d_err;
    SPK_TRY(d_u.alloc(u.size()));
    SPK_TRY(d_off.alloc(off.size()));
    SPK_TRY(d_cp.alloc(cp.size() + 1));
    SPK_TRY(d_out.alloc((size_t)n + 1));
    SPK_TRY(d_err.alloc(1));
    SPK_HIP(hipMemcpyAsync(d_u.p, u.data(), u.size() * 2, hipMemcpyHostToDevice, ctx->stream));
    SPK_HIP(hipMemcpyAsync(d_off.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    if (!cp.empty()) SPK_HIP(hipMemcpyAsync(d_cp.p, cp.data(), cp.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    SPK_HIP(hipMemsetAsync(d_err.p, 0, sizeof(int), ctx->stream));
    if (n) {
        UdfArgs U{n, d_u.p, d_off.p, d_cp.p, op, d_out.p, d_err.p};
        k_udf<<<(unsigned)((n + G_THREADS - 1) / G_THREADS), G_THREADS, 0, ctx->stream>>>(U);
        SPK_HIP(hipGetLastError());
        SPK_HIP(hipMemcpyAsync(out, d_out.p, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
    }
    int err = 0;
    SPK_HIP(hipMemcpyAsync(&err, d_err.p, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    SPK_REQUIRE(!err, SPK_E_LIMIT, "spk udf: a string exceeds 1024 UTF-16 units");
    return SPK_OK;
}

extern "C" int spk_jaro_winkler_sim(spk_ctx *ctx, int64_t n, const int64_t *l_off, const uint8_t *l_utf8,
                                    const int64_t *r_off, const uint8_t *r_utf8, double *out) {
    return run_udf(ctx, 0, n, l_off, l_utf8, r_off, r_utf8, out);
}

extern "C" int spk_levenshtein(spk_ctx *ctx, int64_t n, const int64_t *l_off, const uint8_t *l_utf8,
                               const int64_t *r_off, const uint8_t *r_utf8, double *out) {
    return run_udf(ctx, 1, n, l_off, l_utf8, r_off, r_utf8, out);
}

extern "C" int spk_n_patterns(spk_ctx *ctx, int64_t *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "null arg");
    *out = ctx->n_patterns;
    return SPK_OK;
}

extern "C" int spk_gammas_deferred(spk_ctx *ctx, int64_t *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "null arg");
    *out = ctx->last_deferred;
    return SPK_OK;
}
