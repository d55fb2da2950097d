// Comparison vectors (replaces gammas.py:65-124 evaluating the CASE templates of
// case_statements.py:62-277 with the jar's jaro_winkler_sim and Spark's levenshtein).
//
// Every comparison column is a small program of WHEN branches; each branch is an RPN predicate
// over SQL three-valued logic (NULL = branch not taken).  The program is uniform across a wave,
// so instruction fetch and dispatch are scalar; only the string work diverges.
//
// One lane per pair diverges badly if a wave must wait for its slowest lane's Jaro-Winkler or
// Levenshtein, so the evaluation is split:
//   1. filter pass (one lane per pair): NULL tests, equality (hash first), numeric tests and
//      *bounds* for the string similarities -- a Jaro-Winkler upper bound and a Levenshtein
//      lower / upper bound from 32-byte per-row metadata (lengths, hash, bucket sketch).  A
//      fourth truth value, UNDECIDED, propagates through AND / OR / NOT; a column whose WHEN
//      sequence is decided gets its level here, the others are appended (wave-aggregated) to
//      that column's work list.
//   2. exact pass (one lane per listed (pair, column)): the full interpreter with the exact
//      similarities computed from registers: match masks from per-row bit-planes (8 planes of
//      Latin-1 units, <= 64 units), Levenshtein after stripping the common prefix / suffix,
//      32-bit masks when the (trimmed) pattern fits.  Strings beyond 64 units, and surrogate
//      strings under Levenshtein, go to
//   3. the global-memory pass (two-row DP / flag words in scratch, any length up to SLOW_LIMIT).
// The filter pass writes each pair's code = Σ_k (γ_k + 1) · Π_{j<k}(L_j + 1) over the columns it
// decided (uint16 when the pattern space fits, else uint32); passes 2 and 3 add the rest in place.
// Bounds are exact decisions (never approximations), so the result is the exact evaluation.
#include <algorithm>
#include <cstring>
#include <type_traits>
#include <cmath>

#include "spk_strsim.h"

namespace spk {

constexpr int F_THREADS = 256;  // filter pass
constexpr int X_THREADS = 256;  // exact pass
constexpr int U_THREADS = 128;  // UDF kernel: 2 x 64 x 128 x 2 B = 32 KiB of LDS per block

enum Mode { M_FILTER = 0, M_EXACT = 1, M_SLOW = 2 };
enum Status { ST_DONE = 0, ST_UNDECIDED = 1, ST_NEEDS_SLOW = 2 };

// A "simple" comparison column: the shape every case_statements.py template has --
//   WHEN x_l IS NULL OR x_r IS NULL THEN null_level
//   WHEN test_1(x_l, x_r) THEN level_1 ... WHEN test_n(x_l, x_r) THEN level_n ELSE else_level
// with each test one leaf (=, <>, jaro_winkler_sim cmp t, levenshtein [ratio] cmp t, numeric
// compare / abs diff / percent diff) over the same two plain operands.  The filter pass evaluates
// these straight from the two rows' metadata records, loaded for several columns at once; every
// other program runs through the general interpreter.  Both give identical levels.
constexpr int MAX_TESTS = 6;
constexpr int SIMPLE_GROUP = 4;  // simple columns whose row records are in flight together
constexpr int MAX_SIMPLE = 64;   // = the column limit of set_pattern_space
enum SimpleKind : int32_t { SK_STR = 1, SK_NUM = 2 };
struct SimpleCol {
    int32_t k;  // comparison column (position in the code)
    int32_t kind;
    int32_t col;  // table column, the same index on both sides
    int32_t null_level, else_level, n_tests;
    int32_t op[MAX_TESTS], cmp[MAX_TESTS], level[MAX_TESTS];
    double t[MAX_TESTS];
    int64_t stride;
};

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
    void *codes;                  // packed code per pair: uint16 (code16) or uint32
    int code16;
    int32_t *work;                // [K][P] pair indices per column needing the exact pass, by region
    unsigned int *region_count;   // [K][n_regions] list length of each region
    int64_t region_len;           // pair ordinals per region (one filter workgroup each)
    int n_regions;
    int32_t *slow;             // slow-pass lists, column k at slow_off[k]
    const int64_t *slow_off;
    unsigned int *slow_count;  // [K]
    int *err;
    const SimpleCol *simple;   // filter pass: simple columns ...
    int n_simple;
    const int32_t *complex_k;  // ... and the columns the interpreter evaluates
    int n_complex;
};

// Codes are written in place: the filter pass sets each pair's code, the exact / slow passes of
// column k add to it.  A pair occurs at most once in column k's lists and the passes are ordered
// launches on one stream, so the read-modify-write needs no atomic -- and a 2-byte store leaves
// the neighbouring pair's code alone.
__device__ inline void code_set(const GammaArgs &A, int64_t p, uint32_t v) {
    if (A.code16) static_cast<uint16_t *>(A.codes)[p] = (uint16_t)v;
    else static_cast<uint32_t *>(A.codes)[p] = v;
}
__device__ inline void code_add(const GammaArgs &A, int64_t p, uint32_t d) {
    if (A.code16) {
        uint16_t *c = static_cast<uint16_t *>(A.codes) + p;
        *c = (uint16_t)(*c + d);
    } else {
        static_cast<uint32_t *>(A.codes)[p] += d;
    }
}

enum : int { KF = 0, KT = 1, KN = 2, KU = 3 };  // false, true, NULL, undecided (filter pass)

__device__ inline int k_and(int a, int b) {
    if (a == KF || b == KF) return KF;
    if (a == KU || b == KU) return KU;
    return (a == KN || b == KN) ? KN : KT;
}
__device__ inline int k_or(int a, int b) {
    if (a == KT || b == KT) return KT;
    if (a == KU || b == KU) return KU;
    return (a == KN || b == KN) ? KN : KF;
}
__device__ inline int k_not(int a) { return (a == KN || a == KU) ? a : (a == KT ? KF : KT); }

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

// `v cmp t` for an unknown v in [lo, hi]: decided only if every v in the interval agrees.
__device__ inline int decide(double lo, double hi, int cmp, double t) {
    if (lo == hi) return cmpd(lo, t, cmp);
    switch (cmp) {
        case SPK_CMP_GT: return lo > t ? KT : (hi <= t ? KF : KU);
        case SPK_CMP_GE: return lo >= t ? KT : (hi < t ? KF : KU);
        case SPK_CMP_LT: return hi < t ? KT : (lo >= t ? KF : KU);
        case SPK_CMP_LE: return hi <= t ? KT : (lo > t ? KF : KU);
        case SPK_CMP_EQ: return (t < lo || t > hi) ? KF : KU;
        default: return (t < lo || t > hi) ? KT : KU;
    }
}

// Spark UTF8String.substringSQL(pos, len) on a code-point range, mapped to UTF-16 units.
__device__ inline void apply_substr(StrView &s, int pos, int len) {
    int nc = s.ncp;
    int start = pos > 0 ? pos - 1 : (pos < 0 ? nc + pos : 0);
    long end = (long)start + len;
    if (start < 0) start = 0;
    if (end > nc) end = nc;
    s.has_meta = 0;
    s.planes = nullptr;
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
    return plain_view(A.lit_units + A.lit_off[lit], A.lit_len[lit], A.lit_cplen[lit]);
}

// A row's string view from its metadata record.
__device__ inline StrView row_view(const ColDesc &c, const RecMeta &m, int64_t row, int col) {
    StrView s = plain_view(c.units + meta_off(m), m.len16, meta_cplen(m));
    s.planes = (m.cpf & CPF_PLANES) ? c.planes + row * N_PLANES : nullptr;
    s.has_meta = 1;
    s.exact_key = (m.cpf & CPF_ID) ? col + 1 : 0;  // ids are per column (both sides share)
    s.key = m.key;
    s.sketch = m.sketch;
    return s;
}

__device__ inline StrView get_str(const GammaArgs &A, const spk_operand &op, int32_t x, int32_t y) {
    StrView s;
    if (op.kind == 0) {
        const ColDesc &c = (op.side ? A.cols1 : A.cols0)[op.col];
        const int32_t row = op.side ? y : x;
        const RecMeta m = c.meta[row];
        if (m.len16 >= 0) {
            s = row_view(c, m, row, op.col);
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
    const ColDesc &c = (op.side ? A.cols1 : A.cols0)[op.col];
    const int32_t row = op.side ? y : x;
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

struct Memo {
    int jw_key, lev_key;
    double jw;
    int lev;
    int staged_a, staged_b;  // operand ids currently in the LDS slots
};

// One WHEN predicate.  Sets *slow when the exact pass needs the global-memory pass.
template <int MODE>
__device__ int eval_pred(const GammaArgs &A, int first, int count, int32_t x, int32_t y, uint16_t *slot_a,
                         uint16_t *slot_b, Memo &mm, bool *slow) {
    uint32_t st = 0;  // stack of truth values, 2 bits per entry
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
                if (o.kind == 2 || (o.kind == 0 && (o.side ? A.cols1 : A.cols0)[o.col].kind == COL_NUM)) {
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
                    double d = fabs(a > b ? a : b);
                    r = d == 0.0 ? KN : cmpd(fabs(a - b) / d, in.t, in.cmp);
                }
                break;
            }
            case SPK_OP_STR_CMP: {
                StrView a = get_str(A, A.ops[in.a], x, y), b = get_str(A, A.ops[in.b], x, y);
                if (a.null || b.null) { r = KN; break; }
                if (in.cmp == SPK_CMP_EQ || in.cmp == SPK_CMP_NE) {
                    r = (units_equal(a, b) == (in.cmp == SPK_CMP_EQ)) ? KT : KF;
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
                    } else if (MODE == M_FILTER) {
                        const double hi = jw_upper(a, b);
                        if (hi < 0.0) {
                            v = 0.0;  // no common unit: m = 0
                        } else {
                            r = decide(0.0, hi + 1e-12, in.cmp, in.t);  // margin >> rounding of either side
                            break;
                        }
                    } else if (MODE == M_SLOW) {
                        if (a.n > SLOW_LIMIT || b.n > SLOW_LIMIT) { atomicOr(A.err, 1); v = 0.0; }
                        else if (a.n <= 64 && b.n <= 64) v = jw_small(GlbAcc{a.p}, a.n, GlbAcc{b.p}, b.n);
                        else v = jw_long(GlbAcc{a.p}, a.n, GlbAcc{b.p}, b.n);
                    } else {
                        if (a.n > 64 || b.n > 64) { *slow = true; return KN; }
                        v = jw_exact(a, b);
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
                const double den = (double)(a.ncp + b.ncp) / 2.0;
                if (in.op == SPK_OP_LEVRATIO && den == 0.0) { r = KN; break; }
                const int key = in.a * 4096 + in.b;
                if (mm.lev_key != key) {
                    int v;
                    if (a.n == b.n && units_equal(a, b)) {
                        v = 0;
                    } else if (MODE == M_FILTER) {
                        const int lo = lev_lower(a, b);
                        const int hi = a.ncp > b.ncp ? a.ncp : b.ncp;
                        if (in.op == SPK_OP_LEV) r = decide((double)lo, (double)hi, in.cmp, in.t);
                        else r = decide((double)lo / den, (double)hi / den, in.cmp, in.t);
                        break;
                    } else if (MODE == M_SLOW) {
                        if (a.n > SLOW_LIMIT || b.n > SLOW_LIMIT) { atomicOr(A.err, 1); v = 0; }
                        else v = lev_long(a, b);
                    } else {
                        if (a.n > 64 || b.n > 64 || a.ncp != a.n || b.ncp != b.n) { *slow = true; return KN; }
                        v = lev_exact(a, b);
                    }
                    mm.lev = v;
                    mm.lev_key = key;
                }
                r = in.op == SPK_OP_LEV ? cmpd((double)mm.lev, in.t, in.cmp) : cmpd((double)mm.lev / den, in.t, in.cmp);
                break;
            }
            default: atomicOr(A.err, 2); r = KN; break;
        }
        st = (st << 2) | (uint32_t)r;
    }
    return (int)(st & 3);
}

template <int MODE>
__device__ int eval_column(const GammaArgs &A, int k, int32_t x, int32_t y, uint16_t *slot_a, uint16_t *slot_b,
                           int &level) {
    const spk_column_program prog = A.progs[k];
    Memo mm{-1, -1, 0.0, 0, -1, -1};
    for (int w = 0; w < prog.n_when; ++w) {
        const int wi = prog.first_when + w;
        bool slow = false;
        const int r = eval_pred<MODE>(A, A.when_first[wi], A.when_n[wi], x, y, slot_a, slot_b, mm, &slow);
        if (slow) return ST_NEEDS_SLOW;
        if (r == KU) return ST_UNDECIDED;
        if (r == KT) {
            level = A.when_level[wi];
            return ST_DONE;
        }
    }
    level = prog.else_level;
    return ST_DONE;
}

// Append `val` for every lane with `want`; one atomic per wave.  Call with the whole wave converged.
__device__ inline void wave_append(int32_t *list, unsigned int *count, bool want, int32_t val) {
    const unsigned long long mask = __ballot(want);
    if (!mask) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll(mask) - 1;
    unsigned int base = 0;
    if (lane == leader) base = atomicAdd(count, (unsigned int)__popcll(mask));
    base = __shfl(base, leader);
    if (want) list[base + __popcll(mask & ((1ull << lane) - 1ull))] = val;
}

// Work lists of the filter pass.  Each workgroup owns one contiguous region of pair ordinals and
// appends the region's undecided pairs of column k to work[k][region start ...] under a counter
// in LDS: no device-scope atomic on a shared counter (those serialise at ~12 ns each across the
// whole chip), deterministic list order, and a region's rows stay in one XCD's L2.
struct Region {
    int64_t r0, r1;  // pair ordinals [r0, r1)
};

__device__ inline Region my_region(const GammaArgs &A) {
    const int64_t r0 = (int64_t)blockIdx.x * A.region_len;
    const int64_t r1 = r0 + A.region_len < A.P ? r0 + A.region_len : A.P;
    return Region{r0, r1};
}

__device__ inline int32_t *region_list(const GammaArgs &A, int k, const Region &r) {
    return A.work + (int64_t)k * A.P + r.r0;
}

// ---- simple columns in the filter pass ----------------------------------------------------------
// Upper bound of jaro_winkler_sim(a, b) for unequal rows from their records alone (jw_upper with
// the prefix bounded by the four head units: exact below 4, else by the shorter length).
__device__ inline double jw_upper_meta(const RecMeta &a, const RecMeta &b) {
    const int lf = a.len16, ls = b.len16;
    const int lmn = lf < ls ? lf : ls, lmx = lf < ls ? ls : lf;
    if (lmn == 0) return -1.0;
    const int M = sketch_inter_ub(a.sketch, b.sketch, lf, ls);
    if (M == 0) return -1.0;
    const uint64_t d = a.head ^ b.head;
    const int cp = d ? (__ffsll((unsigned long long)d) - 1) / 16 : 4;
    const int prefix = cp < 4 ? (cp < lmn ? cp : lmn) : lmn;
    // M/lf + M/ls with one division; the caller's 1e-12 margin covers the few-ulp difference from
    // the reference's operation order (a bound only has to be >= the true value), and the Winkler
    // boost is applied unless j is clearly below its 0.7 threshold
    const double j = ((double)M * (double)(lf + ls) / ((double)lf * (double)ls) + 1.0) * (1.0 / 3.0);
    if (j < 0.7 - 1e-9) return j;
    const double pw = lmx > 10 ? (double)prefix / (double)lmx : 0.1 * (double)prefix;
    return j + pw * (1.0 - j);
}

__device__ inline int lev_lower_meta(const RecMeta &a, const RecMeta &b) {
    const int na = meta_cplen(a), nb = meta_cplen(b);
    int lb = na > nb ? na - nb : nb - na;
    if (na == a.len16 && nb == b.len16) {  // BMP: units are code points, so the bag bound holds
        const int bag = (na > nb ? na : nb) - sketch_inter_ub(a.sketch, b.sketch, na, nb);
        if (bag > lb) lb = bag;
    }
    return lb;
}

// 1 equal, 0 unequal, -1 needs the units (hash match on rows without dictionary ids).
__device__ inline int meta_equal(const RecMeta &a, const RecMeta &b) {
    if (a.cpf & b.cpf & CPF_ID) return a.key == b.key ? 1 : 0;
    const bool keyed = ((a.cpf | b.cpf) & CPF_ID) == 0;
    if (a.len16 != b.len16 || a.head != b.head || (keyed && a.key != b.key)) return 0;
    return a.len16 <= 4 ? 1 : -1;
}

__device__ int simple_str(const SimpleCol &sc, const RecMeta &a, const RecMeta &b, int &level) {
    if (a.len16 < 0 || b.len16 < 0) {
        level = sc.null_level;
        return ST_DONE;
    }
    const int eq = meta_equal(a, b);
    for (int i = 0; i < sc.n_tests; ++i) {
        const int op = sc.op[i], cmp = sc.cmp[i];
        const double t = sc.t[i];
        int r;
        if (op == SPK_OP_STR_CMP) {
            r = eq < 0 ? KU : (((eq == 1) == (cmp == SPK_CMP_EQ)) ? KT : KF);
        } else if (op == SPK_OP_JW) {
            if (eq == 1) {
                r = cmpd(a.len16 > 0 ? 1.0 : 0.0, t, cmp);
            } else if (eq == 0) {
                const double hi = jw_upper_meta(a, b);
                r = hi < 0.0 ? cmpd(0.0, t, cmp) : decide(0.0, hi + 1e-12, cmp, t);
            } else {
                r = KU;
            }
        } else {  // SPK_OP_LEV / SPK_OP_LEVRATIO
            const int na = meta_cplen(a), nb = meta_cplen(b);
            const double den = (double)(na + nb) / 2.0;
            if (op == SPK_OP_LEVRATIO && den == 0.0) {
                r = KN;
            } else if (eq == 1) {
                r = cmpd(0.0, t, cmp);  // 0 / den == 0
            } else if (eq == 0) {
                const double lo = (double)lev_lower_meta(a, b), hi = (double)(na > nb ? na : nb);
                r = op == SPK_OP_LEV ? decide(lo, hi, cmp, t) : decide(lo / den, hi / den, cmp, t);
            } else {
                r = KU;
            }
        }
        if (r == KU) return ST_UNDECIDED;
        if (r == KT) {
            level = sc.level[i];
            return ST_DONE;
        }
    }
    level = sc.else_level;
    return ST_DONE;
}

__device__ int simple_num(const SimpleCol &sc, bool va, double a, bool vb, double b) {
    if (!va || !vb) return sc.null_level;
    for (int i = 0; i < sc.n_tests; ++i) {
        const int op = sc.op[i], cmp = sc.cmp[i];
        int r;
        if (op == SPK_OP_NUM_CMP) {
            r = cmpd(a, b, cmp);
        } else if (op == SPK_OP_ABSDIFF) {
            r = cmpd(fabs(a - b), sc.t[i], cmp);
        } else {  // SPK_OP_PERCDIFF
            const double d = fabs(a > b ? a : b);
            r = d == 0.0 ? KN : cmpd(fabs(a - b) / d, sc.t[i], cmp);
        }
        if (r == KT) return sc.level[i];
    }
    return sc.else_level;
}

// Filter pass, simple columns: initialises code[p] with their levels.  The column descriptors
// and the table pointers are staged in LDS once per workgroup: read from global memory inside the
// divergent per-pair code they would be per-lane vector loads on the critical path of every pair.
struct SimpleSrc {
    const RecMeta *m0, *m1;
    const double *v0, *v1;
    const uint8_t *ok0, *ok1;
};

__global__ __launch_bounds__(F_THREADS) void k_gamma_simple(GammaArgs A) {
    __shared__ SimpleCol s_sc[MAX_SIMPLE];
    __shared__ SimpleSrc s_src[MAX_SIMPLE];
    __shared__ unsigned int s_cnt[MAX_SIMPLE];
    for (int i = threadIdx.x; i < A.n_simple; i += F_THREADS) {
        const SimpleCol sc = A.simple[i];
        const ColDesc &c0 = A.cols0[sc.col], &c1 = A.cols1[sc.col];
        s_sc[i] = sc;
        s_src[i] = SimpleSrc{c0.meta, c1.meta, c0.val, c1.val, c0.valid, c1.valid};
        s_cnt[i] = 0;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const Region R = my_region(A);
    for (int64_t base = R.r0 + (threadIdx.x & ~63); base < R.r1; base += F_THREADS) {  // wave-uniform
        const int64_t p = base + lane;
        const bool active = p < R.r1;
        const int32_t x = active ? A.pl[p] : 0;  // inactive lanes read row 0 harmlessly
        const int32_t y = active ? A.pr[p] : 0;
        uint32_t acc = 0;
        for (int g = 0; g < A.n_simple; g += SIMPLE_GROUP) {
            // issue every record load of the group before the first use
            RecMeta ma[SIMPLE_GROUP], mb[SIMPLE_GROUP];
            double va[SIMPLE_GROUP], vb[SIMPLE_GROUP];
            bool oka[SIMPLE_GROUP], okb[SIMPLE_GROUP];
#pragma unroll
            for (int j = 0; j < SIMPLE_GROUP; ++j) {
                if (g + j < A.n_simple) {
                    const SimpleSrc &src = s_src[g + j];
                    if (s_sc[g + j].kind == SK_STR) {
                        ma[j] = src.m0[x];
                        mb[j] = src.m1[y];
                    } else {
                        oka[j] = src.ok0[x] != 0;
                        okb[j] = src.ok1[y] != 0;
                        va[j] = src.v0[x];
                        vb[j] = src.v1[y];
                    }
                }
            }
            // one copy of the evaluation code: slot 0 is evaluated, then the slots rotate down
            const int n_here = A.n_simple - g < SIMPLE_GROUP ? A.n_simple - g : SIMPLE_GROUP;
            for (int j = 0; j < n_here; ++j) {
                const SimpleCol &sc = s_sc[g + j];
                bool undecided = false;
                if (active) {
                    int level;
                    if (sc.kind == SK_STR) {
                        if (simple_str(sc, ma[0], mb[0], level) != ST_DONE) undecided = true;
                    } else {
                        level = simple_num(sc, oka[0], va[0], okb[0], vb[0]);
                    }
                    if (!undecided) acc += (uint32_t)(level + 1) * (uint32_t)sc.stride;
                }
                wave_append(region_list(A, sc.k, R), &s_cnt[g + j], undecided, (int32_t)p);
#pragma unroll
                for (int q = 0; q + 1 < SIMPLE_GROUP; ++q) {
                    ma[q] = ma[q + 1];
                    mb[q] = mb[q + 1];
                    va[q] = va[q + 1];
                    vb[q] = vb[q + 1];
                    oka[q] = oka[q + 1];
                    okb[q] = okb[q + 1];
                }
            }
        }
        if (active) code_set(A, p, acc);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < A.n_simple; i += F_THREADS)
        A.region_count[(int64_t)s_sc[i].k * A.n_regions + blockIdx.x] = s_cnt[i];
}

// Filter pass, every other column through the interpreter: adds to code[p].
__global__ __launch_bounds__(F_THREADS) void k_gamma_filter(GammaArgs A) {
    __shared__ unsigned int s_cnt[MAX_SIMPLE];
    for (int i = threadIdx.x; i < A.n_complex; i += F_THREADS) s_cnt[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const Region R = my_region(A);
    for (int64_t base = R.r0 + (threadIdx.x & ~63); base < R.r1; base += F_THREADS) {  // wave-uniform
        const int64_t p = base + lane;
        const bool active = p < R.r1;
        int32_t x = 0, y = 0;
        if (active) {
            x = A.pl[p];
            y = A.pr[p];
        }
        uint32_t acc = 0;
        for (int i = 0; i < A.n_complex; ++i) {
            const int k = A.complex_k[i];
            bool undecided = false;
            if (active) {
                int level = 0;
                const int st = eval_column<M_FILTER>(A, k, x, y, nullptr, nullptr, level);
                if (st == ST_DONE) acc += (uint32_t)(level + 1) * (uint32_t)A.stride[k];
                else undecided = true;
            }
            wave_append(region_list(A, k, R), &s_cnt[i], undecided, (int32_t)p);
        }
        if (active) code_add(A, p, acc);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < A.n_complex; i += F_THREADS)
        A.region_count[(int64_t)A.complex_k[i] * A.n_regions + blockIdx.x] = s_cnt[i];
}

// Exact pass over column k: workgroup b takes region b's list.
__global__ __launch_bounds__(X_THREADS) void k_gamma_exact(GammaArgs A, int k) {
    uint16_t *slot_a = nullptr, *slot_b = nullptr;  // the exact pass works from registers and L1/L2
    const Region R = my_region(A);
    const int32_t *items = region_list(A, k, R);
    const int64_t n = A.region_count[(int64_t)k * A.n_regions + blockIdx.x];
    for (int64_t base = 0; base < n; base += X_THREADS) {  // block-uniform trip count
        const int64_t i = base + threadIdx.x;
        bool to_slow = false;
        int32_t p = 0;
        if (i < n) {
            p = items[i];
            int level = 0;
            const int st = eval_column<M_EXACT>(A, k, A.pl[p], A.pr[p], slot_a, slot_b, level);
            if (st == ST_DONE) code_add(A, p, (uint32_t)(level + 1) * (uint32_t)A.stride[k]);
            else to_slow = true;
        }
        wave_append(A.slow + A.slow_off[k], A.slow_count + k, to_slow, p);
    }
}

// Exact pass over a simple string column (the template shapes): the tests run straight on the two
// rows' records, bit-planes and units -- no interpreter, no re-evaluation of the NULL / equality
// branches the filter pass already settled, each similarity computed at most once.  Levenshtein
// tests of the `<=` / `<` kind need the distance only up to the largest value any of them accepts
// (lev_cut), so the bit-parallel scan stops as soon as the distance provably exceeds it.
__device__ inline int simple_lev_cut(const SimpleCol &sc, int ncp_a, int ncp_b) {
    const double den = (double)(ncp_a + ncp_b) / 2.0;
    int cut = 0;
    for (int i = 0; i < sc.n_tests; ++i) {
        if (sc.op[i] != SPK_OP_LEV && sc.op[i] != SPK_OP_LEVRATIO) continue;
        if (sc.cmp[i] != SPK_CMP_LE && sc.cmp[i] != SPK_CMP_LT) return 1 << 30;
        // every v > bound fails `v cmp t` (resp. `v / den cmp t`): one unit of margin over t * den
        const double lim = sc.op[i] == SPK_OP_LEV ? sc.t[i] : sc.t[i] * den;
        if (!(lim < 1e9)) return 1 << 30;
        const int bound = lim < 0.0 ? 0 : (int)floor(lim) + 1;
        cut = bound > cut ? bound : cut;
    }
    return cut;
}

__device__ int simple_exact(const GammaArgs &A, const SimpleCol &sc, const ColDesc &c0, const ColDesc &c1, int32_t x,
                            int32_t y, int &level) {
    const RecMeta ma = c0.meta[x], mb = c1.meta[y];
    if (ma.len16 < 0 || mb.len16 < 0) {
        level = sc.null_level;
        return ST_DONE;
    }
    const StrView a = row_view(c0, ma, x, sc.col), b = row_view(c1, mb, y, sc.col);
    int eq = meta_equal(ma, mb);
    if (eq < 0) eq = units_equal(a, b) ? 1 : 0;
    double jw = -1.0;
    int lev = -1;
    for (int i = 0; i < sc.n_tests; ++i) {
        const int op = sc.op[i], cmp = sc.cmp[i];
        const double t = sc.t[i];
        int r;
        if (op == SPK_OP_STR_CMP) {
            r = ((eq == 1) == (cmp == SPK_CMP_EQ)) ? KT : KF;
        } else if (op == SPK_OP_JW) {
            if (jw < 0.0) {
                if (eq == 1) jw = a.n > 0 ? 1.0 : 0.0;
                else if (a.n > 64 || b.n > 64) return ST_NEEDS_SLOW;
                else jw = jw_exact(a, b);
            }
            r = cmpd(jw, t, cmp);
        } else {  // SPK_OP_LEV / SPK_OP_LEVRATIO
            const double den = (double)(a.ncp + b.ncp) / 2.0;
            if (op == SPK_OP_LEVRATIO && den == 0.0) {
                r = KN;
            } else {
                if (lev < 0) {
                    if (eq == 1) lev = 0;
                    else if (a.n > 64 || b.n > 64 || a.ncp != a.n || b.ncp != b.n) return ST_NEEDS_SLOW;
                    else lev = lev_exact(a, b, simple_lev_cut(sc, a.ncp, b.ncp));
                }
                r = op == SPK_OP_LEV ? cmpd((double)lev, t, cmp) : cmpd((double)lev / den, t, cmp);
            }
        }
        if (r == KT) {
            level = sc.level[i];
            return ST_DONE;
        }
    }
    level = sc.else_level;
    return ST_DONE;
}

__global__ __launch_bounds__(X_THREADS) void k_gamma_exact_simple(GammaArgs A, int si) {
    __shared__ SimpleCol s_sc;
    __shared__ ColDesc s_c0, s_c1;
    if (threadIdx.x == 0) {
        s_sc = A.simple[si];
        s_c0 = A.cols0[s_sc.col];
        s_c1 = A.cols1[s_sc.col];
    }
    __syncthreads();
    const SimpleCol &sc = s_sc;
    const int k = sc.k;
    const Region R = my_region(A);
    const int32_t *items = region_list(A, k, R);
    const int64_t n = A.region_count[(int64_t)k * A.n_regions + blockIdx.x];
    // software pipeline: the next item's pair rows are in flight while this one is evaluated
    int64_t i = threadIdx.x;
    int32_t p = 0, x = 0, y = 0;
    if (i < n) {
        p = items[i];
        x = A.pl[p];
        y = A.pr[p];
    }
    for (int64_t base = 0; base < n; base += X_THREADS) {  // block-uniform trip count
        const bool have = i < n;
        const int64_t i2 = i + X_THREADS;
        int32_t p2 = 0, x2 = 0, y2 = 0;
        if (i2 < n) {
            p2 = items[i2];
            x2 = A.pl[p2];
            y2 = A.pr[p2];
        }
        bool to_slow = false;
        if (have) {
            int level = 0;
            if (simple_exact(A, sc, s_c0, s_c1, x, y, level) == ST_DONE)
                code_add(A, p, (uint32_t)(level + 1) * (uint32_t)sc.stride);
            else
                to_slow = true;
        }
        wave_append(A.slow + A.slow_off[k], A.slow_count + k, to_slow, p);
        i = i2;
        p = p2;
        x = x2;
        y = y2;
    }
}

__global__ __launch_bounds__(64) void k_gamma_slow(GammaArgs A, int k, const int32_t *items, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const int32_t p = items[i];
    int level = 0;
    eval_column<M_SLOW>(A, k, A.pl[p], A.pr[p], nullptr, nullptr, level);
    code_add(A, p, (uint32_t)(level + 1) * (uint32_t)A.stride[k]);
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

// Recognise a simple column (see SimpleCol); false leaves it to the interpreter.
static bool classify_simple(int k, const spk_column_program &prog, const int32_t *wf, const int32_t *wn,
                            const int32_t *wl, const spk_instr *instr, const spk_operand *ops, const Table &t0,
                            const Table &t1, const std::vector<int64_t> &stride, SimpleCol *out) {
    if (prog.n_when < 1 || prog.n_when - 1 > MAX_TESTS) return false;
    const int w0 = prog.first_when;
    if (wn[w0] != 3) return false;
    const spk_instr *n = instr + wf[w0];
    if (n[0].op != SPK_OP_ISNULL || n[1].op != SPK_OP_ISNULL || n[2].op != SPK_OP_OR) return false;
    auto plain = [&](int i, int side) {
        const spk_operand &o = ops[i];
        return o.kind == 0 && o.side == side && o.lit < 0 && !o.has_num_default && o.substr_start == 0;
    };
    int a = n[0].a, b = n[1].a;
    if (plain(b, 0) && plain(a, 1)) std::swap(a, b);
    if (!plain(a, 0) || !plain(b, 1) || ops[a].col != ops[b].col) return false;
    const int col = ops[a].col;
    const ColKind ka = t0.cols[col]->kind, kb = t1.cols[col]->kind;
    if (ka != kb || (ka != COL_STR && ka != COL_NUM)) return false;
    SimpleCol s{};
    s.k = k;
    s.kind = ka == COL_STR ? SK_STR : SK_NUM;
    s.col = col;
    s.null_level = wl[w0];
    s.else_level = prog.else_level;
    s.n_tests = prog.n_when - 1;
    s.stride = stride[k];
    for (int i = 0; i < s.n_tests; ++i) {
        const int w = w0 + 1 + i;
        if (wn[w] != 1) return false;
        const spk_instr &in = instr[wf[w]];
        if (in.a != a || in.b != b) return false;
        const bool str_op = (in.op == SPK_OP_STR_CMP && (in.cmp == SPK_CMP_EQ || in.cmp == SPK_CMP_NE)) ||
                            in.op == SPK_OP_JW || in.op == SPK_OP_LEV || in.op == SPK_OP_LEVRATIO;
        const bool num_op = in.op == SPK_OP_NUM_CMP || in.op == SPK_OP_ABSDIFF || in.op == SPK_OP_PERCDIFF;
        if (!(s.kind == SK_STR ? str_op : num_op)) return false;
        s.op[i] = in.op;
        s.cmp[i] = in.cmp;
        s.level[i] = wl[w];
        s.t[i] = in.t;
    }
    *out = s;
    return true;
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
        bool logical = in.op == SPK_OP_AND || in.op == SPK_OP_OR || in.op == SPK_OP_NOT || in.op == SPK_OP_CONST;
        if (!logical) {
            SPK_REQUIRE(in.a >= 0 && in.a < n_operands, SPK_E_INVALID, "spk_gammas: operand index");
            bool two = !(in.op == SPK_OP_ISNULL || in.op == SPK_OP_NOTNULL || in.op == SPK_OP_LEN);
            if (two) SPK_REQUIRE(in.b >= 0 && in.b < n_operands, SPK_E_INVALID, "spk_gammas: operand index");
        }
        if (in.op == SPK_OP_CONST) SPK_REQUIRE(in.i0 >= 0 && in.i0 <= 2, SPK_E_INVALID, "spk_gammas: constant");
    }
    ctx->codes_valid = false;  // codes are rewritten in place below
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
    lu.resize(lu.size() + 8, 0);  // 4-unit vector reads past a literal's end stay in the buffer
    loff.push_back((int64_t)lu.size());
    llen.push_back(0);
    lcp.push_back(0);

    SPK_TRY(ensure_desc(ctx, t0));
    SPK_TRY(ensure_desc(ctx, t1));
    const int K = n_cols;
    std::vector<SimpleCol> simple;
    std::vector<int32_t> complex_k;
    for (int k = 0; k < K; ++k) {
        SimpleCol sc;
        if (ctx->simple_columns &&
            classify_simple(k, cols[k], when_first_instr, when_n_instr, when_level, instr, operands, t0, t1,
                            ctx->stride, &sc))
            simple.push_back(sc);
        else
            complex_k.push_back(k);
    }
    // Every program array goes up in one packed copy into a buffer the context keeps.
    std::vector<uint8_t> blob;
    auto put = [&](const auto *src, size_t n) -> size_t {
        const size_t off = (blob.size() + 15) & ~(size_t)15;
        blob.resize(off + (n ? n : 1) * sizeof(*src), 0);
        if (n) std::memcpy(blob.data() + off, src, n * sizeof(*src));
        return off;
    };
    const size_t o_prog = put(cols, (size_t)K), o_wf = put(when_first_instr, (size_t)n_when),
                 o_wn = put(when_n_instr, (size_t)n_when), o_wl = put(when_level, (size_t)n_when),
                 o_instr = put(instr, (size_t)n_instr), o_ops = put(operands, (size_t)n_operands),
                 o_lu = put(lu.data(), lu.size()), o_loff = put(loff.data(), loff.size()),
                 o_llen = put(llen.data(), llen.size()), o_lcp = put(lcp.data(), lcp.size()),
                 o_stride = put(ctx->stride.data(), ctx->stride.size()), o_simple = put(simple.data(), simple.size()),
                 o_complex = put(complex_k.data(), complex_k.size());
    const int32_t zero = 0;
    const size_t o_err = put(&zero, 1);
    SPK_TRY(ctx->prog_blob.alloc(blob.size()));
    SPK_HIP(hipMemcpyAsync(ctx->prog_blob.p, blob.data(), blob.size(), hipMemcpyHostToDevice, ctx->stream));
    uint8_t *base = ctx->prog_blob.p;
    auto at = [&](auto *&dst, size_t off) { dst = reinterpret_cast<std::remove_reference_t<decltype(dst)>>(base + off); };
    const int64_t P = ctx->n_pairs;
    SPK_TRY(ctx->work.alloc((size_t)K * (size_t)P + 1));
    SPK_TRY(ctx->work_count.alloc((size_t)K));
    SPK_TRY(ctx->codes.alloc((size_t)(P + 1) * ctx->code_bytes));
    // one filter workgroup per region of consecutive pair ordinals (a multiple of the wave size)
    const int n_regions = (int)std::max<int64_t>(1, std::min<int64_t>(2048, (P + F_THREADS - 1) / F_THREADS));
    const int64_t region_len = ((P + n_regions - 1) / n_regions + 63) / 64 * 64;
    SPK_TRY(ctx->region_count.alloc((size_t)K * n_regions));
    SPK_HIP(hipMemsetAsync(ctx->region_count.p, 0, sizeof(unsigned int) * K * n_regions, ctx->stream));
    SPK_HIP(hipMemsetAsync(ctx->work_count.p, 0, sizeof(unsigned int) * K, ctx->stream));

    GammaArgs A{};
    A.cols0 = t0.d_desc.p;
    A.cols1 = t1.d_desc.p;
    A.pl = ctx->pl.p;
    A.pr = ctx->pr.p;
    A.P = P;
    A.K = K;
    at(A.progs, o_prog);
    at(A.when_first, o_wf);
    at(A.when_n, o_wn);
    at(A.when_level, o_wl);
    at(A.instr, o_instr);
    at(A.ops, o_ops);
    at(A.lit_units, o_lu);
    at(A.lit_off, o_loff);
    at(A.lit_len, o_llen);
    at(A.lit_cplen, o_lcp);
    at(A.stride, o_stride);
    at(A.simple, o_simple);
    at(A.complex_k, o_complex);
    at(A.err, o_err);
    A.codes = ctx->codes.p;
    A.code16 = ctx->code_bytes == 2;
    A.work = ctx->work.p;
    A.region_count = ctx->region_count.p;
    A.region_len = region_len;
    A.n_regions = n_regions;
    A.slow_count = ctx->work_count.p;
    A.n_simple = (int)simple.size();
    A.n_complex = (int)complex_k.size();
    ctx->last_simple = (int)simple.size();

    SPK_TRY(ctx->begin(K_GAMMA));
    if (P > 0) {
        k_gamma_simple<<<(unsigned)n_regions, F_THREADS, 0, ctx->stream>>>(A);
        SPK_HIP(hipGetLastError());
        if (A.n_complex) {
            k_gamma_filter<<<(unsigned)n_regions, F_THREADS, 0, ctx->stream>>>(A);
            SPK_HIP(hipGetLastError());
        }
    }
    std::vector<unsigned int> rc((size_t)K * n_regions, 0);
    SPK_HIP(hipMemcpyAsync(rc.data(), ctx->region_count.p, sizeof(unsigned int) * rc.size(), hipMemcpyDeviceToHost,
                           ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    std::vector<int64_t> counts((size_t)2 * K, 0);
    for (int k = 0; k < K; ++k)
        for (int b = 0; b < n_regions; ++b) counts[k] += rc[(size_t)k * n_regions + b];
    std::vector<int64_t> slow_off(K + 1, 0);
    for (int k = 0; k < K; ++k) slow_off[k + 1] = slow_off[k] + counts[k];
    SPK_TRY(ctx->slow.alloc((size_t)slow_off[K] + 1));
    SPK_TRY(ctx->slow_off.alloc(slow_off.size()));
    SPK_HIP(hipMemcpyAsync(ctx->slow_off.p, slow_off.data(), slow_off.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    A.slow = ctx->slow.p;
    A.slow_off = ctx->slow_off.p;
    std::vector<int> simple_of(K, -1);
    for (size_t i = 0; i < simple.size(); ++i) simple_of[simple[i].k] = (int)i;
    for (int k = 0; k < K; ++k) {
        if (!counts[k]) continue;
        if (simple_of[k] >= 0 && simple[simple_of[k]].kind == SK_STR)
            k_gamma_exact_simple<<<(unsigned)n_regions, X_THREADS, 0, ctx->stream>>>(A, simple_of[k]);
        else
            k_gamma_exact<<<(unsigned)n_regions, X_THREADS, 0, ctx->stream>>>(A, k);
        SPK_HIP(hipGetLastError());
    }
    std::vector<unsigned int> slow_counts((size_t)K, 0);
    SPK_HIP(hipMemcpyAsync(slow_counts.data(), ctx->work_count.p, sizeof(unsigned int) * K, hipMemcpyDeviceToHost,
                           ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    for (int k = 0; k < K; ++k) counts[K + k] = slow_counts[k];
    int64_t n_slow = 0;
    for (int k = 0; k < K; ++k) {
        const unsigned int ns = counts[K + k];
        n_slow += ns;
        if (!ns) continue;
        k_gamma_slow<<<(unsigned)((ns + 63) / 64), 64, 0, ctx->stream>>>(A, k, ctx->slow.p + slow_off[k], ns);
        SPK_HIP(hipGetLastError());
    }
    SPK_TRY(ctx->end(K_GAMMA));
    int err = 0;
    SPK_HIP(hipMemcpyAsync(&err, A.err, sizeof(err), hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    SPK_REQUIRE(!(err & 1), SPK_E_LIMIT, "spk_gammas: a compared string exceeds 1024 UTF-16 units");
    SPK_REQUIRE(!(err & 2), SPK_E_INVALID, "spk_gammas: unknown instruction");
    ctx->codes_valid = true;
    ctx->mpat_valid = false;
    ctx->last_deferred = n_slow;
    ctx->last_exact.assign(counts.begin(), counts.begin() + K);
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
// Same device code as the comparison passes: LDS-staged jw_small / lev_myers for short strings,
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

__global__ __launch_bounds__(U_THREADS) void k_udf(UdfArgs U) {
    __shared__ uint16_t lds[2][MAXU][U_THREADS];
    uint16_t *slot_a = &lds[0][0][threadIdx.x];
    uint16_t *slot_b = &lds[1][0][threadIdx.x];
    int64_t p = (int64_t)blockIdx.x * U_THREADS + threadIdx.x;
    if (p >= U.n) return;
    const StrView a = plain_view(U.u16 + U.off[2 * p], (int32_t)(U.off[2 * p + 1] - U.off[2 * p]), U.cp[2 * p]);
    const StrView b =
        plain_view(U.u16 + U.off[2 * p + 1], (int32_t)(U.off[2 * p + 2] - U.off[2 * p + 1]), U.cp[2 * p + 1]);
    if (a.n > SLOW_LIMIT || b.n > SLOW_LIMIT) {
        atomicOr(U.err, 1);
        U.out[p] = NAN;
        return;
    }
    if (U.op == 0) {
        double v;
        if (a.n <= MAXU && b.n <= MAXU) {
            stage<U_THREADS>(slot_a, a);
            stage<U_THREADS>(slot_b, b);
            v = jw_small(LdsAcc<U_THREADS>{slot_a}, a.n, LdsAcc<U_THREADS>{slot_b}, b.n);
        } else {
            v = jw_long(GlbAcc{a.p}, a.n, GlbAcc{b.p}, b.n);
        }
        U.out[p] = v;
    } else {
        int v;
        if (a.n <= MAXU && b.n <= MAXU && a.ncp == a.n && b.ncp == b.n) {
            stage<U_THREADS>(slot_a, a);
            stage<U_THREADS>(slot_b, b);
            v = lev_myers(LdsAcc<U_THREADS>{slot_a}, a.n, LdsAcc<U_THREADS>{slot_b}, b.n);
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
    if (n) {
        UdfArgs U{n, d_u.p, d_off.p, d_cp.p, op, d_out.p, d_err.p};
        k_udf<<<(unsigned)((n + U_THREADS - 1) / U_THREADS), U_THREADS, 0, ctx->stream>>>(U);
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

extern "C" int spk_gammas_exact_counts(spk_ctx *ctx, int64_t *out, int n) {
    SPK_REQUIRE(ctx && out && n >= (int)ctx->last_exact.size(), SPK_E_INVALID, "spk_gammas_exact_counts: bad args");
    for (size_t k = 0; k < ctx->last_exact.size(); ++k) out[k] = ctx->last_exact[k];
    return SPK_OK;
}

extern "C" int spk_gammas_set_simple(spk_ctx *ctx, int on) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    ctx->simple_columns = on != 0;
    return SPK_OK;
}

extern "C" int spk_gammas_simple_count(spk_ctx *ctx, int *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "null arg");
    *out = ctx->last_simple;
    return SPK_OK;
}
