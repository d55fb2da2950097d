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
#include <chrono>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <type_traits>
#include <cmath>

#include "spk_gamma.h"

namespace spk {

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
                         uint16_t *slot_b, Memo &mm, bool *slow, const Scratch &S) {
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
                    } else if (MODE == M_HUGE) {
                        v = jw_long(GlbAcc{a.p}, a.n, GlbAcc{b.p}, b.n, S.at<uint64_t>(0), S.at<uint64_t>(S.words));
                    } else if (MODE == M_SLOW) {
                        if (a.n > SLOW_LIMIT || b.n > SLOW_LIMIT) { *slow = true; return KN; }  // huge pass
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
                    } else if (MODE == M_HUGE) {
                        v = lev_long(a, b, S.at<uint32_t>(0), S.at<int32_t>(S.units));
                    } else if (MODE == M_SLOW) {
                        if (a.n > SLOW_LIMIT || b.n > SLOW_LIMIT) { *slow = true; return KN; }  // huge pass
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
                           int &level, const Scratch &S = Scratch{}) {
    const spk_column_program prog = A.progs[k];
    Memo mm{-1, -1, 0.0, 0, -1, -1};
    for (int w = 0; w < prog.n_when; ++w) {
        const int wi = prog.first_when + w;
        bool slow = false;
        const int r = eval_pred<MODE>(A, A.when_first[wi], A.when_n[wi], x, y, slot_a, slot_b, mm, &slow, S);
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

template <class SC>
__device__ __attribute__((always_inline)) inline int simple_str(const SC &sc, const RecMeta &a, const RecMeta &b, int &level) {
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

// rows_img: the image's row capacity (its chunk stride); rows [0, n) are filled.
__global__ void k_build_image(int64_t n, const ColDesc *__restrict__ cols, const SimpleCol *__restrict__ simple,
                              int n_simple, uint8_t *__restrict__ img, int64_t rows_img) {
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= n) return;
    for (int j = 0; j < n_simple; ++j) {
        const SimpleCol &sc = simple[j];
        const ColDesc &c = cols[sc.col];
        if (sc.cls == SC_NUM) {
            const bool ok = c.valid[row] != 0;
            *reinterpret_cast<double *>(img + img_at(rows_img, row, sc.off)) = ok ? c.val[row] : 0.0;
            *reinterpret_cast<uint2 *>(img + img_at(rows_img, row, sc.off + 8)) = make_uint2(ok ? 1u : 0u, 0u);
            continue;
        }
        const RecMeta m = c.meta[row];
        uint32_t lens = LENS_NULL;
        if (m.len16 >= 0) {
            const int l16 = m.len16 < LEN_SAT ? m.len16 : LEN_SAT;
            const int lcp = meta_cplen(m) < LEN_SAT ? meta_cplen(m) : LEN_SAT;
            lens = (uint32_t)l16 | ((uint32_t)lcp << 16);
        }
        if (sc.eq4) {  // half of a JW gap: the id alone (NULL = all ones; ids are dense, < 2^32 - 1)
            *reinterpret_cast<uint32_t *>(img + img_at(rows_img, row, sc.off)) = m.len16 < 0 ? 0xFFFFFFFFu : m.key;
            continue;
        }
        *reinterpret_cast<uint2 *>(img + img_at(rows_img, row, sc.off)) = make_uint2(m.key, lens);
        if (sc.cls != SC_EQ) *reinterpret_cast<uint64_t *>(img + img_at(rows_img, row, sc.off + 8)) = m.sketch;
        if (sc.cls == SC_JW) *reinterpret_cast<uint64_t *>(img + img_at(rows_img, row, sc.off2)) = m.head;
    }
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
        A.region_count[(int64_t)A.complex_k[i] * A.n_regions + A.region_base + blockIdx.x] = s_cnt[i];
}

// The exact passes run over column k's compacted work list -- every region's undecided pairs back
// to back (k_compact) -- with a grid-stride loop, so every CU gets the same share of cells however
// unevenly they fall over the regions (a region of one large block can hold several times the
// average).  Block b of k_compact copies region b's list to its prefix offset.
//
// The lists are sized on the device, so the pass needs no host round trip between the filter and
// the exact kernels: k_prefix scans the region counts of every column (one workgroup) into
// xpref[k][b] and xinfo = [col_base[K] | col_count[K] | overflow | total].  Column k's list
// starts at xlist + col_base[k]; its slow-pass list (a subset) at the same offset in the second
// half of xlist.  If the lists exceed the capacity, `overflow` makes every exact kernel a no-op
// and the host re-runs the phase with room for `total` (codes are untouched until then).
constexpr int PFX_THREADS = 1024;
constexpr int PFX_PER = 8;  // region counts a k_prefix thread keeps in registers
__global__ __launch_bounds__(PFX_THREADS) void k_prefix(const unsigned int *__restrict__ region_count, int K,
                                                        int n_regions, int64_t cap, int64_t *__restrict__ xpref,
                                                        int64_t *__restrict__ xinfo, unsigned long long *__restrict__ done) {
    // One workgroup per column (blockIdx.x): wave-level inclusive scans (shuffles) and one scan of the
    // 16 wave totals, two barriers.  A thread's counts (<= PFX_PER of them, 5 at 20 regions per CU)
    // stay in registers.  The last workgroup to finish (device-scope counter) lays the columns' lists
    // out one after another and flags an overflow of `cap`.
    constexpr int NW = PFX_THREADS / 64;
    __shared__ int64_t wsum[NW];
    __shared__ bool s_last;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int per = (n_regions + PFX_THREADS - 1) / PFX_THREADS;
    const int b0 = threadIdx.x * per;
    const bool in_regs = per <= PFX_PER;  // block-uniform
    const int k = blockIdx.x;
    const unsigned int *rc = region_count + (int64_t)k * n_regions;
    unsigned int cur[PFX_PER];
    int64_t mine = 0;
    if (in_regs) {
#pragma unroll
        for (int q = 0; q < PFX_PER; ++q) {
            cur[q] = (q < per && b0 + q < n_regions) ? rc[b0 + q] : 0u;
            mine += cur[q];
        }
    } else {
        for (int b = b0; b < b0 + per && b < n_regions; ++b) mine += rc[b];
    }
    int64_t v = mine;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    if (wave == 0) {
        int64_t w = lane < NW ? wsum[lane] : 0;
#pragma unroll
        for (int off = 1; off < NW; off <<= 1) {
            const int64_t t = __shfl_up(w, off, 64);
            if (lane >= off) w += t;
        }
        if (lane < NW) wsum[lane] = w;
    }
    __syncthreads();
    int64_t acc = v - mine + (wave > 0 ? wsum[wave - 1] : 0);  // exclusive
    int64_t *pf = xpref + (int64_t)k * (n_regions + 1);
    if (in_regs) {
#pragma unroll
        for (int q = 0; q < PFX_PER; ++q) {
            if (q < per && b0 + q < n_regions) pf[b0 + q] = acc;
            acc += cur[q];
        }
    } else {
        for (int b = b0; b < b0 + per && b < n_regions; ++b) {
            pf[b] = acc;
            acc += rc[b];
        }
    }
    if (threadIdx.x == 0) {
        const int64_t tot = wsum[NW - 1];
        pf[n_regions] = tot;
        xinfo[K + k] = tot;
        __threadfence();
        s_last = atomicAdd(done, 1ull) == (unsigned long long)(K - 1);
    }
    __syncthreads();
    if (s_last && threadIdx.x == 0) {
        __threadfence();
        int64_t base = 0;
        for (int c = 0; c < K; ++c) {
            xinfo[c] = base;
            base += (int64_t)atomicAdd(reinterpret_cast<unsigned long long *>(&xinfo[K + c]), 0ull);  // from L2
        }
        xinfo[2 * K] = base > cap ? 1 : 0;
        xinfo[2 * K + 1] = base;
        *done = 0;  // ready for a re-run of the phase
    }
}

// Up to four columns per launch (blockIdx.y picks the column): the JW template columns' lists are
// compacted, their slow lists evaluated, in one launch each instead of one per column.
struct ColSet {
    int n;
    int k[4];
};

__global__ void k_compact(GammaArgs A, ColSet cs, const int64_t *__restrict__ xpref, int32_t *__restrict__ xlist,
                          const int64_t *__restrict__ xinfo) {
    if (xinfo[2 * A.K]) return;  // overflow: the host re-runs the phase
    const int k = cs.k[blockIdx.y];
    const int64_t *pref = xpref + (int64_t)k * (A.n_regions + 1);
    const Region R = my_region(A);
    const int32_t *src = region_list(A, k, R);
    const int64_t n = A.region_count[(int64_t)k * A.n_regions + blockIdx.x];
    int32_t *dst = xlist + xinfo[k] + pref[blockIdx.x];
    // four entries per thread in flight before their stores (a long region's copy is latency-bound otherwise)
    const int64_t bd = blockDim.x;
    for (int64_t i = threadIdx.x; i < n; i += 4 * bd) {
        int32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i + u * bd < n ? src[i + u * bd] : 0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * bd < n) dst[i + u * bd] = v[u];
    }
}

__device__ inline int64_t exact_count(const GammaArgs &A, const int64_t *xinfo, int k) {
    return xinfo[2 * A.K] ? 0 : xinfo[A.K + k];
}

__device__ inline int simple_lev_cut(const SimpleCol &sc, int ncp_a, int ncp_b);
__device__ inline int lev_level_of(const SimpleCol &sc, int eq, int lev, int nsum);

// Upper bound on the multiset intersection of two rows from their character-bag rows (k_bag_rows), or -1 when
// a bucket is saturated on both sides.  Σ min(a, b) = (Σ a + Σ b - Σ |a - b|) / 2 over the nibbles, spread to
// bytes (v_sad_u8 sums four absolute byte differences).
__device__ inline int bag_inter_ub(const uint4 &a0, const uint4 &a1, const uint4 &b0, const uint4 &b1) {
    const uint32_t wa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w & 0xFFFFu};
    const uint32_t wb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w & 0xFFFFu};
    uint32_t sad = 0, sa = 0, sb = 0, sat = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const uint32_t la = wa[q] & 0x0F0F0F0Fu, ha = (wa[q] >> 4) & 0x0F0F0F0Fu;
        const uint32_t lb = wb[q] & 0x0F0F0F0Fu, hb = (wb[q] >> 4) & 0x0F0F0F0Fu;
        sad = __builtin_amdgcn_sad_u8(la, lb, sad);
        sad = __builtin_amdgcn_sad_u8(ha, hb, sad);
        sa = __builtin_amdgcn_sad_u8(la, 0u, sa);
        sa = __builtin_amdgcn_sad_u8(ha, 0u, sa);
        sb = __builtin_amdgcn_sad_u8(lb, 0u, sb);
        sb = __builtin_amdgcn_sad_u8(hb, 0u, sb);
        const uint32_t t = wa[q] & wb[q];
        sat |= t & (t >> 1) & (t >> 2) & (t >> 3) & 0x11111111u;
    }
    if (sat) return -1;
    const int oa = (int)((a1.w >> 16) & 0xFFu), ob = (int)((b1.w >> 16) & 0xFFu);
    return (int)((sa + sb - sad) / 2u) + (oa < ob ? oa : ob);
}

// k_compact for a Levenshtein column: a listed cell whose rows' bag distance already exceeds the cut is decided
// here (its level is lev_cell's for any distance past the cut), one with a row past 64 units goes straight to
// the slow list; the others are packed to the front of the
// region's slice of the list in order, and the slice's tail is -1, which the exact passes skip (whole waves of
// it, mostly).  0.206 ms per cfg5 call (round 5); four cells per thread per round (their loads in flight together)
// took 0.260, and unordered packing through one LDS counter per workgroup (no barriers) 0.210.  Round 6 sorts the
// slow cells (0.272 ms) and pipelines the loads across rounds (0.242 ms, profiles/r6_ab_compact_lev_pipeline.log).
constexpr int CL_THREADS = 256;
constexpr int CL_SLOW = 1024;  // LDS buffer of slow-list cells per workgroup
__global__ __launch_bounds__(CL_THREADS) void k_compact_lev(GammaArgs A, int k, int si, const int64_t *__restrict__ xpref,
                                                            int32_t *__restrict__ xlist, const int64_t *__restrict__ xinfo) {
    if (xinfo[2 * A.K]) return;  // overflow: the host re-runs the phase
    __shared__ SimpleCol s_sc;
    __shared__ int s_kept[CL_THREADS / 64];
    __shared__ int32_t s_slow[CL_SLOW];
    __shared__ uint8_t s_skey[CL_SLOW];     // the buffered slow cells' shorter row length (sort key)
    __shared__ uint16_t s_srank[CL_SLOW];   // rank of each among the cells of its key
    __shared__ unsigned int s_sbin[3 * 64];  // counting-sort bins (keys 0 .. 128)
    __shared__ int s_ns;
    __shared__ unsigned int s_sbase;
    if (threadIdx.x == 0) {
        s_sc = A.simple[si];
        s_ns = 0;
    }
    __syncthreads();
    const SimpleCol &sc = s_sc;
    const int64_t *pref = xpref + (int64_t)k * (A.n_regions + 1);
    const Region R = my_region(A);
    const int32_t *src = region_list(A, k, R);
    const int64_t n = A.region_count[(int64_t)k * A.n_regions + blockIdx.x];
    int32_t *dst = xlist + xinfo[k] + pref[blockIdx.x];
    const uint4 *bag0 = A.cols0[sc.col].bag, *bag1 = A.cols1[sc.col].bag;
    const uint32_t stride = (uint32_t)sc.stride;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int32_t *slow_list = A.slow + A.slow_off[k];
    // The buffered slow cells to the slow list (one device atomic), in order of their shorter row's length: the
    // 128-bit pass runs a wave as long as its slowest lane, and cells of similar lengths scan similarly long
    // (host simulation over cfg5's bag-filtered slow cells: lane utilisation 0.53 -> 0.60 sorted per 1,024 cells).
    // A counting sort through LDS: one LDS atomic per cell, a 192-bin scan in wave 0, one scatter.
    auto flush_slow = [&]() {
        const int c = s_ns;
        if (threadIdx.x == 0) s_sbase = atomicAdd(A.slow_count + k, (unsigned int)c);
        if (threadIdx.x < 3 * 64) s_sbin[threadIdx.x] = 0;
        __syncthreads();
        for (int j = threadIdx.x; j < c; j += CL_THREADS) s_srank[j] = (uint16_t)atomicAdd(&s_sbin[s_skey[j]], 1u);
        __syncthreads();
        if (threadIdx.x < 64) {  // wave 0: exclusive scan, three bins per lane
            const int t = threadIdx.x;
            const unsigned int a = s_sbin[3 * t], b = s_sbin[3 * t + 1], d = s_sbin[3 * t + 2];
            unsigned int v = a + b + d;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const unsigned int u = __shfl_up(v, off, 64);
                if (t >= off) v += u;
            }
            const unsigned int ex = v - a - b - d;
            s_sbin[3 * t] = ex;
            s_sbin[3 * t + 1] = ex + a;
            s_sbin[3 * t + 2] = ex + a + b;
        }
        __syncthreads();
        for (int j = threadIdx.x; j < c; j += CL_THREADS) slow_list[s_sbase + s_sbin[s_skey[j]] + s_srank[j]] = s_slow[j];
        __syncthreads();
        if (threadIdx.x == 0) s_ns = 0;
    };
    int64_t kept = 0;  // block-uniform
    // software pipeline: the next round's pair rows and the list entry after that are in flight with this
    // round's bag rows, so a round waits on one memory round trip instead of three
    int32_t pc = 0, xc = 0, yc = 0;
    if (threadIdx.x < n) {
        pc = src[threadIdx.x];
        xc = A.pl[pc];
        yc = A.pr[pc];
    }
    int32_t pn = threadIdx.x + CL_THREADS < n ? src[threadIdx.x + CL_THREADS] : 0;
    for (int64_t i0 = 0; i0 < n; i0 += CL_THREADS) {
        const int64_t i = i0 + threadIdx.x;
        // unconditional loads at clamped indices (pair 0's rows, the list's last entry), no branch around them:
        // this round's bag rows, the next round's pair rows, the list entry after that
        const uint4 a0 = bag0[2 * (int64_t)xc], a1 = bag0[2 * (int64_t)xc + 1];
        const uint4 b0 = bag1[2 * (int64_t)yc], b1 = bag1[2 * (int64_t)yc + 1];
        const int64_t i2 = i + CL_THREADS, i3 = i2 + CL_THREADS;
        const int32_t p2 = i2 < n ? pn : 0;
        const int32_t x2 = A.pl[p2], y2 = A.pr[p2];
        pn = src[i3 < n ? i3 : n - 1];
        __builtin_amdgcn_sched_barrier(0);  // all issued before the first wait
        // the bound before any branch on the rows' lengths, so no load is sunk into one (two round trips)
        const int la = (int)(a1.w >> 24), lb = (int)(b1.w >> 24);
        int inter = bag_inter_ub(a0, a1, b0, b1);
        bool keep = false, slow = false;
        const int32_t p = pc;
        int skey = 0;
        if (i < n) {
            keep = true;
            if (la != 255 && lb != 255) {
                // a row past 64 units has no 64-bit planes: the exact pass would only pass the cell on to the
                // 128-bit slow pass, after loading its rows -- it goes to the slow list from here
                slow = la > 64 || lb > 64;
                skey = la < lb ? la : lb;  // <= 128: rows with bag rows have at most 128 units
                if (inter >= 0) {
                    const int mn = la < lb ? la : lb, mx = la < lb ? lb : la;
                    inter = inter < mn ? inter : mn;
                    const int cut = simple_lev_cut(sc, la, lb);
                    if (mx - inter > cut) {  // unequal rows (a positive bag distance), distance past the cut
                        code_add_atomic(A, p, (uint32_t)(lev_level_of(sc, 0, cut + 1, la + lb) + 1) * stride);
                        keep = slow = false;
                    }
                }
            }
        }
        const unsigned long long ms = __ballot(keep && slow);
        if (ms) {  // into the workgroup's LDS buffer (the device counter once per CL_SLOW cells: a shared
                   // counter per wave serialised, 2.9 ms per cfg5 call)
            int sb = 0;
            if (lane == 0) sb = atomicAdd(&s_ns, __popcll(ms));
            sb = __shfl(sb, 0);
            if (keep && slow) {
                const int q = sb + __popcll(ms & ((1ull << lane) - 1ull));
                s_slow[q] = p;
                s_skey[q] = (uint8_t)skey;
            }
            keep = keep && !slow;
        }
        const unsigned long long m = __ballot(keep);
        if (lane == 0) s_kept[wv] = __popcll(m);
        __syncthreads();
        int off = 0, tot = 0;
#pragma unroll
        for (int q = 0; q < CL_THREADS / 64; ++q) {
            off += q < wv ? s_kept[q] : 0;
            tot += s_kept[q];
        }
        if (keep) dst[kept + off + __popcll(m & ((1ull << lane) - 1ull))] = p;
        kept += tot;
        if (s_ns > CL_SLOW - CL_THREADS || i0 + CL_THREADS >= n) flush_slow();  // block-uniform (after the barrier)
        __syncthreads();
        pc = p2;
        xc = x2;
        yc = y2;
    }
    for (int64_t i = kept + threadIdx.x; i < n; i += CL_THREADS) dst[i] = -1;
}

// Exact pass over column k through the interpreter.
__global__ __launch_bounds__(X_THREADS) void k_gamma_exact(GammaArgs A, int k, const int32_t *xlist,
                                                            const int64_t *xinfo) {
    const int64_t n = exact_count(A, xinfo, k);
    const int32_t *items = xlist + xinfo[k];
    uint16_t *slot_a = nullptr, *slot_b = nullptr;  // the exact pass works from registers and L1/L2
    const int64_t stride = (int64_t)gridDim.x * X_THREADS;
    for (int64_t base = (int64_t)blockIdx.x * X_THREADS; base < n; base += stride) {  // block-uniform
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

// Per len_l + len_r (S < S_MAX): the scan's cut and each test's largest passing distance for unequal strings
// (the filter's integer forms: lev_a, the host's ratio tables), and *tab = 1 when every test is a `<=` / `<` on
// the distance or a string (in)equality, so a cell's level is a table lookup.  Callers barrier after it.
template <int S_MAX, int CUT_MAX>
__device__ inline void lev_tables(const GammaArgs &A, const SimpleCol &sc, uint8_t *s_cut, int16_t (*s_bp)[MAX_TESTS],
                                  int *tab) {
    for (int S = threadIdx.x; S < S_MAX; S += X_THREADS) {  // blocks of X_THREADS
        const int c = simple_lev_cut(sc, S, 0);
        s_cut[S] = (uint8_t)(c < CUT_MAX ? c : CUT_MAX);
        for (int i = 0; i < sc.n_tests; ++i) {
            int bp = -1;
            if (sc.op[i] == SPK_OP_STR_CMP) bp = sc.cmp[i] == SPK_CMP_EQ ? -1 : CUT_MAX + 1;
            else if (sc.op[i] == SPK_OP_LEV) bp = sc.lev_a[i];
            else if (sc.thr_off[i] >= 0 && S < THR_S) bp = A.thr[sc.thr_off[i] + S];
            else if (sc.thr_off[i] >= 0) {  // len_l + len_r past the host tables (WW = 2: S = 256): the same scan
                const double den = (double)S / 2.0;
                for (int v = 0; v <= CUT_MAX + 1 && cmpd((double)v / den, sc.t[i], sc.cmp[i]) == KT; ++v) bp = v;
            }
            s_bp[S][i] = (int16_t)(bp < -1 ? -1 : (bp > CUT_MAX + 1 ? CUT_MAX + 1 : bp));
        }
    }
    if (threadIdx.x == 0) {
        int ok = 1;
        for (int i = 0; i < sc.n_tests; ++i) {
            const int op = sc.op[i];
            if (op == SPK_OP_LEV) ok &= (sc.tflag[i] & (TF_GE | TF_EXACT)) ? 0 : 1;
            else if (op == SPK_OP_LEVRATIO) ok &= sc.thr_off[i] >= 0 ? 1 : 0;
            else ok &= op == SPK_OP_STR_CMP ? 1 : 0;
        }
        *tab = ok;
    }
}

__device__ int simple_exact(const GammaArgs &A, const SimpleCol &sc, const ColDesc &c0, const ColDesc &c1, int32_t x,
                            int32_t y, int &level) {
    uint64_t pa[N_PLANES], pb[N_PLANES];
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
                    else if (a.planes && b.planes) {
#pragma unroll
                        for (int q = 0; q < N_PLANES; ++q) {
                            pa[q] = a.planes[q];
                            pb[q] = b.planes[q];
                        }
                        lev = lev_rows_planes(pa, a.n, pb, b.n, simple_lev_cut(sc, a.ncp, b.ncp), sc.np);
                    } else {
                        lev = lev_exact(a, b, simple_lev_cut(sc, a.ncp, b.ncp));
                    }
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

// Exact pass cell of a Jaro-Winkler template column (every test `jaro_winkler_sim > / >= t`): the JW
// code alone, so its kernel keeps a small register budget (X_JW).
__device__ int jw_cell(const SimpleCol &sc, const ColDesc &c0, const ColDesc &c1, int32_t x, int32_t y, int &level) {
    const RecMeta ma = c0.meta[x], mb = c1.meta[y];
    if (ma.len16 < 0 || mb.len16 < 0) {
        level = sc.null_level;
        return ST_DONE;
    }
    const StrView a = row_view(c0, ma, x, sc.col), b = row_view(c1, mb, y, sc.col);
    int eq = meta_equal(ma, mb);
    if (eq < 0) eq = units_equal(a, b) ? 1 : 0;
    double jw;
    if (eq == 1) jw = a.n > 0 ? 1.0 : 0.0;
    else if (a.n > 64 || b.n > 64) return ST_NEEDS_SLOW;
    else jw = jw_exact(a, b);
    for (int i = 0; i < sc.n_tests; ++i) {
        if (cmpd(jw, sc.t[i], sc.cmp[i]) == KT) {
            level = sc.level[i];
            return ST_DONE;
        }
    }
    level = sc.else_level;
    return ST_DONE;
}

// Exact pass cell of a Levenshtein-class template column (tests: `=` / `<>`, levenshtein [ratio]):
// both rows' bit-planes are loaded in the same round trip as the records and the distance comes
// from them alone (lev_rows_planes).  Rows without planes (> 64 units or a unit >= 256) go to the
// global-memory pass.  A kernel of its own, so its register budget is not the JW path's.
// The column descriptors come from LDS, so their pointers are generic: the records and planes are read through
// global-address-space views (global_load, not flat -- a flat load also counts against lgkmcnt, so every wait on
// it waits for the LDS reads too).
typedef const __attribute__((address_space(1))) uint64_t GU64;
__device__ __attribute__((always_inline)) inline RecMeta load_meta_global(const RecMeta *m, int64_t row) {
    static_assert(sizeof(RecMeta) == 32, "RecMeta: four 8-byte words");
    GU64 *q = (GU64 *)(m + row);
    uint64_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = q[i];
    RecMeta out;
    __builtin_memcpy(&out, w, sizeof(out));
    return out;
}
// cutt / bpt: lev_tables' per len_l + len_r cut and thresholds for a 64-bit scan (nullptr: the tests one by one)
__device__ int lev_cell(const SimpleCol &sc, const ColDesc &c0, const ColDesc &c1, int32_t x, int32_t y, int &level,
                        const uint8_t *cutt = nullptr, const int16_t (*bpt)[MAX_TESTS] = nullptr) {
    uint64_t pa[N_PLANES], pb[N_PLANES];
    {
        GU64 *qa = (GU64 *)(c0.planes + (int64_t)x * N_PLANES);
        GU64 *qb = (GU64 *)(c1.planes + (int64_t)y * N_PLANES);
#pragma unroll
        for (int i = 0; i < N_PLANES; ++i) {
            pa[i] = qa[i];
            pb[i] = qb[i];
        }
    }
    const RecMeta ma = load_meta_global(c0.meta, x), mb = load_meta_global(c1.meta, y);
    if (ma.len16 < 0 || mb.len16 < 0) {
        level = sc.null_level;
        return ST_DONE;
    }
    int eq = meta_equal(ma, mb);
    if (eq < 0) eq = units_equal(row_view(c0, ma, x, sc.col), row_view(c1, mb, y, sc.col)) ? 1 : 0;
    const int na = meta_cplen(ma), nb = meta_cplen(mb);
    const bool planes = (ma.cpf & mb.cpf & CPF_PLANES) != 0;
    int lev = -1;
    for (int i = 0; i < sc.n_tests; ++i) {
        const int op = sc.op[i], cmp = sc.cmp[i];
        const double t = sc.t[i];
        int r;
        if (op == SPK_OP_STR_CMP) {
            r = ((eq == 1) == (cmp == SPK_CMP_EQ)) ? KT : KF;
        } else {
            const double den = (double)(na + nb) / 2.0;
            if (op == SPK_OP_LEVRATIO && den == 0.0) {
                r = KN;
            } else {
                if (lev < 0) {
                    if (eq == 1) lev = 0;
                    else if (!planes) return ST_NEEDS_SLOW;
                    else {
                        const int S = na + nb;  // <= 128: rows of <= 64 units
                        lev = lev_rows_planes(pa, ma.len16, pb, mb.len16, bpt != nullptr ? (int)cutt[S] : simple_lev_cut(sc, na, nb),
                                              sc.np);
                        if (bpt != nullptr) {  // levels by table: the tests before this one failed for eq = 0 too
                            int lv = sc.else_level;
                            for (int j = sc.n_tests - 1; j >= 0; --j) lv = lev <= bpt[S][j] ? sc.level[j] : lv;
                            level = lv;
                            return ST_DONE;
                        }
                    }
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

// The Levenshtein variant is latency-bound (record + plane loads per cell): it keeps registers to
// LEV_WAVES waves per SIMD so enough cells are in flight.
// Work bins of a Levenshtein cell: the scan runs over the shorter row (trip count) with a word as
// wide as the longer one needs, and a wave runs as long as its slowest lane and at the widest word
// any lane needs.  So each workgroup's 256 cells are regrouped by (longer > 32 units, shorter length)
// before they are evaluated: lanes of a wave then get similar trip counts and most waves stay at
// 32-bit words.  Only the assignment of cells to lanes changes; every cell is evaluated once, as
// before.  Cells with a row past 64 units (no 64-bit planes: the 128-bit slow pass takes them) get bins
// of their own, 128 + shorter length, so their waves hold no cell the exact pass evaluates and they
// reach the slow list sorted by that pass's trip count.  Bin LEV_BINS - 1 also holds the empty slots
// past the end of the list.
constexpr int LEV_BINS = 192;
__device__ inline int lev_work_bin(int la, int lb) {
    if (la < 0 || lb < 0) return 0;  // a NULL row: lev_cell settles it at once (not the slow list)
    const int mn = la < lb ? la : lb, mx = la < lb ? lb : la;
    return (mx > 64 ? 128 : (mx > 32 ? 64 : 0)) + (mn < 63 ? mn : 63);
}

// Counting sort of the workgroup's (key, item) by key through LDS: one LDS atomic per lane, a
// LEV_BINS exclusive scan in wave 0 (three bins per lane), one scatter and one gather.  Three barriers.
__device__ inline void lev_sort_items(int &key, bool &have, int32_t &p, int32_t &x, int32_t &y) {
    __shared__ unsigned int s_bin[LEV_BINS];
    __shared__ int32_t s_p[X_THREADS], s_x[X_THREADS], s_y[X_THREADS];
    __shared__ uint8_t s_have[X_THREADS], s_key[X_THREADS];
    const int t = threadIdx.x;
    if (t < LEV_BINS) s_bin[t] = 0;
    __syncthreads();
    const unsigned int r = atomicAdd(&s_bin[key], 1u);
    __syncthreads();
    static_assert(LEV_BINS == 3 * 64, "lev_sort_items scans three bins per lane");
    if (t < 64) {  // wave 0: three bins per lane
        const unsigned int a = s_bin[3 * t], b = s_bin[3 * t + 1], c = s_bin[3 * t + 2];
        unsigned int v = a + b + c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const unsigned int u = __shfl_up(v, off, 64);
            if (t >= off) v += u;
        }
        const unsigned int ex = v - a - b - c;
        s_bin[3 * t] = ex;
        s_bin[3 * t + 1] = ex + a;
        s_bin[3 * t + 2] = ex + a + b;
    }
    __syncthreads();
    const unsigned int pos = s_bin[key] + r;
    s_p[pos] = p;
    s_x[pos] = x;
    s_y[pos] = y;
    s_have[pos] = have ? 1 : 0;
    s_key[pos] = (uint8_t)key;
    __syncthreads();
    p = s_p[t];
    x = s_x[t];
    y = s_y[t];
    have = s_have[t] != 0;
    key = s_key[t];
}

#ifndef SPK_LEV_WAVES
#define SPK_LEV_WAVES 4
#endif
constexpr int LEV_WAVES = SPK_LEV_WAVES;
// The Jaro-Winkler variant keeps its full register budget (138 VGPRs, 3 waves per SIMD): capped at
// 4 waves (128 VGPRs, 40 B of spills) it measured the same on MI355X (52.1 vs 52.3 us per call).
constexpr int JW_WAVES = 1;
// The JW-only cells (jw_cell) take 120 VGPRs: 4 waves per SIMD, twice the workgroups the generic kernel keeps resident.
constexpr int JWC_WAVES = 4;
// Columns of one exact launch: blocks [c g, (c + 1) g) work through column si[c]'s list, so the
// short Jaro-Winkler lists of several columns share one launch (and its tail).
struct ExactCols {
    int n;
    int g;  // blocks per column
    int si[4];
    int k[4], col[4];  // the columns' code positions and table columns (= simple[si].k / .col): the
                       // list bounds and the column descriptors load in one round, not after simple[si]
};

// Diagnostic build only (-DSPK_X_STAMPS): per-workgroup start / end wall-clock stamps (100 MHz) of the JW
// exact launch and the number of cells each workgroup evaluated, read with spk_debug_x_stamps
// (tools/ab_x_stamps.py).
#ifdef SPK_X_STAMPS
constexpr int X_STAMP_BLOCKS = 16384;
__device__ unsigned long long g_x_stamps[5 * X_STAMP_BLOCKS];
#endif
// MODE: X_GENERIC (simple_exact: any simple string column), X_LEV (lev_cell), X_JW (jw_cell).  Each mode
// is its own kernel so its register budget is that of its own cell code: simple_exact carries the
// Levenshtein scans too, and at its 190 VGPRs the JW cells ran 2 waves per SIMD.
enum XMode : int { X_GENERIC = 0, X_LEV = 1, X_JW = 2 };
template <int MODE, int XW = (MODE == X_LEV ? LEV_WAVES : (MODE == X_JW ? JWC_WAVES : JW_WAVES))>
__global__ __launch_bounds__(X_THREADS, XW) void k_gamma_exact_simple(GammaArgs A, ExactCols C,
                                                                   const int32_t *xlist, const int64_t *xinfo) {
    __shared__ SimpleCol s_sc;
    __shared__ ColDesc s_c0, s_c1;
    constexpr int XS_MAX = MODE == X_LEV ? 129 : 1;  // len_l + len_r of 64-bit rows, plus one
    __shared__ uint8_t s_cut[XS_MAX];
    __shared__ int16_t s_bp[XS_MAX][MAX_TESTS];
    __shared__ int s_tab;
#ifdef SPK_X_STAMPS
    unsigned long long x_t0 = wall_clock64(), x_cells = 0, x_t1 = 0, x_t2 = 0;
#endif
    const int col_slot = (int)(blockIdx.x / (unsigned)C.g);  // block-uniform
    const int64_t bid = (int64_t)blockIdx.x - (int64_t)col_slot * C.g;
    int si = C.si[0], k = C.k[0], colx = C.col[0];
#pragma unroll
    for (int c = 1; c < 4; ++c)
        if (c == col_slot) {
            si = C.si[c];
            k = C.k[c];
            colx = C.col[c];
        }
    // one round of independent loads: the column's descriptors (thread 0), the list bounds and every
    // thread's first item and pair rows
    if (threadIdx.x == 0) {
        s_sc = A.simple[si];
        s_c0 = A.cols0[colx];
        s_c1 = A.cols1[colx];
    }
    const int64_t n = exact_count(A, xinfo, k);
    const int32_t *items = xlist + xinfo[k];
    const int64_t stride = (int64_t)C.g * X_THREADS;
    // software pipeline: the next item's pair rows (and, for Levenshtein, the rows' lengths) are in
    // flight while this one is evaluated, and the list entry after that one is read a round earlier still, so
    // the pair-row loads of the next item never wait on its list entry (one memory round trip per cell, shared
    // with the current cell's records and planes)
    int64_t i = bid * X_THREADS + threadIdx.x;
    int32_t p = -1, x = 0, y = 0, key = LEV_BINS - 1;  // p = -1: no cell (past the list, or a k_compact_lev slot)
    if (i < n) {
        p = items[i];
        x = A.pl[p < 0 ? 0 : p];
        y = A.pr[p < 0 ? 0 : p];
    }
    int32_t pn = i + stride < n ? items[i + stride] : -1;  // the next item's list entry
    __syncthreads();
#ifdef SPK_X_STAMPS
    x_t1 = wall_clock64();
#endif
    const SimpleCol &sc = s_sc;
    constexpr bool LEV = MODE == X_LEV;
    if constexpr (LEV) {
        lev_tables<XS_MAX, XS_MAX - 2>(A, sc, s_cut, s_bp, &s_tab);
        __syncthreads();
    }
    const bool tab = LEV && s_tab != 0;  // block-uniform
    // Regroup by work bin only in free-text columns (rows past 64 units, so planes_hi exists): there the
    // trip counts spread widely (cfg5 addresses: 2.98 -> 2.67 ms per call).  In short-string columns
    // the sort's barriers cost more than it saves (cfg2 email: 475 -> 505 us), so they keep the old order.
    const bool regroup = LEV && s_c0.planes_hi != nullptr && s_c1.planes_hi != nullptr;  // block-uniform
    if (regroup && p >= 0) key = lev_work_bin(s_c0.meta[x].len16, s_c1.meta[y].len16);
    for (int64_t base = bid * X_THREADS; base < n; base += stride) {  // block-uniform
        bool have = p >= 0;
        const int64_t i2 = i + stride;
        // unconditional loads (clamped indices: pair 0 and the list's last entry are read harmlessly), so no
        // divergent branch makes the compiler wait on the loads in flight
        const int32_t p2 = i2 < n ? pn : -1;
        const int32_t q2 = p2 < 0 ? 0 : p2;
        const int32_t x2 = A.pl[q2], y2 = A.pr[q2];
        int32_t key2 = LEV_BINS - 1;
        if (regroup && p2 >= 0) key2 = lev_work_bin(s_c0.meta[x2].len16, s_c1.meta[y2].len16);
        const int64_t i3 = i2 + stride;
        const int32_t pn3 = items[i3 < n ? i3 : n - 1];
        pn = i3 < n ? pn3 : -1;
        if (regroup) lev_sort_items(key, have, p, x, y);
        bool to_slow = false;
        if (have && regroup && key >= 128) {
            // a row past 64 units (work bins 128 +): no 64-bit planes, the 128-bit slow pass takes the cell --
            // straight to its list, without loading the rows' planes and records first
            to_slow = true;
        } else if (have) {
            int level = 0;
            int st;
            if constexpr (MODE == X_LEV)
                st = lev_cell(sc, s_c0, s_c1, x, y, level, s_cut, tab ? s_bp : nullptr);
            else if constexpr (MODE == X_JW) st = jw_cell(sc, s_c0, s_c1, x, y, level);
            else st = simple_exact(A, sc, s_c0, s_c1, x, y, level);
#ifdef SPK_X_STAMPS
            if (x_t2 == 0) x_t2 = wall_clock64() + (unsigned long long)(level & 0);
#endif
            if (st != ST_DONE) to_slow = true;
            else if (C.n > 1) code_add_atomic(A, p, (uint32_t)(level + 1) * (uint32_t)sc.stride);
            else code_add(A, p, (uint32_t)(level + 1) * (uint32_t)sc.stride);
        }
        wave_append(A.slow + A.slow_off[k], A.slow_count + k, to_slow, p);
#ifdef SPK_X_STAMPS
        x_cells += have ? 1 : 0;
#endif
        i = i2;
        p = p2;
        x = x2;
        y = y2;
        key = key2;
    }
#ifdef SPK_X_STAMPS
    if (MODE == X_JW && threadIdx.x == 0 && blockIdx.x < X_STAMP_BLOCKS) {
        g_x_stamps[5 * blockIdx.x] = x_t0;
        g_x_stamps[5 * blockIdx.x + 1] = wall_clock64();
        g_x_stamps[5 * blockIdx.x + 2] = x_cells;
        g_x_stamps[5 * blockIdx.x + 3] = x_t1;
        g_x_stamps[5 * blockIdx.x + 4] = x_t2;
    }
#endif
}
#ifdef SPK_X_STAMPS
extern "C" int spk_debug_x_stamps(uint64_t *out, int n) {
    SPK_HIP(hipDeviceSynchronize());
    SPK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x_stamps), sizeof(uint64_t) * (size_t)std::min(n, 5 * X_STAMP_BLOCKS)));
    return SPK_OK;
}
#endif

// ---- Levenshtein exact pass with lane refill from a per-wave queue ----------------------------------------------
// In k_gamma_exact_simple<X_LEV> one lane scans one cell and a wave runs as long as its slowest lane: nearly every
// wave of 64 cells holds one that runs to the end (a pair within the cut) while most stop early, so a wave ran
// ~2-3x the mean trip count (tools/lev_refill_sim.py over the synthetic data: cfg5 addresses 12.8 steps per cell
// on average with the diagonal exit, 39 for the slowest of 64; cfg2 emails 7.5 vs 14.6).  Here a lane that
// finishes takes another cell, so a wave's steps follow the mean:
//   - batch: all 64 lanes set up the next 64 cells of the wave's range at once (full SIMD width, as the per-lane
//     kernel does): NULL / equal / length-gap / empty-remainder cells finish there, cells with a row past 64
//     units or a unit >= 256 go to the slow list, and the rest -- stripped planes, lengths, cut -- go into the
//     wave's LDS queue.  The batch runs when the queue is empty; its rows' records and planes were loaded by the
//     previous batch (three-stage prefetch: list entries, row ids, records + planes), and it is the only place
//     the loop touches global memory, so no wait in the loop waits on a load issued less than a batch ago;
//   - round (every LEVQ_STEPS scan steps): finished cells' levels (table lookups, no fp64) go to an LDS result
//     buffer (written as code adds at the next batch), and idle lanes take queued cells (LDS reads) when
//     LEVQ_ADOPT or more are idle or few lanes still scan;
//   - step: 32-bit words when every scanning lane's pattern has <= 32 units, else 64-bit; the text bit of
//     step j is read from the fixed text planes (bfe).  Early exit on the end cell's diagonal (D[j + m - n][j] >
//     cut proves the distance > cut: values never decrease along a diagonal), tested every LEVQ_STEPS steps.
// Levels are lev_cell's: the same tests in the same order on the same (cut + 1 clamped) distance.
constexpr int LEVQ_WAVES = 4;       // waves per SIMD (VGPR budget 128; the NP = 8 form takes 3)
#ifndef SPK_LEVQ_ADOPT
#define SPK_LEVQ_ADOPT 16
#endif
#ifndef SPK_LEVQ_STEPS
#define SPK_LEVQ_STEPS 2
#endif
constexpr int LEVQ_ADOPT = SPK_LEVQ_ADOPT;  // idle lanes that trigger a hand-out while many lanes still scan
constexpr int LEVQ_STEPS = SPK_LEVQ_STEPS;  // scan steps between rounds
static_assert(32 % LEVQ_STEPS == 0, "k_lev_refill moves a text's upper plane words down between blocks, at j = 32");
constexpr int LEVQ_WG_PER_CU = 4;

// lev_cell's level of a cell from eq (1 equal / 0 unequal) and the clamped distance; nsum = na + nb.
__device__ inline int lev_level_of(const SimpleCol &sc, int eq, int lev, int nsum) {
    const double den = (double)nsum / 2.0;
    for (int i = 0; i < sc.n_tests; ++i) {
        const int op = sc.op[i], cmp = sc.cmp[i];
        int r;
        if (op == SPK_OP_STR_CMP) r = ((eq == 1) == (cmp == SPK_CMP_EQ)) ? KT : KF;
        else if (op == SPK_OP_LEVRATIO && den == 0.0) r = KN;
        else r = op == SPK_OP_LEV ? cmpd((double)lev, sc.t[i], cmp) : cmpd((double)lev / den, sc.t[i], cmp);
        if (r == KT) return sc.level[i];
    }
    return sc.else_level;
}

// Diagnostic build only (-DSPK_LEVQ_STATS): per-launch totals of k_lev_refill's schedule (tools/ab_lev_refill.py
// prints them): waves, batches, rounds, hand-out rounds, wave-steps by word width, lane-steps, cells scanned,
// cycles in batches / in steps / in the whole loop.
#ifdef SPK_LEVQ_STATS
__device__ unsigned long long g_levq[16];
#define LEVQ_STAT(i, v) (st_[i] += (unsigned long long)(v))
#else
#define LEVQ_STAT(i, v) ((void)0)
#endif
// WW = 64-bit words per plane row: 1 = the exact pass over rows of <= 64 units (cells the filter listed; cells
// with a longer or non-Latin-1 row go on to the slow list), 2 = the slow pass over rows of <= 128 units (cells the
// exact pass listed there; cells with a row past 128 units or a unit >= 256 go on to the rest list).
template <int WW>
struct RefillWord {
    typedef uint64_t type;
};
template <>
struct RefillWord<2> {
    typedef u128 type;
};
template <int WW>
__device__ inline int refill_popc(typename RefillWord<WW>::type x) {
    if constexpr (WW == 1) return __builtin_popcountll((unsigned long long)x);
    else return popc128(x);
}
template <int WW>
__device__ inline typename RefillWord<WW>::type refill_mask(int i) {  // bits [0, i), 1 <= i <= 64 WW
    typedef typename RefillWord<WW>::type W;
    return i >= 64 * WW ? ~(W)0 : (((W)1 << i) - 1);
}

template <int NP, int WW>
__global__ __launch_bounds__(X_THREADS, WW == 2 ? 2 : (NP == 8 ? 3 : LEVQ_WAVES)) void k_lev_refill(
    GammaArgs A, int si, int32_t *xlist, const int64_t *xinfo) {
    typedef typename RefillWord<WW>::type Word;
    constexpr int WPB = X_THREADS / 64;
    constexpr int PW = 2 * WW;                  // 32-bit words per plane row
    constexpr int QP = 2 * PW * NP;             // queue words of the pattern and text planes
    constexpr int QW = QP + (WW == 1 ? 2 : 3);  // + p, m | n | cut (| nsum when WW = 1), nsum (WW = 2)
    constexpr int S_MAX = 128 * WW + 1;         // len_l + len_r of rows this pass scans, plus one
    constexpr int CUT_MAX = 128 * WW - 1;       // distances here are <= 64 WW: a larger cut is no cut
    __shared__ SimpleCol s_sc;
    __shared__ ColDesc s_c0, s_c1;
    __shared__ uint32_t s_q[WPB][QW][64];
    __shared__ int32_t s_slow[WPB][128];
    __shared__ uint32_t s_res[WPB][2][128];      // finished cells: p, code delta
    __shared__ int16_t s_bp[S_MAX][MAX_TESTS];  // largest clamped distance passing test i (eq = 0), -1 none
    __shared__ uint8_t s_cut[S_MAX];
    __shared__ int s_tab;
    if (threadIdx.x == 0) {
        s_sc = A.simple[si];
        s_c0 = A.cols0[s_sc.col];
        s_c1 = A.cols1[s_sc.col];
    }
    __syncthreads();
    const SimpleCol &sc = s_sc;
    lev_tables<S_MAX, CUT_MAX>(A, sc, s_cut, s_bp, &s_tab);
    __syncthreads();
    const bool tab = s_tab != 0;
    const int k = sc.k, n_tests = sc.n_tests;
    const uint32_t stride = (uint32_t)sc.stride;
    auto level_of = [&](int lev, int S) -> int {  // eq = 0
        if (!tab) return lev_level_of(sc, 0, lev, S);
        int level = sc.else_level;
        for (int i = n_tests - 1; i >= 0; --i) level = lev <= s_bp[S][i] ? sc.level[i] : level;
        return level;
    };
    // the input list and where the cells this pass cannot scan go
    const int64_t n_items = WW == 1 ? exact_count(A, xinfo, k) : (int64_t)A.slow_count[k];
    const int32_t *items = WW == 1 ? xlist + xinfo[k] : A.slow + A.slow_off[k];
    int32_t *out_list = WW == 1 ? A.slow + A.slow_off[k] : xlist + xinfo[k];
    unsigned int *out_count = A.slow_count + (WW == 1 ? k : A.K + k);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long below = (1ull << lane) - 1ull;
    // the wave's contiguous range of batches (64 list entries each)
    const int64_t n_batches = (n_items + 63) / 64;
    const int64_t n_waves = (int64_t)gridDim.x * WPB;
    const int64_t per = (n_batches + n_waves - 1) / n_waves;
    const int64_t w = (int64_t)blockIdx.x * WPB + wv;
    const int64_t b_end = (w + 1) * per < n_batches ? (w + 1) * per : n_batches;
    int64_t bn = w * per < b_end ? w * per : b_end;  // wave-uniform: next batch to set up
    if (bn >= b_end) return;  // whole waves only: no barrier follows
    // global-address-space views of the rows' records and planes (global_load, not flat: a flat load also
    // counts against lgkmcnt, so the LDS reads after it would wait for the gather)
    typedef const __attribute__((address_space(1))) uint32_t GWord;
    typedef const __attribute__((address_space(1))) uint64_t GPlane;
    // (read through the kernel-argument pointers, so they stay in scalar registers)
    const int colx = A.simple[si].col;
    GWord *meta0 = (GWord *)A.cols0[colx].meta, *meta1 = (GWord *)A.cols1[colx].meta;
    GPlane *plane0 = (GPlane *)A.cols0[colx].planes, *plane1 = (GPlane *)A.cols1[colx].planes;
    GPlane *hi0 = (GPlane *)A.cols0[colx].planes_hi, *hi1 = (GPlane *)A.cols1[colx].planes_hi;
    // list entry of this lane in batch b, clamped into the range (unconditional loads: no divergent skips)
    auto entry = [&](int64_t b) -> int32_t {
        const int64_t bb = b < b_end ? b : b_end - 1;
        int64_t i = bb * 64 + lane;
        i = i < n_items ? i : n_items - 1;
        return items[i];
    };
    // staged batch: records (key, len16, head, cpf) and planes 0 .. NP - 1 of both rows (WW = 2: both words)
    uint32_t ska = 0, skb = 0, sfa = 0, sfb = 0;
    int32_t sla = 0, slb = 0;
    uint64_t sha = 0, shb = 0;
    uint64_t sqa[WW][NP], sqb[WW][NP];
#pragma unroll
    for (int h = 0; h < WW; ++h)
#pragma unroll
        for (int b = 0; b < NP; ++b) sqa[h][b] = sqb[h][b] = 0;
    auto stage = [&](int32_t x, int32_t y) {
        GWord *ma = meta0 + (int64_t)x * 8, *mb = meta1 + (int64_t)y * 8;
        ska = ma[0];
        sla = (int32_t)ma[1];
        sha = ((uint64_t)ma[5] << 32) | ma[4];
        sfa = ma[7];
        skb = mb[0];
        slb = (int32_t)mb[1];
        shb = ((uint64_t)mb[5] << 32) | mb[4];
        sfb = mb[7];
        GPlane *qa = plane0 + (int64_t)x * N_PLANES, *qb = plane1 + (int64_t)y * N_PLANES;
#pragma unroll
        for (int b = 0; b < NP; ++b) {
            sqa[0][b] = qa[b];
            sqb[0][b] = qb[b];
        }
        if constexpr (WW == 2) {  // units 64 .. 127 (zero in rows of <= 64 units); a side without them: zero
            GPlane *ra = hi0 ? hi0 + (int64_t)x * N_PLANES : nullptr, *rb = hi1 ? hi1 + (int64_t)y * N_PLANES : nullptr;
#pragma unroll
            for (int b = 0; b < NP; ++b) {
                sqa[1][b] = ra ? ra[b] : 0ull;
                sqb[1][b] = rb ? rb[b] : 0ull;
            }
        }
    };
    // prefetch pipeline: p0 = entry(bn) with its rows staged, p1 = entry(bn + 1) with row ids x1 / y1, p2 =
    // entry(bn + 2)
    // (-1: a cell k_compact_lev decided; its loads read pair 0 harmlessly)
    auto pair_of = [](int32_t q) { return q < 0 ? 0 : q; };
    int32_t p0 = entry(bn), p1 = entry(bn + 1), p2 = entry(bn + 2);
    int32_t x1 = A.pl[pair_of(p1)], y1 = A.pr[pair_of(p1)];
    stage(A.pl[pair_of(p0)], A.pr[pair_of(p0)]);
    int q_head = 0, q_count = 0, n_res = 0, n_slow = 0;  // wave-uniform
#ifdef SPK_LEVQ_STATS
    unsigned long long st_[16] = {};
    const unsigned long long t_loop = clock64();
#endif
    // the lane's cell: `active` while it holds one, `run` while its scan has text units left
    bool active = false, run = false;
    int32_t p = 0;
    uint32_t P[PW * NP], T[PW * NP];  // plane b: words [PW b, PW b + PW) of the pattern / text planes
#pragma unroll
    for (int b = 0; b < PW * NP; ++b) P[b] = T[b] = 0;
    Word VP = 0, VN = 0;
    int m = 1, n = 0, j = 0, cut = 0, S = 0;
    auto flush_res = [&]() {  // the buffered code adds (fire-and-forget atomics)
        for (int i = lane; i < n_res; i += 64) code_add_atomic(A, (int32_t)s_res[wv][0][i], s_res[wv][1][i]);
        n_res = 0;
    };
    auto flush_slow = [&](int cnt) {  // the first cnt (<= 64) buffered cells to the output list
        unsigned int base = 0;
        if (lane == 0) base = atomicAdd(out_count, (unsigned int)cnt);
        base = __shfl(base, 0);
        if (lane < cnt) out_list[base + lane] = s_slow[wv][lane];
        const int rest = n_slow - cnt;
        const int32_t moved = lane < rest ? s_slow[wv][cnt + lane] : 0;
        __builtin_amdgcn_wave_barrier();
        if (lane < rest) s_slow[wv][lane] = moved;
        __builtin_amdgcn_wave_barrier();
        n_slow = rest;
    };
    for (;;) {
        // ---- round: cells whose scan reached the end of the text, or whose end-cell diagonal passed the cut
        // (D[j + m - n][j] > cut proves the distance > cut: values never decrease along a diagonal), get their
        // level into the result buffer
        {
            bool fin = false;
            int lev = 0;
            if (active) {
                const int i_end = run ? j + (m - n) : m;  // the end cell's diagonal, or row m at j = n
                const Word M = refill_mask<WW>(i_end);
                const int d = j + refill_popc<WW>(VP & M) - refill_popc<WW>(VN & M);
                fin = !run || d > cut;
                lev = d > cut ? cut + 1 : d;
            }
            const unsigned long long fm = __ballot(fin);
            if (fm) {
                if (fin) {
                    const int r = n_res + __popcll(fm & below);
                    s_res[wv][0][r] = (uint32_t)p;
                    s_res[wv][1][r] = (uint32_t)(level_of(lev, S) + 1) * stride;
                    active = run = false;
                }
                __builtin_amdgcn_wave_barrier();
                n_res += __popcll(fm);
                if (n_res > 64) flush_res();  // (a batch flushes it; this only when batches ran out)
            }
        }
        // a text past 32 units: its next plane words move down whenever the scan reaches a multiple of 32 units
        // (blocks of LEVQ_STEPS steps start at multiples of LEVQ_STEPS, a divisor of 32)
        if (__any(run && j > 0 && (j & 31) == 0)) {
            if (run && j > 0 && (j & 31) == 0) {
#pragma unroll
                for (int b = 0; b < NP; ++b)
#pragma unroll
                    for (int h = 0; h + 1 < PW; ++h) T[PW * b + h] = T[PW * b + h + 1];
            }
        }
        const int n_act = __popcll(__ballot(active));
        // ---- batch: set up the next 64 cells when the queue is empty
        LEVQ_STAT(2, 1);
        if (q_count == 0 && bn < b_end && (64 - n_act >= LEVQ_ADOPT || n_act == 0)) {
#ifdef SPK_LEVQ_STATS
            const unsigned long long t_b = clock64();
            LEVQ_STAT(1, 1);
#endif
            // Order: (0) a full output buffer's device atomic (its return waits for everything in flight -- here
            // only the previous batch's loads and code adds), (1) the setup from the staged registers, (2) the
            // next prefetch loads, (3) LDS writes and fire-and-forget code adds: nothing after (2) waits on a load
            if (n_slow >= 64) flush_slow(64);
            const int32_t pc = p0;
            const int64_t left = n_items - bn * 64;
            const bool valid = lane < left && pc >= 0;
            bool to_slow = false, done = false, scan = false, a_pat = false;
            int level = 0, pre = 0, mm = 0, nn = 0, c = 0, s2 = 0;
            if (valid) {
                const RecMeta ma = {ska, sla, 0, sha, 0, sfa}, mb = {skb, slb, 0, shb, 0, sfb};
                const int la = sla, lb = slb;
                const int na = meta_cplen(ma), nb = meta_cplen(mb);
                s2 = na + nb;
                // WW = 1: 64-bit planes on both sides; WW = 2: 64- or 128-bit planes (a row of 65 .. 128
                // units has its units 64 .. 127 in planes_hi)
                constexpr uint32_t ANY = WW == 1 ? CPF_PLANES : (CPF_PLANES | CPF_PLANES2);
                const bool planes = (sfa & ANY) && (sfb & ANY) && (WW == 1 || ((!(sfa & CPF_PLANES2) || hi0) &&
                                                                                (!(sfb & CPF_PLANES2) || hi1)));
                if (la < 0 || lb < 0) {
                    level = sc.null_level;
                    done = true;
                } else {
                    int eq = meta_equal(ma, mb);
                    if (eq < 0 && planes) {  // hash match without dictionary ids: the planes are the units
                        bool same = la == lb;
#pragma unroll
                        for (int h = 0; h < WW; ++h)
#pragma unroll
                            for (int b = 0; b < NP; ++b) same = same && sqa[h][b] == sqb[h][b];
                        eq = same ? 1 : 0;
                    }
                    if (eq == 1) {
                        level = lev_level_of(sc, 1, 0, s2);
                        done = true;
                    } else if (!planes) {
                        to_slow = true;  // WW = 1: the slow list; WW = 2: the rest list (the interpreter)
                    } else {
                        c = s_cut[s2];
                        int lev = -1;
                        if (la == 0 || lb == 0) {
                            lev = la + lb;
                        } else {
                            const int mn = la < lb ? la : lb;
                            Word d = 0, e = 0;
#pragma unroll
                            for (int b = 0; b < NP; ++b) {
                                Word wa = sqa[0][b], wb = sqb[0][b];
                                if constexpr (WW == 2) {
                                    wa |= (Word)sqa[1][b] << 64;
                                    wb |= (Word)sqb[1][b] << 64;
                                }
                                d |= wa ^ wb;
                                e |= (wa << (64 * WW - la)) ^ (wb << (64 * WW - lb));
                            }
                            if constexpr (WW == 1) {
                                pre = d ? __ffsll((unsigned long long)d) - 1 : 64;
                            } else {
                                pre = ctz128(d);
                            }
                            if (pre > mn) pre = mn;
                            int suf;
                            if constexpr (WW == 1) suf = e ? __clzll((long long)e) : 64;
                            else suf = clz128(e);
                            if (suf > mn - pre) suf = mn - pre;
                            const int ra = la - pre - suf, rb = lb - pre - suf;
                            if (ra == 0 || rb == 0) {
                                lev = ra + rb;
                            } else {
                                a_pat = ra >= rb;
                                mm = a_pat ? ra : rb;
                                nn = a_pat ? rb : ra;
                                if (mm - nn > c) lev = c + 1;  // the length gap alone exceeds the cut
                                else scan = true;
                            }
                        }
                        if (!scan) {
                            level = level_of(lev > c ? c + 1 : lev, s2);
                            done = true;
                        }
                    }
                }
            }
            // scan cells into the (empty) queue: the stripped planes, the longer remainder as the pattern
            const unsigned long long sm = __ballot(scan);
            if (scan) {
                const int r = __popcll(sm & below);
#pragma unroll
                for (int b = 0; b < NP; ++b) {
                    Word wa = sqa[0][b], wb = sqb[0][b];
                    if constexpr (WW == 2) {
                        wa |= (Word)sqa[1][b] << 64;
                        wb |= (Word)sqb[1][b] << 64;
                    }
                    const Word pp = (a_pat ? wa : wb) >> pre;
                    const Word tt = (a_pat ? wb : wa) >> pre;
#pragma unroll
                    for (int h = 0; h < PW; ++h) {
                        s_q[wv][PW * b + h][r] = (uint32_t)(pp >> (32 * h));
                        s_q[wv][PW * NP + PW * b + h][r] = (uint32_t)(tt >> (32 * h));
                    }
                }
                s_q[wv][QP][r] = (uint32_t)pc;
                if constexpr (WW == 1) {
                    s_q[wv][QP + 1][r] = (uint32_t)mm | ((uint32_t)nn << 8) | ((uint32_t)c << 16) | ((uint32_t)s2 << 24);
                } else {
                    s_q[wv][QP + 1][r] = (uint32_t)mm | ((uint32_t)nn << 8) | ((uint32_t)c << 16);
                    s_q[wv][QP + 2][r] = (uint32_t)s2;
                }
            }
            q_head = 0;
            q_count = __popcll(sm);
            LEVQ_STAT(8, q_count);
            // cells this pass cannot scan into the output buffer
            const unsigned long long wm = __ballot(to_slow);
            if (wm) {
                if (to_slow) s_slow[wv][n_slow + __popcll(wm & below)] = pc;
                n_slow += __popcll(wm);
            }
            __builtin_amdgcn_wave_barrier();
            // the prefetch pipeline moves one batch on: rows of bn + 1, row ids of bn + 2, entries of bn + 3
            ++bn;
            stage(x1, y1);
            x1 = A.pl[pair_of(p2)];
            y1 = A.pr[pair_of(p2)];
            p0 = p1;
            p1 = p2;
            p2 = entry(bn + 2);
            // settled cells' and buffered code adds (fire-and-forget)
            if (done) code_add_atomic(A, pc, (uint32_t)(level + 1) * stride);
            if (n_res) flush_res();
            __builtin_amdgcn_wave_barrier();
#ifdef SPK_LEVQ_STATS
            LEVQ_STAT(9, clock64() - t_b);
#endif
        }
        // ---- round: idle lanes take queued cells
        if (q_count > 0) {
            const unsigned long long im = __ballot(!active);
            const int n_idle = __popcll(im);
            if (n_idle >= LEVQ_ADOPT || 64 - n_idle < LEVQ_ADOPT) {
                LEVQ_STAT(3, 1);
                const int r = __popcll(im & below);
                if (!active && r < q_count) {
                    const int e = q_head + r;
#pragma unroll
                    for (int b = 0; b < PW * NP; ++b) {
                        P[b] = s_q[wv][b][e];
                        T[b] = s_q[wv][PW * NP + b][e];
                    }
                    p = (int32_t)s_q[wv][QP][e];
                    const uint32_t pk = s_q[wv][QP + 1][e];
                    m = (int)(pk & 0xFF);
                    n = (int)((pk >> 8) & 0xFF);
                    cut = (int)((pk >> 16) & 0xFF);
                    S = WW == 1 ? (int)(pk >> 24) : (int)s_q[wv][QP + 2][e];
                    VP = ~(Word)0;
                    VN = 0;
                    j = 0;
                    active = run = true;
                }
                const int taken = n_idle < q_count ? n_idle : q_count;
                q_head += taken;
                q_count -= taken;
            }
        }
        if (!__any(active)) {
            if (bn >= b_end && q_count == 0) break;
            continue;
        }
        // ---- LEVQ_STEPS scan steps of the lanes whose text has units left (a lane stops at j = n: its exec
        // bit drops, no branch).  The word width is a wave-uniform choice per block of steps: the full width only
        // when some scanning lane needs it in the block.  A pattern of more than H = 32 WW units needs it from
        // text unit J0 = (H - 1) - cut on (Ukkonen, as myers_plane_text_lazy): D[i][j] >= i - j, so rows > H
        // cannot hold a value <= cut before it, and until then a half-width step leaves rows H + 1 .. m at
        // D[H][j] + (i - H) (VP bits set, VN bits clear above row H) -- upper bounds that differ from the true
        // values only where both are > cut, so the cut tests and the clamped distance read the same.  The text's
        // plane words are read at bit j & 31 of T[PW b]; a lane's next words move down at multiples of 32 (in
        // the round, above).
        constexpr int H = 32 * WW;
        bool need_full = false;
        if (run && m > H) need_full = j + LEVQ_STEPS > (cut < H - 1 ? H - 1 - cut : 0);
        const bool wide = __any(need_full);
#ifdef SPK_LEVQ_STATS
        const unsigned long long t_s = clock64();
        LEVQ_STAT(wide ? 5 : 4, LEVQ_STEPS);
        LEVQ_STAT(7, __popcll(__ballot(run)));
#endif
        if (!wide) {
            typedef typename std::conditional<WW == 1, uint32_t, uint64_t>::type Half;
            for (int s = 0; s < LEVQ_STEPS; ++s) {
                if (run) {
                    const uint32_t jj = (uint32_t)j & 31u;
                    Half eq = ~(Half)0;
#pragma unroll
                    for (int b = 0; b < NP; ++b) {
                        const uint32_t mb = (uint32_t)__builtin_amdgcn_sbfe((int)T[PW * b], jj, 1);
                        if constexpr (WW == 1) {
                            eq = eq_plane(eq, mb, P[PW * b]);
                        } else {
                            eq = eq_plane(eq, mb, ((uint64_t)P[PW * b + 1] << 32) | P[PW * b]);
                        }
                    }
                    Half vp = (Half)VP, vn = (Half)VN;
                    const Half x = eq | vn;
                    const Half d0 = (((x & vp) + vp) ^ vp) | x;
                    const Half hp = (vn | ~(d0 | vp)) << 1 | (Half)1;
                    const Half hn = (d0 & vp) << 1;
                    vp = hn | ~(d0 | hp);
                    vn = hp & d0;
                    VP = (~(Word)0 << H) | (Word)vp;  // rows H + 1 .. m: D[H][j] + (i - H)
                    VN = (Word)vn;
                    ++j;
                    run = j < n;
                }
            }
        } else {
            for (int s = 0; s < LEVQ_STEPS; ++s) {
                if (run) {
                    const uint32_t jj = (uint32_t)j & 31u;
                    uint32_t e[PW];
#pragma unroll
                    for (int h = 0; h < PW; ++h) e[h] = ~0u;
#pragma unroll
                    for (int b = 0; b < NP; ++b) {
                        const uint32_t mb = (uint32_t)__builtin_amdgcn_sbfe((int)T[PW * b], jj, 1);
#pragma unroll
                        for (int h = 0; h < PW; ++h) e[h] = eq_plane(e[h], mb, P[PW * b + h]);
                    }
                    Word eq = 0;
#pragma unroll
                    for (int h = 0; h < PW; ++h) eq |= (Word)e[h] << (32 * h);
                    const Word x = eq | VN;
                    const Word d0 = (((x & VP) + VP) ^ VP) | x;
                    const Word hp = (VN | ~(d0 | VP)) << 1 | (Word)1;
                    const Word hn = (d0 & VP) << 1;
                    VP = hn | ~(d0 | hp);
                    VN = hp & d0;
                    ++j;
                    run = j < n;
                }
            }
        }
#ifdef SPK_LEVQ_STATS
        LEVQ_STAT(10, clock64() - t_s);
#endif
    }
#ifdef SPK_LEVQ_STATS
    LEVQ_STAT(11, clock64() - t_loop);
    LEVQ_STAT(0, 1);
    if (lane == 0)
        for (int i = 0; i < 12; ++i) atomicAdd(&g_levq[i], st_[i]);
#endif
    if (n_res) flush_res();
    if (n_slow >= 64) flush_slow(64);
    if (n_slow) flush_slow(n_slow);
}

// Global-memory pass over column k's slow list (length on the device; usually empty).  Cells with a
// string past SLOW_LIMIT units go on to the huge pass: their list (counter slow_count[2K + k]) takes
// column k's exact-list region, free once the exact pass ran and at least as long as the slow list.
__global__ __launch_bounds__(64) void k_gamma_slow(GammaArgs A, ColSet cs, int32_t *xlist, const int64_t *xinfo) {
    const int k = cs.k[blockIdx.y];
    const int64_t n = A.slow_count[k];
    const int32_t *items = A.slow + A.slow_off[k];
    int32_t *huge = xlist + xinfo[k];
    for (int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 64) {
        const int32_t p = items[i];
        int level = 0;
        const bool done = eval_column<M_SLOW>(A, k, A.pl[p], A.pr[p], nullptr, nullptr, level) == ST_DONE;
        // several columns in one launch (the fused JW lists) can hold the same pair: their adds to its code race
        if (done && cs.n > 1) code_add_atomic(A, p, (uint32_t)(level + 1) * (uint32_t)A.stride[k]);
        else if (done) code_add(A, p, (uint32_t)(level + 1) * (uint32_t)A.stride[k]);
        wave_append(huge, A.slow_count + 2 * A.K + k, !done, p);
    }
}

// Huge pass: cells with a string longer than SLOW_LIMIT units, one lane per cell, DP rows and flag
// words in device scratch sized by the host to the longest string the column's program can meet.
__global__ __launch_bounds__(64) void k_gamma_huge(GammaArgs A, int k, const int32_t *items, int64_t n, Scratch S) {
    S.slot = (int64_t)blockIdx.x * 64 + threadIdx.x;
    for (int64_t i = S.slot; i < n; i += S.n_slots) {
        const int32_t p = items[i];
        int level = 0;
        eval_column<M_HUGE>(A, k, A.pl[p], A.pr[p], nullptr, nullptr, level, S);
        code_add(A, p, (uint32_t)(level + 1) * (uint32_t)A.stride[k]);
    }
}

// Slow list of a Levenshtein template column: cells whose rows are Latin-1 and at most
// PLANES2_MAX units (CPF_PLANES / CPF_PLANES2) are exact from 128-bit planes in registers
// (lev_rows_planes128) -- free-text columns such as cfg5's addresses land here; any other cell
// (non-Latin-1 or longer rows) runs the global-memory evaluation of k_gamma_slow.
template <bool P8>
__device__ int lev_cell128(const SimpleCol &sc, const ColDesc &c0, const ColDesc &c1, int32_t x, int32_t y,
                           int &level) {
    // One memory round trip: both rows' records, planes and upper planes are requested together (the upper
    // planes unconditionally -- from the lower planes' own row when the column has none -- and masked by the
    // records' flags afterwards), through global-address-space views.  Loading the upper planes only after the
    // records said a row has them took two round trips more per cell (item, pair rows, records, planes).
    const RecMeta ma = load_meta_global(c0.meta, x), mb = load_meta_global(c1.meta, y);
    uint64_t la[N_PLANES], lb[N_PLANES], ua[N_PLANES], ub[N_PLANES];
    {
        GU64 *qa = (GU64 *)(c0.planes + (int64_t)x * N_PLANES), *qb = (GU64 *)(c1.planes + (int64_t)y * N_PLANES);
        GU64 *ra = (GU64 *)((c0.planes_hi ? c0.planes_hi : c0.planes) + (int64_t)x * N_PLANES);
        GU64 *rb = (GU64 *)((c1.planes_hi ? c1.planes_hi : c1.planes) + (int64_t)y * N_PLANES);
#pragma unroll
        for (int i = 0; i < N_PLANES; ++i) {
            la[i] = qa[i];
            lb[i] = qb[i];
            ua[i] = ra[i];
            ub[i] = rb[i];
        }
    }
    if (ma.len16 < 0 || mb.len16 < 0) {
        level = sc.null_level;
        return ST_DONE;
    }
    constexpr uint32_t ANY = CPF_PLANES | CPF_PLANES2;
    if (!(ma.cpf & ANY) || !(mb.cpf & ANY)) return ST_NEEDS_SLOW;
    if (((ma.cpf & CPF_PLANES2) && !c0.planes_hi) || ((mb.cpf & CPF_PLANES2) && !c1.planes_hi)) return ST_NEEDS_SLOW;
    const uint64_t ka = (ma.cpf & CPF_PLANES2) ? ~0ull : 0ull, kb = (mb.cpf & CPF_PLANES2) ? ~0ull : 0ull;
    u128 pa[N_PLANES], pb[N_PLANES];
#pragma unroll
    for (int i = 0; i < N_PLANES; ++i) {
        pa[i] = ((u128)(ua[i] & ka) << 64) | la[i];
        pb[i] = ((u128)(ub[i] & kb) << 64) | lb[i];
    }
    int eq = meta_equal(ma, mb);
    if (eq < 0) {  // equal keys without dictionary ids: the planes are the units
        eq = ma.len16 == mb.len16 ? 1 : 0;
#pragma unroll
        for (int b = 0; b < N_PLANES; ++b) eq &= pa[b] == pb[b] ? 1 : 0;
    }
    const int na = meta_cplen(ma), nb = meta_cplen(mb);  // = len16: Latin-1 rows
    int lev = -1;
    for (int i = 0; i < sc.n_tests; ++i) {
        const int op = sc.op[i], cmp = sc.cmp[i];
        const double t = sc.t[i];
        int r;
        if (op == SPK_OP_STR_CMP) {
            r = ((eq == 1) == (cmp == SPK_CMP_EQ)) ? KT : KF;
        } else {
            const double den = (double)(na + nb) / 2.0;
            if (op == SPK_OP_LEVRATIO && den == 0.0) {
                r = KN;
            } else {
                if (lev < 0)
                    lev = eq == 1 ? 0 : lev_rows_planes128<P8>(pa, ma.len16, pb, mb.len16, simple_lev_cut(sc, na, nb), sc.np);
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

// Cells without planes on both rows are handed on (rest list: column k's exact-list region, free
// once the exact pass ran, and counter slow_count[K + k]) to k_gamma_rest, so this kernel does not
// carry the general interpreter's registers (the 128-bit scan alone holds ~100).
template <bool P8>  // the column's scans read all 8 planes (SimpleCol.np == 8)
__global__ __launch_bounds__(X_THREADS) void k_gamma_slow_lev(GammaArgs A, int si, int32_t *xlist,
                                                              const int64_t *xinfo) {
    __shared__ SimpleCol s_sc;
    __shared__ ColDesc s_c0, s_c1;
    if (threadIdx.x == 0) {
        s_sc = A.simple[si];
        s_c0 = A.cols0[s_sc.col];
        s_c1 = A.cols1[s_sc.col];
    }
    __syncthreads();
    const int k = s_sc.k;
    const int64_t n = A.slow_count[k];
    const int32_t *items = A.slow + A.slow_off[k];
    int32_t *rest = xlist + xinfo[k];
    // (regrouping these cells by work bin, as k_gamma_exact_simple does for free-text columns,
    // measured no faster here: 2.43-2.47 ms per cfg5 call either way)
    // Software pipeline as the exact pass: the next cell's pair rows are in flight during this cell's scan, and
    // the list entry after that one a round earlier still (unconditional loads at clamped indices).
    const int64_t stride = (int64_t)gridDim.x * X_THREADS;
    int64_t i = (int64_t)blockIdx.x * X_THREADS + threadIdx.x;
    if (n <= 0) return;
    int32_t p = items[i < n ? i : n - 1];
    int32_t x = A.pl[p], y = A.pr[p];
    int32_t pn = items[i + stride < n ? i + stride : n - 1];
    for (; i < n; i += stride) {
        const int32_t x2 = A.pl[pn], y2 = A.pr[pn];
        const int64_t i3 = i + 2 * stride;
        const int32_t pn3 = items[i3 < n ? i3 : n - 1];
        int level = 0;
        const bool done = lev_cell128<P8>(s_sc, s_c0, s_c1, x, y, level) == ST_DONE;
        if (done) code_add(A, p, (uint32_t)(level + 1) * (uint32_t)A.stride[k]);
        wave_append(rest, A.slow_count + A.K + k, !done, p);
        p = pn;
        x = x2;
        y = y2;
        pn = pn3;
    }
}

// The rest list of k_gamma_slow_lev through the global-memory evaluation; cells past SLOW_LIMIT
// units go to the huge list, in column k's slow-list region (free once k_gamma_slow_lev ran).
__global__ __launch_bounds__(64) void k_gamma_rest(GammaArgs A, int k, const int32_t *xlist, const int64_t *xinfo) {
    const int64_t n = A.slow_count[A.K + k];
    const int32_t *items = xlist + xinfo[k];
    int32_t *huge = A.slow + A.slow_off[k];
    for (int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 64) {
        const int32_t p = items[i];
        int level = 0;
        const bool done = eval_column<M_SLOW>(A, k, A.pl[p], A.pr[p], nullptr, nullptr, level) == ST_DONE;
        if (done) code_add(A, p, (uint32_t)(level + 1) * (uint32_t)A.stride[k]);
        wave_append(huge, A.slow_count + 2 * A.K + k, !done, p);
    }
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

static bool host_cmp(double a, double b, int cmp) {
    switch (cmp) {
        case SPK_CMP_EQ: return a == b;
        case SPK_CMP_NE: return a != b;
        case SPK_CMP_LT: return a < b;
        case SPK_CMP_LE: return a <= b;
        case SPK_CMP_GT: return a > b;
        default: return a >= b;
    }
}

static int32_t clamp_i32(double v) { return (int32_t)std::max(-1073741824.0, std::min(1073741824.0, v)); }

// The filter's per-test decision parameters (SimpleCol.tflag / lev_a / jw_cf), so the device decides
// each test with compares and selects only.
static void prepare_tests(SimpleCol &s) {
    for (int i = 0; i < s.n_tests; ++i) {
        const int op = s.op[i], cmp = s.cmp[i];
        const double t = s.t[i];
        int32_t f = 0;
        if (op == SPK_OP_STR_CMP) f |= cmp == SPK_CMP_EQ ? TF_EQ : 0;
        if (op == SPK_OP_JW || op == SPK_OP_LEVRATIO) {
            f |= host_cmp(0.0, t, cmp) ? TF_ZERO : 0;
            f |= host_cmp(1.0, t, cmp) ? TF_ONE : 0;
        }
        s.lev_a[i] = 0;
        s.jw_cf[i] = 0.f;
        if (op == SPK_OP_LEV) {  // integer v: v cmp t as v >= A or v <= A
            switch (cmp) {
                case SPK_CMP_GT: f |= TF_GE; s.lev_a[i] = clamp_i32(std::floor(t) + 1.0); break;
                case SPK_CMP_GE: f |= TF_GE; s.lev_a[i] = clamp_i32(std::ceil(t)); break;
                case SPK_CMP_LT: s.lev_a[i] = clamp_i32(std::ceil(t) - 1.0); break;
                case SPK_CMP_LE: s.lev_a[i] = clamp_i32(std::floor(t)); break;
                default: f |= TF_EXACT; break;
            }
        }
        if (op == SPK_OP_JW) {
            // an fp32 upper bound hi (of a double value) proves `v > t` false iff hi <= t, i.e. hi <=
            // the largest float <= t; `v >= t` false iff hi < t, i.e. hi < the smallest float >= t
            float fl = (float)t;
            if ((double)fl > t) fl = std::nextafter(fl, -INFINITY);
            float fu = (float)t;
            if ((double)fu < t) fu = std::nextafter(fu, INFINITY);
            s.jw_cf[i] = cmp == SPK_CMP_GT ? std::nextafter(fl, INFINITY) : fu;
        }
        s.tflag[i] = f;
    }
}

// Level of a simple string column for two equal, non-NULL, non-empty strings: `=` holds, jw = 1.0,
// levenshtein = 0 and its ratio 0.0 (den > 0); the first test that holds decides.
static int32_t equal_level(const SimpleCol &s) {
    for (int i = 0; i < s.n_tests; ++i) {
        const int op = s.op[i], cmp = s.cmp[i];
        bool r;
        if (op == SPK_OP_STR_CMP) r = cmp == SPK_CMP_EQ;
        else if (op == SPK_OP_JW) r = host_cmp(1.0, s.t[i], cmp);
        else r = host_cmp(0.0, s.t[i], cmp);  // SPK_OP_LEV / SPK_OP_LEVRATIO
        if (r) return s.level[i];
    }
    return s.else_level;
}

// The pairs of one blocking rule are contiguous in the pair order; a rule whose key includes the
// plain term `l.c = r.c` on the raw columns column c was decoded from puts equal, non-NULL strings
// of c in every pair it emits (keys are byte-verified dense ids; NULL keys emit nothing).  The
// longest run of such pairs becomes the column's implied range (SimpleCol.imp_lo / imp_hi).
static void implied_equal(const spk_ctx *ctx, const Table &t0, const Table &t1, SimpleCol &sc) {
    sc.imp_lo = sc.imp_hi = 0;
    sc.eq_level = 0;
    if (sc.kind != SK_STR || !(sc.cls == SC_EQ || sc.cls == SC_JW || sc.cls == SC_LEV)) return;
    const Column *c0 = t0.cols[sc.col], *c1 = t1.cols[sc.col];
    if (!c0 || !c1 || !c0->src[0] || !c1->src[1] || c0->has_empty || c1->has_empty) return;
    int64_t lo = -1, hi = -1;
    for (size_t r = 0; r < ctx->pair_terms.size(); ++r) {
        bool imp = false;
        for (const KeyTerm &k : ctx->pair_terms[r]) imp = imp || (k.plain && k.src_l == c0->src[0] && k.src_r == c1->src[1]);
        if (!imp) continue;
        if (lo >= 0 && ctx->pair_rule_lo[r] == hi) hi = ctx->pair_rule_hi[r];  // adjacent rules merge
        else lo = ctx->pair_rule_lo[r], hi = ctx->pair_rule_hi[r];
        if (hi - lo > sc.imp_hi - sc.imp_lo) sc.imp_lo = lo, sc.imp_hi = hi;
    }
    sc.eq_level = equal_level(sc);
}

// Filter class of a simple column (see SimpleCol); SC_NONE leaves it to the interpreter.
static int32_t simple_class(const SimpleCol &s) {
    if (s.kind == SK_NUM) return SC_NUM;
    bool all_eq = true, all_jw = s.n_tests > 0, lev_ok = true;
    int n_lev = 0;
    for (int i = 0; i < s.n_tests; ++i) {
        const int op = s.op[i], cmp = s.cmp[i];
        all_eq = all_eq && op == SPK_OP_STR_CMP;
        all_jw = all_jw && op == SPK_OP_JW && (cmp == SPK_CMP_GT || cmp == SPK_CMP_GE);
        if (op == SPK_OP_LEV) {
            ++n_lev;
        } else if (op == SPK_OP_LEVRATIO) {
            ++n_lev;
            lev_ok = lev_ok && (cmp == SPK_CMP_LE || cmp == SPK_CMP_LT);
        } else if (op != SPK_OP_STR_CMP) {
            lev_ok = false;
        }
    }
    if (all_eq) return SC_EQ;
    if (all_jw) return SC_JW;
    if (lev_ok && n_lev > 0) return SC_LEV;
    return SC_NONE;
}

// Row-image offsets; returns the row stride (a multiple of 16), 0 when nothing uses the image.
// JW fields take 24 B at a 16-byte boundary (key, lens, sketch; head units at off + 16, the low half
// of the next chunk), LEV / NUM 16 B at a boundary, EQ in the 8-byte gaps JW leaves (an EQ column with
// dictionary ids takes 4 B there -- its id, two to a gap, so one head-chunk load serves a JW column and
// two equality columns -- one without ids the whole gap), then 8 B each at the end.
// Columns that do not fit in IMG_MAX bytes, or past the filter kernel's slots of their class
// (FJ_MAX ...), go to the interpreter (SC_NONE).
static int64_t layout_image(std::vector<SimpleCol> &simple) {
    int64_t off = 0;
    std::vector<int64_t> gaps;  // free 8-byte slots
    int nj = 0, nl = 0, nn = 0, ne = 0;
    for (SimpleCol &s : simple) {
        if (s.cls != SC_JW) continue;
        if (off + 32 > IMG_MAX || nj == FJ_MAX) {
            s.cls = SC_NONE;
            continue;
        }
        ++nj;
        s.off = (int32_t)off;
        s.off2 = (int32_t)(off + 16);
        gaps.push_back(off + 24);
        off += 32;
    }
    for (SimpleCol &s : simple) {
        if (s.cls != SC_LEV && s.cls != SC_NUM) continue;
        int &n = s.cls == SC_LEV ? nl : nn;
        if (off + 16 > IMG_MAX || n == (s.cls == SC_LEV ? FL_MAX : FN_MAX)) {
            s.cls = SC_NONE;
            continue;
        }
        ++n;
        s.off = (int32_t)off;
        off += 16;
    }
    std::vector<int> used(gaps.size(), 0);  // 4-byte halves taken in each gap
    for (SimpleCol &s : simple) s.eq4 = 0;
    for (int pass = 0; pass < 2; ++pass) {  // ids first (half gaps), then the others (whole gaps)
        for (SimpleCol &s : simple) {
            if (s.cls != SC_EQ || (pass == 0) != (s.has_ids != 0)) continue;
            if (ne == FE_MAX) {
                s.cls = SC_NONE;
                continue;
            }
            size_t g = 0;
            const int need = pass == 0 ? 1 : 2;
            while (g < gaps.size() && used[g] + need > 2) ++g;
            if (g < gaps.size()) {
                s.off = (int32_t)(gaps[g] + 4 * used[g]);
                s.eq4 = pass == 0 ? 1 : 0;
                used[g] += need;
                ++ne;
                continue;
            }
            if (off + 8 > IMG_MAX) {
                s.cls = SC_NONE;
                continue;
            }
            ++ne;
            s.off = (int32_t)off;
            off += 8;
        }
    }
    int64_t end = off;
    if (!gaps.empty() && used.back() == 0 && gaps.back() + 8 == off) end = off - 8;  // trailing unused JW gap
    return (end + 15) & ~(int64_t)15;
}

// Row image in a rule's view order: chunk c of view position v = chunk c of table row rows[v]; the
// same chunk stride (row capacity) as the table's image.
__global__ void k_view_image(int64_t nv, const int32_t *__restrict__ rows, int nq, const uint4 *__restrict__ src,
                             uint4 *__restrict__ dst, int64_t cap) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv * nq) return;
    const int64_t v = i % nv, c = i / nv;
    dst[c * cap + v] = src[c * cap + rows[v]];
}

// View-ordered copies of the row images for rule 1's pairs (RuleView), rebuilt when the image or the
// pair set changes.  Returns false when there is no view to use.
struct ViewLaunch {
    const uint8_t *img0, *img1;
    const int32_t *rows0, *rows1;  // view position -> table row
    int64_t lo, hi;                // rule 1's pair ordinals
};

static int build_view_images(spk_ctx *ctx, const GammaArgs &A, int64_t stride, ViewLaunch *out, bool *ok) {
    *ok = false;
    if (stride <= 0 || A.n_simple == 0 || ctx->n_views < 1 || !A.img0) return SPK_OK;
    const int nq = (int)(stride / 16);
    const int r = 1;
    RuleView &v = ctx->views[r];
    for (int s = 0; s < 2; ++s) {
        const int64_t nv = (s == 0 || v.tri) ? v.nL : v.nR;
        const int32_t *rows = (s == 0 || v.tri) ? v.rowsL.p : v.rowsR.p;
        if (s == 1 && v.tri) {  // symmetric self-join: both sides index the same view
            out->img1 = out->img0;
            out->rows1 = out->rows0;
            continue;
        }
        const int64_t cap = s == 0 ? A.img_rows0 : A.img_rows1;
        const uint8_t *src = s == 0 ? A.img0 : A.img1;
        std::vector<int64_t> key = ctx->img_key[(s == 1 && A.img1 != A.img0) ? 1 : 0];
        key.push_back((int64_t)ctx->pairs_epoch);
        key.push_back(s);
        const bool fresh = ctx->vimg[r][s].p && ctx->vimg_key[r][s] == key;
        SPK_TRY(ctx->vimg[r][s].alloc((size_t)cap * (size_t)stride));
        if (!fresh && nv > 0) {
            k_view_image<<<(unsigned)((nv * nq + 255) / 256), 256, 0, ctx->stream>>>(
                nv, rows, nq, reinterpret_cast<const uint4 *>(src), reinterpret_cast<uint4 *>(ctx->vimg[r][s].p), cap);
            SPK_HIP(hipGetLastError());
        }
        ctx->vimg_key[r][s] = key;
        (s == 0 ? out->img0 : out->img1) = ctx->vimg[r][s].p;
        (s == 0 ? out->rows0 : out->rows1) = rows;
    }
    out->lo = v.pair_lo;
    out->hi = v.pair_hi;
    *ok = true;
    return SPK_OK;
}

// The image is a re-layout of the resident records for the current set of simple columns: it is
// rebuilt only when a table (or one of its columns) was replaced or the column layout changed.
static int build_images(spk_ctx *ctx, Table &t0, Table &t1, GammaArgs &A, int64_t stride,
                        const std::vector<SimpleCol> &simple) {
    A.img0 = A.img1 = nullptr;
    A.img_stride = stride;
    if (stride <= 0 || A.n_simple == 0) return SPK_OK;
    Table *ts[2] = {&t0, &t1};
    for (int s = 0; s < 2; ++s) {
        if (s == 1 && &t1 == &t0) {
            A.img1 = A.img0;
            A.img_rows1 = A.img_rows0;
            break;
        }
        Table &t = *ts[s];
        std::vector<int64_t> key = {(int64_t)t.version, t.n, stride};
        for (const SimpleCol &sc : simple) {
            key.push_back(sc.cls);
            key.push_back(sc.col);
            key.push_back(sc.off);
            key.push_back(sc.off2);
            key.push_back(sc.eq4);
        }
        const bool fresh = ctx->img[s].p && ctx->img_key[s] == key;
        SPK_TRY(ctx->img[s].alloc((size_t)(t.n + 1) * (size_t)stride));
        ctx->img_key[s] = key;
        if (t.n > 0 && !fresh) {
            k_build_image<<<(unsigned)((t.n + 255) / 256), 256, 0, ctx->stream>>>(t.n, t.d_desc.p, A.simple, A.n_simple,
                                                                                 ctx->img[s].p, t.n + 1);
            SPK_HIP(hipGetLastError());
        }
        (s == 0 ? A.img0 : A.img1) = ctx->img[s].p;
        (s == 0 ? A.img_rows0 : A.img_rows1) = t.n + 1;
    }
    return SPK_OK;
}

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

// Device scratch of a huge pass over `cells` cells whose strings have at most `units` UTF-16 units: a
// slot per lane (JW: two flag-word arrays; Levenshtein: code points + one DP row), lanes = one per
// cell, at most ~1 GiB of slots, at least one wave.
static int huge_scratch(int64_t units, int64_t cells, DevBuf<uint8_t> &buf, Scratch &S) {
    SPK_REQUIRE(units < INT32_MAX / 2, SPK_E_LIMIT, "a compared string is longer than 2^30 UTF-16 units");
    S.units = (int32_t)units;
    S.words = (int32_t)((units + 63) / 64);
    const int64_t slot_bytes = std::max<int64_t>(16 * (int64_t)S.words, 4 * (2 * units + 1));
    const int64_t budget = std::max<int64_t>(64, ((int64_t)1 << 30) / slot_bytes / 64 * 64);
    S.n_slots = std::min<int64_t>(budget, (cells + 63) / 64 * 64);
    SPK_TRY(buf.alloc((size_t)(S.n_slots * slot_bytes)));
    S.base = buf.p;
    return SPK_OK;
}

// What the exact / slow / huge passes of the last spk_gammas need, kept so that an overflow of the work
// lists or cells past SLOW_LIMIT can be settled after the call returned (settle_gammas).
namespace spk {
struct GammaPlan {
    GammaArgs A{};
    std::vector<SimpleCol> simple;
    std::vector<int> simple_of;
    std::vector<char> may_exact, huge_in_slow, free_text, bag;
    std::vector<char> slow_skipped;  // columns whose slow-list kernels this call did not launch
    int K = 0, n_regions = 0, n_info = 0, n_cnt = 0, n_all = 0;
    int64_t g_exact = 1, max_units = 1;
};
}  // namespace spk

template <class T>
static void swap_buf(spk::DevBuf<T> &a, spk::DevBuf<T> &b) {
    std::swap(a.p, b.p);
    std::swap(a.n, b.n);
}

void spk_ctx::swap_slot() {
    swap_buf(work, alt.work);
    swap_buf(xlist, alt.xlist);
    swap_buf(xpref, alt.xpref);
    swap_buf(xinfo, alt.xinfo);
    swap_buf(region_count, alt.region_count);
    std::swap(xcap, alt.xcap);
    std::swap(h_info, alt.h_info);
    std::swap(h_info_n, alt.h_info_n);
    std::swap(ev_info, alt.ev_info);
    std::swap(gplan, alt.gplan);
    std::swap(gamma_pending, alt.gamma_pending);
    std::swap(stream, alt.stream);
    std::swap(xev0, alt.xev0);
    std::swap(xev1, alt.xev1);
    std::swap(xev_used, alt.xev_used);
}

// The exact and slow passes over the lists the filter wrote (list capacity `cap`).  k_prefix sizes the
// lists on the device; if they exceed `cap` every exact kernel is a no-op and settle_gammas re-runs
// this phase with the right capacity.
// The slow-list kernels of column k (or of the fused JW columns jk): the cells the exact pass left.
static int enqueue_slow(spk_ctx *ctx, GammaPlan &G, int k, const ColSet *jk) {
    GammaArgs &A = G.A;
    if (jk) {
        k_gamma_slow<<<dim3((unsigned)(4 * ctx->n_cu), (unsigned)jk->n), 64, 0, ctx->stream>>>(A, *jk, ctx->xlist.p,
                                                                                              ctx->xinfo.p);
    } else {
        const int si = G.simple_of[k];
        const bool lev = si >= 0 && G.simple[si].cls == SC_LEV;
        const ColSet one_k{1, {k, 0, 0, 0}};
        if (lev) {
            // (a lane-refill form of this pass over 128-bit planes lost 0.5 ms per cfg5 γ pass and was removed in
            // round 6)
            constexpr int SLOWLEV_WG_PER_CU = 8;  // the 128-bit scan holds 3 waves per SIMD: 3 workgroups per CU at once
            const int64_t g_sl = std::max<int64_t>(1, std::min<int64_t>(G.g_exact, (int64_t)SLOWLEV_WG_PER_CU * ctx->n_cu));
            if (G.simple[si].np >= N_PLANES)
                k_gamma_slow_lev<true><<<(unsigned)g_sl, X_THREADS, 0, ctx->stream>>>(A, si, ctx->xlist.p, ctx->xinfo.p);
            else
                k_gamma_slow_lev<false><<<(unsigned)g_sl, X_THREADS, 0, ctx->stream>>>(A, si, ctx->xlist.p, ctx->xinfo.p);
            k_gamma_rest<<<(unsigned)(4 * ctx->n_cu), 64, 0, ctx->stream>>>(A, k, ctx->xlist.p, ctx->xinfo.p);
        } else {
            k_gamma_slow<<<(unsigned)(4 * ctx->n_cu), 64, 0, ctx->stream>>>(A, one_k, ctx->xlist.p, ctx->xinfo.p);
        }
    }
    SPK_HIP(hipGetLastError());
    return SPK_OK;
}

// skip: leave out the slow-list kernels of columns whose slow lists were empty in the last settled call
static int enqueue_phase(spk_ctx *ctx, GammaPlan &G, int64_t cap, bool skip = false) {
    GammaArgs &A = G.A;
    const int K = G.K;
    G.slow_skipped.assign((size_t)K, 0);
    auto quiet = [&](int k) {
        return skip && (ctx->slow_force_skip ||
                        (ctx->slow_seen_valid && k < (int)ctx->slow_seen.size() && !ctx->slow_seen[k]));
    };
    SPK_TRY(ctx->xlist.alloc((size_t)(2 * cap)));
    A.slow = ctx->xlist.p + cap;
    A.slow_off = ctx->xinfo.p;
    ctx->xcap = cap;
    if (A.P <= 0) {
        SPK_HIP(hipMemsetAsync(ctx->xinfo.p, 0, (size_t)G.n_info * 8, ctx->stream));
        return SPK_OK;
    }
    k_prefix<<<(unsigned)K, PFX_THREADS, 0, ctx->stream>>>(
        ctx->region_count.p, K, G.n_regions, cap, ctx->xpref.p, ctx->xinfo.p,
        reinterpret_cast<unsigned long long *>(ctx->xinfo.p + G.n_info + G.n_cnt + 1));
    const std::vector<SimpleCol> &simple = G.simple;
    // Jaro-Winkler template columns: compact every list, then one exact launch over all of them
    // JW exact launches: a JW cell is one short latency-bound evaluation, and the kernel holds 3 waves per
    // SIMD, so a grid of 8 workgroups per CU ran in rounds of dispatch latency; JW_WG_PER_CU per column
    // keeps it near one resident round with the grid-stride loop's prefetch
    constexpr int JW_WG_PER_CU = 8;
    const int64_t g_jw = std::max<int64_t>(1, std::min<int64_t>(G.g_exact, (int64_t)JW_WG_PER_CU * ctx->n_cu));
    ExactCols jw{};
    jw.g = (int)g_jw;
    ColSet jk{};
    for (int k = 0; k < K; ++k) {
        if (!G.may_exact[k] || G.simple_of[k] < 0) continue;
        const SimpleCol &sc = simple[G.simple_of[k]];
        if (sc.cls != SC_JW || sc.kind != SK_STR || jw.n == 4) continue;
        jk.k[jk.n++] = k;
        jw.k[jw.n] = sc.k;
        jw.col[jw.n] = sc.col;
        jw.si[jw.n++] = G.simple_of[k];
    }
    // One compaction launch for the JW lists and the other plain-compacted lists (up to four columns): the
    // launch is one workgroup per region and column, and a short list's workgroups cost dispatch rounds alone
    // (cfg2: the JW lists' launch took as long as the email list's, 15 us each)
    ColSet pre = jk;
    for (int k = 0; k < K && pre.n < 4; ++k) {
        if (!G.may_exact[k]) continue;
        const int si = G.simple_of[k];
        bool in_jw = false;
        for (int c = 0; c < jw.n; ++c) in_jw = in_jw || jw.si[c] == si;
        if (in_jw || (si >= 0 && simple[si].cls == SC_LEV && G.bag[k])) continue;
        pre.k[pre.n++] = k;
    }
    auto precompacted = [&](int k) {
        for (int c = 0; c < pre.n; ++c)
            if (pre.k[c] == k) return true;
        return false;
    };
    if (pre.n)
        k_compact<<<dim3((unsigned)G.n_regions, (unsigned)pre.n), 256, 0, ctx->stream>>>(A, pre, ctx->xpref.p,
                                                                                        ctx->xlist.p, ctx->xinfo.p);
    // (running this launch on a second stream beside the Levenshtein pass measured no faster:
    // 1.198-1.205 ms per cfg2 pass either way)
    for (int c = 0; c < K; ++c)
        if (c < (int)ctx->xev_used.size()) ctx->xev_used[c] = 0;
    if (jw.n) {
        SPK_TRY(ctx->xbegin(jk.k[0]));
        k_gamma_exact_simple<X_JW><<<(unsigned)(g_jw * jw.n), X_THREADS, 0, ctx->stream>>>(A, jw, ctx->xlist.p,
                                                                                                ctx->xinfo.p);
        SPK_TRY(ctx->xend(jk.k[0]));
        bool all_quiet = true;
        for (int c = 0; c < jk.n; ++c) all_quiet = all_quiet && quiet(jk.k[c]);
        if (all_quiet) {
            for (int c = 0; c < jk.n; ++c) G.slow_skipped[jk.k[c]] = 1;
        } else {
            SPK_TRY(enqueue_slow(ctx, G, -1, &jk));
        }
    }
    for (int k = 0; k < K; ++k) {
        if (!G.may_exact[k]) continue;
        const int si = G.simple_of[k];
        const bool lev = si >= 0 && simple[si].cls == SC_LEV;
        bool fused = false;
        for (int c = 0; c < jw.n; ++c) fused = fused || jw.si[c] == si;
        if (fused) continue;
        const ColSet one_k{1, {k, 0, 0, 0}};
        const bool refill = lev && (ctx->lev_kernel == 1 || (ctx->lev_kernel == 2 && G.free_text[k]));
        if (lev && G.bag[k])
            k_compact_lev<<<(unsigned)G.n_regions, CL_THREADS, 0, ctx->stream>>>(A, k, si, ctx->xpref.p, ctx->xlist.p,
                                                                                ctx->xinfo.p);
        else if (!precompacted(k))
            k_compact<<<(unsigned)G.n_regions, 256, 0, ctx->stream>>>(A, one_k, ctx->xpref.p, ctx->xlist.p, ctx->xinfo.p);
        if (refill) {
            // one resident round (LEVQ_WAVES per SIMD, 3 for NP = 8): every wave owns a contiguous range of the list
            const int64_t wg_cu = simple[si].np >= 8 ? 3 : LEVQ_WG_PER_CU;
            const int64_t g_lev = std::max<int64_t>(1, std::min<int64_t>(G.g_exact, wg_cu * ctx->n_cu));
            SPK_TRY(ctx->xbegin(k));
            switch (simple[si].np) {
                case 5: k_lev_refill<5, 1><<<(unsigned)g_lev, X_THREADS, 0, ctx->stream>>>(A, si, ctx->xlist.p, ctx->xinfo.p); break;
                case 6: k_lev_refill<6, 1><<<(unsigned)g_lev, X_THREADS, 0, ctx->stream>>>(A, si, ctx->xlist.p, ctx->xinfo.p); break;
                case 7: k_lev_refill<7, 1><<<(unsigned)g_lev, X_THREADS, 0, ctx->stream>>>(A, si, ctx->xlist.p, ctx->xinfo.p); break;
                default: k_lev_refill<8, 1><<<(unsigned)g_lev, X_THREADS, 0, ctx->stream>>>(A, si, ctx->xlist.p, ctx->xinfo.p); break;
            }
            SPK_TRY(ctx->xend(k));
            if (quiet(k)) G.slow_skipped[k] = 1;
            else SPK_TRY(enqueue_slow(ctx, G, k, nullptr));
        } else if (lev) {
            ExactCols one{};
            one.n = 1;
            // one resident round: the grid-stride loop gives every block a fixed share of the list, so a
            // grid larger than what fits at once (LEV_WAVES per SIMD) runs a second, partly empty round
            constexpr int LEV_WG_PER_CU = 8;
            const int64_t g_lev = std::max<int64_t>(1, std::min<int64_t>(G.g_exact, (int64_t)LEV_WG_PER_CU * ctx->n_cu));
            one.g = (int)g_lev;
            one.si[0] = si;
            one.k[0] = simple[si].k;
            one.col[0] = simple[si].col;
            SPK_TRY(ctx->xbegin(k));
            k_gamma_exact_simple<X_LEV><<<(unsigned)g_lev, X_THREADS, 0, ctx->stream>>>(A, one, ctx->xlist.p,
                                                                                      ctx->xinfo.p);
            SPK_TRY(ctx->xend(k));
            if (quiet(k)) G.slow_skipped[k] = 1;
            else SPK_TRY(enqueue_slow(ctx, G, k, nullptr));
        } else if (si >= 0 && simple[si].kind == SK_STR) {
            ExactCols one{};
            one.n = 1;
            one.g = (int)G.g_exact;
            one.si[0] = si;
            one.k[0] = simple[si].k;
            one.col[0] = simple[si].col;
            k_gamma_exact_simple<X_GENERIC><<<(unsigned)G.g_exact, X_THREADS, 0, ctx->stream>>>(A, one, ctx->xlist.p,
                                                                                           ctx->xinfo.p);
            if (quiet(k)) G.slow_skipped[k] = 1;
            else SPK_TRY(enqueue_slow(ctx, G, k, nullptr));
        } else {
            k_gamma_exact<<<(unsigned)G.g_exact, X_THREADS, 0, ctx->stream>>>(A, k, ctx->xlist.p, ctx->xinfo.p);
            k_gamma_slow<<<(unsigned)(4 * ctx->n_cu), 64, 0, ctx->stream>>>(A, one_k, ctx->xlist.p, ctx->xinfo.p);
        }
    }
    SPK_HIP(hipGetLastError());
    return SPK_OK;
}

namespace spk {
// Completes the last spk_gammas once its info block is on the host: a work-list overflow re-runs the
// exact phase with room for every listed cell, and cells with a string past SLOW_LIMIT units go through
// the huge pass.  *fixed = true when codes changed after the call returned (a consumer that already
// read them must read them again).  Called at the consumers' own synchronisation points.
static int settle_info(spk_ctx *ctx, bool *fixed);

int settle_gammas(spk_ctx *ctx, bool *fixed) {
    bool f = false;
    SPK_TRY(settle_info(ctx, &f));
    if (fixed) *fixed = f;
    // an asynchronous EM iteration enqueued on these codes read them before the correction: repeat it
    if (f && ctx->em_pending && ctx->em_seq == ctx->gamma_seq) {
        SPK_REQUIRE(ctx->em_kind == 0, SPK_E_STATE, "codes corrected under a pending finalize (settle before the histogram)");
        SPK_TRY(em_requeue(ctx));
    }
    return SPK_OK;
}

static int settle_slot(spk_ctx *ctx, bool *fixed);
// Both windows of a two-stream split: the own slot, then the alternate one (its counts added to the first's
// through the window carry, its slow-list flags or-ed in).
static int settle_info(spk_ctx *ctx, bool *fixed) {
    if (fixed) *fixed = false;
    const bool two = ctx->gamma_pending && ctx->alt.gamma_pending;
    bool f0 = false, f1 = false;
    SPK_TRY(settle_slot(ctx, &f0));
    if (two) {
        ctx->exact_carry = ctx->last_exact;
        ctx->deferred_carry = ctx->last_deferred;
        ctx->split_first = ctx->last_exact;
        const std::vector<int64_t> xbase0 = ctx->last_xbase;
        const std::vector<uint8_t> seen = ctx->slow_seen;
        ctx->swap_slot();
        const int rc = settle_slot(ctx, &f1);
        ctx->swap_slot();
        ctx->alt_xbase = ctx->last_xbase;
        ctx->last_xbase = xbase0;
        ctx->exact_carry.clear();
        ctx->deferred_carry = 0;
        SPK_TRY(rc);
        for (size_t k = 0; k < seen.size() && k < ctx->slow_seen.size(); ++k) ctx->slow_seen[k] |= seen[k];
    } else if (ctx->alt.gamma_pending) {
        ctx->alt.gamma_pending = false;  // its call's codes were replaced before the own slot was settled
    }
    if (fixed) *fixed = f0 || f1;
    return SPK_OK;
}

static int settle_slot(spk_ctx *ctx, bool *fixed) {
    if (fixed) *fixed = false;
    if (!ctx->gamma_pending) return SPK_OK;
    // the info block is on the host once the readback behind it completed (later work -- an EM
    // iteration enqueued meanwhile -- keeps running)
    SPK_HIP(hipEventSynchronize(ctx->ev_info));
    ctx->gamma_pending = false;
    if (!ctx->codes_valid || !ctx->gplan) return SPK_OK;  // the codes were replaced or invalidated since
    GammaPlan &G = *ctx->gplan;
    const int K = G.K;
    if (ctx->h_info[2 * K]) {
        // the exact lists did not fit: nothing of the phase ran; grow them and run the phase again
        const int64_t cap = ctx->h_info[2 * K + 1];
        SPK_HIP(hipMemsetAsync(ctx->xinfo.p + G.n_info, 0, (size_t)(G.n_cnt + 2) * 8, ctx->stream));
        SPK_TRY(enqueue_phase(ctx, G, cap));
        SPK_HIP(hipMemcpyAsync(ctx->h_info, ctx->xinfo.p, (size_t)G.n_all * 8, hipMemcpyDeviceToHost, ctx->stream));
        SPK_HIP(hipStreamSynchronize(ctx->stream));
        if (fixed) *fixed = true;
        if (ctx->h_info[2 * K]) {
            ctx->codes_valid = false;
            SPK_REQUIRE(false, SPK_E_STATE, "spk_gammas: exact work list sizing failed");
        }
    }
    const unsigned int *h_slow = reinterpret_cast<const unsigned int *>(ctx->h_info + G.n_info);
    {  // slow-list kernels this call left out although the exact pass did list cells: run them now
        bool ran = false;
        ColSet jk{};
        for (int k = 0; k < K; ++k) {
            if (k >= (int)G.slow_skipped.size() || !G.slow_skipped[k] || !h_slow[k]) continue;
            const int si = G.simple_of[k];
            const bool lev = si >= 0 && G.simple[si].cls == SC_LEV;
            if (!lev && jk.n < 4) jk.k[jk.n++] = k;
            else SPK_TRY(enqueue_slow(ctx, G, k, nullptr));
            ran = true;
        }
        if (jk.n) SPK_TRY(enqueue_slow(ctx, G, -1, &jk));
        if (ran) {
            SPK_HIP(hipMemcpyAsync(ctx->h_info, ctx->xinfo.p, (size_t)G.n_all * 8, hipMemcpyDeviceToHost, ctx->stream));
            SPK_HIP(hipStreamSynchronize(ctx->stream));
            if (fixed) *fixed = true;
        }
        G.slow_skipped.assign((size_t)K, 0);
    }
    ctx->slow_seen.assign((size_t)K, 0);
    for (int k = 0; k < K; ++k) ctx->slow_seen[k] = h_slow[k] ? 1 : 0;
    ctx->slow_seen_valid = true;
    int err = 0;
    std::memcpy(&err, ctx->h_info + G.n_info + G.n_cnt, sizeof(err));
    if (err & 2) {
        ctx->codes_valid = false;
        SPK_REQUIRE(false, SPK_E_INVALID, "spk_gammas: unknown instruction");
    }
    int64_t n_slow = 0, n_huge = 0, max_huge = 0;
    ctx->last_exact.assign((size_t)K, 0);
    const bool carry = (int)ctx->exact_carry.size() == K;  // earlier windows of the same call
    for (int k = 0; k < K; ++k) {
        ctx->last_exact[k] = ctx->h_info[K + k] + (carry ? ctx->exact_carry[k] : 0);
        n_slow += h_slow[k];
        n_huge += h_slow[2 * K + k];
        max_huge = std::max<int64_t>(max_huge, h_slow[2 * K + k]);
    }
    ctx->last_xbase.assign(ctx->h_info, ctx->h_info + K);
    ctx->last_deferred = n_slow + ctx->deferred_carry;
    if (n_huge) {  // cells with a string longer than SLOW_LIMIT units (none in the benchmark configs)
        Scratch S;
        DevBuf<uint8_t> scratch;
        SPK_TRY(huge_scratch(G.max_units, max_huge, scratch, S));
        for (int k = 0; k < K; ++k) {
            const int64_t nk = h_slow[2 * K + k];
            if (!nk) continue;
            const int32_t *items = (G.huge_in_slow[k] ? G.A.slow : ctx->xlist.p) + ctx->h_info[k];  // + xinfo[k]
            k_gamma_huge<<<(unsigned)(S.n_slots / 64), 64, 0, ctx->stream>>>(G.A, k, items, nk, S);
            SPK_HIP(hipGetLastError());
        }
        SPK_HIP(hipStreamSynchronize(ctx->stream));
        if (fixed) *fixed = true;
    }
    return SPK_OK;
}
}  // namespace spk

extern "C" int spk_gammas(spk_ctx *ctx, int n_cols, const spk_column_program *cols, int n_when,
                          const int32_t *when_first_instr, const int32_t *when_n_instr, const int32_t *when_level,
                          int n_instr, const spk_instr *instr, int n_operands, const spk_operand *operands, int n_lits,
                          const int64_t *lit_offsets, const uint8_t *lit_utf8) {
    SPK_REQUIRE(ctx && cols && n_cols >= 1, SPK_E_INVALID, "spk_gammas: bad args");
    SPK_REQUIRE(ctx->pairs_valid, SPK_E_STATE, "spk_gammas: no pairs");
    SPK_REQUIRE(n_operands < 4096 && n_instr >= 0 && n_when >= 0, SPK_E_LIMIT, "spk_gammas: program too large");
    SPK_HIP(hipSetDevice(ctx->device));
#ifdef SPK_HOST_TIMING
    const auto ht0 = std::chrono::steady_clock::now();
#endif
    SPK_TRY(settle_gammas(ctx, nullptr));  // the previous call's capacity feedback (its codes are replaced)
#ifdef SPK_HOST_TIMING
    const auto ht1 = std::chrono::steady_clock::now();
#endif
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
        if (ctx->filter_mode != 0 &&
            classify_simple(k, cols[k], when_first_instr, when_n_instr, when_level, instr, operands, t0, t1,
                            ctx->stride, &sc))
            simple.push_back(sc);
        else
            complex_k.push_back(k);
    }
    for (SimpleCol &sc : simple) {
        sc.cls = simple_class(sc);
        prepare_tests(sc);
        sc.np = N_PLANES;
        if (sc.kind == SK_STR && t0.cols[sc.col]->unit_bits && t1.cols[sc.col]->unit_bits) {
            const uint32_t any = t0.cols[sc.col]->unit_or | t1.cols[sc.col]->unit_or;
            const uint32_t all = t0.cols[sc.col]->unit_and & t1.cols[sc.col]->unit_and;
            while (sc.np > 5 && (((any ^ all) >> (sc.np - 1)) & 1u) == 0) --sc.np;  // top bit constant
        }
        sc.has_ids = (t0.cols[sc.col]->has_ids && t1.cols[sc.col]->has_ids) ? 1 : 0;
        implied_equal(ctx, t0, t1, sc);
    }
    // character-bag rows of the free-text Levenshtein columns' strings (k_compact_lev), built on first use.
    // Free-text only: in cfg2's emails the bound decided 15 % of the listed cells (1.23 of 8.10 M), and the
    // compaction's gathers cost more than the scans it saved (γ pass 1.070 -> 1.168 ms; cfg5's addresses
    // 4.88 -> 3.85 ms; profiles/r5_ab_lev_bag.log).
    if (ctx->lev_bag) {
        bool built[2] = {false, false};
        for (const SimpleCol &sc : simple) {
            if (sc.cls != SC_LEV || sc.kind != SK_STR || !t0.cols[sc.col]->planes_hi.n || !t1.cols[sc.col]->planes_hi.n)
                continue;
            for (int s = 0; s < 2; ++s) {
                Table &t = s ? t1 : t0;
                Column *c = t.cols[sc.col];
                if (c->kind != COL_STR || c->bag.n || t.n <= 0) continue;
                SPK_TRY(build_bag_rows(ctx, t.n, c));
                t.desc_dirty = true;
                built[s] = true;
            }
        }
        if (built[0]) SPK_TRY(ensure_desc(ctx, t0));
        if (built[1]) SPK_TRY(ensure_desc(ctx, t1));
    }
    // threshold tables of the Levenshtein-ratio tests (SimpleCol.thr_off)
    std::vector<int16_t> thr_tab;
    for (SimpleCol &sc : simple) {
        for (int i = 0; i < MAX_TESTS; ++i) sc.thr_off[i] = -1;
        if (sc.cls != SC_LEV) continue;
        for (int i = 0; i < sc.n_tests; ++i) {
            if (sc.op[i] != SPK_OP_LEVRATIO || (sc.cmp[i] != SPK_CMP_LE && sc.cmp[i] != SPK_CMP_LT)) continue;
            sc.thr_off[i] = (int32_t)thr_tab.size();
            for (int S = 0; S < THR_S; ++S) {
                // `v / den cmp t` holds for v <= the entry (monotone in v); S = 0 is NULL (den = 0)
                int th = -1;
                const double den = (double)S / 2.0;
                for (int v = 0; v < THR_S && S > 0; ++v)
                    if (host_cmp((double)v / den, sc.t[i], sc.cmp[i])) th = v;
                    else break;
                thr_tab.push_back((int16_t)th);
            }
        }
    }
    const int64_t img_stride = layout_image(simple);
    // simple columns the filter kernel cannot take (no filter class, no room in the image) join the
    // interpreter's columns
    for (size_t i = 0; i < simple.size();) {
        if (simple[i].cls == SC_NONE) {
            complex_k.push_back(simple[i].k);
            simple.erase(simple.begin() + (long)i);
        } else {
            ++i;
        }
    }
    std::sort(complex_k.begin(), complex_k.end());
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
                 o_complex = put(complex_k.data(), complex_k.size()), o_thr = put(thr_tab.data(), thr_tab.size());
    // the device keeps the last blob: an unchanged program (every call of an EM run) is not re-sent
    const bool fresh_blob = ctx->prog_blob.p && ctx->prog_blob.n >= blob.size() && ctx->last_blob == blob;
    if (!fresh_blob || ctx->slow_key_pairs != ctx->pairs_epoch || ctx->slow_key_tables != ctx->table_epoch)
        ctx->slow_seen_valid = false;
    ctx->slow_key_pairs = ctx->pairs_epoch;
    ctx->slow_key_tables = ctx->table_epoch;
    if (!fresh_blob) {
        SPK_TRY(ctx->prog_blob.alloc(blob.size()));
        SPK_HIP(hipMemcpyAsync(ctx->prog_blob.p, blob.data(), blob.size(), hipMemcpyHostToDevice, ctx->stream));
        ctx->last_blob = blob;
    }
#ifdef SPK_HOST_TIMING
    const auto ht2 = std::chrono::steady_clock::now();
#endif
    uint8_t *base = ctx->prog_blob.p;
    auto at = [&](auto *&dst, size_t off) { dst = reinterpret_cast<std::remove_reference_t<decltype(dst)>>(base + off); };
    const int64_t P = ctx->n_pairs;
    // Ordinal windows: the filter's work lists and the exact / slow passes hold window-relative pair
    // ordinals as int32 (and the filter walks them in uint32), so a pair set of more than ~2^31 pairs runs
    // as consecutive windows of equal size.  Every window but the last is settled (list overflow, skipped
    // slow lists, huge cells) before the next one reuses the lists; the last is left pending as usual.
    const int64_t WMAX = ((int64_t)1 << 31) - ((int64_t)1 << 22);
    const int64_t wcap = ctx->gamma_window > 0 ? std::min<int64_t>(ctx->gamma_window, WMAX) : WMAX;
    const int64_t n_win0 = std::max<int64_t>(1, (P + wcap - 1) / wcap);
    // the two-stream split (spk_ctx::alt): two windows of half the pairs at once, one per stream
    const bool split = ctx->gamma_streams >= 2 && ctx->gamma_window == 0 && n_win0 == 1 &&
                       P >= std::max<int64_t>(ctx->split_min, 256);
    // Window 0 (the context stream, which starts first and continues after the join) takes 60 % of the pairs, or half
    // when a free-text Levenshtein column's long exact and slow passes dominate the pass: measured best shares, cfg2
    // 0.966 -> 0.943 ms per step at 60 %, cfg5 best at 50 % (profiles/r6_ab_split_share.log)
    bool long_exact = false;
    for (const SimpleCol &sc : simple) {
        const Column *a = t0.cols[sc.col], *b = t1.cols[sc.col];
        long_exact = long_exact || (sc.cls == SC_LEV && a && b && a->planes_hi.n && b->planes_hi.n);
    }
    const int64_t W = split ? (P * (long_exact ? 500 : 600) / 1000 + 63) / 64 * 64
                            : (n_win0 == 1 ? P : ((P + n_win0 - 1) / n_win0 + 63) / 64 * 64);  // pairs per window
    // rounding W up to a multiple of 64 can leave trailing windows empty (small test windows): count the
    // windows from W itself
    const int64_t n_win = split ? 2 : (n_win0 == 1 ? 1 : (P + W - 1) / W);
    if (split && !ctx->split_ready) {
        SPK_HIP(hipStreamCreateWithFlags(&ctx->alt.stream, hipStreamNonBlocking));
        SPK_HIP(hipEventCreateWithFlags(&ctx->alt.ev_info, hipEventDisableTiming));
        SPK_HIP(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
        SPK_HIP(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
        ctx->split_ready = true;
    }
    // work lists only for the columns whose filter can leave cells undecided (a dictionary-id equality
    // or numeric column never does): one slot of W pair indices each
    std::vector<int32_t> wslot(K, 0);
    int n_wslots = 0;
    for (int k = 0; k < K; ++k) {
        bool may = true;
        for (const SimpleCol &sc : simple)
            if (sc.k == k && (sc.kind == SK_NUM || sc.cls == SC_NUM || (sc.cls == SC_EQ && sc.has_ids))) may = false;
        wslot[k] = may ? n_wslots++ : 0;
    }
    SPK_TRY(ctx->codes.alloc((size_t)(P + 1) * ctx->code_bytes));
    // one filter workgroup per region of consecutive pair ordinals (a multiple of the wave size)
    // 20 regions (256-thread workgroups) per CU: four rounds of the 5 resident workgroups a CU holds
    // at the filter's 96-VGPR cap, so the regions' uneven work evens out (measured best of 1280 ..
    // 20480 on MI355X: 5120 regions 1.76 ms vs 2048 regions 1.86 ms for the cfg2 pass)
    const int64_t max_regions = 20 * (int64_t)ctx->n_cu;
    auto regions_of = [&](int64_t pw) {
        return (int)std::max<int64_t>(1, std::min<int64_t>(max_regions, (pw + F_THREADS - 1) / F_THREADS));
    };
    const int n_regions_max = regions_of(W);  // (window 0 is the larger one)
    // One device info block, read back with one copy: xinfo (k_prefix: list bases and counts, overflow,
    // total), then the slow / rest / huge list lengths (3K uint32) and the error word, both zeroed per window.
    const int n_info = 2 * K + 2;
    const int n_cnt = (3 * K + 1) / 2;  // int64 slots of the 3K uint32 list lengths
    const int n_all = n_info + n_cnt + 2;  // + the error word and k_prefix's completion counter
    // the per-window buffers (of the alternate slot too when split): every (column, region) count is written
    // by the filter launch that covers the region, so region_count needs no memset
    auto alloc_slot = [&]() -> int {
        SPK_TRY(ctx->work.alloc((size_t)std::max(n_wslots, 1) * (size_t)W + 1));
        SPK_TRY(ctx->region_count.alloc((size_t)K * n_regions_max));
        SPK_TRY(ctx->xinfo.alloc((size_t)n_all));
        SPK_TRY(ctx->pinned_info((size_t)n_all));
        SPK_TRY(ctx->xpref.alloc((size_t)K * (n_regions_max + 1)));
        return SPK_OK;
    };
    SPK_TRY(alloc_slot());
    if (split) {
        ctx->swap_slot();
        const int rc = alloc_slot();
        ctx->swap_slot();
        SPK_TRY(rc);
    }

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
    at(A.thr, o_thr);
    A.n_thr = (int)thr_tab.size();
    A.codes = ctx->codes.p;
    A.code16 = ctx->code_bytes == 2;
    for (int k = 0; k < K; ++k) A.wslot[k] = wslot[k];
    A.n_simple = (int)simple.size();
    A.n_complex = (int)complex_k.size();
    ctx->last_simple = (int)simple.size();

    // ---- the plan of the exact and slow passes (host decisions only; sized on the device by k_prefix).
    // It is kept in the context: the lists' overflow and the huge pass are settled at the next sync
    // (settle_gammas), not by a round trip inside this call.
    if (!ctx->gplan) {
        ctx->gplan = new GammaPlan();
        ctx->gplan_free = [](GammaPlan *g) { delete g; };
    }
    GammaPlan &G = *ctx->gplan;
    G.simple = simple;
    G.simple_of.assign(K, -1);
    for (size_t i = 0; i < simple.size(); ++i) G.simple_of[simple[i].k] = (int)i;
    G.may_exact.assign(K, 1);  // columns whose filter can leave cells undecided
    for (const SimpleCol &sc : simple)
        if (sc.kind == SK_NUM || sc.cls == SC_NUM || (sc.cls == SC_EQ && sc.has_ids)) G.may_exact[sc.k] = 0;
    G.free_text.assign(K, 0);  // simple columns with rows past 64 UTF-8 bytes on both sides (planes_hi)
    G.bag.assign(K, 0);        // free-text Levenshtein columns with character-bag rows (k_compact_lev)
    for (const SimpleCol &sc : simple) {
        const Column *a = t0.cols[sc.col], *b = t1.cols[sc.col];
        G.free_text[sc.k] = (a && b && a->planes_hi.n && b->planes_hi.n) ? 1 : 0;
        G.bag[sc.k] = (G.free_text[sc.k] && sc.cls == SC_LEV && a->bag.n && b->bag.n && ctx->lev_bag) ? 1 : 0;
    }
    G.huge_in_slow.assign(K, 0);  // column k's huge list: slow-list region (Levenshtein) or exact-list region
    for (int k = 0; k < K; ++k)
        G.huge_in_slow[k] = (G.may_exact[k] && G.simple_of[k] >= 0 && simple[G.simple_of[k]].cls == SC_LEV) ? 1 : 0;
    G.K = K;
    G.n_info = n_info;
    G.n_cnt = n_cnt;
    G.n_all = n_all;
    // every string a program can meet is a row of a loaded string column (UTF-8 bytes bound its UTF-16
    // units), a substring of one, or a literal: the huge pass's scratch per lane
    G.max_units = 1;
    for (const Table *t : {&t0, &t1})
        for (const Column *c : t->cols)
            if (c && c->kind == COL_STR) G.max_units = std::max<int64_t>(G.max_units, c->max_bytes);
    for (int i = 0; i < n_lits; ++i) G.max_units = std::max<int64_t>(G.max_units, llen[i]);

    ctx->exact_carry.clear();
    ctx->deferred_carry = 0;
    ctx->last_windows = n_win;
    ctx->last_split = split;
    ctx->split_w = split ? W : 0;
    SPK_TRY(ctx->begin(K_GAMMA));
    // row images and rule-view images: kernels only when a table, the column layout or the pairs changed
    ViewLaunch V{};
    bool have_view = false;
    ctx->last_view_regions = 0;
    if (P > 0) {
        SPK_TRY(build_images(ctx, t0, t1, A, img_stride, simple));
        // regions wholly inside rule 1's pairs read its view-ordered image (view launch); the others, and a
        // region straddling a rule boundary, the table image (table launches).  Only when the image
        // outgrows the caches: at 1M rows (80 MB, held by the 256 MB Infinity Cache) the second launch's
        // tail cost 4 % (1.41 vs 1.34 ms, cfg2); at 20M rows (1.6 GB) the view launch took the pass from
        // 31.1 to 22.8 ms (profiles/archive/r2_ab_views.log).
        const bool big = (A.img_rows0 + A.img_rows1) * img_stride > VIEW_MIN_IMAGE_BYTES;
        if ((ctx->use_views == 1 && big) || ctx->use_views == 2) SPK_TRY(build_view_images(ctx, A, img_stride, &V, &have_view));
    }
    // ---- graph replay: everything the launches' arguments and decisions depend on
    std::vector<int64_t> gkey;
    {
        auto ptr = [](const void *q) { return (int64_t)(uintptr_t)q; };
        gkey = {P, n_win, split ? 1 : 0, W, K, ctx->code_bytes, (int64_t)ctx->pairs_epoch, (int64_t)ctx->table_epoch,
                (int64_t)std::hash<std::string>()(std::string(blob.begin(), blob.end())), ctx->lev_kernel,
                ctx->lev_bag ? 1 : 0, ctx->filter_mode, ctx->use_views, ctx->slow_force_skip ? 1 : 0,
                have_view ? 1 : 0, ptr(ctx->stream), ptr(ctx->codes.p), ptr(ctx->pl.p), ptr(ctx->pr.p), ptr(ctx->pvl.p),
                ptr(ctx->prog_blob.p), ptr(ctx->img[0].p), ptr(ctx->img[1].p), ptr(ctx->work.p), ptr(ctx->xlist.p),
                ptr(ctx->xinfo.p), ptr(ctx->xpref.p), ptr(ctx->region_count.p), ctx->xcap, ptr(ctx->alt.work.p),
                ptr(ctx->alt.xlist.p), ptr(ctx->alt.xinfo.p), ptr(ctx->alt.xpref.p), ptr(ctx->alt.region_count.p),
                ctx->alt.xcap, ptr(ctx->alt.stream), ctx->slow_seen_valid ? 1 : 0, (int64_t)ctx->timing};
        for (uint8_t f : ctx->slow_seen) gkey.push_back(f);
        for (int v = 0; v < MAX_VIEWS; ++v) gkey.push_back(ptr(ctx->vimg[v][0].p));
    }
    const bool graphable = ctx->use_graph && !ctx->timing_exact && P > 0 && fresh_blob && (split || n_win == 1);
    const bool replay = graphable && ctx->gexec && gkey == ctx->gkey;
    const bool capture = graphable && !replay && gkey == ctx->gkey_prev;  // the second call with this key
    ctx->gkey_prev = gkey;
    if (split && !replay) {  // window 1's plan: the same program, its own window arguments
        if (!ctx->alt.gplan) ctx->alt.gplan = new GammaPlan();
        *ctx->alt.gplan = G;
    }
    bool via_graph = replay;
    if (replay) {
        // the plans as the captured call left them; the slow-list launches it skipped
        ctx->gplan->slow_skipped = ctx->gskip0;
        if (split) ctx->alt.gplan->slow_skipped = ctx->gskip1;
        ctx->last_view_regions = ctx->gview_regions;
        SPK_HIP(hipGraphLaunch(ctx->gexec, ctx->stream));
        ++ctx->graph_launches;
    } else {
    auto run_windows = [&](bool in_graph) -> int {
    if (split) {
        // window 1's stream starts after everything queued so far (images, program blob, earlier reads of the
        // codes), together with window 0.  Starting it after window 0's filter instead (so that its filter runs
        // beside window 0's exact passes) measured slower: the short JW launch then waited behind the second
        // filter's workgroups (cfg2 0.99 -> 1.02 ms per step, profiles/r6_ab_gamma_streams.log).
        SPK_HIP(hipEventRecord(ctx->ev_fork, ctx->stream));
        SPK_HIP(hipStreamWaitEvent(ctx->alt.stream, ctx->ev_fork, 0));
    }
    for (int64_t w = 0; w < n_win; ++w) {
        if (split && w == 1) ctx->swap_slot();  // window 1: the alternate buffers, plan and stream
        GammaPlan &G = *ctx->gplan;
        const int64_t b = w * W, Pw = std::min<int64_t>(W, P - b);
        const int n_regions = regions_of(Pw);
        const int64_t region_len = ((Pw + n_regions - 1) / n_regions + 63) / 64 * 64;
        GammaArgs AW = A;  // the window [b, b + Pw) as a pair set of its own
        AW.err = reinterpret_cast<int *>(ctx->xinfo.p + n_info + n_cnt);
        AW.work = ctx->work.p;
        AW.region_count = ctx->region_count.p;
        AW.slow_count = reinterpret_cast<unsigned int *>(ctx->xinfo.p + n_info);
        AW.pl = ctx->pl.p + b;
        AW.pr = ctx->pr.p + b;
        AW.P = Pw;
        AW.codes = ctx->codes.p + b * ctx->code_bytes;
        AW.region_len = region_len;
        AW.n_regions = n_regions;
        std::vector<SimpleCol> sw = simple;  // implied ranges relative to the window
        for (SimpleCol &sc : sw) {
            sc.imp_lo = std::min<int64_t>(std::max<int64_t>(sc.imp_lo - b, 0), Pw);
            sc.imp_hi = std::min<int64_t>(std::max<int64_t>(sc.imp_hi - b, 0), Pw);
            if (sc.imp_hi <= sc.imp_lo) sc.imp_lo = sc.imp_hi = 0;
        }
        G.n_regions = n_regions;
        G.g_exact = std::max<int64_t>(1, std::min<int64_t>(8 * (int64_t)ctx->n_cu, (Pw + X_THREADS - 1) / X_THREADS));
        SPK_HIP(hipMemsetAsync(ctx->xinfo.p + n_info, 0, (size_t)(n_cnt + 2) * 8, ctx->stream));
        int64_t va = n_regions, vb = n_regions;  // regions over rule 1's view-ordered image: [va, vb)
        if (Pw > 0) {
            if (have_view) {  // regions [i L, min((i + 1) L, Pw)) inside the window's part of [V.lo, V.hi)
                const int64_t lo = std::min<int64_t>(std::max<int64_t>(V.lo - b, 0), Pw);
                const int64_t hi = std::min<int64_t>(std::max<int64_t>(V.hi - b, 0), Pw);
                va = std::min<int64_t>(n_regions, (lo + region_len - 1) / region_len);
                vb = hi >= Pw ? n_regions : std::min<int64_t>(n_regions, hi / region_len);
                vb = hi > lo ? std::max<int64_t>(va, vb) : va;
            }
            ctx->last_view_regions += vb - va;
            // the filter pass (the interpreter's columns add to the codes the template filter sets)
            if (sw.empty())
                SPK_HIP(hipMemsetAsync(AW.codes, 0, (size_t)Pw * ctx->code_bytes, ctx->stream));
            if (!sw.empty()) {
                SPK_TRY(launch_template_filter(ctx->stream, AW, sw, 0, va));
                if (vb > va) {
                    GammaArgs VA = AW;
                    VA.pl = ctx->pvl.p - ctx->pv_base + b;  // pl[p] = view position of pair b + p (>= pv_base)
                    VA.pr = ctx->pvr.p - ctx->pv_base + b;
                    VA.img0 = V.img0;
                    VA.img1 = V.img1;
                    SPK_TRY(launch_template_filter(ctx->stream, VA, sw, va, vb));
                }
                SPK_TRY(launch_template_filter(ctx->stream, AW, sw, vb, n_regions));
            }
            if (AW.n_complex) {
                k_gamma_filter<<<(unsigned)n_regions, F_THREADS, 0, ctx->stream>>>(AW);
                SPK_HIP(hipGetLastError());
            }
        }
        G.A = AW;
        const int64_t cap = std::max<int64_t>(ctx->xcap, std::max<int64_t>(Pw, 1 << 16));
        SPK_TRY(enqueue_phase(ctx, G, cap, /*skip=*/true));
        if (split) {
            if (w == 0) {  // window 0's info block, on its own stream (not behind the join; a graph reads it after)
                if (!in_graph) {
                    SPK_HIP(hipMemcpyAsync(ctx->h_info, ctx->xinfo.p, (size_t)n_all * 8, hipMemcpyDeviceToHost, ctx->stream));
                    SPK_HIP(hipEventRecord(ctx->ev_info, ctx->stream));
                }
                continue;
            }
            // window 1: the join right after its last kernel (the context stream waits for nothing else of it), then
            // its info block, and the own slot back
            SPK_HIP(hipEventRecord(ctx->ev_join, ctx->stream));
            if (!in_graph) {
                SPK_HIP(hipMemcpyAsync(ctx->h_info, ctx->xinfo.p, (size_t)n_all * 8, hipMemcpyDeviceToHost, ctx->stream));
                SPK_HIP(hipEventRecord(ctx->ev_info, ctx->stream));
            }
            ctx->gamma_pending = true;
            ctx->swap_slot();
            SPK_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
            break;
        }
        if (w + 1 == n_win) break;
        // settle this window before the next one reuses the lists
        SPK_HIP(hipMemcpyAsync(ctx->h_info, ctx->xinfo.p, (size_t)n_all * 8, hipMemcpyDeviceToHost, ctx->stream));
        SPK_HIP(hipEventRecord(ctx->ev_info, ctx->stream));
        ctx->gamma_pending = true;
        ctx->codes_valid = true;
        SPK_TRY(settle_info(ctx, nullptr));
        ctx->exact_carry = ctx->last_exact;
        ctx->deferred_carry = ctx->last_deferred;
    }
        return SPK_OK;
    };
    bool cap = capture;
    if (cap) {
        if (ctx->gexec) (void)hipGraphExecDestroy(ctx->gexec);
        if (ctx->graph) (void)hipGraphDestroy(ctx->graph);
        ctx->gexec = nullptr;
        ctx->graph = nullptr;
        ctx->gkey.clear();
        if (hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
            (void)hipGetLastError();
            cap = false;
            ctx->use_graph = false;
        }
    }
    int rc = run_windows(cap);
    if (cap) {
        hipGraph_t g = nullptr;
        hipError_t e = hipStreamEndCapture(ctx->stream, &g);
        if (rc == SPK_OK && e == hipSuccess) e = hipGraphInstantiate(&ctx->gexec, g, nullptr, nullptr, 0);
        if (rc == SPK_OK && e == hipSuccess) {
            ctx->graph = g;
            ctx->gkey = gkey;
            ctx->gskip0 = ctx->gplan->slow_skipped;
            if (split) ctx->gskip1 = ctx->alt.gplan->slow_skipped;
            ctx->gview_regions = ctx->last_view_regions;
            rc = hipGraphLaunch(ctx->gexec, ctx->stream) == hipSuccess ? SPK_OK : SPK_E_HIP;
        } else {
            // nothing of the captured pass ran: no graphs on this context from now on, the pass enqueued directly
            if (g) (void)hipGraphDestroy(g);
            ctx->gexec = nullptr;
            (void)hipGetLastError();
            ctx->use_graph = false;
            cap = false;
            if (rc == SPK_OK) rc = run_windows(false);
        }
    }
    SPK_TRY(rc);
    via_graph = cap;
    }  // (not a replay)
    SPK_TRY(ctx->end(K_GAMMA));
    if (!split || via_graph) {
        // the info blocks on the context stream behind the pass (a split call without a graph read window 0's back
        // in the loop, window 1's on its own stream)
        SPK_HIP(hipMemcpyAsync(ctx->h_info, ctx->xinfo.p, (size_t)n_all * 8, hipMemcpyDeviceToHost, ctx->stream));
        SPK_HIP(hipEventRecord(ctx->ev_info, ctx->stream));
        if (split) {
            SPK_HIP(hipMemcpyAsync(ctx->alt.h_info, ctx->alt.xinfo.p, (size_t)n_all * 8, hipMemcpyDeviceToHost, ctx->stream));
            SPK_HIP(hipEventRecord(ctx->alt.ev_info, ctx->stream));
            ctx->alt.gamma_pending = true;
        }
    }
    ++ctx->gamma_seq;
    ctx->gamma_pending = true;
    ctx->codes_valid = true;
    ctx->mpat_valid = false;
    ctx->last_implied.assign((size_t)K, 0);
    for (const SimpleCol &sc : simple) ctx->last_implied[sc.k] = sc.imp_hi - sc.imp_lo;
#ifdef SPK_HOST_TIMING
    {  // diagnostic build only: host time per spk_gammas phase (settle wait, program preparation, enqueue)
        static double acc[3] = {0, 0, 0};
        static int calls = 0;
        const auto ht3 = std::chrono::steady_clock::now();
        acc[0] += std::chrono::duration<double, std::micro>(ht1 - ht0).count();
        acc[1] += std::chrono::duration<double, std::micro>(ht2 - ht1).count();
        acc[2] += std::chrono::duration<double, std::micro>(ht3 - ht2).count();
        if (++calls % 20 == 0) {
            std::fprintf(stderr, "[spk host] per call: settle %.1f us, prepare %.1f us, enqueue %.1f us\n", acc[0] / 20,
                         acc[1] / 20, acc[2] / 20);
            acc[0] = acc[1] = acc[2] = 0;
        }
    }
#endif
    return SPK_OK;
}

extern "C" int spk_gammas_load(spk_ctx *ctx, int n_cols, const int32_t *n_levels, int64_t n, const int8_t *gammas) {
    SPK_REQUIRE(ctx && n_levels && n >= 0 && (n == 0 || gammas), SPK_E_INVALID, "spk_gammas_load: bad args");
    SPK_HIP(hipSetDevice(ctx->device));
    SPK_TRY(settle_gammas(ctx, nullptr));
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
    ctx->gamma_pending = false;
    ctx->alt.gamma_pending = false;
    ++ctx->gamma_seq;
    ctx->codes_valid = true;
    return SPK_OK;
}

extern "C" int spk_gammas_copy(spk_ctx *ctx, int64_t start, int64_t count, int8_t *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "spk_gammas_copy: bad args");
    SPK_REQUIRE(ctx->codes_valid, SPK_E_STATE, "spk_gammas_copy: no gammas");
    SPK_REQUIRE(start >= 0 && count >= 0 && start + count <= ctx->n_pairs, SPK_E_INVALID, "range out of bounds");
    SPK_HIP(hipSetDevice(ctx->device));
    SPK_TRY(settle_gammas(ctx, nullptr));
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
// the global-memory jw_long / lev_long for the rest, and pairs with a string past SLOW_LIMIT units
// through the huge pass (device scratch sized to the longest string).
struct UdfArgs {
    int64_t n;
    const uint16_t *u16;
    const int64_t *off;  // [2n+1]: string i of pair p is 2p (left) and 2p+1 (right)
    const int32_t *cp;   // code points per string
    int op;              // 0 JW, 1 Levenshtein
    double *out;
    int32_t *huge;              // pairs for k_udf_huge
    unsigned int *n_huge;
};

__device__ inline StrView udf_view(const UdfArgs &U, int64_t s) {
    return plain_view(U.u16 + U.off[s], (int32_t)(U.off[s + 1] - U.off[s]), U.cp[s]);
}

__global__ __launch_bounds__(U_THREADS) void k_udf(UdfArgs U) {
    __shared__ uint16_t lds[2][MAXU][U_THREADS];
    uint16_t *slot_a = &lds[0][0][threadIdx.x];
    uint16_t *slot_b = &lds[1][0][threadIdx.x];
    int64_t p = (int64_t)blockIdx.x * U_THREADS + threadIdx.x;
    if (p >= U.n) return;
    const StrView a = udf_view(U, 2 * p), b = udf_view(U, 2 * p + 1);
    if (a.n > SLOW_LIMIT || b.n > SLOW_LIMIT) {
        U.huge[atomicAdd(U.n_huge, 1u)] = (int32_t)p;
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

__global__ __launch_bounds__(64) void k_udf_huge(UdfArgs U, int64_t n, Scratch S) {
    S.slot = (int64_t)blockIdx.x * 64 + threadIdx.x;
    for (int64_t i = S.slot; i < n; i += S.n_slots) {
        const int64_t p = U.huge[i];
        const StrView a = udf_view(U, 2 * p), b = udf_view(U, 2 * p + 1);
        U.out[p] = U.op == 0 ? jw_long(GlbAcc{a.p}, a.n, GlbAcc{b.p}, b.n, S.at<uint64_t>(0), S.at<uint64_t>(S.words))
                             : (double)lev_long(a, b, S.at<uint32_t>(0), S.at<int32_t>(S.units));
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
    DevBuf<int32_t> d_huge;
    DevBuf<unsigned int> d_nhuge;
    SPK_TRY(d_u.alloc(u.size()));
    SPK_TRY(d_off.alloc(off.size()));
    SPK_TRY(d_cp.alloc(cp.size() + 1));
    SPK_TRY(d_out.alloc((size_t)n + 1));
    SPK_TRY(d_huge.alloc((size_t)n + 1));
    SPK_TRY(d_nhuge.alloc(1));
    SPK_HIP(hipMemsetAsync(d_nhuge.p, 0, sizeof(unsigned int), ctx->stream));  // hipMalloc does not zero
    SPK_HIP(hipMemcpyAsync(d_u.p, u.data(), u.size() * 2, hipMemcpyHostToDevice, ctx->stream));
    SPK_HIP(hipMemcpyAsync(d_off.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    if (!cp.empty()) SPK_HIP(hipMemcpyAsync(d_cp.p, cp.data(), cp.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    if (!n) return SPK_OK;
    UdfArgs U{n, d_u.p, d_off.p, d_cp.p, op, d_out.p, d_huge.p, d_nhuge.p};
    k_udf<<<(unsigned)((n + U_THREADS - 1) / U_THREADS), U_THREADS, 0, ctx->stream>>>(U);
    SPK_HIP(hipGetLastError());
    unsigned int n_huge = 0;
    SPK_HIP(hipMemcpyAsync(&n_huge, d_nhuge.p, sizeof(n_huge), hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    DevBuf<uint8_t> scratch;
    if (n_huge) {
        int64_t units = 1;
        for (size_t i = 0; i + 1 < off.size(); ++i) units = std::max<int64_t>(units, off[i + 1] - off[i]);
        Scratch S;
        SPK_TRY(huge_scratch(units, n_huge, scratch, S));
        k_udf_huge<<<(unsigned)(S.n_slots / 64), 64, 0, ctx->stream>>>(U, (int64_t)n_huge, S);
        SPK_HIP(hipGetLastError());
    }
    SPK_HIP(hipMemcpyAsync(out, d_out.p, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
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

extern "C" int spk_gammas_exact_ms(spk_ctx *ctx, double *out, int n) {
    SPK_REQUIRE(ctx && out && n >= 0, SPK_E_INVALID, "spk_gammas_exact_ms: bad args");
    SPK_HIP(hipSetDevice(ctx->device));
    SPK_TRY(settle_gammas(ctx, nullptr));
    SPK_HIP(hipStreamSynchronize(ctx->stream));
    // a two-stream split timed each window's launch on its own stream: the sum of both
    const bool two = ctx->last_windows == 2 && ctx->split_ready && ctx->alt.xev_used.size();
    for (int k = 0; k < n; ++k) {
        out[k] = -1.0;
        if (k < (int)ctx->xev_used.size() && ctx->xev_used[k]) {
            float ms = 0.f;
            SPK_HIP(hipEventElapsedTime(&ms, ctx->xev0[k], ctx->xev1[k]));
            out[k] = (double)ms;
        }
        if (two && k < (int)ctx->alt.xev_used.size() && ctx->alt.xev_used[k]) {
            float ms = 0.f;
            SPK_HIP(hipEventElapsedTime(&ms, ctx->alt.xev0[k], ctx->alt.xev1[k]));
            out[k] = (out[k] < 0 ? 0.0 : out[k]) + (double)ms;
        }
    }
    return SPK_OK;
}

extern "C" int spk_gammas_deferred(spk_ctx *ctx, int64_t *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "null arg");
    SPK_TRY(settle_gammas(ctx, nullptr));
    *out = ctx->last_deferred;
    return SPK_OK;
}

extern "C" int spk_gammas_exact_list(spk_ctx *ctx, int k, int32_t *out, int64_t n) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    SPK_TRY(settle_gammas(ctx, nullptr));
    SPK_REQUIRE(out && k >= 0 && k < (int)ctx->last_exact.size() && n >= 0, SPK_E_INVALID,
                "spk_gammas_exact_list: bad args");
    const int64_t m = std::min<int64_t>(n, ctx->last_exact[k]);
    if (!ctx->last_split) {
        if (m > 0)
            SPK_HIP(hipMemcpy(out, ctx->xlist.p + ctx->last_xbase[k], (size_t)m * sizeof(int32_t), hipMemcpyDeviceToHost));
        return SPK_OK;
    }
    // a split call: window 0's list, then window 1's with its window-relative ordinals made global
    const int64_t m0 = std::min<int64_t>(m, ctx->split_first[k]), m1 = m - m0;
    if (m0 > 0)
        SPK_HIP(hipMemcpy(out, ctx->xlist.p + ctx->last_xbase[k], (size_t)m0 * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (m1 > 0) {
        SPK_HIP(hipMemcpy(out + m0, ctx->alt.xlist.p + ctx->alt_xbase[k], (size_t)m1 * sizeof(int32_t), hipMemcpyDeviceToHost));
        for (int64_t i = m0; i < m; ++i)
            if (out[i] >= 0) out[i] += (int32_t)ctx->split_w;
    }
    return SPK_OK;
}

extern "C" int spk_gammas_exact_counts(spk_ctx *ctx, int64_t *out, int n) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    SPK_TRY(settle_gammas(ctx, nullptr));
    SPK_REQUIRE(out && n >= (int)ctx->last_exact.size(), SPK_E_INVALID, "spk_gammas_exact_counts: bad args");
    for (size_t k = 0; k < ctx->last_exact.size(); ++k) out[k] = ctx->last_exact[k];
    return SPK_OK;
}

extern "C" int spk_gammas_implied_pairs(spk_ctx *ctx, int64_t *out, int n) {
    SPK_REQUIRE(ctx && out && n >= (int)ctx->last_implied.size(), SPK_E_INVALID, "spk_gammas_implied_pairs: bad args");
    for (size_t k = 0; k < ctx->last_implied.size(); ++k) out[k] = ctx->last_implied[k];
    return SPK_OK;
}

extern "C" int spk_gammas_set_simple(spk_ctx *ctx, int on) {
    SPK_REQUIRE(ctx && on >= 0 && on % 10 <= 1 && on % 100 < 30 && on < 200, SPK_E_INVALID,
                "spk_gammas_set_simple: mode 0, 1 (+10 / +20) (+100)");
    ctx->use_views = on % 100 >= 20 ? 2 : (on % 100 >= 10 ? 0 : 1);
    ctx->filter_mode = on % 10;
    ctx->slow_force_skip = on >= 100;
    return SPK_OK;
}

extern "C" int spk_ctx_memory(spk_ctx *ctx, int64_t *out8) {
    SPK_REQUIRE(ctx && out8, SPK_E_INVALID, "spk_ctx_memory: null arg");
    auto b = [](const auto &buf) { return (int64_t)(buf.n * sizeof(*buf.p)); };
    int64_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (const RawCol *r : ctx->raw)
        if (r) m[0] += b(r->off) + b(r->bytes) + b(r->i64) + b(r->valid);
    for (const Table &t : ctx->table) {
        m[1] += b(t.perm) + b(t.rank) + b(t.d_desc);
        for (int w = 0; w < 2; ++w)
            for (const DevBuf<int64_t> *k : t.key[w])
                if (k) m[1] += b(*k);
        for (const Column *c : t.cols)
            if (c) m[1] += b(c->units) + b(c->meta) + b(c->planes) + b(c->planes_hi) + b(c->bag) + b(c->val) + b(c->valid);
    }
    for (int s = 0; s < 2; ++s) {
        m[2] += b(ctx->img[s]);
        for (int v = 0; v < MAX_VIEWS; ++v) m[2] += b(ctx->vimg[v][s]);
    }
    m[3] = b(ctx->pl) + b(ctx->pr) + b(ctx->pvl) + b(ctx->pvr);
    for (int v = 0; v < MAX_VIEWS; ++v) m[3] += b(ctx->views[v].rowsL) + b(ctx->views[v].rowsR);
    m[4] = b(ctx->codes);
    m[5] = b(ctx->work) + b(ctx->xlist) + b(ctx->xpref) + b(ctx->xinfo) + b(ctx->region_count) + b(ctx->prog_blob) +
           b(ctx->alt.work) + b(ctx->alt.xlist) + b(ctx->alt.xpref) + b(ctx->alt.xinfo) + b(ctx->alt.region_count);
    m[6] = b(ctx->hist) + b(ctx->mpat) + b(ctx->llpat) + b(ctx->cpat) + b(ctx->stats) + b(ctx->mu) + b(ctx->em_ticket) +
           b(ctx->em_row) + b(ctx->em_hot) + b(ctx->mp) + b(ctx->mpat_score) + b(ctx->tf_uniq) + b(ctx->tf_runs) +
           b(ctx->tf_nruns) + b(ctx->tf_mp) + b(ctx->tf_hist) +
           b(ctx->tf_sort);
    for (int i = 0; i < 7; ++i) m[7] += m[i];
    for (int i = 0; i < 8; ++i) out8[i] = m[i];
    return SPK_OK;
}

extern "C" int spk_ctx_lds_per_block(spk_ctx *ctx, int *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "null arg");
    *out = ctx->lds_per_block;
    return SPK_OK;
}

extern "C" int spk_gammas_view_regions(spk_ctx *ctx, int64_t *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "null arg");
    *out = ctx->last_view_regions;
    return SPK_OK;
}

extern "C" int spk_gammas_simple_count(spk_ctx *ctx, int *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "null arg");
    *out = ctx->last_simple;
    return SPK_OK;
}

extern "C" int spk_gammas_set_window(spk_ctx *ctx, int64_t pairs) {
    SPK_REQUIRE(ctx && pairs >= 0, SPK_E_INVALID, "spk_gammas_set_window: bad args");
    ctx->gamma_window = pairs;
    return SPK_OK;
}

extern "C" int spk_gammas_set_graph(spk_ctx *ctx, int on) {
    SPK_REQUIRE(ctx, SPK_E_INVALID, "null ctx");
    ctx->use_graph = on != 0;
    ctx->gkey_prev.clear();
    return SPK_OK;
}

extern "C" int spk_gammas_graph_launches(spk_ctx *ctx, int64_t *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "null arg");
    *out = ctx->graph_launches;
    return SPK_OK;
}

extern "C" int spk_gammas_set_streams(spk_ctx *ctx, int streams, int64_t min_pairs) {
    SPK_REQUIRE(ctx && (streams == 1 || streams == 2) && min_pairs >= 0, SPK_E_INVALID,
                "spk_gammas_set_streams: 1 or 2 streams, min_pairs >= 0");
    SPK_TRY(settle_gammas(ctx, nullptr));
    ctx->gamma_streams = streams;
    ctx->split_min = min_pairs;
    return SPK_OK;
}

extern "C" int spk_gammas_windows(spk_ctx *ctx, int64_t *out) {
    SPK_REQUIRE(ctx && out, SPK_E_INVALID, "spk_gammas_windows: bad args");
    *out = ctx->last_windows;
    return SPK_OK;
}

extern "C" int spk_gammas_set_lev_kernel(spk_ctx *ctx, int mode) {
    SPK_REQUIRE(ctx && mode >= 0 && mode <= 3, SPK_E_INVALID, "spk_gammas_set_lev_kernel: mode 0 .. 3");
    ctx->lev_kernel = mode == 3 ? 2 : mode;
    ctx->lev_bag = mode != 3;
    return SPK_OK;
}

#ifdef SPK_LEVQ_STATS
extern "C" int spk_debug_levq_stats(uint64_t *out, int reset) {
    SPK_HIP(hipDeviceSynchronize());
    SPK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_levq), sizeof(uint64_t) * 16));
    if (reset) {
        static const unsigned long long zero[16] = {};
        SPK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_levq), zero, sizeof(zero)));
    }
    return SPK_OK;
}
#endif
