// Shared definitions of the comparison-vector passes (spk_gamma.hip: interpreter, exact / slow / huge
// passes, host orchestration; spk_filter.hip: the template-column filter pass).
#pragma once

#include <vector>

#include "spk_strsim.h"

namespace spk {

constexpr int F_THREADS = 256;  // filter pass
constexpr int X_THREADS = 256;  // exact pass
constexpr int U_THREADS = 128;  // UDF kernel: 2 x 64 x 128 x 2 B = 32 KiB of LDS per block

enum Mode { M_FILTER = 0, M_EXACT = 1, M_SLOW = 2, M_HUGE = 3 };
enum Status { ST_DONE = 0, ST_UNDECIDED = 1, ST_NEEDS_SLOW = 2 };

// A "simple" comparison column: the shape every case_statements.py template has --
//   WHEN x_l IS NULL OR x_r IS NULL THEN null_level
//   WHEN test_1(x_l, x_r) THEN level_1 ... WHEN test_n(x_l, x_r) THEN level_n ELSE else_level
// with each test one leaf (=, <>, jaro_winkler_sim cmp t, levenshtein [ratio] cmp t, numeric
// compare / abs diff / percent diff) over the same two plain operands.  The filter pass evaluates
// these straight from the two rows' metadata records, loaded for several columns at once; every
// other program runs through the general interpreter.  Both give identical levels.
constexpr int MAX_TESTS = 6;
constexpr int MAX_SIMPLE = 64;   // = the column limit of set_pattern_space
enum SimpleKind : int32_t { SK_STR = 1, SK_NUM = 2 };
// Filter class of a simple column, chosen on the host: which row-image fields the filter reads and
// which bound logic decides the column (spk_filter.hip).  A simple column of no class (other tests,
// or no room left in the image) is evaluated by the general interpreter instead.
enum SimpleClass : int32_t { SC_NONE = 0, SC_EQ = 1, SC_JW = 2, SC_LEV = 3, SC_NUM = 4 };
struct SimpleCol {
    int32_t k;  // comparison column (position in the code)
    int32_t kind;
    int32_t col;  // table column, the same index on both sides
    int32_t null_level, else_level, n_tests;
    int32_t op[MAX_TESTS], cmp[MAX_TESTS], level[MAX_TESTS];
    double t[MAX_TESTS];
    int64_t stride;
    int32_t cls;      // SimpleClass
    int32_t off;      // byte offset of the column's fields in a row-image row
    int32_t off2;     // SC_JW: offset of the four head units
    int32_t has_ids;  // both sides carry dictionary ids (equal keys = equal strings)
    int32_t eq4;      // SC_EQ with ids in half of a JW gap: a 4-byte field, the id or 0xFFFFFFFF (NULL)
    // Per-test decision parameters, precomputed on the host (prepare_tests) so the filter decides
    // every test with compares and selects only -- no divergent branches:
    int32_t tflag[MAX_TESTS];  // TF_* bits
    int32_t lev_a[MAX_TESTS];  // LEV (absolute): integer bound of the equivalent integer test
    float jw_cf[MAX_TESTS];    // JW: an upper bound hi < jw_cf proves the test false
    // Pairs [imp_lo, imp_hi) come from a blocking rule whose key includes `l.c = r.c` on this
    // column's own raw columns: their strings are equal, non-NULL (and non-empty: no empty value
    // in the column), so their level is eq_level and the filter reads nothing for them.
    int64_t imp_lo, imp_hi;
    int32_t eq_level;
    // LEVRATIO tests: offset of the test's threshold table in GammaArgs.thr (-1: none).  Entry S is
    // the largest distance v with `v / (S / 2.0) cmp t` true in fp64 (Spark's division), for
    // S = len_l + len_r (code points) < THR_S: the filter decides the test with integer compares.
    int32_t thr_off[MAX_TESTS];
    // Bit-planes the Levenshtein scans need: bits np..7 of every plane-row unit of the column (both
    // sides) are the same (Column.unit_or / unit_and), so those planes' match-mask terms are no-ops.
    int32_t np;
};
constexpr int THR_S = 256;
constexpr int32_t TF_ZERO = 1;     // the value 0.0 passes the test (JW of strings without a common unit; lev ratio 0)
constexpr int32_t TF_ONE = 2;      // JW: the value 1.0 passes (equal non-empty strings)
constexpr int32_t TF_GE = 4;       // LEV: the test is `lev >= lev_a` (else `lev <= lev_a`)
constexpr int32_t TF_EXACT = 8;    // LEV `=` / `<>`: decided only when the bounds meet
constexpr int32_t TF_EQ = 16;      // `=` (else `<>`)

// ---- filter row image ----------------------------------------------------------------------------
// The filter needs a few bytes per (row, column) -- equality key, lengths, unit sketch, head units --
// but reading them from each column's own 32-byte records costs a cache line per row AND column,
// and the pairs of a second blocking rule land on random rows.  So before the filter pass the
// fields of every simple column are packed, per row, into one row of a row image (<= IMG_MAX
// bytes, 16-byte aligned): a pair then reads two rows' lines whatever the number of columns.
//   SC_EQ   8 B {key u32, lens u32}            SC_LEV 16 B {key, lens, sketch u64}
//   SC_JW  16 B {key, lens, sketch} + 8 B head units at off2
//   SC_NUM 16 B {value f64, valid u32, pad}
// lens = UTF-16 length | code points << 16, each saturating at LEN_SAT; LENS_NULL = NULL.
constexpr int IMG_MAX = 256;
constexpr int64_t VIEW_MIN_IMAGE_BYTES = (int64_t)192 << 20;  // rule-view images only past this size
constexpr uint32_t LENS_NULL = 0xFFFFFFFFu;
constexpr int LEN_SAT = 0xFFFE;
// A chunk plane of the image as a buffer resource: gathers then take a 32-bit per-lane byte offset
// (row x 16) against a wave-uniform descriptor -- no 64-bit address arithmetic per load
// (cdna_hip_programming.md T8).  One plane holds at most 2^31 bytes (2^27 rows).
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
__device__ inline __amdgpu_buffer_rsrc_t image_rsrc(const uint8_t *base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)bytes, 0x00020000);
}
constexpr int64_t IMG_MAX_ROWS = ((int64_t)1 << 27) - 1;

// Chunk-major image: the 16-byte chunk c of every row is contiguous, so the lanes of a wave that
// read the same field of consecutive rows (a block's pairs) share a few cache lines.
__host__ __device__ inline int64_t img_at(int64_t rows, int64_t row, int off) {
    return ((int64_t)(off >> 4) * rows + row) * 16 + (off & 15);
}

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
    int32_t *work;                // [slots][P] pair indices per column needing the exact pass, by region
    int32_t wslot[MAX_SIMPLE];    // column k's work-list slot (columns whose filter can leave cells undecided)
    unsigned int *region_count;   // [K][n_regions] list length of each region
    int64_t region_len;           // pair ordinals per region (one filter workgroup each)
    int n_regions;
    int32_t *slow;             // slow-pass lists, column k at slow_off[k]
    const int64_t *slow_off;
    unsigned int *slow_count;  // [3K]: slow lists, k_gamma_slow_lev's rest lists, huge lists
    int *err;
    const SimpleCol *simple;   // filter pass: simple columns ...
    int n_simple;
    const int32_t *complex_k;  // ... and the columns the interpreter evaluates
    int n_complex;
    const uint8_t *img0, *img1;  // filter row images of the l- and r-side tables (k_build_image)
    int64_t img_stride;          // bytes of one row's fields (a multiple of 16)
    int64_t img_rows0, img_rows1;  // rows of each image (chunk-major layout: chunk c of row r at (c * rows + r) * 16)
    // per filter launch: regions [region_base, region_base + gridDim.x); a view launch (rule 1's pairs)
    // reads pl / pr = their view positions and img0 / img1 = view-ordered images
    int region_base;
    const int16_t *thr;  // LEVRATIO threshold tables (SimpleCol.thr_off), n_thr entries
    int n_thr;
};

// Codes are written in place: the filter pass sets each pair's code (a 2-byte store leaves the
// neighbouring pair's code alone), the exact / slow passes of column k add to it (a pair occurs at
// most once in column k's lists).
__device__ inline void code_set(const GammaArgs &A, int64_t p, uint32_t v) {
    if (A.code16) static_cast<uint16_t *>(A.codes)[p] = (uint16_t)v;
    else static_cast<uint32_t *>(A.codes)[p] = v;
}
// The exact and slow passes add their column's digit to the code the filter set.  Launches of one
// column run in stream order and a pair occurs once in a column's lists: a plain read-modify-write
// (an atomic add measured 2.4x the HBM writes of the Levenshtein pass at the same kernel time,
// profiles/r2b_traffic.json).
__device__ inline void code_add(const GammaArgs &A, int64_t p, uint32_t d) {
    if (A.code16) {
        uint16_t *c = static_cast<uint16_t *>(A.codes) + p;
        *c = (uint16_t)(*c + d);
    } else {
        static_cast<uint32_t *>(A.codes)[p] += d;
    }
}

// Several columns in one launch (ExactCols) may update one pair's code at once: an atomic add on
// the aligned dword (a 16-bit code never carries into its neighbour -- a code stays below the
// pattern count, <= 65536).
__device__ inline void code_add_atomic(const GammaArgs &A, int64_t p, uint32_t d) {
    if (A.code16) {
        uint32_t *w = reinterpret_cast<uint32_t *>(static_cast<uint16_t *>(A.codes) + (p & ~(int64_t)1));
        atomicAdd(w, d << (16 * (uint32_t)(p & 1)));
    } else {
        atomicAdd(static_cast<uint32_t *>(A.codes) + p, d);
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

// Fold one WHEN test into the branch chain: the first test that is TRUE (or UNDECIDED) ends it;
// FALSE and NULL fall through to the next WHEN (a NULL predicate is a branch not taken).  r is
// KF 0 / KT 1 / KN 2 / KU 3, so "ends the chain" is r & 1 and "undecided" r >> 1 on top: the chain
// state stays in integer registers (VALU bit ops) instead of per-lane condition masks, and the
// lanes of a wave never diverge over which test decided them.
struct Chain {
    int open = 1, und = 0, lvl = 0;
    Chain() = default;
    __device__ explicit Chain(int else_level) : lvl(else_level) {}
    __device__ __attribute__((always_inline)) void fold(int r, int lvl_i) {
        const int hit = r & open;  // bit 0: TRUE / UNDECIDED while open
        und |= hit & (r >> 1);
        lvl += hit * (lvl_i - lvl);
        open &= ~hit;
    }
};


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
    const int64_t r0 = (int64_t)(A.region_base + blockIdx.x) * A.region_len;
    const int64_t r1 = r0 + A.region_len < A.P ? r0 + A.region_len : A.P;
    return Region{r0, r1};
}

__device__ inline int32_t *region_list(const GammaArgs &A, int k, const Region &r) {
    return A.work + (int64_t)A.wslot[k] * A.P + r.r0;
}

template <class SC>
__device__ __attribute__((always_inline)) inline int simple_num(const SC &sc, bool va, double a, bool vb, double b) {
    Chain c(sc.else_level);
    const double diff = fabs(a - b), big = fabs(a > b ? a : b);
    for (int i = 0; i < sc.n_tests; ++i) {
        const int op = sc.op[i], cmp = sc.cmp[i];
        int r;
        if (op == SPK_OP_NUM_CMP) r = cmpd(a, b, cmp);
        else if (op == SPK_OP_ABSDIFF) r = cmpd(diff, sc.t[i], cmp);
        else r = big == 0.0 ? KN : cmpd(diff / big, sc.t[i], cmp);  // SPK_OP_PERCDIFF
        c.fold(r, sc.level[i]);
    }
    return (!va || !vb) ? sc.null_level : c.lvl;
}

__device__ inline int lens_u16(uint32_t l) { return (int)(l & 0xFFFFu); }
__device__ inline int lens_cp(uint32_t l) { return (int)(l >> 16); }
__device__ inline uint64_t img_sketch(const uint4 &v) { return ((uint64_t)v.w << 32) | v.z; }

// sketch_inter_ub without the data-dependent branch (both saturated buckets add min(rest_a, rest_b)).
__device__ __attribute__((always_inline)) inline int sketch_inter_ub_bf(uint64_t sa, uint64_t sb, int la, int lb) {
    const uint32_t aL = (uint32_t)sa, aH = (uint32_t)(sa >> 32);
    const uint32_t bL = (uint32_t)sb, bH = (uint32_t)(sb >> 32);
    const uint32_t gt = (aH & ~bH) | (~(aH ^ bH) & aL & ~bL);
    const uint32_t mL = (aL & ~gt) | (bL & gt), mH = (aH & ~gt) | (bH & gt);
    const uint32_t both_sat = aL & aH & bL & bH, rest = ~both_sat;
    const int lmn = la < lb ? la : lb;
    if (!__any(both_sat != 0u)) {  // wave-uniform: no bucket saturated on both sides (rest = all ones)
        const int inter = __builtin_popcount(mL) + 2 * __builtin_popcount(mH);
        return inter < lmn ? inter : lmn;
    }
    int inter = __builtin_popcount(mL & rest) + 2 * __builtin_popcount(mH & rest);
    const int ra = la - (__builtin_popcount(aL & rest) + 2 * __builtin_popcount(aH & rest));
    const int rb = lb - (__builtin_popcount(bL & rest) + 2 * __builtin_popcount(bH & rest));
    inter += both_sat ? (ra < rb ? ra : rb) : 0;
    return inter < lmn ? inter : lmn;
}

__device__ inline double bits_to_double(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Append the lanes' wanted values of FP ballots to a list: one LDS atomic per call.  The wave must be
// converged (lane 0 active).
template <int FP>
__device__ inline void wave_append_batch(int32_t *list, unsigned int *count, const bool (&want)[FP],
                                         const int64_t (&val)[FP]) {
    unsigned long long m[FP];
    unsigned int total = 0;
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        m[u] = __ballot(want[u]);
        total += (unsigned int)__popcll(m[u]);
    }
    if (!total) return;
    const int lane = threadIdx.x & 63;
    unsigned int base = 0;
    if (lane == 0) base = atomicAdd(count, total);
    base = __shfl(base, 0);
    const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
    for (int u = 0; u < FP; ++u) {
        if (want[u]) list[base + __popcll(m[u] & below)] = (int32_t)val[u];
        base += (unsigned int)__popcll(m[u]);
    }
}

// ---- template-column filter pass (spk_filter.hip) -------------------------------------------------
// Filter regions [region_lo, region_hi) of A's pair range over the simple columns (every one of class
// SC_EQ / SC_JW / SC_LEV / SC_NUM, laid out in A's row image), `shm` bytes of LDS for the threshold
// tables.  Writes each pair's code over those columns, their work lists and region counts.
int launch_template_filter(hipStream_t stream, const GammaArgs &A, const std::vector<SimpleCol> &simple,
                           int64_t region_lo, int64_t region_hi);
// Columns of each class the filter kernel handles (more go to the interpreter).
constexpr int FJ_MAX = 4, FL_MAX = 3, FE_MAX = 6, FN_MAX = 4;

}  // namespace spk
