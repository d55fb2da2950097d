/*
 * splink_hip.h -- C ABI of libsplink_hip.so, the MI355X (gfx950) execution engine for
 * splink's pairwise-comparison + EM hot path.
 *
 * The reference (splink 0.1.7) has no native boundary: every stage is a Python
 * function that emits Spark SQL.  These entry points replace the
 * Spark execution (L0) of those stages; the Python layer in splink_amd/ keeps the
 * reference's stage-function API and calls them through ctypes.  Each entry point
 * names the reference interface it replaces.
 *
 * Conventions
 *   - Every function returns SPK_OK (0) or a negative SPK_E_* code; spk_last_error()
 *     gives a thread-local message.
 *   - Host buffers passed in are BORROWED for the duration of the call; outputs are
 *     caller-allocated.  Device state is owned by the context.
 *   - A context is bound to one HIP device and one stream and is not re-entrant;
 *     callers serialise.  Multi-GPU = one process (one context) per GPU; the only
 *     cross-GPU exchange is the EM pattern histogram (spk_em_histogram writes it to a
 *     caller-provided device buffer, the caller all-reduces it, spk_em_finalize reads it).
 */
#ifndef SPLINK_HIP_H
#define SPLINK_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPK_OK 0
#define SPK_E_INVALID (-1) /* bad argument / shape (Python: ValueError) */
#define SPK_E_HIP (-2)     /* HIP runtime failure */
#define SPK_E_OOM (-3)     /* device allocation failed */
#define SPK_E_STATE (-4)   /* call out of order (e.g. gammas before pairs) */
#define SPK_E_LIMIT (-5)   /* input beyond a supported limit (e.g. 2^31 rows in one table) */

#define SPK_LINK_DEDUPE 0        /* "dedupe_only"     */
#define SPK_LINK_ONLY 1          /* "link_only"       */
#define SPK_LINK_AND_DEDUPE 2    /* "link_and_dedupe" */

typedef struct spk_ctx spk_ctx;

const char *spk_last_error(void);
int spk_version(void);
int spk_device_count(int *out);

/* ---- context ------------------------------------------------------------------ */
int spk_ctx_create(int device, spk_ctx **out);
void spk_ctx_destroy(spk_ctx *ctx);
/* Run all work on `hip_stream` (a hipStream_t; NULL = the context's own stream). */
int spk_ctx_set_stream(spk_ctx *ctx, void *hip_stream);
int spk_ctx_sync(spk_ctx *ctx);
/* Link type of the loaded tables (needed before spk_pairs_load / spk_gammas when spk_block is not used). */
int spk_ctx_set_link_type(spk_ctx *ctx, int link_type);
/* Elapsed milliseconds of the last launch of each kernel family, measured with HIP events
 * on the context stream: [0] block, [1] gamma, [2] em_hist, [3] em_final, [4] score. */
int spk_ctx_kernel_ms(spk_ctx *ctx, double *out5);
/* The same without synchronising: per family the newest launch that has completed (-1 = none), so a
 * caller can read the timings of iteration i while iteration i + 1 is still queued. */
int spk_ctx_kernel_ms_done(spk_ctx *ctx, double *out5);
/* on = 1: HIP events around each kernel family (spk_ctx_kernel_ms); on = 2: also around each column's exact-pass
 * launch (spk_gammas_exact_ms); 0: off. */
int spk_ctx_enable_timing(spk_ctx *ctx, int on);
/* LDS bytes one workgroup may allocate on the context's device (sizes the E/M histogram copies). */
int spk_ctx_lds_per_block(spk_ctx *ctx, int *out);
/* Device memory the context holds, by what it stores (bytes allocated): [0] raw input columns (Arrow
 * buffers as handed over), [1] record encodings (decoded columns: units, metadata, bit-planes, bag rows,
 * numeric values; row permutations, ranks, blocking keys), [2] filter row images, [3] candidate pairs (row
 * indices, rule-view positions and rows), [4] comparison codes, [5] comparison work lists (filter lists,
 * exact / slow lists, region counts), [6] EM, scoring and tf state, [7] the sum.  For sizing a share of a
 * job against a device's memory (there is no reference counterpart: Spark spills). */
int spk_ctx_memory(spk_ctx *ctx, int64_t *out8);

/* ---- record tables (replaces createOrReplaceTempView of df / df_l / df_r,
 *      blocking.py:209-222, and the vertical concatenation of :70-93) ------------ */
/* side 0 = df (dedupe_only, link_and_dedupe after concatenation) or df_l; side 1 = df_r. */
int spk_table_create(spk_ctx *ctx, int side, int64_t n_rows, int n_cols);
/* String column from Arrow-style UTF-8: offsets[n_rows+1] into data; valid[n_rows] (1 = non-null).
 * Decoded on the device to UTF-16 code units (Jaro-Winkler alphabet) + code-point lengths.
 * value_ids (optional, may be NULL): a dictionary id per row, equal iff the strings are equal, in
 * one id space for side 0 and side 1 (Arrow dictionary encoding), in [0, 2^32) for non-NULL rows.
 * With ids, string equality in comparison programs is one integer compare; without, a hash then
 * a unit compare.  A column holds at most 2^34 UTF-16 units. */
int spk_table_add_utf8(spk_ctx *ctx, int side, int col, const int64_t *offsets, const uint8_t *data,
                       const uint8_t *valid, const int64_t *value_ids);
int spk_table_add_float64(spk_ctx *ctx, int side, int col, const double *values, const uint8_t *valid);
/* Order rank per row for the link-type predicate: dedupe `l.uid < r.uid` (blocking.py:136),
 * link_and_dedupe `(l.src < r.src) or (l.uid < r.uid and same src)` (:139).  Equal rank = equal key.
 * Per-row host arrays (rank, keys) are in INPUT row order; after spk_cluster they are taken through the
 * table's permutation.  A new rank clears the NULL-id layout (declare it again with spk_table_set_rank_null). */
int spk_table_set_rank(spk_ctx *ctx, int side, const int64_t *rank);
/* NULL unique ids (blocking.py:136, :139: `l.uid < r.uid` is NULL, so the pair is dropped, unless
 * `l._source_table < r._source_table` holds).  divisor > 0 declares the rank layout
 * rank = source * divisor + r with r = divisor - 1 for a row whose unique id is NULL; 0 = no NULL ids. */
int spk_table_set_rank_null(spk_ctx *ctx, int side, int64_t divisor);
/* Blocking key ids of rule `rule` for each row (-1 = NULL: the row never matches the rule).
 * which = 0: key of the row as the join's l-side; which = 1: as the r-side. */
int spk_table_set_key(spk_ctx *ctx, int side, int rule, int which, const int64_t *keys);

/* ---- device ingest (replaces the per-row key / value preparation that Spark does inside the
 *      equi-joins of blocking.py:95-160 and the projections of gammas.py:65-89) ----------------
 * Input columns are handed over once as Arrow buffers ("raw" columns, input row order, indexed by
 * `raw`, borrowed for the call).  Everything derived from them is computed on the device. */
int spk_raw_utf8(spk_ctx *ctx, int raw, int64_t n, const int64_t *offsets, const uint8_t *data, const uint8_t *valid);
/* The same from Arrow buffers as they are (zero-copy on the host side): `offsets` (n + 1, any base: a
 * sliced array's first offset may be past 0), `data` the value buffer those offsets index, `validity`
 * the Arrow validity bitmap (LSB first, from bit validity_bit_offset; NULL = no NULLs; offset -1: one byte
 * per row instead, 0 = NULL).  on_device = 1:
 * all three are device pointers (e.g. rows all-gathered from the ranks that uploaded them) and are
 * copied device to device.  Rebasing, validity expansion and the length scan run on the device. */
int spk_raw_utf8_arrow(spk_ctx *ctx, int raw, int64_t n, const int64_t *offsets, const uint8_t *data,
                       const uint8_t *validity, int64_t validity_bit_offset, int on_device);
/* A chunked Arrow column (pyarrow ChunkedArray: one call instead of a host-side combine_chunks copy):
 * chunk c has rows[c] rows, its own offsets (any base), data and validity (bit_offsets[c] as above, -1 for
 * one byte per row; validity[c] NULL = no NULLs).  The chunks' rows are concatenated in order. */
int spk_raw_utf8_arrow_chunks(spk_ctx *ctx, int raw, int n_chunks, const int64_t *rows, const int64_t *const *offsets,
                              const uint8_t *const *data, const uint8_t *const *validity, const int64_t *bit_offsets);
/* 64-bit digest of a table's encoded device form (row permutation, ranks, every comparison column's
 * metadata / bit-planes / values, blocking keys): two contexts that ingested the same rows by
 * different routes (local upload, or rows gathered from other ranks) give the same digest. */
int spk_table_digest(spk_ctx *ctx, int side, uint64_t *out);
/* Free a raw column's device buffers (its keys and decoded columns stay; using it again is SPK_E_STATE
 * until it is uploaded again under the same index). */
int spk_raw_release(spk_ctx *ctx, int raw);
/* 8-byte values compared as bit patterns (int64 ids, canonical float64 bits, host-computed key ids). */
int spk_raw_i64(spk_ctx *ctx, int raw, int64_t n, const int64_t *values, const uint8_t *valid);
/* One equality term of a blocking rule: l-side column `raw_l` (table 0) = r-side column `raw_r` (the
 * r table; -1 = the same column, a symmetric term), each with an optional Spark substr(start, len)
 * on code points (len < 0 = none). */
typedef struct {
    int32_t raw_l, raw_r;
    int32_t l_substr_start, l_substr_len;
    int32_t r_substr_start, r_substr_len;
} spk_key_term;
/* Blocking key of rule `rule` (the conjunction of its terms; NULL if a term is NULL): hash, radix sort
 * and verified dense ids on the device, one id space for both sides.  Same result as
 * spk_table_set_key with host-computed ids (which stays available for other key expressions). */
int spk_key_build(spk_ctx *ctx, int rule, int n_terms, const spk_key_term *terms);
/* Rank for the link predicate from int64 unique ids (raw column, NULL allowed): dense rank, rows
 * [right_from, n) being the 'right' source of link_and_dedupe (-1 = none).  Also sets the NULL-id
 * layout of spk_table_set_rank_null. */
int spk_rank_from_raw(spk_ctx *ctx, int raw_uid, int64_t right_from);
/* Reorder the tables' rows by rule 0's key, then rank (NULL keys last), so a block's rows are
 * contiguous on the device.  Keys and ranks move with the rows; comparison columns must be added
 * after this (they are decoded through the permutation); keys built and ranks set after it follow the
 * table's row order too (calling it again composes the permutations).  out_perm0 / out_perm1 (host,
 * optional): input row of each table row. */
int spk_cluster(spk_ctx *ctx, int32_t *out_perm0, int32_t *out_perm1);
/* String comparison column `col` from raw column raw0 (table 0) and, for link_only, raw1 (table 1):
 * decoded to UTF-16 through the tables' row permutations, with dictionary ids computed on the
 * device in one id space for both sides. */
int spk_table_add_raw_utf8(spk_ctx *ctx, int col, int raw0, int raw1);

/* ---- blocking (replaces block_using_rules / cartesian_block, blocking.py:162-318) -- */
/* Generates candidate pairs for rules 0..n_rules-1 in order, each excluding pairs an earlier
 * rule matched (`AND NOT ifnull(rule_j, false)`, :59-68), with the link-type predicate.
 * rule_symmetric[r] = 1 when the rule's l- and r-side keys are the same function of a row.
 * Pairs are generated for the shard [shard/n_shards] of the global candidate-ordinal space
 * and stay on the device (int32 row indices). */
int spk_block(spk_ctx *ctx, int link_type, int n_rules, const int32_t *rule_symmetric, int shard,
              int n_shards, int64_t *out_n_pairs, int64_t *out_n_candidates_total);
int spk_pairs_count(spk_ctx *ctx, int64_t *out);
int spk_pairs_copy(spk_ctx *ctx, int64_t start, int64_t count, int32_t *out_l, int32_t *out_r);
/* Use caller-provided pairs (e.g. add_gammas on an externally built comparison frame). */
int spk_pairs_load(spk_ctx *ctx, int64_t n, const int32_t *rows_l, const int32_t *rows_r);

/* ---- comparison programs (replaces add_gammas / the CASE templates,
 *      gammas.py:65-124, case_statements.py:62-277) ----------------------------- */
/* Operand of a predicate: a column of the pair's l- or r-record, or a literal, with an
 * optional ifnull() default and an optional substr(start, len) (code points, Spark rules). */
typedef struct {
    int32_t kind;        /* 0 column, 1 string literal, 2 number literal */
    int32_t side;        /* 0 = `_l` record, 1 = `_r` record */
    int32_t col;         /* column index in the side's table */
    int32_t lit;         /* string literal index (kind 1) or ifnull default string (-1 none) */
    double num;          /* number literal (kind 2) or ifnull default number */
    int32_t has_num_default;
    int32_t substr_start; /* 1-based Spark substr position; 0 = no substr */
    int32_t substr_len;
    int32_t pad;
} spk_operand;

/* Predicate instruction (RPN over Kleene booleans). */
#define SPK_OP_ISNULL 1     /* a IS NULL */
#define SPK_OP_NOTNULL 2    /* a IS NOT NULL */
#define SPK_OP_STR_CMP 3    /* a cmp b (strings; = / != / < / <= / > / >=, UTF-8 byte order) */
#define SPK_OP_NUM_CMP 4    /* a cmp b (numbers) */
#define SPK_OP_JW 5         /* jaro_winkler_sim(a, b) cmp t */
#define SPK_OP_LEV 6        /* levenshtein(a, b) cmp t */
#define SPK_OP_LEVRATIO 7   /* levenshtein(a,b)/((length(a)+length(b))/2) cmp t */
#define SPK_OP_ABSDIFF 8    /* abs(a - b) cmp t */
#define SPK_OP_PERCDIFF 9   /* abs(a - b)/abs(case when a > b then a else b end) cmp t */
#define SPK_OP_CONST 10     /* constant: i0 = 0 false, 1 true, 2 null */
#define SPK_OP_AND 20
#define SPK_OP_OR 21
#define SPK_OP_NOT 22
#define SPK_OP_LEN 11       /* length(a) cmp t */

#define SPK_CMP_EQ 0
#define SPK_CMP_NE 1
#define SPK_CMP_LT 2
#define SPK_CMP_LE 3
#define SPK_CMP_GT 4
#define SPK_CMP_GE 5

typedef struct {
    int32_t op;
    int32_t a, b;   /* operand indices */
    int32_t cmp;    /* SPK_CMP_* */
    int32_t i0;
    int32_t pad;
    double t;       /* threshold */
} spk_instr;

typedef struct {
    int32_t n_levels;    /* L_k; gamma values are -1..L_k-1 */
    int32_t else_level;
    int32_t n_when;
    int32_t first_when;  /* index into the when arrays */
} spk_column_program;

/* Install the comparison programs and evaluate them over the current pairs, producing one
 * packed comparison-vector code per pair: code = Σ_k (γ_k + 1) · Π_{j<k} (L_j + 1).
 * Asynchronous: returns once the passes are queued on the context stream.  A work-list overflow
 * or cells past the exact passes' string limit are completed at the next synchronising call that
 * reads the codes (spk_em_iteration, spk_em_finalize, spk_em_histogram with a caller buffer,
 * spk_score, spk_gammas_copy, the tf calls, spk_ctx_sync), so results are always complete. */
int spk_gammas(spk_ctx *ctx, int n_cols, const spk_column_program *cols, int n_when,
               const int32_t *when_first_instr, const int32_t *when_n_instr, const int32_t *when_level,
               int n_instr, const spk_instr *instr, int n_operands, const spk_operand *operands,
               int n_lits, const int64_t *lit_offsets, const uint8_t *lit_utf8);
/* Decode codes to int8 gamma columns, [count x K] row-major. */
int spk_gammas_copy(spk_ctx *ctx, int64_t start, int64_t count, int8_t *out);
/* Use a caller-provided gamma matrix (int8 [n x K], values -1..L_k-1). */
int spk_gammas_load(spk_ctx *ctx, int n_cols, const int32_t *n_levels, int64_t n, const int8_t *gammas);
int spk_n_patterns(spk_ctx *ctx, int64_t *out);
/* Pairs the last spk_gammas evaluated in the global-memory pass (strings beyond LDS staging). */
int spk_gammas_deferred(spk_ctx *ctx, int64_t *out);
/* Per comparison column: pairs the last spk_gammas could not decide from bounds in the filter pass
 * and evaluated with the exact similarity (out[n], n >= number of columns). */
int spk_gammas_exact_counts(spk_ctx *ctx, int64_t *out, int n);
/* With timing on at level 2 (spk_ctx_enable_timing): milliseconds of each column's exact-pass launch in the last
 * spk_gammas (HIP events; -1 = none; the Jaro-Winkler columns share one launch, reported at the first
 * of them).  Synchronises. */
int spk_gammas_exact_ms(spk_ctx *ctx, double *out, int n);
/* Diagnostics: the first n pair ordinals of column k's exact list of the last spk_gammas (host). */
int spk_gammas_exact_list(spk_ctx *ctx, int k, int32_t *out, int64_t n);
/* Per comparison column: pairs of the last spk_gammas whose level the filter took from the blocking
 * key instead of the rows -- a rule built by spk_key_build whose key includes the plain term
 * `l.c = r.c` on the raw columns the column was decoded from (spk_table_add_raw_utf8) emits only
 * pairs with equal, non-NULL values of c (the longest such run of the pair order; 0 when the
 * column holds an empty string, or was not built from raw columns). */
int spk_gammas_implied_pairs(spk_ctx *ctx, int64_t *out, int n);
/* Columns in the shape of the case_statements.py templates (NULL branch, then single-leaf tests
 * on the same two plain operands) are filtered from a packed per-row image of their fields
 * (spk_filter.hip); every other column by the general interpreter.  on = 1 (default): template
 * columns through the filter kernel; on = 0: every column through the interpreter; + 10: the second
 * blocking rule's pairs always read the table-ordered row image, + 20: always their rule's
 * view-ordered copy (default: the copy once the image outgrows the caches); + 100: leave every slow-list
 * launch to the settlement at the next synchronising call (by default only those of columns whose slow
 * lists were empty in the last call with the same pairs, tables and program).  All modes give
 * identical results (for testing).  spk_gammas_simple_count: how many columns the last spk_gammas
 * took as template columns. */
int spk_gammas_set_simple(spk_ctx *ctx, int on);
int spk_gammas_simple_count(spk_ctx *ctx, int *out);
/* Ordinal windows.  The reference joins and projects any number of pairs (blocking.py:95-160,
 * gammas.py:65-89); spk_gammas runs a pair set of more than ~2^31 pairs as consecutive windows of equal
 * size (the exact passes' work lists hold window-relative int32 ordinals), so one context takes any pair
 * count its device memory holds.  spk_gammas_set_window caps the window at `pairs` (0 = default, just under
 * 2^31; smaller windows give identical codes -- for testing); spk_gammas_windows: windows the last
 * spk_gammas ran. */
int spk_gammas_set_window(spk_ctx *ctx, int64_t pairs);
int spk_gammas_windows(spk_ctx *ctx, int64_t *out);
/* Two-stream split (an implementation choice, not a reference interface): with streams = 2 (default), a pair
 * set that fits one window and holds at least min_pairs pairs (default 2^22) runs as two windows of half the
 * pairs at once, the second on a stream of its own joined back before spk_gammas returns, so one window's
 * filter and the other's exact passes share the device.  streams = 1: one window on the context stream.
 * Identical codes either way (spk_gammas_windows reports 2 for a split call). */
int spk_gammas_set_streams(spk_ctx *ctx, int streams, int64_t min_pairs);
/* Graph replay (an implementation choice): a call whose program, pairs, tables, buffers, window layout and
 * slow-list decisions equal the previous call's records the pass's launches as a HIP graph; later such calls
 * (an EM run's iterations) replay it with one launch.  Off by default (on MI355X the replay measured slower than
 * direct launches); on = 0 enqueues every call directly.  Identical codes.
 * spk_gammas_graph_launches: replays so far on this context (diagnostics). */
int spk_gammas_set_graph(spk_ctx *ctx, int on);
int spk_gammas_graph_launches(spk_ctx *ctx, int64_t *out);
/* Levenshtein pass kernels (same codes in every mode; for A/B tests): 2 = lane refill (a lane that finishes its
 * cell takes the next one from its wave's queue) in the exact pass of free-text columns -- rows past 64 units on
 * both sides -- and one cell per lane elsewhere (default), 1 = lane refill in every exact pass (the 128-bit slow
 * pass stays one cell per lane), 0 = one cell per lane everywhere, 3 = as 2 without the character-bag decisions that precede a
 * refill pass over a free-text column (k_compact_lev: cells whose bag distance exceeds the cut take their level
 * there).  Modes 1 and 2 make those decisions too. */
int spk_gammas_set_lev_kernel(spk_ctx *ctx, int mode);
/* Filter regions (workgroups) the last spk_gammas ran over the second rule's view-ordered image. */
int spk_gammas_view_regions(spk_ctx *ctx, int64_t *out);

/* ---- the jar's similarity UDFs as bulk device functions ---------------------------------
 * spk_jaro_winkler_sim replaces uk.gov.moj.dash.linkage.JaroWinklerSimilarity.call(String, String)
 * (commons-text 1.4 JaroWinklerDistance.apply, registered as `jaro_winkler_sim`, tests/test_spark.py:45);
 * spk_levenshtein replaces Spark's levenshtein(l, r) (case_statements.py:121).  n pairs of UTF-8 strings
 * (Arrow offsets, no NULLs), results in out[n] (host).  Same device code as the comparison kernel. */
int spk_jaro_winkler_sim(spk_ctx *ctx, int64_t n, const int64_t *l_offsets, const uint8_t *l_utf8,
                         const int64_t *r_offsets, const uint8_t *r_utf8, double *out);
int spk_levenshtein(spk_ctx *ctx, int64_t n, const int64_t *l_offsets, const uint8_t *l_utf8,
                    const int64_t *r_offsets, const uint8_t *r_utf8, double *out);

/* ---- EM (replaces run_expectation_step + run_maximisation_step's aggregate,
 *      expectation_step.py:25-221, maximisation_step.py:41-90) ------------------ */
/* One EM iteration over this context's pairs in ONE launch: streams every pair's code into the
 * pattern histogram, and the workgroup that finishes last evaluates mp per pattern and the M-step
 * sums.  out_stats / m / u / lambda as spk_em_finalize.  For a single GPU (no exchange). */
int spk_em_iteration(spk_ctx *ctx, double lambda, double one_minus, const double *m, const double *u,
                     double *out_stats, int n_stats);
/* spk_em_iteration in two halves: _start enqueues the launch and the statistics readback (pinned host
 * memory) and returns; _wait returns the statistics.  In between the caller may enqueue the next
 * spk_gammas pass and compute the previous M-step on the host, so the device never waits for the host
 * (the reference's iterate loop, iterate.py:36-56, runs E, M, E, M ...: only the M-step of iteration i
 * must precede the E-step of i + 1).  If the codes the iteration read are corrected after spk_gammas
 * returned (work-list overflow, strings past the exact passes), the iteration is repeated before _wait
 * returns.  One iteration may be pending per context (SPK_E_STATE otherwise). */
int spk_em_iteration_start(spk_ctx *ctx, double lambda, double one_minus, const double *m, const double *u,
                           int n_stats);
int spk_em_iteration_wait(spk_ctx *ctx, double *out_stats, int n_stats);
/* Multi-GPU form of the same iteration: spk_em_histogram streams every pair's code once and writes
 * the pattern histogram (uint64 [n_patterns]) to d_hist, a DEVICE buffer (NULL = context-owned);
 * with a caller buffer it returns once the histogram is final.  Callers sharding pairs over GPUs
 * all-reduce it (exact integer sum), then spk_em_finalize. */
int spk_em_histogram(spk_ctx *ctx, uint64_t *d_hist);
/* Histogram kernel choice (same result): 1 = lane-private LDS counters when the pattern space fits, with an
 * agent-scope release fence before each last-arriver ticket (default: the memory model's own ordering; it
 * measured within 1 us of the unfenced form on MI355X, tools/ab_em_fence.py), 0 = wave-ballot aggregation
 * into one LDS histogram, 2 = as 1 without the fence (relies on gfx950 draining the row atomics before the
 * ticket).  For testing and measurement. */
int spk_em_set_lane_histogram(spk_ctx *ctx, int on);
/* E-step per pattern with the reference's literal arithmetic, then the M-step sums:
 * out_stats (host) = [Σmp, rows, non-null rows, Σ ln(λΠm + (1-λ)Πu), non-null ln rows] + per column k,
 * per level v in -1..L_k-1:
 * [rows, non-null rows, Σmp, Σ(1-mp)].  m/u are flattened [Σ L_k], already quantised as
 * `cast({p:.35f} as double)`; lambda/one_minus are `cast({λ} as double)`/`cast({1-λ} as double)`. */
int spk_em_finalize(spk_ctx *ctx, const uint64_t *d_hist, double lambda, double one_minus, const double *m,
                    const double *u, double *out_stats, int n_stats);
/* The multi-GPU iteration without host synchronisation: spk_em_histogram_async settles the last
 * spk_gammas (so every rank counts final codes and reduces exactly once) and enqueues the histogram into
 * d_hist; the caller enqueues its all-reduce on the context stream (spk_ctx_set_stream); then
 * spk_em_finalize_start enqueues the E-step + M-step sums and the statistics readback, and
 * spk_em_iteration_wait returns them. */
int spk_em_histogram_async(spk_ctx *ctx, uint64_t *d_hist);
int spk_em_finalize_start(spk_ctx *ctx, const uint64_t *d_hist, double lambda, double one_minus, const double *m,
                          const double *u, int n_stats);
/* Final E-step: match_probability per pair (NaN = NULL).  out_mp = host buffer for
 * [start, start+count), or NULL to keep the result on the device only. */
int spk_score(spk_ctx *ctx, double lambda, double one_minus, const double *m, const double *u, int64_t start,
              int64_t count, double *out_mp);

/* ---- term-frequency adjustment (term_frequencies.py:122-168) ------------------- */
/* For value ids of one column (per row, -1 NULL; both sides in one id space) accumulate, over
 * pairs with equal non-null values, Σ mp and count(mp) per value id (n_values slots), after spk_score.
 * The sums are exact and order-free, so they are identical for any run, grid and sharding.  Each value
 * has a scale E_v (spk_tf_scales: ilogb of its largest term + 1, INT32_MIN for none) and is summed in
 * fixed point relative to 2^E_v (20-bit limbs down to 2^(E_v - 260)), so tiny match probabilities keep
 * their relative precision.  Ranks holding shards of the pairs all-reduce the scales with MAX, pass
 * them to the _exact forms, all-reduce the returned accumulators (int64 [n_values x SPK_TF_LIMBS],
 * sum) and convert them with spk_tf_limbs_to_sum; the double forms do all of that for one context. */
#define SPK_TF_LIMBS 14
int spk_tf_accumulate(spk_ctx *ctx, int64_t n_values, const int64_t *ids_side0, const int64_t *ids_side1,
                      double *out_sum, int64_t *out_count);
int spk_tf_scales(spk_ctx *ctx, int64_t n_values, const int64_t *ids_side0, const int64_t *ids_side1,
                  int32_t *out_scale);
int spk_tf_accumulate_exact(spk_ctx *ctx, int64_t n_values, const int64_t *ids_side0, const int64_t *ids_side1,
                            const int32_t *scale, int64_t *out_limbs, int64_t *out_count);
/* Host only (no device): Σ mp per value from (all-reduced) accumulators and their scales. */
int spk_tf_limbs_to_sum(int64_t n_values, const int64_t *limbs, const int32_t *scale, double *out_sum);
/* The same with the value ids taken on the device from a string column's dictionary ids (columns
 * added with spk_table_add_raw_utf8: dense in [0, n_values), one id space for both sides, NULL
 * rows excluded), so no host-side factorisation of the tf column is needed.  spk_tf_column_values
 * gives n_values (SPK_E_STATE for a column without device ids). */
int spk_tf_column_values(spk_ctx *ctx, int col, int64_t *out_n_values);
int spk_tf_accumulate_column(spk_ctx *ctx, int col, int64_t n_values, double *out_sum, int64_t *out_count);
int spk_tf_scales_column(spk_ctx *ctx, int col, int64_t n_values, int32_t *out_scale);
int spk_tf_accumulate_column_exact(spk_ctx *ctx, int col, int64_t n_values, const int32_t *scale,
                                   int64_t *out_limbs, int64_t *out_count);
int spk_tf_apply_columns(spk_ctx *ctx, int n_tf_cols, const int32_t *cols, const double *const *adj_tables,
                         const int64_t *table_sizes, int64_t start, int64_t count, double *out_tf_mp,
                         double *out_adj /* [count x n_tf_cols] or NULL */);
/* tf_adjusted_match_prob = bayes(mp, adj_1, ..., adj_n) (:98-117) with adj_c = table_c[id] for pairs
 * with equal non-null values and 0.5 otherwise.  out (host) [start, start+count); out_tf_mp = NULL keeps
 * the results on the device (as spk_score with out = NULL), read back by range with spk_tf_copy. */
int spk_tf_apply(spk_ctx *ctx, int n_tf_cols, const int64_t *const *ids_side0, const int64_t *const *ids_side1,
                 const double *const *adj_tables, const int64_t *table_sizes, int64_t start, int64_t count,
                 double *out_tf_mp, double *out_adj /* [count x n_tf_cols] or NULL */);
/* Pairs [start, start + count) of the tf_adjusted_match_prob the last spk_tf_apply* call with out_tf_mp = NULL
 * kept on the device (SPK_E_STATE when there is none for the current pair set; the range must lie inside the
 * applied one).  Replaces collecting the reference's tf_adjusted_match_prob column (term_frequencies.py:159-168). */
int spk_tf_copy(spk_ctx *ctx, int64_t start, int64_t count, double *out_tf_mp);
/* How the per-value sums find the (value, pattern) counts: 0 (default) a direct histogram when n_values x
 * n_patterns <= min(2^30, max(4 x pairs, 2^24)), else keys (value x n_patterns + pattern, 32-bit when they fit) + radix sort + run-length
 * encode; 1 always the sort; 2 the sort with 64-bit keys (tests hold the three identical).  No reference
 * counterpart (an implementation choice below term_frequencies.py:49-65). */
int spk_tf_set_mode(spk_ctx *ctx, int mode);

#ifdef __cplusplus
}
#endif
#endif /* SPLINK_HIP_H */
