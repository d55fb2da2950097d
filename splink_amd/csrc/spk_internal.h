// Internal definitions shared by the libsplink_hip.so translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/splink_hip.h"

namespace spk {

// ---- error plumbing -------------------------------------------------------------------
void set_error(const std::string &msg);

#define SPK_HIP(expr)                                                                         \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            ::spk::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));              \
            return _e == hipErrorOutOfMemory ? SPK_E_OOM : SPK_E_HIP;                         \
        }                                                                                     \
    } while (0)

#define SPK_REQUIRE(cond, code, msg)                                                          \
    do {                                                                                      \
        if (!(cond)) {                                                                        \
            ::spk::set_error(msg);                                                            \
            return code;                                                                      \
        }                                                                                     \
    } while (0)

#define SPK_TRY(expr)                                                                         \
    do {                                                                                      \
        int _r = (expr);                                                                      \
        if (_r != SPK_OK) return _r;                                                          \
    } while (0)

// ---- device column layout ---------------------------------------------------------------
// String columns keep the UTF-16 code units of row i at a 4-unit (8-byte) aligned start derived
// from its UTF-8 byte offset, (off8[i] + 3i + 3) & ~3: UTF-16 never needs more units than UTF-8
// has bytes, so the starts are monotone, rows never overlap and no scan is needed on upload.
// Each row also has a 32-byte metadata record (two 16-byte loads) that holds everything the
// comparison filter needs -- NULL flag, lengths, equality key, sketch and the first four units --
// so most (pair, column) cells are decided without touching the units at all.
enum ColKind : int32_t { COL_NONE = 0, COL_STR = 1, COL_NUM = 2 };

struct alignas(16) RecMeta {
    uint32_t key;     // dictionary id of the value (CPF_ID: equal iff the strings are) or a 32-bit
                      // FNV-1a fold of the units (unequal keys prove unequal strings)
    int32_t len16;    // UTF-16 length, -1 = NULL
    uint64_t sketch;  // unit sketch (sketch_bucket / sketch_add)
    uint64_t head;    // units 0..3, zero beyond len16
    uint32_t off4;    // first UTF-16 unit of the row / 4 (rows start 8-byte aligned)
    uint32_t cpf;     // bits 0..23: code-point length; bit 24: bit-planes valid (<= 64 units, all < 256);
                      // bit 25: `key` is an exact dictionary id; bit 26: two-word bit-planes valid
                      // (65..128 units, all < 256: units 0..63 in planes, 64..127 in planes_hi)
};
static_assert(sizeof(RecMeta) == 32, "RecMeta layout");
constexpr uint32_t CPF_PLANES = 1u << 24;
constexpr uint32_t CPF_ID = 1u << 25;
constexpr uint32_t CPF_PLANES2 = 1u << 26;
constexpr int PLANES2_MAX = 128;  // longest row with two-word planes
__host__ __device__ inline int32_t meta_cplen(const RecMeta &m) { return (int32_t)(m.cpf & 0xFFFFFFu); }
__host__ __device__ inline int64_t meta_off(const RecMeta &m) { return (int64_t)m.off4 * 4; }

// Bit-planes of a row whose units are all < 256 and that has <= 64 units: plane b (0..7) holds
// bit b of unit i at bit i.  The Levenshtein / Jaro-Winkler match masks of a character c are then
// AND_b (bit b of c ? plane_b : ~plane_b), eight register ops instead of a scan of the string.
constexpr int N_PLANES = 8;

// Unit sketch: 32 buckets of saturating 2-bit unit counts (0, 1, 2, >=3) held as two bit-planes,
// bits 0..31 the low count bit and bits 32..63 the high count bit of each bucket.  ASCII letters
// get a bucket each (case folded), digits three, other ASCII three; other units are hashed.
// Merging units into a bucket only raises the per-bucket minima, so the multiset-intersection
// bound derived from two sketches (sketch_inter_ub) holds for any bucket map.
__host__ __device__ inline uint32_t sketch_bucket(uint32_t u) {
    if (u < 128u) {
        if (u >= 'a' && u <= 'z') return u - 'a';
        if (u >= 'A' && u <= 'Z') return u - 'A';
        if (u >= '0' && u <= '9') return 26u + (u - '0') % 3u;
        return 29u + u % 3u;
    }
    return ((u * 2654435761u) >> 16) & 31u;
}

__host__ __device__ inline void sketch_add(uint64_t &sk, uint32_t unit) {
    const uint32_t b = sketch_bucket(unit);
    const uint64_t lo = 1ull << b, hi = 1ull << (32 + b);
    if ((sk & lo) && (sk & hi)) return;  // saturated at 3
    if (sk & lo) sk = (sk & ~lo) | hi;   // 1 -> 2
    else sk |= lo;                       // 0 -> 1, 2 -> 3
}

struct ColDesc {
    int32_t kind;
    int32_t pad;
    const uint16_t *units;   // COL_STR
    const RecMeta *meta;     // COL_STR
    const uint64_t *planes;  // COL_STR, [n][N_PLANES]
    const uint64_t *planes_hi;  // COL_STR, [n][N_PLANES] units 64..127 (CPF_PLANES2 rows), or null
    const uint4 *bag;        // COL_STR: [n][2] character-bag rows (k_bag_rows), or null (not built)
    const double *val;       // COL_NUM
    const uint8_t *valid;   // COL_NUM
};

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    int alloc(size_t count) {
        if (count <= n && p) return SPK_OK;
        release();
        if (count == 0) return SPK_OK;
        hipError_t e = hipMalloc(&p, count * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            set_error(std::string("hipMalloc failed: ") + hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SPK_E_OOM : SPK_E_HIP;
        }
        n = count;
        return SPK_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DevBuf() { release(); }
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
};

struct Column {
    ColKind kind = COL_NONE;
    DevBuf<uint16_t> units;
    int64_t units_len = 0;  // units written by the last decode (zeroed first); the buffer may be larger (reused)
    DevBuf<RecMeta> meta;
    DevBuf<uint64_t> planes;
    DevBuf<uint64_t> planes_hi;  // allocated only when some row has more than 64 UTF-8 bytes
    DevBuf<uint4> bag;           // 32-byte character-bag row per row (k_bag_rows; built when a Levenshtein
                                 // comparison reads the column)
    DevBuf<double> val;
    DevBuf<uint8_t> valid;
    bool has_ids = false;  // COL_STR: RecMeta.key is a dictionary id
    int64_t max_bytes = 0; // COL_STR: longest row in UTF-8 bytes (>= its UTF-16 units)
    uint64_t src[2] = {0, 0};  // spk_table_add_raw_utf8: serials of the raw columns of the l / r side (0: other)
    bool has_empty = false;    // some non-NULL row is the empty string
    int64_t n_ids = -1;        // spk_table_add_raw_utf8: distinct non-NULL values (ids are dense in [0, n_ids))
    // OR / AND of the units of every row that has bit-planes (bits 0..7), set by launch_unit_bits
    bool unit_bits = false;
    uint32_t unit_or = 0, unit_and = 0xFFu;
};

// A blocking-key term as spk_key_build saw it, by raw-column serial: the comparison filter skips a
// string column for the pairs of a rule whose key includes `l.c = r.c` on that column's own raw
// columns (the strings are then equal and non-NULL; see spk_gammas).
struct KeyTerm {
    uint64_t src_l = 0, src_r = 0;
    bool plain = false;  // no substr on either side
};

// An input column as handed over (Arrow buffers), kept on the device in input row order: the source
// of blocking keys, dictionary ids and (through a table's row permutation) comparison columns.
enum RawKind : int32_t { RAW_UTF8 = 1, RAW_I64 = 2 };
struct RawCol {
    RawKind kind = RAW_UTF8;
    uint64_t serial = 0;     // ctx-wide upload counter (a replaced raw column gets a new one)
    bool has_empty = false;  // RAW_UTF8: some non-NULL value is the empty string
    int64_t n = 0;
    int64_t max_len = 0;     // longest value in bytes (UTF-8)
    DevBuf<int64_t> off;     // RAW_UTF8: n + 1 byte offsets
    DevBuf<uint8_t> bytes;   // RAW_UTF8
    DevBuf<int64_t> i64;     // RAW_I64: values (compared as 8-byte patterns)
    DevBuf<uint8_t> valid;   // 1 = non-NULL
    bool released = false;   // spk_raw_release: buffers freed, serial kept
};

struct Table {
    int64_t n = -1;
    DevBuf<int32_t> perm;    // row i of the table is input row perm[i] (spk_cluster); empty = identity
    std::vector<Column *> cols;
    DevBuf<ColDesc> d_desc;
    bool desc_dirty = true;
    uint64_t version = 0;  // bumped (ctx-wide counter) whenever the table or one of its columns is replaced
    DevBuf<int64_t> rank;
    int64_t null_div = 0;  // rank layout for NULL unique ids (spk_table_set_rank_null), 0 = none
    std::vector<DevBuf<int64_t> *> key[2];  // [which][rule]
    ~Table();
};

template <typename T>
inline void take_buf(DevBuf<T> &dst, DevBuf<T> &src) {  // move src's allocation into dst
    dst.release();
    dst.p = src.p;
    dst.n = src.n;
    src.p = nullptr;
    src.n = 0;
}

// Blocking rule r >= 1 as its own row order ("view"): the rows with a non-NULL key r sorted by
// (key r, rank), so a block of rule r is contiguous in it.  Pairs of rule r also carry their view
// positions (spk_ctx::pvl / pvr), and the comparison filter reads a copy of the row image laid out
// in view order: the pairs of a later rule then touch a block's rows in a few cache lines, as the
// first rule's pairs do in the table (clustered by rule 0) itself.
constexpr int MAX_VIEWS = 2;  // rules 1 .. MAX_VIEWS - 1 get views (one: registers of the filter)
struct RuleView {
    DevBuf<int32_t> rowsL, rowsR;  // view position -> table row (l side; r side unless tri)
    int64_t nL = 0, nR = 0;
    bool tri = true;               // symmetric self-join: both sides index rowsL
    int64_t pair_lo = 0, pair_hi = 0;  // this rule's pair ordinals (local shard)
};

struct GammaPlan;
enum Kern { K_BLOCK = 0, K_GAMMA = 1, K_EMHIST = 2, K_EMFIN = 3, K_SCORE = 4, K_COUNT = 5 };

}  // namespace spk

struct spk_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    spk::Table table[2];
    int link_type = SPK_LINK_DEDUPE;

    // candidate pairs (row indices into table 0 / table side_r)
    spk::DevBuf<int32_t> pl, pr;
    int64_t n_pairs = 0;
    bool pairs_valid = false;
    uint64_t pairs_epoch = 0;          // bumped whenever the pair set is replaced
    std::vector<spk::KeyTerm> rule_terms[32];   // spk_key_build terms per rule (cleared by spk_table_set_key)
    std::vector<std::vector<spk::KeyTerm>> pair_terms;  // the terms of each rule of the current pair set
    std::vector<int64_t> pair_rule_lo, pair_rule_hi;   // local pair ordinals of each rule (spk_block)
    uint64_t raw_serial = 0;
    spk::RuleView views[spk::MAX_VIEWS];  // views[r] for rules 1 .. n_views
    int n_views = 0;
    spk::DevBuf<int32_t> pvl, pvr;     // view positions of pairs [pv_base, n_pairs)
    int64_t pv_base = 0;

    // packed comparison-vector codes
    spk::DevBuf<uint8_t> codes;
    int code_bytes = 2;
    int K = 0;
    std::vector<int32_t> n_levels;
    std::vector<int64_t> stride;
    int64_t n_patterns = 0;
    bool codes_valid = false;
    int64_t last_deferred = 0;
    std::vector<int64_t> last_exact;  // per column: pairs the last spk_gammas evaluated exactly
    std::vector<int64_t> last_xbase;  // per column: start of its exact list in xlist (diagnostics)
    std::vector<int64_t> last_implied;  // per column: pairs whose level the blocking key implied
    int filter_mode = 1;              // 1: template-shaped columns through the filter kernel (spk_filter.hip),
                                      // 0: every column through the interpreter (spk_gammas_set_simple)
    int use_views = 1;                // rule 1's pairs read a view-ordered row image: 0 never, 1 when the
                                      // image outgrows the caches, 2 always (tests)
    int64_t last_view_regions = 0;    // filter regions the last spk_gammas ran as a view launch
    int last_simple = 0;
    // ordinal windows: spk_gammas runs the filter / exact / slow passes over windows of at most this many
    // pairs (0: the default, just under 2^31 -- the work lists hold window-relative int32 ordinals); each
    // window but the last is settled before the next one reuses the lists
    int64_t gamma_window = 0;
    int64_t last_windows = 0;             // windows the last spk_gammas ran
    std::vector<int64_t> exact_carry;     // exact-pass cells of the windows settled before the last one
    int64_t deferred_carry = 0;           // their slow-list cells

    // comparison-vector work buffers (reused across calls)
    spk::DevBuf<int32_t> work;
    spk::DevBuf<int32_t> xlist;       // [2 x xcap]: compacted exact-pass lists, column after column | slow lists
    spk::DevBuf<int64_t> xpref;       // [K][regions + 1] offsets of each region's list in its column's list
    spk::DevBuf<int64_t> xinfo;       // [col_base K | col_count K | overflow | total] (k_prefix)
    int64_t xcap = 0;
    int64_t *h_info = nullptr;        // pinned readback of xinfo + slow counts
    size_t h_info_n = 0;
    int pinned_info(size_t n) {
        if (n <= h_info_n) return SPK_OK;
        if (h_info) (void)hipHostFree(h_info);
        h_info = nullptr;
        h_info_n = 0;
        if (hipHostMalloc(reinterpret_cast<void **>(&h_info), n * 8, hipHostMallocDefault) != hipSuccess) {
            h_info = nullptr;
            spk::set_error("hipHostMalloc failed");
            return SPK_E_OOM;
        }
        h_info_n = n;
        return SPK_OK;
    }
    spk::DevBuf<uint8_t> img[2];      // filter row images of table 0 / table 1
    std::vector<int64_t> img_key[2];  // what img[s] was built from: table version, rows, column layout
    spk::DevBuf<uint8_t> vimg[spk::MAX_VIEWS][2];  // row images in rule-view order (views[r])
    std::vector<int64_t> vimg_key[spk::MAX_VIEWS][2];
    uint64_t table_epoch = 0;
    spk::DevBuf<uint8_t> prog_blob;   // comparison programs, literals, strides (uploaded when they change)
    std::vector<uint8_t> last_blob;   // host copy of what prog_blob holds
    // the last spk_gammas: the plan its exact / huge passes ran with, and whether its info block still
    // has to be read (settle_gammas, at the next synchronisation of a consumer)
    spk::GammaPlan *gplan = nullptr;
    void (*gplan_free)(spk::GammaPlan *) = nullptr;
    bool gamma_pending = false;
    // per column: whether the last settled spk_gammas found cells on its slow list; with the same pairs,
    // tables and program the next call does not launch the slow-list kernels of columns that had none
    // (settle_gammas runs them if the list is not empty after all)
    std::vector<uint8_t> slow_seen;
    bool slow_seen_valid = false;
    bool lev_bag = true;           // k_compact_lev's bag-distance decisions before a refill pass (mode 3: off)
    int lev_kernel = 2;            // Levenshtein exact pass: 0 k_gamma_exact_simple<X_LEV>, 1 k_lev_refill, 2 refill in
                                   // free-text columns (rows past 64 units), one cell per lane elsewhere
    bool slow_force_skip = false;  // tests: leave every slow-list launch to settle_gammas
    uint64_t slow_key_pairs = 0, slow_key_tables = 0;
    spk::DevBuf<unsigned int> region_count;  // [K][regions] filter work-list lengths

    // Two-stream split (spk_gammas_set_streams): a pair set that fits one ordinal window but holds at least
    // split_min pairs runs as two windows at once, window 0 on `stream`, window 1 on alt.stream, so one
    // window's filter (texture-address bound) shares the CUs with the other's exact passes (VALU bound).  `alt`
    // is a second set of the per-window state; swap_slot() exchanges it with the members above, so the phase,
    // slow-list and settle functions run unchanged on either window.
    struct Slot {
        spk::DevBuf<int32_t> work, xlist;
        spk::DevBuf<int64_t> xpref, xinfo;
        spk::DevBuf<unsigned int> region_count;
        int64_t xcap = 0;
        int64_t *h_info = nullptr;
        size_t h_info_n = 0;
        hipEvent_t ev_info = nullptr;
        spk::GammaPlan *gplan = nullptr;
        bool gamma_pending = false;
        hipStream_t stream = nullptr;
        std::vector<hipEvent_t> xev0, xev1;
        std::vector<char> xev_used;
    } alt;
    int gamma_streams = 2;
    int64_t split_min = (int64_t)1 << 22;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    bool split_ready = false;  // alt.stream and the events exist
    // The pass's launches as a captured HIP graph (spk_gammas_set_graph, off by default): a call whose key -- program,
    // pairs, tables, buffers, window layout, slow-list decisions -- equals the previous call's is captured, later
    // calls with that key replay it (one launch instead of ~25 API calls).  Measured slower than direct launches
    // on MI355X (cfg2 0.939 -> 0.954 ms per step, profiles/r6_ab_gamma_graph.log), so it is opt-in.
    bool use_graph = false;
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    std::vector<int64_t> gkey, gkey_prev;
    std::vector<char> gskip0, gskip1;  // the slots' slow_skipped at capture
    int64_t gview_regions = 0;
    int64_t graph_launches = 0;        // replays so far (diagnostics)
    bool last_split = false;   // the last spk_gammas ran split: window 1 = pairs [split_w, P)
    int64_t split_w = 0;
    std::vector<int64_t> split_first, alt_xbase;  // per column: window 0's exact cells; window 1's list base
    void swap_slot();

    // EM state
    spk::DevBuf<uint64_t> hist;
    spk::DevBuf<double> mpat, llpat, cpat, stats, mu;  // per pattern: mp, ln(...), count; statistics; m / u
    spk::DevBuf<unsigned int> em_ticket;  // k_em_iter's last-workgroup ticket (kept zero between launches)
    spk::DevBuf<uint32_t> em_row;         // its reduction rows (kept zero between launches)
    spk::DevBuf<int32_t> em_hot;          // the pattern it does not count with R < 64 lane copies (-1: none yet)
    std::vector<int64_t> em_hot_key;      // the pair set / pattern space it was found for
    double *h_stats = nullptr;        // pinned host copy of the statistics vector
    size_t h_stats_n = 0;
    int n_cu = 256;                   // compute units of the device (grid sizing)
    int lds_per_block = 64 * 1024;    // LDS a workgroup may allocate (device attribute)
    int pinned_stats(size_t n) {
        if (n <= h_stats_n) return SPK_OK;
        if (h_stats) (void)hipHostFree(h_stats);
        h_stats = nullptr;
        h_stats_n = 0;
        if (hipHostMalloc(reinterpret_cast<void **>(&h_stats), n * 8, hipHostMallocDefault) != hipSuccess) {
            h_stats = nullptr;
            spk::set_error("hipHostMalloc failed");
            return SPK_E_OOM;
        }
        h_stats_n = n;
        return SPK_OK;
    }
    spk::DevBuf<double> mp;  // per-pair scores (final E-step)
    // tf_adjusted_match_prob kept on the device (spk_tf_apply* with out_tf_mp = NULL): pairs [tf_start, tf_start +
    // tf_count) of the pair set tf_epoch (pairs_epoch then); read back by range with spk_tf_copy
    spk::DevBuf<double> tf_mp;
    int64_t tf_start = 0, tf_count = -1;
    uint64_t tf_epoch = 0;
    // mp per pattern of the last spk_score (the tf sums read it): a table of its own, since every EM
    // launch rewrites mpat with its iteration's parameters
    spk::DevBuf<double> mpat_score;
    std::vector<spk::RawCol *> raw;  // device copies of the input columns (spk_raw_*)
    ~spk_ctx() {
        for (spk::RawCol *r : raw) delete r;
        if (gplan && gplan_free) gplan_free(gplan);
        if (alt.gplan && gplan_free) gplan_free(alt.gplan);
    }
    bool mpat_valid = false;  // mpat_score holds the mp per pattern of the current codes' last spk_score
    uint64_t score_seq = 0;   // spk_score calls so far (the tf runs depend on their mp per pattern)
    // the (value, pattern) runs of the last tf scale pass over a device-id column, reused by its sum pass
    spk::DevBuf<unsigned long long> tf_uniq;
    spk::DevBuf<unsigned int> tf_runs, tf_nruns;
    // or, when n_values x n_patterns is small enough, the (value, pattern) pair counts themselves (tf_pass)
    spk::DevBuf<unsigned long long> tf_hist;
    spk::DevBuf<uint8_t> tf_sort;  // the sort form's keys, sorted keys and sort scratch (scale pass to sum pass)
    std::vector<int64_t> tf_key;
    int tf_mode = 0;  // spk_tf_set_mode: 0 auto (histogram when it fits), 1 always the sort, 2 the sort with 64-bit keys
    bool hist_lanes = true;  // k_hist_lanes (lane-private LDS counters) when the pattern space fits
    bool em_fence = true;    // k_em_iter: release fence before each ticket (spk_em_set_lane_histogram 2: none)

    // asynchronous EM iteration (spk_em_iteration_start / _wait): the statistics land in h_stats behind
    // ev_stats; the arguments are kept so that the launch can be repeated when the codes it read are
    // corrected after spk_gammas returned (settle_gammas -> em_requeue)
    bool em_pending = false;
    uint64_t gamma_seq = 0;           // spk_gammas calls so far (the codes' generation)
    uint64_t em_seq = 0;              // the generation the pending EM iteration read
    double em_lambda = 0.0, em_one_minus = 0.0;
    std::vector<double> em_m, em_u;
    int em_n_stats = 0;
    int em_kind = 0;                  // 0: one-launch iteration (re-enqueued on a code fix), 1: finalize of a
                                      // caller's (all-reduced) histogram, whose codes were settled before
    hipEvent_t ev_info = nullptr;     // after spk_gammas' info-block readback
    hipEvent_t ev_stats = nullptr;    // after the EM statistics readback

    // timing: two event pairs per kind, alternating, so the last completed launch of a kind can be read
    // while a newer one is still in flight (spk_ctx_kernel_ms_done)
    bool timing = false;
    bool timing_exact = false;  // also each column's exact-pass launch (spk_ctx_enable_timing 2): events cost host time per launch
    hipEvent_t ev0[2][spk::K_COUNT] = {}, ev1[2][spk::K_COUNT] = {};
    bool ev_used[2][spk::K_COUNT] = {};
    int ev_slot[spk::K_COUNT] = {};

    // per comparison column: HIP events around its exact-pass launch in the last spk_gammas (timing on;
    // the fused Jaro-Winkler launch is shared by its columns)
    std::vector<hipEvent_t> xev0, xev1;
    std::vector<char> xev_used;
    int xbegin(int k);
    int xend(int k);

    int begin(spk::Kern k);
    int end(spk::Kern k);
    spk::Table &side_table(int operand_side) { return table[(operand_side == 1 && link_type == SPK_LINK_ONLY) ? 1 : 0]; }
};

namespace spk {
int ensure_desc(spk_ctx *ctx, Table &t);
// Finishes the last spk_gammas (work-list overflow, huge pass) once the stream is synchronised;
// *fixed = true when codes changed after spk_gammas returned.  No-op when nothing is pending.
int settle_gammas(spk_ctx *ctx, bool *fixed);
// Enqueue the pending asynchronous EM iteration again (its codes were corrected after it was enqueued).
int em_requeue(spk_ctx *ctx);
int new_column(spk_ctx *ctx, int side, int col, Column **out);
int launch_unit_bits(spk_ctx *ctx, int64_t n, Column *c);
int build_bag_rows(spk_ctx *ctx, int64_t n, Column *c);
int launch_utf8_decode(spk_ctx *ctx, int64_t n, const int64_t *off8, const int64_t *src_off, const int32_t *perm,
                       const uint8_t *bytes, const uint8_t *valid, Column *c, bool long_rows, const int64_t *ids);
}
