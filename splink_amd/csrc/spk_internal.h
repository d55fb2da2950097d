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
// String columns keep the UTF-16 code units of every row at the row's UTF-8 byte offset
// (UTF-16 never needs more units than UTF-8 has bytes), so no scan is needed on upload.
enum ColKind : int32_t { COL_NONE = 0, COL_STR = 1, COL_NUM = 2 };

struct ColDesc {
    int32_t kind;
    int32_t pad;
    const uint16_t *units;  // COL_STR
    const int64_t *off;     // row start (in units)
    const int32_t *len16;   // UTF-16 length, -1 = NULL
    const int32_t *cplen;   // code-point length
    const uint64_t *hash;   // FNV-1a over the units (inequality fast path)
    const double *val;      // COL_NUM
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
    DevBuf<int64_t> off;
    DevBuf<int32_t> len16, cplen;
    DevBuf<uint64_t> hash;
    DevBuf<double> val;
    DevBuf<uint8_t> valid;
};

struct Table {
    int64_t n = -1;
    std::vector<Column *> cols;
    DevBuf<ColDesc> d_desc;
    bool desc_dirty = true;
    DevBuf<int64_t> rank;
    std::vector<DevBuf<int64_t> *> key[2];  // [which][rule]
    ~Table();
};

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

    // packed comparison-vector codes
    spk::DevBuf<uint8_t> codes;
    int code_bytes = 2;
    int K = 0;
    std::vector<int32_t> n_levels;
    std::vector<int64_t> stride;
    int64_t n_patterns = 0;
    bool codes_valid = false;
    int64_t last_deferred = 0;

    // EM state
    spk::DevBuf<uint64_t> hist;
    spk::DevBuf<double> mpat, llpat, stats, mu;
    spk::DevBuf<double> mp;  // per-pair scores (final E-step)
    bool mpat_valid = false;

    // timing
    bool timing = false;
    hipEvent_t ev0[spk::K_COUNT] = {}, ev1[spk::K_COUNT] = {};
    bool ev_used[spk::K_COUNT] = {};

    int begin(spk::Kern k);
    int end(spk::Kern k);
    spk::Table &side_table(int operand_side) { return table[(operand_side == 1 && link_type == SPK_LINK_ONLY) ? 1 : 0]; }
};

namespace spk {
int ensure_desc(spk_ctx *ctx, Table &t);
}
