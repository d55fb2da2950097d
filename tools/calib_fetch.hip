// Calibration of rocprofv3's FETCH_SIZE for the access shapes of the comparison pass (run under
// `rocprofv3 --pmc FETCH_SIZE --kernel-trace`; tools/traffic.py reads the dispatches by name).
//
//   k_stream16   : every byte of a 2 GiB buffer once, 16 B per lane, coalesced (the guide's case:
//                  FETCH_SIZE = half the bytes on gfx950)
//   k_gather16   : 32M lanes, each one 16-byte load from a distinct random 128-byte line of the buffer
//   k_gather8    : the same with 8-byte loads
//   k_gather4    : the same with 4-byte loads
// The buffer (2 GiB) is far larger than the 256 MB Infinity Cache and the L2s, and lines are not
// revisited, so each gather fetches its line from HBM once: FETCH_SIZE / (32M x 128 B) is the factor
// that turns the counter into bytes for scattered loads.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/calib_fetch tools/calib_fetch.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void k_stream16(const uint4 *__restrict__ a, int64_t n, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

template <typename T>
__global__ void k_gather(const uint8_t *__restrict__ a, const uint32_t *__restrict__ line, int64_t n,
                         uint32_t *__restrict__ sink) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const T v = *reinterpret_cast<const T *>(a + (uint64_t)line[i] * 128);
    uint32_t acc;
    if constexpr (sizeof(T) == 16) acc = v.x ^ v.y ^ v.z ^ v.w;
    else if constexpr (sizeof(T) == 8) acc = (uint32_t)v ^ (uint32_t)(v >> 32);
    else acc = v;
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void k_lines(uint32_t *line, int64_t n, uint32_t n_lines) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // a permutation of distinct lines: odd multiplier modulo a power of two
    line[i] = (uint32_t)(((uint64_t)i * 2654435761ull + 12345ull) & (n_lines - 1));
}

int main() {
    const size_t bytes = (size_t)2 << 30;           // 2 GiB
    const uint32_t n_lines = (uint32_t)(bytes / 128);  // 16M lines
    const int64_t n_gather = n_lines;                 // every line once
    uint8_t *a;
    uint32_t *line, *sink;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&line, n_gather * 4) != hipSuccess ||
        hipMalloc(&sink, 4) != hipSuccess) {
        std::printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(a, 1, bytes);
    k_lines<<<(unsigned)((n_gather + 255) / 256), 256>>>(line, n_gather, n_lines);
    (void)hipDeviceSynchronize();
    for (int rep = 0; rep < 2; ++rep) {
        k_stream16<<<8192, 256>>>(reinterpret_cast<const uint4 *>(a), (int64_t)(bytes / 16), sink);
        k_gather<uint4><<<(unsigned)((n_gather + 255) / 256), 256>>>(a, line, n_gather, sink);
        k_gather<uint64_t><<<(unsigned)((n_gather + 255) / 256), 256>>>(a, line, n_gather, sink);
        k_gather<uint32_t><<<(unsigned)((n_gather + 255) / 256), 256>>>(a, line, n_gather, sink);
        (void)hipDeviceSynchronize();
    }
    std::printf("stream bytes %zu, gathers %lld (one per 128-byte line)\n", bytes, (long long)n_gather);
    (void)hipFree(a);
    (void)hipFree(line);
    (void)hipFree(sink);
    return 0;
}
