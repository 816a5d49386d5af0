// Shared helpers for the Robust-NeRF MI355X (gfx950) HIP kernels.
//
// Every extern "C" entry point in this library follows one contract
// (include/nerf_hip.h): it returns 0 on success, a positive hipError_t on a
// runtime failure, or NR_EARG on an argument error, and records a message that
// nr_last_error() returns.  Pointers are caller-owned device pointers; no entry
// point allocates, frees or synchronises, so every launch can be captured into
// a hipGraph.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "nerf_hip.h"

namespace nr {

void set_error(const char* fmt, ...);
void clear_error();

// Launch-and-check helper: returns the hipError_t of the most recent launch.
inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return static_cast<int>(e);
    }
    return NR_OK;
}

#define NR_REQUIRE(cond, ...)                                  \
    do {                                                       \
        if (!(cond)) {                                         \
            ::nr::set_error(__VA_ARGS__);                      \
            return NR_EARG;                                    \
        }                                                      \
    } while (0)

#define NR_LAUNCH_CHECK(what)                                  \
    do {                                                       \
        int _rc = ::nr::check_launch(what);                    \
        if (_rc) return _rc;                                   \
    } while (0)

constexpr int kWave = 64;

__host__ __device__ inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ inline long long ceil_div_ll(long long a, long long b) { return (a + b - 1) / b; }

__device__ __forceinline__ float norm3(float x, float y, float z) { return sqrtf(x * x + y * y + z * z); }

// Grid for a grid-stride memory-bound kernel (cdna_hip_programming.md G11).
inline int stream_grid(long long work, int block) {
    long long g = ceil_div_ll(work, block);
    if (g > 2048) g = 2048;
    if (g < 1) g = 1;
    return static_cast<int>(g);
}

}  // namespace nr
