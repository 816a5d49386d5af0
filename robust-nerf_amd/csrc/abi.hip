// Library-level entry points: error reporting, version and the toolchain probe.
#include <cstdarg>

#include "common.hpp"

namespace nr {

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

void clear_error() { g_last_error[0] = '\0'; }

__global__ void probe_fill_kernel(float* out, int n, float value) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = value + static_cast<float>(i);
}

}  // namespace nr

extern "C" {

const char* nr_last_error(void) { return nr::g_last_error; }

int nr_abi_version(void) { return 5; }

int nr_probe_fill(float* out, int n, float value, nr_stream_t stream) {
    NR_REQUIRE(out != nullptr && n >= 0, "nr_probe_fill: bad arguments");
    if (n == 0) return NR_OK;
    hipLaunchKernelGGL(nr::probe_fill_kernel, dim3(nr::ceil_div(n, 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), out, n, value);
    NR_LAUNCH_CHECK("nr_probe_fill");
    return NR_OK;
}

}  // extern "C"
