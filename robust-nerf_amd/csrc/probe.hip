// Diagnostic entry point: runs ONE MFMA tile so host tests can check the lane
// maps of mfma.hpp on real hardware (asymmetric A and B, full tile compare).
#include "common.hpp"
#include "mfma.hpp"

namespace nr {

// kind 0: bf16 32x32x16 (A 32x16, B 16x32); kind 1: f32 32x32x2 (A 32x2, B 2x32).
// D is written row-major 32x32.  One wave.
__global__ void probe_mfma_kernel(int kind, const float* A, const float* B, float* D) {
    const int l = threadIdx.x;
    const bool raw = kind >= 2;
    kind &= 1;
    const int r = l & 31, h = l >> 5;
    f32x16 acc;
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    if (kind == 0) {
        bf16x8 a, b;
        for (int j = 0; j < 8; ++j) {
            a[j] = to_bf16(A[r * 16 + 8 * h + j]);
            b[j] = to_bf16(B[(8 * h + j) * 32 + r]);
        }
        acc = mfma_bf16(a, b, acc);
    } else {
        acc = mfma_f32(A[r * 2 + h], B[h * 32 + r], acc);
    }
    if (raw) {
        for (int reg = 0; reg < 16; ++reg) D[l * 16 + reg] = acc[reg];
    } else {
        for (int reg = 0; reg < 16; ++reg) D[acc_row(reg, h) * 32 + r] = acc[reg];
    }
}

}  // namespace nr

extern "C" int nr_probe_mfma(int kind, const float* A, const float* B, float* D,
                             nr_stream_t stream) {
    NR_REQUIRE(A && B && D && (kind >= 0 && kind <= 3), "nr_probe_mfma: bad arguments");
    hipLaunchKernelGGL(nr::probe_mfma_kernel, dim3(1), dim3(64), 0,
                       static_cast<hipStream_t>(stream), kind, A, B, D);
    NR_LAUNCH_CHECK("nr_probe_mfma");
    return NR_OK;
}
