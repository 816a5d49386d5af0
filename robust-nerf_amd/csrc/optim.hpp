// Device helpers of the optimizer tail shared by optim.hip (clip, Adam) and the fused
// step in mlp.hip (Adam that also refreshes the packed MFMA images).
#pragma once

#include "common.hpp"

namespace nr {

constexpr int kSumsqBlocks = 256;
constexpr int kSumsqThreads = 256;
static_assert(kSumsqBlocks == kSumsqThreads, "the final pass reads one partial per thread");
constexpr int kMaxAdamSpans = 8;

// Sum of a block's values in a fixed order: wave butterfly, then waves in index order.
// Every thread of the (kSumsqThreads-wide) block must call it.
__device__ __forceinline__ float block_sum_fixed(float s) {
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    __shared__ float part[kSumsqThreads / 64];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    float t = 0.f;
    for (int i = 0; i < kSumsqThreads / 64; ++i) t += part[i];
    return t;
}

// block_sum_fixed over kSumsqThreads values x[0..), computed by ONE wave without LDS or a
// barrier: lane l folds x[64 w + l] through the same xor tree per w, then the four wave
// sums in the same order -- the identical float result in every wave of every block
__device__ __forceinline__ float wave_sum_fixed(const float* __restrict__ x) {
    static_assert(kSumsqThreads == 256, "four waves' worth of values");
    const int l = threadIdx.x & 63;
    float r[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) r[w] = x[64 * w + l];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int w = 0; w < 4; ++w) r[w] += __shfl_xor(r[w], off);
    return ((r[0] + r[1]) + r[2]) + r[3];
}

// clip_grad_norm_ coefficient from a squared norm (train.py:115)
__device__ __forceinline__ float clip_coef(float sumsq, float max_norm) {
    const float c = max_norm / (sqrtf(sumsq) + 1e-6f);
    return c < 1.0f ? c : 1.0f;
}

// torch.optim.Adam (train.py:402) on one element, the grad first scaled by the clip
__device__ __forceinline__ void adam_one(float& p, float& g, float& m, float& v, float coef, float omb1, float b2,
                                         float omb2, float step_size, float bc2_sqrt, float eps) {
    g = g * coef;
    m = m + omb1 * (g - m);  // exp_avg.lerp_(grad, 1 - beta1)
    v = v * b2 + (omb2 * g) * g;  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p - step_size * (m / denom);
}

}  // namespace nr
