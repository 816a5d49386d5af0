// Optimizer tail: global-norm gradient clipping and Adam on flat fp32 buffers.
//
// Reference semantics (ShawnnnLiu/Robust-NeRF):
//   torch.nn.utils.clip_grad_norm_(params, max_norm)  noisy_src/train.py:115,
//       noisy_src/train_pose_opt.py:398-404: coef = min(1, max_norm / (||g||_2 + 1e-6))
//   torch.optim.Adam(lr, betas=(0.9, 0.999), eps=1e-8)  noisy_src/train.py:402
//       m.lerp_(g, 1-b1); v = b2 v + (1-b2) g^2; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
//   LambdaLR 0.1^(step/250000)                          noisy_src/train.py:405-411 (host)
// HBM-bound: ~20 B read + 16 B written per parameter; 16-B vector accesses.
//
// Determinism: the sum of squares is a fixed-shape two-pass reduction (a constant
// grid of kSumsqBlocks partials, then one block that sums them in index order), so
// the clip coefficient — and with it every data-parallel replica's Adam update — is
// bit-identical from run to run (the reference is bit-deterministic).
#include <cmath>

#include "optim.hpp"

namespace nr {

__global__ void __launch_bounds__(kSumsqThreads) sumsq_partial_kernel(const float* x, int64_t n, float* partials) {
    float s = 0.f;
    const int64_t stride = static_cast<int64_t>(kSumsqBlocks) * kSumsqThreads;
    const int64_t n4 = n / 4;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kSumsqThreads + threadIdx.x; i < n4; i += stride) {
        const float4 v = x4[i];
        s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (int64_t i = 4 * n4 + static_cast<int64_t>(blockIdx.x) * kSumsqThreads + threadIdx.x; i < n; i += stride)
        s += x[i] * x[i];
    const float t = block_sum_fixed(s);
    if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// One clip group's buffers as one sequence: block b sums the elements it strides over
// in every span, in span order, so the partials are a fixed function of the inputs.
struct SumsqSpans {
    const float* x[kMaxAdamSpans];
    int64_t n[kMaxAdamSpans];
    int nspan;
};

__global__ void __launch_bounds__(kSumsqThreads) sumsq_spans_kernel(SumsqSpans sp, float* partials) {
    float s = 0.f;
    const int64_t stride = static_cast<int64_t>(kSumsqBlocks) * kSumsqThreads;
    const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kSumsqThreads + threadIdx.x;
    for (int k = 0; k < sp.nspan; ++k) {
        const float* x = sp.x[k];
        const int64_t n = sp.n[k], n4 = ((reinterpret_cast<uintptr_t>(x) & 15) == 0) ? n / 4 : 0;
        const float4* x4 = reinterpret_cast<const float4*>(x);
        for (int64_t i = t0; i < n4; i += stride) {
            const float4 v = x4[i];
            s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        }
        for (int64_t i = 4 * n4 + t0; i < n; i += stride) s += x[i] * x[i];
    }
    const float t = block_sum_fixed(s);
    if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

__global__ void __launch_bounds__(kSumsqThreads) sumsq_final_kernel(const float* partials, float* acc) {
    const float t = block_sum_fixed(partials[threadIdx.x]);
    if (threadIdx.x == 0) *acc += t;
}

__global__ void adam_kernel(float* p, float* g, float* m, float* v, int64_t n, float omb1, float b2, float omb2,
                            float eps,
                            float step_size, float bc2_sqrt, const float* sumsq, float max_norm) {
    const float coef = sumsq ? clip_coef(*sumsq, max_norm) : 1.0f;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    const int64_t n4 = n / 4;
    float4* p4 = reinterpret_cast<float4*>(p);
    float4* g4 = reinterpret_cast<float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 P = p4[i], G = g4[i], M = m4[i], V = v4[i];
        adam_one(P.x, G.x, M.x, V.x, coef, omb1, b2, omb2, step_size, bc2_sqrt, eps);
        adam_one(P.y, G.y, M.y, V.y, coef, omb1, b2, omb2, step_size, bc2_sqrt, eps);
        adam_one(P.z, G.z, M.z, V.z, coef, omb1, b2, omb2, step_size, bc2_sqrt, eps);
        adam_one(P.w, G.w, M.w, V.w, coef, omb1, b2, omb2, step_size, bc2_sqrt, eps);
        p4[i] = P;
        g4[i] = G;
        m4[i] = M;
        v4[i] = V;
    }
    for (int64_t i = 4 * n4 + static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        adam_one(p[i], g[i], m[i], v[i], coef, omb1, b2, omb2, step_size, bc2_sqrt, eps);
}

}  // namespace nr

using namespace nr;

extern "C" {

int64_t nr_sumsq_workspace_bytes(void) { return static_cast<int64_t>(kSumsqBlocks) * sizeof(float); }

int nr_sumsq(const float* x, int64_t n, float* acc, void* workspace, nr_stream_t stream) {
    NR_REQUIRE(x && acc && workspace && n >= 0, "nr_sumsq: bad arguments");
    NR_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0, "nr_sumsq: x must be 16-byte aligned");
    if (n == 0) return NR_OK;
    float* partials = static_cast<float*>(workspace);
    hipLaunchKernelGGL(sumsq_partial_kernel, dim3(kSumsqBlocks), dim3(kSumsqThreads), 0,
                       static_cast<hipStream_t>(stream), x, n, partials);
    NR_LAUNCH_CHECK("nr_sumsq");
    hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(kSumsqThreads), 0, static_cast<hipStream_t>(stream),
                       partials, acc);
    NR_LAUNCH_CHECK("nr_sumsq");
    return NR_OK;
}

int nr_sumsq_partials(const float* const* xs, const int64_t* ns, int nspan, float* partials, nr_stream_t stream) {
    NR_REQUIRE(xs && ns && partials && nspan >= 1 && nspan <= kMaxAdamSpans,
               "nr_sumsq_partials: bad arguments (1..%d spans)", kMaxAdamSpans);
    SumsqSpans sp;
    std::memset(&sp, 0, sizeof(sp));
    sp.nspan = nspan;
    for (int k = 0; k < nspan; ++k) {
        NR_REQUIRE(ns[k] >= 0 && (xs[k] || ns[k] == 0), "nr_sumsq_partials: span %d: bad buffer", k);
        sp.x[k] = xs[k];
        sp.n[k] = ns[k];
    }
    hipLaunchKernelGGL(sumsq_spans_kernel, dim3(kSumsqBlocks), dim3(kSumsqThreads), 0,
                       static_cast<hipStream_t>(stream), sp, partials);
    NR_LAUNCH_CHECK("nr_sumsq_partials");
    return NR_OK;
}

int nr_adam_step(float* p, float* g, float* m, float* v, int64_t n, double lr, double b1, double b2, double eps,
                 int64_t step, const float* sumsq, float max_norm, nr_stream_t stream) {
    NR_REQUIRE(p && g && m && v && n >= 0 && step >= 1, "nr_adam_step: bad arguments");
    NR_REQUIRE(((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
                 reinterpret_cast<uintptr_t>(v)) & 15) == 0,
               "nr_adam_step: buffers must be 16-byte aligned");
    if (n == 0) return NR_OK;
    // bias corrections in double on the host, as torch's _single/_multi_tensor_adam do
    const double bc1 = 1.0 - std::pow(b1, static_cast<double>(step));
    const double bc2 = 1.0 - std::pow(b2, static_cast<double>(step));
    const float step_size = static_cast<float>(lr / bc1);
    const float bc2_sqrt = static_cast<float>(std::sqrt(bc2));
    const int grid = stream_grid(ceil_div_ll(n, 4), 256);
    hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), p, g, m, v, n,
                       static_cast<float>(1.0 - b1), static_cast<float>(b2), static_cast<float>(1.0 - b2),
                       static_cast<float>(eps), step_size, bc2_sqrt, sumsq, max_norm);
    NR_LAUNCH_CHECK("nr_adam_step");
    return NR_OK;
}

}  // extern "C"
