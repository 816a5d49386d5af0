// Volume-rendering alpha composite (forward + backward) and the MSE loss seed.
//
// Reference semantics (ShawnnnLiu/Robust-NeRF):
//   raw2outputs  noisy_src/rendering.py:20-116
//   loss         noisy_src/train.py:89,98 (mean((rgb - target)^2))
// One thread per ray walks its S samples in order, so the transmittance is the
// same sequential product as torch's CPU cumprod:
//   delta_i = (z_{i+1} - z_i | 1e10) * |d|;  a_i = 1 - exp(-relu(sigma_i + n_i) * delta_i)
//   T_0 = 1, T_{i+1} = T_i * (1 - a_i + 1e-10);  w_i = a_i T_i
//   rgb = sum w c (+ 1 - acc if white), depth = sum w z, acc = sum w.
// Backward uses the division-free form of torch's cumprod gradient:
//   dL/da_i = T_i (G_i - R_i),  R_i = G_{i+1} a_{i+1} + t_{i+1} R_{i+1},  R_{S-1} = 0
// (equal to G_i T_i - (sum_{k>i} G_k w_k) / t_i, the formula autograd evaluates).
#include "common.hpp"

namespace nr {

struct SampleTerms {
    float delta_raw, alpha, e, sig;  // sig = relu'd sigma after noise
};

__device__ __forceinline__ SampleTerms sample_terms(const float* sigma, const float* z, const float* noise,
                                                    int64_t base, int i, int S, float dnorm) {
    SampleTerms t;
    t.delta_raw = i < S - 1 ? z[base + i + 1] - z[base + i] : 1e10f;
    float s = sigma[base + i];
    if (noise) s = s + noise[base + i];
    t.sig = s > 0.f ? s : 0.f;
    t.e = expf(-t.sig * (t.delta_raw * dnorm));
    t.alpha = 1.0f - t.e;
    return t;
}

__global__ void composite_fwd_kernel(const float* rgb, const float* sigma, const float* z, const float* rd,
                                     const float* noise, int B, int S, int white, float* rgb_map, float* depth,
                                     float* acc, float* weights) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const float dnorm = sqrtf(rd[3 * b] * rd[3 * b] + rd[3 * b + 1] * rd[3 * b + 1] + rd[3 * b + 2] * rd[3 * b + 2]);
    const int64_t base = static_cast<int64_t>(b) * S;
    float T = 1.0f, r = 0.f, g = 0.f, bl = 0.f, d = 0.f, a = 0.f;
    for (int i = 0; i < S; ++i) {
        const SampleTerms st = sample_terms(sigma, z, noise, base, i, S, dnorm);
        const float w = st.alpha * T;
        T = T * (1.0f - st.alpha + 1e-10f);
        if (weights) weights[base + i] = w;
        const int64_t q = 3 * (base + i);
        r += w * rgb[q];
        g += w * rgb[q + 1];
        bl += w * rgb[q + 2];
        d += w * z[base + i];
        a += w;
    }
    if (white) {
        r = r + (1.0f - a);
        g = g + (1.0f - a);
        bl = bl + (1.0f - a);
    }
    rgb_map[3 * b] = r;
    rgb_map[3 * b + 1] = g;
    rgb_map[3 * b + 2] = bl;
    if (depth) depth[b] = d;
    if (acc) acc[b] = a;
}

// g_sigma doubles as scratch for T_i between the two passes.
__global__ void composite_bwd_kernel(const float* rgb, const float* sigma, const float* z, const float* rd,
                                     const float* noise, int B, int S, int white, const float* g_map,
                                     const float* g_depth, const float* g_acc, const float* g_w, float* g_rgb,
                                     float* g_sigma, float* g_rd) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const float dx = rd[3 * b], dy = rd[3 * b + 1], dz = rd[3 * b + 2];
    const float dnorm = sqrtf(dx * dx + dy * dy + dz * dz);
    const int64_t base = static_cast<int64_t>(b) * S;
    const float gr = g_map[3 * b], gg = g_map[3 * b + 1], gb = g_map[3 * b + 2];
    const float gd = g_depth ? g_depth[b] : 0.f;
    const float ga = (g_acc ? g_acc[b] : 0.f) - (white ? (gr + gg) + gb : 0.f);
    // pass 1: transmittance T_i -> g_sigma scratch
    float T = 1.0f;
    for (int i = 0; i < S; ++i) {
        const SampleTerms st = sample_terms(sigma, z, noise, base, i, S, dnorm);
        g_sigma[base + i] = T;
        T = T * (1.0f - st.alpha + 1e-10f);
    }
    // pass 2: reverse recurrence
    float R = 0.f, Gn = 0.f, an = 0.f, tn = 0.f, g_norm = 0.f;
    for (int i = S - 1; i >= 0; --i) {
        const SampleTerms st = sample_terms(sigma, z, noise, base, i, S, dnorm);
        const int64_t q = 3 * (base + i);
        const float Ti = g_sigma[base + i];
        const float w = st.alpha * Ti;
        const float c0 = rgb[q], c1 = rgb[q + 1], c2 = rgb[q + 2];
        float G = ((gr * c0 + gg * c1) + gb * c2) + gd * z[base + i] + ga;
        if (g_w) G += g_w[base + i];
        g_rgb[q] = gr * w;
        g_rgb[q + 1] = gg * w;
        g_rgb[q + 2] = gb * w;
        if (i < S - 1) R = Gn * an + tn * R;
        const float g_alpha = Ti * (G - R);
        // alpha = 1 - exp(x), x = -relu(s) * delta_raw * |d|
        const float g_x = -g_alpha * st.e;
        const float delta = st.delta_raw * dnorm;
        g_sigma[base + i] = (st.sig > 0.f) ? -g_x * delta : 0.f;
        g_norm += g_x * (-st.sig * st.delta_raw);
        Gn = G;
        an = st.alpha;
        tn = 1.0f - st.alpha + 1e-10f;
    }
    if (g_rd) {
        g_rd[3 * b] += g_norm * dx / dnorm;
        g_rd[3 * b + 1] += g_norm * dy / dnorm;
        g_rd[3 * b + 2] += g_norm * dz / dnorm;
    }
}

// ---- wave-per-ray forms (S <= 64 * kCompK): one 64-lane wave per ray, lane j
// owns samples [jK, jK + K) (K = ceil(S / 64)), all loads contiguous per lane.
// Transmittance: lane-local running product times the wave's exclusive product
// scan of the per-lane products (the thread-per-ray kernels above walk the ray
// serially through strided loads: 64 rays per launch-wide wave set, latency-bound).
// The backward's reverse recurrence R_i = u_{i+1} + t_{i+1} R_{i+1} (u = G a)
// becomes a lane-local affine map R_i = A_i + B_i X_j of the lane's boundary value
// X_j, and X_j = alpha_{j+1} + beta_{j+1} X_{j+1} is a suffix scan of affine maps
// across lanes.  Samples past S are padded with a = 0, t = 1, G = 0.  Only the
// association of the products and sums differs from the serial walk.
constexpr int kCompK = 8;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

__global__ __launch_bounds__(256) void composite_fwd_wave_kernel(const float* rgb, const float* sigma,
                                                                 const float* z, const float* rd,
                                                                 const float* noise, int B, int S, int K,
                                                                 int white, float* rgb_map, float* depth,
                                                                 float* acc, float* weights) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b >= B) return;  // wave-uniform
    const float dnorm = sqrtf(rd[3 * b] * rd[3 * b] + rd[3 * b + 1] * rd[3 * b + 1] + rd[3 * b + 2] * rd[3 * b + 2]);
    const int64_t base = static_cast<int64_t>(b) * S;
    const int i0 = lane * K;
    float al[kCompK], L[kCompK];
    float P = 1.0f;
#pragma unroll
    for (int k = 0; k < kCompK; ++k) {
        al[k] = 0.f;
        L[k] = P;
        const int i = i0 + k;
        if (k < K && i < S) {
            const SampleTerms st = sample_terms(sigma, z, noise, base, i, S, dnorm);
            al[k] = st.alpha;
            P = P * (1.0f - st.alpha + 1e-10f);
        }
    }
    // exclusive product scan of P over lanes
    float incl = P;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const float o = __shfl_up(incl, d);
        if (lane >= d) incl *= o;
    }
    float E = __shfl_up(incl, 1);
    if (lane == 0) E = 1.0f;
    float r = 0.f, g = 0.f, bl = 0.f, dd = 0.f, a = 0.f;
#pragma unroll
    for (int k = 0; k < kCompK; ++k) {
        const int i = i0 + k;
        if (k < K && i < S) {
            const float w = al[k] * (E * L[k]);
            if (weights) weights[base + i] = w;
            const int64_t q = 3 * (base + i);
            r += w * rgb[q];
            g += w * rgb[q + 1];
            bl += w * rgb[q + 2];
            dd += w * z[base + i];
            a += w;
        }
    }
    r = wave_sum(r);
    g = wave_sum(g);
    bl = wave_sum(bl);
    dd = wave_sum(dd);
    a = wave_sum(a);
    if (lane == 0) {
        if (white) {
            r = r + (1.0f - a);
            g = g + (1.0f - a);
            bl = bl + (1.0f - a);
        }
        rgb_map[3 * b] = r;
        rgb_map[3 * b + 1] = g;
        rgb_map[3 * b + 2] = bl;
        if (depth) depth[b] = dd;
        if (acc) acc[b] = a;
    }
}

__global__ __launch_bounds__(256) void composite_bwd_wave_kernel(
    const float* rgb, const float* sigma, const float* z, const float* rd, const float* noise, int B, int S, int K,
    int white, const float* g_map, const float* g_depth, const float* g_acc, const float* g_w, float* g_rgb,
    float* g_sigma, float* g_rd) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b >= B) return;
    const float dx = rd[3 * b], dy = rd[3 * b + 1], dz = rd[3 * b + 2];
    const float dnorm = sqrtf(dx * dx + dy * dy + dz * dz);
    const int64_t base = static_cast<int64_t>(b) * S;
    const float gr = g_map[3 * b], gg = g_map[3 * b + 1], gb = g_map[3 * b + 2];
    const float gd = g_depth ? g_depth[b] : 0.f;
    const float ga = (g_acc ? g_acc[b] : 0.f) - (white ? (gr + gg) + gb : 0.f);
    const int i0 = lane * K;
    float al[kCompK], tt[kCompK], ee[kCompK], sg[kCompK], dr[kCompK], GG[kCompK], L[kCompK];
    float P = 1.0f;
#pragma unroll
    for (int k = 0; k < kCompK; ++k) {
        al[k] = 0.f;
        tt[k] = 1.0f;
        ee[k] = 1.0f;
        sg[k] = 0.f;
        dr[k] = 0.f;
        GG[k] = 0.f;
        L[k] = P;
        const int i = i0 + k;
        if (k < K && i < S) {
            const SampleTerms st = sample_terms(sigma, z, noise, base, i, S, dnorm);
            al[k] = st.alpha;
            tt[k] = 1.0f - st.alpha + 1e-10f;
            ee[k] = st.e;
            sg[k] = st.sig;
            dr[k] = st.delta_raw;
            const int64_t q = 3 * (base + i);
            float G = ((gr * rgb[q] + gg * rgb[q + 1]) + gb * rgb[q + 2]) + gd * z[base + i] + ga;
            if (g_w) G += g_w[base + i];
            GG[k] = G;
            P = P * tt[k];
        }
    }
    float incl = P;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const float o = __shfl_up(incl, d);
        if (lane >= d) incl *= o;
    }
    float E = __shfl_up(incl, 1);
    if (lane == 0) E = 1.0f;
    // lane-local affine maps R_i = A_i + B_i X (X = R at the lane's last sample)
    float A[kCompK], Bc[kCompK];
    float an = 0.f, bn = 1.0f;
#pragma unroll
    for (int k = kCompK - 1; k >= 0; --k) {
        if (k < K) {
            if (k == K - 1) {
                an = 0.f;
                bn = 1.0f;
            } else {
                an = GG[k + 1] * al[k + 1] + tt[k + 1] * an;
                bn = tt[k + 1] * bn;
            }
        }
        A[k] = an;
        Bc[k] = bn;
    }
    // this lane's map for its predecessor: X_{j-1} = alpha + beta X_j
    float qa = GG[0] * al[0] + tt[0] * A[0];
    float qb = tt[0] * Bc[0];
    // suffix composition Q_j = N_j o N_{j+1} o ... o N_63
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const float oa = __shfl_down(qa, d), ob = __shfl_down(qb, d);
        if (lane + d < 64) {
            qa = qa + qb * oa;
            qb = qb * ob;
        }
    }
    float X = __shfl_down(qa, 1);
    if (lane == 63) X = 0.f;
    float g_norm = 0.f;
#pragma unroll
    for (int k = 0; k < kCompK; ++k) {
        const int i = i0 + k;
        if (k < K && i < S) {
            const float Ti = E * L[k];
            const float w = al[k] * Ti;
            const int64_t q = 3 * (base + i);
            g_rgb[q] = gr * w;
            g_rgb[q + 1] = gg * w;
            g_rgb[q + 2] = gb * w;
            const float R = A[k] + Bc[k] * X;
            const float g_alpha = Ti * (GG[k] - R);
            const float g_x = -g_alpha * ee[k];
            g_sigma[base + i] = (sg[k] > 0.f) ? -g_x * (dr[k] * dnorm) : 0.f;
            g_norm += g_x * (-sg[k] * dr[k]);
        }
    }
    g_norm = wave_sum(g_norm);
    if (g_rd && lane == 0) {
        g_rd[3 * b] += g_norm * dx / dnorm;
        g_rd[3 * b + 1] += g_norm * dy / dnorm;
        g_rd[3 * b + 2] += g_norm * dz / dnorm;
    }
}

// One ray of composite_mse_wave_kernel (lane = the wave's lane).
__device__ __forceinline__ void composite_mse_ray(const float* rgb, const float* sigma, const float* z, const float* rd,
                                                  const float* noise, const float* target, int b, int S, int K,
                                                  int white, float inv, float scale, float* rgb_map, float* depth,
                                                  float* acc, float* weights, float* sqerr, float* g_rgb,
                                                  float* g_sigma, float* g_rd, int lane) {
    const float dx = rd[3 * b], dy = rd[3 * b + 1], dz = rd[3 * b + 2];
    const float dnorm = sqrtf(dx * dx + dy * dy + dz * dz);
    const int64_t base = static_cast<int64_t>(b) * S;
    const int i0 = lane * K;
    float al[kCompK], tt[kCompK], ee[kCompK], sg[kCompK], dr[kCompK], L[kCompK], c[kCompK][3], zz[kCompK];
    float P = 1.0f;
#pragma unroll
    for (int k = 0; k < kCompK; ++k) {
        al[k] = 0.f;
        tt[k] = 1.0f;
        ee[k] = 1.0f;
        sg[k] = 0.f;
        dr[k] = 0.f;
        zz[k] = 0.f;
        c[k][0] = c[k][1] = c[k][2] = 0.f;
        L[k] = P;
        const int i = i0 + k;
        if (k < K && i < S) {
            const SampleTerms st = sample_terms(sigma, z, noise, base, i, S, dnorm);
            al[k] = st.alpha;
            tt[k] = 1.0f - st.alpha + 1e-10f;
            ee[k] = st.e;
            sg[k] = st.sig;
            dr[k] = st.delta_raw;
            zz[k] = z[base + i];
            const int64_t q = 3 * (base + i);
            c[k][0] = rgb[q];
            c[k][1] = rgb[q + 1];
            c[k][2] = rgb[q + 2];
            P = P * tt[k];
        }
    }
    float incl = P;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const float o = __shfl_up(incl, d);
        if (lane >= d) incl *= o;
    }
    float E = __shfl_up(incl, 1);
    if (lane == 0) E = 1.0f;
    // forward
    float r = 0.f, g = 0.f, bl = 0.f, dd = 0.f, a = 0.f;
#pragma unroll
    for (int k = 0; k < kCompK; ++k) {
        const int i = i0 + k;
        if (k < K && i < S) {
            const float w = al[k] * (E * L[k]);
            if (weights) weights[base + i] = w;
            r += w * c[k][0];
            g += w * c[k][1];
            bl += w * c[k][2];
            dd += w * zz[k];
            a += w;
        }
    }
    r = wave_sum(r);
    g = wave_sum(g);
    bl = wave_sum(bl);
    dd = wave_sum(dd);
    a = wave_sum(a);
    if (white) {
        r = r + (1.0f - a);
        g = g + (1.0f - a);
        bl = bl + (1.0f - a);
    }
    // loss seed
    const float d0 = r - target[3 * b], d1 = g - target[3 * b + 1], d2 = bl - target[3 * b + 2];
    const float gr = (2.0f * d0) * inv * scale, gg = (2.0f * d1) * inv * scale, gb = (2.0f * d2) * inv * scale;
    if (lane == 0) {
        rgb_map[3 * b] = r;
        rgb_map[3 * b + 1] = g;
        rgb_map[3 * b + 2] = bl;
        if (depth) depth[b] = dd;
        if (acc) acc[b] = a;
        sqerr[b] = (d0 * d0 + d1 * d1) + d2 * d2;
    }
    // backward (composite_bwd_wave_kernel with g_depth = g_acc = g_w = 0)
    const float gd = 0.f;
    const float ga = 0.f - (white ? (gr + gg) + gb : 0.f);
    float GG[kCompK];
#pragma unroll
    for (int k = 0; k < kCompK; ++k) {
        GG[k] = 0.f;
        if (k < K && i0 + k < S) GG[k] = ((gr * c[k][0] + gg * c[k][1]) + gb * c[k][2]) + gd * zz[k] + ga;
    }
    float A[kCompK], Bc[kCompK];
    float an = 0.f, bn = 1.0f;
#pragma unroll
    for (int k = kCompK - 1; k >= 0; --k) {
        if (k < K) {
            if (k == K - 1) {
                an = 0.f;
                bn = 1.0f;
            } else {
                an = GG[k + 1] * al[k + 1] + tt[k + 1] * an;
                bn = tt[k + 1] * bn;
            }
        }
        A[k] = an;
        Bc[k] = bn;
    }
    float qa = GG[0] * al[0] + tt[0] * A[0];
    float qb = tt[0] * Bc[0];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const float oa = __shfl_down(qa, d), ob = __shfl_down(qb, d);
        if (lane + d < 64) {
            qa = qa + qb * oa;
            qb = qb * ob;
        }
    }
    float X = __shfl_down(qa, 1);
    if (lane == 63) X = 0.f;
    float g_norm = 0.f;
#pragma unroll
    for (int k = 0; k < kCompK; ++k) {
        const int i = i0 + k;
        if (k < K && i < S) {
            const float Ti = E * L[k];
            const float w = al[k] * Ti;
            const int64_t q = 3 * (base + i);
            g_rgb[q] = gr * w;
            g_rgb[q + 1] = gg * w;
            g_rgb[q + 2] = gb * w;
            const float R = A[k] + Bc[k] * X;
            const float g_alpha = Ti * (GG[k] - R);
            const float g_x = -g_alpha * ee[k];
            g_sigma[base + i] = (sg[k] > 0.f) ? -g_x * (dr[k] * dnorm) : 0.f;
            g_norm += g_x * (-sg[k] * dr[k]);
        }
    }
    g_norm = wave_sum(g_norm);
    if (g_rd && lane == 0) {
        g_rd[3 * b] += g_norm * dx / dnorm;
        g_rd[3 * b + 1] += g_norm * dy / dnorm;
        g_rd[3 * b + 2] += g_norm * dz / dnorm;
    }
}


// The last workgroup to finish (an agent-scope ticket; the recipe of
// cdna_hip_programming.md §6 Guideline 16: plain stores, release fence, relaxed
// fetch_add, acquire fence in the reducer) sums the per-ray squared errors in a fixed
// order and leaves the ticket at 0 for the next call.
__device__ __forceinline__ void sum_loss_last_block(const float* sqerr, int B, float inv, unsigned* ticket,
                                                    float* loss) {
    __shared__ float part[5];  // [0..3]: wave sums, [4]: the "last" flag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        part[4] = t == gridDim.x - 1 ? 1.f : 0.f;
    }
    __syncthreads();
    if (part[4] == 0.f) return;  // workgroup-uniform
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    float sum = 0.f;
    for (int i = threadIdx.x; i < B; i += blockDim.x) sum += sqerr[i];
    sum = wave_sum(sum);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        float tot = 0.f;
        for (int w = 0; w < static_cast<int>(blockDim.x >> 6); ++w) tot += part[w];
        *loss = tot * inv;
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Training form: raw2outputs (rendering.py:20-116) + the MSE loss seed (train.py:89,98:
// mean over 3B of (rgb_map - target)^2, gradient 2 (rgb_map - target) / 3B * scale) + the
// backward of both, in one wave-per-ray pass.  Every value is the expression
// composite_fwd_wave_kernel, mse_kernel and composite_bwd_wave_kernel evaluate (the
// backward's depth / acc / weight terms are the zeros those kernels read for absent
// gradients), so g_rgb / g_sigma / g_rd are bit-identical to the three launches.  The
// loss is summed per ray (sqerr), then over the rays by the last workgroup (ticket) or,
// without a ticket, by loss_sum_kernel.
__global__ __launch_bounds__(256) void composite_mse_wave_kernel(
    const float* rgb, const float* sigma, const float* z, const float* rd, const float* noise, const float* target,
    int B, int S, int K, int white, float inv, float scale, float* rgb_map, float* depth, float* acc, float* weights,
    float* sqerr, float* g_rgb, float* g_sigma, float* g_rd, unsigned* ticket, float* loss) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b < B) composite_mse_ray(rgb, sigma, z, rd, noise, target, b, S, K, white, inv, scale, rgb_map, depth, acc,
                                 weights, sqerr, g_rgb, g_sigma, g_rd, lane);
    if (ticket) sum_loss_last_block(sqerr, B, inv, ticket, loss);
}

// loss = inv * sum of the per-ray squared errors, in a fixed order.  One block.
__global__ __launch_bounds__(1024) void loss_sum_kernel(const float* sqerr, int B, float inv, float* loss) {
    __shared__ float part[16];
    float s = 0.f;
    for (int i = threadIdx.x; i < B; i += blockDim.x) s += sqerr[i];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float tot = 0.f;
        for (int i = 0; i < static_cast<int>(blockDim.x >> 6); ++i) tot += part[i];
        *loss = tot * inv;
    }
}

// loss = mean((p - t)^2) over n = 3B; g = 2 (p - t) / n * scale.  One block.
__global__ void mse_kernel(const float* p, const float* t, int n, float scale, float* loss, float* g) {
    __shared__ float part[16];
    float s = 0.f;
    const float inv = 1.0f / static_cast<float>(n);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float d = p[i] - t[i];
        s += d * d;
        if (g) g[i] = (2.0f * d) * inv * scale;
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) part[w] = s;
    __syncthreads();
    if (threadIdx.x == 0 && loss) {
        float tot = 0.f;
        for (int i = 0; i < static_cast<int>(blockDim.x >> 6); ++i) tot += part[i];
        *loss = tot * inv;
    }
}

}  // namespace nr

using namespace nr;

extern "C" {

int nr_composite_fwd(const float* rgb, const float* sigma, const float* z, const float* rd, const float* noise, int B,
                     int S, int white, float* rgb_map, float* depth, float* acc, float* weights,
                     nr_stream_t stream) {
    NR_REQUIRE(rgb && sigma && z && rd && rgb_map && B >= 0 && S > 0, "nr_composite_fwd: bad arguments");
    if (B == 0) return NR_OK;
    if (S <= 64 * kCompK)
        hipLaunchKernelGGL(composite_fwd_wave_kernel, dim3(ceil_div(B, 4)), dim3(256), 0,
                           static_cast<hipStream_t>(stream), rgb, sigma, z, rd, noise, B, S, (S + 63) / 64, white,
                           rgb_map, depth, acc, weights);
    else
        hipLaunchKernelGGL(composite_fwd_kernel, dim3(ceil_div(B, 64)), dim3(64), 0, static_cast<hipStream_t>(stream),
                           rgb, sigma, z, rd, noise, B, S, white, rgb_map, depth, acc, weights);
    NR_LAUNCH_CHECK("nr_composite_fwd");
    return NR_OK;
}

int nr_composite_bwd(const float* rgb, const float* sigma, const float* z, const float* rd, const float* noise, int B,
                     int S, int white, const float* g_map, const float* g_depth, const float* g_acc,
                     const float* g_w, float* g_rgb, float* g_sigma, float* g_rd, nr_stream_t stream) {
    NR_REQUIRE(rgb && sigma && z && rd && g_map && g_rgb && g_sigma && B >= 0 && S > 0,
               "nr_composite_bwd: bad arguments");
    if (B == 0) return NR_OK;
    if (S <= 64 * kCompK)
        hipLaunchKernelGGL(composite_bwd_wave_kernel, dim3(ceil_div(B, 4)), dim3(256), 0,
                           static_cast<hipStream_t>(stream), rgb, sigma, z, rd, noise, B, S, (S + 63) / 64, white,
                           g_map, g_depth, g_acc, g_w, g_rgb, g_sigma, g_rd);
    else
        hipLaunchKernelGGL(composite_bwd_kernel, dim3(ceil_div(B, 64)), dim3(64), 0, static_cast<hipStream_t>(stream),
                           rgb, sigma, z, rd, noise, B, S, white, g_map, g_depth, g_acc, g_w, g_rgb, g_sigma, g_rd);
    NR_LAUNCH_CHECK("nr_composite_bwd");
    return NR_OK;
}

int nr_composite_mse(const float* rgb, const float* sigma, const float* z, const float* rd, const float* noise,
                     const float* target, int B, int S, int white, float scale, float* rgb_map, float* depth,
                     float* acc, float* weights, float* loss, float* g_rgb, float* g_sigma, float* g_rd,
                     unsigned* ticket, void* workspace, nr_stream_t stream) {
    NR_REQUIRE(rgb && sigma && z && rd && target && rgb_map && loss && g_rgb && g_sigma && workspace && B > 0 && S > 0,
               "nr_composite_mse: bad arguments");
    const hipStream_t s = static_cast<hipStream_t>(stream);
    float* sqerr = static_cast<float*>(workspace);
    const float inv = 1.0f / static_cast<float>(3 * B);
    // the in-launch loss sum pays up to ~256 workgroups; beyond, the agent-scope release and
    // ticket of every workgroup cost more than a second one-block launch (measured: 1024
    // workgroups, 4096 rays, 61 vs 26 + 5 us)
    if (ticket && ceil_div(B, 4) > 256) ticket = nullptr;
    if (S <= 64 * kCompK) {
        hipLaunchKernelGGL(composite_mse_wave_kernel, dim3(ceil_div(B, 4)), dim3(256), 0, s, rgb, sigma, z, rd, noise,
                           target, B, S, (S + 63) / 64, white, inv, scale, rgb_map, depth, acc, weights, sqerr, g_rgb,
                           g_sigma, g_rd, ticket, loss);
        NR_LAUNCH_CHECK("nr_composite_mse");
        if (!ticket) {
            hipLaunchKernelGGL(loss_sum_kernel, dim3(1), dim3(1024), 0, s, sqerr, B, inv, loss);
            NR_LAUNCH_CHECK("nr_composite_mse (loss)");
        }
        return NR_OK;
    }
    // long rays: the three separate passes (the seed gradient lives in the workspace)
    float* g_map = sqerr + B;
    int rc = nr_composite_fwd(rgb, sigma, z, rd, noise, B, S, white, rgb_map, depth, acc, weights, stream);
    if (rc) return rc;
    rc = nr_mse_fwd_bwd(rgb_map, target, B, scale, loss, g_map, stream);
    if (rc) return rc;
    return nr_composite_bwd(rgb, sigma, z, rd, noise, B, S, white, g_map, nullptr, nullptr, nullptr, g_rgb, g_sigma,
                            g_rd, stream);
}

int64_t nr_composite_mse_workspace_bytes(int B) { return B > 0 ? int64_t{16} * B : 0; }

int nr_mse_fwd_bwd(const float* pred, const float* target, int B, float scale, float* loss, float* g,
                   nr_stream_t stream) {
    NR_REQUIRE(pred && target && B > 0, "nr_mse_fwd_bwd: bad arguments");
    hipLaunchKernelGGL(mse_kernel, dim3(1), dim3(1024), 0, static_cast<hipStream_t>(stream), pred, target, 3 * B,
                       scale, loss, g);
    NR_LAUNCH_CHECK("nr_mse_fwd_bwd");
    return NR_OK;
}

}  // extern "C"
