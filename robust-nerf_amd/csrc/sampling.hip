// Inverse-CDF (hierarchical) sampling, one wave per ray.
//
// Reference semantics (ShawnnnLiu/Robust-NeRF):
//   sample_pdf           noisy_src/rays.py:213-279
//   sample_hierarchical  noisy_src/rays.py:282-333
// Per ray: w += 1e-5; pdf = w / sum(w); cdf = [0, cumsum(pdf)] (sequential
// order, as torch's CPU cumsum); u = linspace(0,1,Ns) if det else the caller's
// uniforms; idx = searchsorted(cdf, u, right=True); below/above clamped; the
// `denom < 1e-5 -> 1` rule; s = b0 + (u-c0)/denom * (b1-b0).  The hierarchical
// form then sorts cat(z_coarse, s) — here a bitonic sort in the wave's registers, whose
// output values equal torch.sort's whatever the order of u.
#include "common.hpp"

namespace nr {

// Lanes of one wave exchanging values through LDS: the wave barrier alone is not a
// memory fence at the IR level, so release / acquire at wavefront scope around it keep
// the compiler from moving or forwarding LDS accesses across it (rocPRIM's wave sync).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kRaysPerBlock = 4;  // one wave per ray
constexpr int kMaxPerLane = 8;    // Nc + Nf <= 512

__device__ __forceinline__ float linspace01(int n, int i) {
    if (n == 1) return 0.f;
    const float step = 1.0f / static_cast<float>(n - 1);
    return i < n / 2 ? step * static_cast<float>(i) : 1.0f - step * static_cast<float>(n - 1 - i);
}

// Build cdf[0..nb-1] from wbuf[0..nb-2] (raw weights, +1e-5 applied here).
// Every lane runs the same sequential recurrence; the owner lane stores.
// The divisions pdf_k = w_k / sum run in parallel (written over wbuf); the serial
// chain is the cumsum alone (the caller syncs the workgroup before reading cdf).
__device__ __forceinline__ void build_cdf(float* wbuf, float* cdf, int nb, int lane) {
    const int nw = nb - 1;
    float sum = 0.f;
    for (int k = 0; k < nw; ++k) sum += wbuf[k] + 1e-5f;
    float pdf[8];  // nw <= 512 (64 lanes x 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = lane + 64 * j;
        pdf[j] = k < nw ? (wbuf[k] + 1e-5f) / sum : 0.f;
    }
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = lane + 64 * j;
        if (k < nw) wbuf[k] = pdf[j];
    }
    wave_lds_sync();
    float run = 0.f;
    if (lane == 0) cdf[0] = 0.f;
    for (int k = 0; k < nw; ++k) {
        run += wbuf[k];
        if (((k + 1) & 63) == lane) cdf[k + 1] = run;
    }
}

__device__ __forceinline__ float invert_cdf(const float* cdf, const float* bins, int nb, float u) {
    int lo = 0, hi = nb;  // first index with cdf[idx] > u  (searchsorted right=True)
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf[mid] > u)
            hi = mid;
        else
            lo = mid + 1;
    }
    const int below = lo - 1 > 0 ? lo - 1 : 0;
    const int above = lo < nb - 1 ? lo : nb - 1;
    const float c0 = cdf[below], c1 = cdf[above];
    const float b0 = bins[below], b1 = bins[above];
    float denom = c1 - c0;
    denom = denom < 1e-5f ? 1.0f : denom;
    const float t = (u - c0) / denom;
    return b0 + t * (b1 - b0);
}

// LDS per wave: bins[nb] | cdf[nb] | wbuf[nb] | uni[T]
__global__ void sample_pdf_kernel(const float* bins_g, const float* w_g, const float* u_g, int B, int Nb, int Ns,
                                  float* out) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.x * kRaysPerBlock + wv;
    float* bins = smem + wv * (3 * Nb);
    float* cdf = bins + Nb;
    float* wbuf = cdf + Nb;
    const bool live = b < B;
    if (live) {
        for (int i = lane; i < Nb; i += 64) bins[i] = bins_g[static_cast<int64_t>(b) * Nb + i];
        for (int i = lane; i < Nb - 1; i += 64) wbuf[i] = w_g[static_cast<int64_t>(b) * (Nb - 1) + i];
    }
    __syncthreads();
    if (live) build_cdf(wbuf, cdf, Nb, lane);
    __syncthreads();
    if (!live) return;
    for (int j = lane; j < Ns; j += 64) {
        const float u = u_g ? u_g[static_cast<int64_t>(b) * Ns + j] : linspace01(Ns, j);
        out[static_cast<int64_t>(b) * Ns + j] = invert_cdf(cdf, bins, Nb, u);
    }
}

// Bitonic sort (ascending) of R * 64 values held R per lane (element 64 i + lane in
// register i), fully unrolled: strides below 64 exchange across lanes (__shfl_xor),
// strides of 64 and more between a lane's own registers.  Compare-exchange is
// fminf / fmaxf, so the output is the sorted multiset whatever the input order (equal
// values are interchangeable: only values leave the sort, as in torch.sort(...)[0]).
template <int R, int K, int J>
__device__ __forceinline__ void bitonic_step(float (&v)[R], int lane) {
    if constexpr (J >= 64) {
        constexpr int M = J / 64;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            if ((i & M) == 0) {
                const bool asc = ((i * 64) & K) == 0;  // K > J >= 64: the lane bits do not matter
                const float x = v[i], y = v[i ^ M];
                v[i] = asc ? fminf(x, y) : fmaxf(x, y);
                v[i ^ M] = asc ? fmaxf(x, y) : fminf(x, y);
            }
        }
    } else {
        const bool lo = (lane & J) == 0;  // the lower element of its pair
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const bool asc = K >= 64 ? ((i * 64) & K) == 0 : (lane & K) == 0;
            const float y = __shfl_xor(v[i], J);
            v[i] = lo == asc ? fminf(v[i], y) : fmaxf(v[i], y);
        }
    }
    if constexpr (J > 1) bitonic_step<R, K, J / 2>(v, lane);
}
template <int R, int K = 2>
__device__ __forceinline__ void bitonic_sort(float (&v)[R], int lane) {
    bitonic_step<R, K, K / 2>(v, lane);
    if constexpr (K < R * 64) bitonic_sort<R, K * 2>(v, lane);
}

// One wave per ray.  The wave's T = Nc + Nf values (coarse z, then the inverse-CDF
// samples) live in registers, R = P / 64 per lane for the padded length P (+inf past T),
// and are sorted there: the LDS form (v1) spent 11-14 us of 19-26 in its 36 LDS
// exchange rounds (tools/proto_sample_hier.hip).  LDS holds only bins, cdf and weights.
template <int R>
__global__ void sample_hier_kernel(const float* ro, const float* rd, const float* zc_g, const float* wc_g,
                                   const float* u_g, int B, int Nc, int Nf, float* zf_out, float* pts_out,
                                   float* vd_out) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.x * kRaysPerBlock + wv;
    const int Nb = Nc - 1, T = Nc + Nf;
    float* bins = smem + wv * (3 * Nb);
    float* cdf = bins + Nb;
    float* wbuf = cdf + Nb;
    const bool live = b < B;
    const int64_t zb = static_cast<int64_t>(b) * Nc;
    float v[R];
#pragma unroll
    for (int i = 0; i < R; ++i) v[i] = 0.f;
    if (live) {
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (i * 64 + lane < Nc) v[i] = zc_g[zb + i * 64 + lane];
        for (int i = lane; i < Nc - 2; i += 64) wbuf[i] = wc_g[zb + 1 + i];  // weights[..., 1:-1]
        // z_vals_mid: z[e + 1] from the next lane (lane 63: lane 0 of the next register)
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const float nxt = __shfl(v[i], (lane + 1) & 63);
            const float wrap = __shfl(v[i + 1 < R ? i + 1 : i], 0);
            const int e = i * 64 + lane;
            if (e < Nb) bins[e] = 0.5f * ((lane == 63 ? wrap : nxt) + v[i]);
        }
    }
    __syncthreads();
    if (live) build_cdf(wbuf, cdf, Nb, lane);
    __syncthreads();
    if (!live) return;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int e = i * 64 + lane;
        if (e >= Nc) {
            if (e < T) {
                const int j = e - Nc;
                const float u = u_g ? u_g[static_cast<int64_t>(b) * Nf + j] : linspace01(Nf, j);
                v[i] = invert_cdf(cdf, bins, Nb, u);
            } else {
                v[i] = __builtin_inff();
            }
        }
    }
    bitonic_sort<R>(v, lane);
    const int64_t ob = static_cast<int64_t>(b) * T;
    float ox = 0.f, oy = 0.f, oz = 0.f, dx = 0.f, dy = 0.f, dz = 0.f;
    if (pts_out || vd_out) {
        ox = ro ? ro[3 * b] : 0.f, oy = ro ? ro[3 * b + 1] : 0.f, oz = ro ? ro[3 * b + 2] : 0.f;
        dx = rd[3 * b], dy = rd[3 * b + 1], dz = rd[3 * b + 2];
    }
    float vx = 0.f, vy = 0.f, vz = 0.f;
    if (vd_out) {  // rendering.py:165 (expand_viewdirs_kernel's values)
        const float dn = norm3(dx, dy, dz);
        vx = dx / dn, vy = dy / dn, vz = dz / dn;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int e = i * 64 + lane;
        if (e < T) {
            const int64_t o = ob + e;
            zf_out[o] = v[i];
            if (pts_out) {
                pts_out[3 * o] = ox + dx * v[i];
                pts_out[3 * o + 1] = oy + dy * v[i];
                pts_out[3 * o + 2] = oz + dz * v[i];
            }
            if (vd_out) {
                vd_out[3 * o] = vx;
                vd_out[3 * o + 1] = vy;
                vd_out[3 * o + 2] = vz;
            }
        }
    }
}

}  // namespace nr

using namespace nr;

extern "C" {

int nr_sample_pdf(const float* bins, const float* weights, const float* u, int B, int Nb, int Ns, float* samples,
                  nr_stream_t stream) {
    NR_REQUIRE(bins && weights && samples && B >= 0 && Nb >= 2 && Ns > 0, "nr_sample_pdf: bad arguments");
    if (B == 0) return NR_OK;
    const size_t lds = sizeof(float) * kRaysPerBlock * 3 * Nb;
    NR_REQUIRE(lds <= 64 * 1024 && Nb - 1 <= 512, "nr_sample_pdf: Nb=%d too large", Nb);
    hipLaunchKernelGGL(sample_pdf_kernel, dim3(ceil_div(B, kRaysPerBlock)), dim3(64 * kRaysPerBlock), lds,
                       static_cast<hipStream_t>(stream), bins, weights, u, B, Nb, Ns, samples);
    NR_LAUNCH_CHECK("nr_sample_pdf");
    return NR_OK;
}

int nr_sample_hierarchical(const float* ro, const float* rd, const float* zc, const float* wc, const float* u,
                           int B, int Nc, int Nf, float* zf, float* pts, float* viewdirs, nr_stream_t stream) {
    NR_REQUIRE(zc && wc && zf && B >= 0 && Nc >= 3 && Nf > 0 && (!pts || (ro && rd)) && (!viewdirs || rd),
               "nr_sample_hierarchical: bad arguments");
    NR_REQUIRE(Nc + Nf <= 64 * kMaxPerLane, "nr_sample_hierarchical: Nc+Nf=%d exceeds %d", Nc + Nf,
               64 * kMaxPerLane);
    if (B == 0) return NR_OK;
    int P2 = 64;  // the kernel's sort pads Nc + Nf to a power of two, at least one wave
    while (P2 < Nc + Nf) P2 <<= 1;
    const size_t lds = sizeof(float) * kRaysPerBlock * 3 * (Nc - 1);
    const dim3 grid(ceil_div(B, kRaysPerBlock)), block(64 * kRaysPerBlock);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    switch (P2 / 64) {  // values per lane
        case 1: hipLaunchKernelGGL(sample_hier_kernel<1>, grid, block, lds, st, ro, rd, zc, wc, u, B, Nc, Nf, zf, pts, viewdirs); break;
        case 2: hipLaunchKernelGGL(sample_hier_kernel<2>, grid, block, lds, st, ro, rd, zc, wc, u, B, Nc, Nf, zf, pts, viewdirs); break;
        case 4: hipLaunchKernelGGL(sample_hier_kernel<4>, grid, block, lds, st, ro, rd, zc, wc, u, B, Nc, Nf, zf, pts, viewdirs); break;
        default: hipLaunchKernelGGL(sample_hier_kernel<8>, grid, block, lds, st, ro, rd, zc, wc, u, B, Nc, Nf, zf, pts, viewdirs); break;
    }
    NR_LAUNCH_CHECK("nr_sample_hierarchical");
    return NR_OK;
}

}  // extern "C"
