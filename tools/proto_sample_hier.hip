// Prototype (not product code): where sample_hier_kernel's time goes.  Timing-only
// variants of its body (parts removed) beside the real entry point, HIP events.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -I../robust-nerf_amd/csrc \
//         proto_sample_hier.hip -o proto_bin/sample_hier && proto_bin/sample_hier
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "sampling.hip"

using namespace nr;

template <bool LOADS, bool CDF, bool INV, bool SORT, bool STORE>
__global__ void sh_var(const float* ro, const float* rd, const float* zc_g, const float* wc_g, const float* u_g, int B,
                       int Nc, int Nf, float* zf_out, float* pts_out, float* vd_out) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.x * kRaysPerBlock + wv;
    const int Nb = Nc - 1, T = Nc + Nf;
    int P2 = 1;
    while (P2 < T) P2 <<= 1;
    float* bins = smem + wv * (3 * Nb + P2);
    float* cdf = bins + Nb;
    float* wbuf = cdf + Nb;
    float* uni = wbuf + Nb;
    const bool live = b < B;
    const int64_t zb = static_cast<int64_t>(b) * Nc;
    if (live) {
        for (int i = lane; i < Nc; i += 64) uni[i] = LOADS ? zc_g[zb + i] : 0.5f * i;
        for (int i = lane; i < Nc - 2; i += 64) wbuf[i] = LOADS ? wc_g[zb + 1 + i] : 1.f;
    }
    __syncthreads();
    if (live) {
        for (int i = lane; i < Nb; i += 64) bins[i] = 0.5f * (uni[i + 1] + uni[i]);
        if (CDF) build_cdf(wbuf, cdf, Nb, lane);
        else for (int i = lane; i < Nb; i += 64) cdf[i] = i / float(Nb);
    }
    __syncthreads();
    if (live) {
        for (int j = lane; j < Nf; j += 64) {
            const float u = LOADS ? u_g[static_cast<int64_t>(b) * Nf + j] : 0.3f;
            uni[Nc + j] = INV ? invert_cdf(cdf, bins, Nb, u) : u;
        }
    }
    __syncthreads();
    if (!live) return;
    const int P = P2;
    if (SORT) {
        for (int e = T + lane; e < P; e += 64) uni[e] = __builtin_inff();
        wave_lds_sync();
        for (int k = 2; k <= P; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int t = lane; t < (P >> 1); t += 64) {
                    const int lo = ((t & ~(j - 1)) << 1) | (t & (j - 1)), hi = lo + j;
                    const float x = uni[lo], y = uni[hi];
                    const bool swap = (lo & k) == 0 ? (x > y) : (x < y);
                    if (swap) {
                        uni[lo] = y;
                        uni[hi] = x;
                    }
                }
                wave_lds_sync();
            }
        }
    }
    if (!STORE) {
        if (uni[lane] == 12345.f) zf_out[0] = 1.f;  // keep the work
        return;
    }
    const int64_t ob = static_cast<int64_t>(b) * T;
    const float ox = ro[3 * b], oy = ro[3 * b + 1], oz = ro[3 * b + 2];
    const float dx = rd[3 * b], dy = rd[3 * b + 1], dz = rd[3 * b + 2];
    const float dn = norm3(dx, dy, dz);
    const float vx = dx / dn, vy = dy / dn, vz = dz / dn;
    for (int e = lane; e < T; e += 64) {
        const float v = uni[e];
        const int64_t o = ob + e;
        zf_out[o] = v;
        pts_out[3 * o] = ox + dx * v;
        pts_out[3 * o + 1] = oy + dy * v;
        pts_out[3 * o + 2] = oz + dz * v;
        vd_out[3 * o] = vx;
        vd_out[3 * o + 1] = vy;
        vd_out[3 * o + 2] = vz;
    }
}

// bitonic compare-exchange of registers i and i ^ M (M = j / 64), same lane
template <int M>
__device__ __forceinline__ void reg_cx(float (&v)[8], int R, int k, int lane) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if ((i & M) == 0 && i < R) {
            const int e = i * 64 + lane;
            const bool asc = (e & k) == 0;
            const float x = v[i], y = v[i ^ M];
            v[i] = asc ? fminf(x, y) : fmaxf(x, y);
            v[i ^ M] = asc ? fmaxf(x, y) : fminf(x, y);
        }
    }
}

__global__ void sh_reg(const float* ro, const float* rd, const float* zc_g, const float* wc_g, const float* u_g, int B,
                       int Nc, int Nf, float* zf_out, float* pts_out, float* vd_out) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.x * kRaysPerBlock + wv;
    const int Nb = Nc - 1, T = Nc + Nf;
    int P = 64;
    while (P < T) P <<= 1;
    const int R = P >> 6;  // values per lane
    float* bins = smem + wv * (3 * Nb + 64);
    float* cdf = bins + Nb;
    float* wbuf = cdf + Nb;
    float* zl = wbuf + Nb;  // unused tail
    (void)zl;
    const bool live = b < B;
    const int64_t zb = static_cast<int64_t>(b) * Nc;
    // element e = 64 i + lane of the padded sequence lives in register i of this lane
    float v[8];
    if (live) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (i < R && i * 64 + lane < Nc) ? zc_g[zb + i * 64 + lane] : 0.f;
        for (int i = lane; i < Nc - 2; i += 64) wbuf[i] = wc_g[zb + 1 + i];
        // bins from the z values: z[i + 1] by shuffle (lane 63 takes the next register's lane 0)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i < R) {
                const float nxt = __shfl(v[i], (lane + 1) & 63);
                const float up = lane == 63 ? (i + 1 < 8 ? __shfl(v[i + 1 < 8 ? i + 1 : i], 0) : 0.f) : nxt;
                const int e = i * 64 + lane;
                if (e < Nb) bins[e] = 0.5f * (up + v[i]);
            }
        }
    }
    __syncthreads();
    if (live) build_cdf(wbuf, cdf, Nb, lane);
    __syncthreads();
    if (!live) return;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (i < R) {
            const int e = i * 64 + lane;
            if (e >= Nc) v[i] = e < T ? invert_cdf(cdf, bins, Nb, u_g[static_cast<int64_t>(b) * Nf + (e - Nc)])
                                      : __builtin_inff();
        }
    }
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
                const int m = j >> 6;
                if (m == 1) reg_cx<1>(v, R, k, lane);
                else if (m == 2) reg_cx<2>(v, R, k, lane);
                else reg_cx<4>(v, R, k, lane);
            } else {
                const bool lo = (lane & j) == 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if (i < R) {
                        const int e = i * 64 + lane;
                        const bool asc = (e & k) == 0;
                        const float y = __shfl_xor(v[i], j);
                        v[i] = (lo == asc) ? fminf(v[i], y) : fmaxf(v[i], y);
                    }
                }
            }
        }
    }
    const int64_t ob = static_cast<int64_t>(b) * T;
    const float ox = ro[3 * b], oy = ro[3 * b + 1], oz = ro[3 * b + 2];
    const float dx = rd[3 * b], dy = rd[3 * b + 1], dz = rd[3 * b + 2];
    const float dn = norm3(dx, dy, dz);
    const float vx = dx / dn, vy = dy / dn, vz = dz / dn;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int e = i * 64 + lane;
        if (i < R && e < T) {
            const int64_t o = ob + e;
            zf_out[o] = v[i];
            pts_out[3 * o] = ox + dx * v[i];
            pts_out[3 * o + 1] = oy + dy * v[i];
            pts_out[3 * o + 2] = oz + dz * v[i];
            vd_out[3 * o] = vx;
            vd_out[3 * o + 1] = vy;
            vd_out[3 * o + 2] = vz;
        }
    }
}

// fully unrolled register bitonic sort of R = P / 64 values per lane (element 64 i + lane
// in register i), ascending
template <int R, int K, int J>
__device__ __forceinline__ void bitonic_step(float (&v)[8], int lane) {
    if constexpr (J >= 64) {
        constexpr int M = J / 64;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            if ((i & M) == 0) {
                const bool asc = ((i * 64) & K) == 0;  // K >= 128 here: lane bits do not matter
                const float x = v[i], y = v[i ^ M];
                v[i] = asc ? fminf(x, y) : fmaxf(x, y);
                v[i ^ M] = asc ? fmaxf(x, y) : fminf(x, y);
            }
        }
    } else {
        const bool lo = (lane & J) == 0;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const bool asc = (K >= 64) ? (((i * 64) & K) == 0) : ((lane & K) == 0);
            const float y = __shfl_xor(v[i], J);
            v[i] = (lo == asc) ? fminf(v[i], y) : fmaxf(v[i], y);
        }
    }
    if constexpr (J > 1) bitonic_step<R, K, J / 2>(v, lane);
}
template <int R, int K>
__device__ __forceinline__ void bitonic_all(float (&v)[8], int lane) {
    bitonic_step<R, K, K / 2>(v, lane);
    if constexpr (K < R * 64) bitonic_all<R, K * 2>(v, lane);
}

template <int R>
__global__ void sh_reg2(const float* ro, const float* rd, const float* zc_g, const float* wc_g, const float* u_g, int B,
                        int Nc, int Nf, float* zf_out, float* pts_out, float* vd_out) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.x * kRaysPerBlock + wv;
    const int Nb = Nc - 1, T = Nc + Nf;
    float* bins = smem + wv * (3 * Nb + 64);
    float* cdf = bins + Nb;
    float* wbuf = cdf + Nb;
    float* zs = wbuf + Nb;  // unused
    (void)zs;
    const bool live = b < B;
    const int64_t zb = static_cast<int64_t>(b) * Nc;
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
    if (live) {
#pragma unroll
        for (int i = 0; i < R; ++i) v[i] = (i * 64 + lane < Nc) ? zc_g[zb + i * 64 + lane] : 0.f;
        for (int i = lane; i < Nc - 2; i += 64) wbuf[i] = wc_g[zb + 1 + i];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const float nxt = __shfl(v[i], (lane + 1) & 63);
            const float first_next = __shfl(v[i + 1 < R ? i + 1 : i], 0);
            const float up = lane == 63 ? first_next : nxt;
            const int e = i * 64 + lane;
            if (e < Nb) bins[e] = 0.5f * (up + v[i]);
        }
    }
    __syncthreads();
    if (live) build_cdf(wbuf, cdf, Nb, lane);
    __syncthreads();
    if (!live) return;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int e = i * 64 + lane;
        if (e >= Nc) v[i] = e < T ? invert_cdf(cdf, bins, Nb, u_g[static_cast<int64_t>(b) * Nf + (e - Nc)])
                                  : __builtin_inff();
    }
    bitonic_all<R, 2>(v, lane);
    const int64_t ob = static_cast<int64_t>(b) * T;
    const float ox = ro[3 * b], oy = ro[3 * b + 1], oz = ro[3 * b + 2];
    const float dx = rd[3 * b], dy = rd[3 * b + 1], dz = rd[3 * b + 2];
    const float dn = norm3(dx, dy, dz);
    const float vx = dx / dn, vy = dy / dn, vz = dz / dn;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int e = i * 64 + lane;
        if (e < T) {
            const int64_t o = ob + e;
            zf_out[o] = v[i];
            pts_out[3 * o] = ox + dx * v[i];
            pts_out[3 * o + 1] = oy + dy * v[i];
            pts_out[3 * o + 2] = oz + dz * v[i];
            vd_out[3 * o] = vx;
            vd_out[3 * o + 1] = vy;
            vd_out[3 * o + 2] = vz;
        }
    }
}

int main() {
    const int Nc = 64, Nf = 128, T = Nc + Nf;
    for (int B : {512, 4096}) {
        std::vector<float> zc(size_t(B) * Nc), wc(size_t(B) * Nc), u(size_t(B) * Nf), o(3 * B), d(3 * B);
        srand(1);
        for (int b = 0; b < B; ++b) {
            for (int i = 0; i < Nc; ++i) zc[size_t(b) * Nc + i] = 2.f + 4.f * (i + rand() / float(RAND_MAX)) / Nc;
            for (int i = 0; i < Nc; ++i) wc[size_t(b) * Nc + i] = rand() / float(RAND_MAX) * (i > 20 && i < 30);
            for (int i = 0; i < Nf; ++i) u[size_t(b) * Nf + i] = rand() / float(RAND_MAX);
            for (int c = 0; c < 3; ++c) { o[3 * b + c] = 0.1f * c; d[3 * b + c] = c == 2 ? -1.f : 0.1f; }
        }
        float *dzc, *dwc, *du, *dro, *drd, *dzf, *dpts, *dvd;
        hipMalloc(&dzc, zc.size() * 4); hipMalloc(&dwc, wc.size() * 4); hipMalloc(&du, u.size() * 4);
        hipMalloc(&dro, o.size() * 4); hipMalloc(&drd, d.size() * 4);
        hipMalloc(&dzf, size_t(B) * T * 4); hipMalloc(&dpts, size_t(B) * T * 12); hipMalloc(&dvd, size_t(B) * T * 12);
        hipMemcpy(dzc, zc.data(), zc.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(dwc, wc.data(), wc.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(du, u.data(), u.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(dro, o.data(), o.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(drd, d.data(), d.size() * 4, hipMemcpyHostToDevice);
        const size_t lds = sizeof(float) * kRaysPerBlock * (3 * (Nc - 1) + 256);
        const dim3 grid((B + kRaysPerBlock - 1) / kRaysPerBlock), block(64 * kRaysPerBlock);
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        auto timeit = [&](const char* name, auto launch) {
            for (int i = 0; i < 5; ++i) launch();
            hipEventRecord(e0);
            for (int i = 0; i < 50; ++i) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("B=%5d %-28s %7.2f us\n", B, name, 1e3f * ms / 50);
        };
        timeit("entry point (full)", [&] { nr_sample_hierarchical(dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd, nullptr); });
        timeit("variant full", [&] { hipLaunchKernelGGL((sh_var<true, true, true, true, true>), grid, block, lds, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd); });
        timeit("no sort", [&] { hipLaunchKernelGGL((sh_var<true, true, true, false, true>), grid, block, lds, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd); });
        timeit("no cdf", [&] { hipLaunchKernelGGL((sh_var<true, false, true, true, true>), grid, block, lds, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd); });
        timeit("no invert", [&] { hipLaunchKernelGGL((sh_var<true, true, false, true, true>), grid, block, lds, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd); });
        timeit("no store", [&] { hipLaunchKernelGGL((sh_var<true, true, true, true, false>), grid, block, lds, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd); });
        timeit("no loads", [&] { hipLaunchKernelGGL((sh_var<false, true, true, true, true>), grid, block, lds, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd); });
        timeit("loads+store only", [&] { hipLaunchKernelGGL((sh_var<true, false, false, false, true>), grid, block, lds, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd); });
        {
            std::vector<float> r1(size_t(B) * T), r2(size_t(B) * T), p1(size_t(B) * T * 3), p2(size_t(B) * T * 3);
            nr_sample_hierarchical(dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd, nullptr);
            hipMemcpy(r1.data(), dzf, r1.size() * 4, hipMemcpyDeviceToHost);
            hipMemcpy(p1.data(), dpts, p1.size() * 4, hipMemcpyDeviceToHost);
            const size_t lds2 = sizeof(float) * kRaysPerBlock * (3 * (Nc - 1) + 64);
            hipLaunchKernelGGL(sh_reg2<4>, grid, block, lds2, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd);
            hipMemcpy(r2.data(), dzf, r2.size() * 4, hipMemcpyDeviceToHost);
            hipMemcpy(p2.data(), dpts, p2.size() * 4, hipMemcpyDeviceToHost);
            size_t bad = 0;
            for (size_t i = 0; i < r1.size(); ++i) bad += r1[i] != r2[i];
            for (size_t i = 0; i < p1.size(); ++i) bad += p1[i] != p2[i];
            printf("B=%5d register sort: %zu mismatches\n", B, bad);
            timeit("register sort (runtime)", [&] { hipLaunchKernelGGL(sh_reg, grid, block, lds2, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd); });
            timeit("register sort (unrolled)", [&] { hipLaunchKernelGGL(sh_reg2<4>, grid, block, lds2, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd); });
        }
        timeit("empty (loads only)", [&] { hipLaunchKernelGGL((sh_var<true, false, false, false, false>), grid, block, lds, 0, dro, drd, dzc, dwc, du, B, Nc, Nf, dzf, dpts, dvd); });
    }
    return 0;
}
