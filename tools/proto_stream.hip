// Structural prototype of the fused-MLP weight stream (timing only, no numerics):
// a workgroup streams NQ chunks of 16 KB bf16 A fragments (8 row blocks x 2
// k-steps) through an LDS ring of NS slots (LDS-DMA, counted vmcnt, raw
// s_barrier); each wave applies every fragment to TPW 32-sample tiles whose B
// operands sit in registers.  Prints cycles per MFMA and TF/s.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -DNT=256 -DTPW=2 ... proto_stream.hip -o proto
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef NT
#define NT 512
#endif
#ifndef TPW
#define TPW 1
#endif
#ifndef NS
#define NS 2
#endif
#ifndef PD
#define PD 2
#endif
#ifndef BARRIER
#define BARRIER 1
#endif
#ifndef DMA
#define DMA 1
#endif
#ifndef GROUPS
#define GROUPS 1
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kChunk = 16384, kWaves = NT / 64, kPieces = kChunk / 1024 / kWaves;

__device__ __forceinline__ uint32_t lane16() {
    uint32_t v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\tv_lshlrev_b32 %0, 4, %0" : "=v"(v));
    return v;
}

__global__ __launch_bounds__(NT, 1) void proto(const char* __restrict__ w, int nq, int reps, float* out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    f32x16 acc[TPW][8];
    bf16x8 b[TPW][2];
    for (int t = 0; t < TPW; ++t) {
        for (int j = 0; j < 8; ++j) {
            b[t][0][j] = static_cast<__bf16>(0.001f * (threadIdx.x + j + t));
            b[t][1][j] = static_cast<__bf16>(0.002f * (threadIdx.x + j));
        }
        for (int r = 0; r < 8; ++r)
            for (int e = 0; e < 16; ++e) acc[t][r][e] = 0.f;
    }
    const int total = nq * reps;
    auto dma = [&](int q) {
        const char* src = w + static_cast<size_t>(q % nq) * kChunk + lane16();
        char* slot = lds + (q % NS) * kChunk;
#pragma unroll
        for (int p = 0; p < kPieces; ++p) {
            const int pc = wv + p * kWaves;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + pc * 1024),
                                             (__attribute__((address_space(3))) void*)(slot + pc * 1024), 16, 0, 0);
        }
    };
#if DMA
    for (int q = 0; q < NS - 1; ++q) dma(q);
#endif
    for (int q = 0; q < total; ++q) {
#if DMA
        // chunk q must have landed: NS-2 younger chunks may stay in flight
        if constexpr (NS == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if constexpr (NS == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPieces) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kPieces) : "memory");
#endif
#if BARRIER
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#endif
#if DMA
        if (q + NS - 1 < total) dma(q + NS - 1);
#endif
        const char* slot = lds + (q % NS) * kChunk + lane16();
        bf16x8 fa[8][2];
#pragma unroll
        for (int r = 0; r < PD; ++r) {
            fa[r][0] = *reinterpret_cast<const bf16x8*>(slot + r * 2048);
            fa[r][1] = *reinterpret_cast<const bf16x8*>(slot + r * 2048 + 1024);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if (r + PD < 8) {
                fa[r + PD][0] = *reinterpret_cast<const bf16x8*>(slot + (r + PD) * 2048);
                fa[r + PD][1] = *reinterpret_cast<const bf16x8*>(slot + (r + PD) * 2048 + 1024);
            }
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                acc[t][r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[r][0], b[t][0], acc[t][r], 0, 0, 0);
                acc[t][r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[r][1], b[t][1], acc[t][r], 0, 0, 0);
            }
        }
#if GROUPS
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * PD, 0);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2 * TPW, 0);
            if (r + PD < 8) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
#endif
    }
    float s = 0.f;
    for (int t = 0; t < TPW; ++t)
        for (int r = 0; r < 8; ++r)
            for (int e = 0; e < 16; ++e) s += acc[t][r][e];
    out[blockIdx.x * NT + threadIdx.x] = s;
}

int main(int argc, char** argv) {
    const int nq = 77, reps = argc > 1 ? atoi(argv[1]) : 24;
    const int grid = argc > 2 ? atoi(argv[2]) : 256;
    std::vector<unsigned short> h(static_cast<size_t>(nq) * kChunk / 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3c00 + (i % 64);
    char* w;
    float* out;
    hipMalloc(&w, h.size() * 2);
    hipMalloc(&out, static_cast<size_t>(grid) * NT * 4);
    hipMemcpy(w, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    const size_t lds = static_cast<size_t>(NS) * kChunk;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int it = 0; it < 3; ++it) proto<<<grid, NT, lds>>>(w, nq, reps, out);
    hipEventRecord(a);
    const int iters = 10;
    for (int it = 0; it < iters; ++it) proto<<<grid, NT, lds>>>(w, nq, reps, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= iters;
    const double mfma = static_cast<double>(grid) * kWaves * nq * reps * 16 * TPW;
    const double flop = mfma * 32 * 32 * 16 * 2;
    // cycles per MFMA per SIMD at 2.4 GHz (per CU: 4 SIMDs; grid/256 workgroups per CU)
    const double per_simd = mfma / (grid / 256.0 * 256 * 4);
    printf("NT=%d TPW=%d NS=%d PD=%d BAR=%d DMA=%d GROUPS=%d: %.3f ms  %.1f TF/s  %.1f cyc/MFMA@2.4GHz\n", NT, TPW, NS,
           PD, BARRIER, DMA, GROUPS, ms, flop / ms / 1e9, ms * 1e-3 * 2.4e9 / per_simd);
    return 0;
}
