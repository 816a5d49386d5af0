// Structural prototype (timing only, no numerics) of the fused-MLP weight stream
// with the workgroup barrier moved INSIDE a step: at row block MID of step s every
// wave waits for step s+1's LDS-DMA and barriers; then it issues the DMA of step
// s+2 (NS = 3 slots: that slot held step s-1, which every wave has finished) and
// may already read step s+1's A fragments while row blocks MID..7 of step s
// multiply.  MID = -1 is the current scheme (NS = 2, barrier + lgkmcnt(0) between
// steps, then the pipe refills).  A step is FH k16-halves of all 8 row blocks
// (FH = 2: 16-KB chunk, FH = 1: 8-KB half chunk).  BLDS = 1 reads the B operand
// (activations) from the wave's own LDS region, as the real forward does.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -DMID=4 -DNS=3 -DF=1 proto_midbar.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef NT
#define NT 512
#endif
#ifndef NS
#define NS 3
#endif
#ifndef MID
#define MID 4
#endif
#ifndef FH
#define FH 1
#endif
#ifndef BLDS
#define BLDS 1
#endif
#ifndef BARRIER
#define BARRIER 1
#endif
#ifndef VALU
#define VALU 0  // extra v_fma per row block (epilogue-like filler)
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kPD = 3;                          // A prefetch distance in row blocks (ring of 4)
constexpr int kStep = 8 * FH * 1024;             // bytes per step
constexpr int kWaves = NT / 64;
constexpr int kPieces = kStep / 1024 / kWaves;  // LDS-DMA pieces per wave per step
constexpr int kBRegion = 8 * 2 * 1024;          // per-wave activation image (16 KB)
static_assert(kPieces >= 1, "pieces");

__device__ __forceinline__ uint32_t lane16() {
    uint32_t v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\tv_lshlrev_b32 %0, 4, %0" : "=v"(v));
    return v;
}
__device__ __forceinline__ void dsr(bf16x8& d, uint32_t a) { asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(a)); }
#define LGK(n, ...) case n: asm volatile("s_waitcnt lgkmcnt(" #n ")" : __VA_ARGS__); break;
// n is a compile-time constant after unrolling: the switch folds away
__device__ __forceinline__ void lgkm(int n, bf16x8& a) {
    switch (n) { LGK(0, "+v"(a)) LGK(1, "+v"(a)) LGK(2, "+v"(a)) LGK(3, "+v"(a)) LGK(4, "+v"(a)) LGK(5, "+v"(a))
                 LGK(6, "+v"(a)) LGK(7, "+v"(a)) default: asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(a)); }
}
__device__ __forceinline__ void lgkm3(int n, bf16x8& a, bf16x8& b0, bf16x8& b1) {
    switch (n) { LGK(0, "+v"(a), "+v"(b0), "+v"(b1)) LGK(1, "+v"(a), "+v"(b0), "+v"(b1)) LGK(2, "+v"(a), "+v"(b0), "+v"(b1))
                 LGK(3, "+v"(a), "+v"(b0), "+v"(b1)) LGK(4, "+v"(a), "+v"(b0), "+v"(b1)) LGK(5, "+v"(a), "+v"(b0), "+v"(b1))
                 LGK(6, "+v"(a), "+v"(b0), "+v"(b1))
                 default: asm volatile("s_waitcnt lgkmcnt(7)" : "+v"(a), "+v"(b0), "+v"(b1)); }
}

// LDS reads issued after A(row r)'s reads and before its use (see the schedule below)
constexpr int younger(int r) { return kPD * FH + ((BLDS && r >= 4 && r - kPD <= 4) ? FH : 0); }

__global__ __launch_bounds__(NT, 1) void proto(const char* __restrict__ w, int nsteps, int reps, float* out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t l16 = lane16();
    const uint32_t lbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds));
    const uint32_t breg = lbase + NS * kStep + wv * kBRegion + l16;
    f32x16 acc[8];
    for (int r = 0; r < 8; ++r)
        for (int e = 0; e < 16; ++e) acc[r][e] = 0.f;
    bf16x8 b[FH], bn[FH];
    for (int f = 0; f < FH; ++f)
        for (int j = 0; j < 8; ++j) b[f][j] = bn[f][j] = static_cast<__bf16>(0.001f * (threadIdx.x + j + f));
    const int total = nsteps * reps;
    auto dma = [&](int s) {
        const char* src = w + static_cast<size_t>(s % nsteps) * kStep + l16;
        char* slot = lds + (s % NS) * kStep;
#pragma unroll
        for (int p = 0; p < kPieces; ++p) {
            const int pc = wv + p * kWaves;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + pc * 1024),
                                             (__attribute__((address_space(3))) void*)(slot + pc * 1024), 16, 0, 0);
        }
    };
    bf16x8 fa[kPD + 1][FH];
    // prologue: steps 0 (and 1 for MID >= 0) landed and published, A(0..PD-1) of step 0 in flight
    dma(0);
    if (MID >= 0) dma(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPD; ++r)
#pragma unroll
        for (int f = 0; f < FH; ++f) dsr(fa[r][f], lbase + r * FH * 1024 + f * 1024 + l16);
    for (int s = 0; s < total; ++s) {
        const uint32_t cur = lbase + (s % NS) * kStep + l16;
        const uint32_t nxt = lbase + ((s + 1) % NS) * kStep + l16;
        if (MID < 0) {
            // current scheme: chunk s+1 issued now into the other slot (NS = 2)
            if (s + 1 < total) dma(s + 1);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if (MID >= 0 && r == MID) {
                if (BARRIER) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    asm volatile("" ::: "memory");
                }
                if (s + 2 < total) dma(s + 2);
            }
            // prefetch A of row r + PD (next step once past the barrier)
            const int rp = r + kPD;
            if (rp < 8) {
#pragma unroll
                for (int f = 0; f < FH; ++f) dsr(fa[rp % (kPD + 1)][f], cur + rp * FH * 1024 + f * 1024);
            } else if (MID >= 0 && r >= MID) {
#pragma unroll
                for (int f = 0; f < FH; ++f) dsr(fa[rp % (kPD + 1)][f], nxt + (rp - 8) * FH * 1024 + f * 1024);
            }
            if (BLDS && r == 4)
#pragma unroll
                for (int f = 0; f < FH; ++f) dsr(bn[f], breg + ((s + 1) % 8) * 2048 + f * 1024);
            bf16x8 a0 = fa[r % (kPD + 1)][0];
            if (BLDS && r == 0) {
                // B of this step (read at row 4 of the previous one) is older than A(0)
                lgkm3(younger(0) + FH - 1, a0, bn[0], bn[FH - 1]);
#pragma unroll
                for (int f = 0; f < FH; ++f) b[f] = bn[f];
            } else {
                lgkm(younger(r) + FH - 1, a0);
            }
            acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[0], acc[r], 0, 0, 0);
            if (FH == 2) {
                bf16x8 a1 = fa[r % (kPD + 1)][FH - 1];
                lgkm(younger(r), a1);
                acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[FH - 1], acc[r], 0, 0, 0);
            }
            if (VALU) {
#pragma unroll
                for (int e = 0; e < VALU; ++e) acc[(r + 4) & 7][e] = acc[(r + 4) & 7][e] * 0.999f + 1e-7f;
            }
        }
        if (MID < 0) {
            // drain, publish chunk s+1, refill the A ring from it
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (BARRIER) __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
#pragma unroll
            for (int r = 0; r < kPD; ++r)
#pragma unroll
                for (int f = 0; f < FH; ++f) dsr(fa[r][f], nxt + r * FH * 1024 + f * 1024);
        }
    }
    float sum = 0.f;
    for (int r = 0; r < 8; ++r)
        for (int e = 0; e < 16; ++e) sum += acc[r][e];
    out[blockIdx.x * NT + threadIdx.x] = sum;
}

int main(int argc, char** argv) {
    const int nsteps = 77 * 2 / FH, reps = argc > 1 ? atoi(argv[1]) : 24;
    const int grid = argc > 2 ? atoi(argv[2]) : 256;
    std::vector<unsigned short> h(static_cast<size_t>(nsteps) * kStep / 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3c00 + (i % 64);
    char* w;
    float* out;
    hipMalloc(&w, h.size() * 2);
    hipMalloc(&out, static_cast<size_t>(grid) * NT * 4);
    hipMemcpy(w, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    const size_t lds = static_cast<size_t>(NS) * kStep + (BLDS ? kWaves * kBRegion : 0);
    if (lds > 163840) {
        printf("MID=%d NS=%d FH=%d BLDS=%d: LDS %zu too large\n", MID, NS, FH, BLDS, lds);
        return 0;
    }
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int it = 0; it < 3; ++it) proto<<<grid, NT, lds>>>(w, nsteps, reps, out);
    hipEventRecord(a);
    const int iters = 10;
    for (int it = 0; it < iters; ++it) proto<<<grid, NT, lds>>>(w, nsteps, reps, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= iters;
    const double mfma = static_cast<double>(grid) * kWaves * nsteps * reps * 8 * FH;
    const double flop = mfma * 32 * 32 * 16 * 2;
    const double per_simd = mfma / (grid / 256.0 * 256 * 4);
    printf("MID=%d NS=%d FH=%d BLDS=%d BAR=%d VALU=%d NT=%d: %.3f ms  %.1f TF/s  %.1f cyc/MFMA@2.4GHz\n", MID, NS, FH,
           BLDS, BARRIER, VALU, NT, ms, flop / ms / 1e9, ms * 1e-3 * 2.4e9 / per_simd);
    return 0;
}
