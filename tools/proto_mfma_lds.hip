// Microbenchmark (prototype, not product): MFMA issue rate when every
// v_mfma_f32_32x32x16_bf16 takes its A operand from LDS (one ds_read_b128 per lane per
// MFMA, read PD items ahead, counted lgkmcnt waits) -- the forward kernel's inner loop
// without its epilogues, stores or weight DMA -- at 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int OFF>
__device__ __forceinline__ void dsr(bf16x8& d, unsigned a) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "i"(OFF));
}
template <int N>
__device__ __forceinline__ void lgkm(bf16x8& a) {
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "n"(N));
}

template <int PD>
__global__ __launch_bounds__(512) void k(const bf16x8* in, float* out, int iters, long long* cyc) {
    __shared__ bf16x8 lds[16 * 64];  // 16 KB: 16 fragments of 1 KB
    for (int i = threadIdx.x; i < 16 * 64; i += blockDim.x) lds[i] = in[i & 63];
    bf16x8 b = in[(threadIdx.x + 7) & 63];
    f32x16 acc[2];
    for (int q = 0; q < 2; ++q)
        for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
    __syncthreads();
    const unsigned base = static_cast<unsigned>(reinterpret_cast<uintptr_t>(lds)) + (threadIdx.x & 63) * 16;
    long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) {
        bf16x8 fa[PD + 1];
        // prologue: PD reads in flight
        if constexpr (PD >= 1) dsr<0 * 1024>(fa[0], base);
        if constexpr (PD >= 2) dsr<1 * 1024>(fa[1], base);
        if constexpr (PD >= 3) dsr<2 * 1024>(fa[2], base);
        if constexpr (PD >= 4) dsr<3 * 1024>(fa[3], base);
#define STEP(j)                                                                                     \
    {                                                                                               \
        if constexpr (j + PD < 16) dsr<((j + PD) % 16) * 1024>(fa[(j + PD) % (PD + 1)], base);       \
        constexpr int younger = (16 - 1 - j) < PD ? (16 - 1 - j) : PD;                              \
        lgkm<younger>(fa[j % (PD + 1)]);                                                            \
        acc[(j / 8) & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[j % (PD + 1)], b, acc[(j / 8) & 1], 0, 0, 0); \
    }
        STEP(0) STEP(1) STEP(2) STEP(3) STEP(4) STEP(5) STEP(6) STEP(7)
        STEP(8) STEP(9) STEP(10) STEP(11) STEP(12) STEP(13) STEP(14) STEP(15)
#undef STEP
    }
    __syncthreads();
    long long t1 = __builtin_readcyclecounter();
    float s = 0.f;
    for (int q = 0; q < 2; ++q)
        for (int r = 0; r < 16; ++r) s += acc[q][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int PD>
void run(int threads, const bf16x8* in, float* out, long long* cyc, int cus) {
    const int iters = 2000;
    hipLaunchKernelGGL(k<PD>, dim3(cus), dim3(threads), 0, 0, in, out, iters, cyc);
    hipDeviceSynchronize();
    long long h[1024];
    (void)hipMemcpy(h, cyc, sizeof(long long) * cus, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < cus; ++i) avg += h[i];
    avg /= cus;
    const int wps = threads / 64 / 4;
    printf("PD %d, %d wave(s)/SIMD: %.1f cycles per MFMA per SIMD\n", PD, wps, avg / (double(iters) * 16 * wps));
}

int main() {
    bf16x8* in;
    float* out;
    long long* cyc;
    (void)hipMalloc(&in, 64 * sizeof(bf16x8));
    (void)hipMemset(in, 0, 64 * sizeof(bf16x8));
    (void)hipMalloc(&out, 1024 * 512 * sizeof(float));
    (void)hipMalloc(&cyc, 1024 * sizeof(long long));
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int threads : {256, 512}) {
        run<1>(threads, in, out, cyc, cus);
        run<2>(threads, in, out, cyc, cus);
        run<3>(threads, in, out, cyc, cus);
        run<4>(threads, in, out, cyc, cus);
    }
    return 0;
}
