// Microbenchmark (prototype, not product): issue rate of v_mfma_f32_32x32x16_bf16 when
// consecutive MFMAs accumulate into the SAME accumulator (one dependent chain per wave)
// vs alternating between 2 or 4 accumulators, at 1 and 2 waves per SIMD.  Prints cycles
// per MFMA per SIMD.  hipcc --offload-arch=gfx950 -O3 tools/proto_mfma_chain.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int NACC>
__global__ __launch_bounds__(512) void chain(const bf16x8* in, float* out, int iters, long long* cyc) {
    bf16x8 a = in[threadIdx.x & 63], b = in[(threadIdx.x + 7) & 63];
    f32x16 acc[NACC];
    for (int k = 0; k < NACC; ++k)
        for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;
    __syncthreads();
    long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j % NACC] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j % NACC], 0, 0, 0);
    }
    __syncthreads();
    long long t1 = __builtin_readcyclecounter();
    float s = 0.f;
    for (int k = 0; k < NACC; ++k)
        for (int r = 0; r < 16; ++r) s += acc[k][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NACC>
void run(int threads, const bf16x8* in, float* out, long long* cyc, int cus) {
    const int iters = 2000;
    hipLaunchKernelGGL(chain<NACC>, dim3(cus), dim3(threads), 0, 0, in, out, iters, cyc);
    hipDeviceSynchronize();
    long long h[1024];
    hipMemcpy(h, cyc, sizeof(long long) * cus, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < cus; ++i) avg += h[i];
    avg /= cus;
    const int waves_per_simd = threads / 64 / 4;
    // per SIMD: waves_per_simd x iters x 16 MFMAs; readcyclecounter ticks at the shader clock
    printf("accumulators %d, %d wave(s)/SIMD: %.1f cycles per MFMA per SIMD\n", NACC, waves_per_simd,
           avg / (double(iters) * 16 * waves_per_simd));
}

int main() {
    bf16x8* in;
    float* out;
    long long* cyc;
    hipMalloc(&in, 64 * sizeof(bf16x8));
    hipMemset(in, 0, 64 * sizeof(bf16x8));
    hipMalloc(&out, 1024 * 512 * sizeof(float));
    hipMalloc(&cyc, 1024 * sizeof(long long));
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int threads : {256, 512}) {
        run<1>(threads, in, out, cyc, cus);
        run<2>(threads, in, out, cyc, cus);
        run<4>(threads, in, out, cyc, cus);
    }
    return 0;
}
