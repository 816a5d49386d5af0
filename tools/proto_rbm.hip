// Structural prototype (timing only, no numerics) of a ROW-BLOCK-MAJOR fused-MLP
// forward: a stream chunk is RB row blocks x all 8 k blocks of one 256x256 layer
// (16 KB per row block), so a row block's accumulator is final after its 16
// MFMAs and its epilogue (bias MFMA, bf16 packing, ReLU, mask bits) runs while
// the next row block multiplies.  The layer input h_{i-1} (8 blocks, 64 VGPRs)
// and the output h_i being built stay in registers (ping-pong over two layers);
// LDS holds only the weight ring (NS slots).  EPI = 0 drops the epilogue work.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -DRB=1 -DNS=3 proto_rbm.hip
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
#ifndef RB
#define RB 1
#endif
#ifndef EPI
#define EPI 1
#endif
#ifndef PD
#define PD 3
#endif
#ifndef STORE
#define STORE 0  // training: store each finished output block (2 x 1 KB per wave, non-temporal)
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kChunk = RB * 16384;
constexpr int kWaves = NT / 64;
constexpr int kPieces = kChunk / 1024 / kWaves;
constexpr int kRing = PD + 1;

__device__ __forceinline__ uint32_t lane16() {
    uint32_t v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\tv_lshlrev_b32 %0, 4, %0" : "=v"(v));
    return v;
}
template <int OFF>
__device__ __forceinline__ void dsr(bf16x8& d, uint32_t a) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "i"(OFF));
}
#define DSR(d, a, off) \
    switch (off) { case 0: dsr<0>(d, a); break; case 1: dsr<1024>(d, a); break; case 2: dsr<2048>(d, a); break; \
        case 3: dsr<3072>(d, a); break; case 4: dsr<4096>(d, a); break; case 5: dsr<5120>(d, a); break; \
        case 6: dsr<6144>(d, a); break; case 7: dsr<7168>(d, a); break; case 8: dsr<8192>(d, a); break; \
        case 9: dsr<9216>(d, a); break; case 10: dsr<10240>(d, a); break; case 11: dsr<11264>(d, a); break; \
        case 12: dsr<12288>(d, a); break; case 13: dsr<13312>(d, a); break; case 14: dsr<14336>(d, a); break; \
        default: dsr<15360>(d, a); break; }
#define LGK(n) case n: asm volatile("s_waitcnt lgkmcnt(" #n ")" : "+v"(a)); break;
__device__ __forceinline__ void lgkm(int n, bf16x8& a) {
    switch (n) { LGK(0) LGK(1) LGK(2) LGK(3) LGK(4) LGK(5) LGK(6) default: asm volatile("s_waitcnt lgkmcnt(7)" : "+v"(a)); }
}
__device__ __forceinline__ unsigned relu_pk(unsigned w) {
    unsigned r;
    asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(w));
    return r;
}
__device__ __forceinline__ unsigned nz_pk(unsigned w) {
    unsigned r;
    asm("v_pk_min_u16 %0, %1, 1" : "=v"(r) : "v"(w));
    return r;
}

// epilogue of one finished row block: bias by MFMA, pack to bf16, ReLU, mask bits
__device__ __forceinline__ void epi(f32x16& a, bf16x8 (&o)[2], const bf16x8& bias, const bf16x8& ones, unsigned& mw,
                                    int sh) {
    a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bias, ones, a, 0, 0, 0);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        u32x4 w;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            unsigned p;
            asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(p) : "v"(a[8 * hf + 2 * m]), "v"(a[8 * hf + 2 * m + 1]));
            p = relu_pk(p);
            mw |= nz_pk(p) << (sh + 4 * hf + m);
            w[m] = p;
        }
        o[hf] = __builtin_bit_cast(bf16x8, w);
    }
}

__global__ __launch_bounds__(NT, 1) void proto(const char* __restrict__ wts, int nlayers, int reps, float* out,
                                               char* sink) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t l16 = lane16();
    const uint32_t lbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds)) + l16;
    bf16x8 hA[8][2], hB[8][2];
    for (int b = 0; b < 8; ++b)
        for (int f = 0; f < 2; ++f)
            for (int j = 0; j < 8; ++j) {
                hA[b][f][j] = static_cast<__bf16>(0.001f * (threadIdx.x + j + b));
                hB[b][f][j] = hA[b][f][j];
            }
    bf16x8 bias, ones;
    for (int j = 0; j < 8; ++j) {
        bias[j] = static_cast<__bf16>(0.01f * j);
        ones[j] = static_cast<__bf16>(1.f);
    }
    unsigned mw = 0;
    const int nchunk = nlayers * 8 / RB;  // weight chunks per pass
    const int total = nchunk * reps;
    auto dma = [&](int q) {
        const char* src = wts + static_cast<size_t>(q % nchunk) * kChunk + l16;
        char* slot = lds + (q % NS) * kChunk;
#pragma unroll
        for (int p = 0; p < kPieces; ++p) {
            const int pc = wv + p * kWaves;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + pc * 1024),
                                             (__attribute__((address_space(3))) void*)(slot + pc * 1024), 16, 0, 0);
        }
    };
    for (int q = 0; q < NS - 1; ++q) dma(q);
    int q = 0;
    char* sk = sink + (static_cast<size_t>(blockIdx.x) * kWaves + wv) * 16384 + l16;
    f32x16 acc[2];
    for (int e = 0; e < 16; ++e) acc[0][e] = acc[1][e] = 0.f;
    // one layer: 8 row blocks, input hin, output hout
    auto layer = [&](bf16x8 (&hin)[8][2], bf16x8 (&hout)[8][2]) {
        // current / previous row block (EPI = 0: two running sums)
#pragma unroll
        for (int rb = 0; rb < 8; ++rb) {
            const int sub = rb % RB;
            if (sub == 0) {
                // chunk q landed (NS-2 younger chunks may be in flight), previous slot free
                if constexpr (NS == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                else if constexpr (NS == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPieces) : "memory");
                else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kPieces) : "memory");
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                if (q + NS - 1 < total) dma(q + NS - 1);
            }
            const uint32_t slot = lbase + (q % NS) * kChunk + sub * 16384;
            f32x16& a = acc[rb & 1];
            if (EPI)
#pragma unroll
                for (int e = 0; e < 16; ++e) a[e] = 0.f;
            bf16x8 fa[kRing];
#pragma unroll
            for (int k = 0; k < PD; ++k) DSR(fa[k], slot, k)
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (k + PD < 16) DSR(fa[(k + PD) % kRing], slot, k + PD)
                bf16x8 x = fa[k % kRing];
                lgkm(k + PD < 16 ? PD : 15 - k, x);
                a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, hin[k >> 1][k & 1], a, 0, 0, 0);
                if (EPI && rb > 0 && k == 4) {
                    epi(acc[(rb - 1) & 1], hout[rb - 1], bias, ones, mw, 8 * ((rb - 1) & 1));
                    if (STORE) {
                        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, hout[rb - 1][0]),
                                                    reinterpret_cast<u32x4*>(sk + (rb - 1) * 2048));
                        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, hout[rb - 1][1]),
                                                    reinterpret_cast<u32x4*>(sk + (rb - 1) * 2048 + 1024));
                    }
                }
            }
            if (sub == RB - 1) ++q;
        }
        if (EPI) epi(acc[1], hout[7], bias, ones, mw, 8);
        // the layer's mask word is consumed (stored, in the real kernel) at the layer end
        asm volatile("" ::"v"(mw));
        mw = 0;
    };
    for (int it = 0; it < total / 8 * RB; it += 2) {
        layer(hA, hB);
        layer(hB, hA);
    }
    float s = 0.f;
    for (int b = 0; b < 8; ++b)
        for (int j = 0; j < 8; ++j) s += static_cast<float>(hA[b][0][j]);
    for (int e = 0; e < 16; ++e) s += acc[0][e] + acc[1][e];
    out[blockIdx.x * NT + threadIdx.x] = s + mw;
}

int main(int argc, char** argv) {
    const int nlayers = 10, reps = argc > 1 ? atoi(argv[1]) : 24;
    const int grid = argc > 2 ? atoi(argv[2]) : 256;
    const size_t nchunk = nlayers * 8 / RB;
    std::vector<unsigned short> h(nchunk * kChunk / 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3c00 + (i % 64);
    char *w, *sink;
    float* out;
    (void)hipMalloc(&w, h.size() * 2);
    (void)hipMalloc(&out, static_cast<size_t>(grid) * NT * 4);
    (void)hipMalloc(&sink, static_cast<size_t>(grid) * kWaves * 16384);
    (void)hipMemcpy(w, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    const size_t lds = static_cast<size_t>(NS) * kChunk;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int it = 0; it < 3; ++it) proto<<<grid, NT, lds>>>(w, nlayers, reps, out, sink);
    (void)hipEventRecord(a);
    const int iters = 10;
    for (int it = 0; it < iters; ++it) proto<<<grid, NT, lds>>>(w, nlayers, reps, out, sink);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= iters;
    // useful MFMAs only (the bias MFMA is overhead)
    const double mfma = static_cast<double>(grid) * kWaves * nchunk * RB * reps * 16;
    const double flop = mfma * 32 * 32 * 16 * 2;
    const double per_simd = mfma / (grid / 256.0 * 256 * 4);
    printf("RBM RB=%d NS=%d EPI=%d PD=%d STORE=%d NT=%d: %.3f ms  %.1f TF/s  %.1f cyc/MFMA@2.4GHz\n", RB, NS, EPI, PD,
           STORE, NT, ms, flop / ms / 1e9, ms * 1e-3 * 2.4e9 / per_simd);
    return 0;
}
