// Fused NeRF MLP on MFMA (gfx950): weight packing, training/inference forward,
// backward dX chain, and the dW GEMM with a deterministic split-M reduction.
//
// Reference: noisy_src/model.py:20-221 — PositionalEncoding (no pi), 8x256 ReLU
// trunk with skip cat([x_enc, h]) after layer 4, sigma = relu(W h), feat = W h
// (no activation), h_c = relu(W [feat, d_enc]), rgb = sigmoid(W h_c).
//
// Formulation.  Every layer computes out^T = W . in^T on 32-sample tiles.  In
// the MFMA C/D layout a lane holds 16 features of ONE sample, so a layer's
// accumulator tile is already the next layer's B operand (packed to bf16, or
// as-is in fp32): activations stay in registers through the whole network.
// The A operand (weights) is a packed image whose per-lane 16 bytes per MFMA
// are contiguous, with the k order permuted to match the accumulator rows:
//   bf16 32x32x16, k-step s: element j <-> input feature 16s + 8(j>>2) + 4h + (j&3)
//   fp32 32x32x2,  k-step t: lane half h <-> input feature (t&3) + 8(t>>2) + 4h
// The images are chunk-major (a chunk = all row blocks of one k block) and are
// streamed through an LDS double buffer shared by the workgroup's 4 waves;
// each wave applies every fragment to TPW sample tiles.
//
// Training saves activations (and the backward its dz) as B-operand images:
// per tile and 32-feature block, FPB wave-wide 1-KB fragments, so each store
// is one coalesced 1-KB wave write.  The dW GEMM reduces over samples, i.e.
// over the lanes of those images; it stages whole tiles in LDS (LDS-DMA) and
// rebuilds sample-major operands with the gfx950 transpose read
// ds_read_b64_tr_b16 (bf16) or strided ds_read_b32 (fp32).
#include <cmath>
#include <cstring>
#include <type_traits>
#include <utility>

#include "common.hpp"
#include "mfma.hpp"
#include "mlp_plan.hpp"
#include "optim.hpp"

#include "mlp_plan.cpp.inc"

namespace nr {

// 16-bit MFMA operands (bf16 or fp16; both stored as 16-bit patterns in bf16x8
// registers, the MFMA and the conversions pick the format) or fp32.
template <int PREC>
constexpr bool k16 = PREC != NR_PREC_FP32;

template <int PREC>
struct InBlk {
    bf16x8 s[2];
};
template <>
struct InBlk<NR_PREC_FP32> {
    f32x16 v;
};

template <int PREC>
constexpr int kFPB = k16<PREC> ? 2 : 4;  // 1-KB fragments per 32x32 block

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// fp16 backward runs on dz scaled by 2^14 (the per-sample gradients of a mean
// loss over 4096 rays sit near 1e-6, in fp16's subnormal range); the dW reduce and
// the input gradients divide it out exactly.
inline float grad_scale(int prec) { return prec == NR_PREC_FP16 ? 16384.0f : 1.0f; }

// D += A.B on 16-bit operand images of either format
template <int PREC>
__device__ __forceinline__ f32x16 mfma16(bf16x8 a, bf16x8 b, f32x16 c) {
    if constexpr (PREC == NR_PREC_FP16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                      0, 0, 0);
    else
        return mfma_bf16(a, b, c);
}

// Two fp32 -> one word of two bf16 (RNE), low half = lo: one v_cvt_pk_bf16_f32
// (element-wise casts compile to one convert per element plus a v_perm per pair;
// not inline asm: the hazard recognizer does not see an asm def that an MFMA reads).
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned cvt_pk_bf16(float lo, float hi) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{lo, hi}, bf16x2));
}
template <int PREC>
__device__ __forceinline__ unsigned cvt_pk16(float lo, float hi) {
    if constexpr (PREC == NR_PREC_FP16)
        return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{lo, hi}, f16x2));
    else
        return cvt_pk_bf16(lo, hi);
}
// 16-bit pattern of x (round to nearest even)
template <int PREC>
__device__ __forceinline__ float from16_lo(unsigned w) {
    if constexpr (PREC == NR_PREC_FP16)
        return static_cast<float>(__builtin_bit_cast(f16x2, w)[0]);
    else
        return __uint_as_float(w << 16);
}

// registers 8 hf .. 8 hf + 7 of an accumulator as a 16-bit operand
template <int PREC = NR_PREC_BF16>
__device__ __forceinline__ bf16x8 pack8(const f32x16& a, int hf) {
    u32x4 w;
#pragma unroll
    for (int m = 0; m < 4; ++m) w[m] = cvt_pk16<PREC>(a[8 * hf + 2 * m], a[8 * hf + 2 * m + 1]);
    return __builtin_bit_cast(bf16x8, w);
}

template <int PREC>
__device__ __forceinline__ void to_in(const f32x16& a, InBlk<PREC>& o) {
    if constexpr (k16<PREC>) {
        o.s[0] = pack8<PREC>(a, 0);
        o.s[1] = pack8<PREC>(a, 1);
    } else {
        o.v = a;
    }
}

__device__ __forceinline__ void zero(f32x16& a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = 0.f;
}

#ifndef NR_SIN
#define NR_SIN sinf
#define NR_COS cosf
#endif
// lane * 16 recomputed in place (2 VALU): lane-derived offsets are otherwise kept
// live across the whole kernel, and under register pressure spilled and
// reloaded with a vmcnt(0) that also drains the in-flight weight stream.
__device__ __forceinline__ uint32_t lane16() {
    uint32_t v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\tv_lshlrev_b32 %0, 4, %0" : "=v"(v));
    return v;
}

// Positional-encoding feature f of a 3-vector (model.py:72-80): [x | sin 2^0 x | cos 2^0 x | ...].
__device__ __forceinline__ float pe_feat(float x0, float x1, float x2, int f, int L) {
    if (f < 3) return f == 0 ? x0 : (f == 1 ? x1 : x2);
    const int fp = f - 3;
    const int k = fp / 6;
    if (k >= L) return 0.f;  // padding column
    const int rem = fp - 6 * k;
    const int c = rem % 3;
    const float xv = c == 0 ? x0 : (c == 1 ? x1 : x2);
    const float v = exp2f(static_cast<float>(k)) * xv;
    return rem < 3 ? NR_SIN(v) : NR_COS(v);
}

// d gamma_f / d x_c contracted with g (torch: (g * cos(fx)) * f, (g * -sin(fx)) * f).
__device__ __forceinline__ void pe_feat_bwd(float x0, float x1, float x2, int f, int L, float g, float& g0,
                                            float& g1, float& g2) {
    int c;
    float d;
    if (f < 3) {
        c = f;
        d = g;
    } else {
        const int fp = f - 3;
        const int k = fp / 6;
        if (k >= L) return;
        const int rem = fp - 6 * k;
        c = rem % 3;
        const float xv = c == 0 ? x0 : (c == 1 ? x1 : x2);
        const float fr = exp2f(static_cast<float>(k));
        const float v = fr * xv;
        d = rem < 3 ? (g * cosf(v)) * fr : (g * -sinf(v)) * fr;
    }
    // selects, not branches: the branches became a run-time-indexed scratch array
    g0 += c == 0 ? d : 0.f;
    g1 += c == 1 ? d : 0.f;
    g2 += c == 2 ? d : 0.f;
}

// bf16 positional encoding.  sin/cos by the hardware v_sin_f32 (argument in
// revolutions) after an exact two-term reduction: x/(2 pi) = hi + lo with
// hi = x*C1 rounded and lo = fma(x, C1, -hi) + x*C2, so 2^k x/(2 pi) mod 1 =
// fract(2^k hi) + 2^k lo (2^k hi exact).  Absolute error ~1e-6, far below the
// bf16 rounding (2^-9 relative) the encoding goes through; the fp32 path keeps
// sinf/cosf.  cos(v) = sin(v + 1/4 revolution).
#ifndef NR_EPI_HOOK
#define NR_EPI_HOOK 1  // 16-bit: layer epilogue overlapped with the last chunk's MFMAs
#endif
#ifndef NR_APF
#define NR_APF 3  // 16-bit weight-stream A fragments read ahead (row blocks)
#endif
#ifndef NR_NT_STORE
#define NR_NT_STORE 1
#endif
#ifndef NR_FASTPE
#define NR_FASTPE 1
#endif
#ifndef NR_BIASMFMA
#define NR_BIASMFMA 1
#endif
struct PeRev {
    float x[3], hi[3], lo[3];
};

__device__ __forceinline__ PeRev pe_rev(float x0, float x1, float x2) {
    constexpr float C1 = 0.15915494f, C2 = 6.4206382e-09f;  // fp32(1/2pi), 1/2pi - C1
    PeRev p;
    const float xs[3] = {x0, x1, x2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        p.x[c] = xs[c];
        p.hi[c] = xs[c] * C1;
        p.lo[c] = fmaf(xs[c], C1, -p.hi[c]) + xs[c] * C2;
    }
    return p;
}

// feature f (compile-time after unrolling) for lane half 0 and f1 for half 1
__device__ __forceinline__ float pe_fast(const PeRev& p, int f0, int f1, bool h1, int L) {
    auto kind = [](int f) { return f < 3 ? 0 : 1; };
    auto trig = [&](int f, float& hi, float& lo) {  // 2^k (hi, lo) + phase of feature f
        const int fp = f - 3, k = fp / 6, rem = fp - 6 * k, c = rem % 3;
        const float sc = static_cast<float>(1 << (k < 24 ? k : 0));
        hi = p.hi[c] * sc;
        lo = fmaf(p.lo[c], sc, rem < 3 ? 0.f : 0.25f);
        return k < L;
    };
    if (kind(f0) == 1 && kind(f1) == 1) {
        float h0, l0, hh, lh;
        const bool v0 = trig(f0, h0, l0), v1 = trig(f1, hh, lh);
        const float hi = h1 ? hh : h0, lo = h1 ? lh : l0;
        const float v = __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(hi) + lo);
        return (h1 ? v1 : v0) ? v : 0.f;
    }
    auto one = [&](int f) -> float {
        if (f < 3) return p.x[f];
        float hi, lo;
        const bool ok = trig(f, hi, lo);
        return ok ? __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(hi) + lo) : 0.f;
    };
    const float a0 = one(f0), a1 = one(f1);
    return h1 ? a1 : a0;
}

// Backward of pe_fast: d gamma_f / d x_c contracted with g, for feature f0 (lane
// half 0) / f1 (half 1).  d sin(theta + phi)/d theta = sin(theta + phi + 1/4 rev), so
// the derivative is the same hardware sine a quarter revolution on (sin -> cos,
// cos -> -sin), times 2^k.  16-bit paths only (the fp32 path keeps sinf/cosf).
__device__ __forceinline__ void pe_fast_bwd(const PeRev& p, int f0, int f1, bool h1, int L, float g, float& g0,
                                            float& g1, float& g2) {
    auto chan = [](int f) { return f < 3 ? f : ((f - 3) - 6 * ((f - 3) / 6)) % 3; };
    // selects: a run-time index into p.hi / p.lo put them in scratch
    auto sel = [](const float (&v)[3], int c) { return c == 0 ? v[0] : (c == 1 ? v[1] : v[2]); };
    auto live = [&](int f) { return f < 3 || (f - 3) / 6 < L; };
    auto dgamma = [&](int f) -> float {  // d gamma_f / d x_c (f >= 3, live)
        const int fp = f - 3, k = fp / 6, rem = fp - 6 * k, c = rem % 3;
        const float sc = static_cast<float>(1 << (k < 24 ? k : 0));
        const float hi = sel(p.hi, c) * sc, lo = fmaf(sel(p.lo, c), sc, rem < 3 ? 0.25f : 0.5f);
        return __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(hi) + lo) * sc;
    };
    float d;
    if (f0 >= 3 && f1 >= 3) {
        const int fp0 = f0 - 3, k0 = fp0 / 6, r0 = fp0 - 6 * k0;
        const int fp1 = f1 - 3, k1 = fp1 / 6, r1 = fp1 - 6 * k1;
        const float s0 = static_cast<float>(1 << (k0 < 24 ? k0 : 0)), s1 = static_cast<float>(1 << (k1 < 24 ? k1 : 0));
        const float hi = h1 ? sel(p.hi, r1 % 3) * s1 : sel(p.hi, r0 % 3) * s0;
        const float lo = h1 ? fmaf(sel(p.lo, r1 % 3), s1, r1 < 3 ? 0.25f : 0.5f) : fmaf(sel(p.lo, r0 % 3), s0, r0 < 3 ? 0.25f : 0.5f);
        d = g * (__builtin_amdgcn_sinf(__builtin_amdgcn_fractf(hi) + lo) * (h1 ? s1 : s0));
    } else {
        const float a0 = f0 < 3 ? 1.f : (live(f0) ? dgamma(f0) : 0.f);
        const float a1 = f1 < 3 ? 1.f : (live(f1) ? dgamma(f1) : 0.f);
        d = g * (h1 ? a1 : a0);
    }
    if (!(h1 ? live(f1) : live(f0))) return;
    const int c = h1 ? chan(f1) : chan(f0);
    g0 += c == 0 ? d : 0.f;
    g1 += c == 1 ? d : 0.f;
    g2 += c == 2 ? d : 0.f;
}

// ---- bf16 epilogue: bias by MFMA, ReLU and mask bits on packed bf16 pairs ----
// Bias of row block nb as an MFMA A fragment against an all-ones B operand:
// lanes 0..31 hold bias[32 nb + lane] split exactly into bf16 hi + mid + lo,
// lanes 32..63 zeros, so D += bias broadcast over the 32 samples of the tile.
template <int PREC>
__device__ __forceinline__ bf16x8 bias_frag(float b) {
    const unsigned w0 = cvt_pk16<PREC>(b, 0.f);            // hi
    const float r1 = b - from16_lo<PREC>(w0);
    const unsigned w1 = cvt_pk16<PREC>(r1, 0.f);           // mid
    const float r2 = r1 - from16_lo<PREC>(w1);
    const unsigned w2 = cvt_pk16<PREC>(r2, 0.f);           // lo
    return __builtin_bit_cast(bf16x8, u32x4{w0 | (w1 << 16), w2, 0u, 0u});
}

template <int PREC>
__device__ __forceinline__ bf16x8 ones16() {
    const unsigned one = PREC == NR_PREC_FP16 ? 0x3C003C00u : 0x3F803F80u;
    return __builtin_bit_cast(bf16x8, u32x4{one, one, one, one});
}

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Word w (0..7) of a bf16 block holds accumulator registers 2w (low half) and
// 2w+1 (high half).  bf16 ReLU = max as int16 against 0 (negative bf16 has the
// sign bit set).  Mask bits of a layer, 4 words per lane: block nb, word w sets
// bit j = 8 (nb & 1) + w (register 2w > 0) and bit 16 + j (register 2w+1 > 0)
// of word nb >> 1.
__device__ __forceinline__ unsigned relu_pk(unsigned w) {
    return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(s16x2, w), s16x2{0, 0}));
}
// (asm: after the ReLU the compiler knows w >= 0 and rewrites the min into
// per-half compares and selects, six instructions instead of one)
__device__ __forceinline__ unsigned nz_pk(unsigned w) {
    unsigned r;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(w), "s"(0x10001u));
    return r;
}

// fp32 accumulators (bias included) -> bf16 B operands; ReLU in fp32 when a VALU
// head reads the same activations, else on the packed pairs; optional mask bits.
template <int PREC, int NBO, bool RELU, bool RELU_F32, bool MASK>
__device__ __forceinline__ void epi16(f32x16 (&acc)[NBO], bf16x8 (&out)[NBO][2], unsigned (&mw)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) mw[q] = 0u;
#pragma unroll
    for (int nb = 0; nb < NBO; ++nb) {
        if constexpr (RELU && RELU_F32)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[nb][r] = __int_as_float(max(__float_as_int(acc[nb][r]), 0));
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            u32x4 wd = __builtin_bit_cast(u32x4, pack8<PREC>(acc[nb], hf));
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                if constexpr (RELU && !RELU_F32) wd[m] = relu_pk(wd[m]);
                if constexpr (MASK) mw[nb >> 1] |= nz_pk(wd[m]) << (8 * (nb & 1) + 4 * hf + m);
            }
            out[nb][hf] = __builtin_bit_cast(bf16x8, wd);
        }
    }
}

// Backward: zero the packed dz pairs whose forward activation was not positive.
__device__ __forceinline__ void mask_pk(bf16x8 (&v)[2], unsigned word, int nb) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        u32x4 wd = __builtin_bit_cast(u32x4, v[hf]);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const unsigned t = (word >> (8 * (nb & 1) + 4 * hf + m)) & 0x10001u;
            wd[m] &= t * 0xFFFFu;
        }
        v[hf] = __builtin_bit_cast(bf16x8, wd);
    }
}

// dz block -> B operand with the ReLU mask of its forward activation applied
// (bf16: packed-pair mask words of epi_bf16; fp32: bit (nb&1)*16 + r of word nb>>1).
template <int PREC>
__device__ __forceinline__ void to_in_masked(f32x16 a, const u32x4& mw, int nb, InBlk<PREC>& o) {
    if constexpr (k16<PREC>) {
        to_in<PREC>(a, o);
        mask_pk(o.s, mw[nb >> 1], nb);
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const unsigned bit = (mw[nb >> 1] >> ((nb & 1) * 16 + r)) & 1u;
            a[r] = bit ? a[r] : 0.f;
        }
        o.v = a;
    }
}

// One 32-feature block of a tile as a B-operand image: FPB fragments of 1 KB.
template <int PREC>
__device__ __forceinline__ void store_img(char* __restrict__ region, int64_t tile, int nblk, int blk,
                                          const InBlk<PREC>& v, int) {
    // wave-uniform base (tile is per wave) + the lane's 16 B: saddr + voffset stores
    char* base = region + ((tile * nblk + blk) * kFPB<PREC>) * static_cast<int64_t>(kFragBytes) + lane16();
    if constexpr (k16<PREC>) {
#if NR_NT_STORE
        // streaming (non-temporal) stores: the 4 GB of images must not evict the
        // L2-resident weight stream every workgroup re-reads
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v.s[0]), reinterpret_cast<u32x4*>(base));
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v.s[1]), reinterpret_cast<u32x4*>(base + kFragBytes));
#else
        *reinterpret_cast<bf16x8*>(base) = v.s[0];
        *reinterpret_cast<bf16x8*>(base + kFragBytes) = v.s[1];
#endif
    } else {
#pragma unroll
        for (int tq = 0; tq < 4; ++tq)
            *reinterpret_cast<f32x4*>(base + tq * kFragBytes) =
                f32x4{v.v[4 * tq], v.v[4 * tq + 1], v.v[4 * tq + 2], v.v[4 * tq + 3]};
    }
}

template <int PREC>
__device__ __forceinline__ void load_img(const char* __restrict__ region, int64_t tile, int nblk, int blk,
                                         InBlk<PREC>& v, int) {
    const char* base = region + ((tile * nblk + blk) * kFPB<PREC>) * static_cast<int64_t>(kFragBytes) + lane16();
    if constexpr (k16<PREC>) {
        v.s[0] = *reinterpret_cast<const bf16x8*>(base);
        v.s[1] = *reinterpret_cast<const bf16x8*>(base + kFragBytes);
    } else {
#pragma unroll
        for (int tq = 0; tq < 4; ++tq) {
            const f32x4 q = *reinterpret_cast<const f32x4*>(base + tq * kFragBytes);
#pragma unroll
            for (int e = 0; e < 4; ++e) v.v[4 * tq + e] = q[e];
        }
    }
}

// bias + optional ReLU on NBO blocks; mask bits (bit (nb&1)*16+r of word nb>>1) into w[4].
// Vector images (mlp_plan.hpp): 16 fp32 per (block, lane half) in accumulator order.
// Vector images (biases, w_sigma, W_rgb: 16 fp32 per (block, lane half)) are
// read with SCALAR loads through the constant address space and selected per
// lane half, so they cost no vector registers; the opaque pointer copy keeps the
// loads from being hoisted out of the layer loops as invariants.
typedef const __attribute__((address_space(4))) float cfloat;

struct VImg {
    cfloat* p;
    bool hi;
    // registers 4g..4g+3 of block nb, for this lane's half
    __device__ __forceinline__ f32x4 g4(int nb, int g) const {
        f32x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float lo = p[(2 * nb) * 16 + 4 * g + e], up = p[(2 * nb + 1) * 16 + 4 * g + e];
            r[e] = hi ? up : lo;
        }
        return r;
    }
};

__device__ __forceinline__ VImg vimg(const char* packed, int64_t off, int lane) {
    const char* q = packed + off;
    asm volatile("" : "+s"(q));
    return VImg{(cfloat*)(q), (lane >> 5) != 0};
}
#define NR_VEC(img, nb, g) ((img).g4((nb), (g)))

// Pair images (w_sigma, the rows of W_rgb): element nb*16 + r holds the weights of
// accumulator register r of block nb for lane half 0 and for lane half 1, read with
// one 64-bit scalar load; a packed FMA evaluates both halves and each lane keeps
// its own (no per-lane selects of scalar weights: VOP3 reads one SGPR at most).
typedef const __attribute__((address_space(4))) f32x2 cf32x2;
struct PImg {
    cf32x2* p;
    __device__ __forceinline__ f32x2 at(int nb, int r) const { return p[nb * 16 + r]; }
};
__device__ __forceinline__ PImg pimg(const char* packed, int64_t off) {
    const char* q = packed + off;
    asm volatile("" : "+s"(q));
    return PImg{(cf32x2*)(q)};
}
__device__ __forceinline__ f32x2 bcast2(float x) { return f32x2{x, x}; }
// ReLU as an integer max (negative floats, -0 included, are negative as int32):
// one v_max_i32, where the float compare-select also canonicalises its input
__device__ __forceinline__ float relu_f(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

template <int NBO, bool RELU>
__device__ __forceinline__ void bias_act(f32x16 (&acc)[NBO], const VImg& bias, unsigned (&w)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = 0u;
#pragma unroll
    for (int nb = 0; nb < NBO; ++nb) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 b = NR_VEC(bias, nb, g);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * g + e;
                float v = acc[nb][r] + b[e];
                if (RELU) v = v > 0.f ? v : 0.f;
                acc[nb][r] = v;
                w[nb >> 1] |= (v > 0.f ? 1u : 0u) << ((nb & 1) * 16 + r);
            }
        }
    }
}

template <int NBO>
__device__ __forceinline__ void apply_mask(f32x16 (&acc)[NBO], u32x4 mw) {
#pragma unroll
    for (int nb = 0; nb < NBO; ++nb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const unsigned bit = (mw[nb >> 1] >> ((nb & 1) * 16 + r)) & 1u;
            acc[nb][r] = bit ? acc[nb][r] : 0.f;
        }
}

// ------------------------------------------------------ weight stream -----
// A sequence of chunks (all row blocks of one k block of one layer image)
// consumed in order through an LDS double buffer, register-staged one chunk
// ahead: load(q+1) is issued before chunk q's MFMAs and written to the other
// slot after them, then one barrier.  The slot written at step q was last read
// at step q-1, which every wave finished before the previous barrier.
constexpr int kMaxChunks = 176;  // >= sum of KB (forward) or NB (backward) over the MFMA layers

struct StreamDesc {
    int64_t base;                  // byte offset of the stream's first chunk in `packed`
    int nq;                        // chunks
    int ckb[kMaxChunks];           // bytes loaded per chunk, in KB
    int cadv[kMaxChunks];          // bytes to the next chunk, in KB (>= ckb: a chunk may be loaded in part)
};

struct Ring {
    char* lds;
    int slot_bytes;
    int q;                         // chunk in the current slot
    const char* src;               // next chunk to load
    int wv;                        // wave index in the workgroup (wave-uniform)
};

#ifndef NR_SINK_BWD
#define NR_SINK_BWD 0  // 1: store each dz while the next stream consumes it (measured slower: 1.50 vs 1.35 ms)
#endif
#ifndef NR_BWD_RBM
#define NR_BWD_RBM 1  // 16-bit dX chain: 1 row-block major (mlp_bwd_rbm.inc), 0 chunk-major mlp_bwd_kernel
#endif
#ifndef NR_DIN_FUSED
#define NR_DIN_FUSED 0  // 1: 16-bit g_x / g_d through the 4-wave input-gradient dX variant (A/B)
#endif
#ifndef NR_STAGE_GLDS
#define NR_STAGE_GLDS 1
#endif
template <int G, int NT>
struct Stager {
#if NR_STAGE_GLDS
    // LDS-DMA staging: chunk q goes straight into its slot (no registers); the
    // barrier that publishes it is preceded by vmcnt(0).
    __device__ __forceinline__ void load(Ring& ring, const StreamDesc& sd, int q, int tid) {
        if (q >= sd.nq) return;
        load_sized(ring, q, sd.ckb[q], sd.cadv[q], tid);
    }
    // chunk q of ckb KB (advance cadv KB): sizes from the caller, no scalar loads
    __device__ __forceinline__ void load_sized(Ring& ring, int q, int ckb, int cadv, int) {
        const int bytes = ckb * 1024;
        char* slot = ring.lds + (q & 1) * ring.slot_bytes;
        const uint32_t l16 = lane16();
        for (int pc = ring.wv; pc * 1024 < bytes; pc += NT / 64)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(ring.src + pc * 1024 + l16),
                (__attribute__((address_space(3))) void*)(slot + pc * 1024), 16, 0, 0);
        ring.src += cadv * 1024;
    }

    // Wait for this wave's pieces of the next chunk only: the `after` vector-memory
    // ops issued since (the chunk's saved-activation / dz stores) may stay in flight
    // across the barrier (vmcnt retires in issue order).
    __device__ __forceinline__ void store(char*, const StreamDesc&, int, int, int after = 0) {
        switch (after) {
            case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
            case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
            case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
            default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        }
    }
#else
    // register staging: load(q) before chunk q-1's MFMAs, store after them
    u32x4 v[G];

    __device__ __forceinline__ void load(Ring& ring, const StreamDesc& sd, int q, int tid) {
        if (q >= sd.nq) return;
        load_sized(ring, q, sd.ckb[q], sd.cadv[q], tid);
    }
    __device__ __forceinline__ void load_sized(Ring& ring, int, int ckb, int cadv, int tid) {
        const int bytes = ckb * 1024;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int b = (g * NT + tid) * 16;
            if (b < bytes) v[g] = *reinterpret_cast<const u32x4*>(ring.src + b);
        }
        ring.src += cadv * 1024;
    }

    __device__ __forceinline__ void store(char* slot, const StreamDesc& sd, int q, int tid, int = 0) {
        if (q >= sd.nq) return;
        const int bytes = sd.ckb[q] * 1024;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int b = (g * NT + tid) * 16;
            if (b < bytes) *reinterpret_cast<u32x4*>(slot + b) = v[g];
        }
    }
#endif
};

// Per-wave activation storage of NBLK 32-feature blocks for TPW tiles: in
// registers, or (bf16) in the wave's own LDS region as B-operand images (frees
// the 64 registers that let two waves share a SIMD without spilling).
template <int PREC, int TPW, int NBLK, bool LDS>
struct Act {
    static constexpr bool kLds = false;
    InBlk<PREC> v[TPW][NBLK];
    __device__ __forceinline__ InBlk<PREC> operator()(int t, int kb) const { return v[t][kb]; }
    __device__ __forceinline__ void put(int t, int nb, const InBlk<PREC>& x) { v[t][nb] = x; }
};
template <int PREC, int TPW, int NBLK>
struct Act<PREC, TPW, NBLK, true> {
    static constexpr bool kLds = true;
    char* base;  // the wave's region (wave-uniform)
    // LDS byte address of this lane's 16 B of block kb of tile t (first fragment)
    __device__ __forceinline__ uint32_t addr(int t, int kb) const {
        return static_cast<uint32_t>(reinterpret_cast<uintptr_t>(base)) + lane16() +
               static_cast<uint32_t>((t * NBLK + kb) * 2 * kFragBytes);
    }
    static constexpr int kBytes = TPW * NBLK * 2 * kFragBytes;
    __device__ __forceinline__ InBlk<PREC> operator()(int t, int kb) const {
        const char* p = base + lane16() + (t * NBLK + kb) * 2 * kFragBytes;
        InBlk<PREC> r;
        r.s[0] = *reinterpret_cast<const bf16x8*>(p);
        r.s[1] = *reinterpret_cast<const bf16x8*>(p + kFragBytes);
        return r;
    }
    __device__ __forceinline__ void put(int t, int nb, const InBlk<PREC>& x) {
        char* p = base + lane16() + (t * NBLK + nb) * 2 * kFragBytes;
        *reinterpret_cast<bf16x8*>(p) = x.s[0];
        *reinterpret_cast<bf16x8*>(p + kFragBytes) = x.s[1];
    }
};

// Saves each B operand a stream consumes (= the previous layer's output block kb)
// as its B-operand image, one block per chunk: the saved-activation / dz stores
// spread over the stream instead of bursting at every layer end.
template <int PREC, int TPW>
struct Sink {
    char* region;  // nullptr: no store
    int nblk;
    int64_t tile0;
    unsigned tok;  // bit t: tile t exists
    __device__ __forceinline__ void operator()(int t, int kb, const InBlk<PREC>& v) const {
        if (region != nullptr && ((tok >> t) & 1u)) store_img<PREC>(region, tile0 + t, nblk, kb, v, 0);
    }
    // vector-memory stores one chunk issues (wave-uniform)
    __device__ __forceinline__ int stores() const {
        return region == nullptr ? 0 : kFPB<PREC> * __builtin_popcount(tok & ((1u << TPW) - 1u));
    }
};

// Workgroup barrier of the weight stream.  Not __syncthreads(): its release fence
// would also drain every in-flight global store (vmcnt(0)) at every chunk.  LDS
// writes (activations, register-staged chunks) and this wave's reads of the slot
// about to be refilled complete first (lgkmcnt(0)); LDS-DMA completion is the
// stager's counted vmcnt.
__device__ __forceinline__ void stream_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// ds_read_b128 of the two 1-KB fragments of one 32x32 16-bit block (inline asm:
// see stream_gemm) and the counted wait that publishes them.
__device__ __forceinline__ void ds_read_pair(bf16x8 (&dst)[2], uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1" : "=v"(dst[0]) : "v"(addr));
    asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(dst[1]) : "v"(addr));
}
// wait until at most n LDS/SMEM ops are outstanding (n: the reads issued after
// these two, all younger LDS reads; SMEM only ever makes this wait longer)
__device__ __forceinline__ void lgkm_wait_pair(int n, bf16x8& a0, bf16x8& a1) {
    switch (n) {
        case 0: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a0), "+v"(a1)); break;
        case 2: asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(a0), "+v"(a1)); break;
        case 4: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(a0), "+v"(a1)); break;
        case 6: asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(a0), "+v"(a1)); break;
        default: asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(a0), "+v"(a1)); break;
    }
}

// fp32 A operands: the four 1-KB fragments of one row block, read by asm
__device__ __forceinline__ void ds_read_quad(f32x4 (&dst)[4], uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1" : "=v"(dst[0]) : "v"(addr));
    asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(dst[1]) : "v"(addr));
    asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(dst[2]) : "v"(addr));
    asm volatile("ds_read_b128 %0, %1 offset:3072" : "=v"(dst[3]) : "v"(addr));
}
__device__ __forceinline__ void lgkm_wait_one(int n, f32x4& a) {
    switch (n) {
        case 0: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a)); break;
        case 1: asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(a)); break;
        case 2: asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(a)); break;
        case 3: asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(a)); break;
        case 4: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(a)); break;
        case 5: asm volatile("s_waitcnt lgkmcnt(5)" : "+v"(a)); break;
        case 6: asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(a)); break;
        default: asm volatile("s_waitcnt lgkmcnt(7)" : "+v"(a)); break;
    }
}

// Epilogue hooks of stream_gemm's last chunk (16-bit, one tile per wave): as the
// MFMAs of row block r issue, the bias MFMA of block r-1 and the packing / ReLU /
// mask bits / LDS store of block r-2 run, so the layer epilogue overlaps the
// matrix pipe instead of following it with every wave of the workgroup idle.
struct NoEpi {
    static constexpr bool kOn = false;
    __device__ __forceinline__ void bias(int) const {}
    __device__ __forceinline__ void finish(int) const {}
};

template <int PREC, bool RELU, bool MASK>
__device__ __forceinline__ void epi16_blk(const f32x16& a, bf16x8 (&out)[2], unsigned* mw, int nb) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        u32x4 wd = __builtin_bit_cast(u32x4, pack8<PREC>(a, hf));
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            if constexpr (RELU) wd[m] = relu_pk(wd[m]);
            if constexpr (MASK) mw[nb >> 1] |= nz_pk(wd[m]) << (8 * (nb & 1) + 4 * hf + m);
        }
        out[hf] = __builtin_bit_cast(bf16x8, wd);
    }
}

template <int PREC, int TPW, bool RELU, bool MASK, class Dst>
struct LayerEpi {
    static constexpr bool kOn = true;
    f32x16 (*acc)[kHB];  // the layer's accumulators, acc[TPW][kHB]
    const float* bl;     // bias, lane < 32 holds row 32 nb + lane
    Dst* dst;            // where the 16-bit output blocks go (activations)
    unsigned (*mw)[4];   // mask words per tile (MASK)
    __device__ __forceinline__ void bias(int nb) const {
#pragma unroll
        for (int t = 0; t < TPW; ++t) acc[t][nb] = mfma16<PREC>(bias_frag<PREC>(bl[nb]), ones16<PREC>(), acc[t][nb]);
    }
    __device__ __forceinline__ void finish(int nb) const {
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            bf16x8 o[2];
            epi16_blk<PREC, RELU, MASK>(acc[t][nb], o, mw[t], nb);
            dst->put(t, nb, InBlk<PREC>{{o[0], o[1]}});
        }
    }
};

// acc1[t][r] += A(row block nb0 + r) . in[t]   (r < N1)
// acc2[t][r] += A(row block nb0 + N1 + r) . in[t]   (r < N2)
// over KBN consecutive stream chunks (k blocks).
template <int PREC, int TPW, int N1, int N2, int KBN, int G, int NT, class Src, class Epi = NoEpi>
__device__ __forceinline__ void stream_gemm(f32x16 (&acc1)[TPW][N1 > 0 ? N1 : 1],
                                            f32x16 (&acc2)[TPW][N2 > 0 ? N2 : 1], int nb0, const Src& src,
                                            Ring& ring, Stager<G, NT>& st, const char* __restrict__ packed,
                                            const StreamDesc& sd, int tid, int lane,
                                            const Sink<PREC, TPW>& sink = Sink<PREC, TPW>{nullptr, 0, 0, 0u},
                                            const Epi& epi = Epi{}) {
    static_assert(!Epi::kOn || (k16<PREC> && N2 == 0), "epilogue hook: 16-bit");
    // Chunk sizes, read once per segment: every chunk of a segment has this
    // segment's size; the prefetch in its last step is the next segment's first chunk.
    const int q0 = ring.q;
    const int ckb_this = sd.ckb[q0], adv_this = sd.cadv[q0];
    const bool has_next = q0 + KBN < sd.nq;
    const int ckb_next = has_next ? sd.ckb[q0 + KBN] : 0, adv_next = has_next ? sd.cadv[q0 + KBN] : 0;
#pragma unroll
    for (int kb = 0; kb < KBN; ++kb) {
        if (kb < KBN - 1)
            st.load_sized(ring, ring.q + 1, ckb_this, adv_this, tid);
        else if (has_next)
            st.load_sized(ring, ring.q + 1, ckb_next, adv_next, tid);
        asm volatile("" ::: "memory");  // the sink stores below stay younger than the DMA
        const char* slot = ring.lds + (ring.q & 1) * ring.slot_bytes + lane16();
        InBlk<PREC> in[TPW];
        constexpr bool B_ASM = k16<PREC> && Src::kLds;  // B operands read by asm (see A below)
        if constexpr (B_ASM) {
#pragma unroll
            for (int t = 0; t < TPW; ++t) ds_read_pair(in[t].s, src.addr(t, kb));
        } else {
#pragma unroll
            for (int t = 0; t < TPW; ++t) in[t] = src(t, kb);
        }
        // 16-bit: the two A fragments of row block r + PF are read (inline asm) while
        // row block r multiplies, and each MFMA pair waits (counted lgkmcnt, tied to its
        // registers) only for its own reads.  Plain loads here get sunk by the compiler
        // next to their use: one read, lgkmcnt(0), one MFMA, every time.
        constexpr int NRB = N1 + N2;
        constexpr int PF = NR_APF < NRB ? NR_APF : NRB;
        bf16x8 aring[PF + 1][2];
        const uint32_t abase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(slot)) +
                               static_cast<uint32_t>(nb0 * kFPB<PREC> * kFragBytes);
        f32x4 aq[2][4];  // fp32: row block r + 1 is read while row block r multiplies
        if constexpr (k16<PREC>) {
#pragma unroll
            for (int r = 0; r < PF; ++r) ds_read_pair(aring[r], abase + r * 2 * kFragBytes);
        } else if constexpr (NR_APF > 0) {
            ds_read_quad(aq[0], abase);
        }
        if constexpr (B_ASM)
#pragma unroll
            for (int t = 0; t < TPW; ++t) lgkm_wait_pair(2 * PF + 2 * (TPW - 1 - t), in[t].s[0], in[t].s[1]);
#pragma unroll
        for (int t = 0; t < TPW; ++t) sink(t, kb, in[t]);
#pragma unroll
        for (int r = 0; r < N1 + N2; ++r) {
            const char* fp = slot + (nb0 + r) * kFPB<PREC> * kFragBytes;
            constexpr int I1 = N1 > 0 ? N1 : 1;
            constexpr int I2 = N2 > 0 ? N2 : 1;
            const int r1 = r < N1 ? r : 0;
            const int r2 = r >= N1 ? (r - N1) % I2 : 0;
            (void)I1;
            if constexpr (k16<PREC>) {
                if (r + PF < NRB) ds_read_pair(aring[(r + PF) % (PF + 1)], abase + (r + PF) * 2 * kFragBytes);
                bf16x8 a0 = aring[r % (PF + 1)][0];
                bf16x8 a1 = aring[r % (PF + 1)][1];
                const int younger = 2 * (NRB - 1 - r < PF ? NRB - 1 - r : PF);
                lgkm_wait_pair(younger, a0, a1);
#pragma unroll
                for (int t = 0; t < TPW; ++t) {
                    if (r < N1) {
                        acc1[t][r1] = mfma16<PREC>(a0, in[t].s[0], acc1[t][r1]);
                        acc1[t][r1] = mfma16<PREC>(a1, in[t].s[1], acc1[t][r1]);
                    } else {
                        acc2[t][r2] = mfma16<PREC>(a0, in[t].s[0], acc2[t][r2]);
                        acc2[t][r2] = mfma16<PREC>(a1, in[t].s[1], acc2[t][r2]);
                    }
                }
                if constexpr (Epi::kOn) {
                    if (kb == KBN - 1) {
                        if (r >= 1) epi.bias(r - 1);
                        if (r >= 2) epi.finish(r - 2);
                    }
                }
            } else {
                if constexpr (NR_APF > 0)
                    if (r + 1 < NRB) ds_read_quad(aq[(r + 1) & 1], abase + (r + 1) * 4 * kFragBytes);
#pragma unroll
                for (int tq = 0; tq < 4; ++tq) {
                    f32x4 a;
                    if constexpr (NR_APF > 0) {
                        a = aq[r & 1][tq];
                        lgkm_wait_one((r + 1 < NRB ? 4 : 0) + 3 - tq, a);
                    } else {
                        a = *reinterpret_cast<const f32x4*>(fp + tq * kFragBytes);
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e)
#pragma unroll
                        for (int t = 0; t < TPW; ++t) {
                            if (r < N1)
                                acc1[t][r1] = mfma_f32(a[e], in[t].v[4 * tq + e], acc1[t][r1]);
                            else
                                acc2[t][r2] = mfma_f32(a[e], in[t].v[4 * tq + e], acc2[t][r2]);
                        }
                }
            }
        }
        if constexpr (Epi::kOn) {
            if (kb == KBN - 1) {
                epi.bias(NRB - 1);
                if (NRB >= 2) epi.finish(NRB - 2);
                epi.finish(NRB - 1);
            }
        }
        st.store(ring.lds + ((ring.q + 1) & 1) * ring.slot_bytes, sd, ring.q + 1, tid, sink.stores());
        stream_barrier();
        ++ring.q;
    }
}

template <int G, int NT>
__device__ __forceinline__ void stream_begin(Ring& ring, Stager<G, NT>& st, const char* __restrict__ packed,
                                             const StreamDesc& sd, int tid) {
    ring.q = 0;
    ring.src = packed + sd.base;
    st.load(ring, sd, 0, tid);
    st.store(ring.lds, sd, 0, tid);
    __syncthreads();
}

// ------------------------------------------------------------ forward -----
struct FwdArgs {
    const char* packed;
    const float* params;
    const float* x;
    const float* d;
    float* rgb;
    float* sigma;
    char* saved;
    int64_t M, tiles;
    int L, Ld, n_layers;
    uint32_t skips;
    int slot_bytes;
    StreamDesc sd;  // W images: trunk 0..n-1, feat, dir
    int64_t vb[kMaxMfmaLayers];
    int64_t bo[kMaxMfmaLayers];  // bias offsets in params (bf16: bias by MFMA)
    int64_t vsig, vrgb, sig_b, rgb_b;
    int64_t sv_off[kMaxTrunk + 4];
    int sv_feat, sv_denc, sv_hc;
    int64_t mask_off;
    int n_mask;
};

template <int PREC, int XB, int DB, bool TRAIN, int TPW, int G, int NT>
__global__ __launch_bounds__(NT, 1) void mlp_fwd_kernel(FwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, ml = lane & 31;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t tile0 = (static_cast<int64_t>(blockIdx.x) * (NT / 64) + wv) * TPW;
    const int n = a.n_layers;
    float px[TPW][3];
    bool tok[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const int64_t m = (tile0 + t) * 32 + ml;
        tok[t] = tile0 + t < a.tiles;
        const bool valid = m < a.M;
        px[t][0] = valid ? a.x[3 * m] : 0.f;
        px[t][1] = valid ? a.x[3 * m + 1] : 0.f;
        px[t][2] = valid ? a.x[3 * m + 2] : 0.f;
    }
    u32x4* masks = reinterpret_cast<u32x4*>(a.saved + a.mask_off);
    unsigned tokm = 0u;
#pragma unroll
    for (int t = 0; t < TPW; ++t) tokm |= (tok[t] ? 1u : 0u) << t;
    // training saves each layer input as the next stream consumes it
    auto sink_of = [&](int sv, int nblk) {
        return Sink<PREC, TPW>{TRAIN ? a.saved + a.sv_off[sv] : nullptr, nblk, tile0, tokm};
    };

    Ring ring{lds, a.slot_bytes, 0, nullptr, wv};
    Stager<G, NT> st;
    stream_begin(ring, st, a.packed, a.sd, tid);

    f32x16 acc[TPW][kHB];
    constexpr bool ACT_LDS = k16<PREC> && (NT == 512 || TPW >= 2);
    Act<PREC, TPW, kHB, ACT_LDS> hin;
    if constexpr (ACT_LDS)
        hin.base = lds + 2 * a.slot_bytes + wv * Act<PREC, TPW, kHB, ACT_LDS>::kBytes;
    f32x16 dummy[TPW][1];
    unsigned w[TPW][4];
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
            for (int nb = 0; nb < kHB; ++nb) zero(acc[t][nb]);
        float bl[kHB];  // bf16: this layer's bias, lane < 32 holds rows 32 nb + lane
        if constexpr (k16<PREC>)
#pragma unroll
            for (int nb = 0; nb < kHB; ++nb) bl[nb] = lane < 32 ? a.params[a.bo[i] + 32 * nb + lane] : 0.f;
        const bool skip_in = i > 0 && ((a.skips >> (i - 1)) & 1u);
        // 16-bit: the epilogue runs inside the layer's last chunk
        constexpr bool HOOK = k16<PREC> && NR_EPI_HOOK;
        if constexpr (HOOK)
#pragma unroll
            for (int t = 0; t < TPW; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) w[t][q] = 0u;
        const LayerEpi<PREC, TPW, true, TRAIN, decltype(hin)> ep{acc, bl, &hin, w};
        if (i == 0 || skip_in) {
            // x_enc is not kept in registers: the skip layer reloads the saved
            // copy (training) or recomputes it (inference)
            Act<PREC, TPW, XB, false> xe;
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                if (TRAIN && i > 0) {
#pragma unroll
                    for (int kb = 0; kb < XB; ++kb) {
                        if (tok[t])
                            load_img<PREC>(a.saved + a.sv_off[SV_XENC], tile0 + t, XB, kb, xe.v[t][kb], lane);
                        else
                            xe.v[t][kb] = InBlk<PREC>{};
                    }
                    continue;
                }
                // opaque copy: keeps the encoding from being hoisted out of the
                // layer loop (and spilled) as a loop invariant
                float p0 = px[t][0], p1 = px[t][1], p2 = px[t][2];
                asm volatile("" : "+v"(p0), "+v"(p1), "+v"(p2));
                const PeRev pr = pe_rev(p0, p1, p2);
#pragma unroll
                for (int kb = 0; kb < XB; ++kb) {
                    f32x16 v;
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        v[r] = (k16<PREC> && NR_FASTPE)
                                   ? pe_fast(pr, 32 * kb + acc_row(r, 0), 32 * kb + acc_row(r, 1), h != 0, a.L)
                                   : pe_feat(p0, p1, p2, 32 * kb + acc_row(r, h), a.L);
                    InBlk<PREC> o;
                    to_in<PREC>(v, o);
                    if constexpr (TRAIN)
                        if (tok[t]) store_img<PREC>(a.saved + a.sv_off[SV_XENC], tile0 + t, XB, kb, o, lane);
                    // constant indices: the fp32 body (accurate sinf) is too big for the
                    // pragma to unroll, and a run-time index put xe in scratch, whose
                    // reloads in the stream then drained the in-flight weight DMA
#pragma unroll
                    for (int k2 = 0; k2 < XB; ++k2)
                        if (k2 == kb) xe.v[t][k2] = o;
                }
            }
            bool hooked = false;
            if constexpr (HOOK) {
                if (i == 0) {
                    stream_gemm<PREC, TPW, kHB, 0, XB, G, NT>(acc, dummy, 0, xe, ring, st, a.packed, a.sd, tid, lane,
                                                              Sink<PREC, TPW>{nullptr, 0, 0, 0u}, ep);
                    hooked = true;
                }
            }
            if (!hooked)
                stream_gemm<PREC, TPW, kHB, 0, XB, G, NT>(acc, dummy, 0, xe, ring, st, a.packed, a.sd, tid, lane);
        }
        if (i > 0) {
            if constexpr (HOOK)
                stream_gemm<PREC, TPW, kHB, 0, kHB, G, NT>(acc, dummy, 0, hin, ring, st, a.packed, a.sd, tid, lane,
                                                           sink_of(SV_H0 + i - 1, kHB), ep);
            else
                stream_gemm<PREC, TPW, kHB, 0, kHB, G, NT>(acc, dummy, 0, hin, ring, st, a.packed, a.sd, tid, lane,
                                                           sink_of(SV_H0 + i - 1, kHB));
        }
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            if constexpr (HOOK) {
                // done inside the stream
            } else if constexpr (k16<PREC>) {
                bf16x8 hv[kHB][2];
                if (NR_BIASMFMA) {
#pragma unroll
                    for (int nb = 0; nb < kHB; ++nb) acc[t][nb] = mfma16<PREC>(bias_frag<PREC>(bl[nb]), ones16<PREC>(), acc[t][nb]);
                } else {
                    unsigned wt[4];
                    bias_act<kHB, false>(acc[t], vimg(a.packed, a.vb[i], lane), wt);
                }
                epi16<PREC, kHB, true, false, TRAIN>(acc[t], hv, w[t]);
#pragma unroll
                for (int nb = 0; nb < kHB; ++nb) hin.put(t, nb, InBlk<PREC>{{hv[nb][0], hv[nb][1]}});
            } else {
                bias_act<kHB, true>(acc[t], vimg(a.packed, a.vb[i], lane), w[t]);
#pragma unroll
                for (int nb = 0; nb < kHB; ++nb) {
                    InBlk<PREC> v;
                    to_in<PREC>(acc[t][nb], v);
                    hin.put(t, nb, v);
                }
            }
            if constexpr (TRAIN)
                if (tok[t]) masks[((tile0 + t) * a.n_mask + i) * 64 + lane] = u32x4{w[t][0], w[t][1], w[t][2], w[t][3]};
        }
    }

    // sigma head (VALU): relu(w_sigma . h + b), from the fp32 activations
    float sp[TPW];
    {
        const PImg ws = pimg(a.packed, a.vsig);
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            f32x2 s2 = {0.f, 0.f};
#pragma unroll
            for (int nb = 0; nb < kHB; ++nb)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    s2 = __builtin_elementwise_fma(bcast2(relu_f(acc[t][nb][r])), ws.at(nb, r), s2);
            sp[t] = h ? s2[1] : s2[0];
        }
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            sp[t] += __shfl_xor(sp[t], 32);
            sp[t] = sp[t] + a.params[a.sig_b];
            sp[t] = sp[t] > 0.f ? sp[t] : 0.f;
        }
    }

    // feature_linear (no activation)
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) zero(acc[t][nb]);
    constexpr bool HOOKF = k16<PREC> && NR_EPI_HOOK;
    if constexpr (HOOKF) {
        float bf[kHB];
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) bf[nb] = lane < 32 ? a.params[a.bo[n] + 32 * nb + lane] : 0.f;
        const LayerEpi<PREC, TPW, false, false, decltype(hin)> epf{acc, bf, &hin, w};
        stream_gemm<PREC, TPW, kHB, 0, kHB, G, NT>(acc, dummy, 0, hin, ring, st, a.packed, a.sd, tid, lane,
                                                   sink_of(SV_H0 + n - 1, kHB), epf);
    } else {
        stream_gemm<PREC, TPW, kHB, 0, kHB, G, NT>(acc, dummy, 0, hin, ring, st, a.packed, a.sd, tid, lane,
                                                   sink_of(SV_H0 + n - 1, kHB));
    }
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        if constexpr (HOOKF) {
            // done inside the stream
        } else if constexpr (k16<PREC>) {
            bf16x8 hv[kHB][2];
#pragma unroll
            for (int nb = 0; nb < kHB; ++nb) {
                const float b = lane < 32 ? a.params[a.bo[n] + 32 * nb + lane] : 0.f;
                if (NR_BIASMFMA) acc[t][nb] = mfma16<PREC>(bias_frag<PREC>(b), ones16<PREC>(), acc[t][nb]);
            }
            if (!NR_BIASMFMA) {
                unsigned wt[4];
                bias_act<kHB, false>(acc[t], vimg(a.packed, a.vb[n], lane), wt);
            }
            epi16<PREC, kHB, false, false, false>(acc[t], hv, w[t]);
#pragma unroll
            for (int nb = 0; nb < kHB; ++nb) hin.put(t, nb, InBlk<PREC>{{hv[nb][0], hv[nb][1]}});
        } else {
            bias_act<kHB, false>(acc[t], vimg(a.packed, a.vb[n], lane), w[t]);
#pragma unroll
            for (int nb = 0; nb < kHB; ++nb) {
                InBlk<PREC> v;
                to_in<PREC>(acc[t][nb], v);
                hin.put(t, nb, v);
            }
        }
    }

    // dir_linear over [feat, d_enc], ReLU
    constexpr int NC = kHB / 2;
    f32x16 ac[TPW][NC];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int nb = 0; nb < NC; ++nb) zero(ac[t][nb]);
    stream_gemm<PREC, TPW, NC, 0, kHB, G, NT>(ac, dummy, 0, hin, ring, st, a.packed, a.sd, tid, lane,
                                              sink_of(a.sv_feat, kHB));
    if constexpr (DB > 0) {
        Act<PREC, TPW, DB, false> de;
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            const int64_t m = (tile0 + t) * 32 + ml;
            const bool valid = m < a.M;
            const float d0 = valid ? a.d[3 * m] : 0.f, d1 = valid ? a.d[3 * m + 1] : 0.f,
                        d2 = valid ? a.d[3 * m + 2] : 0.f;
            const PeRev pr = pe_rev(d0, d1, d2);
#pragma unroll
            for (int kb = 0; kb < DB; ++kb) {
                f32x16 v;
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    v[r] = (k16<PREC> && NR_FASTPE)
                               ? pe_fast(pr, 32 * kb + acc_row(r, 0), 32 * kb + acc_row(r, 1), h != 0, a.Ld)
                               : pe_feat(d0, d1, d2, 32 * kb + acc_row(r, h), a.Ld);
                to_in<PREC>(v, de.v[t][kb]);
                if constexpr (TRAIN)
                    if (tok[t]) store_img<PREC>(a.saved + a.sv_off[a.sv_denc], tile0 + t, DB, kb, de.v[t][kb], lane);
            }
        }
        stream_gemm<PREC, TPW, NC, 0, DB, G, NT>(ac, dummy, 0, de, ring, st, a.packed, a.sd, tid, lane);
    }
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        bf16x8 hcv[NC][2];
        if constexpr (k16<PREC>) {
#pragma unroll
            for (int nb = 0; nb < NC; ++nb) {
                const float b = lane < 32 ? a.params[a.bo[n + 1] + 32 * nb + lane] : 0.f;
                if (NR_BIASMFMA) ac[t][nb] = mfma16<PREC>(bias_frag<PREC>(b), ones16<PREC>(), ac[t][nb]);
            }
            if (!NR_BIASMFMA) {
                unsigned wt[4];
                bias_act<NC, false>(ac[t], vimg(a.packed, a.vb[n + 1], lane), wt);
            }
            epi16<PREC, NC, true, true, TRAIN>(ac[t], hcv, w[t]);
        } else {
            bias_act<NC, true>(ac[t], vimg(a.packed, a.vb[n + 1], lane), w[t]);
        }
        if constexpr (TRAIN) {
            if (tok[t]) {
#pragma unroll
                for (int nb = 0; nb < NC; ++nb) {
                    InBlk<PREC> v;
                    if constexpr (k16<PREC>)
                        v = InBlk<PREC>{{hcv[nb][0], hcv[nb][1]}};
                    else
                        to_in<PREC>(ac[t][nb], v);
                    store_img<PREC>(a.saved + a.sv_off[a.sv_hc], tile0 + t, NC, nb, v, lane);
                }
                masks[((tile0 + t) * a.n_mask + n) * 64 + lane] = u32x4{w[t][0], w[t][1], w[t][2], w[t][3]};
            }
        }
        // rgb head (VALU): sigmoid(W_rgb h_c + b)
        float pr[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const PImg wr = pimg(a.packed, a.vrgb + c * NC * 128);
            f32x2 s2 = {0.f, 0.f};
#pragma unroll
            for (int nb = 0; nb < NC; ++nb)
#pragma unroll
                for (int r = 0; r < 16; ++r) s2 = __builtin_elementwise_fma(bcast2(ac[t][nb][r]), wr.at(nb, r), s2);
            float s = h ? s2[1] : s2[0];
            s += __shfl_xor(s, 32);
            s = s + a.params[a.rgb_b + c];
            pr[c] = 1.0f / (1.0f + expf(-s));
        }
        const int64_t m = (tile0 + t) * 32 + ml;
        if (m < a.M && h == 0) {
            a.rgb[3 * m] = pr[0];
            a.rgb[3 * m + 1] = pr[1];
            a.rgb[3 * m + 2] = pr[2];
            a.sigma[m] = sp[t];
        }
    }
}

// Active tiles of a segment from its flags (tile_flags_kernel), one wave: lane l holds
// flag word l (tiles 4l .. 4l+3 of the segment, one byte each, 0 or 1), its count and the
// wave's inclusive scan of the counts.
struct SegFlags {
    uint32_t word;
    int count, incl, total;
};
__device__ __forceinline__ uint32_t seg_flag_word(const uint8_t* __restrict__ flags, int64_t sg) {
    static_assert(kSegTiles == 4 * 64, "one flag word per lane");
    return reinterpret_cast<const uint32_t*>(flags + sg * kSegTiles)[threadIdx.x & 63];
}
__device__ __forceinline__ SegFlags seg_scan(uint32_t word) {
    const int lane = threadIdx.x & 63;
    SegFlags f;
    f.word = word;
    f.count = __popc(f.word);
    f.incl = f.count;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(f.incl, d);
        if (lane >= d) f.incl += o;
    }
    f.total = __builtin_amdgcn_readfirstlane(__shfl(f.incl, 63));
    return f;
}

// The tile of the segment's k-th active tile (k < f.total; wave-uniform result).
__device__ __forceinline__ int64_t seg_entry(const SegFlags& f, int64_t sg, int k) {
    const uint64_t over = __ballot(f.incl > k);
    const int L = __builtin_ctzll(over);  // the lane whose word holds entry k
    const uint32_t w = __builtin_amdgcn_readfirstlane(__shfl(f.word, L));
    int r = k - __builtin_amdgcn_readfirstlane(__shfl(f.incl - f.count, L));
    int b = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bool set = (w >> (8 * q)) & 1u;
        if (set && r == 0) b = q;
        r -= set ? 1 : 0;
        if (r < 0) r = 1 << 20;  // found: no later byte matches
    }
    return sg * kSegTiles + 4 * L + b;
}

// The dW kernel's work list: every active tile once, in increasing order, and their
// total.  Each segment's tiles are placed by wave 0 of the dX workgroup that leads the
// segment (part 0), after its own tiles, from `before` (the active tiles of the segments
// before it, select_tile): each lane writes the active tiles of its flag word.
__device__ __forceinline__ void place_segment(const SegFlags& f, uint32_t before, int64_t nseg, int64_t sg,
                                              uint32_t* __restrict__ list, uint32_t* __restrict__ count) {
    const int lane = threadIdx.x & 63;
    uint32_t slot = before + static_cast<uint32_t>(f.incl - f.count);
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if ((f.word >> (8 * q)) & 1u) list[slot++] = static_cast<uint32_t>(sg * kSegTiles + 4 * lane + q);
    if (sg == nseg - 1 && lane == 0) *count = before + static_cast<uint32_t>(f.total);
}

// A dX wave's tile.  Every workgroup reads the 64-tile block counts of the whole launch
// (tile_flags_kernel; one uint4 per segment, from L2) and its segment's flags, in one
// round of loads:
//  * every tile active (the dense case: bare-init training, cfg->dense_backward):
//    workgroup b runs tiles W b .. W b + W - 1, the layout's own order (no lists; dW
//    takes its identity path on count == tiles);
//  * otherwise, segment-minor: workgroup b takes part j = b / nseg of segment
//    (b - j) mod nseg, i.e. the active tiles W j .. W j + W - 1 of that segment, so the
//    workgroups with active tiles are dispatched first and spread over every XCD
//    (blocks are dealt to XCDs round-robin); parts past a segment's count have nothing
//    to do.
// Measured (fine bf16 M=786432 dX, profiles/r06_tile_map_ab.txt): segment-minor in the
// dense case costs ~7 % at M=786432 and ~20 % at 262144 (locality), segment-major in
// the skipping case 1.67x at 37 % active.
constexpr int64_t kDenseCheckSegs = 1024;  // launches up to 262,144 tiles check for "all active"

struct TileSel {
    SegFlags sf;
    int64_t seg, tile;
    uint32_t before;   // skipping form: active tiles of the segments before seg
    bool dense, live, idle, leader;
};
__device__ __forceinline__ TileSel select_tile(const uint8_t* __restrict__ flags,
                                               const uint32_t* __restrict__ blk_count, int64_t nseg,
                                               int64_t tiles, int W, int wv) {
    constexpr int BPS = kSegTiles / 64;  // 64-tile blocks per segment
    const int lane = threadIdx.x & 63;
    const int64_t b = blockIdx.x;
    TileSel t;
    // skipping form: part-major over the segments (the parts with active tiles go first),
    // the segment rotated by the part, so that one segment's parts land on different
    // XCDs (b % 8) even when nseg is a multiple of 8: segments whose counts differ (a
    // trained field's rays hit or miss as a whole) then load every XCD alike
    const int part = static_cast<int>(b / nseg);
    t.seg = (b % nseg + nseg - part % nseg) % nseg;
    // every load first (one round trip): the segment's flag word and the block counts,
    // one uint4 (a segment's four blocks) per lane and 64 segments.  Past
    // kDenseCheckSegs segments (M > 8.4M samples) reading every count in every workgroup
    // would grow with M^2: such launches take the skipping form, which is right for any
    // flags, and only the leaders read the counts before their segment
    static_assert(BPS == 4, "a segment's block counts are one uint4");
    const bool check = nseg <= kDenseCheckSegs;  // launch-uniform
    const int64_t lim = check ? nseg : (part == 0 && wv == 0 ? t.seg : 0);
    const uint32_t word = seg_flag_word(flags, t.seg);
    const uint4* __restrict__ bc4 = reinterpret_cast<const uint4*>(blk_count);
    uint32_t all = 0, before = 0;
    for (int64_t s0 = 0; s0 < lim; s0 += 4 * 64) {
        uint4 c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t sg = s0 + i * 64 + lane;
            c[i] = sg < lim ? bc4[sg] : uint4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t n = ((c[i].x + c[i].y) + c[i].z) + c[i].w;
            all += n;
            before += (s0 + i * 64 + lane) < t.seg ? n : 0u;
        }
    }
    t.sf = seg_scan(word);
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        all += __shfl_xor(all, d);
        before += __shfl_xor(before, d);
    }
    t.before = __builtin_amdgcn_readfirstlane(before);
    t.dense = check && static_cast<int64_t>(__builtin_amdgcn_readfirstlane(all)) == tiles;
    if (t.dense) {
        const int64_t first = b * W;
        t.tile = first + wv;
        t.live = t.tile < tiles;
        t.idle = first >= tiles;
        t.leader = b == 0 && wv == 0;
    } else {
        const int k = part * W + wv;
        t.idle = part * W >= t.sf.total;
        t.live = k < t.sf.total;
        t.tile = t.live ? seg_entry(t.sf, t.seg, k) : 0;
        t.leader = part == 0 && wv == 0;
    }
    return t;
}

// the leader's share of the dW list (skipping form) or the dense count
__device__ __forceinline__ void finish_tiles(const TileSel& t, int64_t nseg, int64_t tiles, uint32_t* __restrict__ list,
                                             uint32_t* __restrict__ count) {
    if (!t.leader) return;
    if (t.dense) {
        if ((threadIdx.x & 63) == 0) *count = static_cast<uint32_t>(tiles);
    } else {
        place_segment(t.sf, t.before, nseg, t.seg, list, count);
    }
}

#include "mlp_fwd_rbm.inc"
#include "mlp_bwd_rbm.inc"

// ----------------------------------------------------------- backward -----
struct BwdArgs {
    float gscale, inv_gscale;  // fp16 loss scale applied to dL/d(rgb, sigma); 1 otherwise
    const char* packed;
    const float* params;
    const float* x;
    const float* d;
    const float* rgb;
    const float* sigma;
    const float* g_rgb;
    const float* g_sigma;
    float* g_x;
    float* g_d;
    const char* saved;
    char* ws;
    int64_t M, tiles;
    const uint8_t* flags;       // active tiles (tile_flags_kernel) and their 64-tile block counts
    const uint32_t* blk_count;
    int64_t nseg;
    uint32_t* dw_list;          // the dW kernel's list and count (place_segment)
    uint32_t* count;
    int L, Ld, n_layers;
    uint32_t skips;
    int slot_bytes;
    StreamDesc sd;  // W^T images: dir, feat, trunk n-1..1 [, trunk 0 when g_x/g_d]
    int64_t vsig, vrgb;
    int64_t mask_off;
    int n_mask;
    int64_t ws_off[kMaxTrunk + 3];
    int ws_feat, ws_dir, ws_heads;
};

template <int PREC, int XB, int DB, int TPW, int G, int NT, bool WANT_X>
__global__ __launch_bounds__(NT, 1) void mlp_bwd_kernel(BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, ml = lane & 31;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    // wave -> its tile (select_tile; one tile per wave); waves without one run on zero
    // inputs and store nothing
    static_assert(TPW == 1, "the active-tile selection gives each wave one tile");
    const TileSel ts = select_tile(a.flags, a.blk_count, a.nseg, a.tiles, NT / 64, wv);
    if (ts.idle) {  // workgroup-uniform
        finish_tiles(ts, a.nseg, a.tiles, a.dw_list, a.count);
        return;
    }
    const bool live = ts.live;
    const int64_t tile0 = live ? ts.tile : 0;
    const int n = a.n_layers;
    const u32x4* masks = reinterpret_cast<const u32x4*>(a.saved + a.mask_off);
    bool tok[TPW];
    unsigned tokm = 0u;
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        tok[t] = live;
        tokm |= (tok[t] ? 1u : 0u) << t;
    }
    // each dz image is saved while the next stream consumes it
    auto sink_of = [&](int wsid, int nblk) {
        return Sink<PREC, TPW>{NR_SINK_BWD ? a.ws + a.ws_off[wsid] : nullptr, nblk, tile0, tokm};
    };
    auto store_dz = [&](int wsid, int nblk, int t, int nb, const InBlk<PREC>& v) {
        if (tok[t]) store_img<PREC>(a.ws + a.ws_off[wsid], tile0 + t, nblk, nb, v, lane);
    };
    auto put_dz = [&](int wsid, int nblk, int t, int nb, const InBlk<PREC>& v) {
        if (!NR_SINK_BWD) store_dz(wsid, nblk, t, nb, v);
    };
    auto mask_of = [&](int t, int layer) -> u32x4 {
        return tok[t] ? masks[((tile0 + t) * a.n_mask + layer) * 64 + lane] : u32x4{0u, 0u, 0u, 0u};
    };

    Ring ring{lds, a.slot_bytes, 0, nullptr, wv};
    Stager<G, NT> st;
    stream_begin(ring, st, a.packed, a.sd, tid);

    // heads: sigmoid / relu backward (torch: g * (1 - y) * y ; g * (y > 0))
    constexpr int NC = kHB / 2;
    float dzs[TPW];
    Act<PREC, TPW, NC, false> cin;
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const int64_t m = (tile0 + t) * 32 + ml;
        const bool valid = tok[t] && m < a.M;
        float dr[3] = {0.f, 0.f, 0.f};
        dzs[t] = 0.f;
        if (valid) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float y = a.rgb[3 * m + c];
                dr[c] = ((a.g_rgb[3 * m + c] * (1.0f - y)) * y) * a.gscale;
            }
            dzs[t] = (a.sigma[m] > 0.f ? a.g_sigma[m] : 0.f) * a.gscale;
        }
        if (tok[t]) {
            // dz of the heads as one 32-feature block: feature 0 sigma, 1..3 rgb
            f32x16 hb;
            zero(hb);
            if (h == 0) {
                hb[0] = dzs[t];
                hb[1] = dr[0];
                hb[2] = dr[1];
                hb[3] = dr[2];
            }
            InBlk<PREC> hv;
            to_in<PREC>(hb, hv);
            store_img<PREC>(a.ws + a.ws_off[a.ws_heads], tile0 + t, 1, 0, hv, lane);
        }
        // dz_c = (W_rgb^T dz_rgb) * [h_c > 0]
        f32x16 dc[NC];
        const PImg wr0 = pimg(a.packed, a.vrgb), wr1 = pimg(a.packed, a.vrgb + NC * 128),
                   wr2 = pimg(a.packed, a.vrgb + 2 * NC * 128);
#pragma unroll
        for (int nb = 0; nb < NC; ++nb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                f32x2 v = wr0.at(nb, r) * bcast2(dr[0]);
                v = __builtin_elementwise_fma(wr1.at(nb, r), bcast2(dr[1]), v);
                v = __builtin_elementwise_fma(wr2.at(nb, r), bcast2(dr[2]), v);
                dc[nb][r] = h ? v[1] : v[0];
            }
        const u32x4 mwc = mask_of(t, n);
#pragma unroll
        for (int nb = 0; nb < NC; ++nb) {
            to_in_masked<PREC>(dc[nb], mwc, nb, cin.v[t][nb]);
            put_dz(a.ws_dir, NC, t, nb, cin.v[t][nb]);
        }
    }

    // d [feat | d_enc] = W_dir^T dz_c   (feature_linear has no activation: dz_feat = d feat)
    f32x16 acc[TPW][kHB];
    constexpr bool ACT_LDS = k16<PREC> && NT == 512;
    Act<PREC, TPW, kHB, ACT_LDS> hin;
    if constexpr (ACT_LDS)
        hin.base = lds + 2 * a.slot_bytes + wv * Act<PREC, TPW, kHB, ACT_LDS>::kBytes;
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) zero(acc[t][nb]);
    constexpr int DBX = (WANT_X && DB > 0) ? DB : 0;
    f32x16 dd[TPW][DBX > 0 ? DBX : 1];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int k = 0; k < (DBX > 0 ? DBX : 1); ++k) zero(dd[t][k]);
    stream_gemm<PREC, TPW, kHB, DBX, NC, G, NT>(acc, dd, 0, cin, ring, st, a.packed, a.sd, tid, lane,
                                                sink_of(a.ws_dir, NC));
    if constexpr (DBX > 0) {
        if (a.g_d) {
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                const int64_t m = (tile0 + t) * 32 + ml;
                const bool valid = tok[t] && m < a.M;
                const float d0 = valid ? a.d[3 * m] : 0.f, d1 = valid ? a.d[3 * m + 1] : 0.f,
                            d2 = valid ? a.d[3 * m + 2] : 0.f;
                float g0 = 0.f, g1 = 0.f, g2 = 0.f;
#pragma unroll
                for (int kb = 0; kb < DBX; ++kb)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        pe_feat_bwd(d0, d1, d2, 32 * kb + acc_row(r, h), a.Ld, dd[t][kb][r], g0, g1, g2);
                g0 += __shfl_xor(g0, 32);
                g1 += __shfl_xor(g1, 32);
                g2 += __shfl_xor(g2, 32);
                if (valid && h == 0) {
                    a.g_d[3 * m] = g0 * a.inv_gscale;
                    a.g_d[3 * m + 1] = g1 * a.inv_gscale;
                    a.g_d[3 * m + 2] = g2 * a.inv_gscale;
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) {
            InBlk<PREC> v;
            to_in<PREC>(acc[t][nb], v);
            hin.put(t, nb, v);
            put_dz(a.ws_feat, kHB, t, nb, v);
        }

    // d h_{n-1} = W_feat^T dz_feat + w_sigma dz_sigma, then * [h_{n-1} > 0]
    f32x16 dummy[TPW][1];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) zero(acc[t][nb]);
    // the ReLU masks this stream's output needs are loaded before it (the stream's
    // asm barriers keep loads from being hoisted over it by the compiler)
    u32x4 mwf[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) mwf[t] = mask_of(t, n - 1);
    stream_gemm<PREC, TPW, kHB, 0, kHB, G, NT>(acc, dummy, 0, hin, ring, st, a.packed, a.sd, tid, lane,
                                               sink_of(a.ws_feat, kHB));
    {
        const PImg ws = pimg(a.packed, a.vsig);
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb)
#pragma unroll
            for (int r = 0; r < 16; ++r)
#pragma unroll
                for (int t = 0; t < TPW; ++t) {
                    const f32x2 v = __builtin_elementwise_fma(ws.at(nb, r), bcast2(dzs[t]), bcast2(acc[t][nb][r]));
                    acc[t][nb][r] = h ? v[1] : v[0];
                }
    }
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) {
            InBlk<PREC> v;
            to_in_masked<PREC>(acc[t][nb], mwf[t], nb, v);
            hin.put(t, nb, v);
            if ((n == 1 && !WANT_X) || !NR_SINK_BWD)  // (dz_0 without g_x has no consumer stream)
                store_dz(WS_DZ0 + n - 1, kHB, t, nb, v);
        }
    }

    // trunk: dz_{i-1} = (W_i^T dz_i)[h rows] * [h_{i-1} > 0]; x_enc rows feed g_x
    constexpr int XBX = WANT_X ? XB : 0;
    f32x16 dxe[TPW][XBX > 0 ? XBX : 1];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int k = 0; k < (XBX > 0 ? XBX : 1); ++k) zero(dxe[t][k]);
    for (int i = n - 1; i >= 1; --i) {
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
            for (int nb = 0; nb < kHB; ++nb) zero(acc[t][nb]);
        u32x4 mwt[TPW];
#pragma unroll
        for (int t = 0; t < TPW; ++t) mwt[t] = mask_of(t, i - 1);
        if ((a.skips >> (i - 1)) & 1u) {
            // W^T row blocks of a skip layer are [h (8) | x_enc (XB)]; without g_x
            // only the h rows are streamed
            if constexpr (XBX > 0)
                stream_gemm<PREC, TPW, kHB, XBX, kHB, G, NT>(acc, dxe, 0, hin, ring, st, a.packed, a.sd, tid, lane,
                                                             sink_of(WS_DZ0 + i, kHB));
            else
                stream_gemm<PREC, TPW, kHB, 0, kHB, G, NT>(acc, dummy, 0, hin, ring, st, a.packed, a.sd, tid, lane,
                                                           sink_of(WS_DZ0 + i, kHB));
        } else {
            stream_gemm<PREC, TPW, kHB, 0, kHB, G, NT>(acc, dummy, 0, hin, ring, st, a.packed, a.sd, tid, lane,
                                                       sink_of(WS_DZ0 + i, kHB));
        }
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
#pragma unroll
            for (int nb = 0; nb < kHB; ++nb) {
                InBlk<PREC> v;
                to_in_masked<PREC>(acc[t][nb], mwt[t], nb, v);
                hin.put(t, nb, v);
                if ((i == 1 && !WANT_X) || !NR_SINK_BWD)  // (dz_0 without g_x has no consumer stream)
                    store_dz(WS_DZ0 + i - 1, kHB, t, nb, v);
            }
        }
    }
    if constexpr (XBX > 0) {
        stream_gemm<PREC, TPW, XBX, 0, kHB, G, NT>(dxe, dummy, 0, hin, ring, st, a.packed, a.sd, tid, lane,
                                                   sink_of(WS_DZ0, kHB));
        if (a.g_x) {
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                const int64_t m = (tile0 + t) * 32 + ml;
                const bool valid = tok[t] && m < a.M;
                const float x0 = valid ? a.x[3 * m] : 0.f, x1 = valid ? a.x[3 * m + 1] : 0.f,
                            x2 = valid ? a.x[3 * m + 2] : 0.f;
                float g0 = 0.f, g1 = 0.f, g2 = 0.f;
#pragma unroll
                for (int kb = 0; kb < XBX; ++kb)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        pe_feat_bwd(x0, x1, x2, 32 * kb + acc_row(r, h), a.L, dxe[t][kb][r], g0, g1, g2);
                g0 += __shfl_xor(g0, 32);
                g1 += __shfl_xor(g1, 32);
                g2 += __shfl_xor(g2, 32);
                if (valid && h == 0) {
                    a.g_x[3 * m] = g0 * a.inv_gscale;
                    a.g_x[3 * m + 1] = g1 * a.inv_gscale;
                    a.g_x[3 * m + 2] = g2 * a.inv_gscale;
                }
            }
        }
    }
    finish_tiles(ts, a.nseg, a.tiles, a.dw_list, a.count);
}

// ------------------------------------------------ input gradients ------
// dL/dx and dL/dd of the 16-bit path (the pose-optimisation gradient, BASELINE
// cfg #3) as a separate pass over the dz images the dX chain stores anyway:
//   d x_enc = sum over the x_enc-reading layers l (0 and every skip layer) of
//             W_l[:, x_enc]^T dz_l,        d d_enc = W_dir[:, d_enc]^T dz_dir,
// then the positional-encoding backward.  Replaces the input-gradient variant of
// mlp_bwd_kernel, which carries d x_enc through the whole trunk and therefore runs
// 4 waves per CU (2.23 ms vs 1.17 ms for the plain dX chain).
// One wave per 32-sample tile; the A fragments are the W^T images' x_enc / d_enc
// row blocks (gathered into LDS once per workgroup), the B operands the stored dz
// blocks.  fp32 accumulation, the same products as the fused variant.  HBM-bound:
// 1.28 KB of dz per sample for the default model (dz_0, dz_skip, dz_c).
struct DinArgs {
    const char* packed;
    const char* ws;
    const float* x;
    const float* d;
    float* g_x;
    float* g_d;
    int64_t M, tiles;
    const uint8_t* flags;         // active tiles (tile_flags_kernel): the others have dz == 0
    int L, Ld;
    float inv_gscale;
    int nsrc;                     // x_enc-reading layers
    int64_t a_off[kMaxTrunk];     // byte offset of the layer's W^T image
    int a_kb[kMaxTrunk];          // row blocks per chunk of that image
    int a_p0[kMaxTrunk];          // first x_enc row block within a chunk
    int64_t dz_off[kMaxTrunk];    // byte offset of the layer's dz image in ws
    int64_t dir_a_off, dz_dir_off;
    int dir_kb, dir_p0, nc;       // dir W^T chunk rows, first d_enc row, dz_dir blocks
};

constexpr int kDinNT = 512;

// The x_enc / d_enc row blocks of every source W^T image, gathered fragment by
// fragment: [source][dz block][row block][2] then [dz_c block][row block][2] (1 KB each).
__host__ __device__ inline int din_frags(int nsrc, int XB, int DB, int nc) { return 2 * (nsrc * kHB * XB + nc * DB); }

template <int PREC, int XB, int DB, bool ALDS>
__global__ __launch_bounds__(kDinNT) void mlp_dinput_kernel(DinArgs a) {
    static_assert(k16<PREC>, "16-bit images only");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int lane = threadIdx.x & 63, h = lane >> 5, ml = lane & 31;
    // A operands: staged once per workgroup into LDS (72 KB for the default model), or
    // read from the L2-resident packed buffer when they do not fit
    auto frag_src = [&](int f) -> const char* {  // global address of gathered fragment f (lane 0)
        const int nx = 2 * a.nsrc * kHB * XB;
        if (f < nx) {
            const int s = f / (2 * kHB * XB), r = f % (2 * kHB * XB);
            const int ob = r / (2 * XB), q = r % (2 * XB);
            return a.packed + a.a_off[s] + static_cast<int64_t>((ob * a.a_kb[s] + a.a_p0[s]) * 2 + q) * kFragBytes;
        }
        const int r = f - nx, ob = r / (2 * DB > 0 ? 2 * DB : 1), q = r % (2 * DB > 0 ? 2 * DB : 1);
        return a.packed + a.dir_a_off + static_cast<int64_t>((ob * a.dir_kb + a.dir_p0) * 2 + q) * kFragBytes;
    };
    if constexpr (ALDS) {
        const int nf = din_frags(a.nsrc, XB, DB, a.nc);
        for (int i = threadIdx.x; i < nf * 64; i += kDinNT) {
            const int f = i >> 6, l = i & 63;
            *reinterpret_cast<u32x4*>(lds + f * kFragBytes + l * 16) =
                *reinterpret_cast<const u32x4*>(frag_src(f) + l * 16);
        }
        __syncthreads();
    }
    auto afrag = [&](int f) -> bf16x8 {
        if constexpr (ALDS)
            return *reinterpret_cast<const bf16x8*>(lds + f * kFragBytes + lane * 16);
        else
            return *reinterpret_cast<const bf16x8*>(frag_src(f) + lane * 16);
    };
    const int64_t waves = static_cast<int64_t>(gridDim.x) * (kDinNT / 64);
    for (int64_t tile = static_cast<int64_t>(blockIdx.x) * (kDinNT / 64) + (threadIdx.x >> 6); tile < a.tiles;
         tile += waves) {
        const int64_t tile_u = __builtin_amdgcn_readfirstlane(static_cast<int>(tile));
        const int64_t m = tile * 32 + ml;
        const bool valid = m < a.M;
        if (!a.flags[tile_u]) {
            // no incoming gradient in this tile: its dz were never computed, and its input
            // gradients are exactly zero
            if (valid && h == 0)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    if (a.g_x) a.g_x[3 * m + c] = 0.f;
                    if (a.g_d) a.g_d[3 * m + c] = 0.f;
                }
            continue;
        }
        if (a.g_x) {
            f32x16 dxe[XB];
#pragma unroll
            for (int q = 0; q < XB; ++q) zero(dxe[q]);
            for (int s = 0; s < a.nsrc; ++s) {
                InBlk<PREC> b[kHB];
#pragma unroll
                for (int ob = 0; ob < kHB; ++ob) load_img<PREC>(a.ws + a.dz_off[s], tile_u, kHB, ob, b[ob], lane);
#pragma unroll
                for (int ob = 0; ob < kHB; ++ob)
#pragma unroll
                    for (int q = 0; q < XB; ++q) {
                        const int f = ((s * kHB + ob) * XB + q) * 2;
                        dxe[q] = mfma16<PREC>(afrag(f), b[ob].s[0], dxe[q]);
                        dxe[q] = mfma16<PREC>(afrag(f + 1), b[ob].s[1], dxe[q]);
                    }
            }
            const PeRev pr = pe_rev(valid ? a.x[3 * m] : 0.f, valid ? a.x[3 * m + 1] : 0.f,
                                    valid ? a.x[3 * m + 2] : 0.f);
            float g0 = 0.f, g1 = 0.f, g2 = 0.f;
#pragma unroll
            for (int kb = 0; kb < XB; ++kb)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    pe_fast_bwd(pr, 32 * kb + acc_row(r, 0), 32 * kb + acc_row(r, 1), h != 0, a.L, dxe[kb][r], g0, g1,
                                g2);
            g0 += __shfl_xor(g0, 32);
            g1 += __shfl_xor(g1, 32);
            g2 += __shfl_xor(g2, 32);
            if (valid && h == 0) {
                a.g_x[3 * m] = g0 * a.inv_gscale;
                a.g_x[3 * m + 1] = g1 * a.inv_gscale;
                a.g_x[3 * m + 2] = g2 * a.inv_gscale;
            }
        }
        if constexpr (DB > 0) {
            if (a.g_d) {
                f32x16 dd[DB];
#pragma unroll
                for (int q = 0; q < DB; ++q) zero(dd[q]);
                const int f0 = 2 * a.nsrc * kHB * XB;
                for (int ob = 0; ob < a.nc; ++ob) {
                    InBlk<PREC> b;
                    load_img<PREC>(a.ws + a.dz_dir_off, tile_u, a.nc, ob, b, lane);
#pragma unroll
                    for (int q = 0; q < DB; ++q) {
                        const int f = f0 + (ob * DB + q) * 2;
                        dd[q] = mfma16<PREC>(afrag(f), b.s[0], dd[q]);
                        dd[q] = mfma16<PREC>(afrag(f + 1), b.s[1], dd[q]);
                    }
                }
                const PeRev pr = pe_rev(valid ? a.d[3 * m] : 0.f, valid ? a.d[3 * m + 1] : 0.f,
                                        valid ? a.d[3 * m + 2] : 0.f);
                float g0 = 0.f, g1 = 0.f, g2 = 0.f;
#pragma unroll
                for (int kb = 0; kb < DB; ++kb)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        pe_fast_bwd(pr, 32 * kb + acc_row(r, 0), 32 * kb + acc_row(r, 1), h != 0, a.Ld, dd[kb][r], g0,
                                    g1, g2);
                g0 += __shfl_xor(g0, 32);
                g1 += __shfl_xor(g1, 32);
                g2 += __shfl_xor(g2, 32);
                if (valid && h == 0) {
                    a.g_d[3 * m] = g0 * a.inv_gscale;
                    a.g_d[3 * m + 1] = g1 * a.inv_gscale;
                    a.g_d[3 * m + 2] = g2 * a.inv_gscale;
                }
            }
        }
    }
}

// ----------------------------------------------------- active tiles ----
// The backward's work list.  A sample whose sigma is exactly 0 (alpha = w = 0, and
// ReLU'(0) = 0 on sigma: reference rendering.py:83) or whose transmittance has
// underflowed to 0 (the cumprod of 1 - alpha + 1e-10, rendering.py:87-96) receives
// exactly zero g_rgb and g_sigma, so every layer's dz for it is zero.  A 32-sample
// tile of such samples only adds exact zeros to dW, so the dX chain, the dW GEMM and
// the input gradients run over the tiles with ANY nonzero incoming gradient (computed
// from the values, never assumed).  One launch, no global scan: the tiles form
// segments of kSegTiles; the launch writes one flag byte per tile and the active count
// of every 64-tile block.  The dX workgroups pick their tiles from those (select_tile:
// the dense order when every tile is active, else eight (four) of a segment's active
// tiles found by a wave scan of its 256 flag bytes), and the segments' leaders
// concatenate them into the dW kernel's list (place_segment), which that kernel splits
// evenly over its chunks.  With every tile active, each kernel sees exactly the dense
// form's tiles in order.
constexpr int kTileFlagThreads = 256;  // 4 waves x 16 tiles: one 64-tile block per workgroup

__global__ __launch_bounds__(kTileFlagThreads) void tile_flags_kernel(const float* __restrict__ g_rgb,
                                                                      const float* __restrict__ g_sigma, int64_t M,
                                                                      int dense,
                                                                      uint8_t* __restrict__ flags,
                                                                      uint32_t* __restrict__ blk_count) {
    __shared__ uint32_t wcnt[kTileFlagThreads / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t tw = static_cast<int64_t>(blockIdx.x) * 64 + wv * 16;
    bool nz[8];
    // lanes 0-31: tile tw + 2 it, lanes 32-63: tile tw + 2 it + 1 (one sample each)
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int64_t m = (tw + 2 * it + (lane >> 5)) * 32 + (lane & 31);
        bool v = false;
        if (m < M) {
            if (dense) {
                v = true;
            } else {
                const float r0 = g_rgb[3 * m], r1 = g_rgb[3 * m + 1], r2 = g_rgb[3 * m + 2], s0 = g_sigma[m];
                v = (r0 != 0.f) | (r1 != 0.f) | (r2 != 0.f) | (s0 != 0.f);  // NaN counts as nonzero
            }
        }
        nz[it] = v;
    }
    uint32_t mask = 0;  // bit k: tile tw + k is active (wave-uniform); tiles past the last sample: 0
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const uint64_t b = __ballot(nz[it]);
        mask |= (static_cast<uint32_t>(b & 0xffffffffull) != 0 ? 1u : 0u) << (2 * it);
        mask |= (static_cast<uint32_t>(b >> 32) != 0 ? 1u : 0u) << (2 * it + 1);
    }
    if (lane < 16) flags[tw + lane] = static_cast<uint8_t>((mask >> lane) & 1u);
    if (lane == 0) wcnt[wv] = __popc(mask);
    __syncthreads();
    if (threadIdx.x == 0) blk_count[blockIdx.x] = ((wcnt[0] + wcnt[1]) + wcnt[2]) + wcnt[3];
}

// ------------------------------------------------------------------ dW ----
// Workgroup = (job, chunk of tiles): 8 waves, each accumulating its planned share
// (DwWave: up to 5x2 blocks) of the job's NBz x KB output grid.  Per tile the
// job's dz and input blocks (every tensor once: h_{n-1} feeds the feature layer
// and the sigma head in one job) are staged into LDS by LDS-DMA (a 4-stage ring of
// 1-KB wave pieces) and the sample-major MFMA operands are rebuilt from the
// B-operand images.  Bias partials are v_dot2 sums of the dz operands.  Output
// slab per chunk: [dz row][input col | bias] fp32.  The kernel runs at its staging
// ceiling: the same staging with the MFMAs compiled out (a timing-only variant,
// r02) is within 1 % of it.
#ifndef NR_DW_NSTAGE
#define NR_DW_NSTAGE 4  // LDS staging ring depth of the dW kernel (tiles)
#endif
#ifndef NR_DW_AUX
#define NR_DW_AUX 0  // cache-policy bits of the dW staging loads (2: nt)
#endif
#ifndef NR_DW_ONESHAPE
#define NR_DW_ONESHAPE 0  // A/B only: every 16-bit wave share runs as 5x2
#endif
constexpr int kDwThreads = 512;
constexpr int kDwWaves = kDwThreads / 64;
static_assert(kDwWaves == kDwMaxWaves, "dW wave shares are planned for 8-wave workgroups");

constexpr int kDwMaxWgs = 256;  // one round of workgroups (make_sizes: NR_DW_WGS)
struct DwArgs {
    float* slabs;
    int njobs;
    int64_t tiles;
    const uint32_t* list;           // active tiles in order and their count (built during the dX launch)
    const uint32_t* count;
    int list_lds;                   // LDS byte offset the chunk's list entries are staged to (0: read them global)
    int job_chunks[kMaxJobs];       // chunks of each job: list entries split evenly in order
    uint16_t wg_map[kDwMaxWgs];     // workgroup -> job | chunk << 5 (chunk-major: one chunk of every job in a row)
    int stage_bytes, nstage;
    int64_t slab_floats_per_chunk;
    int job_NBz[kMaxJobs], job_KB[kMaxJobs];
    int64_t job_slab[kMaxJobs];
    const char* seg_ptr[kMaxJobs][2 * kMaxJobSeg];  // tensor region: dz segments, then inputs
    uint8_t seg_blocks[kMaxJobs][2 * kMaxJobSeg];
    // wave share (DwWave) packed: row0 | np << 6 | col0 << 9 | nq << 15 | bias << 17; 0 = idle
    int job_wave[kMaxJobs][kDwWaves];
};
static_assert(sizeof(DwArgs) <= 4096, "dW kernel arguments exceed 4 KiB");

__host__ __device__ constexpr int dw_wave_pack(int row0, int np, int col0, int nq, int bias) {
    return row0 | np << 6 | col0 << 9 | nq << 15 | bias << 17;
}

// Block-local feature of dW operand row/col index r: r = 16h + i <-> accumulator
// register i of lane half h in the B-operand image.
__device__ __forceinline__ int dw_feat(int r) { return acc_row(r & 15, r >> 4); }

// bf16 staging swizzle: image lane L of fragment s sits in LDS slot
// L ^ 4*(L>>5 & 1) ^ 8*s (an involution), which makes the transpose reads of
// dw_frag_bf16 bank-conflict free (the 16 slots a 32-lane half reads are
// distinct mod 16).  glds writes lane-linear, so the swizzle goes on the source.
__device__ __forceinline__ int dw_slot(int L, int s) { return L ^ (((L >> 5) & 1) << 2) ^ (s << 3); }
// fp32 staging: fragment f's 16-B chunk c lands at chunk position c ^ 2 (f + 4 (c >> 5))
// (an involution: bits 1-3 only), so the per-sample reads of mlp_dw_kernel's fp32 path
// spread over all 16 four-bank groups instead of 2 (8-way conflicts)
__device__ __forceinline__ int dw_slot32(int L, int f) { return L ^ (2 * (f + 4 * ((L >> 5) & 1))); }

// ds_read_b64_tr_b16 through inline asm: the builtin makes hipcc wait vmcnt(0)
// (every in-flight LDS-DMA stage) before each read, which would serialise the
// staging pipeline.  The caller waits lgkmcnt itself (tr_wait) before use.
template <int OFF>
__device__ __forceinline__ void tr16(uint64_t& out, uint32_t addr) {
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(out) : "v"(addr), "i"(OFF));
}

// the two 64-bit halves of a transpose-read operand as one bf16x8 (a pure bit cast, so
// the register allocator can place the two asm outputs as the halves: no copies)
typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
// ds_read_b32 through inline asm (as tr16: no compiler drain of in-flight LDS-DMA)
template <int OFF>
__device__ __forceinline__ void ds_rd32(float& out, uint32_t addr) {
    asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(out) : "v"(addr), "i"(OFF));
}

__device__ __forceinline__ bf16x8 tr_pair(uint64_t lo, uint64_t hi) {
    return __builtin_bit_cast(bf16x8, u64x2_t{lo, hi});
}

// LDS byte offsets, within a staged block, of the two transpose reads that give
// lane l its bf16 operand for k-step ks: lane l = 16g + i (h = g&1, hh = g>>1)
// receives feature acc_row(i, h) of samples 16ks + 8hh + 0..7 (two reads of 4
// samples x 16 features; lane 4q+p of a group addresses sample q, features
// 4p..4p+3: cdna_hip_programming.md T10).
__device__ __forceinline__ uint32_t dw_tr_off(int ks, int half, int lane) {
    const int g = lane >> 4, h = g & 1, hh = g >> 1;
    const int lam = lane & 15, q = lam >> 2, p = lam & 3;
    const int s = p >> 1;
    const int L = 16 * ks + 8 * hh + q + 32 * h + 4 * half;
    return static_cast<uint32_t>(s * kFragBytes + dw_slot(L, s) * 16 + 8 * (p & 1));
}

// acc + the four 16-bit values of a transpose read (bias partial sums): two
// v_dot2c_f32_{bf16,f16} against (1, 1), fp32 accumulation
template <int PREC>
__device__ __forceinline__ float dw_acc4(uint64_t v, float acc) {
    const unsigned w0 = static_cast<unsigned>(v), w1 = static_cast<unsigned>(v >> 32);
    if constexpr (PREC == NR_PREC_FP16) {
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        const h2 one = __builtin_bit_cast(h2, 0x3c003c00u);
        acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, w0), one, acc, false);
        return __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, w1), one, acc, false);
    } else {
        typedef __bf16 b2 __attribute__((ext_vector_type(2)));
        const b2 one = __builtin_bit_cast(b2, 0x3f803f80u);
        acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b2, w0), one, acc, false);
        return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b2, w1), one, acc, false);
    }
}

template <int PREC>
__global__ __launch_bounds__(kDwThreads, 1) void mlp_dw_kernel(DwArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar staging loop
    // chunk-major (wg_map): every job of a chunk runs at about the same time (an input two
    // jobs share, x_enc of the x-jobs beyond the first, is re-read from L2/MALL)
    const int wmap = a.wg_map[blockIdx.x];
    const int j = wmap & 31, chunk = wmap >> 5;
    const int NBz = a.job_NBz[j], KB = a.job_KB[j];
    const int winfo = a.job_wave[j][wv];
    const int row0 = winfo & 63, np = (winfo >> 6) & 7, col0 = (winfo >> 9) & 63, nq = (winfo >> 15) & 3;
    const bool active = np > 0;
    const bool do_bias = active && ((winfo >> 17) & 1);
    // this chunk's entries [t0, t1) of the active-tile list: ceil(count / chunks) each, in
    // list order (with every tile active, exactly the dense form's contiguous ranges)
    const int64_t cnt = *a.count;
    const int64_t tpc = (cnt + a.job_chunks[j] - 1) / a.job_chunks[j];
    const int64_t t0 = static_cast<int64_t>(chunk) * tpc;
    int64_t t1 = t0 + tpc;
    if (t1 > cnt) t1 = cnt;
    constexpr int FPB = kFPB<PREC>;
    constexpr int BLK = FPB * kFragBytes;

    // Stage tile t into buffer b (the job's blocks, dz segments first).  Every wave
    // issues exactly `per_wave` 1-KB LDS-DMA pieces per tile (padding pieces re-load
    // piece 0 into a scratch KB), so a counted vmcnt can retire one stage while the
    // next NS-2 stay in flight across the barrier.  Each piece's per-lane source
    // address, per-tile stride and LDS offset are resolved once per workgroup: the
    // per-tile staging is one pointer bump and one DMA per piece (the segment walk
    // per piece and tile made this kernel SALU-bound).
    const int total = (NBz + KB) * FPB;
    const int per_wave = (total + kDwWaves - 1) / kDwWaves;
    constexpr int kMaxPW = dw_max_pieces(k16<PREC>);  // the plan keeps per_wave <= kMaxPW
    const char* psrc[kMaxPW];  // piece k of tile 0 (lane's 16 B); tile t adds t * pstride[k]
    int64_t pstride[kMaxPW];
    int pdst[kMaxPW];  // LDS offset within a stage, or -1: scratch KB
#pragma unroll
    for (int k = 0; k < kMaxPW; ++k) {
        psrc[k] = nullptr;
        pstride[k] = 0;
        pdst[k] = -1;
        if (k < per_wave) {
            int pc = wv + k * kDwWaves;
            const bool pad = pc >= total;
            if (pad) pc = 0;
            int sg = 0, p0 = 0;
            while (pc >= p0 + a.seg_blocks[j][sg] * FPB) p0 += a.seg_blocks[j][sg++] * FPB;
            const int nb = a.seg_blocks[j][sg];
            const int L = k16<PREC> ? dw_slot(lane, (pc - p0) % FPB) : dw_slot32(lane, (pc - p0) % FPB);
            pstride[k] = static_cast<int64_t>(nb) * BLK;
            psrc[k] = a.seg_ptr[j][sg] + (pc - p0) * kFragBytes + L * 16;
            pdst[k] = pad ? -1 : pc * kFragBytes;
        }
    }
    // this chunk's list entries, copied into LDS once when they fit (a scalar load per
    // stage would wait on the L2 inside the tile loop: lgkmcnt also counts the transpose reads)
    const uint32_t* lds_list = nullptr;
    if (a.list_lds && cnt != a.tiles) {  // (every tile active: the list is the identity)
        uint32_t* dst = reinterpret_cast<uint32_t*>(lds + a.list_lds);
        for (int64_t q = t0 + tid; q < t1; q += kDwThreads) dst[q - t0] = a.list[q];
        __syncthreads();  // (before any staging DMA is in flight)
        lds_list = dst;
    }
    // the tile of list entry pos: with every tile active the list is the identity (no read:
    // the dense form's cost); else from the LDS copy through asm with its own wait (a
    // compiler-visible LDS load behind the staging DMA makes hipcc wait vmcnt(0) for the
    // DMA, which writes LDS), or from the global list when the copy did not fit
    const bool ident = cnt == a.tiles;
    const uint32_t list_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds_list));
    auto tile_at = [&](int64_t pos) -> int64_t {
        if (ident) return pos;
        if (!lds_list) return a.list[pos];
        uint32_t v;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(v)
                     : "v"(list_base + 4u * static_cast<uint32_t>(pos - t0))
                     : "memory");
        return __builtin_amdgcn_readfirstlane(v);
    };
    // stage `tile` into buffer b
    auto stage = [&](int b, int64_t tile) {
        char* dst = lds + b * a.stage_bytes;
        char* scratch = lds + a.nstage * a.stage_bytes;
#pragma unroll
        for (int k = 0; k < kMaxPW; ++k) {
            if (k < per_wave) {
                char* d = pdst[k] < 0 ? scratch : dst + pdst[k];
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(psrc[k] + tile * pstride[k]),
                    (__attribute__((address_space(3))) void*)(d), 16, 0, NR_DW_AUX);
            }
        }
    };
    // wait until at most n of this wave's pieces are outstanding (n: wave-uniform)
    auto wait_pieces = [](int n) {
        switch (n) {
            case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
            case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
            case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
            case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
            default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        }
    };

    uint32_t trof[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) trof[ks][hf] = dw_tr_off(ks, hf, lane);
    const int NS = a.nstage;
    float* slab = a.slabs + static_cast<int64_t>(chunk) * a.slab_floats_per_chunk + a.job_slab[j];
    const int ld = KB * 32 + 1;
    const int hl = lane >> 5, ml = lane & 31;

    // The tile loop and the slab write for a compile-time share shape NP x NQ (16-bit:
    // the share's np x nq blocks run as the next compiled shape up, the extra blocks
    // accumulate garbage that is never written; fp32: kDwMaxP x kDwMaxQ with runtime
    // validity).  Each shape's accumulators live only inside its own instantiation.
    using std::integral_constant;
    auto run = [&](auto npc, auto nqc) {
        constexpr int NP = decltype(npc)::value, NQ = decltype(nqc)::value;
        f32x16 acc[NP][NQ];
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int q = 0; q < NQ; ++q) zero(acc[p][q]);
        float bsum[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) bsum[p] = 0.f;
        bool nval[NP], kval[NQ];
#pragma unroll
        for (int p = 0; p < NP; ++p) nval[p] = p < np;
#pragma unroll
        for (int q = 0; q < NQ; ++q) kval[q] = q < nq;

        for (int k = 0; k < NS - 1; ++k)
            if (t0 + k < t1) stage(k, tile_at(t0 + k));
        int bcur = 0, bnext = NS - 1;  // stage of tile t, stage tile t+NS-1 goes to
        for (int64_t t = t0; t < t1; ++t) {
            // stages t+1 .. t+NS-2 may stay in flight
            int64_t ahead = t1 - 1 - t;
            if (ahead > NS - 2) ahead = NS - 2;
            wait_pieces(per_wave * static_cast<int>(ahead));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (t + NS - 1 < t1) stage(bnext, tile_at(t + NS - 1));
            bnext = bnext + 1 == NS ? 0 : bnext + 1;
            const char* buf = lds + bcur * a.stage_bytes;
            bcur = bcur + 1 == NS ? 0 : bcur + 1;
            if (!active) continue;
            if constexpr (k16<PREC>) {
                const uint32_t base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(buf));
                const uint32_t bufA = base + row0 * BLK, bufB = base + (NBz + col0) * BLK;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    uint64_t ra[NP][2], rb[NQ][2];
#pragma unroll
                    for (int hf = 0; hf < 2; ++hf) {
                        const uint32_t oa = bufA + trof[ks][hf], ob = bufB + trof[ks][hf];
                        rbm_static_for<NP>(
                            [&](auto pp) { tr16<decltype(pp)::value * BLK>(ra[decltype(pp)::value][hf], oa); });
                        rbm_static_for<NQ>(
                            [&](auto qq) { tr16<decltype(qq)::value * BLK>(rb[decltype(qq)::value][hf], ob); });
                    }
                    // the wait publishes the transpose reads: tie every destination to it
                    // (volatile asm keeps its order) so no use is scheduled above it
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
                        for (int p = 0; p < NP; ++p) asm volatile("" : "+v"(ra[p][hf]));
#pragma unroll
                        for (int q = 0; q < NQ; ++q) asm volatile("" : "+v"(rb[q][hf]));
                    }
                    bf16x8 A[NP], Bm[NQ];
#pragma unroll
                    for (int p = 0; p < NP; ++p) A[p] = tr_pair(ra[p][0], ra[p][1]);
#pragma unroll
                    for (int q = 0; q < NQ; ++q) Bm[q] = tr_pair(rb[q][0], rb[q][1]);
                    // branch-free: per-MFMA validity branches made this loop SALU-bound
#pragma unroll
                    for (int p = 0; p < NP; ++p)
#pragma unroll
                        for (int q = 0; q < NQ; ++q) acc[p][q] = mfma16<PREC>(A[p], Bm[q], acc[p][q]);
                    // bias gradient = dz summed over samples: lane-local fp32 partials
                    if (do_bias)
#pragma unroll
                        for (int p = 0; p < NP; ++p) bsum[p] = dw_acc4<PREC>(ra[p][1], dw_acc4<PREC>(ra[p][0], bsum[p]));
                }
            } else {
                // fp32 image [tq][L][4]: operand row r <-> (hh = r>>4, reg i = r&15 -> frag i>>2,
                // elem i&3); sample m = 2 ss + kk is 16-B chunk 32 hh + m of the fragment,
                // staged at chunk position 32 hh + 2 (ss ^ k2) + kk (dw_slot32, k2 = frag + 4 hh):
                // the 16 chunks one read instruction touches fall in 16 distinct 4-bank groups
                const int r = lane & 31, kk = lane >> 5;
                const int hh = r >> 4, i = r & 15;
                const int k2 = (i >> 2) + 4 * hh;
                const uint32_t base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(buf)) +
                                      ((i >> 2) * 64 + 32 * hh + kk) * 16 + (i & 3) * 4;
                const uint32_t bufA = base + row0 * BLK, bufB = base + (NBz + col0) * BLK;
                const uint32_t kx = static_cast<uint32_t>(k2) << 5;
                // operands through asm reads (a plain LDS load makes the compiler drain every
                // in-flight staging DMA first), one sample pair read ahead; the compiled
                // share shape runs branch-free (blocks past np x nq accumulate garbage that
                // is never written, as in the 16-bit path)
                float Ar[2][NP], Br[2][NQ];
                auto rd = [&](auto sc) {
                    constexpr int ss = decltype(sc)::value;
                    // (ss ^ k2) << 5 computed in place: sixteen hoisted per-lane offsets would
                    // cost sixteen registers across the tile loop
                    uint32_t o;
                    asm volatile("v_xor_b32 %0, %1, %2" : "=v"(o) : "i"(ss << 5), "v"(kx));
                    const uint32_t oa = bufA + o, ob = bufB + o;
                    rbm_static_for<NP>([&](auto pp) { ds_rd32<decltype(pp)::value * BLK>(Ar[ss & 1][decltype(pp)::value], oa); });
                    rbm_static_for<NQ>([&](auto qq) { ds_rd32<decltype(qq)::value * BLK>(Br[ss & 1][decltype(qq)::value], ob); });
                };
                rd(integral_constant<int, 0>{});
                rbm_static_for<16>([&](auto sc) {
                    constexpr int ss = decltype(sc)::value;
                    if constexpr (ss + 1 < 16) {
                        rd(integral_constant<int, ss + 1>{});
                        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NP + NQ) : "memory");
                    } else {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    }
#pragma unroll
                    for (int p = 0; p < NP; ++p) asm volatile("" : "+v"(Ar[ss & 1][p]));
#pragma unroll
                    for (int q = 0; q < NQ; ++q) asm volatile("" : "+v"(Br[ss & 1][q]));
#pragma unroll
                    for (int p = 0; p < NP; ++p) {
                        bsum[p] += Ar[ss & 1][p];  // summed by every wave, written by the bias share's
#pragma unroll
                        for (int q = 0; q < NQ; ++q) acc[p][q] = mfma_f32(Ar[ss & 1][p], Br[ss & 1][q], acc[p][q]);
                    }
                });
            }
        }
        if (!active) return;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if (!nval[p]) continue;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                if (!kval[q]) continue;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = 32 * (row0 + p) + dw_feat(acc_row(r, hl));
                    const int col = 32 * (col0 + q) + dw_feat(ml);
                    slab[static_cast<int64_t>(row) * ld + col] = acc[p][q][r];
                }
            }
            if (do_bias) {
                // lanes l and l+32 summed the two sample halves of operand row l & 31
                const float tot = bsum[p] + __shfl_xor(bsum[p], 32);
                if (hl == 0) slab[static_cast<int64_t>(32 * (row0 + p) + dw_feat(ml)) * ld + KB * 32] = tot;
            }
        }
    };
    if constexpr (!k16<PREC> && !NR_DW_ONESHAPE) {
        // fp32: the plan keeps every share within 4 x 2 (the sigma head is its own job), so
        // one compiled 4x2 share: a wave pair on one SIMD runs 16 blocks per tile of an
        // h-job instead of the 20 of the 5x2 shape (a second shape in the kernel spills)
        run(integral_constant<int, 4>{}, integral_constant<int, kDwMaxQ>{});
    } else if constexpr (k16<PREC> && !NR_DW_ONESHAPE) {
        // compiled shares: 1x2, 4x1, 4x2, 5x2 (a smaller share runs the next one up)
        if (np <= 1)
            run(integral_constant<int, 1>{}, integral_constant<int, 2>{});
        else if (np <= 4 && nq <= 1)
            run(integral_constant<int, 4>{}, integral_constant<int, 1>{});
        else if (np <= 4)
            run(integral_constant<int, 4>{}, integral_constant<int, 2>{});
        else
            run(integral_constant<int, kDwMaxP>{}, integral_constant<int, kDwMaxQ>{});
    } else {
        run(integral_constant<int, kDwMaxP>{}, integral_constant<int, kDwMaxQ>{});
    }
}

// g_params[param] = sum over chunks of its slab entry (fixed chunk order: deterministic).
struct ReduceArgs {
    const float* slabs;
    float* g;
    float inv_gscale;  // fp16: undo the backward's loss scale (a power of two: exact)
    int64_t param_count;
    int64_t slab_floats_per_chunk;
    int n_red;
    int rows[kMaxRed], in[kMaxRed], nseg[kMaxRed], bjob[kMaxRed], brow0[kMaxRed];
    int64_t w_off[kMaxRed], b_off[kMaxRed];
    RedSeg seg[kMaxRed][kMaxSeg];
    int64_t job_slab[kMaxJobs];
    int job_KB[kMaxJobs];
    int job_chunks[kMaxJobs];  // slab sets of each job, summed in chunk order
};

// One workgroup per (reduce range k = blockIdx.y, output row r = blockIdx.x): the row's
// weight columns and its bias (column `in`) across the threads, so neither an index
// search per parameter nor a division; consecutive columns read consecutive slab floats.
__global__ void mlp_dw_reduce_kernel(ReduceArgs a) {
    const int k = blockIdx.y, r = blockIdx.x;
    if (r >= a.rows[k]) return;
    const int in = a.in[k];
    const int64_t st = a.slab_floats_per_chunk;
    for (int c = threadIdx.x; c <= in; c += blockDim.x) {
        int job = -1, row = 0, col = 0;
        int64_t dst;
        if (c < in) {
            for (int q = 0; q < a.nseg[k]; ++q) {
                const RedSeg& sg = a.seg[k][q];
                if (c >= sg.col0 && c < sg.col0 + sg.width) {
                    job = sg.job;
                    row = sg.slab_row0 + r;
                    col = sg.slab_col0 + (c - sg.col0);
                }
            }
            dst = a.w_off[k] + static_cast<int64_t>(r) * in + c;
        } else {
            job = a.bjob[k];
            row = a.brow0[k] + r;
            col = a.job_KB[job] * 32;
            dst = a.b_off[k] + r;
        }
        if (job < 0) continue;
        const int ld = a.job_KB[job] * 32 + 1;
        const float* s = a.slabs + a.job_slab[job] + static_cast<int64_t>(row) * ld + col;
        // chunk order fixed (deterministic); loads issued four at a time
        const int nch = a.job_chunks[job];
        float acc = 0.f;
        int ch = 0;
        for (; ch + 4 <= nch; ch += 4) {
            const float v0 = s[ch * st], v1 = s[(ch + 1) * st], v2 = s[(ch + 2) * st], v3 = s[(ch + 3) * st];
            acc = (((acc + v0) + v1) + v2) + v3;
        }
        for (; ch < nch; ++ch) acc += s[ch * st];
        a.g[dst] = acc * a.inv_gscale;
    }
}

// ---------------------------------------------------------------- pack ----
// Every pack kernel has an index mode (IDX): instead of writing a parameter's value
// into an image it records where it goes, in the destination table of the fused
// optimizer step (nr_adam_multi): table[slot * n + i] = kind << 29 | byte offset
// for flat parameter i.  Slot 0: the forward W image, a bias fragment or a pair
// image; 1: the W^T image or a vector image; 2: the 16-bit dX-chain image.  The
// same index maps fill both, so a refresh through the table writes exactly the
// bytes nr_mlp_pack writes.
constexpr int kPackSlots = 3;
enum : uint32_t { kDstNone = 0, kDstF32 = 1, kDstBf16 = 2, kDstF16 = 3, kDstFragBf16 = 4, kDstFragF16 = 5 };
constexpr int64_t kDstMaxOff = int64_t(1) << 29;
struct PackIdx {
    uint32_t* table;
    int64_t n;  // flat parameters
};
__device__ __forceinline__ void put_dst(const PackIdx& t, int slot, int64_t pidx, int64_t off, uint32_t kind) {
    t.table[slot * t.n + pidx] = (kind << 29) | static_cast<uint32_t>(off);
}
__device__ __forceinline__ uint32_t dst16(int prec) { return prec == NR_PREC_FP16 ? kDstF16 : kDstBf16; }

// Image element e of layer l (fwd: W, bwd: W^T), chunk-major:
//   e = (((kblock * ROWBLOCKS + rowblock) * FPB + frag) * 64 + lane) * EPL + el
struct PackArgs {
    const float* params;
    char* packed;
    int n_lin;
    int prec;
    int64_t w_off[kMaxMfmaLayers];
    int in[kMaxMfmaLayers], NB[kMaxMfmaLayers], KB[kMaxMfmaLayers], nseg[kMaxMfmaLayers];
    int seg_col0[kMaxMfmaLayers][kMaxSeg], seg_w[kMaxMfmaLayers][kMaxSeg], seg_blk[kMaxMfmaLayers][kMaxSeg];
    int64_t pk[kMaxMfmaLayers], pkb[kMaxMfmaLayers];
    int bwd_rot[kMaxMfmaLayers];  // W^T row-block rotation: skip layers put the h rows first
    int64_t cum[kMaxMfmaLayers + 1];
};

// W column of local input index c (0..31) in input block kb, or -1 for padding.
__device__ __forceinline__ int pack_col(const PackArgs& a, int l, int kb, int c) {
    int blk0 = 0;
    for (int s = 0; s < a.nseg[l]; ++s) {
        if (kb < blk0 + a.seg_blk[l][s]) {
            const int cs = 32 * (kb - blk0) + c;
            return cs < a.seg_w[l][s] ? a.seg_col0[l][s] + cs : -1;
        }
        blk0 += a.seg_blk[l][s];
    }
    return -1;
}

template <bool IDX>
__global__ void mlp_pack_kernel(PackArgs a, PackIdx t) {
    const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g >= a.cum[a.n_lin]) return;
    int l = 0;
    while (g >= a.cum[l + 1]) ++l;
    const int64_t img = (a.cum[l + 1] - a.cum[l]) / 2;
    int64_t e = g - a.cum[l];
    const bool bwd = e >= img;
    if (bwd) e -= img;
    const bool bf = a.prec != NR_PREC_FP32;  // 16-bit image (bf16 or fp16)
    const int epl = bf ? 8 : 4, fpb = bf ? 2 : 4;
    const int64_t frag = e / (64 * epl);
    const int lane = static_cast<int>((e / epl) % 64);
    const int el = static_cast<int>(e % epl);
    const int64_t blk = frag / fpb;
    const int sub = static_cast<int>(frag % fpb);
    const int h = lane >> 5, i = lane & 31;
    const int kk = bf ? 16 * sub + 8 * (el >> 2) + 4 * h + (el & 3) : acc_row(4 * sub + el, h);
    int row, col;
    int64_t dst_e = e;
    if (!bwd) {  // W: A[i][k] = W[32nb + i][col(kb, k)]
        // fp32: chunk kb, row block nb (chunk-major); 16-bit: row block nb, k block kb,
        // then the row block's bias fragment (row-block major, mlp_fwd_rbm.inc)
        const int kb = static_cast<int>(bf ? blk % a.KB[l] : blk / a.NB[l]);
        const int nb = static_cast<int>(bf ? blk / a.KB[l] : blk % a.NB[l]);
        row = 32 * nb + i;
        col = pack_col(a, l, kb, kk);
        if (bf) dst_e = ((static_cast<int64_t>(nb) * (2 * a.KB[l] + 1) + 2 * kb + sub) * 64 + lane) * epl + el;
    } else {  // W^T: A[i][k] = W[32ob + k][col(ib, i)], chunk ob, row block ib
        const int ob = static_cast<int>(blk / a.KB[l]);
        const int ib = static_cast<int>((blk % a.KB[l] + a.bwd_rot[l]) % a.KB[l]);
        row = 32 * ob + kk;
        col = pack_col(a, l, ib, i);
    }
    if constexpr (IDX) {
        if (col >= 0)
            put_dst(t, bwd ? 1 : 0, a.w_off[l] + static_cast<int64_t>(row) * a.in[l] + col,
                    (bwd ? a.pkb[l] : a.pk[l]) + dst_e * (bf ? 2 : 4), bf ? dst16(a.prec) : kDstF32);
        return;
    }
    const float v = col >= 0 ? a.params[a.w_off[l] + static_cast<int64_t>(row) * a.in[l] + col] : 0.f;
    char* dst = a.packed + (bwd ? a.pkb[l] : a.pk[l]);
    if (bf)
        reinterpret_cast<unsigned short*>(dst)[dst_e] =
            a.prec == NR_PREC_FP16 ? __builtin_bit_cast(unsigned short, static_cast<_Float16>(v)) : bf16_bits(v);
    else
        reinterpret_cast<float*>(dst)[dst_e] = v;
}

// 16-bit dX-chain images (pk_bwdr): for layers l >= 1, A[i][k] = W[32 ob + k][hcol0 +
// 32 ib + i] with ib the hidden input block (row block), ob the output block (k
// block), row-block major: e = ((ib * NB + ob) * 2 + frag) * 512 + lane * 8 + el.
struct PackBwdrArgs {
    const float* params;
    char* packed;
    int prec;
    int l0, n_lin;                         // layers l0 .. n_lin-1
    int64_t w_off[kMaxMfmaLayers], pk[kMaxMfmaLayers];
    int in[kMaxMfmaLayers], NB[kMaxMfmaLayers], out[kMaxMfmaLayers], hcol0[kMaxMfmaLayers];
    int64_t cum[kMaxMfmaLayers + 1];       // element prefix over layers l0..
};

template <bool IDX>
__global__ void mlp_pack_bwdr_kernel(PackBwdrArgs a, PackIdx t) {
    const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g >= a.cum[a.n_lin]) return;
    int l = a.l0;
    while (g >= a.cum[l + 1]) ++l;
    const int64_t e = g - a.cum[l];
    const int el = static_cast<int>(e % 8), lane = static_cast<int>((e / 8) % 64);
    const int64_t frag = e / 512;
    const int sub = static_cast<int>(frag % 2);
    const int64_t blk = frag / 2;
    const int ob = static_cast<int>(blk % a.NB[l]), ib = static_cast<int>(blk / a.NB[l]);
    const int h = lane >> 5, i = lane & 31;
    const int kk = 16 * sub + 8 * (el >> 2) + 4 * h + (el & 3);
    const int row = 32 * ob + kk, col = a.hcol0[l] + 32 * ib + i;
    if constexpr (IDX) {
        if (row < a.out[l]) put_dst(t, 2, a.w_off[l] + static_cast<int64_t>(row) * a.in[l] + col, a.pk[l] + 2 * e, dst16(a.prec));
        return;
    }
    const float v = row < a.out[l] ? a.params[a.w_off[l] + static_cast<int64_t>(row) * a.in[l] + col] : 0.f;
    unsigned short* dst = reinterpret_cast<unsigned short*>(a.packed + a.pk[l]);
    dst[e] = a.prec == NR_PREC_FP16 ? __builtin_bit_cast(unsigned short, static_cast<_Float16>(v)) : bf16_bits(v);
}

// 16-bit forward images: the bias fragment that follows each row block's weights
// (bias_frag of bias[32 nb + lane] in lanes 0..31, zeros in 32..63).
struct PackBiasArgs {
    const float* params;
    char* packed;
    int prec;
    int n_lin;
    int64_t pk[kMaxMfmaLayers], b_off[kMaxMfmaLayers];
    int NB[kMaxMfmaLayers], KB[kMaxMfmaLayers], out[kMaxMfmaLayers];
};

template <int PREC, bool IDX>
__device__ void pack_bias_one(const PackBiasArgs& a, const PackIdx& t, int l, int nb, int lane) {
    const int row = 32 * nb + lane;
    if constexpr (IDX) {
        if (lane < 32 && row < a.out[l])
            put_dst(t, 0, a.b_off[l] + row,
                    a.pk[l] + (static_cast<int64_t>(nb) * (2 * a.KB[l] + 1) + 2 * a.KB[l]) * kFragBytes + 16 * lane,
                    PREC == NR_PREC_FP16 ? kDstFragF16 : kDstFragBf16);
        return;
    }
    const float b = (lane < 32 && row < a.out[l]) ? a.params[a.b_off[l] + row] : 0.f;
    const bf16x8 f = bias_frag<PREC>(b);
    char* dst = a.packed + a.pk[l] + (static_cast<int64_t>(nb) * (2 * a.KB[l] + 1) + 2 * a.KB[l]) * kFragBytes;
    reinterpret_cast<bf16x8*>(dst)[lane] = lane < 32 ? f : bf16x8{};
}

template <bool IDX>
__global__ void mlp_pack_bias_kernel(PackBiasArgs a, PackIdx t) {
    const int l = blockIdx.x / kMaxTrunk, nb = blockIdx.x % kMaxTrunk, lane = threadIdx.x;
    if (l >= a.n_lin || nb >= a.NB[l]) return;
    if (a.prec == NR_PREC_FP16)
        pack_bias_one<NR_PREC_FP16, IDX>(a, t, l, nb, lane);
    else
        pack_bias_one<NR_PREC_BF16, IDX>(a, t, l, nb, lane);
}

// Vector images: element idx of a vector of NB blocks <-> feature 32*(idx>>5) + acc_row(idx&15, (idx>>4)&1).
struct PackVecArgs {
    const float* params;
    char* packed;
    int nv;                                   // vectors: n_lin biases, w_sigma, 3 rows of W_rgb
    int64_t src[kMaxMfmaLayers + 8];          // float offset in params
    int len[kMaxMfmaLayers + 8];              // valid features
    int64_t dst[kMaxMfmaLayers + 8];          // byte offset in packed
    int cum[kMaxMfmaLayers + 9];              // image elements (NB*32) prefix
    int pair[kMaxMfmaLayers + 8];             // 1: pair image (PImg), 0: vector image (VImg)
    int slot[kMaxMfmaLayers + 8];             // destination-table slot (IDX mode)
};

template <bool IDX>
__global__ void mlp_pack_vec_kernel(PackVecArgs a, PackIdx t) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.cum[a.nv]) return;
    int v = 0;
    while (g >= a.cum[v + 1]) ++v;
    const int idx = g - a.cum[v];
    const int f = a.pair[v] ? 32 * (idx >> 5) + acc_row((idx >> 1) & 15, idx & 1)
                            : 32 * (idx >> 5) + acc_row(idx & 15, (idx >> 4) & 1);
    if constexpr (IDX) {
        if (f < a.len[v]) put_dst(t, a.slot[v], a.src[v] + f, a.dst[v] + 4 * static_cast<int64_t>(idx), kDstF32);
        return;
    }
    reinterpret_cast<float*>(a.packed + a.dst[v])[idx] = f < a.len[v] ? a.params[a.src[v] + f] : 0.f;
}

// ------------------------------------------------- fused optimizer step ----
// Adam over up to kMaxAdamSpans flat buffers (blockIdx.y = span), the clip
// coefficient from the span's clip-group partials (nr_sumsq_partials, summed in the
// fixed block order by every block), and the packed images refreshed through the
// span's destination table: nr_mlp_pack's four kernels are not run after the step.
struct AdamSpanDev {
    float *p, *g, *m, *v;
    int64_t n;
    const float* partials;
    float max_norm;
    const uint32_t* table;
    char* packed;
};
struct AdamMultiArgs {
    AdamSpanDev s[kMaxAdamSpans];
    float omb1, b2, omb2, eps, step_size, bc2_sqrt;
    const float* sched;  // nullable: {step_size, bc2_sqrt} read on the device (graph replay)
};

__device__ __forceinline__ void put_image(char* packed, uint32_t e, float p) {
    char* q = packed + (e & 0x1fffffffu);
    switch (e >> 29) {
        case kDstF32: *reinterpret_cast<float*>(q) = p; break;
        case kDstBf16: *reinterpret_cast<unsigned short*>(q) = bf16_bits(p); break;
        case kDstF16: *reinterpret_cast<unsigned short*>(q) = __builtin_bit_cast(unsigned short, static_cast<_Float16>(p)); break;
        case kDstFragBf16: *reinterpret_cast<bf16x8*>(q) = bias_frag<NR_PREC_BF16>(p); break;
        case kDstFragF16: *reinterpret_cast<bf16x8*>(q) = bias_frag<NR_PREC_FP16>(p); break;
        default: break;
    }
}

__global__ void __launch_bounds__(kSumsqThreads) adam_multi_kernel(AdamMultiArgs a) {
    const AdamSpanDev& s = a.s[blockIdx.y];
    const float step_size = a.sched ? a.sched[0] : a.step_size, bc2_sqrt = a.sched ? a.sched[1] : a.bc2_sqrt;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    const int64_t t0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t n = s.n;
    // 16-B accesses when every buffer (and the table's slot rows) allows them
    const int64_t n4 = (n % 4 == 0) ? n / 4 : 0;
    float4 P, G, M, V;
    u32x4 E[kPackSlots];
    auto load = [&](int64_t i) {
        P = reinterpret_cast<const float4*>(s.p)[i];
        G = reinterpret_cast<const float4*>(s.g)[i];
        M = reinterpret_cast<const float4*>(s.m)[i];
        V = reinterpret_cast<const float4*>(s.v)[i];
        if (s.table)
#pragma unroll
            for (int sl = 0; sl < kPackSlots; ++sl) E[sl] = reinterpret_cast<const u32x4*>(s.table + sl * n)[i];
    };
    // the first element's loads go out before the clip coefficient's 256 partials are
    // summed (per wave, no barrier: the grid is one element per thread at NeRF sizes)
    if (t0 < n4) load(t0);
    const float coef = s.partials ? clip_coef(wave_sum_fixed(s.partials), s.max_norm) : 1.0f;
    for (int64_t i = t0; i < n4; i += stride) {
        if (i != t0) load(i);
        adam_one(P.x, G.x, M.x, V.x, coef, a.omb1, a.b2, a.omb2, step_size, bc2_sqrt, a.eps);
        adam_one(P.y, G.y, M.y, V.y, coef, a.omb1, a.b2, a.omb2, step_size, bc2_sqrt, a.eps);
        adam_one(P.z, G.z, M.z, V.z, coef, a.omb1, a.b2, a.omb2, step_size, bc2_sqrt, a.eps);
        adam_one(P.w, G.w, M.w, V.w, coef, a.omb1, a.b2, a.omb2, step_size, bc2_sqrt, a.eps);
        reinterpret_cast<float4*>(s.p)[i] = P;
        reinterpret_cast<float4*>(s.g)[i] = G;
        reinterpret_cast<float4*>(s.m)[i] = M;
        reinterpret_cast<float4*>(s.v)[i] = V;
        if (s.table) {
#pragma unroll
            for (int sl = 0; sl < kPackSlots; ++sl) {
                put_image(s.packed, E[sl].x, P.x);
                put_image(s.packed, E[sl].y, P.y);
                put_image(s.packed, E[sl].z, P.z);
                put_image(s.packed, E[sl].w, P.w);
            }
        }
    }
    for (int64_t i = 4 * n4 + t0; i < n; i += stride) {
        float P1 = s.p[i], G1 = s.g[i], M1 = s.m[i], V1 = s.v[i];
        adam_one(P1, G1, M1, V1, coef, a.omb1, a.b2, a.omb2, step_size, bc2_sqrt, a.eps);
        s.p[i] = P1;
        s.g[i] = G1;
        s.m[i] = M1;
        s.v[i] = V1;
        if (s.table)
#pragma unroll
            for (int sl = 0; sl < kPackSlots; ++sl) put_image(s.packed, s.table[sl * n + i], P1);
    }
}

}  // namespace nr

using namespace nr;

namespace {

bool plan_or_error(const NrMlpConfig* cfg, MlpPlan* p) {
    const char* why = "";
    if (!make_plan(cfg, p, &why)) {
        set_error("NrMlpConfig unsupported: %s", why);
        return false;
    }
    return true;
}

// Workgroup shape of the bf16 forward / backward kernels: NT threads, one
// 32-sample tile per wave, all waves sharing one LDS weight stream.  256 = 4
// waves with the full 512-register budget (1 wave per SIMD); 512 = 8 waves at
// 256 registers (2 waves per SIMD).  Measured on MI355X at M = 786,432 (r01):
// forward (training) 3.25 ms at 256 vs 4.09 ms at 512 (the 512 build spills);
// backward dX 2.12 ms at 256 vs 1.70 ms at 512.
#ifndef NR_FWD_NT
#define NR_FWD_NT 512
#endif
#ifndef NR_BWD_NT
#define NR_BWD_NT 512
#endif
#ifndef NR_FWD_TPW
#define NR_FWD_TPW 1
#endif

void add_stream_layer(StreamDesc& sd, int nchunks, int chunk_kb, int load_kb = -1) {
    for (int c = 0; c < nchunks && sd.nq < kMaxChunks; ++c) {
        sd.ckb[sd.nq] = load_kb < 0 ? chunk_kb : load_kb;
        sd.cadv[sd.nq++] = chunk_kb;
    }
}

int max_chunk(const StreamDesc& sd) {
    int m = 0;
    for (int q = 0; q < sd.nq; ++q) m = sd.ckb[q] * 1024 > m ? sd.ckb[q] * 1024 : m;
    return m;
}

template <int PREC, bool TRAIN>
int launch_fwd(const MlpPlan& p, FwdArgs& a, hipStream_t s) {
    constexpr int TPW = NR_FWD_TPW, NT = k16<PREC> ? NR_FWD_NT : 256;
    constexpr int G = (k16<PREC> ? 16384 : 32768) / (NT * 16);  // one 16 / 32 KB chunk
    const int mc = max_chunk(a.sd);
    if (mc > G * NT * 16) {
        set_error("nr_mlp_forward: chunk of %d bytes exceeds the stager", mc);
        return NR_EARG;
    }
    a.slot_bytes = mc;
    constexpr bool ACT_LDS = k16<PREC> && (NT == 512 || TPW >= 2);
    const size_t lds = 2 * static_cast<size_t>(mc) + (ACT_LDS ? (NT / 64) * TPW * kHB * 2 * kFragBytes : 0);
    if (lds > 160 * 1024) {
        set_error("nr_mlp_forward: %zu bytes of LDS exceed 160 KiB", lds);
        return NR_EARG;
    }
    const dim3 grid(static_cast<unsigned>(ceil_div_ll(a.tiles, (NT / 64) * TPW))), block(NT);
#define NR_FWD(XB_, DB_)                                                                                 \
    if (p.XB == XB_ && p.DB == DB_) {                                                                    \
        hipLaunchKernelGGL((mlp_fwd_kernel<PREC, XB_, DB_, TRAIN, TPW, G, NT>), grid, block, lds, s, a); \
        return check_launch("nr_mlp_forward");                                                           \
    }
    NR_FWD(2, 1)
#ifndef NR_MLP_DEV  // dev builds (register/ISA inspection) compile the default model only
    NR_FWD(2, 0)
    NR_FWD(1, 1)
    NR_FWD(1, 0)
#endif
#undef NR_FWD
    set_error("nr_mlp_forward: no kernel instance for XB=%d DB=%d", p.XB, p.DB);
    return NR_EARG;
}

template <int PREC, bool TRAIN>
int launch_fwd_rbm(const MlpPlan& p, const RbmArgs& a, hipStream_t s) {
    // every chunk fits a slot (checked at compile time per layer shape).  Eight waves per
    // workgroup at every size: four- and six-wave workgroups for small launches (all CUs
    // busy, or even rounds) were faster in isolation at 1,024 tiles but slower inside the
    // graph-replayed 512-ray step, where the coarse backward shares the chip
    // (profiles/r06_rbm_waves.txt; r04 found the same)
    constexpr int W = kRbmWaves;
    const dim3 grid(static_cast<unsigned>(ceil_div_ll(a.tiles, W))), block(W * 64);
    const size_t lds = rbm_lds_bytes(p.XB, W);
#define NR_FWDR(XB_, DB_)                                                                           \
    if (p.XB == XB_ && p.DB == DB_) {                                                               \
        hipLaunchKernelGGL((mlp_fwd_rbm_kernel<PREC, XB_, DB_, TRAIN, W>), grid, block, lds, s, a); \
        return check_launch("nr_mlp_forward");                                                      \
    }
    NR_FWDR(2, 1)
#ifndef NR_MLP_DEV
    NR_FWDR(2, 0)
    NR_FWDR(1, 1)
    NR_FWDR(1, 0)
#endif
#undef NR_FWDR
    set_error("nr_mlp_forward: no kernel instance for XB=%d DB=%d", p.XB, p.DB);
    return NR_EARG;
}

template <int PREC>
int launch_bwd_rbm(const MlpPlan& p, const BwdrArgs& a, hipStream_t s) {
    constexpr int W = kRbmWaves;
    const size_t lds = bwdr_lds_bytes(p.n_mask, W);
    if (lds > 160 * 1024) {
        set_error("nr_mlp_backward_dx: %zu bytes of LDS exceed 160 KiB", lds);
        return NR_EARG;
    }
    // every part of every segment (mlp_bwd_rbm_kernel's workgroup mapping)
    const dim3 grid(static_cast<unsigned>(a.nseg * (kSegTiles / W))), block(W * 64);
    hipLaunchKernelGGL((mlp_bwd_rbm_kernel<PREC, W>), grid, block, lds, s, a);
    return check_launch("nr_mlp_backward_dx");
}

template <int PREC, bool WX>
int launch_bwd(const MlpPlan& p, BwdArgs& a, hipStream_t s) {
    // the input-gradient variant also carries d x_enc through the trunk: 4 waves, 512 registers
    constexpr int TPW = 1, NT = (WX || !k16<PREC>) ? 256 : NR_BWD_NT;
    // one chunk of the skip layer's W^T: (XB + 8) blocks, at most 20 / 40 KB
    constexpr int G = ((k16<PREC> ? 20480 : 40960) + NT * 16 - 1) / (NT * 16);
    const int mc = max_chunk(a.sd);
    if (mc > G * NT * 16) {
        set_error("nr_mlp_backward_dx: chunk of %d bytes exceeds the stager", mc);
        return NR_EARG;
    }
    a.slot_bytes = mc;
    constexpr bool ACT_LDS = k16<PREC> && NT == 512;
    const size_t lds = 2 * static_cast<size_t>(mc) + (ACT_LDS ? (NT / 64) * TPW * kHB * 2 * kFragBytes : 0);
    if (lds > 160 * 1024) {
        set_error("nr_mlp_backward_dx: %zu bytes of LDS exceed 160 KiB", lds);
        return NR_EARG;
    }
    // every part of every segment (mlp_bwd_kernel's workgroup mapping)
    const dim3 grid(static_cast<unsigned>(a.nseg * (kSegTiles / (NT / 64)))), block(NT);
#define NR_BWD(XB_, DB_)                                                                              \
    if (p.XB == XB_ && p.DB == DB_) {                                                                 \
        hipLaunchKernelGGL((mlp_bwd_kernel<PREC, XB_, DB_, TPW, G, NT, WX>), grid, block, lds, s, a); \
        return check_launch("nr_mlp_backward_dx");                                                    \
    }
    NR_BWD(2, 1)
#ifndef NR_MLP_DEV  // dev builds (register/ISA inspection) compile the default model only
    NR_BWD(2, 0)
    NR_BWD(1, 1)
    NR_BWD(1, 0)
#endif
#undef NR_BWD
    set_error("nr_mlp_backward_dx: no kernel instance for XB=%d DB=%d", p.XB, p.DB);
    return NR_EARG;
}

template <int PREC>
int launch_dinput(const MlpPlan& p, const DinArgs& a, hipStream_t s) {
    const size_t lds = static_cast<size_t>(din_frags(a.nsrc, p.XB, p.DB, a.nc)) * kFragBytes;
    const bool alds = lds <= 160 * 1024;
    // enough workgroups for 2 per CU (the staging is amortised over ~6 tiles per wave)
    const dim3 grid(static_cast<unsigned>(std::min<int64_t>(ceil_div_ll(a.tiles, kDinNT / 64), 512))),
        block(kDinNT);
#define NR_DIN(XB_, DB_)                                                                                  \
    if (p.XB == XB_ && p.DB == DB_) {                                                                     \
        if (alds)                                                                                         \
            hipLaunchKernelGGL((mlp_dinput_kernel<PREC, XB_, DB_, true>), grid, block, lds, s, a);        \
        else                                                                                              \
            hipLaunchKernelGGL((mlp_dinput_kernel<PREC, XB_, DB_, false>), grid, block, 0, s, a);         \
        return check_launch("nr_mlp_backward_dx (input gradients)");                                     \
    }
    NR_DIN(2, 1)
#ifndef NR_MLP_DEV
    NR_DIN(2, 0)
    NR_DIN(1, 1)
    NR_DIN(1, 0)
#endif
#undef NR_DIN
    set_error("nr_mlp_backward_dx: no input-gradient kernel for XB=%d DB=%d", p.XB, p.DB);
    return NR_EARG;
}

// 16-bit g_x / g_d: one MFMA pass over the stored dz images of the x_enc-reading
// layers and of dz_c (mlp_dinput_kernel), after either backward form wrote them
int input_grads16(const MlpPlan& p, const MlpSizes& z, const char* packed, const float* x, const float* d, float* g_x,
                  float* g_d, const char* ws, int64_t M, hipStream_t s) {
    const int n = p.n_layers;
    DinArgs da;
    std::memset(&da, 0, sizeof(da));
    da.packed = packed;
    da.ws = ws;
    da.flags = reinterpret_cast<const uint8_t*>(ws + z.flags_off);
    da.x = x;
    da.d = d;
    da.g_x = g_x;
    da.g_d = g_d;
    da.M = M;
    da.tiles = z.tiles;
    da.L = p.L;
    da.Ld = p.Ld;
    da.inv_gscale = 1.0f / grad_scale(p.prec);
    // layer 0 reads x_enc alone; a skip layer's W^T chunk is [h (8) | x_enc (XB)]
    for (int l = 0; l < n; ++l) {
        if (l > 0 && !is_skip(p, l - 1)) continue;
        da.a_off[da.nsrc] = p.lin[l].pk_bwd;
        da.a_kb[da.nsrc] = p.lin[l].KB;
        da.a_p0[da.nsrc] = p.lin[l].KB - p.XB;
        da.dz_off[da.nsrc] = z.ws_off[WS_DZ0 + l];
        da.nsrc++;
    }
    // dir's W^T chunk is [feat (8) | d_enc (DB)], one chunk per dz_c block
    da.dir_a_off = p.lin[n + 1].pk_bwd;
    da.dir_kb = p.lin[n + 1].KB;
    da.dir_p0 = kHB;
    da.nc = p.lin[n + 1].NB;
    da.dz_dir_off = z.ws_off[p.ws_dir];
    return p.prec == NR_PREC_BF16 ? launch_dinput<NR_PREC_BF16>(p, da, s) : launch_dinput<NR_PREC_FP16>(p, da, s);
}


}  // namespace

namespace {

// nr_mlp_pack's four kernels; IDX: their index mode, filling the destination table
template <bool IDX>
int launch_pack(const MlpPlan& p, const float* params, void* packed, PackIdx t, hipStream_t s) {
    const char* what = IDX ? "nr_mlp_pack_table" : "nr_mlp_pack";
    PackArgs a;
    std::memset(&a, 0, sizeof(a));
    a.params = params;
    a.packed = static_cast<char*>(packed);
    a.n_lin = p.n_lin;
    a.prec = p.prec;
    a.cum[0] = 0;
    for (int l = 0; l < p.n_lin; ++l) {
        const LinearDesc& d = p.lin[l];
        a.w_off[l] = d.w_off;
        a.in[l] = d.in;
        a.NB[l] = d.NB;
        a.KB[l] = d.KB;
        a.nseg[l] = d.nseg;
        for (int s = 0; s < d.nseg; ++s) {
            a.seg_col0[l][s] = d.seg[s].col0;
            a.seg_w[l][s] = d.seg[s].width;
            a.seg_blk[l][s] = d.seg[s].blocks;
        }
        a.pk[l] = d.pk_fwd;
        a.pkb[l] = d.pk_bwd;
        a.bwd_rot[l] = (l > 0 && l < p.n_layers && is_skip(p, l - 1)) ? d.seg[0].blocks : 0;
        const int64_t elems = static_cast<int64_t>(d.NB) * d.KB * 1024;  // 32x32 elements per block
        a.cum[l + 1] = a.cum[l] + 2 * elems;
    }
    const int64_t total = a.cum[p.n_lin];
    hipLaunchKernelGGL(mlp_pack_kernel<IDX>, dim3(static_cast<unsigned>(ceil_div_ll(total, 256))), dim3(256), 0, s, a, t);
    NR_LAUNCH_CHECK(what);
    if (p.prec != NR_PREC_FP32) {
        PackBiasArgs pb;
        std::memset(&pb, 0, sizeof(pb));
        pb.params = params;
        pb.packed = static_cast<char*>(packed);
        pb.prec = p.prec;
        pb.n_lin = p.n_lin;
        for (int l = 0; l < p.n_lin; ++l) {
            pb.pk[l] = p.lin[l].pk_fwd;
            pb.b_off[l] = p.lin[l].b_off;
            pb.NB[l] = p.lin[l].NB;
            pb.KB[l] = p.lin[l].KB;
            pb.out[l] = p.lin[l].out;
        }
        hipLaunchKernelGGL(mlp_pack_bias_kernel<IDX>, dim3(p.n_lin * kMaxTrunk), dim3(64), 0, s, pb, t);
        NR_LAUNCH_CHECK(what);
        if (p.n_lin > 1) {
            PackBwdrArgs pr;
            std::memset(&pr, 0, sizeof(pr));
            pr.params = params;
            pr.packed = static_cast<char*>(packed);
            pr.prec = p.prec;
            pr.l0 = 1;
            pr.n_lin = p.n_lin;
            pr.cum[1] = 0;
            for (int l = 1; l < p.n_lin; ++l) {
                const LinearDesc& d = p.lin[l];
                pr.w_off[l] = d.w_off;
                pr.pk[l] = d.pk_bwdr;
                pr.in[l] = d.in;
                pr.NB[l] = d.NB;
                pr.out[l] = d.out;
                // the hidden input columns: after x_enc in a skip layer (cat([x_enc, h])), first otherwise
                pr.hcol0[l] = (l < p.n_layers && is_skip(p, l - 1)) ? p.pos_dim : 0;
                pr.cum[l + 1] = pr.cum[l] + static_cast<int64_t>(kHB) * d.NB * 1024;
            }
            const int64_t tot = pr.cum[p.n_lin];
            hipLaunchKernelGGL(mlp_pack_bwdr_kernel<IDX>, dim3(static_cast<unsigned>(ceil_div_ll(tot, 256))), dim3(256),
                               0, s, pr, t);
            NR_LAUNCH_CHECK(what);
        }
    }
    PackVecArgs v;
    std::memset(&v, 0, sizeof(v));
    v.params = params;
    v.packed = static_cast<char*>(packed);
    auto add_vec = [&](int64_t src, int len, int64_t dst, int nblk, int pair, int slot) {
        v.pair[v.nv] = pair;
        v.slot[v.nv] = slot;
        v.src[v.nv] = src;
        v.len[v.nv] = len;
        v.dst[v.nv] = dst;
        v.cum[v.nv + 1] = v.cum[v.nv] + nblk * 32;
        v.nv++;
    };
    // table slots: biases 1 (slot 0 holds their 16-bit fragment), the head weights'
    // pair images 0 and their vector images 1
    for (int l = 0; l < p.n_lin; ++l) add_vec(p.lin[l].b_off, p.lin[l].out, p.lin[l].vb, p.lin[l].NB, 0, 1);
    add_vec(p.sig_w, kHidden, p.vsig, kHB, 1, 0);
    for (int c = 0; c < 3; ++c)
        add_vec(p.rgb_w + c * (kHidden / 2), kHidden / 2, p.vrgb + c * (kHidden / 2) * 4, kHB / 2, 1, 0);
    add_vec(p.sig_w, kHidden, p.vhead, kHB, 0, 1);
    for (int c = 0; c < 3; ++c)
        add_vec(p.rgb_w + c * (kHidden / 2), kHidden / 2, p.vhead + 1024 + c * (kHidden / 2) * 4, kHB / 2, 0, 1);
    hipLaunchKernelGGL(mlp_pack_vec_kernel<IDX>, dim3(ceil_div(v.cum[v.nv], 256)), dim3(256), 0, s, v, t);
    NR_LAUNCH_CHECK(what);
    return NR_OK;
}

}  // namespace

extern "C" {

int64_t nr_mlp_param_count(const NrMlpConfig* cfg) {
    MlpPlan p;
    return plan_or_error(cfg, &p) ? p.param_count : -1;
}

int64_t nr_mlp_packed_bytes(const NrMlpConfig* cfg) {
    MlpPlan p;
    return plan_or_error(cfg, &p) ? p.packed_bytes : -1;
}

int64_t nr_mlp_saved_bytes(const NrMlpConfig* cfg, int64_t M) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p) || M < 0) return -1;
    return make_sizes(p, M).saved_bytes;
}

int64_t nr_mlp_workspace_bytes(const NrMlpConfig* cfg, int64_t M) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p) || M < 0) return -1;
    return make_sizes(p, M).ws_bytes;
}

int nr_mlp_pack(const NrMlpConfig* cfg, const float* params, void* packed, nr_stream_t stream) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p)) return NR_EARG;
    NR_REQUIRE(params && packed, "nr_mlp_pack: null pointer");
    NR_REQUIRE((reinterpret_cast<uintptr_t>(packed) & 15) == 0, "nr_mlp_pack: packed must be 16-byte aligned");
    return launch_pack<false>(p, params, packed, PackIdx{nullptr, 0}, static_cast<hipStream_t>(stream));
}

int64_t nr_mlp_pack_table_bytes(const NrMlpConfig* cfg) {
    MlpPlan p;
    return plan_or_error(cfg, &p) ? static_cast<int64_t>(kPackSlots) * p.param_count * 4 : -1;
}

int nr_mlp_pack_table(const NrMlpConfig* cfg, uint32_t* table, nr_stream_t stream) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p)) return NR_EARG;
    NR_REQUIRE(table, "nr_mlp_pack_table: null pointer");
    NR_REQUIRE((reinterpret_cast<uintptr_t>(table) & 15) == 0, "nr_mlp_pack_table: table must be 16-byte aligned");
    NR_REQUIRE(p.packed_bytes < kDstMaxOff, "nr_mlp_pack_table: packed images beyond 512 MB");
    const hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = hipMemsetAsync(table, 0, static_cast<size_t>(kPackSlots) * p.param_count * 4, s);
    if (e != hipSuccess) {
        set_error("nr_mlp_pack_table: %s", hipGetErrorString(e));
        return static_cast<int>(e);
    }
    return launch_pack<true>(p, nullptr, nullptr, PackIdx{table, p.param_count}, s);
}

int nr_adam_multi(const NrAdamSpan* spans, int nspan, double lr, double b1, double b2, double eps, int64_t step,
                  const float* sched, nr_stream_t stream) {
    NR_REQUIRE(spans && nspan >= 1 && nspan <= kMaxAdamSpans && step >= 1,
               "nr_adam_multi: bad arguments (1..%d spans, step >= 1)", kMaxAdamSpans);
    AdamMultiArgs a;
    std::memset(&a, 0, sizeof(a));
    int64_t nmax = 0;
    for (int k = 0; k < nspan; ++k) {
        const NrAdamSpan& x = spans[k];
        NR_REQUIRE(x.params && x.grads && x.exp_avg && x.exp_avg_sq && x.n >= 0, "nr_adam_multi: span %d: null buffer", k);
        NR_REQUIRE(((reinterpret_cast<uintptr_t>(x.params) | reinterpret_cast<uintptr_t>(x.grads) |
                     reinterpret_cast<uintptr_t>(x.exp_avg) | reinterpret_cast<uintptr_t>(x.exp_avg_sq) |
                     reinterpret_cast<uintptr_t>(x.pack_table)) & 15) == 0,
                   "nr_adam_multi: span %d: buffers must be 16-byte aligned", k);
        NR_REQUIRE(!x.pack_table || x.packed, "nr_adam_multi: span %d: pack_table without packed", k);
        a.s[k] = AdamSpanDev{x.params, x.grads, x.exp_avg, x.exp_avg_sq, x.n, x.sumsq_partials, x.max_norm,
                             x.pack_table, static_cast<char*>(x.packed)};
        nmax = x.n > nmax ? x.n : nmax;
    }
    if (nmax == 0) return NR_OK;
    // bias corrections in double on the host, as torch's _single/_multi_tensor_adam do
    const double bc1 = 1.0 - std::pow(b1, static_cast<double>(step));
    const double bc2 = 1.0 - std::pow(b2, static_cast<double>(step));
    a.omb1 = static_cast<float>(1.0 - b1);
    a.b2 = static_cast<float>(b2);
    a.omb2 = static_cast<float>(1.0 - b2);
    a.eps = static_cast<float>(eps);
    a.step_size = static_cast<float>(lr / bc1);
    a.bc2_sqrt = static_cast<float>(std::sqrt(bc2));
    a.sched = sched;
    const int grid = stream_grid(ceil_div_ll(nmax, 4), kSumsqThreads);
    hipLaunchKernelGGL(adam_multi_kernel, dim3(grid, nspan), dim3(kSumsqThreads), 0, static_cast<hipStream_t>(stream), a);
    NR_LAUNCH_CHECK("nr_adam_multi");
    return NR_OK;
}

int nr_mlp_forward(const NrMlpConfig* cfg, const void* packed, const float* params, const float* x, const float* d,
                   int64_t M, float* rgb, float* sigma, void* saved, nr_stream_t stream) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p)) return NR_EARG;
    NR_REQUIRE(packed && params && x && rgb && sigma && M >= 0, "nr_mlp_forward: null pointer");
    NR_REQUIRE(!p.use_vd || d, "nr_mlp_forward: use_view_dirs needs d (model.py:187-191)");
    NR_REQUIRE((reinterpret_cast<uintptr_t>(saved) & 15) == 0, "nr_mlp_forward: saved must be 16-byte aligned");
    NR_REQUIRE((reinterpret_cast<uintptr_t>(packed) & 15) == 0, "nr_mlp_forward: packed must be 16-byte aligned");
    if (M == 0) return NR_OK;
    const MlpSizes z = make_sizes(p, M);
    FwdArgs a;
    std::memset(&a, 0, sizeof(a));
    a.packed = static_cast<const char*>(packed);
    a.params = params;
    a.x = x;
    a.d = d;
    a.rgb = rgb;
    a.sigma = sigma;
    a.saved = static_cast<char*>(saved);
    a.M = M;
    a.tiles = z.tiles;
    a.L = p.L;
    a.Ld = p.Ld;
    a.n_layers = p.n_layers;
    a.skips = p.skips;
    a.sd.base = p.lin[0].pk_fwd;
    for (int l = 0; l < p.n_lin; ++l) {
        const LinearDesc& dl = p.lin[l];
        add_stream_layer(a.sd, dl.KB, dl.NB * p.fpb);
        a.vb[l] = dl.vb;
        a.bo[l] = dl.b_off;
    }
    a.vsig = p.vsig;
    a.vrgb = p.vrgb;
    a.sig_b = p.sig_b;
    a.rgb_b = p.rgb_b;
    for (int t = 0; t < p.n_saved; ++t) a.sv_off[t] = z.saved_off[t];
    a.sv_feat = p.sv_feat;
    a.sv_denc = p.sv_denc;
    a.sv_hc = p.sv_hc;
    a.mask_off = z.mask_off;
    a.n_mask = p.n_mask;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    if (p.prec != NR_PREC_FP32) {
        RbmArgs r;
        std::memset(&r, 0, sizeof(r));
        r.packed = a.packed;
        r.params = params;
        r.x = x;
        r.d = d;
        r.rgb = rgb;
        r.sigma = sigma;
        r.saved = a.saved;
        r.M = M;
        r.tiles = z.tiles;
        r.L = p.L;
        r.Ld = p.Ld;
        r.n_layers = p.n_layers;
        r.skips = p.skips;
        r.base = p.lin[0].pk_fwd;
        r.vhead = p.vhead;
        r.sig_b = p.sig_b;
        r.rgb_b = p.rgb_b;
        for (int t = 0; t < p.n_saved; ++t) r.sv_off[t] = z.saved_off[t];
        r.sv_feat = p.sv_feat;
        r.sv_denc = p.sv_denc;
        r.sv_hc = p.sv_hc;
        r.mask_off = z.mask_off;
        r.n_mask = p.n_mask;
        if (p.prec == NR_PREC_BF16)
            return saved ? launch_fwd_rbm<NR_PREC_BF16, true>(p, r, s) : launch_fwd_rbm<NR_PREC_BF16, false>(p, r, s);
        return saved ? launch_fwd_rbm<NR_PREC_FP16, true>(p, r, s) : launch_fwd_rbm<NR_PREC_FP16, false>(p, r, s);
    }
    return saved ? launch_fwd<NR_PREC_FP32, true>(p, a, s) : launch_fwd<NR_PREC_FP32, false>(p, a, s);
}

int nr_mlp_backward_dx(const NrMlpConfig* cfg, const void* packed, const float* params, const float* x,
                       const float* d, int64_t M, const float* rgb, const float* sigma, const void* saved,
                       const float* g_rgb, const float* g_sigma, float* g_x, float* g_d, void* workspace,
                       nr_stream_t stream) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p)) return NR_EARG;
    NR_REQUIRE(packed && params && x && rgb && sigma && saved && g_rgb && g_sigma && workspace && M >= 0,
               "nr_mlp_backward_dx: null pointer");
    NR_REQUIRE(!g_d || (d && p.use_vd), "nr_mlp_backward_dx: g_d needs d and use_view_dirs");
    NR_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0,
               "nr_mlp_backward_dx: workspace must be 16-byte aligned");
    if (M == 0) return NR_OK;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const MlpSizes z = make_sizes(p, M);
    NR_REQUIRE(z.tiles_alloc < (int64_t{1} << 32), "nr_mlp_backward_dx: M beyond 2^37 samples");
    // the active tiles' flags (every tile with cfg->dense_backward); the dX launch
    // concatenates each segment's into the dW kernel's list (place_segment)
    char* wsb = static_cast<char*>(workspace);
    uint8_t* tflags = reinterpret_cast<uint8_t*>(wsb + z.flags_off);
    uint32_t* blkcnt = reinterpret_cast<uint32_t*>(wsb + z.blkcnt_off);
    uint32_t* dwlist = reinterpret_cast<uint32_t*>(wsb + z.dwlist_off);
    uint32_t* tcount = reinterpret_cast<uint32_t*>(wsb + z.count_off);
    hipLaunchKernelGGL(tile_flags_kernel, dim3(static_cast<unsigned>(z.nseg * (kSegTiles / 64))),
                       dim3(kTileFlagThreads), 0, s, g_rgb, g_sigma, M, p.dense_bwd, tflags, blkcnt);
    NR_LAUNCH_CHECK("nr_mlp_backward_dx (tile flags)");
    BwdArgs b;
    std::memset(&b, 0, sizeof(b));
    b.packed = static_cast<const char*>(packed);
    b.gscale = grad_scale(p.prec);
    b.inv_gscale = 1.0f / b.gscale;
    b.params = params;
    b.x = x;
    b.d = d;
    b.rgb = rgb;
    b.sigma = sigma;
    b.g_rgb = g_rgb;
    b.g_sigma = g_sigma;
    b.g_x = g_x;
    b.g_d = g_d;
    b.saved = static_cast<const char*>(saved);
    b.ws = static_cast<char*>(workspace);
    b.M = M;
    b.tiles = z.tiles;
    b.flags = tflags;
    b.blk_count = blkcnt;
    b.nseg = z.nseg;
    b.dw_list = dwlist;
    b.count = tcount;
    b.L = p.L;
    b.Ld = p.Ld;
    b.n_layers = p.n_layers;
    b.skips = p.skips;
    const int n = p.n_layers;
    // 16-bit: g_x / g_d come from a separate pass over the stored dz images
    // (mlp_dinput_kernel), so the dX chain itself always runs the 8-wave variant
    const bool want_in = g_x != nullptr || g_d != nullptr;
    const bool split_in = want_in && p.prec != NR_PREC_FP32 && !NR_DIN_FUSED;
    const bool wx = want_in && !split_in;
    // a skip layer's W^T chunk is [h rows | x_enc rows] and dir's is [feat rows |
    // d_enc rows]: without g_x / g_d only the first 8 row blocks are loaded
    auto add_T = [&](int l) {
        const bool partial = !wx && ((l > 0 && l < n && is_skip(p, l - 1)) || l == n + 1);
        add_stream_layer(b.sd, p.lin[l].NB, p.lin[l].KB * p.fpb, partial ? kHB * p.fpb : -1);
    };
    b.sd.base = p.lin[n + 1].pk_bwd;
    add_T(n + 1);  // dir^T
    add_T(n);      // feat^T
    for (int i = n - 1; i >= 1; --i) add_T(i);
    if (wx) add_T(0);
    b.vsig = p.vsig;
    b.vrgb = p.vrgb;
    b.mask_off = z.mask_off;
    b.n_mask = p.n_mask;
    for (int t = 0; t < p.n_ws; ++t) b.ws_off[t] = z.ws_off[t];
    b.ws_feat = p.ws_feat;
    b.ws_dir = p.ws_dir;
    b.ws_heads = p.ws_heads;
    // 16-bit dX chain: row-block major (mlp_bwd_rbm.inc)
    auto chain16 = [&]() -> int {
#if NR_BWD_RBM
        BwdrArgs r;
        std::memset(&r, 0, sizeof(r));
        r.gscale = b.gscale;
        r.packed = b.packed;
        r.rgb = rgb;
        r.sigma = sigma;
        r.g_rgb = g_rgb;
        r.g_sigma = g_sigma;
        r.saved = b.saved;
        r.ws = b.ws;
        r.M = M;
        r.tiles = z.tiles;
        r.flags = tflags;
        r.blk_count = blkcnt;
        r.nseg = z.nseg;
        r.dw_list = dwlist;
        r.count = tcount;
        r.scratch_base = z.tiles_alloc - kScratchTiles;
        r.n_layers = n;
        r.base = p.lin[n + 1].pk_bwdr;
        r.vrgb = p.vrgb;
        r.vhead = p.vhead;
        r.mask_off = z.mask_off;
        r.n_mask = p.n_mask;
        for (int t = 0; t < p.n_ws; ++t) r.ws_off[t] = z.ws_off[t];
        r.ws_feat = p.ws_feat;
        r.ws_dir = p.ws_dir;
        r.ws_heads = p.ws_heads;
        return p.prec == NR_PREC_BF16 ? launch_bwd_rbm<NR_PREC_BF16>(p, r, s) : launch_bwd_rbm<NR_PREC_FP16>(p, r, s);
#else
        return p.prec == NR_PREC_BF16 ? launch_bwd<NR_PREC_BF16, false>(p, b, s)
                                      : launch_bwd<NR_PREC_FP16, false>(p, b, s);
#endif
    };
    if (split_in) {
        const int rc = chain16();
        if (rc != NR_OK) return rc;
        return input_grads16(p, z, b.packed, x, d, g_x, g_d, b.ws, M, s);
    }
    if (p.prec != NR_PREC_FP32 && !wx) return chain16();
    if (!p.dense_bwd) {
        // the chain writes g_x / g_d of the active tiles only: the rest are exactly zero
        for (float* g : {g_x, g_d})
            if (g) {
                const hipError_t e = hipMemsetAsync(g, 0, sizeof(float) * 3 * static_cast<size_t>(M), s);
                if (e != hipSuccess) {
                    set_error("nr_mlp_backward_dx: %s", hipGetErrorString(e));
                    return static_cast<int>(e);
                }
            }
    }
    if (p.prec == NR_PREC_BF16) return launch_bwd<NR_PREC_BF16, true>(p, b, s);
    if (p.prec == NR_PREC_FP16) return launch_bwd<NR_PREC_FP16, true>(p, b, s);
    return wx ? launch_bwd<NR_PREC_FP32, true>(p, b, s) : launch_bwd<NR_PREC_FP32, false>(p, b, s);
}

int nr_mlp_backward_dw(const NrMlpConfig* cfg, int64_t M, const void* saved, void* workspace, nr_stream_t stream) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p)) return NR_EARG;
    NR_REQUIRE(saved && workspace && M >= 0, "nr_mlp_backward_dw: null pointer");
    NR_REQUIRE((reinterpret_cast<uintptr_t>(saved) & 15) == 0 && (reinterpret_cast<uintptr_t>(workspace) & 15) == 0,
               "nr_mlp_backward_dw: saved and workspace must be 16-byte aligned");
    if (M == 0) return NR_OK;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const MlpSizes z = make_sizes(p, M);
    const char* sv = static_cast<const char*>(saved);
    char* ws = static_cast<char*>(workspace);
    DwArgs w;
    std::memset(&w, 0, sizeof(w));
    w.slabs = reinterpret_cast<float*>(ws + z.slab_off);
    w.tiles = z.tiles;
    w.list = reinterpret_cast<const uint32_t*>(ws + z.dwlist_off);  // written by nr_mlp_backward_dx
    w.count = reinterpret_cast<const uint32_t*>(ws + z.count_off);
    w.njobs = p.n_jobs;
    int nwg = 0;
    NR_REQUIRE(p.n_jobs <= 32 && z.max_chunks < 2048, "nr_mlp_backward_dw: %d jobs x %d chunks beyond the map",
               p.n_jobs, z.max_chunks);
    for (int c = 0; c < z.max_chunks; ++c)
        for (int j = 0; j < p.n_jobs; ++j)
            if (c < z.job_chunks[j]) {
                NR_REQUIRE(nwg < kDwMaxWgs, "nr_mlp_backward_dw: more than %d workgroups", kDwMaxWgs);
                w.wg_map[nwg++] = static_cast<uint16_t>(j | c << 5);
            }
    for (int j = 0; j < p.n_jobs; ++j) w.job_chunks[j] = z.job_chunks[j];
    w.slab_floats_per_chunk = p.slab_floats_per_chunk;
    int max_blk = 0;
    for (int j = 0; j < p.n_jobs; ++j) {
        const DwJob& jb = p.job[j];
        w.job_NBz[j] = jb.NBz;
        w.job_KB[j] = jb.KB;
        for (int v = 0; v < kDwWaves; ++v) {
            if (v >= jb.nwaves) {
                w.job_wave[j][v] = 0;
                continue;
            }
            const DwWave& sh = jb.w[v];
            NR_REQUIRE(sh.np >= 1 && sh.np <= kDwMaxP && sh.nq >= 1 && sh.nq <= kDwMaxQ && sh.row0 >= 0 &&
                           sh.row0 + sh.np <= jb.NBz && sh.col0 >= 0 && sh.col0 + sh.nq <= jb.KB && jb.NBz < 64 &&
                           jb.KB < 64,
                       "nr_mlp_backward_dw: job %d wave %d share out of its %dx%d grid", j, v, jb.NBz, jb.KB);
            w.job_wave[j][v] = dw_wave_pack(sh.row0, sh.np, sh.col0, sh.nq, sh.bias);
        }
        int ns = 0;
        for (int q = 0; q < jb.ndz; ++q, ++ns) {
            w.seg_ptr[j][ns] = (jb.dz[q].is_ws ? ws : sv) + (jb.dz[q].is_ws ? z.ws_off : z.saved_off)[jb.dz[q].tensor];
            w.seg_blocks[j][ns] = static_cast<uint8_t>(jb.dz[q].blocks);
        }
        for (int q = 0; q < jb.nin; ++q, ++ns) {
            w.seg_ptr[j][ns] = (jb.in[q].is_ws ? ws : sv) + (jb.in[q].is_ws ? z.ws_off : z.saved_off)[jb.in[q].tensor];
            w.seg_blocks[j][ns] = static_cast<uint8_t>(jb.in[q].blocks);
        }
        w.job_slab[j] = jb.slab_off;
        NR_REQUIRE((jb.NBz + jb.KB) * p.fpb <= kDwWaves * dw_max_pieces(p.fpb == 2),
                   "nr_mlp_backward_dw: job %d stages %d blocks, beyond the kernel's per-wave pieces", j, jb.NBz + jb.KB);
        max_blk = jb.NBz + jb.KB > max_blk ? jb.NBz + jb.KB : max_blk;
    }
    w.stage_bytes = max_blk * p.fpb * kFragBytes;
    // as many stages as fit in 160 KiB (+1 KB scratch): 4 for bf16, 2 for fp32
    w.nstage = static_cast<int>((160 * 1024 - kFragBytes) / w.stage_bytes);
    if (w.nstage > NR_DW_NSTAGE) w.nstage = NR_DW_NSTAGE;
    size_t lds = static_cast<size_t>(w.nstage) * w.stage_bytes + kFragBytes;
    // the largest chunk's list entries behind the stages, when they fit
    int min_chunks = z.job_chunks[0];
    for (int j = 1; j < p.n_jobs; ++j) min_chunks = z.job_chunks[j] < min_chunks ? z.job_chunks[j] : min_chunks;
    const size_t list_bytes = (static_cast<size_t>(ceil_div_ll(z.tiles, min_chunks)) * 4 + 15) / 16 * 16;
    if (lds + list_bytes <= 160 * 1024) {
        w.list_lds = static_cast<int>(lds);
        lds += list_bytes;
    }
    NR_REQUIRE(w.nstage >= 2, "nr_mlp_backward_dw: a %d-byte stage does not fit twice in LDS", w.stage_bytes);
    NR_REQUIRE(lds <= 160 * 1024, "nr_mlp_backward_dw: %zu bytes of LDS staging exceeds 160 KiB", lds);
    const dim3 grid(static_cast<unsigned>(nwg)), block(kDwThreads);
    if (p.prec == NR_PREC_BF16)
        hipLaunchKernelGGL(mlp_dw_kernel<NR_PREC_BF16>, grid, block, lds, s, w);
    else if (p.prec == NR_PREC_FP16)
        hipLaunchKernelGGL(mlp_dw_kernel<NR_PREC_FP16>, grid, block, lds, s, w);
    else
        hipLaunchKernelGGL(mlp_dw_kernel<NR_PREC_FP32>, grid, block, lds, s, w);
    NR_LAUNCH_CHECK("nr_mlp_backward_dw");
    return NR_OK;
}

int nr_mlp_backward_reduce(const NrMlpConfig* cfg, int64_t M, const void* workspace, float* g_params,
                           nr_stream_t stream) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p)) return NR_EARG;
    NR_REQUIRE(workspace && g_params && M >= 0, "nr_mlp_backward_reduce: null pointer");
    const hipStream_t s = static_cast<hipStream_t>(stream);
    if (M == 0) {
        (void)hipMemsetAsync(g_params, 0, sizeof(float) * p.param_count, s);
        return check_launch("nr_mlp_backward_reduce");
    }
    const MlpSizes z = make_sizes(p, M);
    ReduceArgs r;
    std::memset(&r, 0, sizeof(r));
    r.slabs = reinterpret_cast<const float*>(static_cast<const char*>(workspace) + z.slab_off);
    r.g = g_params;
    r.inv_gscale = 1.0f / grad_scale(p.prec);
    r.param_count = p.param_count;
    r.slab_floats_per_chunk = p.slab_floats_per_chunk;
    r.n_red = p.n_red;
    for (int k = 0; k < p.n_red; ++k) {
        const ReduceRange& rr = p.red[k];
        r.rows[k] = rr.rows;
        r.in[k] = rr.in;
        r.nseg[k] = rr.nseg;
        r.bjob[k] = rr.bjob;
        r.brow0[k] = rr.brow0;
        r.w_off[k] = rr.w_off;
        r.b_off[k] = rr.b_off;
        for (int q = 0; q < rr.nseg; ++q) r.seg[k][q] = rr.seg[q];
    }
    for (int j = 0; j < p.n_jobs; ++j) {
        r.job_slab[j] = p.job[j].slab_off;
        r.job_KB[j] = p.job[j].KB;
        r.job_chunks[j] = z.job_chunks[j];
    }
    int max_rows = 1;
    for (int k = 0; k < p.n_red; ++k) max_rows = p.red[k].rows > max_rows ? p.red[k].rows : max_rows;
    hipLaunchKernelGGL(mlp_dw_reduce_kernel, dim3(static_cast<unsigned>(max_rows), static_cast<unsigned>(p.n_red)),
                       dim3(256), 0, s, r);
    NR_LAUNCH_CHECK("nr_mlp_backward_reduce");
    return NR_OK;
}

int64_t nr_mlp_active_tiles_offset(const NrMlpConfig* cfg, int64_t M) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p) || M <= 0) return -1;
    return make_sizes(p, M).count_off;
}

int nr_mlp_backward(const NrMlpConfig* cfg, const void* packed, const float* params, const float* x, const float* d,
                    int64_t M, const float* rgb, const float* sigma, const void* saved, const float* g_rgb,
                    const float* g_sigma, float* g_params, float* g_x, float* g_d, void* workspace,
                    nr_stream_t stream) {
    NR_REQUIRE(g_params, "nr_mlp_backward: null g_params");
    // the split form: dX chain (dz images), then the dW GEMM over them
    int rc = nr_mlp_backward_dx(cfg, packed, params, x, d, M, rgb, sigma, saved, g_rgb, g_sigma, g_x, g_d, workspace,
                                stream);
    if (rc) return rc;
    rc = nr_mlp_backward_dw(cfg, M, saved, workspace, stream);
    if (rc) return rc;
    return nr_mlp_backward_reduce(cfg, M, workspace, g_params, stream);
}

}  // extern "C"
