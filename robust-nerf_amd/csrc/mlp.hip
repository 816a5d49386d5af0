// Fused NeRF MLP on MFMA (gfx950): weight packing, training/inference forward,
// backward dX chain, and the dW GEMM with a deterministic split-M reduction.
//
// Reference: noisy_src/model.py:20-221 — PositionalEncoding (no pi), 8x256 ReLU
// trunk with skip cat([x_enc, h]) after layer 4, sigma = relu(W h), feat = W h
// (no activation), h_c = relu(W [feat, d_enc]), rgb = sigmoid(W h_c).
//
// Formulation: every layer computes out^T = W . in^T with one 32-sample tile
// per wave.  In the MFMA C/D layout a lane holds 16 features of ONE sample, so
// a layer's accumulator tile is already the next layer's B operand (after a
// pack to bf16, or as-is in fp32): activations stay in registers for the whole
// network and never touch LDS.  The A operand (weights) comes from a packed
// image in which each lane's 16 bytes for one MFMA are contiguous, with the
// k order permuted to match the accumulator's row order:
//   bf16 32x32x16, k-step s: element j <-> input feature 16s + 8(j>>2) + 4h + (j&3)
//   fp32 32x32x2,  k-step t: lane half h <-> input feature (t&3) + 8(t>>2) + 4h
// The same images are built for W^T, so the backward chain has the same form.
#include <cstring>

#include "common.hpp"
#include "mfma.hpp"
#include "mlp_plan.hpp"

#include "mlp_plan.cpp.inc"

namespace nr {

constexpr int kWavesPerBlock = 4;

template <int PREC>
struct InBlk;
template <>
struct InBlk<NR_PREC_BF16> {
    bf16x8 s[2];
};
template <>
struct InBlk<NR_PREC_FP32> {
    f32x16 v;
};

template <int PREC>
constexpr int kFPB = PREC == NR_PREC_BF16 ? 2 : 4;  // 1-KB fragments per 32x32 block

template <int PREC>
__device__ __forceinline__ void to_in(const f32x16& a, InBlk<PREC>& o) {
    if constexpr (PREC == NR_PREC_BF16) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            o.s[0][j] = static_cast<__bf16>(a[j]);
            o.s[1][j] = static_cast<__bf16>(a[8 + j]);
        }
    } else {
        o.v = a;
    }
}

// The flat nn.Module parameter layout has odd offsets (feature_linear starts at
// 493,313 floats for the default model), so parameter reads are scalar.
__device__ __forceinline__ f32x4 ld4u(const float* __restrict__ p) { return f32x4{p[0], p[1], p[2], p[3]}; }

__device__ __forceinline__ void zero(f32x16& a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = 0.f;
}

// acc[nb] += A(nb0+nb, kb0+kb) . in[kb]  for a packed image with KBtot column blocks.
template <int PREC, int NBO, int KBN>
__device__ __forceinline__ void gemm(f32x16 (&acc)[NBO], int nb0, const InBlk<PREC> (&in)[KBN], int kb0,
                                     const char* __restrict__ base, int KBtot, int lane) {
#pragma unroll
    for (int kb = 0; kb < KBN; ++kb) {
#pragma unroll
        for (int nb = 0; nb < NBO; ++nb) {
            const char* p = base + static_cast<int64_t>(((nb0 + nb) * KBtot + kb0 + kb) * kFPB<PREC>) * kFragBytes +
                            lane * 16;
            if constexpr (PREC == NR_PREC_BF16) {
                const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(p);
                const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(p + kFragBytes);
                acc[nb] = mfma_bf16(a0, in[kb].s[0], acc[nb]);
                acc[nb] = mfma_bf16(a1, in[kb].s[1], acc[nb]);
            } else {
#pragma unroll
                for (int tq = 0; tq < 4; ++tq) {
                    const f32x4 a = *reinterpret_cast<const f32x4*>(p + tq * kFragBytes);
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[nb] = mfma_f32(a[e], in[kb].v[4 * tq + e], acc[nb]);
                }
            }
        }
    }
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
    return rem < 3 ? sinf(v) : cosf(v);
}

// d gamma_f / d x_c, contracted with g: adds into gx[c].
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
    if (c == 0)
        g0 += d;
    else if (c == 1)
        g1 += d;
    else
        g2 += d;
}

// Store one accumulator block (32 features x 32 samples) into a tile-blocked,
// feature-major tensor: (f, m) at tile*F*32 + f*32 + m.
template <int PREC>
__device__ __forceinline__ void store_block(char* __restrict__ region, int64_t tile, int F, int blk, const f32x16& v,
                                            int lane) {
    const int h = lane >> 5, ml = lane & 31;
    const int64_t e0 = tile * F * 32 + static_cast<int64_t>(blk) * 32 * 32 + ml;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t e = e0 + acc_row(r, h) * 32;
        if constexpr (PREC == NR_PREC_BF16)
            reinterpret_cast<unsigned short*>(region)[e] = bf16_bits(v[r]);
        else
            reinterpret_cast<float*>(region)[e] = v[r];
    }
}

// bias + optional ReLU on NBO blocks; returns mask bits (bit nb*16+r) in w[4].
template <int NBO, bool RELU>
__device__ __forceinline__ void bias_act(f32x16 (&acc)[NBO], const float* __restrict__ bias, int lane,
                                         unsigned (&w)[4]) {
    const int h = lane >> 5;
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = 0u;
#pragma unroll
    for (int nb = 0; nb < NBO; ++nb) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 b = ld4u(bias + 32 * nb + 8 * g + 4 * h);
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
    int64_t pk[kMaxMfmaLayers];
    int KB[kMaxMfmaLayers];
    int64_t bias[kMaxMfmaLayers];
    int64_t sig_w, sig_b, rgb_w, rgb_b;
    int64_t sv_off[kMaxTrunk + 4];
    int sv_F[kMaxTrunk + 4];
    int sv_feat, sv_denc, sv_hc;
    int64_t mask_off;
    int n_mask;
};

template <int PREC, int XB, int DB, bool TRAIN>
__global__ __launch_bounds__(64 * kWavesPerBlock) void mlp_fwd_kernel(FwdArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, ml = lane & 31;
    const int64_t tile = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
    if (tile >= a.tiles) return;
    const int64_t m = tile * 32 + ml;
    const bool valid = m < a.M;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f;
    if (valid) {
        x0 = a.x[3 * m];
        x1 = a.x[3 * m + 1];
        x2 = a.x[3 * m + 2];
    }
    const int n = a.n_layers;
    unsigned* masks = reinterpret_cast<unsigned*>(a.saved + a.mask_off);

    InBlk<PREC> xe[XB];
#pragma unroll
    for (int kb = 0; kb < XB; ++kb) {
        f32x16 t;
#pragma unroll
        for (int r = 0; r < 16; ++r) t[r] = pe_feat(x0, x1, x2, 32 * kb + acc_row(r, h), a.L);
        to_in<PREC>(t, xe[kb]);
        if constexpr (TRAIN) store_block<PREC>(a.saved + a.sv_off[SV_XENC], tile, a.sv_F[SV_XENC], kb, t, lane);
    }

    f32x16 acc[kHB];
    InBlk<PREC> hin[kHB];
    unsigned w[4];
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) zero(acc[nb]);
        const char* base = a.packed + a.pk[i];
        if (i == 0) {
            gemm<PREC, kHB, XB>(acc, 0, xe, 0, base, a.KB[i], lane);
        } else if ((a.skips >> (i - 1)) & 1u) {
            gemm<PREC, kHB, XB>(acc, 0, xe, 0, base, a.KB[i], lane);
            gemm<PREC, kHB, kHB>(acc, 0, hin, XB, base, a.KB[i], lane);
        } else {
            gemm<PREC, kHB, kHB>(acc, 0, hin, 0, base, a.KB[i], lane);
        }
        bias_act<kHB, true>(acc, a.params + a.bias[i], lane, w);
        if constexpr (TRAIN) {
            char* region = a.saved + a.sv_off[SV_H0 + i];
#pragma unroll
            for (int nb = 0; nb < kHB; ++nb) store_block<PREC>(region, tile, kHidden, nb, acc[nb], lane);
            reinterpret_cast<u32x4*>(masks)[(tile * a.n_mask + i) * 64 + lane] = u32x4{w[0], w[1], w[2], w[3]};
        }
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) to_in<PREC>(acc[nb], hin[nb]);
    }

    // sigma head (VALU): relu(w_sigma . h + b)
    float sp = 0.f;
    {
        const float* ws = a.params + a.sig_w;
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 wv = ld4u(ws + 32 * nb + 8 * g + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; ++e) sp += wv[e] * acc[nb][4 * g + e];
            }
        sp += __shfl_xor(sp, 32);
        sp = sp + a.params[a.sig_b];
        sp = sp > 0.f ? sp : 0.f;
    }

    // feature_linear (no activation)
#pragma unroll
    for (int nb = 0; nb < kHB; ++nb) zero(acc[nb]);
    gemm<PREC, kHB, kHB>(acc, 0, hin, 0, a.packed + a.pk[n], a.KB[n], lane);
    bias_act<kHB, false>(acc, a.params + a.bias[n], lane, w);
    if constexpr (TRAIN) {
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) store_block<PREC>(a.saved + a.sv_off[a.sv_feat], tile, kHidden, nb, acc[nb], lane);
    }
#pragma unroll
    for (int nb = 0; nb < kHB; ++nb) to_in<PREC>(acc[nb], hin[nb]);

    // dir_linear over [feat, d_enc], ReLU
    constexpr int NC = kHB / 2;
    f32x16 ac[NC];
#pragma unroll
    for (int nb = 0; nb < NC; ++nb) zero(ac[nb]);
    const char* dbase = a.packed + a.pk[n + 1];
    gemm<PREC, NC, kHB>(ac, 0, hin, 0, dbase, a.KB[n + 1], lane);
    if constexpr (DB > 0) {
        float d0 = 0.f, d1 = 0.f, d2 = 0.f;
        if (valid) {
            d0 = a.d[3 * m];
            d1 = a.d[3 * m + 1];
            d2 = a.d[3 * m + 2];
        }
        InBlk<PREC> de[DB];
#pragma unroll
        for (int kb = 0; kb < DB; ++kb) {
            f32x16 t;
#pragma unroll
            for (int r = 0; r < 16; ++r) t[r] = pe_feat(d0, d1, d2, 32 * kb + acc_row(r, h), a.Ld);
            to_in<PREC>(t, de[kb]);
            if constexpr (TRAIN) store_block<PREC>(a.saved + a.sv_off[a.sv_denc], tile, DB * 32, kb, t, lane);
        }
        gemm<PREC, NC, DB>(ac, 0, de, kHB, dbase, a.KB[n + 1], lane);
    }
    bias_act<NC, true>(ac, a.params + a.bias[n + 1], lane, w);
    if constexpr (TRAIN) {
#pragma unroll
        for (int nb = 0; nb < NC; ++nb) store_block<PREC>(a.saved + a.sv_off[a.sv_hc], tile, kHidden / 2, nb, ac[nb], lane);
        reinterpret_cast<u32x4*>(masks)[(tile * a.n_mask + n) * 64 + lane] = u32x4{w[0], w[1], w[2], w[3]};
    }

    // rgb head (VALU): sigmoid(W_rgb h_c + b)
    float pr[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float* wr = a.params + a.rgb_w + c * (kHidden / 2);
        float s = 0.f;
#pragma unroll
        for (int nb = 0; nb < NC; ++nb)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 wv = ld4u(wr + 32 * nb + 8 * g + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; ++e) s += wv[e] * ac[nb][4 * g + e];
            }
        s += __shfl_xor(s, 32);
        s = s + a.params[a.rgb_b + c];
        pr[c] = 1.0f / (1.0f + expf(-s));
    }
    if (valid && h == 0) {
        a.rgb[3 * m] = pr[0];
        a.rgb[3 * m + 1] = pr[1];
        a.rgb[3 * m + 2] = pr[2];
        a.sigma[m] = sp;
    }
}

struct BwdArgs {
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
    int L, Ld, n_layers;
    uint32_t skips;
    int64_t pkT[kMaxMfmaLayers];
    int NB[kMaxMfmaLayers];
    int64_t sig_w, rgb_w;
    int64_t mask_off;
    int n_mask;
    int64_t ws_off[kMaxTrunk + 3];
    int ws_feat, ws_dir, ws_heads;
};

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

template <int PREC, int XB, int DB>
__global__ __launch_bounds__(64 * kWavesPerBlock) void mlp_bwd_kernel(BwdArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, ml = lane & 31;
    const int64_t tile = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
    if (tile >= a.tiles) return;
    const int64_t m = tile * 32 + ml;
    const bool valid = m < a.M;
    const int n = a.n_layers;
    const u32x4* masks = reinterpret_cast<const u32x4*>(a.saved + a.mask_off);
    auto mask_of = [&](int layer) { return masks[(tile * a.n_mask + layer) * 64 + lane]; };

    // heads: sigmoid / relu backward (torch: g * (1 - y) * y ; g * (y > 0))
    float dz_rgb[3] = {0.f, 0.f, 0.f}, dz_s = 0.f;
    if (valid) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float y = a.rgb[3 * m + c];
            dz_rgb[c] = (a.g_rgb[3 * m + c] * (1.0f - y)) * y;
        }
        dz_s = a.sigma[m] > 0.f ? a.g_sigma[m] : 0.f;
    }
    {
        f32x16 hb;
        zero(hb);
        if (h == 0) {
            hb[0] = dz_s;
            hb[1] = dz_rgb[0];
            hb[2] = dz_rgb[1];
            hb[3] = dz_rgb[2];
        }
        store_block<PREC>(a.ws + a.ws_off[a.ws_heads], tile, 32, 0, hb, lane);
    }

    // dz_c = (W_rgb^T dz_rgb) * [h_c > 0]
    constexpr int NC = kHB / 2;
    f32x16 dc[NC];
    {
        const float* wr = a.params + a.rgb_w;
#pragma unroll
        for (int nb = 0; nb < NC; ++nb)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int f0 = 32 * nb + 8 * g + 4 * h;
                const f32x4 w0 = ld4u(wr + f0);
                const f32x4 w1 = ld4u(wr + kHidden / 2 + f0);
                const f32x4 w2 = ld4u(wr + kHidden + f0);
#pragma unroll
                for (int e = 0; e < 4; ++e) dc[nb][4 * g + e] = (w0[e] * dz_rgb[0] + w1[e] * dz_rgb[1]) + w2[e] * dz_rgb[2];
            }
        apply_mask<NC>(dc, mask_of(n));
    }
    InBlk<PREC> cin[NC];
#pragma unroll
    for (int nb = 0; nb < NC; ++nb) {
        store_block<PREC>(a.ws + a.ws_off[a.ws_dir], tile, kHidden / 2, nb, dc[nb], lane);
        to_in<PREC>(dc[nb], cin[nb]);
    }

    // d feat = W_dir^T dz_c  (feature_linear has no activation: dz_feat = d feat)
    f32x16 acc[kHB];
    InBlk<PREC> hin[kHB];
#pragma unroll
    for (int nb = 0; nb < kHB; ++nb) zero(acc[nb]);
    const char* dirT = a.packed + a.pkT[n + 1];
    gemm<PREC, kHB, NC>(acc, 0, cin, 0, dirT, a.NB[n + 1], lane);
    if constexpr (DB > 0) {
        if (a.g_d) {
            f32x16 dd[DB];
#pragma unroll
            for (int kb = 0; kb < DB; ++kb) zero(dd[kb]);
            gemm<PREC, DB, NC>(dd, kHB, cin, 0, dirT, a.NB[n + 1], lane);
            float d0 = 0.f, d1 = 0.f, d2 = 0.f;
            if (valid) {
                d0 = a.d[3 * m];
                d1 = a.d[3 * m + 1];
                d2 = a.d[3 * m + 2];
            }
            float g0 = 0.f, g1 = 0.f, g2 = 0.f;
#pragma unroll
            for (int kb = 0; kb < DB; ++kb)
#pragma unroll
                for (int r = 0; r < 16; ++r) pe_feat_bwd(d0, d1, d2, 32 * kb + acc_row(r, h), a.Ld, dd[kb][r], g0, g1, g2);
            g0 += __shfl_xor(g0, 32);
            g1 += __shfl_xor(g1, 32);
            g2 += __shfl_xor(g2, 32);
            if (valid && h == 0) {
                a.g_d[3 * m] = g0;
                a.g_d[3 * m + 1] = g1;
                a.g_d[3 * m + 2] = g2;
            }
        }
    }
#pragma unroll
    for (int nb = 0; nb < kHB; ++nb) {
        store_block<PREC>(a.ws + a.ws_off[a.ws_feat], tile, kHidden, nb, acc[nb], lane);
        to_in<PREC>(acc[nb], hin[nb]);
    }

    // d h_{n-1} = W_feat^T dz_feat + w_sigma dz_sigma, then * [h_{n-1} > 0]
#pragma unroll
    for (int nb = 0; nb < kHB; ++nb) zero(acc[nb]);
    gemm<PREC, kHB, kHB>(acc, 0, hin, 0, a.packed + a.pkT[n], a.NB[n], lane);
    {
        const float* ws = a.params + a.sig_w;
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 wv = ld4u(ws + 32 * nb + 8 * g + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[nb][4 * g + e] = acc[nb][4 * g + e] + wv[e] * dz_s;
            }
    }
    apply_mask<kHB>(acc, mask_of(n - 1));
#pragma unroll
    for (int nb = 0; nb < kHB; ++nb) {
        store_block<PREC>(a.ws + a.ws_off[WS_DZ0 + n - 1], tile, kHidden, nb, acc[nb], lane);
        to_in<PREC>(acc[nb], hin[nb]);
    }

    // trunk: dz_{i-1} = (W_i^T dz_i)[h part] * [h_{i-1} > 0]
    f32x16 dxe[XB];
#pragma unroll
    for (int kb = 0; kb < XB; ++kb) zero(dxe[kb]);
    const bool want_x = a.g_x != nullptr;
    for (int i = n - 1; i >= 1; --i) {
        const char* baseT = a.packed + a.pkT[i];
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) zero(acc[nb]);
        if ((a.skips >> (i - 1)) & 1u) {
            if (want_x) gemm<PREC, XB, kHB>(dxe, 0, hin, 0, baseT, a.NB[i], lane);
            gemm<PREC, kHB, kHB>(acc, XB, hin, 0, baseT, a.NB[i], lane);
        } else {
            gemm<PREC, kHB, kHB>(acc, 0, hin, 0, baseT, a.NB[i], lane);
        }
        apply_mask<kHB>(acc, mask_of(i - 1));
#pragma unroll
        for (int nb = 0; nb < kHB; ++nb) {
            store_block<PREC>(a.ws + a.ws_off[WS_DZ0 + i - 1], tile, kHidden, nb, acc[nb], lane);
            to_in<PREC>(acc[nb], hin[nb]);
        }
    }
    if (want_x) {
        gemm<PREC, XB, kHB>(dxe, 0, hin, 0, a.packed + a.pkT[0], a.NB[0], lane);
        float x0 = 0.f, x1 = 0.f, x2 = 0.f;
        if (valid) {
            x0 = a.x[3 * m];
            x1 = a.x[3 * m + 1];
            x2 = a.x[3 * m + 2];
        }
        float g0 = 0.f, g1 = 0.f, g2 = 0.f;
#pragma unroll
        for (int kb = 0; kb < XB; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) pe_feat_bwd(x0, x1, x2, 32 * kb + acc_row(r, h), a.L, dxe[kb][r], g0, g1, g2);
        g0 += __shfl_xor(g0, 32);
        g1 += __shfl_xor(g1, 32);
        g2 += __shfl_xor(g2, 32);
        if (valid && h == 0) {
            a.g_x[3 * m] = g0;
            a.g_x[3 * m + 1] = g1;
            a.g_x[3 * m + 2] = g2;
        }
    }
}

// ------------------------------------------------------------------ dW ----
// slab[job][chunk][row][col] += sum over the chunk's tiles of dz[row] x in[col];
// column KB*32 of each row holds the bias partial sum_m dz[row].
struct DwArgs {
    const char* saved;
    const char* ws;
    float* slabs;
    int64_t tiles;
    int chunks, tiles_per_chunk;
    int n_jobs;
    int job_wg0[kMaxJobs + 1];  // first workgroup of each job (cumulative)
    int job_sg[kMaxJobs];        // 4x4-block subgrids per job
    int job_nbg[kMaxJobs];       // subgrid rows (ceil(NB/4))
    int job_NB[kMaxJobs], job_KB[kMaxJobs], job_row0[kMaxJobs];
    int job_nin[kMaxJobs];
    int64_t job_dz_off[kMaxJobs];  // bytes
    int job_dz_F[kMaxJobs];
    int64_t job_in_off[kMaxJobs][kMaxSeg];
    int job_in_F[kMaxJobs][kMaxSeg];
    int job_in_blocks[kMaxJobs][kMaxSeg];
    int64_t job_slab[kMaxJobs];    // floats
    int64_t slab_floats_per_chunk;
};

// Operand fragment of a tile-blocked feature-major tensor for reduction over samples.
// bf16 32x32x16: lane (row i, half h), k-step s: 8 samples 16s+8h .. +7 of feature row.
template <int PREC>
__device__ __forceinline__ void load_rowfrag(const char* __restrict__ region, int64_t tile, int F, int row, int lane,
                                             bf16x8 (&b)[2], f32x4 (&f)[4]) {
    const int h = lane >> 5, i = lane & 31;
    if constexpr (PREC == NR_PREC_BF16) {
        const __bf16* p = reinterpret_cast<const __bf16*>(region) + (tile * F + row + i) * 32 + 8 * h;
        b[0] = *reinterpret_cast<const bf16x8*>(p);
        b[1] = *reinterpret_cast<const bf16x8*>(p + 16);
    } else {
        const float* p = reinterpret_cast<const float*>(region) + (tile * F + row + i) * 32 + 16 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) f[q] = *reinterpret_cast<const f32x4*>(p + 4 * q);
    }
}

template <int PREC>
__global__ __launch_bounds__(64 * kWavesPerBlock) void mlp_dw_kernel(DwArgs a) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wg = blockIdx.x;
    int j = 0;
    while (j + 1 < a.n_jobs && wg >= a.job_wg0[j + 1]) ++j;
    const int per_chunk = (a.job_sg[j] + kWavesPerBlock - 1) / kWavesPerBlock;
    const int local = wg - a.job_wg0[j];
    const int chunk = local / per_chunk;
    const int sg = (local % per_chunk) * kWavesPerBlock + wv;
    if (sg >= a.job_sg[j]) return;
    const int nbg = sg % a.job_nbg[j], kbg = sg / a.job_nbg[j];
    const int NB = a.job_NB[j], KB = a.job_KB[j];
    const int64_t t0 = static_cast<int64_t>(chunk) * a.tiles_per_chunk;
    int64_t t1 = t0 + a.tiles_per_chunk;
    if (t1 > a.tiles) t1 = a.tiles;

    // input block kb -> (segment, block in segment)
    int in_seg[4], in_blk[4];
    bool kval[4], nval[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int kb = 4 * kbg + q;
        kval[q] = kb < KB;
        const int s = (a.job_nin[j] > 1 && kb >= a.job_in_blocks[j][0]) ? 1 : 0;
        in_seg[q] = s;
        in_blk[q] = kb - (s ? a.job_in_blocks[j][0] : 0);
        nval[q] = 4 * nbg + q < NB;
    }
    const bool do_bias = kbg == 0;

    f32x16 acc[4][4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) zero(acc[p][q]);
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};

    const char* dz = a.ws + a.job_dz_off[j];
    for (int64_t t = t0; t < t1; ++t) {
        bf16x8 ab[4][2], bb[4][2];
        f32x4 af[4][4], bf[4][4];
#pragma unroll
        for (int p = 0; p < 4; ++p)
            if (nval[p]) load_rowfrag<PREC>(dz, t, a.job_dz_F[j], 32 * (4 * nbg + p), lane, ab[p], af[p]);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (kval[q])
                load_rowfrag<PREC>(a.saved + a.job_in_off[j][in_seg[q]], t, a.job_in_F[j][in_seg[q]], 32 * in_blk[q],
                                   lane, bb[q], bf[q]);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if (!nval[p]) continue;
            if (do_bias) {
                if constexpr (PREC == NR_PREC_BF16) {
#pragma unroll
                    for (int s = 0; s < 2; ++s)
#pragma unroll
                        for (int e = 0; e < 8; ++e) bsum[p] += static_cast<float>(ab[p][s][e]);
                } else {
#pragma unroll
                    for (int s = 0; s < 4; ++s)
#pragma unroll
                        for (int e = 0; e < 4; ++e) bsum[p] += af[p][s][e];
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (!kval[q]) continue;
                if constexpr (PREC == NR_PREC_BF16) {
                    acc[p][q] = mfma_bf16(ab[p][0], bb[q][0], acc[p][q]);
                    acc[p][q] = mfma_bf16(ab[p][1], bb[q][1], acc[p][q]);
                } else {
#pragma unroll
                    for (int s = 0; s < 4; ++s)
#pragma unroll
                        for (int e = 0; e < 4; ++e) acc[p][q] = mfma_f32(af[p][s][e], bf[q][s][e], acc[p][q]);
                }
            }
        }
    }
    // write the slab: row = dz row n, col = input feature k (padded)
    float* slab = a.slabs + static_cast<int64_t>(chunk) * a.slab_floats_per_chunk + a.job_slab[j];
    const int ld = KB * 32 + 1;
    const int h = lane >> 5, ml = lane & 31;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        if (!nval[p]) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (!kval[q]) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = 32 * (4 * nbg + p) + acc_row(r, h);
                const int col = 32 * (4 * kbg + q) + ml;
                slab[static_cast<int64_t>(row) * ld + col] = acc[p][q][r];
            }
        }
        if (do_bias) {
            const float tot = bsum[p] + __shfl_xor(bsum[p], 32);
            if (h == 0) slab[static_cast<int64_t>(32 * (4 * nbg + p) + ml) * ld + KB * 32] = tot;
        }
    }
}

// g_params[param] = sum over chunks of the slab entry it maps to (chunk order:
// deterministic).  One thread per parameter.
struct ReduceArgs {
    const float* slabs;
    float* g;
    int64_t param_count;
    int chunks;
    int64_t slab_floats_per_chunk;
    int n_jobs;
    int64_t job_p0[kMaxJobs + 1];  // first flat parameter of each job (weights then bias)
    int64_t job_w_off[kMaxJobs], job_b_off[kMaxJobs];
    int job_rows[kMaxJobs], job_in[kMaxJobs], job_KB[kMaxJobs], job_row0[kMaxJobs];
    int job_nseg[kMaxJobs];
    int job_seg_col0[kMaxJobs][kMaxSeg], job_seg_w[kMaxJobs][kMaxSeg], job_seg_blk0[kMaxJobs][kMaxSeg];
    int64_t job_slab[kMaxJobs];
};

__global__ void mlp_dw_reduce_kernel(ReduceArgs a) {
    const int64_t pidx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (pidx >= a.param_count) return;
    // find the job whose weight or bias range holds pidx
    int j = -1;
    int64_t row = 0, col = -1;  // col = -1 => bias
    for (int q = 0; q < a.n_jobs; ++q) {
        const int64_t wsz = static_cast<int64_t>(a.job_rows[q]) * a.job_in[q];
        if (pidx >= a.job_w_off[q] && pidx < a.job_w_off[q] + wsz) {
            j = q;
            const int64_t e = pidx - a.job_w_off[q];
            row = e / a.job_in[q];
            const int c = static_cast<int>(e % a.job_in[q]);
            // W column c -> padded slab column
            for (int s = 0; s < a.job_nseg[q]; ++s)
                if (c >= a.job_seg_col0[q][s] && c < a.job_seg_col0[q][s] + a.job_seg_w[q][s])
                    col = 32 * a.job_seg_blk0[q][s] + (c - a.job_seg_col0[q][s]);
            break;
        }
        if (pidx >= a.job_b_off[q] && pidx < a.job_b_off[q] + a.job_rows[q]) {
            j = q;
            row = pidx - a.job_b_off[q];
            col = static_cast<int64_t>(a.job_KB[q]) * 32;
            break;
        }
    }
    if (j < 0) return;
    const int ld = a.job_KB[j] * 32 + 1;
    const float* s = a.slabs + a.job_slab[j] + (row + a.job_row0[j]) * ld + col;
    float acc = 0.f;
    for (int c = 0; c < a.chunks; ++c) acc += s[static_cast<int64_t>(c) * a.slab_floats_per_chunk];
    a.g[pidx] = acc;
}

// ---------------------------------------------------------------- pack ----
struct PackArgs {
    const float* params;
    char* packed;
    int n_lin;
    int prec;
    int64_t w_off[kMaxMfmaLayers];
    int in[kMaxMfmaLayers], NB[kMaxMfmaLayers], KB[kMaxMfmaLayers], nseg[kMaxMfmaLayers];
    int seg_col0[kMaxMfmaLayers][kMaxSeg], seg_w[kMaxMfmaLayers][kMaxSeg], seg_blk[kMaxMfmaLayers][kMaxSeg];
    int64_t pk[kMaxMfmaLayers];   // byte offset of the fwd image; bwd image follows
    int64_t cum[kMaxMfmaLayers + 1];  // cumulative element counts (fwd+bwd per layer)
};

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

__global__ void mlp_pack_kernel(PackArgs a) {
    const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g >= a.cum[a.n_lin]) return;
    int l = 0;
    while (g >= a.cum[l + 1]) ++l;
    const int64_t img = (a.cum[l + 1] - a.cum[l]) / 2;
    int64_t e = g - a.cum[l];
    const bool bwd = e >= img;
    if (bwd) e -= img;
    const bool bf = a.prec == NR_PREC_BF16;
    const int epl = bf ? 8 : 4, fpb = bf ? 2 : 4;
    const int64_t frag = e / (64 * epl);
    const int lane = static_cast<int>((e / epl) % 64);
    const int el = static_cast<int>(e % epl);
    const int64_t blk = frag / fpb;
    const int sub = static_cast<int>(frag % fpb);
    const int h = lane >> 5, i = lane & 31;
    const int kk = bf ? 16 * sub + 8 * (el >> 2) + 4 * h + (el & 3) : acc_row(4 * sub + el, h);
    int row, col;
    if (!bwd) {  // W fragment (nb, kb): A[i][k] = W[32nb+i][col(kb,k)]
        const int nb = static_cast<int>(blk / a.KB[l]), kb = static_cast<int>(blk % a.KB[l]);
        row = 32 * nb + i;
        col = pack_col(a, l, kb, kk);
    } else {  // W^T fragment (ib, ob): A[i][k] = W[32ob+k][col(ib,i)]
        const int ib = static_cast<int>(blk / a.NB[l]), ob = static_cast<int>(blk % a.NB[l]);
        row = 32 * ob + kk;
        col = pack_col(a, l, ib, i);
    }
    const float v = col >= 0 ? a.params[a.w_off[l] + static_cast<int64_t>(row) * a.in[l] + col] : 0.f;
    char* dst = a.packed + a.pk[l] + (bwd ? img * (bf ? 2 : 4) : 0);
    if (bf)
        reinterpret_cast<unsigned short*>(dst)[e] = bf16_bits(v);
    else
        reinterpret_cast<float*>(dst)[e] = v;
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

template <int PREC, bool TRAIN>
int launch_fwd(const MlpPlan& p, const FwdArgs& a, hipStream_t s) {
    const dim3 grid(static_cast<unsigned>(ceil_div_ll(a.tiles, kWavesPerBlock))), block(64 * kWavesPerBlock);
#define NR_FWD(XB_, DB_)                                                                         \
    if (p.XB == XB_ && p.DB == DB_) {                                                            \
        hipLaunchKernelGGL((mlp_fwd_kernel<PREC, XB_, DB_, TRAIN>), grid, block, 0, s, a);       \
        return check_launch("nr_mlp_forward");                                                   \
    }
    NR_FWD(2, 1)
    NR_FWD(2, 0)
    NR_FWD(1, 1)
#undef NR_FWD
    set_error("nr_mlp_forward: no kernel instance for XB=%d DB=%d (pos_freqs/dir_freqs)", p.XB, p.DB);
    return NR_EARG;
}

template <int PREC>
int launch_bwd(const MlpPlan& p, const BwdArgs& a, hipStream_t s) {
    const dim3 grid(static_cast<unsigned>(ceil_div_ll(a.tiles, kWavesPerBlock))), block(64 * kWavesPerBlock);
#define NR_BWD(XB_, DB_)                                                                   \
    if (p.XB == XB_ && p.DB == DB_) {                                                      \
        hipLaunchKernelGGL((mlp_bwd_kernel<PREC, XB_, DB_>), grid, block, 0, s, a);        \
        return check_launch("nr_mlp_backward");                                            \
    }
    NR_BWD(2, 1)
    NR_BWD(2, 0)
    NR_BWD(1, 1)
#undef NR_BWD
    set_error("nr_mlp_backward: no kernel instance for XB=%d DB=%d (pos_freqs/dir_freqs)", p.XB, p.DB);
    return NR_EARG;
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
        const int64_t elems = static_cast<int64_t>(d.NB) * d.KB * 1024;  // 32x32 elements per block
        a.cum[l + 1] = a.cum[l] + 2 * elems;
    }
    const int64_t total = a.cum[p.n_lin];
    hipLaunchKernelGGL(mlp_pack_kernel, dim3(static_cast<unsigned>(ceil_div_ll(total, 256))), dim3(256), 0,
                       static_cast<hipStream_t>(stream), a);
    NR_LAUNCH_CHECK("nr_mlp_pack");
    return NR_OK;
}

int nr_mlp_forward(const NrMlpConfig* cfg, const void* packed, const float* params, const float* x, const float* d,
                   int64_t M, float* rgb, float* sigma, void* saved, nr_stream_t stream) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p)) return NR_EARG;
    NR_REQUIRE(packed && params && x && rgb && sigma && M >= 0, "nr_mlp_forward: null pointer");
    NR_REQUIRE(!p.use_vd || d, "nr_mlp_forward: use_view_dirs needs d (model.py:187-191)");
    NR_REQUIRE((reinterpret_cast<uintptr_t>(saved) & 15) == 0, "nr_mlp_forward: saved must be 16-byte aligned");
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
    for (int l = 0; l < p.n_lin; ++l) {
        a.pk[l] = p.lin[l].pk_fwd;
        a.KB[l] = p.lin[l].KB;
        a.bias[l] = p.lin[l].b_off;
    }
    a.sig_w = p.sig_w;
    a.sig_b = p.sig_b;
    a.rgb_w = p.rgb_w;
    a.rgb_b = p.rgb_b;
    for (int t = 0; t < p.n_saved; ++t) {
        a.sv_off[t] = z.saved_off[t];
        a.sv_F[t] = p.sv_F[t];
    }
    a.sv_feat = p.sv_feat;
    a.sv_denc = p.sv_denc;
    a.sv_hc = p.sv_hc;
    a.mask_off = z.mask_off;
    a.n_mask = p.n_mask;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    if (p.prec == NR_PREC_BF16)
        return saved ? launch_fwd<NR_PREC_BF16, true>(p, a, s) : launch_fwd<NR_PREC_BF16, false>(p, a, s);
    return saved ? launch_fwd<NR_PREC_FP32, true>(p, a, s) : launch_fwd<NR_PREC_FP32, false>(p, a, s);
}

int nr_mlp_backward(const NrMlpConfig* cfg, const void* packed, const float* params, const float* x, const float* d,
                    int64_t M, const float* rgb, const float* sigma, const void* saved, const float* g_rgb,
                    const float* g_sigma, float* g_params, float* g_x, float* g_d, void* workspace,
                    nr_stream_t stream) {
    MlpPlan p;
    if (!plan_or_error(cfg, &p)) return NR_EARG;
    NR_REQUIRE(packed && params && x && rgb && sigma && saved && g_rgb && g_sigma && g_params && workspace && M >= 0,
               "nr_mlp_backward: null pointer");
    NR_REQUIRE(!g_d || (d && p.use_vd), "nr_mlp_backward: g_d needs d and use_view_dirs");
    const hipStream_t s = static_cast<hipStream_t>(stream);
    if (M == 0) {
        hipMemsetAsync(g_params, 0, sizeof(float) * p.param_count, s);
        return check_launch("nr_mlp_backward");
    }
    const MlpSizes z = make_sizes(p, M);
    char* ws = static_cast<char*>(workspace);

    BwdArgs b;
    std::memset(&b, 0, sizeof(b));
    b.packed = static_cast<const char*>(packed);
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
    b.ws = ws;
    b.M = M;
    b.tiles = z.tiles;
    b.L = p.L;
    b.Ld = p.Ld;
    b.n_layers = p.n_layers;
    b.skips = p.skips;
    for (int l = 0; l < p.n_lin; ++l) {
        b.pkT[l] = p.lin[l].pk_bwd;
        b.NB[l] = p.lin[l].NB;
    }
    b.sig_w = p.sig_w;
    b.rgb_w = p.rgb_w;
    b.mask_off = z.mask_off;
    b.n_mask = p.n_mask;
    for (int t = 0; t < p.n_ws; ++t) b.ws_off[t] = z.ws_off[t];
    b.ws_feat = p.ws_feat;
    b.ws_dir = p.ws_dir;
    b.ws_heads = p.ws_heads;
    int rc = p.prec == NR_PREC_BF16 ? launch_bwd<NR_PREC_BF16>(p, b, s) : launch_bwd<NR_PREC_FP32>(p, b, s);
    if (rc) return rc;

    // dW over all jobs, split into z.chunks sample chunks
    DwArgs w;
    std::memset(&w, 0, sizeof(w));
    w.saved = static_cast<const char*>(saved);
    w.ws = ws;
    w.slabs = reinterpret_cast<float*>(ws + z.slab_off);
    w.tiles = z.tiles;
    w.chunks = z.chunks;
    w.tiles_per_chunk = static_cast<int>(ceil_div_ll(z.tiles, z.chunks));
    w.n_jobs = p.n_jobs;
    w.slab_floats_per_chunk = p.slab_floats_per_chunk;
    int wg = 0;
    for (int j = 0; j < p.n_jobs; ++j) {
        const DwJob& jb = p.job[j];
        w.job_wg0[j] = wg;
        w.job_nbg[j] = (jb.NB + 3) / 4;
        w.job_sg[j] = w.job_nbg[j] * ((jb.KB + 3) / 4);
        wg += z.chunks * ((w.job_sg[j] + kWavesPerBlock - 1) / kWavesPerBlock);
        w.job_NB[j] = jb.NB;
        w.job_KB[j] = jb.KB;
        w.job_row0[j] = jb.dz_row0;
        w.job_nin[j] = jb.nin;
        w.job_dz_off[j] = z.ws_off[jb.dz_tensor];
        w.job_dz_F[j] = p.ws_F[jb.dz_tensor];
        for (int q = 0; q < jb.nin; ++q) {
            w.job_in_off[j][q] = z.saved_off[jb.in_tensor[q]];
            w.job_in_F[j][q] = p.sv_F[jb.in_tensor[q]];
            w.job_in_blocks[j][q] = jb.in_blocks[q];
        }
        w.job_slab[j] = jb.slab_off;
    }
    w.job_wg0[p.n_jobs] = wg;
    if (p.prec == NR_PREC_BF16)
        hipLaunchKernelGGL(mlp_dw_kernel<NR_PREC_BF16>, dim3(wg), dim3(64 * kWavesPerBlock), 0, s, w);
    else
        hipLaunchKernelGGL(mlp_dw_kernel<NR_PREC_FP32>, dim3(wg), dim3(64 * kWavesPerBlock), 0, s, w);
    NR_LAUNCH_CHECK("nr_mlp_backward (dW)");

    ReduceArgs r;
    std::memset(&r, 0, sizeof(r));
    r.slabs = w.slabs;
    r.g = g_params;
    r.param_count = p.param_count;
    r.chunks = z.chunks;
    r.slab_floats_per_chunk = p.slab_floats_per_chunk;
    r.n_jobs = p.n_jobs;
    for (int j = 0; j < p.n_jobs; ++j) {
        const DwJob& jb = p.job[j];
        if (jb.layer >= 0) {
            const LinearDesc& ld = p.lin[jb.layer];
            r.job_w_off[j] = ld.w_off;
            r.job_b_off[j] = ld.b_off;
            r.job_in[j] = ld.in;
            r.job_nseg[j] = ld.nseg;
            int blk = 0;
            for (int q = 0; q < ld.nseg; ++q) {
                r.job_seg_col0[j][q] = ld.seg[q].col0;
                r.job_seg_w[j][q] = ld.seg[q].width;
                r.job_seg_blk0[j][q] = blk;
                blk += ld.seg[q].blocks;
            }
        } else if (jb.layer == -1) {  // sigma head: W (1, hidden)
            r.job_w_off[j] = p.sig_w;
            r.job_b_off[j] = p.sig_b;
            r.job_in[j] = kHidden;
            r.job_nseg[j] = 1;
            r.job_seg_col0[j][0] = 0;
            r.job_seg_w[j][0] = kHidden;
            r.job_seg_blk0[j][0] = 0;
        } else {  // rgb head: W (3, hidden/2)
            r.job_w_off[j] = p.rgb_w;
            r.job_b_off[j] = p.rgb_b;
            r.job_in[j] = kHidden / 2;
            r.job_nseg[j] = 1;
            r.job_seg_col0[j][0] = 0;
            r.job_seg_w[j][0] = kHidden / 2;
            r.job_seg_blk0[j][0] = 0;
        }
        r.job_rows[j] = jb.rows;
        r.job_KB[j] = jb.KB;
        r.job_row0[j] = jb.dz_row0;
        r.job_slab[j] = jb.slab_off;
    }
    hipLaunchKernelGGL(mlp_dw_reduce_kernel, dim3(static_cast<unsigned>(ceil_div_ll(p.param_count, 256))), dim3(256),
                       0, s, r);
    NR_LAUNCH_CHECK("nr_mlp_backward (dW reduce)");
    return NR_OK;
}

}  // extern "C"
