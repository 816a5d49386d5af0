// MFMA fragment helpers for gfx950 (CDNA4).
//
// Two instructions carry the NeRF MLP:
//   v_mfma_f32_32x32x16_bf16 : D[32x32] += A[32x16] * B[16x32], bf16 in, f32 acc
//   v_mfma_f32_32x32x2_f32   : D[32x32] += A[32x2]  * B[2x32],  f32 in, f32 acc (exact fmaf chain)
// Lane maps (cdna_hip_programming.md §3):
//   bf16: lane l (r = l&31, h = l>>5) holds A[r][8h+j], B[8h+j][r], j = 0..7
//   f32 : lane l holds A[l&31][l>>5], B[l>>5][l&31]
//   C/D (both): col = l&31, row = (reg&3) + 8*(reg>>2) + 4*(l>>5), reg = 0..15
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

namespace nr {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Row of the 32x32 C/D tile held in accumulator register `reg` by lane half `h`.
__host__ __device__ constexpr int acc_row(int reg, int h) {
    return (reg & 3) + 8 * (reg >> 2) + 4 * h;
}

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Round-to-nearest-even f32 -> bf16 (hipcc lowers the cast to v_cvt_pk_bf16_f32).
__device__ __forceinline__ __bf16 to_bf16(float x) { return static_cast<__bf16>(x); }

__device__ __forceinline__ float bf16_to_f32(unsigned short u) {
    return __uint_as_float(static_cast<unsigned int>(u) << 16);
}

__device__ __forceinline__ unsigned short bf16_bits(float x) {
    __bf16 b = to_bf16(x);
    return __builtin_bit_cast(unsigned short, b);
}

}  // namespace nr
