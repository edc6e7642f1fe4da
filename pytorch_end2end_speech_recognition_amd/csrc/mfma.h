// MFMA fragment helpers for gfx950 (wave64).
//   bf16 path: v_mfma_f32_16x16x32_bf16  (lane l: A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15])
//   f32  path: v_mfma_f32_16x16x4_f32    (lane l: A[l&15][l>>4],      B[l>>4][l&15])
//   C/D (both): col = l&15, row = 4*(l>>4) + r, r = 0..3
#pragma once
#include "common.h"

namespace asr {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 mfma_f32(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 as_bf16x8(const u16x8& v) {
  return __builtin_bit_cast(bf16x8, v);
}

// 8 consecutive f32 -> packed bf16x8 (round to nearest even).
__device__ __forceinline__ bf16x8 cvt8(const float* p) {
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(p[j]);
  return as_bf16x8(r);
}

__device__ __forceinline__ bf16x8 load_bf16x8_from_f32(const float* p) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  float t[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return cvt8(t);
}

__device__ __forceinline__ bf16x8 load_bf16x8(const uint16_t* p) {
  return as_bf16x8(*reinterpret_cast<const u16x8*>(p));
}

}  // namespace asr
