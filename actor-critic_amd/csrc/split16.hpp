// 16-bit split-operand primitives for the f32-accurate products on the
// 16-bit matrix cores: bf16x3 (three bf16 terms per value, six MFMAs per
// product; the arithmetic is described in symred3.hpp) -- the packed types,
// the split, the transposed LDS fragment read and the six-MFMA step.  The
// f16x2 form (two scaled f16 terms, three MFMAs) builds on these in f16x2.hpp.
#pragma once

#include "gemm.hpp"  // f32x16, common.hpp

namespace acmi {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

// (a, b) -> packed bf16 pair, round-to-nearest-even (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const f32x2v v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
}

// three-term split of the pair (a, b): h + m + l == (a, b) to 2^-24 relative
__device__ __forceinline__ void split3(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = pk_bf16(a, b);
  const float ra = a - __uint_as_float(h << 16);
  const float rb = b - __uint_as_float(h & 0xffff0000u);
  m = pk_bf16(ra, rb);
  const float sa = ra - __uint_as_float(m << 16);
  const float sb = rb - __uint_as_float(m & 0xffff0000u);
  l = pk_bf16(sa, sb);
}

__device__ __forceinline__ s16x4 ds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat8(s16x4 a, s16x4 b) {
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// six-product bf16x3 step on one accumulator
__device__ __forceinline__ f32x16 mfma_x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
  return c;
}

}  // namespace acmi
