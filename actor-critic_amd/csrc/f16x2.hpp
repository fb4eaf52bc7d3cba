// "f16x2" split operands: f32-accurate products on the f16 matrix cores at three
// MFMAs per 32x32x16 product tile (bf16x3 takes six).
//
// A tensor is scaled by a power of two s chosen from a bound of its magnitude
// (f16x2_scale: the bound lands below 2^14 < 65504), and every scaled value
// x s is split into h = f16_rn(x s) and l = f16_rn(x s - h) -- the subtraction is
// exact, so x s = h + l to 2^-22 relative (elements below the f16 normal range
// keep an absolute error <= 2^-25 in scaled units, < 2^-30 of the bound when the
// bound is tight to 2^9).  A product tile takes l*h + h*l + h*h on
// v_mfma_f32_32x32x16_f16 (every f16 product exact in f32; the dropped l*l is
// <= 2^-22 |a||b|) and the accumulator is multiplied by 1/(s_a s_b) -- exact --
// before it is used.  f32-class sums: the accumulation error (~sqrt(K) 2^-24)
// dominates the 2^-22 operand error.
//
// Bounds come from where the tensor is made: the exact max of a dX epilogue
// (gemm.hpp has_amax), the max |W| of a weight matrix, or a weight-derived
// bound of a ReLU activation (band.hpp band_bounds_kernel).
#pragma once

#include "split16.hpp"  // f32x2v, s16x4/8, ds_tr16

namespace acmi {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));

constexpr int F16X2_MAX_SCALE_EXP = 60;

// power of two putting a bound mx at < 2^14; 1 for a zero / non-finite bound.
// The exponent is capped at 2^60 so that the product of two scales (<= 2^120) and
// its reciprocal (>= 2^-120) stay finite normal floats: a bound below 2^-46 then
// loses precision gracefully (its scaled values sit below 2^14) instead of the
// scale overflowing to inf and the unscale 1/(s_a s_b) zeroing the product.
__device__ __forceinline__ float f16x2_scale(float mx) {
  if (!(mx > 0.f) || !(mx < 3.0e38f)) return 1.f;
  int e;
  (void)frexpf(mx, &e);  // mx < 2^e
  return ldexpf(1.f, min(14 - e, F16X2_MAX_SCALE_EXP));
}
// the scale of a published bound (common.hpp amax_read: all 64 lanes active)
__device__ __forceinline__ float f16x2_scale_of_bits(const unsigned* mx) {
  return f16x2_scale(amax_read(mx));
}

__device__ __forceinline__ uint32_t pk_f16(float a, float b) {
  const f32x2v v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2v));
}
// (a, b) * s = h + l (the residual as fma(x, s, -h): v_fma_mix_f32 reads h from
// the packed f16 register)
__device__ __forceinline__ void split2(float a, float b, float s, uint32_t& h, uint32_t& l) {
  h = pk_f16(a * s, b * s);
  const f16x2v hv = __builtin_bit_cast(f16x2v, h);
  l = pk_f16(fmaf(a, s, -(float)hv[0]), fmaf(b, s, -(float)hv[1]));
}
// eight consecutive values as their (h, l) fragments
__device__ __forceinline__ void split2x8(const float4& x0, const float4& x1, float s, f16x8& h, f16x8& l) {
  uint4 hh, ll;
  split2(x0.x, x0.y, s, hh.x, ll.x);
  split2(x0.z, x0.w, s, hh.y, ll.y);
  split2(x1.x, x1.y, s, hh.z, ll.z);
  split2(x1.z, x1.w, s, hh.w, ll.w);
  h = __builtin_bit_cast(f16x8, hh);
  l = __builtin_bit_cast(f16x8, ll);
}
__device__ __forceinline__ f16x8 cat8h(s16x4 a, s16x4 b) {
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(f16x8, v);
}
__device__ __forceinline__ f16x8 as_f16x8(const uint4& u) { return __builtin_bit_cast(f16x8, u); }

// eight u8 pixels n as the f16 SUBNORMALS n * 2^-24 (exact; one byte permute per
// two: the byte is the significand, the exponent field zero) -- the products'
// 2^-24 is taken out with the other operand's scale when they are stored
__device__ __forceinline__ f16x8 u8x8_to_f16(uint2 u) {
  const uint32_t w0 = __builtin_amdgcn_perm(0u, u.x, 0x0c010c00u), w1 = __builtin_amdgcn_perm(0u, u.x, 0x0c030c02u);
  const uint32_t w2 = __builtin_amdgcn_perm(0u, u.y, 0x0c010c00u), w3 = __builtin_amdgcn_perm(0u, u.y, 0x0c030c02u);
  return __builtin_bit_cast(f16x8, make_uint4(w0, w1, w2, w3));
}

// three-product f16x2 step on one accumulator: a = {h, l}, b = {h, l}
__device__ __forceinline__ f32x16 mfma_x2(const f16x8 (&a)[2], const f16x8 (&b)[2], f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], c, 0, 0, 0);
  return c;
}

// max |x| over n floats (a weight matrix) into *out (zeroed by the caller):
// grid-stride loads, one atomicMax per wave
static __global__ __launch_bounds__(256) void absmax_kernel(const float* x, long long n, unsigned* out) {
  float m = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    m = fmaxf(m, fabsf(x[i]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) amax_update(out, m);
}

}  // namespace acmi
