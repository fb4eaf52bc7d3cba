// Shared device/host helpers for libacmi (MI355X / gfx950 only).
//
// Everything here is stream-ordered and allocation-free: entry points take
// caller-owned device buffers and a hipStream_t, never synchronise, and report
// errors through an int status + acmi_last_error() (see include/acmi.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/acmi.h"

namespace acmi {

// ---------------------------------------------------------------------------
// error reporting (host)
// ---------------------------------------------------------------------------
void set_error(const char* fmt, ...);

#define ACMI_REQUIRE(cond, code, ...)        \
  do {                                       \
    if (!(cond)) {                           \
      ::acmi::set_error(__VA_ARGS__);        \
      return (code);                         \
    }                                        \
  } while (0)

#define ACMI_LAUNCH_CHECK(what)                                              \
  do {                                                                       \
    hipError_t e_ = hipGetLastError();                                       \
    if (e_ != hipSuccess) {                                                  \
      ::acmi::set_error("%s: HIP launch failed: %s", what,                   \
                        hipGetErrorString(e_));                              \
      return ACMI_ERR_HIP;                                                   \
    }                                                                        \
  } while (0)

// ---------------------------------------------------------------------------
// fixed-order sum of p[c * stride], c = 0..n-1, with 8 loads in flight: the
// loads of a group are issued before its (sequential, in-order) adds; a
// missing tail element reads p[0] and is multiplied by 0 (no branch, no
// select on a loaded value)
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T chunk_sum(const T* p, int n, long long stride) {
  T s = 0;
  for (int c0 = 0; c0 < n; c0 += 8) {
    T v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(c0 + u < n ? (long long)(c0 + u) : 0LL) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += (c0 + u < n) ? v[u] : T(0);
  }
  return s;
}

// ---------------------------------------------------------------------------
// counter-based hashing (bit-identical restatement in oracle/oracle.py:mix32)
// lowbias32 finaliser (C. Wellons); all arithmetic mod 2^32.
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// key of a 4-field counter; the fields are folded one at a time
__host__ __device__ __forceinline__ uint32_t key4(uint32_t a, uint32_t b,
                                                 uint32_t c, uint32_t d) {
  uint32_t h = mix32(a ^ 0x9e3779b9U);
  h = mix32(h ^ b);
  h = mix32(h ^ c);
  h = mix32(h ^ d);
  return h;
}

// uniform in [0, 1) with 24 random bits, exactly representable in f32
__host__ __device__ __forceinline__ float u01(uint32_t h) {
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------------------
// wave helpers (wave64)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Published maxima (the f16x2 operand scales, f16x2.hpp): a bound m >= 0 lives
// in kAmaxSlots words kAmaxStride words apart (kAmaxWords in all, zeroed before
// the producing launch; non-negative floats order as their bits); block b
// publishes into slot b % 64 (an atomicMax only when m exceeds the value already
// there), and a consumer wave reads the 64 slots one per lane and takes their max
// (every lane of the wave must be active).  scripts/probes/amax_probe.hip, a
// 10240 x 512 float4 stream (20480 waves, 8.4 us alone): one publication per wave
// into ONE word 238 us (check first: 162; one per block: 55), into 64 adjacent
// words 104 (one cache line), into 64 words 256 B apart 15.9, one per block into
// those 12.0; reading them lane-parallel in 2048 blocks 2.9 us against 2.3 for
// one word.
constexpr int kAmaxSlots = 64, kAmaxStride = 64, kAmaxWords = kAmaxSlots * kAmaxStride;
__device__ __forceinline__ void amax_update(unsigned* p, float m) {
  unsigned* q = p + kAmaxStride * ((blockIdx.x + 7 * blockIdx.y) & (kAmaxSlots - 1));
  const unsigned v = __float_as_uint(m);
  if (v > __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(q, v);
}
__device__ __forceinline__ float amax_read(const unsigned* p) {
  return wave_max(__uint_as_float(p[kAmaxStride * (threadIdx.x & 63)]));
}

// GEMM arithmetic mode (ACMI_GEMM_X3 / ACMI_GEMM_F32, acmi_set_gemm_mode; net.hip)
// (the calling thread's mode for the current entry point: its net's or the process default)
extern thread_local int g_gemm_mode;

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// afactor_u8.hip: exact-integer conv1 A factor on the i8 matrix cores
long long conv1_afactor_ws_ints(long long rows);
// d1 != nullptr (bf16x3 mode): the conv1 weight gradient's per-chunk partials
// [chunk][257][32] are computed in the same pass (*wpart_out, in ws;
// conv1_afactor_fused_chunks chunks)
int conv1_afactor_u8(const uint8_t* obs, long long img_stride, int B, float* astat, int* ws,
                     long long ws_ints, hipStream_t s, const float* d1, float** wpart_out,
                     const unsigned* d1max);
int conv1_afactor_fused_chunks(long long rows);

}  // namespace acmi
