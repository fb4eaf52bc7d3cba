// PROBE ONLY (not in libacmi): measured no faster than gemm_kernel at rollout batch.
// Wave-split GEMM for the rollout-size forward convolutions (B = 512 images).
//
// At rollout batch the forward GEMMs are latency-bound, not MFMA-bound: conv3
// has 25,088 output rows, i.e. 196 blocks of 128 rows for 256 CUs, so every
// SIMD runs ONE wave whose K loop alternates a short MFMA burst (16 MFMAs per
// K-tile) with the staging round trip and a block barrier, ~50% MFMA busy at
// best.  Here a block's 4 waves split the K-tiles (wave q takes k-tiles
// q, q+WK, ...) of a small output tile (WM row groups of 32 x WTN*32 columns)
// and run them as independent pipelines: each wave stages its own k-tiles into
// its own LDS region (register prefetch of the next tile across the MFMAs, no
// block barrier inside the loop), so a conv3 launch becomes 784 blocks / 3136
// waves.  The WK partial accumulators of a row group are added in a fixed order
// (q = 0, 1, .., WK-1) through LDS at the end and the q = 0 wave runs the
// epilogue (same store_tile as gemm_kernel).  Deterministic; the k order inside
// a partial is the k-ordered MFMA chain of gemm_kernel.
//
// OpA: KCONTIG row source (RowsAsK<ConvRows<..>>), OpB: MatI (B[k][n] row-major).
#pragma once

#include "../../actor-critic_amd/csrc/gemm.hpp"

namespace acmi {

template <int WM, int WK, int WTN, int BK>
struct WsTile {
  static_assert(WM * WK == 4, "4 waves per block");
  static_assert(BK % 4 == 0 && (32 * BK / 4) % 64 == 0 && (BK * 32 * WTN / 4) % 64 == 0, "staging");
  static constexpr int BM = 32 * WM, BN = 32 * WTN;
  static constexpr int SA = 33;            // A image [k][i], i contiguous (+1 pad)
  static constexpr int SB = BN + 4;        // B image [k][j]
  static constexpr int WAVE_FLOATS = BK * SA + BK * SB;
  static constexpr int RED_FLOATS = 16 * WTN * 64;  // one wave's accumulators
  static constexpr int LDS_FLOATS =
      4 * WAVE_FLOATS > 4 * RED_FLOATS ? 4 * WAVE_FLOATS : 4 * RED_FLOATS;
};

template <int WM, int WK, int WTN, int BK, class OpA, class OpB, class Epi>
__global__ __launch_bounds__(256) void gemm_ws_kernel(OpA opA, OpB opB, Epi epi, int I, int J,
                                                      int K) {
  static_assert(OpA::KCONTIG && !OpB::KCONTIG, "A k-contiguous rows, B row-major [K][N]");
  using T = WsTile<WM, WK, WTN, BK>;
  constexpr int NA = 32 * BK / 4 / 64;        // A float4 slots per lane
  constexpr int NB = BK * T::BN / 4 / 64;     // B float4 slots per lane
  constexpr int AK = BK / 4;                  // A slots per row
  constexpr int BJ = T::BN / 4;               // B slots per k-row
  __shared__ __attribute__((aligned(16))) float lds[T::LDS_FLOATS];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int m = wave / WK, q = wave - (wave / WK) * WK;
  const int i0 = blockIdx.x * T::BM + 32 * m;
  const int j0 = blockIdx.y * T::BN;
  float* As = lds + wave * T::WAVE_FLOATS;
  float* Bs = As + BK * T::SA;

  typename OpA::R rowA[NA];
#pragma unroll
  for (int v = 0; v < NA; ++v) rowA[v] = opA.row(i0 + (lane + 64 * v) / AK);
  typename OpB::C colB[NB];
#pragma unroll
  for (int v = 0; v < NB; ++v) colB[v] = opB.col(j0 + ((lane + 64 * v) % BJ) * 4);

  typename OpA::St ra[NA];
  typename OpB::St rb[NB];
  auto fetch = [&](int k0) {
    const int ka = k0 + (lane % AK) * 4;  // same k for every v (64 % AK == 0)
    const auto ca = opA.col(ka);
#pragma unroll
    for (int v = 0; v < NA; ++v) ra[v] = opA.stage(rowA[v], ca, ka < K);
#pragma unroll
    for (int v = 0; v < NB; ++v) {
      const int k = k0 + (lane + 64 * v) / BJ;
      rb[v] = opB.stage(opB.row(k), colB[v], k < K);
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int v = 0; v < NA; ++v) {
      const int idx = lane + 64 * v;
      const int i = idx / AK, k = (idx - i * AK) * 4;
      const float4 x = finish(ra[v]);
      As[(k + 0) * T::SA + i] = x.x;
      As[(k + 1) * T::SA + i] = x.y;
      As[(k + 2) * T::SA + i] = x.z;
      As[(k + 3) * T::SA + i] = x.w;
    }
#pragma unroll
    for (int v = 0; v < NB; ++v) {
      const int idx = lane + 64 * v;
      const int k = idx / BJ, j = (idx - k * BJ) * 4;
      *reinterpret_cast<float4*>(Bs + k * T::SB + j) = finish(rb[v]);
    }
  };

  f32x16 acc[WTN];
#pragma unroll
  for (int t = 0; t < WTN; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  const int nk = (K + BK - 1) / BK;
  const int khalf = lane >> 5, col = lane & 31;
  if (q < nk) {
    fetch(q * BK);
    commit();
  }
  // the wave's LDS image is private: wave-level ordering suffices
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int kt = q; kt < nk; kt += WK) {
    fetch((kt + WK) * BK);  // past the end: clamped, zero-masked, never committed
    __builtin_amdgcn_sched_barrier(0);
    float a = As[khalf * T::SA + col], b[WTN];
#pragma unroll
    for (int t = 0; t < WTN; ++t) b[t] = Bs[khalf * T::SB + t * 32 + col];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float an = 0.f, bn[WTN];
      if (kk + 2 < BK) {
        an = As[(kk + 2 + khalf) * T::SA + col];
#pragma unroll
        for (int t = 0; t < WTN; ++t) bn[t] = Bs[(kk + 2 + khalf) * T::SB + t * 32 + col];
      }
#pragma unroll
      for (int t = 0; t < WTN; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b[t], acc[t], 0, 0, 0);
      if (kk + 2 < BK) {
        a = an;
#pragma unroll
        for (int t = 0; t < WTN; ++t) b[t] = bn[t];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (kt + WK < nk) commit();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }

  if constexpr (WK > 1) {
    __syncthreads();  // every wave is done with its staging image
    float* red = lds + wave * T::RED_FLOATS;
    if (q > 0) {
#pragma unroll
      for (int t = 0; t < WTN; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(t * 16 + r) * 64 + lane] = acc[t][r];
    }
    __syncthreads();
    if (q > 0) return;
#pragma unroll
    for (int p = 1; p < WK; ++p) {
      const float* o = lds + (wave + p) * T::RED_FLOATS;
#pragma unroll
      for (int t = 0; t < WTN; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] += o[(t * 16 + r) * 64 + lane];
    }
  }
  f32x16 out[1][WTN];
#pragma unroll
  for (int t = 0; t < WTN; ++t) out[0][t] = acc[t];
  store_tile<1, WTN>(epi, out, i0, j0, lane, I, J);
}

template <int WM, int WK, int WTN, int BK, class OpA, class OpB, class Epi>
inline void launch_gemm_ws(const OpA& a, const OpB& b, const Epi& e, int I, int J, int K,
                           hipStream_t s) {
  using T = WsTile<WM, WK, WTN, BK>;
  hipLaunchKernelGGL((gemm_ws_kernel<WM, WK, WTN, BK, OpA, OpB, Epi>),
                     dim3(cdiv(I, T::BM), cdiv(J, T::BN)), dim3(256), 0, s, a, b, e, I, J, K);
}

}  // namespace acmi
