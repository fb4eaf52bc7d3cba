// conv1 forward at rollout batch with the u8 patches kept as BYTES in LDS.
//
// gemm_kernel stages conv1's A operand (the u8 observation patches) as f32 in
// LDS: a 128x32 K-tile of A is 16.5 KB per buffer, so with B a block takes
// 42 KB and only 3 fit on a CU -- 768 resident blocks for the 1600 tiles of a
// 512-image launch, 2.08 rounds.  Here the A image is the raw bytes, [row i][k]
// with k contiguous exactly as the patch row sits in memory, so the commit is a
// plain 4-byte copy per staged word (no conversion, no transpose) and the block
// takes 17 KB.  A lane's MFMA fragment for k-steps kk and kk+2 (k = kk+khalf,
// kk+2+khalf) is two bytes of one ds_read_b32 of its row; v_cvt_f32_ubyte
// turns them into the exact integer values 0..255 the f32 MFMA consumes
// (identical operands, identical k-ordered chain => bit-identical to
// gemm_kernel).  The 1/255 normalisation stays in the epilogue (EpiAct).
#pragma once

#include "gemm.hpp"

namespace acmi {

template <int BK, class Src, class Epi>
__global__ __launch_bounds__(256) void conv1_fwd_u8_kernel(Src src, MatI<true> w, Epi epi, int I,
                                                           int K) {
  static_assert(sizeof(typename Src::elem_t) == 1, "u8 patch rows");
  constexpr int BM = 128, BN = 32;
  constexpr int RS = BK + 4;            // A row stride in bytes (odd word count: no bank conflicts)
  constexpr int SB = BN + 4;            // B row stride in floats
  constexpr int NA = BM * BK / 4 / 256;  // A words per thread
  constexpr int AW = BK / 4;             // words per A row
  static_assert(BK % 8 == 0 && NA >= 1 && (RS / 4) % 2 == 1, "tile");
  constexpr int NBF = (BK * BN / 4 + 255) / 256;  // B float4 per thread
  __shared__ __attribute__((aligned(16))) uint8_t a_img[2][BM * RS];
  __shared__ __attribute__((aligned(16))) float b_img[2][BK * SB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int i0 = blockIdx.x * BM;
  const int nk = (K + BK - 1) / BK;

  typename Src::R rowA[NA];
#pragma unroll
  for (int v = 0; v < NA; ++v) rowA[v] = src.row(i0 + (tid + 256 * v) / AW);
  constexpr int BJ = BN / 4;
  const int bj = (tid % BJ) * 4;

  StU8 ra[NA];
  StF4 rb[NBF];
  auto fetch = [&](int k0) {
    const int k = k0 + (tid % AW) * 4;  // same for every v (256 % AW == 0)
    const auto c = src.col(k);
#pragma unroll
    for (int v = 0; v < NA; ++v) ra[v] = src.stage(rowA[v], c, k < K);
#pragma unroll
    for (int v = 0; v < NBF; ++v) {
      const int t = tid + 256 * v;
      const bool on = t < BK * BJ;
      const int kb = k0 + t / BJ;
      rb[v] = w.stage(w.row(on ? kb : K), w.col(bj), on && kb < K);
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NA; ++v) {
      const int idx = tid + 256 * v;
      const int i = idx / AW, q = idx - i * AW;
      *reinterpret_cast<uint32_t*>(&a_img[buf][i * RS + 4 * q]) = ra[v].u;
    }
#pragma unroll
    for (int v = 0; v < NBF; ++v) {
      const int t = tid + 256 * v;
      if (t < BK * BJ) *reinterpret_cast<float4*>(&b_img[buf][(t / BJ) * SB + bj]) = finish(rb[v]);
    }
  };

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int arow = wave * 32 + (lane & 31);
  const int khalf = lane >> 5;
  const int col = lane & 31;
  const uint32_t sh0 = 8u * khalf, sh1 = 8u * (2 + khalf);

  if (nk > 0) {
    fetch(0);
    commit(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    fetch((kt + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t* As = a_img[cur] + arow * RS;
    const float* Bs = b_img[cur];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const uint32_t u = *reinterpret_cast<const uint32_t*>(As + kk);
      const float a0 = (float)((u >> sh0) & 255u), a1 = (float)((u >> sh1) & 255u);
      const float b0 = Bs[(kk + khalf) * SB + col], b1 = Bs[(kk + 2 + khalf) * SB + col];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) commit(cur ^ 1);
    __syncthreads();
  }
  f32x16 out[1][1];
  out[0][0] = acc;
  store_tile<1, 1>(epi, out, i0 + wave * 32, 0, lane, I, BN);
}

template <int BK, class Src, class Epi>
inline void launch_conv1_fwd_u8(const Src& src, const MatI<true>& w, const Epi& e, int I, int K,
                                hipStream_t s) {
  hipLaunchKernelGGL((conv1_fwd_u8_kernel<BK, Src, Epi>), dim3(cdiv(I, 128)), dim3(256), 0, s, src,
                     w, e, I, K);
}

}  // namespace acmi

namespace acmi {

// conv1 weight gradient  [P;1]^T d1  over the B*400 conv1 locations (split-K
// partials, EpiPartial [chunk][257][32], column sums = the bias gradient), the
// u8 patches again kept as bytes in LDS.  One block covers all 256 patch
// columns (4 waves x 64), so d1 is read once instead of once per 128-column
// tile, and a block takes 2 x (8.3 + 4.6) KB.  A lane's fragment A(k, i) is one
// byte of the [k][i] image (ds_read_u8 + v_cvt_f32_ubyte0); the k-ordered MFMA
// chain is gemm_kernel's, so the partials are bit-identical to it.
template <class Src>
__global__ __launch_bounds__(256) void conv1_wgrad_u8_kernel(Src src, const float* dy, int rows,
                                                             int k_chunk, EpiPartial epi) {
  static_assert(sizeof(typename Src::elem_t) == 1, "u8 patch rows");
  constexpr int BK = 32, NI = 256, NJ = 32;
  constexpr int RA = NI + 4;  // A image row stride (bytes)
  constexpr int SB = NJ + 4;  // B image row stride (floats)
  __shared__ __attribute__((aligned(16))) uint8_t a_img[2][BK * RA];
  __shared__ __attribute__((aligned(16))) float b_img[2][BK * SB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const int total = gridDim.x;
  const int xcd = b & 7, base8 = total >> 3, rem = total & 7;
  const int z = xcd * base8 + min(xcd, rem) + (b >> 3);  // chunk (XCD-contiguous)
  epi.z = z;
  const int kbeg = z * k_chunk, kend = min(rows, kbeg + k_chunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // A staging: 64 threads per k-row, 4 patch bytes each (one word), 4 rows per pass
  const int acol = (tid & 63) * 4;
  const typename Src::Cp ca = src.col(acol);
  // B staging: 8 threads per k-row (one float4 each), 32 rows per pass
  const int bcol = (tid & 7) * 4, brow = tid >> 3;
  StU8 ra[BK / 4];
  StF4 rb;
  auto fetch = [&](int k0) {
#pragma unroll
    for (int v = 0; v < BK / 4; ++v) {
      const int k = k0 + (tid >> 6) + 4 * v;
      ra[v] = src.stage(src.row(k), ca, k < kend);
    }
    const int k = k0 + brow;
    const bool ok = k < kend;
    rb = stage_f4(dy + (uint32_t)(ok ? k : 0) * (uint32_t)NJ + bcol, ok);
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int v = 0; v < BK / 4; ++v)
      *reinterpret_cast<uint32_t*>(&a_img[buf][((tid >> 6) + 4 * v) * RA + acol]) = ra[v].u;
    *reinterpret_cast<float4*>(&b_img[buf][brow * SB + bcol]) = rb;
  };

  f32x16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float csum = 0.f;
  const int khalf = lane >> 5, col = lane & 31;
  const int arow = wave * 64 + col;

  if (nk > 0) {
    fetch(kbeg);
    commit(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    fetch(kbeg + (kt + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t* As = a_img[cur];
    const float* Bs = b_img[cur];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int k = kk + khalf;
      const float a0 = (float)As[k * RA + arow], a1 = (float)As[k * RA + arow + 32];
      const float bb = Bs[k * SB + col];
      csum += bb;  // (stored by wave 0 only)
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bb, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bb, acc[1], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) commit(cur ^ 1);
    __syncthreads();
  }
  f32x16 out[2][1];
  out[0][0] = acc[0];
  out[1][0] = acc[1];
  store_tile<2, 1>(epi, out, wave * 64, 0, lane, NI, NJ);
  if (wave == 0) {
    const float t = csum + __shfl_xor(csum, 32);
    if (lane < 32) epi.colsum(lane, t);
  }
}

// chunks: whole rounds of the resident blocks (LDS: 2 x 12.9 KB per block)
inline void conv1_wgrad_u8_plan(long long rows, int* nchunk, int* chunk) {
  plan_rounds(rows, 1, 256 * std::min(8, 160 * 1024 / (2 * (32 * 260 + 32 * 36 * 4))), nchunk,
              chunk);
}

template <class Src>
inline void launch_conv1_wgrad_u8(const Src& src, const float* dy, int rows, int nchunk,
                                  int chunk, const EpiPartial& e, hipStream_t s) {
  hipLaunchKernelGGL((conv1_wgrad_u8_kernel<Src>), dim3(nchunk), dim3(256), 0, s, src, dy, rows,
                     chunk, e);
}

}  // namespace acmi
