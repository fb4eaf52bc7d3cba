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
#include "gemm3.hpp"

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

// bf16 form of conv1_fwd_u8_kernel (ACMI_GEMM_X3 mode).  The u8 pixels are
// exact in bf16, so only the weights take the three-way split (symred3.hpp):
// three v_mfma_f32_32x32x16_bf16 per 16 k (pixel x w_l, x w_m, x w_h), every
// product exact, f32 accumulation -- vs eight f32 MFMAs of twice the cycles.
// A stays bytes in LDS ([row][k], 40-byte rows: one conflict-free ds_read_b64
// gives a lane the 8 consecutive k of its row that the 32x32x16 operand map
// wants, converted with v_cvt_f32_ubyte + v_cvt_pk_bf16_f32); the 32x32 weight
// tile of each k-step is split at the commit into a [part][k][j] bf16 image
// (64-byte rows) read by ds_read_b64_tr_b16.  22 KB per block: the 1,600 tiles
// of a 512-image launch are resident at once (7 blocks per CU).
__device__ __forceinline__ bf16x8 u8x8_to_bf16(uint2 u) {
  uint32_t w[4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t x = h ? u.y : u.x;
    w[2 * h] = pk_bf16((float)(x & 255u), (float)((x >> 8) & 255u));
    w[2 * h + 1] = pk_bf16((float)((x >> 16) & 255u), (float)(x >> 24));
  }
  return __builtin_bit_cast(bf16x8, make_uint4(w[0], w[1], w[2], w[3]));
}

template <class Src, class Epi>
__global__ __launch_bounds__(256) void conv1_fwd_x3_kernel(Src src, MatI<true> w, Epi epi, int I,
                                                           int K) {
  static_assert(sizeof(typename Src::elem_t) == 1, "u8 patch rows");
  constexpr int BM = 128, BN = 32, BK = 32;
  constexpr int RS = BK + 8;             // A row stride in bytes (8-aligned, conflict-free b64 reads)
  constexpr int NA = BM * BK / 4 / 256;  // A words per thread
  constexpr int AW = BK / 4;             // words per A row
  constexpr int RB = BN * 2;             // B image row bytes
  constexpr int BPART = BK * RB;
  __shared__ __attribute__((aligned(16))) uint8_t a_img[2][BM * RS];
  __shared__ __attribute__((aligned(16))) char b_img[2][3 * BPART];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int i0 = blockIdx.x * BM;
  const int nk = (K + BK - 1) / BK;

  typename Src::R rowA[NA];
#pragma unroll
  for (int v = 0; v < NA; ++v) rowA[v] = src.row(i0 + (tid + 256 * v) / AW);
  const int bk = tid / (BN / 4), bj = (tid % (BN / 4)) * 4;  // one weight float4 per thread

  StU8 ra[NA];
  StF4 rb;
  auto fetch = [&](int k0) {
    const int k = k0 + (tid % AW) * 4;
    const auto c = src.col(k);
#pragma unroll
    for (int v = 0; v < NA; ++v) ra[v] = src.stage(rowA[v], c, k < K);
    const int kb = k0 + bk;
    rb = w.stage(w.row(kb), w.col(bj), kb < K);
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NA; ++v) {
      const int idx = tid + 256 * v;
      const int i = idx / AW, q = idx - i * AW;
      *reinterpret_cast<uint32_t*>(&a_img[buf][i * RS + 4 * q]) = ra[v].u;
    }
    const float4 x = finish(rb);
    uint2 h, m, l;
    split3(x.x, x.y, h.x, m.x, l.x);
    split3(x.z, x.w, h.y, m.y, l.y);
    char* bs = b_img[buf] + bk * RB + 2 * bj;
    *reinterpret_cast<uint2*>(bs) = h;
    *reinterpret_cast<uint2*>(bs + BPART) = m;
    *reinterpret_cast<uint2*>(bs + 2 * BPART) = l;
  };

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int arow = wave * 32 + (lane & 31);
  const int kh = lane >> 5;
  // tr-read address of the weight fragment (rows 8kh + q, columns 16g + 4p)
  const int q = (lane >> 2) & 3, p = lane & 3, g = (lane >> 4) & 1;
  const int boff = (8 * kh + q) * RB + 8 * (4 * g + p);

  if (nk > 0) {
    fetch(0);
    commit(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    fetch((kt + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t* As = a_img[cur] + arow * RS + 8 * kh;
    const char* Bs = b_img[cur];
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const bf16x8 a = u8x8_to_bf16(*reinterpret_cast<const uint2*>(As + 16 * ks));
      bf16x8 b[3];
#pragma unroll
      for (int pt = 0; pt < 3; ++pt) {
        const char* bp = Bs + pt * BPART + 16 * ks * RB + boff;
        b[pt] = cat8(ds_tr16(bp), ds_tr16(bp + 4 * RB));
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[0], acc, 0, 0, 0);
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
  if (g_gemm_mode == ACMI_GEMM_X3)
    hipLaunchKernelGGL((conv1_fwd_x3_kernel<Src, Epi>), dim3(cdiv(I, 128)), dim3(256), 0, s, src, w,
                       e, I, K);
  else
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

// bf16 form of conv1_wgrad_u8_kernel (ACMI_GEMM_X3 mode), computed transposed:
// C^T[j][i] = sum_k d1(k, j) P(k, i), A = d1 (three-way split at the commit,
// [part][k][j] image), B = the u8 patches converted to bf16 at the commit
// (exact) into a [k][i] image (512-byte rows, slots swizzled as gemm3's
// sw_rows), both read by ds_read_b64_tr_b16.  Three MFMAs per 32x32 tile and 16
// k, every product exact.  Each wave owns all 32 channels x 64 patch columns;
// the tile is stored transposed into the same [chunk][257][32] partials (a
// lane's 4 consecutive j of one i are one float4).  The bias gradient (row 256)
// is summed in f32 from the staged d1 at the commit.  44 KB per block.
template <class Src>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
void conv1_wgrad_x3_kernel(Src src, const float* dy, int rows, int k_chunk, EpiPartial epi) {
  static_assert(sizeof(typename Src::elem_t) == 1, "u8 patch rows");
  constexpr int BK = 32, NI = 256, NJ = 32;
  constexpr int RA = NJ * 2;        // d1 image row bytes
  constexpr int APART = BK * RA;    // 2 KB
  constexpr int RB = NI * 2;        // patch image row bytes
  constexpr int BUF = 3 * APART + BK * RB;  // 6 KB + 16 KB
  __shared__ __attribute__((aligned(16))) char img[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const int total = gridDim.x;
  const int xcd = b & 7, base8 = total >> 3, rem = total & 7;
  const int z = xcd * base8 + min(xcd, rem) + (b >> 3);  // chunk (XCD-contiguous)
  epi.z = z;
  const int kbeg = z * k_chunk, kend = min(rows, kbeg + k_chunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // patch staging: 64 threads per k-row, one word (4 bytes) each, 4 rows per pass
  const int pcol = (tid & 63) * 4;
  const typename Src::Cp cp = src.col(pcol);
  // d1 staging: 8 threads per k-row (one float4 each), 32 rows
  const int dcol = (tid & 7) * 4, drow = tid >> 3;
  StU8 rp[BK / 4];
  StF4 rd;
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
  auto fetch = [&](int k0) {
#pragma unroll
    for (int v = 0; v < BK / 4; ++v) {
      const int k = k0 + (tid >> 6) + 4 * v;
      rp[v] = src.stage(src.row(k), cp, k < kend);
    }
    const int k = k0 + drow;
    const bool ok = k < kend;
    rd = stage_f4(dy + (uint32_t)(ok ? k : 0) * (uint32_t)NJ + dcol, ok);
  };
  auto commit = [&](int buf) {
    char* s = img + buf * BUF;
    uint2 h, m, l;
    csum[0] += rd.x;
    csum[1] += rd.y;
    csum[2] += rd.z;
    csum[3] += rd.w;
    split3(rd.x, rd.y, h.x, m.x, l.x);
    split3(rd.z, rd.w, h.y, m.y, l.y);
    char* ds = s + drow * RA + 2 * dcol;
    *reinterpret_cast<uint2*>(ds) = h;
    *reinterpret_cast<uint2*>(ds + APART) = m;
    *reinterpret_cast<uint2*>(ds + 2 * APART) = l;
#pragma unroll
    for (int v = 0; v < BK / 4; ++v) {
      const int k = (tid >> 6) + 4 * v;
      const uint32_t u = rp[v].u;
      const uint2 pb = make_uint2(pk_bf16((float)(u & 255u), (float)((u >> 8) & 255u)),
                                  pk_bf16((float)((u >> 16) & 255u), (float)(u >> 24)));
      *reinterpret_cast<uint2*>(s + 3 * APART + k * RB + 8 * sw_rows<RB>(pcol >> 2, k)) = pb;
    }
  };

  f32x16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const int q = (lane >> 2) & 3, p = lane & 3, g = (lane >> 4) & 1, kh = lane >> 5;
  const int aoff = (8 * kh + q) * RA + 8 * (4 * g + p);  // d1 fragment (32 j)
  int boff[2][2];                                          // [k-step][i block]
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k = 16 * ks + 8 * kh + q;
      boff[ks][t] = 3 * APART + k * RB + 8 * sw_rows<RB>(((wave * 64 + 32 * t) >> 2) + 4 * g + p, k);
    }

  if (nk > 0) {
    fetch(kbeg);
    commit(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    fetch(kbeg + (kt + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);
    const char* s = img + cur * BUF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[3];
#pragma unroll
      for (int pt = 0; pt < 3; ++pt) {
        const char* ap = s + pt * APART + 16 * ks * RA + aoff;
        a[pt] = cat8(ds_tr16(ap), ds_tr16(ap + 4 * RA));
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bf16x8 bb = cat8(ds_tr16(s + boff[ks][t]), ds_tr16(s + boff[ks][t] + 4 * RB));
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], bb, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bb, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb, acc[t], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) commit(cur ^ 1);
    __syncthreads();
  }
  // bias gradient: the 32 k-row threads of each column group through LDS
  float* cs = reinterpret_cast<float*>(img);
#pragma unroll
  for (int e = 0; e < 4; ++e) cs[drow * NJ + dcol + e] = csum[e];
  __syncthreads();
  if (wave == 0 && lane < NJ) {
    float t = 0.f;
    for (int r = 0; r < 32; ++r) t += cs[r * NJ + lane];
    epi.colsum(lane, t);
  }
  // acc[t][r]: j = (r&3) + 8(r>>2) + 4kh, i = wave*64 + 32t + (lane&31) -> part[z][i][j..j+3]
  float* out = epi.part + (long long)z * (NI + 1) * NJ;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int i = wave * 64 + 32 * t + (lane & 31);
#pragma unroll
    for (int gq = 0; gq < 4; ++gq)
      *reinterpret_cast<float4*>(out + i * NJ + 8 * gq + 4 * kh) =
          make_float4(acc[t][4 * gq], acc[t][4 * gq + 1], acc[t][4 * gq + 2], acc[t][4 * gq + 3]);
  }
}

// chunks: whole rounds of the resident blocks (LDS: f32 kernel 2 x 12.9 KB per
// block, bf16 kernel 44 KB)
inline void conv1_wgrad_u8_plan(long long rows, int* nchunk, int* chunk, int mode = g_gemm_mode) {
  const int lds = mode == ACMI_GEMM_X3 ? 2 * (3 * 32 * 64 + 32 * 512) : 2 * (32 * 260 + 32 * 36 * 4);
  plan_rounds(rows, 1, 256 * std::min(8, 160 * 1024 / lds), nchunk, chunk);
}

template <class Src>
inline void launch_conv1_wgrad_u8(const Src& src, const float* dy, int rows, int nchunk,
                                  int chunk, const EpiPartial& e, hipStream_t s) {
  if (g_gemm_mode == ACMI_GEMM_X3)
    hipLaunchKernelGGL((conv1_wgrad_x3_kernel<Src>), dim3(nchunk), dim3(256), 0, s, src, dy, rows,
                       chunk, e);
  else
    hipLaunchKernelGGL((conv1_wgrad_u8_kernel<Src>), dim3(nchunk), dim3(256), 0, s, src, dy, rows,
                       chunk, e);
}

}  // namespace acmi
