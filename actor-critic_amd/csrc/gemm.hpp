// LDS-tiled f32-input MFMA GEMM engine for gfx950 with pluggable operands.
//
//   C[i][j] = sum_k A(k, i) * B(k, j)
//
// Every GEMM-shaped op on the A2C/ACKTR path is an instance of this kernel:
//   * conv forward (implicit im2col, u8/255 fused for conv1)       RowsAsK
//   * conv input-gradient (transposed conv as a per-stride-phase gather)
//   * fc forward / input-gradient
//   * weight gradient fused with the K-FAC A-factor: [P;1]^T [P | dY | 1]
//     over the huge row dimension, split over blockIdx.z into per-chunk
//     partials reduced later in a fixed order (deterministic, no atomics)
//   * K-FAC G-factors and the natural-gradient preconditioning products.
//
// Math is exact f32: v_mfma_f32_32x32x2_f32 is a k-ordered f32 fmaf chain
// (cdna_hip_programming.md §3 "FP32-input MFMA"); fp32 is the reference's
// dtype.  Block = 256 threads = 4 waves; each wave owns a
// (32*WTM) x (32*WTN) sub-tile held in WTM*WTN 16-register accumulators.
//
// Operand concept (template parameter Op):
//   static constexpr bool KCONTIG;   // load4 returns 4 consecutive k (true)
//                                    // or 4 consecutive i/j (false)
//   __device__ float4 load4(int k, int i) const;   // zero outside bounds
// LDS images are [k][i] for both operands so the MFMA fragment read
// (lane l: row k = l>>5, col i = l&31) is one conflict-free ds_read_b32 per
// operand per k-step.  K-contiguous operands are written transposed with a
// row stride == 1 (mod 32) (conflict-free scatter), i-contiguous ones with a
// 16-byte aligned stride (ds_write_b128).
#pragma once

#include "common.hpp"

namespace acmi {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// exact u8 / 255.0f (one rounding), verified exhaustively for 0..255
__device__ __forceinline__ float u8norm(uint32_t u) {
  const float x = (float)u;
  const float inv = 1.0f / 255.0f;
  const float q = x * inv;
  const float r = __builtin_fmaf(-q, 255.0f, x);
  return __builtin_fmaf(r, inv, q);
}

// ---------------------------------------------------------------------------
// Row sources: get4(r, c) returns elements c..c+3 of logical row r.
// ---------------------------------------------------------------------------

// Patches of NHWC images for a VALID conv; row r = (img, oh, ow),
// column c = (kh, kw, ch) with ch fastest (== HWIO flatten == TF
// extract_image_patches order).  T = uint8_t normalises by 1/255.
template <typename T, int H, int W, int C, int KH, int KW, int S>
struct ConvRows {
  static constexpr int OH = (H - KH) / S + 1;
  static constexpr int OW = (W - KW) / S + 1;
  static constexpr int L = OH * OW;
  static constexpr int COLS = KH * KW * C;
  static_assert(C % 4 == 0, "channel runs must hold float4");
  const T* x;
  long long img_stride;  // elements of T between images
  int rows;              // images * L

  __device__ __forceinline__ float4 get4(int r, int c) const {
    if (r >= rows || c >= COLS) return f4zero();
    const int img = r / L;
    const int p = r - img * L;
    const int oh = p / OW;
    const int ow = p - oh * OW;
    const int kh = c / (KW * C);
    const int rem = c - kh * (KW * C);
    const int kw = rem / C;
    const int ch = rem - kw * C;
    const T* src = x + (long long)img * img_stride +
                   ((oh * S + kh) * W + (ow * S + kw)) * C + ch;
    if constexpr (sizeof(T) == 1) {
      const uint32_t u = *reinterpret_cast<const uint32_t*>(src);
      return make_float4(u8norm(u & 255u), u8norm((u >> 8) & 255u),
                         u8norm((u >> 16) & 255u), u8norm(u >> 24));
    } else {
      return *reinterpret_cast<const float4*>(src);
    }
  }
};

// Dense row-major [rows][cols] with leading dimension ld (ld % 4 == 0).
struct DenseRows {
  const float* x;
  int ld;
  int rows;
  int cols;  // multiple of 4 or rows zero-padded to ld
  __device__ __forceinline__ float4 get4(int r, int c) const {
    if (r >= rows || c >= cols) return f4zero();
    return *reinterpret_cast<const float4*>(x + (long long)r * ld + c);
  }
};

// Gradient of a VALID conv w.r.t. its input, one stride phase (ph, pw) per
// blockIdx.z: row r = (img, ih', iw') -> input pixel (S*ih'+ph, S*iw'+pw);
// column c = (kh', kw', co) -> tap (ph+S*kh', pw+S*kw'), output pixel
// (ih'-kh', iw'-kw').  Only taps that hit the phase are enumerated, so the
// stride-2 conv2 gradient does no zero work except at the borders.
template <int IH, int IW, int KH, int KW, int S, int COUT>
struct ConvTRows {
  static constexpr int OH = (IH - KH) / S + 1;
  static constexpr int OW = (IW - KW) / S + 1;
  static_assert(IH % S == 0 && IW % S == 0 && KH % S == 0 && KW % S == 0,
                "phase decomposition needs divisible extents");
  static constexpr int PH = IH / S;   // phase grid extent
  static constexpr int PW = IW / S;
  static constexpr int KHP = KH / S;  // taps per phase
  static constexpr int KWP = KW / S;
  static constexpr int COLS = KHP * KWP * COUT;
  static constexpr int L = PH * PW;   // rows per image per phase
  static_assert(COUT % 4 == 0, "");
  const float* dy;  // [img][OH][OW][COUT]
  int rows;         // images * L

  __device__ __forceinline__ float4 get4(int r, int c) const {
    if (r >= rows || c >= COLS) return f4zero();
    const int img = r / L;
    const int p = r - img * L;
    const int ihp = p / PW;
    const int iwp = p - ihp * PW;
    const int khp = c / (KWP * COUT);
    const int rem = c - khp * (KWP * COUT);
    const int kwp = rem / COUT;
    const int co = rem - kwp * COUT;
    const int oh = ihp - khp;
    const int ow = iwp - kwp;
    if (oh < 0 || ow < 0 || oh >= OH || ow >= OW) return f4zero();
    return *reinterpret_cast<const float4*>(
        dy + (((long long)img * OH + oh) * OW + ow) * COUT + co);
  }
};

// ---------------------------------------------------------------------------
// Operands
// ---------------------------------------------------------------------------

// A(k, i) = src row i, column k   (forward-style; k contiguous)
template <class Src>
struct RowsAsK {
  static constexpr bool KCONTIG = true;
  Src src;
  __device__ __forceinline__ float4 load4(int k, int i) const { return src.get4(i, k); }
};

// A(k, i) = src row k, column i   (reduction-style; i contiguous)
template <class Src>
struct RowsAsI {
  static constexpr bool KCONTIG = false;
  Src src;
  __device__ __forceinline__ float4 load4(int k, int i) const { return src.get4(k, i); }
};

// B(k, j) over row k of [P | dY | 1]:  j < kp -> P(k, j) (kp = 0 skips P),
// kp <= j < kp + cout_pad -> dY(k, j-kp) (zero past cout), j == kp+cout_pad
// -> 1 (homogeneous column, only for rows k < rows).
template <class Src>
struct CatRowsI {
  static constexpr bool KCONTIG = false;
  Src src;
  int kp;
  const float* dy;
  int ldy;
  int cout;
  int cout_pad;  // multiple of 4
  int rows;
  __device__ __forceinline__ float4 load4(int k, int j) const {
    if (k >= rows) return f4zero();
    if (j < kp) return src.get4(k, j);
    const int jj = j - kp;
    if (jj < cout_pad) {
      const float* p = dy + (long long)k * ldy + jj;
      if (jj + 3 < cout) return *reinterpret_cast<const float4*>(p);
      float4 v = f4zero();
      if (jj + 0 < cout) v.x = p[0];
      if (jj + 1 < cout) v.y = p[1];
      if (jj + 2 < cout) v.z = p[2];
      return v;
    }
    if (jj == cout_pad) return make_float4(1.f, 0.f, 0.f, 0.f);
    return f4zero();
  }
};

// B(k, j) = M[k][j], row-major with leading dimension ld (dims K x N).
template <bool ALIGNED>
struct MatI {
  static constexpr bool KCONTIG = false;
  const float* m;
  int ld;
  int K;
  int N;
  __device__ __forceinline__ float4 load4(int k, int j) const {
    if (k >= K || j >= N) return f4zero();
    const float* p = m + (long long)k * ld + j;
    if (ALIGNED && j + 3 < N) return *reinterpret_cast<const float4*>(p);
    float4 v = f4zero();
    v.x = p[0];
    if (j + 1 < N) v.y = p[1];
    if (j + 2 < N) v.z = p[2];
    if (j + 3 < N) v.w = p[3];
    return v;
  }
};

// B(k, j) = M[j][k]  (transposed access; k contiguous; dims K x N; ld%4==0)
struct MatTK {
  static constexpr bool KCONTIG = true;
  const float* m;
  int ld;
  int K;  // multiple of 4
  int N;
  __device__ __forceinline__ float4 load4(int k, int j) const {
    if (k >= K || j >= N) return f4zero();
    return *reinterpret_cast<const float4*>(m + (long long)j * ld + k);
  }
};

// A(k, i) = M[i][k]  (transposed access, any ld/alignment; dims K x N)
struct MatTKu {
  static constexpr bool KCONTIG = true;
  const float* m;
  int ld;
  int K;
  int N;
  __device__ __forceinline__ float4 load4(int k, int j) const {
    if (j >= N || k >= K) return f4zero();
    const float* p = m + (long long)j * ld + k;
    float4 v = f4zero();
    v.x = p[0];
    if (k + 1 < K) v.y = p[1];
    if (k + 2 < K) v.z = p[2];
    if (k + 3 < K) v.w = p[3];
    return v;
  }
};

// Conv weight as the B operand of the input gradient, one stride phase per
// blockIdx.z:  B(k = (kh',kw',co), j = ci) = W[ph+S*kh'][pw+S*kw'][ci][co].
template <int KH, int KW, int S, int CIN, int COUT>
struct ConvTWeights {
  static constexpr bool KCONTIG = true;
  static constexpr int KHP = KH / S;
  static constexpr int KWP = KW / S;
  static constexpr int K = KHP * KWP * COUT;
  const float* w;  // HWIO
  __device__ __forceinline__ float4 load4(int k, int j) const {
    if (k >= K || j >= CIN) return f4zero();
    const int ph = blockIdx.z / S;
    const int pw = blockIdx.z - ph * S;
    const int khp = k / (KWP * COUT);
    const int rem = k - khp * (KWP * COUT);
    const int kwp = rem / COUT;
    const int co = rem - kwp * COUT;
    const int kh = ph + S * khp;
    const int kw = pw + S * kwp;
    return *reinterpret_cast<const float4*>(w + ((kh * KW + kw) * CIN + j) * COUT + co);
  }
};

// ---------------------------------------------------------------------------
// The kernel
// ---------------------------------------------------------------------------
template <int BM, int BN, int BK, int WTM, int WTN>
struct Tile {
  static constexpr int WAVES_M = BM / (32 * WTM);
  static constexpr int WAVES_N = BN / (32 * WTN);
  static_assert(WAVES_M * WAVES_N == 4, "4 waves per block");
  static_assert(BK % 2 == 0 && BK % 4 == 0, "");
  static_assert((BM * BK / 4) % 256 == 0 && (BN * BK / 4) % 256 == 0,
                "staging must split evenly over 256 threads");
};

// SPLITK: blockIdx.z selects the k-chunk [z*k_chunk, min(K, (z+1)*k_chunk))
// (k_chunk % BK == 0); otherwise the full K range and operands/epilogues
// may use blockIdx.z for their own purposes (stride phases).
// COLSUM: blocks with blockIdx.x == 0 also return sum_k B(k, j) through
// epi.colsum(j, v) (the homogeneous row of [P;1]^T [..]).
template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM,
          class OpA, class OpB, class Epi>
__global__ __launch_bounds__(256) void gemm_kernel(OpA opA, OpB opB, Epi epi,
                                                   int I, int J, int K,
                                                   int k_chunk) {
  using TL = Tile<BM, BN, BK, WTM, WTN>;
  constexpr int SA = OpA::KCONTIG ? BM + 1 : BM + 4;
  constexpr int SB = OpB::KCONTIG ? BN + 1 : BN + 4;
  constexpr int NA = BM * BK / 4 / 256;
  constexpr int NB = BN * BK / 4 / 256;
  constexpr int ABUF = BK * SA;
  constexpr int BBUF = BK * SB;
  __shared__ __attribute__((aligned(16))) float lds[2 * (ABUF + BBUF)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / TL::WAVES_N;
  const int wn = wave - wm * TL::WAVES_N;
  const int i0 = blockIdx.x * BM;
  const int j0 = blockIdx.y * BN;
  int kbeg = 0, kend = K;
  if constexpr (SPLITK) {
    kbeg = blockIdx.z * k_chunk;
    kend = min(K, kbeg + k_chunk);
  }
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  float4 ra[NA];
  float4 rb[NB];

  auto fetch = [&](int k0) {
#pragma unroll
    for (int v = 0; v < NA; ++v) {
      const int idx = tid + 256 * v;
      if constexpr (OpA::KCONTIG) {
        const int i = idx / (BK / 4);
        const int k = (idx - i * (BK / 4)) * 4;
        ra[v] = (k0 + k < kend) ? opA.load4(k0 + k, i0 + i) : f4zero();
      } else {
        const int k = idx / (BM / 4);
        const int i = (idx - k * (BM / 4)) * 4;
        ra[v] = (k0 + k < kend) ? opA.load4(k0 + k, i0 + i) : f4zero();
      }
    }
#pragma unroll
    for (int v = 0; v < NB; ++v) {
      const int idx = tid + 256 * v;
      if constexpr (OpB::KCONTIG) {
        const int j = idx / (BK / 4);
        const int k = (idx - j * (BK / 4)) * 4;
        rb[v] = (k0 + k < kend) ? opB.load4(k0 + k, j0 + j) : f4zero();
      } else {
        const int k = idx / (BN / 4);
        const int j = (idx - k * (BN / 4)) * 4;
        rb[v] = (k0 + k < kend) ? opB.load4(k0 + k, j0 + j) : f4zero();
      }
    }
  };

  auto commit = [&](int buf) {
    float* As = lds + buf * ABUF;
    float* Bs = lds + 2 * ABUF + buf * BBUF;
#pragma unroll
    for (int v = 0; v < NA; ++v) {
      const int idx = tid + 256 * v;
      if constexpr (OpA::KCONTIG) {
        const int i = idx / (BK / 4);
        const int k = (idx - i * (BK / 4)) * 4;
        As[(k + 0) * SA + i] = ra[v].x;
        As[(k + 1) * SA + i] = ra[v].y;
        As[(k + 2) * SA + i] = ra[v].z;
        As[(k + 3) * SA + i] = ra[v].w;
      } else {
        const int k = idx / (BM / 4);
        const int i = (idx - k * (BM / 4)) * 4;
        *reinterpret_cast<float4*>(As + k * SA + i) = ra[v];
      }
    }
#pragma unroll
    for (int v = 0; v < NB; ++v) {
      const int idx = tid + 256 * v;
      if constexpr (OpB::KCONTIG) {
        const int j = idx / (BK / 4);
        const int k = (idx - j * (BK / 4)) * 4;
        Bs[(k + 0) * SB + j] = rb[v].x;
        Bs[(k + 1) * SB + j] = rb[v].y;
        Bs[(k + 2) * SB + j] = rb[v].z;
        Bs[(k + 3) * SB + j] = rb[v].w;
      } else {
        const int k = idx / (BN / 4);
        const int j = (idx - k * (BN / 4)) * 4;
        *reinterpret_cast<float4*>(Bs + k * SB + j) = rb[v];
      }
    }
  };

  f32x16 acc[WTM][WTN];
#pragma unroll
  for (int a = 0; a < WTM; ++a)
#pragma unroll
    for (int b = 0; b < WTN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  float csum = 0.f;
  const bool do_colsum = COLSUM && blockIdx.x == 0 && tid < BN;

  if (nk > 0) {
    fetch(kbeg);
    commit(0);
  }
  __syncthreads();

  const int arow = wm * WTM * 32 + (lane & 31);
  const int brow = wn * WTN * 32 + (lane & 31);
  const int khalf = lane >> 5;

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) fetch(kbeg + (kt + 1) * BK);
    const float* As = lds + cur * ABUF;
    const float* Bs = lds + 2 * ABUF + cur * BBUF;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a[WTM], b[WTN];
#pragma unroll
      for (int tm = 0; tm < WTM; ++tm) a[tm] = As[(kk + khalf) * SA + arow + tm * 32];
#pragma unroll
      for (int tn = 0; tn < WTN; ++tn) b[tn] = Bs[(kk + khalf) * SB + brow + tn * 32];
#pragma unroll
      for (int tm = 0; tm < WTM; ++tm)
#pragma unroll
        for (int tn = 0; tn < WTN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm], b[tn], acc[tm][tn], 0, 0, 0);
    }
    if constexpr (COLSUM) {
      if (do_colsum) {
#pragma unroll 8
        for (int kk = 0; kk < BK; ++kk) csum += Bs[kk * SB + tid];
      }
    }
    if (kt + 1 < nk) commit(cur ^ 1);
    __syncthreads();
  }

  // epilogue: acc[tm][tn][r] -> C[i][j],  j = lane&31 (+tile),
  // i = (r&3) + 8*(r>>2) + 4*(lane>>5) (+tile)   (gfx950 32x32 C/D map)
#pragma unroll
  for (int tm = 0; tm < WTM; ++tm)
#pragma unroll
    for (int tn = 0; tn < WTN; ++tn) {
      const int j = j0 + wn * WTN * 32 + tn * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + wm * WTM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
        if (i < I && j < J) epi(i, j, acc[tm][tn][r]);
      }
    }
  if constexpr (COLSUM) {
    if (do_colsum && j0 + tid < J) epi.colsum(j0 + tid, csum);
  }
}

// ---------------------------------------------------------------------------
// Epilogues
// ---------------------------------------------------------------------------
struct EpiStore {
  float* out;
  long long ld;
  __device__ __forceinline__ void operator()(int i, int j, float v) const {
    out[(long long)i * ld + j] = v;
  }
};

// out = relu?(v + bias[j])
struct EpiBiasAct {
  float* out;
  long long ld;
  const float* bias;
  int relu;
  __device__ __forceinline__ void operator()(int i, int j, float v) const {
    v += bias[j];
    if (relu) v = fmaxf(v, 0.f);
    out[(long long)i * ld + j] = v;
  }
};

// fc heads: j < A -> logits[i][j] = v + bpi[j]; j == A -> value[i] = v + bv
struct EpiHeads {
  float* logits;
  int ld;
  float* value;
  const float* bpi;
  const float* bv;
  int A;
  __device__ __forceinline__ void operator()(int i, int j, float v) const {
    if (j < A) logits[(long long)i * ld + j] = v + bpi[j];
    else if (value) value[i] = v + bv[0];
  }
};

// out = v * (act > 0)   (ReLU derivative from the stored post-ReLU output)
struct EpiReluGrad {
  float* out;
  const float* act;
  long long ld;
  __device__ __forceinline__ void operator()(int i, int j, float v) const {
    const long long o = (long long)i * ld + j;
    out[o] = act[o] > 0.f ? v : 0.f;
  }
};

// input-gradient of a strided conv, one phase per blockIdx.z: row i =
// (img, ih', iw') -> NHWC pixel (S*ih'+ph, S*iw'+pw); masked by ReLU'.
template <int IH, int IW, int S, int CIN>
struct EpiConvTPhase {
  float* out;
  const float* act;
  __device__ __forceinline__ void operator()(int i, int j, float v) const {
    constexpr int PH = IH / S, PW = IW / S, L = PH * PW;
    const int ph = blockIdx.z / S;
    const int pw = blockIdx.z - ph * S;
    const int img = i / L;
    const int p = i - img * L;
    const int ihp = p / PW;
    const int iwp = p - ihp * PW;
    const long long o =
        (((long long)img * IH + (S * ihp + ph)) * IW + (S * iwp + pw)) * CIN + j;
    out[o] = act[o] > 0.f ? v : 0.f;
  }
};

// split-K partial: part[z][I+1][J]; row I carries the column sums.
struct EpiPartial {
  float* part;
  int I;
  int J;
  __device__ __forceinline__ void operator()(int i, int j, float v) const {
    part[((long long)blockIdx.z * (I + 1) + i) * J + j] = v;
  }
  __device__ __forceinline__ void colsum(int j, float v) const {
    part[((long long)blockIdx.z * (I + 1) + I) * J + j] = v;
  }
};

template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM,
          class OpA, class OpB, class Epi>
inline void launch_gemm(const OpA& a, const OpB& b, const Epi& e, int I, int J,
                        int K, int zdim, int k_chunk, hipStream_t s) {
  dim3 grid(cdiv(I, BM), cdiv(J, BN), zdim);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WTM, WTN, SPLITK, COLSUM, OpA, OpB, Epi>),
                     grid, dim3(256), 0, s, a, b, e, I, J, K, k_chunk);
}

}  // namespace acmi
