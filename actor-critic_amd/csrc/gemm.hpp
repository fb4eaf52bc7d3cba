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
// Operand concept (template parameter Op; loaders in gemm_ops.hpp):
//   static constexpr bool KCONTIG;   // float4 runs along k (true) or i/j
//   R row(int) const; C col(int) const; St stage(R, C, bool) const;
//   float4 finish(St)   (deferred masking, see gemm_ops.hpp)
// LDS images are [k][i] for both operands so the MFMA fragment read
// (lane l: row k = l>>5, col i = l&31) is one conflict-free ds_read_b32 per
// operand per k-step.  K-contiguous operands are written transposed with a
// row stride == 1 (mod 32) (conflict-free scatter), i-contiguous ones with a
// 16-byte aligned stride (ds_write_b128).
#pragma once

#include "gemm_ops.hpp"

namespace acmi {

typedef float f32x16 __attribute__((ext_vector_type(16)));

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
// sym_cols > 0 (requires BM == BN): the product's top-left sym_cols x sym_cols
// block is symmetric and only its upper triangle is consumed, so blocks
// strictly below the diagonal whose column tile lies inside it exit at once.
template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM,
          class OpA, class OpB, class Epi>
__global__ __launch_bounds__(256) void gemm_kernel(OpA opA, OpB opB, Epi epi,
                                                   int I, int J, int K,
                                                   int k_chunk, int sym_cols) {
  using TL = Tile<BM, BN, BK, WTM, WTN>;
  if (BM == BN && sym_cols > 0 && blockIdx.y < blockIdx.x &&
      (int)(blockIdx.y + 1) * BN <= sym_cols)
    return;
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

  typename OpA::St ra[NA];
  typename OpB::St rb[NB];

  // per-thread element coordinates: KCONTIG operands keep their row (i) fixed
  // across K-tiles, the others their column (i) -> hoist that address part
  constexpr int AK = OpA::KCONTIG ? BK / 4 : BM / 4;  // float4 slots per staging row
  constexpr int BKs = OpB::KCONTIG ? BK / 4 : BN / 4;
  typename OpA::R rowA[OpA::KCONTIG ? NA : 1];
  typename OpA::C colA;
  typename OpB::R rowB[OpB::KCONTIG ? NB : 1];
  typename OpB::C colB;
  if constexpr (OpA::KCONTIG) {
#pragma unroll
    for (int v = 0; v < NA; ++v) rowA[v] = opA.row(i0 + (tid + 256 * v) / AK);
  } else {
    colA = opA.col(i0 + (tid % AK) * 4);
  }
  if constexpr (OpB::KCONTIG) {
#pragma unroll
    for (int v = 0; v < NB; ++v) rowB[v] = opB.row(j0 + (tid + 256 * v) / BKs);
  } else {
    colB = opB.col(j0 + (tid % BKs) * 4);
  }

  // loads are unconditional (operands clamp out-of-range addresses); the K
  // bound and the operand masks are applied at commit (finish)
  auto fetch = [&](int k0) {
    if constexpr (OpA::KCONTIG) {
      const int k = k0 + (tid % AK) * 4;  // same k for every v (256 % AK == 0)
      const auto c = opA.col(k);
#pragma unroll
      for (int v = 0; v < NA; ++v) ra[v] = opA.stage(rowA[v], c, k < kend);
    } else {
#pragma unroll
      for (int v = 0; v < NA; ++v) {
        const int k = k0 + (tid + 256 * v) / AK;
        ra[v] = opA.stage(opA.row(k), colA, k < kend);
      }
    }
    if constexpr (OpB::KCONTIG) {
      const int k = k0 + (tid % BKs) * 4;
      const auto c = opB.col(k);
#pragma unroll
      for (int v = 0; v < NB; ++v) rb[v] = opB.stage(rowB[v], c, k < kend);
    } else {
#pragma unroll
      for (int v = 0; v < NB; ++v) {
        const int k = k0 + (tid + 256 * v) / BKs;
        rb[v] = opB.stage(opB.row(k), colB, k < kend);
      }
    }
  };

  auto commit = [&](int buf) {
    float* As = lds + buf * ABUF;
    float* Bs = lds + 2 * ABUF + buf * BBUF;
#pragma unroll
    for (int v = 0; v < NA; ++v) {
      const int idx = tid + 256 * v;
      const float4 x = finish(ra[v]);
      if constexpr (OpA::KCONTIG) {
        const int i = idx / (BK / 4);
        const int k = (idx - i * (BK / 4)) * 4;
        As[(k + 0) * SA + i] = x.x;
        As[(k + 1) * SA + i] = x.y;
        As[(k + 2) * SA + i] = x.z;
        As[(k + 3) * SA + i] = x.w;
      } else {
        const int k = idx / (BM / 4);
        const int i = (idx - k * (BM / 4)) * 4;
        *reinterpret_cast<float4*>(As + k * SA + i) = x;
      }
    }
#pragma unroll
    for (int v = 0; v < NB; ++v) {
      const int idx = tid + 256 * v;
      const float4 x = finish(rb[v]);
      if constexpr (OpB::KCONTIG) {
        const int j = idx / (BK / 4);
        const int k = (idx - j * (BK / 4)) * 4;
        Bs[(k + 0) * SB + j] = x.x;
        Bs[(k + 1) * SB + j] = x.y;
        Bs[(k + 2) * SB + j] = x.z;
        Bs[(k + 3) * SB + j] = x.w;
      } else {
        const int k = idx / (BN / 4);
        const int j = (idx - k * (BN / 4)) * 4;
        *reinterpret_cast<float4*>(Bs + k * SB + j) = x;
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

  // The loop body is one basic block: the next tile's fetch is unconditional
  // (past kend it reads clamped addresses and is zeroed), so its loads stay in
  // flight across the MFMAs and are only waited for at the LDS commit.
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    fetch(kbeg + (kt + 1) * BK);
    // keep the scheduler from hoisting the commit's finish() (which waits for
    // the loads) into the MFMA block
    __builtin_amdgcn_sched_barrier(0);
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
    __builtin_amdgcn_sched_barrier(0);
    commit(cur ^ 1);
    if constexpr (COLSUM) {
      if (do_colsum) {
#pragma unroll 8
        for (int kk = 0; kk < BK; ++kk) csum += Bs[kk * SB + tid];
      }
    }
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
                        int K, int zdim, int k_chunk, hipStream_t s, int sym_cols = 0) {
  dim3 grid(cdiv(I, BM), cdiv(J, BN), zdim);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WTM, WTN, SPLITK, COLSUM, OpA, OpB, Epi>),
                     grid, dim3(256), 0, s, a, b, e, I, J, K, k_chunk, sym_cols);
}

}  // namespace acmi
