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

#include <algorithm>

#include "gemm_ops.hpp"

// K-loop schedule: 0 = fetch the next tile before the MFMA block; 1 = spread
// the fetch over the k-steps; 2 = as 1 with the order pinned per k-step
#ifndef ACMI_GEMM_SCHED
#define ACMI_GEMM_SCHED 0
#endif

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

// SPLITK: the block's chunk z selects k in [z*k_chunk, min(K, (z+1)*k_chunk))
// (k_chunk % BK == 0) and is handed to the epilogue (epi.z).  The grid is then
// 1-D and XCD-aware (cdna_hip_programming.md §5.5 T1): hardware block b runs
// on XCD b % 8, and each XCD gets a contiguous run of logical blocks, i.e. all
// tiles of a few chunks, so the tiles that read the same rows share one L2.
// Otherwise the grid is (tiles_i, tiles_j, zdim) and operands/epilogues may
// use blockIdx.z for their own purposes (stride phases).
// COLSUM: blocks with blockIdx.x == 0 also return sum_k B(k, j) through
// epi.colsum(j, v) (the homogeneous row of [P;1]^T [..]).
// sym_cols > 0: the product's top-left sym_cols x sym_cols block is symmetric
// and only its upper triangle is consumed, so blocks lying strictly below the
// diagonal (every column < every row) inside it exit at once.
template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM,
          class OpA, class OpB, class Epi>
__global__ __launch_bounds__(256) void gemm_kernel(OpA opA, OpB opB, Epi epi,
                                                   int I, int J, int K,
                                                   int k_chunk, int sym_cols) {
  using TL = Tile<BM, BN, BK, WTM, WTN>;
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if constexpr (SPLITK) {
    // live tiles only: row x skips its first skip(x) column tiles (those
    // strictly below the diagonal of the symmetric block, see sym_cols)
    const int tx = (I + BM - 1) / BM, ty = (J + BN - 1) / BN;
    const int ssym = sym_cols > 0 ? sym_cols / BN : 0;
    int live = 0;
    for (int x = 0; x < tx; ++x) live += ty - min(x * BM / BN, ssym);
    const int total = gridDim.x;
    const int b = blockIdx.x;
#ifndef ACMI_NO_XCD_REMAP
    const int xcd = b & 7, base = total >> 3, rem = total & 7;
    const int l = xcd * base + min(xcd, rem) + (b >> 3);
#else
    const int l = b + 0 * total;
#endif
    bz = l / live;
    int t = l - bz * live;
    bx = 0;
    for (int x = 0; x < tx; ++x) {
      const int n = ty - min(x * BM / BN, ssym);
      if (t >= n) {
        t -= n;
        bx = x + 1;
      } else {
        break;
      }
    }
    by = min(bx * BM / BN, ssym) + t;
    epi.z = bz;
  } else if (sym_cols > 0 && (by + 1) * BN <= bx * BM && (by + 1) * BN <= sym_cols) {
    return;
  }
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
  const int i0 = bx * BM;
  const int j0 = by * BN;
  int kbeg = 0, kend = K;
  if constexpr (SPLITK) {
    kbeg = bz * k_chunk;
    kend = min(K, kbeg + k_chunk);
  }
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  typename OpA::St ra[NA];
  typename OpB::St rb[NB];

  // per-thread element coordinates: KCONTIG operands keep their row (i) fixed
  // across K-tiles, the others their columns (i) -> hoist that address part.
  // i-contiguous staging: TPR threads cover one k-row with RPR float4 runs
  // each (stride 4*TPR), so a thread touches NROW rows per tile; with TPR = 32
  // for both operands A and B visit the same rows and share the row decode.
  constexpr int AK = BK / 4;  // float4 slots per staging row (KCONTIG)
  constexpr int BKs = BK / 4;
  constexpr int TPRA = BM / 4 >= 32 ? 32 : BM / 4, RPRA = BM / 4 / TPRA, RSA = 256 / TPRA;
  constexpr int TPRB = BN / 4 >= 32 ? 32 : BN / 4, RPRB = BN / 4 / TPRB, RSB = 256 / TPRB;
  constexpr int NROWA = OpA::KCONTIG ? 1 : BK / RSA;
  constexpr int NROWB = OpB::KCONTIG ? 1 : BK / RSB;
  static_assert(OpA::KCONTIG || (BK % RSA == 0 && NROWA * RPRA == NA), "A staging map");
  static_assert(OpB::KCONTIG || (BK % RSB == 0 && NROWB * RPRB == NB), "B staging map");
  typename OpA::R rowA[OpA::KCONTIG ? NA : 1];
  typename OpA::C colA[OpA::KCONTIG ? 1 : RPRA];
  typename OpB::R rowB[OpB::KCONTIG ? NB : 1];
  typename OpB::C colB[OpB::KCONTIG ? 1 : RPRB];
  if constexpr (OpA::KCONTIG) {
#pragma unroll
    for (int v = 0; v < NA; ++v) rowA[v] = opA.row(i0 + (tid + 256 * v) / AK);
  } else {
#pragma unroll
    for (int u = 0; u < RPRA; ++u) colA[u] = opA.col(i0 + (tid % TPRA) * 4 + u * TPRA * 4);
  }
  if constexpr (OpB::KCONTIG) {
#pragma unroll
    for (int v = 0; v < NB; ++v) rowB[v] = opB.row(j0 + (tid + 256 * v) / BKs);
  } else {
#pragma unroll
    for (int u = 0; u < RPRB; ++u) colB[u] = opB.col(j0 + (tid % TPRB) * 4 + u * TPRB * 4);
  }

  // loads are unconditional (operands clamp out-of-range addresses); the K
  // bound and the operand masks are applied at commit (finish).  One element
  // (float4 run) at a time, so the K loop can spread them over its k-steps.
  auto fetch_a = [&](int k0, int v) {
    if constexpr (OpA::KCONTIG) {
      const int k = k0 + (tid % AK) * 4;  // same k for every v (256 % AK == 0)
      ra[v] = opA.stage(rowA[v], opA.col(k), k < kend);
    } else {
      const int k = k0 + tid / TPRA + RSA * (v / RPRA);
      ra[v] = opA.stage(opA.row(k), colA[v % RPRA], k < kend);
    }
  };
  auto fetch_b = [&](int k0, int v) {
    if constexpr (OpB::KCONTIG) {
      const int k = k0 + (tid % BKs) * 4;
      rb[v] = opB.stage(rowB[v], opB.col(k), k < kend);
    } else {
      const int k = k0 + tid / TPRB + RSB * (v / RPRB);
      rb[v] = opB.stage(opB.row(k), colB[v % RPRB], k < kend);
    }
  };
  auto fetch = [&](int k0) {
#pragma unroll
    for (int v = 0; v < NA; ++v) fetch_a(k0, v);
#pragma unroll
    for (int v = 0; v < NB; ++v) fetch_b(k0, v);
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
        const int k = tid / TPRA + RSA * (v / RPRA);
        const int i = (tid % TPRA) * 4 + (v % RPRA) * TPRA * 4;
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
        const int k = tid / TPRB + RSB * (v / RPRB);
        const int j = (tid % TPRB) * 4 + (v % RPRB) * TPRB * 4;
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
  // column sums of B ride on the MFMA fragment reads: lane l accumulates the
  // k-steps of parity l>>5 for column (l&31) of each of its WTN tiles; the
  // wm == 0 waves of bx == 0 blocks combine the halves and store them
  float csum[WTN];
#pragma unroll
  for (int tn = 0; tn < WTN; ++tn) csum[tn] = 0.f;

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
    const int knext = kbeg + (kt + 1) * BK;
    const float* As = lds + cur * ABUF;
    const float* Bs = lds + 2 * ABUF + cur * BBUF;
#if ACMI_GEMM_SCHED == 0
    fetch(knext);
    // keep the scheduler from hoisting the commit's finish() (which waits for
    // the loads) into the MFMA block
    __builtin_amdgcn_sched_barrier(0);
#endif
    float a[WTM], b[WTN];
#pragma unroll
    for (int tm = 0; tm < WTM; ++tm) a[tm] = As[khalf * SA + arow + tm * 32];
#pragma unroll
    for (int tn = 0; tn < WTN; ++tn) b[tn] = Bs[khalf * SB + brow + tn * 32];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      // fragments of the next k-step are read before this step's MFMAs
      float an[WTM], bn[WTN];
      if (kk + 2 < BK) {
#pragma unroll
        for (int tm = 0; tm < WTM; ++tm) an[tm] = As[(kk + 2 + khalf) * SA + arow + tm * 32];
#pragma unroll
        for (int tn = 0; tn < WTN; ++tn) bn[tn] = Bs[(kk + 2 + khalf) * SB + brow + tn * 32];
      }
#if ACMI_GEMM_SCHED != 0
      // the next tile's staging loads, one element per operand per k-step,
      // between the MFMAs (a wave's address arithmetic then overlaps its own
      // matrix work instead of preceding it)
      {
        constexpr int NSTEP = BK / 2;
        const int st = kk / 2;
        (void)NSTEP;
        if (st < NA) fetch_a(knext, st);
        if (st < NB) fetch_b(knext, st);
      }
#endif
      if constexpr (COLSUM) {
#pragma unroll
        for (int tn = 0; tn < WTN; ++tn) csum[tn] += b[tn];
      }
#pragma unroll
      for (int tm = 0; tm < WTM; ++tm)
#pragma unroll
        for (int tn = 0; tn < WTN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm], b[tn], acc[tm][tn], 0, 0, 0);
#if ACMI_GEMM_SCHED == 2
      __builtin_amdgcn_sched_barrier(0);
#endif
      if (kk + 2 < BK) {
#pragma unroll
        for (int tm = 0; tm < WTM; ++tm) a[tm] = an[tm];
#pragma unroll
        for (int tn = 0; tn < WTN; ++tn) b[tn] = bn[tn];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    commit(cur ^ 1);
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
    if (bx == 0 && wm == 0) {
#pragma unroll
      for (int tn = 0; tn < WTN; ++tn) {
        const float t = csum[tn] + __shfl_xor(csum[tn], 32);
        const int j = j0 + wn * WTN * 32 + tn * 32 + lane;
        if (lane < 32 && j < J) epi.colsum(j, t);
      }
    }
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
  int z = 0;  // chunk, set by gemm_kernel
  __device__ __forceinline__ void operator()(int i, int j, float v) const {
    part[((long long)z * (I + 1) + i) * J + j] = v;
  }
  __device__ __forceinline__ void colsum(int j, float v) const {
    part[((long long)z * (I + 1) + I) * J + j] = v;
  }
};

// LDS bytes of one gemm_kernel block and the blocks one CU holds (160 KiB LDS,
// 2048 threads)
template <int BM, int BN, int BK, bool KA, bool KB>
constexpr int gemm_lds_bytes() {
  return 2 * BK * ((KA ? BM + 1 : BM + 4) + (KB ? BN + 1 : BN + 4)) * 4;
}
template <int BM, int BN, int BK, bool KA, bool KB>
constexpr int gemm_blocks_per_cu() {
  return std::min(8, 160 * 1024 / gemm_lds_bytes<BM, BN, BK, KA, KB>());
}

// Split a reduction over `rows` into chunks for `live` tiles so the grid fills
// whole rounds of `slots` resident blocks (a partly filled last round idles
// most of the chip for a whole block time).  Chunks are multiples of 32 rows
// and at least min_rows long.
inline void plan_rounds(long long rows, int live, int slots, int* nchunk, int* chunk,
                        int min_rows = 512) {
  int best_nc = 1;
  double best = -1.0;
  for (int r = 1; r <= 8; ++r) {
    const int nc = std::max(1, (r * slots) / std::max(1, live));
    long long ch = (rows + nc - 1) / nc;
    ch = (ch + 31) / 32 * 32;
    if (ch < min_rows && r > 1) break;
    const int ncr = (int)((rows + ch - 1) / ch);
    const int blocks = ncr * live;
    const int rounds = (blocks + slots - 1) / slots;
    const double eff = (double)blocks / ((double)rounds * slots);
    // prefer fewer rounds unless a later one fills noticeably better
    if (eff > best + 0.02) {
      best = eff;
      best_nc = ncr;
    }
  }
  long long ch = (rows + best_nc - 1) / best_nc;
  ch = (ch + 31) / 32 * 32;
  *chunk = (int)ch;
  *nchunk = (int)((rows + ch - 1) / ch);
}

// tiles of an I x J product that gemm_kernel computes (sym_cols skip applied)
template <int BM, int BN>
inline int live_tiles(int I, int J, int sym_cols) {
  const int tx = cdiv(I, BM), ty = cdiv(J, BN);
  const int ssym = sym_cols > 0 ? sym_cols / BN : 0;
  int live = 0;
  for (int x = 0; x < tx; ++x) live += ty - std::min(x * BM / BN, ssym);
  return live;
}

template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM,
          class OpA, class OpB, class Epi>
inline void launch_gemm(const OpA& a, const OpB& b, const Epi& e, int I, int J,
                        int K, int zdim, int k_chunk, hipStream_t s, int sym_cols = 0) {
  dim3 grid(cdiv(I, BM), cdiv(J, BN), zdim);
  if (SPLITK) grid = dim3(live_tiles<BM, BN>(I, J, sym_cols) * zdim);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WTM, WTN, SPLITK, COLSUM, OpA, OpB, Epi>),
                     grid, dim3(256), 0, s, a, b, e, I, J, K, k_chunk, sym_cols);
}

}  // namespace acmi
