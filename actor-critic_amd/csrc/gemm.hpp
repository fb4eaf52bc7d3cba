// LDS-tiled f32-input MFMA GEMM engine for gfx950 with pluggable operands.
//
//   C[i][j] = sum_k A(k, i) * B(k, j)
//
// Every GEMM-shaped op on the A2C/ACKTR path is an instance of this kernel:
//   * conv forward (implicit im2col, u8/255 fused for conv1)       RowsAsK
//   * conv input-gradient (transposed conv as a per-stride-phase gather)
//   * fc forward / input-gradient
//   * weight gradient fused with the K-FAC A-factor: [P;1]^T [P | dY]
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
#include <type_traits>

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

// SPLITK: the block's chunk z selects k in [z*k_chunk, min(K, (z+1)*k_chunk))
// (k_chunk % BK == 0) and is handed to the epilogue (epi.z).  The grid is then
// 1-D and XCD-aware (cdna_hip_programming.md §5.5 T1): hardware block b runs
// on XCD b % 8, and each XCD gets a contiguous run of logical blocks, i.e. all
// tiles of a few chunks, so the tiles that read the same rows share one L2.
// Otherwise the grid is (tiles_i, tiles_j, zdim) and the z coordinate (a
// stride phase) is handed to operands/epilogues that have a member z.
// COLSUM: blocks with blockIdx.x == 0 also return sum_k B(k, j) through
// epi.colsum(j, v) (the homogeneous row of [P;1]^T [..]).
// sym_cols > 0: the product's top-left sym_cols x sym_cols block is symmetric
// and only its upper triangle is consumed, so blocks lying strictly below the
// diagonal (every column < every row) inside it exit at once.
// Epilogue of a wave's (32*WTM) x (32*WTN) sub-tile at (ib, jb):
// acc[tm][tn][r] -> (ib + 32tm + (r&3) + 8(r>>2) + 4(lane>>5), jb + 32tn + (lane&31))
// (gfx950 32x32 C/D map).  All aux loads first (clamped indices), then the
// bounded stores.  Epilogues with VEC4 take the four consecutive rows a lane
// holds (r = 4g..4g+3) as one float4 (aux4/store4 at row i0 = 4-aligned; I % 4
// == 0): one 16-byte access instead of four scalar ones when those rows are
// contiguous in memory.
template <class T, class = void>
struct has_vec4 : std::false_type {};
template <class T>
struct has_vec4<T, std::void_t<decltype(T::VEC4)>> : std::integral_constant<bool, T::VEC4> {};

// Epilogues with a member `unsigned* amax` (nullable) also publish the largest
// |value| they stored: store/store4 return what they wrote, each wave takes the
// max of its lanes and one lane publishes it (amax_update: atomicMax of the bit
// pattern when larger) into *amax, zeroed by the caller before the launch.  The
// band reductions and the f16x2 operand splits scale a tensor by it (band.hpp).
template <class T, class = void>
struct has_amax : std::false_type {};
template <class T>
struct has_amax<T, std::void_t<decltype(std::declval<T&>().amax)>> : std::true_type {};

__device__ __forceinline__ void amax_publish(unsigned* amax, float m, int lane) {
  m = wave_max(m);
  if (amax && lane == 0) amax_update(amax, m);
}
__device__ __forceinline__ float absmax4(float m, float4 v) {
  return fmaxf(fmaxf(m, fmaxf(fabsf(v.x), fabsf(v.y))), fmaxf(fabsf(v.z), fabsf(v.w)));
}

template <int WTM, int WTN, class Epi, class Acc>
__device__ __forceinline__ void store_tile(const Epi& epi, const Acc& acc, int ib, int jb, int lane,
                                           int I, int J) {
  const int khalf = lane >> 5;
  float am = 0.f;
  if constexpr (has_vec4<Epi>::value) {
    float4 x[WTM][WTN][4];
#pragma unroll
    for (int tm = 0; tm < WTM; ++tm)
#pragma unroll
      for (int tn = 0; tn < WTN; ++tn) {
        const int j = min(jb + tn * 32 + (lane & 31), J - 1);
#pragma unroll
        for (int g = 0; g < 4; ++g)
          x[tm][tn][g] = epi.aux4(min(ib + tm * 32 + 8 * g + 4 * khalf, I - 4), j);
      }
#pragma unroll
    for (int tm = 0; tm < WTM; ++tm)
#pragma unroll
      for (int tn = 0; tn < WTN; ++tn) {
        const int j = jb + tn * 32 + (lane & 31);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int i0 = ib + tm * 32 + 8 * g + 4 * khalf;
          const float4 v = make_float4(acc[tm][tn][4 * g], acc[tm][tn][4 * g + 1],
                                       acc[tm][tn][4 * g + 2], acc[tm][tn][4 * g + 3]);
          if (i0 < I && j < J) {
            if constexpr (has_amax<Epi>::value) am = absmax4(am, epi.store4(i0, j, v, x[tm][tn][g]));
            else epi.store4(i0, j, v, x[tm][tn][g]);
          }
        }
      }
  } else {
    float x[WTM][WTN][16];
#pragma unroll
    for (int tm = 0; tm < WTM; ++tm)
#pragma unroll
      for (int tn = 0; tn < WTN; ++tn) {
        const int j = min(jb + tn * 32 + (lane & 31), J - 1);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int i = min(ib + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf, I - 1);
          x[tm][tn][r] = epi.aux(i, j);
        }
      }
#pragma unroll
    for (int tm = 0; tm < WTM; ++tm)
#pragma unroll
      for (int tn = 0; tn < WTN; ++tn) {
        const int j = jb + tn * 32 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int i = ib + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
          if (i < I && j < J) {
            if constexpr (has_amax<Epi>::value) am = fmaxf(am, fabsf(epi.store(i, j, acc[tm][tn][r], x[tm][tn][r])));
            else epi.store(i, j, acc[tm][tn][r], x[tm][tn][r]);
          }
        }
      }
  }
  if constexpr (has_amax<Epi>::value) amax_publish(epi.amax, am, lane);
}

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

// Epilogues with LDS_T take their float4 row runs (aux4/store4, as VEC4) after a
// transpose through LDS: the C map gives a lane 4 consecutive rows of ONE column
// (32 columns per instruction, 16-32 bytes each), so for an output whose rows
// are contiguous in memory (EpiConvT: channels of a pixel) each access touches
// 32 lines.  Through LDS ([col][row] per 32x32 block) 8 lanes cover 32 rows of
// one column: one instruction moves 8 whole 128-byte runs.  The caller has
// synchronised the block (the LDS staging buffers are free); each wave uses
// its own 32x36-float region and reads back only what it wrote.
template <class T, class = void>
struct has_ldst : std::false_type {};
template <class T>
struct has_ldst<T, std::void_t<decltype(T::LDS_T)>> : std::integral_constant<bool, T::LDS_T> {};

template <int WTM, int WTN, class Epi, class Acc>
__device__ __forceinline__ void store_tile_lds(const Epi& epi, const Acc& acc, int ib, int jb,
                                               int lane, float* wlds, int I, int J) {
  constexpr int S = 36;  // [32 columns][32 rows + 4]
  const int khalf = lane >> 5, c = lane & 31;
  const int ri = 4 * (lane & 7), cj = lane >> 3;  // read-back map: rows ri..ri+3 of column cj+8p
  float am = 0.f;
#pragma unroll
  for (int tm = 0; tm < WTM; ++tm)
#pragma unroll
    for (int tn = 0; tn < WTN; ++tn) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(wlds + c * S + 8 * g + 4 * khalf) =
            make_float4(acc[tm][tn][4 * g], acc[tm][tn][4 * g + 1], acc[tm][tn][4 * g + 2],
                        acc[tm][tn][4 * g + 3]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float4 v[4], x[4];
      const int i0 = ib + tm * 32 + ri;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        v[p] = *reinterpret_cast<const float4*>(wlds + (cj + 8 * p) * S + ri);
        x[p] = epi.aux4(min(i0, I - 4), min(jb + tn * 32 + cj + 8 * p, J - 1));
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int j = jb + tn * 32 + cj + 8 * p;
        if (i0 < I && j < J) {
          if constexpr (has_amax<Epi>::value) am = absmax4(am, epi.store4(i0, j, v[p], x[p]));
          else epi.store4(i0, j, v[p], x[p]);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  if constexpr (has_amax<Epi>::value) amax_publish(epi.amax, am, lane);
}

// DEPTH: K-tiles of staging loads in flight (register sets): 1 = the next
// tile's loads overlap the current tile's MFMAs; 2 = two tiles ahead, for
// latency-bound shapes (short per-tile MFMA work, L2-missing gathers).
// The work of one output tile (bx, by) of split-K chunk bz: gemm_kernel maps its
// grid onto tiles, gemm_group_kernel maps one grid over several problems.
template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM, class OpA, class OpB,
          class Epi, int DEPTH>
__device__ __forceinline__ void gemm_block(OpA opA, OpB opB, Epi epi, int I, int J, int K, int k_chunk,
                                           int sym_cols, int bx, int by, int bz) {
  using TL = Tile<BM, BN, BK, WTM, WTN>;
  set_z(opA, bz);
  set_z(opB, bz);
  set_z(epi, bz);
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

  static_assert(DEPTH == 1 || DEPTH == 2, "prefetch depth 1 or 2");
  typename OpA::St ra[DEPTH][NA];
  typename OpB::St rb[DEPTH][NB];

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
  // register set S is a compile-time index (std::integral_constant): a runtime
  // index into ra/rb would put the staging registers in scratch
  auto fetch = [&](int k0, auto S) {
    constexpr int set = decltype(S)::value;
    if constexpr (OpA::KCONTIG) {
      const int k = k0 + (tid % AK) * 4;  // same k for every v (256 % AK == 0)
      const auto c = opA.col(k);
#pragma unroll
      for (int v = 0; v < NA; ++v) ra[set][v] = opA.stage(rowA[v], c, k < kend);
    } else {
#pragma unroll
      for (int rr = 0; rr < NROWA; ++rr) {
        const int k = k0 + tid / TPRA + RSA * rr;
        const auto r = opA.row(k);
#pragma unroll
        for (int u = 0; u < RPRA; ++u) ra[set][rr * RPRA + u] = opA.stage(r, colA[u], k < kend);
      }
    }
    if constexpr (OpB::KCONTIG) {
      const int k = k0 + (tid % BKs) * 4;
      const auto c = opB.col(k);
#pragma unroll
      for (int v = 0; v < NB; ++v) rb[set][v] = opB.stage(rowB[v], c, k < kend);
    } else {
#pragma unroll
      for (int rr = 0; rr < NROWB; ++rr) {
        const int k = k0 + tid / TPRB + RSB * rr;
        const auto r = opB.row(k);
#pragma unroll
        for (int u = 0; u < RPRB; ++u) rb[set][rr * RPRB + u] = opB.stage(r, colB[u], k < kend);
      }
    }
  };

  auto commit = [&](int buf, auto S) {
    constexpr int set = decltype(S)::value;
    float* As = lds + buf * ABUF;
    float* Bs = lds + 2 * ABUF + buf * BBUF;
#pragma unroll
    for (int v = 0; v < NA; ++v) {
      const int idx = tid + 256 * v;
      const float4 x = finish(ra[set][v]);
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
      const float4 x = finish(rb[set][v]);
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

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, DEPTH == 2 ? 1 : 0>;
  if (nk > 0) {
    fetch(kbeg, S0{});
    commit(0, S0{});
    if constexpr (DEPTH == 2) fetch(kbeg + BK, S1{});
  }
  __syncthreads();

  const int arow = wm * WTM * 32 + (lane & 31);
  const int brow = wn * WTN * 32 + (lane & 31);
  const int khalf = lane >> 5;

  // One K-tile: issue the staging loads DEPTH tiles ahead (unconditional:
  // past kend they read clamped addresses and are zeroed), run the MFMAs on
  // LDS buffer `cur`, then write the tile kt+1 held in register set SC to the
  // other buffer.  The body is one basic block and sched_barriers keep the
  // commit (which waits for its loads) behind the MFMA block.
  auto step = [&](int kt, int cur, auto SC, auto SF, auto MF) {
    constexpr bool mf = decltype(MF)::value;
    fetch(kbeg + (kt + DEPTH) * BK, SF);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (mf) {
      const float* As = lds + cur * ABUF;
      const float* Bs = lds + 2 * ABUF + cur * BBUF;
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
        if constexpr (COLSUM) {
#pragma unroll
          for (int tn = 0; tn < WTN; ++tn) csum[tn] += b[tn];
        }
#pragma unroll
        for (int tm = 0; tm < WTM; ++tm)
#pragma unroll
          for (int tn = 0; tn < WTN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm], b[tn], acc[tm][tn], 0, 0, 0);
        if (kk + 2 < BK) {
#pragma unroll
          for (int tm = 0; tm < WTM; ++tm) a[tm] = an[tm];
#pragma unroll
          for (int tn = 0; tn < WTN; ++tn) b[tn] = bn[tn];
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    commit(cur ^ 1, SC);
    __syncthreads();
  };
  // two K-tiles per iteration so the register sets are compile-time indices:
  // with DEPTH 2, tile t lives in set t & 1
  // A wave whose whole sub-tile lies strictly below the diagonal of the
  // symmetric block (diagonal blocks, sym_cols) computes nothing anyone reads:
  // it only stages and syncs (its SIMD serves the co-resident blocks' MFMAs).
  // So does a wave whose sub-tile lies wholly outside I x J (edge tiles).
  const int wrow0 = i0 + wm * WTM * 32, wcol0 = j0 + wn * WTN * 32, wcol1 = wcol0 + WTN * 32;
  const bool wave_idle =
      (sym_cols > 0 && wcol1 <= wrow0 && wcol1 <= sym_cols) || wrow0 >= I || wcol0 >= J;
  using MFon = std::integral_constant<bool, true>;
  using MFoff = std::integral_constant<bool, false>;
  if (!wave_idle) {
    for (int kt = 0; kt < nk; kt += 2) {
      step(kt, 0, S1{}, S0{}, MFon{});
      if (kt + 1 < nk) step(kt + 1, 1, S0{}, S1{}, MFon{});
    }
  } else {
    for (int kt = 0; kt < nk; kt += 2) {
      step(kt, 0, S1{}, S0{}, MFoff{});
      if (kt + 1 < nk) step(kt + 1, 1, S0{}, S1{}, MFoff{});
    }
  }

  // epilogue: acc[tm][tn][r] -> C[i][j],  j = lane&31 (+tile),
  // i = (r&3) + 8*(r>>2) + 4*(lane>>5) (+tile)   (gfx950 32x32 C/D map)
  if constexpr (has_ldst<Epi>::value && 2 * (ABUF + BBUF) >= 4 * 32 * 36) {
    __syncthreads();  // every wave is done with the staging buffers
    store_tile_lds<WTM, WTN>(epi, acc, i0 + wm * WTM * 32, j0 + wn * WTN * 32, lane,
                             lds + wave * 32 * 36, I, J);
  } else {
    store_tile<WTM, WTN>(epi, acc, i0 + wm * WTM * 32, j0 + wn * WTN * 32, lane, I, J);
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

template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM,
          class OpA, class OpB, class Epi, int DEPTH = 1>
// waves_per_eu = the blocks per CU the LDS allows (one wave per SIMD each),
// which plan_rounds counts on for the split-K reductions: for the 128x128x16
// tiles that is 4, and without the hint the compiler parks the accumulators in
// AGPRs next to ~85 VGPRs so only 3 fit.  (The conv2 input gradient spills a
// little at 4 and is still faster than at 3; shapes whose registers cannot
// reach the LDS bound get the compiler's best, -Wno-pass-failed.)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    gemm_blocks_per_cu<BM, BN, BK, OpA::KCONTIG, OpB::KCONTIG>())))
void gemm_kernel(OpA opA, OpB opB, Epi epi, int I, int J, int K, int k_chunk, int sym_cols) {
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
  } else if (sym_cols > 0 && (by + 1) * BN <= bx * BM && (by + 1) * BN <= sym_cols) {
    return;
  }
  gemm_block<BM, BN, BK, WTM, WTN, SPLITK, COLSUM, OpA, OpB, Epi, DEPTH>(opA, opB, epi, I, J, K, k_chunk,
                                                                       sym_cols, bx, by, bz);
}

// ---------------------------------------------------------------------------
// Epilogues.  Two phases per element so no load sits under the tile-edge
// branch (the .s trap (c) again: a load under `if (i < I && j < J)` waits
// vmcnt(0) per element): aux(i, j) loads what the store needs from a clamped,
// always valid (i, j) for every element first; store(i, j, v, aux) then runs
// under the bounds check.
// ---------------------------------------------------------------------------
struct EpiStore {
  float* out;
  long long ld;
  __device__ __forceinline__ float aux(int, int) const { return 0.f; }
  __device__ __forceinline__ void store(int i, int j, float v, float) const {
    out[(long long)i * ld + j] = v;
  }
};

// out = relu?(v + bias[j])
struct EpiBiasAct {
  float* out;
  long long ld;
  const float* bias;
  int relu;
  __device__ __forceinline__ float aux(int, int j) const { return bias[j]; }
  __device__ __forceinline__ void store(int i, int j, float v, float b) const {
    v += b;
    if (relu) v = fmaxf(v, 0.f);
    out[(long long)i * ld + j] = v;
  }
};

// out = v * (act > 0)   (ReLU derivative from the stored post-ReLU output)
// MASK: the activation's ReLU' bits (acmi_acts_t m1..m3: bit e of word e / 32 =
// act[e] > 0) read instead of the f32 activation -- 1/32 of its bytes.  A
// compile-time choice: a runtime one put the epilogue's loads under a branch
// (fc4 dX 91 -> 119 us).
template <bool MASK = false>
struct EpiReluGrad {
  float* out;
  const float* act;  // MASK: the uint32 bit words
  long long ld;
  unsigned* amax = nullptr;  // nullable: max |out| (has_amax)
  __device__ __forceinline__ float aux(int i, int j) const {
    const long long e = (long long)i * ld + j;
    if constexpr (MASK) return (float)((reinterpret_cast<const uint32_t*>(act)[e >> 5] >> (e & 31)) & 1u);
    else return act[e];
  }
  __device__ __forceinline__ float store(int i, int j, float v, float x) const {
    const float o = x > 0.f ? v : 0.f;
    out[(long long)i * ld + j] = o;
    return o;
  }
};

// input-gradient of a strided conv as the TRANSPOSED product: row i =
// (ph, pw, ci) (all stride phases), column j = super-pixel (img, ih', iw') ->
// NHWC pixel (S*ih'+ph, S*iw'+pw), channel ci; masked by ReLU'.  Four
// consecutive rows are four consecutive channels of one pixel (VEC4), written
// after the LDS transpose (LDS_T) as whole 128-byte channel runs.
template <int IH, int IW, int S, int CIN, bool MASK = false>
struct EpiConvT {
  static constexpr bool VEC4 = true;
  static constexpr bool LDS_T = true;
  static_assert(CIN % 4 == 0, "channel runs of 4");
  float* out;
  const float* act;  // MASK: its ReLU' bit words (EpiReluGrad)
  unsigned* amax = nullptr;  // nullable: max |out| (has_amax)
  __device__ __forceinline__ long long offset(int i, int j) const {
    constexpr int PH = IH / S, PW = IW / S, L = PH * PW;
    const uint32_t img = (uint32_t)j / L;
    const uint32_t p = (uint32_t)j - img * L;
    const uint32_t ihp = p / PW;
    const uint32_t iwp = p - ihp * PW;
    const int ph = i / (S * CIN);
    const int rem = i - ph * (S * CIN);
    const int pw = rem / CIN;
    const int ci = rem - pw * CIN;
    return (((long long)img * IH + (S * ihp + ph)) * IW + (S * iwp + pw)) * CIN + ci;
  }
  __device__ __forceinline__ float4 aux4(int i0, int j) const {
    const long long e = offset(i0, j);
    if constexpr (MASK) {  // 4 consecutive channels: 4 bits of one word (CIN % 32 == 0)
      static_assert(CIN % 32 == 0, "mask words of 32 channels");
      const uint32_t b = reinterpret_cast<const uint32_t*>(act)[e >> 5] >> (e & 31);
      return make_float4((float)(b & 1u), (float)((b >> 1) & 1u), (float)((b >> 2) & 1u), (float)((b >> 3) & 1u));
    } else {
      return *reinterpret_cast<const float4*>(act + e);
    }
  }
  __device__ __forceinline__ float4 store4(int i0, int j, float4 v, float4 x) const {
    float4 o;
    o.x = x.x > 0.f ? v.x : 0.f;
    o.y = x.y > 0.f ? v.y : 0.f;
    o.z = x.z > 0.f ? v.z : 0.f;
    o.w = x.w > 0.f ? v.w : 0.f;
    *reinterpret_cast<float4*>(out + offset(i0, j)) = o;
    return o;
  }
};

// split-K partial: part[z][I+1][J]; row I carries the column sums.
struct EpiPartial {
  float* part;
  int I;
  int J;
  int z = 0;  // chunk, set by gemm_kernel
  __device__ __forceinline__ float aux(int, int) const { return 0.f; }
  __device__ __forceinline__ void store(int i, int j, float v, float) const {
    part[((long long)z * (I + 1) + i) * J + j] = v;
  }
  __device__ __forceinline__ void colsum(int j, float v) const {
    part[((long long)z * (I + 1) + I) * J + j] = v;
  }
};

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

template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM, int DEPTH = 1,
          class OpA, class OpB, class Epi>
inline void launch_gemm(const OpA& a, const OpB& b, const Epi& e, int I, int J,
                        int K, int zdim, int k_chunk, hipStream_t s, int sym_cols = 0) {
  dim3 grid(cdiv(I, BM), cdiv(J, BN), zdim);
  if (SPLITK) grid = dim3(live_tiles<BM, BN>(I, J, sym_cols) * zdim);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WTM, WTN, SPLITK, COLSUM, OpA, OpB, Epi, DEPTH>),
                     grid, dim3(256), 0, s, a, b, e, I, J, K, k_chunk, sym_cols);
}

// Several independent problems (same operand types and tile shape, no split-K)
// in one launch: block b runs tile b - tile0[p] of problem p.  For chains of
// small GEMMs whose launches would otherwise each cost a latency.
constexpr int kGemmGroupMax = 6;
template <class OpA, class OpB, class Epi>
struct GemmGroup {
  int n;
  int tile0[kGemmGroupMax + 1];
  int tiles_x[kGemmGroupMax];
  int I[kGemmGroupMax], J[kGemmGroupMax], K[kGemmGroupMax];
  OpA a[kGemmGroupMax];
  OpB b[kGemmGroupMax];
  Epi e[kGemmGroupMax];
};

template <int BM, int BN, int BK, int WTM, int WTN, class OpA, class OpB, class Epi>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    gemm_blocks_per_cu<BM, BN, BK, OpA::KCONTIG, OpB::KCONTIG>())))
void gemm_group_kernel(GemmGroup<OpA, OpB, Epi> g) {
  const int b = blockIdx.x;
  int p = 0;
  while (p + 1 < g.n && b >= g.tile0[p + 1]) ++p;
  p = __builtin_amdgcn_readfirstlane(p);
  const int t = b - g.tile0[p];
  const int bx = t % g.tiles_x[p], by = t / g.tiles_x[p];
  gemm_block<BM, BN, BK, WTM, WTN, false, false, OpA, OpB, Epi, 1>(g.a[p], g.b[p], g.e[p], g.I[p], g.J[p],
                                                                    g.K[p], 0, 0, bx, by, 0);
}

template <int BM, int BN, int BK, int WTM, int WTN, class OpA, class OpB, class Epi>
inline void launch_gemm_group(GemmGroup<OpA, OpB, Epi>& g, hipStream_t s) {
  g.tile0[0] = 0;
  for (int p = 0; p < g.n; ++p) {
    g.tiles_x[p] = cdiv(g.I[p], BM);
    g.tile0[p + 1] = g.tile0[p] + g.tiles_x[p] * cdiv(g.J[p], BN);
  }
  hipLaunchKernelGGL((gemm_group_kernel<BM, BN, BK, WTM, WTN, OpA, OpB, Epi>), dim3(g.tile0[g.n]), dim3(256),
                     0, s, g);
}

}  // namespace acmi
