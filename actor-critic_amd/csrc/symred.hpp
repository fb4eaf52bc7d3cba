// Slab-grouped split-K reduction for the fused weight-gradient / K-FAC A-factor
// product  [P;1]^T [P | dY]  (conv2, conv3, heads).
//
// gemm_kernel covers the product with 128x128 tiles and skips the tiles below
// the diagonal of the symmetric P^T P block, but the 4 diagonal tiles still
// hold a useless lower-left 64x64 quarter and the dY tile a useless right half
// (cout = 64 of 128 columns): 14 tiles of 4 waves for 44 useful 64x64
// sub-tiles (conv2).  Here the unit is the 64-column SLAB of the [P | dY]
// column space.  A block stages up to four slabs (256 columns, the same LDS
// and load volume as a 128x128 tile: A and B are the same rows of the same
// operand) and each of its 4 waves multiplies one (row slab a, column slab b)
// pair with a <= b.  sym_plan() partitions the needed sub-tiles into groups of
// four that use at most four slabs, e.g. for conv2 (8 P slabs + dY):
//   6 groups {2i,2i+1} x {2j,2j+1}                      (off-diagonal, i < j)
//   4 groups (2i,2i+1) (2i+1,2i+1) (2i,dY) (2i+1,dY)    (slabs 2i, 2i+1, dY)
//   1 group  (0,0) (2,2) (4,4) (6,6)                    (diagonal slabs)
// = 11 blocks per row chunk with every wave busy (vs 14).  Same staging,
// fragment maps, MFMA chain order and split-K partial layout as gemm_kernel
// (EpiPartial [chunk][I+1][J], column sums in row I), so finalize_wgrad_kernel
// is unchanged.  The column sums (the homogeneous row) of column slab b come
// from the one wave whose row slab is 0 (sub-tile (0, b) is unique).
#pragma once

#include "gemm.hpp"

namespace acmi {

struct SymGroup {
  int16_t base[4];  // first [P | dY] column of each staged slab (-1: none)
  int8_t wa[4];     // per wave: staged slab of its rows (-1: idle)
  int8_t wb[4];     // per wave: staged slab of its columns
};
constexpr int kSymMaxGroups = 96;
struct SymPlan {
  int ngroups;
  SymGroup g[kSymMaxGroups];
};

// P columns 0..K-1 in slabs 0..nb-1 and one dY slab (cout_pad <= 64) at column
// K.  When K % 64 != 0 (fc4: 1568) the last P slab runs into the first dY
// columns: those products are also made by the (a, dY) sub-tiles from the same
// inputs in the same order, so both write identical values, and its rows >= K
// are never stored.  Returns false when the shape does not fit the scheme.
inline bool sym_plan(int K, int cout_pad, SymPlan* p) {
  if (cout_pad > 64 || cout_pad <= 0 || K <= 0) return false;
  const int nb = (K + 63) / 64, np = nb / 2, dy = K;
  const bool odd = nb & 1;
  const int last = 64 * (nb - 1);
  int n = 0;
  auto add = [&](int b0, int b1, int b2, int b3, int a0, int c0, int a1, int c1, int a2, int c2,
                 int a3, int c3) {
    if (n >= kSymMaxGroups) return false;
    SymGroup& g = p->g[n++];
    const int b[4] = {b0, b1, b2, b3}, a[4] = {a0, a1, a2, a3}, c[4] = {c0, c1, c2, c3};
    for (int s = 0; s < 4; ++s) {
      g.base[s] = (int16_t)b[s];
      g.wa[s] = (int8_t)a[s];
      g.wb[s] = (int8_t)c[s];
    }
    return true;
  };
  bool ok = true;
  for (int i = 0; i < np; ++i)  // off-diagonal rectangles between row pairs
    for (int j = i + 1; j < np; ++j)
      ok &= add(128 * i, 128 * i + 64, 128 * j, 128 * j + 64, 0, 2, 0, 3, 1, 2, 1, 3);
  if (odd) {
    for (int i = 0; i < np; ++i)  // row pair x {last slab, dY}
      ok &= add(128 * i, 128 * i + 64, last, dy, 0, 2, 0, 3, 1, 2, 1, 3);
    // row pair triangles (2i,2i) (2i,2i+1) (2i+1,2i+1); the leftovers (last,last)
    // and (last,dY) ride in the first two groups' fourth wave
    for (int i = 0; i < np; ++i) {
      if (i == 0)
        ok &= add(0, 64, last, -1, 0, 0, 0, 1, 1, 1, 2, 2);
      else if (i == 1)
        ok &= add(128, 192, last, dy, 0, 0, 0, 1, 1, 1, 2, 3);
      else
        ok &= add(128 * i, 128 * i + 64, -1, -1, 0, 0, 0, 1, 1, 1, -1, -1);
    }
    if (np < 2) {  // nb == 1 or 3: the leftovers were not placed
      if (np == 0) ok &= add(last, dy, -1, -1, 0, 0, 0, 1, -1, -1, -1, -1);
      else ok &= add(last, dy, -1, -1, 0, 1, -1, -1, -1, -1, -1, -1);
    }
  } else {
    for (int i = 0; i < np; ++i)  // (2i,2i+1) (2i+1,2i+1) (2i,dY) (2i+1,dY)
      ok &= add(128 * i, 128 * i + 64, dy, -1, 0, 1, 1, 1, 0, 2, 1, 2);
    for (int i = 0; i < np; i += 4) {  // the (2i,2i) diagonals, four per group
      int b[4], a[4];
      for (int w = 0; w < 4; ++w) {
        const bool on = i + w < np;
        b[w] = on ? 128 * (i + w) : -1;
        a[w] = on ? w : -1;
      }
      ok &= add(b[0], b[1], b[2], b[3], a[0], a[0], a[1], a[1], a[2], a[2], a[3], a[3]);
    }
  }
  p->ngroups = n;
  return ok;
}

template <int BK, class Op, class Epi>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
void symred_kernel(Op op, Epi epi, SymPlan plan, int I, int J, int K, int k_chunk) {
  constexpr int SW = 256;      // staged columns (4 slabs)
  constexpr int SS = SW + 4;   // LDS row stride (floats)
  constexpr int BUF = BK * SS;
  constexpr int NR = BK / 8;   // staging k-rows per thread (32 threads per k-row)
  static_assert(BK % 8 == 0, "BK");
  __shared__ __attribute__((aligned(16))) float lds[2 * BUF];

  // XCD-aware 1-D grid over (chunk, group), as gemm_kernel's SPLITK path
  const int total = gridDim.x;
  const int b = blockIdx.x;
  const int xcd = b & 7, base8 = total >> 3, rem = total & 7;
  const int l = xcd * base8 + min(xcd, rem) + (b >> 3);
  const int ng = plan.ngroups;
  const int bz = l / ng;
  const SymGroup& G = plan.g[l - bz * ng];
  set_z(epi, bz);
  const int kbeg = bz * k_chunk;
  const int kend = min(K, kbeg + k_chunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;

  // staging: thread -> 8 consecutive staged columns (two float4 runs) of k-rows
  // tid/32 + 8*rr; a run never crosses a slab (64 % 8 == 0)
  const int scol = (tid & 31) * 8;
  const int sbase = G.base[scol >> 6];
  const int jcol = sbase >= 0 ? sbase + (scol & 63) : J;  // >= J stages zeros
  const typename Op::C c0 = op.col(jcol), c1 = op.col(jcol + 4);
  typename Op::St ra[NR][2];

  auto fetch = [&](int k0) {
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int k = k0 + (tid >> 5) + 8 * rr;
      const auto r = op.row(k);
      ra[rr][0] = op.stage(r, c0, k < kend);
      ra[rr][1] = op.stage(r, c1, k < kend);
    }
  };
  auto commit = [&](int buf) {
    float* s = lds + buf * BUF;
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int k = (tid >> 5) + 8 * rr;
      *reinterpret_cast<float4*>(s + k * SS + scol) = finish(ra[rr][0]);
      *reinterpret_cast<float4*>(s + k * SS + scol + 4) = finish(ra[rr][1]);
    }
  };

  const int sa = G.wa[wave], sb = G.wb[wave];
  const bool idle = sa < 0;
  const int ib = idle ? 0 : G.base[sa];  // row slabs are P slabs: column == row index
  const int jb = idle ? 0 : G.base[sb];
  const bool do_cs = !idle && ib == 0;
  const int aoff = 64 * (idle ? 0 : sa) + (lane & 31);
  const int boff = 64 * (idle ? 0 : sb) + (lane & 31);
  const int khalf = lane >> 5;

  f32x16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[x][y][r] = 0.f;
  float csum[2] = {0.f, 0.f};

  if (nk > 0) {
    fetch(kbeg);
    commit(0);
  }
  __syncthreads();

  // NT: column blocks of 32 the wave multiplies (1 when its second half lies
  // past J: a dY slab of cout_pad <= 32, e.g. conv3's 32 filters)
  auto step = [&](int kt, int cur, auto MF, auto CS, auto NTc) {
    constexpr bool mf = decltype(MF)::value;
    constexpr bool cs = decltype(CS)::value;
    constexpr int NT = decltype(NTc)::value;
    fetch(kbeg + (kt + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (mf) {
      const float* s = lds + cur * BUF;
      float a[2], bb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = s[khalf * SS + aoff + 32 * t];
        bb[t] = s[khalf * SS + boff + 32 * t];
      }
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        float an[2], bn[2];
        if (kk + 2 < BK) {
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            an[t] = s[(kk + 2 + khalf) * SS + aoff + 32 * t];
            bn[t] = s[(kk + 2 + khalf) * SS + boff + 32 * t];
          }
        }
        if constexpr (cs) {
#pragma unroll
          for (int tn = 0; tn < NT; ++tn) csum[tn] += bb[tn];
        }
#pragma unroll
        for (int tm = 0; tm < 2; ++tm)
#pragma unroll
          for (int tn = 0; tn < NT; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm], bb[tn], acc[tm][tn], 0, 0, 0);
        if (kk + 2 < BK) {
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            a[t] = an[t];
            bb[t] = bn[t];
          }
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    commit(cur ^ 1);
    __syncthreads();
  };
  using T = std::integral_constant<bool, true>;
  using F = std::integral_constant<bool, false>;
  using N2 = std::integral_constant<int, 2>;
  using N1 = std::integral_constant<int, 1>;
  const bool half = jb + 32 >= J;
  // wave-uniform loop variants: MFMAs (+ column sums) on 64 or 32 columns, or
  // staging only
  if (idle) {
    for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, F{}, F{}, N2{});
  } else if (do_cs) {
    if (half)
      for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, T{}, T{}, N1{});
    else
      for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, T{}, T{}, N2{});
  } else {
    if (half)
      for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, T{}, F{}, N1{});
    else
      for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, T{}, F{}, N2{});
  }
  if (idle) return;

  store_tile<2, 2>(epi, acc, ib, jb, lane, I, J);
  if (do_cs) {
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const float t = csum[tn] + __shfl_xor(csum[tn], 32);
      const int j = jb + tn * 32 + lane;
      if (lane < 32 && j < J) epi.colsum(j, t);
    }
  }
}

template <int BK>
constexpr int symred_lds_bytes() {
  return 2 * BK * (256 + 4) * 4;
}

template <int BK, class Op, class Epi>
inline void launch_symred(const Op& op, const Epi& e, const SymPlan& plan, int I, int J, int K,
                          int nchunk, int k_chunk, hipStream_t s) {
  hipLaunchKernelGGL((symred_kernel<BK, Op, Epi>), dim3(plan.ngroups * nchunk), dim3(256), 0, s, op,
                     e, plan, I, J, K, k_chunk);
}

}  // namespace acmi
