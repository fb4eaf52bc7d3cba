// Persistent ("stream") variant of the f32-MFMA GEMM for short-K products
// (conv forwards, conv input gradients: K = 256..1568, thousands of row
// tiles).  With one tile per block such a launch pays a full load latency in
// every block's prologue and idles the MFMAs during every epilogue; here each
// block walks the tiles t = blockIdx.x, blockIdx.x + gridDim.x, ... as ONE
// flattened sequence of K-tiles, so the staging loads of the next K-tile —
// including the first K-tile of the next output tile — are always in flight
// across the current MFMAs and the epilogue.  Same operand/epilogue concepts,
// LDS images, fragment maps and numerics (k-ordered fmaf chains) as
// gemm_kernel (gemm.hpp); no split-K, no column sums, no symmetric skip.
#pragma once

#include "gemm.hpp"

namespace acmi {

template <int BM, int BN, int BK, int WTM, int WTN, class OpA, class OpB, class Epi>
__global__ __launch_bounds__(256) void gemm_stream_kernel(OpA opA, OpB opB, Epi epi, int I, int J,
                                                          int K, int zdim) {
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
  const int tx = (I + BM - 1) / BM, ty = (J + BN - 1) / BN;
  const int ntile = tx * ty * zdim;
  const int nk = (K + BK - 1) / BK;
  const int G = gridDim.x;
  if ((int)blockIdx.x >= ntile || nk == 0) return;

  // same staging maps as gemm_kernel
  constexpr int AK = BK / 4;
  constexpr int BKs = BK / 4;
  constexpr int TPRA = BM / 4 >= 32 ? 32 : BM / 4, RPRA = BM / 4 / TPRA, RSA = 256 / TPRA;
  constexpr int TPRB = BN / 4 >= 32 ? 32 : BN / 4, RPRB = BN / 4 / TPRB, RSB = 256 / TPRB;
  constexpr int NROWA = OpA::KCONTIG ? 1 : BK / RSA;
  constexpr int NROWB = OpB::KCONTIG ? 1 : BK / RSB;
  static_assert(OpA::KCONTIG || (BK % RSA == 0 && NROWA * RPRA == NA), "A staging map");
  static_assert(OpB::KCONTIG || (BK % RSB == 0 && NROWB * RPRB == NB), "B staging map");

  typename OpA::St ra[NA];
  typename OpB::St rb[NB];
  typename OpA::R rowA[OpA::KCONTIG ? NA : 1];
  typename OpA::C colA[OpA::KCONTIG ? 1 : RPRA];
  typename OpB::R rowB[OpB::KCONTIG ? NB : 1];
  typename OpB::C colB[OpB::KCONTIG ? 1 : RPRB];

  // tile t -> (x, y, z): z slowest so consecutive tiles share z's B operand
  auto decode = [&](int t, int& x, int& y, int& z) {
    z = t / (tx * ty);
    const int r = t - z * tx * ty;
    y = r / tx;
    x = r - y * tx;
  };
  // per-tile address hoists of the FETCH side; past the last tile the fetch
  // re-reads the last tile (valid addresses, results never committed to a
  // computed tile)
  auto hoist = [&](int t) {
    int x, y, z;
    decode(min(t, ntile - 1), x, y, z);
    set_z(opA, z);
    set_z(opB, z);
    const int i0 = x * BM, j0 = y * BN;
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
  };
  auto fetch = [&](int k0) {
    if constexpr (OpA::KCONTIG) {
      const int k = k0 + (tid % AK) * 4;
      const auto c = opA.col(k);
#pragma unroll
      for (int v = 0; v < NA; ++v) ra[v] = opA.stage(rowA[v], c, k < K);
    } else {
#pragma unroll
      for (int rr = 0; rr < NROWA; ++rr) {
        const int k = k0 + tid / TPRA + RSA * rr;
        const auto r = opA.row(k);
#pragma unroll
        for (int u = 0; u < RPRA; ++u) ra[rr * RPRA + u] = opA.stage(r, colA[u], k < K);
      }
    }
    if constexpr (OpB::KCONTIG) {
      const int k = k0 + (tid % BKs) * 4;
      const auto c = opB.col(k);
#pragma unroll
      for (int v = 0; v < NB; ++v) rb[v] = opB.stage(rowB[v], c, k < K);
    } else {
#pragma unroll
      for (int rr = 0; rr < NROWB; ++rr) {
        const int k = k0 + tid / TPRB + RSB * rr;
        const auto r = opB.row(k);
#pragma unroll
        for (int u = 0; u < RPRB; ++u) rb[rr * RPRB + u] = opB.stage(r, colB[u], k < K);
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
  auto zero_acc = [&]() {
#pragma unroll
    for (int a = 0; a < WTM; ++a)
#pragma unroll
      for (int b = 0; b < WTN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  };
  zero_acc();

  const int arow = wm * WTM * 32 + (lane & 31);
  const int brow = wn * WTN * 32 + (lane & 31);
  const int khalf = lane >> 5;

  // compute position (ct, ck) and fetch position (ft, fk) one K-tile ahead
  int ct = blockIdx.x, ck = 0;
  int ft = ct, fk = 0;
  hoist(ft);
  fetch(0);
  commit(0);
  if (++fk == nk) {
    fk = 0;
    ft += G;
    hoist(ft);
  }
  {
    int x, y, z;
    decode(ct, x, y, z);
    set_z(epi, z);
  }
  __syncthreads();

  int cur = 0;
  while (ct < ntile) {
    fetch(fk * BK);  // next K-tile (possibly of the next tile, or past the end)
    __builtin_amdgcn_sched_barrier(0);
    const float* As = lds + cur * ABUF;
    const float* Bs = lds + 2 * ABUF + cur * BBUF;
    float a[WTM], b[WTN];
#pragma unroll
    for (int tm = 0; tm < WTM; ++tm) a[tm] = As[khalf * SA + arow + tm * 32];
#pragma unroll
    for (int tn = 0; tn < WTN; ++tn) b[tn] = Bs[khalf * SB + brow + tn * 32];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float an[WTM], bn[WTN];
      if (kk + 2 < BK) {
#pragma unroll
        for (int tm = 0; tm < WTM; ++tm) an[tm] = As[(kk + 2 + khalf) * SA + arow + tm * 32];
#pragma unroll
        for (int tn = 0; tn < WTN; ++tn) bn[tn] = Bs[(kk + 2 + khalf) * SB + brow + tn * 32];
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
    __builtin_amdgcn_sched_barrier(0);
    if (++ck == nk) {
      // epilogue of tile ct while the next tile's first loads are in flight
      int x, y, z;
      decode(ct, x, y, z);
      store_tile<WTM, WTN>(epi, acc, x * BM + wm * WTM * 32, y * BN + wn * WTN * 32, lane, I, J);
      zero_acc();
      ck = 0;
      ct += G;
      if (ct < ntile) {
        decode(ct, x, y, z);
        set_z(epi, z);
      }
    }
    commit(cur ^ 1);
    if (++fk == nk) {
      fk = 0;
      ft += G;
      hoist(ft);
    }
    __syncthreads();
    cur ^= 1;
  }
}

// grid = min(tiles, resident blocks): 256 CUs x blocks per CU (LDS-bound)
template <int BM, int BN, int BK, int WTM, int WTN, class OpA, class OpB, class Epi>
inline void launch_gemm_stream(const OpA& a, const OpB& b, const Epi& e, int I, int J, int K,
                               int zdim, hipStream_t s) {
  const long long ntile = (long long)cdiv(I, BM) * cdiv(J, BN) * zdim;
  const int slots = 256 * gemm_blocks_per_cu<BM, BN, BK, OpA::KCONTIG, OpB::KCONTIG>();
  const int grid = (int)std::min<long long>(ntile, slots);
  if (grid <= 0) return;
  hipLaunchKernelGGL((gemm_stream_kernel<BM, BN, BK, WTM, WTN, OpA, OpB, Epi>), dim3(grid),
                     dim3(256), 0, s, a, b, e, I, J, K, zdim);
}

}  // namespace acmi
