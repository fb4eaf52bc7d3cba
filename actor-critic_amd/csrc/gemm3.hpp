// The GEMM engine of gemm.hpp on the bf16 matrix cores with three-way split
// operands (bf16x3, see symred3.hpp for the arithmetic and its error bound):
//
//   C[i][j] = sum_k A(k, i) * B(k, j),  f32-accurate, six
//   v_mfma_f32_32x32x16_bf16 per 32x32 tile and 16 k (2.67x the f32 MFMA rate)
//
// Same operand concept (gemm_ops.hpp), thread->element staging map, split-K /
// live-tile grid, symmetric skip, epilogues (store_tile / store_tile_lds) and
// column-sum contract as gemm_kernel, so every launch_gemm<...> site can run
// either kernel (launch_mm picks by acmi_set_gemm_mode).  What differs is the
// LDS image, written at the commit as three bf16 parts of the staged values:
//  * i-contiguous operands: [part][k][i] bf16 rows of BM*2 bytes, 8-byte column
//    slots XOR-swizzled by k (sw_rows); fragments by ds_read_b64_tr_b16 (two per
//    32-column block and part), as in symred3.
//  * k-contiguous operands: [part][i][k] rows of BK*2 bytes, 16-byte k chunks
//    XOR-swizzled by i (sw_kc); fragments by one ds_read_b128 per 32-row block
//    and part (8 consecutive k of row i = the 32x32x16 operand map).
// Both images are bank-conflict free for their ds_write_b64 commits and their
// fragment reads (MI355X_MICROARCH.md §LDS lane groups; worked out in the
// comments of sw_rows / sw_kc).
// Column sums (COLSUM, i-contiguous B only) are summed in f32 from the staged
// values at the commit and reduced across the k-row threads through LDS.
//
// F16 (launch_gemm3_f16): the same kernel on f16x2 split operands (f16x2.hpp) --
// two f16 parts per operand scaled by the power of two of a published bound
// (amax_a, amax_b: f32 bit patterns in device memory), three MFMAs per product
// instead of six, the accumulators unscaled before the epilogue.
#pragma once

#include "f16x2.hpp"
#include "gemm.hpp"
#include "symred3.hpp"

namespace acmi {

// i-contiguous image: 8-byte slot s (4 bf16 columns) of k-row k.  A transposed
// read gives each 16-lane group 4 k-rows (q = k & 3) x 16 columns; a 32-lane
// half (two groups, 32 columns) must hit 32 distinct 8-byte slots of the
// 256-byte bank window.  Rows of >= 256 B: slot ^ 8q keeps the row's slots in
// their 32-slot window and separates the 4 rows; 128-B rows (2 per window):
// q and q + 2 share a window offset, so toggle the row half by (q >> 1); 64-B
// rows: the 4 rows already fill the window.
template <int RB>
__device__ __forceinline__ int sw_rows(int slot, int k) {
  const int q = k & 3;
  if constexpr (RB >= 256) return slot ^ (8 * q);
  else if constexpr (RB == 128) return slot ^ (8 * ((q >> 1) & 1));
  else return slot;
}

// k-contiguous image: 16-byte k chunk c of row i (BK = 16: 2 chunks, 32-B rows;
// BK = 32: 4 chunks, 64-B rows).  A ds_read_b128 lane group (16 lanes = 16
// rows i, one chunk) must hit 16 distinct slots of the 256-byte window:
// BK = 16 -> c ^ ((i >> 3) & 1), BK = 32 -> c ^ ((i >> 2) & 3) (checked for the
// four gfx950 groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... ).
template <int BK>
__device__ __forceinline__ int sw_kc(int c, int i) {
  if constexpr (BK == 16) return c ^ ((i >> 3) & 1);
  else return c ^ ((i >> 2) & 3);
}

template <int BM, int BN, int BK, int NP = 3>
constexpr int gemm3_lds_bytes() {
  return 2 * NP * (BM + BN) * BK * 2;
}
template <int BM, int BN, int BK, int NP = 3>
constexpr int gemm3_blocks_per_cu() {
  return std::min(8, 160 * 1024 / gemm3_lds_bytes<BM, BN, BK, NP>());
}

// one operand's LDS image: write a staged float4 run, read 32-wide fragments;
// NP = 3: bf16 h/m/l parts, NP = 2: f16 h/l parts of the values times sc
template <bool KC, int BX, int BK, int NP = 3>
struct X3Image {
  static constexpr int PART = BX * BK * 2;  // bytes per part
  static constexpr int BYTES = NP * PART;
  static constexpr int RB = KC ? BK * 2 : BX * 2;  // bytes per LDS row
  // commit of run v at (k, x): KC -> 4 consecutive k of row x; else 4
  // consecutive x of k-row k
  __device__ __forceinline__ static void write(char* s, int k, int x, const float4& f, float sc = 1.f) {
    uint2 h, m, l;
    if constexpr (NP == 3) {
      split3(f.x, f.y, h.x, m.x, l.x);
      split3(f.z, f.w, h.y, m.y, l.y);
    } else {
      split2(f.x, f.y, sc, h.x, m.x);
      split2(f.z, f.w, sc, h.y, m.y);
    }
    int off;
    if constexpr (KC) {
      off = x * RB + 16 * sw_kc<BK>(k >> 3, x) + 8 * ((k >> 2) & 1);
    } else {
      off = k * RB + 8 * sw_rows<RB>(x >> 2, k);
    }
    *reinterpret_cast<uint2*>(s + off) = h;
    *reinterpret_cast<uint2*>(s + PART + off) = m;
    if constexpr (NP == 3) *reinterpret_cast<uint2*>(s + 2 * PART + off) = l;
  }
  // byte offset (within a part) of lane's fragment for k-step ks (16 k) and the
  // 32-wide block starting at x0
  __device__ __forceinline__ static int frag_off(int lane, int ks, int x0) {
    if constexpr (KC) {
      const int x = x0 + (lane & 31);
      return x * RB + 16 * sw_kc<BK>(2 * ks + (lane >> 5), x);
    } else {
      const int q = (lane >> 2) & 3, p = lane & 3, g = (lane >> 4) & 1, kh = lane >> 5;
      const int k = 16 * ks + 8 * kh + q;
      return k * RB + 8 * sw_rows<RB>((x0 >> 2) + 4 * g + p, k);
    }
  }
  __device__ __forceinline__ static bf16x8 frag(const char* part, int off) {
    if constexpr (KC) {
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(part + off));
    } else {
      return cat8(ds_tr16(part + off), ds_tr16(part + off + 4 * RB));
    }
  }
};

template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM, class OpA, class OpB,
          class Epi, bool F16 = false>
__global__ __launch_bounds__(256)
// (occupancy of the three-part LDS image in both forms: the two-part image would
// allow more blocks, but its register budget then spills -- measured 30-390 VGPRs
// of spill and 1.4-3x the time at 64x128 .. 128x256)
__attribute__((amdgpu_waves_per_eu(gemm3_blocks_per_cu<BM, BN, BK, 3>())))
void gemm3_kernel(OpA opA, OpB opB, Epi epi, int I, int J, int K, int k_chunk, int sym_cols,
                  const unsigned* amax_a = nullptr, const unsigned* amax_b = nullptr) {
  using TL = Tile<BM, BN, BK, WTM, WTN>;
  static_assert(BK == 16 || BK == 32, "BK 16 or 32");
  static_assert(!COLSUM || !OpB::KCONTIG, "column sums need an i-contiguous B");
  constexpr int NP = F16 ? 2 : 3;
  using IA = X3Image<OpA::KCONTIG, BM, BK, NP>;
  using IB = X3Image<OpB::KCONTIG, BN, BK, NP>;
  float sa = 1.f, sb = 1.f;
  if constexpr (F16) {
    sa = f16x2_scale_of_bits(amax_a);
    sb = f16x2_scale_of_bits(amax_b);
  }
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if constexpr (SPLITK) {
    const int tx = (I + BM - 1) / BM, ty = (J + BN - 1) / BN;
    const int ssym = sym_cols > 0 ? sym_cols / BN : 0;
    int live = 0;
    for (int x = 0; x < tx; ++x) live += ty - min(x * BM / BN, ssym);
    const int total = gridDim.x;
    const int b = blockIdx.x;
    const int xcd = b & 7, base = total >> 3, rem = total & 7;
    const int l = xcd * base + min(xcd, rem) + (b >> 3);
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
  set_z(opA, bz);
  set_z(opB, bz);
  set_z(epi, bz);
  constexpr int NA = BM * BK / 4 / 256;
  constexpr int NB = BN * BK / 4 / 256;
  __shared__ __attribute__((aligned(16))) char lds[2 * (IA::BYTES + IB::BYTES)];

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

  // staging map of gemm_kernel (see there)
  constexpr int AK = BK / 4;
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

  auto fetch = [&](int k0) {
    if constexpr (OpA::KCONTIG) {
      const int k = k0 + (tid % AK) * 4;
      const auto c = opA.col(k);
#pragma unroll
      for (int v = 0; v < NA; ++v) ra[v] = opA.stage(rowA[v], c, k < kend);
    } else {
#pragma unroll
      for (int rr = 0; rr < NROWA; ++rr) {
        const int k = k0 + tid / TPRA + RSA * rr;
        const auto r = opA.row(k);
#pragma unroll
        for (int u = 0; u < RPRA; ++u) ra[rr * RPRA + u] = opA.stage(r, colA[u], k < kend);
      }
    }
    if constexpr (OpB::KCONTIG) {
      const int k = k0 + (tid % BKs) * 4;
      const auto c = opB.col(k);
#pragma unroll
      for (int v = 0; v < NB; ++v) rb[v] = opB.stage(rowB[v], c, k < kend);
    } else {
#pragma unroll
      for (int rr = 0; rr < NROWB; ++rr) {
        const int k = k0 + tid / TPRB + RSB * rr;
        const auto r = opB.row(k);
#pragma unroll
        for (int u = 0; u < RPRB; ++u) rb[rr * RPRB + u] = opB.stage(r, colB[u], k < kend);
      }
    }
  };

  // COLSUM: per-thread f32 sums of its staged B columns over its k-rows
  float csum[COLSUM ? 4 * RPRB : 1];
#pragma unroll
  for (int e = 0; e < (COLSUM ? 4 * RPRB : 1); ++e) csum[e] = 0.f;

  auto commit = [&](int buf) {
    char* As = lds + buf * IA::BYTES;
    char* Bs = lds + 2 * IA::BYTES + buf * IB::BYTES;
#pragma unroll
    for (int v = 0; v < NA; ++v) {
      const float4 x = finish(ra[v]);
      const int idx = tid + 256 * v;
      if constexpr (OpA::KCONTIG) {
        const int i = idx / (BK / 4);
        IA::write(As, (idx - i * (BK / 4)) * 4, i, x, sa);
      } else {
        IA::write(As, tid / TPRA + RSA * (v / RPRA), (tid % TPRA) * 4 + (v % RPRA) * TPRA * 4, x, sa);
      }
    }
#pragma unroll
    for (int v = 0; v < NB; ++v) {
      const float4 x = finish(rb[v]);
      const int idx = tid + 256 * v;
      if constexpr (OpB::KCONTIG) {
        const int j = idx / (BK / 4);
        IB::write(Bs, (idx - j * (BK / 4)) * 4, j, x, sb);
      } else {
        if constexpr (COLSUM) {
          const int u = v % RPRB;
          csum[4 * u] += x.x;
          csum[4 * u + 1] += x.y;
          csum[4 * u + 2] += x.z;
          csum[4 * u + 3] += x.w;
        }
        IB::write(Bs, tid / TPRB + RSB * (v / RPRB), (tid % TPRB) * 4 + (v % RPRB) * TPRB * 4, x, sb);
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

  if (nk > 0) {
    fetch(kbeg);
    commit(0);
  }
  __syncthreads();

  int aoff[BK / 16][WTM], boff[BK / 16][WTN];
#pragma unroll
  for (int ks = 0; ks < BK / 16; ++ks) {
#pragma unroll
    for (int tm = 0; tm < WTM; ++tm) aoff[ks][tm] = IA::frag_off(lane, ks, wm * WTM * 32 + tm * 32);
#pragma unroll
    for (int tn = 0; tn < WTN; ++tn) boff[ks][tn] = IB::frag_off(lane, ks, wn * WTN * 32 + tn * 32);
  }

  auto step = [&](int kt, int cur, auto MF) {
    constexpr bool mf = decltype(MF)::value;
    fetch(kbeg + (kt + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (mf) {
      const char* As = lds + cur * IA::BYTES;
      const char* Bs = lds + 2 * IA::BYTES + cur * IB::BYTES;
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 a[WTM][3], b[WTN][3];
#pragma unroll
        for (int pt = 0; pt < NP; ++pt) {
#pragma unroll
          for (int tm = 0; tm < WTM; ++tm) a[tm][pt] = IA::frag(As + pt * IA::PART, aoff[ks][tm]);
#pragma unroll
          for (int tn = 0; tn < WTN; ++tn) b[tn][pt] = IB::frag(Bs + pt * IB::PART, boff[ks][tn]);
        }
#pragma unroll
        for (int tm = 0; tm < WTM; ++tm)
#pragma unroll
          for (int tn = 0; tn < WTN; ++tn) {
            if constexpr (F16) {
              const f16x8 ah[2] = {__builtin_bit_cast(f16x8, a[tm][0]), __builtin_bit_cast(f16x8, a[tm][1])};
              const f16x8 bh[2] = {__builtin_bit_cast(f16x8, b[tn][0]), __builtin_bit_cast(f16x8, b[tn][1])};
              acc[tm][tn] = mfma_x2(ah, bh, acc[tm][tn]);
            } else {
              acc[tm][tn] = mfma_x3(a[tm], b[tn], acc[tm][tn]);
            }
          }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    commit(cur ^ 1);
    __syncthreads();
  };
  const int wrow0 = i0 + wm * WTM * 32, wcol0 = j0 + wn * WTN * 32, wcol1 = wcol0 + WTN * 32;
  const bool wave_idle =
      (sym_cols > 0 && wcol1 <= wrow0 && wcol1 <= sym_cols) || wrow0 >= I || wcol0 >= J;
  using MFon = std::integral_constant<bool, true>;
  using MFoff = std::integral_constant<bool, false>;
  if (!wave_idle) {
    for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, MFon{});
  } else {
    for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, MFoff{});
  }

  if constexpr (COLSUM) {
    // [k-row thread][BN columns] f32 sums through the (free) staging LDS
    constexpr int KT = 256 / TPRB;  // threads per column
    static_assert(KT * BN * 4 <= 2 * (IA::BYTES + IB::BYTES), "colsum LDS");
    float* cs = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int u = 0; u < RPRB; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        cs[(tid / TPRB) * BN + (tid % TPRB) * 4 + u * TPRB * 4 + e] = csum[4 * u + e];
    __syncthreads();
    if (bx == 0 && wm == 0) {
#pragma unroll
      for (int tn = 0; tn < WTN; ++tn) {
        const int c = wn * WTN * 32 + tn * 32 + (lane & 31);
        float t = 0.f;
        for (int r = 0; r < KT; ++r) t += cs[r * BN + c];
        const int j = j0 + c;
        if (lane < 32 && j < J) epi.colsum(j, t);
      }
    }
    __syncthreads();
  }

  if constexpr (F16) {
    const float inv = 1.0f / (sa * sb);  // exact: powers of two
#pragma unroll
    for (int a = 0; a < WTM; ++a)
#pragma unroll
      for (int b = 0; b < WTN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] *= inv;
  }
  if constexpr (has_ldst<Epi>::value && 2 * (IA::BYTES + IB::BYTES) >= 4 * 32 * 36 * 4) {
    __syncthreads();
    store_tile_lds<WTM, WTN>(epi, acc, i0 + wm * WTM * 32, j0 + wn * WTN * 32, lane,
                             reinterpret_cast<float*>(lds) + wave * 32 * 36, I, J);
  } else {
    store_tile<WTM, WTN>(epi, acc, i0 + wm * WTM * 32, j0 + wn * WTN * 32, lane, I, J);
  }
}

template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM, class OpA, class OpB,
          class Epi>
inline void launch_gemm3(const OpA& a, const OpB& b, const Epi& e, int I, int J, int K, int zdim,
                         int k_chunk, hipStream_t s, int sym_cols = 0) {
  dim3 grid(cdiv(I, BM), cdiv(J, BN), zdim);
  if (SPLITK) grid = dim3(live_tiles<BM, BN>(I, J, sym_cols) * zdim);
  hipLaunchKernelGGL((gemm3_kernel<BM, BN, BK, WTM, WTN, SPLITK, COLSUM, OpA, OpB, Epi>), grid,
                     dim3(256), 0, s, a, b, e, I, J, K, k_chunk, sym_cols, nullptr, nullptr);
}

// the f16x2 form (no split-K): amax_a / amax_b bound |A|, |B| (f32 bit patterns)
template <int BM, int BN, int BK, int WTM, int WTN, class OpA, class OpB, class Epi>
inline void launch_gemm3_f16(const OpA& a, const OpB& b, const Epi& e, int I, int J, int K,
                             const unsigned* amax_a, const unsigned* amax_b, hipStream_t s) {
  hipLaunchKernelGGL((gemm3_kernel<BM, BN, BK, WTM, WTN, false, false, OpA, OpB, Epi, true>),
                     dim3(cdiv(I, BM), cdiv(J, BN), 1), dim3(256), 0, s, a, b, e, I, J, K, 0, 0, amax_a,
                     amax_b);
}

// the f16x2 form with split-K and the symmetric skip (Gram matrices of tensors
// whose max a dX epilogue published)
template <int BM, int BN, int BK, int WTM, int WTN, class OpA, class OpB, class Epi>
inline void launch_gemm3_f16_splitk(const OpA& a, const OpB& b, const Epi& e, int I, int J, int K, int zdim,
                                    int k_chunk, const unsigned* amax_a, const unsigned* amax_b,
                                    hipStream_t s, int sym_cols = 0) {
  hipLaunchKernelGGL((gemm3_kernel<BM, BN, BK, WTM, WTN, true, false, OpA, OpB, Epi, true>),
                     dim3(live_tiles<BM, BN>(I, J, sym_cols) * zdim), dim3(256), 0, s, a, b, e, I, J, K, k_chunk,
                     sym_cols, amax_a, amax_b);
}

// launch_gemm's interface, run on gemm3_kernel (bf16x3, K-tile BK3) in
// ACMI_GEMM_X3 mode and on gemm_kernel (f32 MFMA, K-tile BK) otherwise
template <int BM, int BN, int BK, int WTM, int WTN, bool SPLITK, bool COLSUM, int BK3 = 16,
          class OpA, class OpB, class Epi>
inline void launch_mm(const OpA& a, const OpB& b, const Epi& e, int I, int J, int K, int zdim,
                      int k_chunk, hipStream_t s, int sym_cols = 0) {
  if (g_gemm_mode == ACMI_GEMM_X3)
    launch_gemm3<BM, BN, BK3, WTM, WTN, SPLITK, COLSUM>(a, b, e, I, J, K, zdim, k_chunk, s, sym_cols);
  else
    launch_gemm<BM, BN, BK, WTM, WTN, SPLITK, COLSUM>(a, b, e, I, J, K, zdim, k_chunk, s, sym_cols);
}

}  // namespace acmi
