// Slab-grouped symmetric reduction [P;1]^T [P | dY] on the bf16 matrix cores
// with three-way split operands ("bf16x3"): fp32-accurate, 2.67x the f32-MFMA
// issue rate.
//
// Every f32 operand value x is split at the LDS commit into three bf16 terms
//   h = bf16_rn(x),  m = bf16_rn(x - h),  l = bf16_rn(x - h - m)
// (both subtractions are exact in f32), so |x - (h + m + l)| <= 2^-24 |x|: the
// split itself is as accurate as an f32 value.  Each 32x32x16 product tile then
// takes the six v_mfma_f32_32x32x16_bf16 of the terms with i + j <= 2
//   l*h + h*l + m*m + m*h + h*m + h*h     (small terms first)
// into one f32 accumulator; the three dropped terms (m*l, l*m, l*l) are
// <= 2^-24 |a||b| together, i.e. below f32 rounding of the product, and every
// bf16 x bf16 product is exact in the MFMA's f32 arithmetic.  The result is an
// f32 dot product with f32-class error (checked against float64 in
// tests/test_gpu_kernels.py and the symred A/B probe), not a bf16 one.
// Rate: 6 x 32 cycles per 32x32x16 tile vs 8 x 64 for the same K on
// v_mfma_f32_32x32x2_f32 (MI355X_MICROARCH.md constants table).
//
// Same slab plan (sym_plan), grid, staging loads, split-K partial layout and
// column-sum contract as symred_kernel (symred.hpp), so finalize_wgrad_kernel is
// shared.  What differs:
//  * LDS image: per stage of BK = 16 k-rows, three parts (h, m, l), each
//    [16 k][256 columns] of bf16 (512-byte rows) with 8-byte column slots
//    XOR-swizzled by 8*(k & 3): the 16-byte commit stores (8 lanes of one
//    k-row) and the ds_read_b64_tr_b16 transposed fragment reads (4 k-rows x 16
//    columns per 16 lanes) are both bank-conflict free.  24 KB per stage, 48 KB
//    double-buffered -> 3 blocks per CU.
//  * Fragments come from ds_read_b64_tr_b16 (cdna_hip_programming.md T10): two
//    per 32-column block and part give lane l the 8 consecutive k of column
//    l & 31 that the 32x32x16 operand map wants (A[r][8h + e], B[8h + e][r]).
//  * Column sums (the homogeneous row) are summed in f32 from the staged
//    values at the commit (each thread: its 8 columns over its k-rows), then
//    reduced over the 8 k-row threads of a column through LDS at the end.
#pragma once

#include <stdlib.h>

#include "symred.hpp"

namespace acmi {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

// (a, b) -> packed bf16 pair, round-to-nearest-even (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const f32x2v v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
}

// three-term split of the pair (a, b): h + m + l == (a, b) to 2^-24 relative
__device__ __forceinline__ void split3(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = pk_bf16(a, b);
  const float ra = a - __uint_as_float(h << 16);
  const float rb = b - __uint_as_float(h & 0xffff0000u);
  m = pk_bf16(ra, rb);
  const float sa = ra - __uint_as_float(m << 16);
  const float sb = rb - __uint_as_float(m & 0xffff0000u);
  l = pk_bf16(sa, sb);
}

__device__ __forceinline__ s16x4 ds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat8(s16x4 a, s16x4 b) {
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// six-product bf16x3 step on one accumulator
__device__ __forceinline__ f32x16 mfma_x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
  return c;
}

constexpr int kX3Rows = 16;                 // k-rows per stage
constexpr int kX3RowBytes = 512;            // 256 bf16 columns
constexpr int kX3Part = kX3Rows * kX3RowBytes;
constexpr int kX3Buf = 3 * kX3Part;         // h, m, l
constexpr int symred3_lds_bytes() { return 2 * kX3Buf; }

template <class Op, class Epi, int DBG = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
void symred3_kernel(Op op, Epi epi, SymPlan plan, int I, int J, int K, int k_chunk) {
  constexpr int BK = kX3Rows;
  constexpr int NR = BK / 8;  // staging k-rows per thread (32 threads per k-row)
  __shared__ __attribute__((aligned(16))) char lds[2 * kX3Buf];

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

  // staging: thread -> 8 consecutive staged columns (16-byte chunk c16 of a
  // 512-byte LDS row) of k-rows tid/32 + 8*rr
  const int c16 = tid & 31;
  const int scol = c16 * 8;
  const int sbase = G.base[scol >> 6];
  const int jcol = sbase >= 0 ? sbase + (scol & 63) : J;  // >= J stages zeros
  const typename Op::CB c0 = op.col_base(jcol), c1 = op.col_base(jcol + 4);
  typename Op::St ra[NR][2];
  float csum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) csum[e] = 0.f;
  // rows kbeg + tid/32 + 8rr, advanced BK per fetch (fetches run in k order)
  typename Op::It it[NR];
#pragma unroll
  for (int rr = 0; rr < NR; ++rr) it[rr] = op.iter(kbeg + (tid >> 5) + 8 * rr);

  auto fetch = [&](int k0) {
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int k = k0 + (tid >> 5) + 8 * rr;
      ra[rr][0] = op.stage_it(it[rr], c0, k < kend);
      ra[rr][1] = op.stage_it(it[rr], c1, k < kend);
      op.template advance<BK>(it[rr]);
    }
  };
  auto commit = [&](int buf) {
    char* s = lds + buf * kX3Buf;
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int k = (tid >> 5) + 8 * rr;
      const float4 x0 = finish(ra[rr][0]);
      const float4 x1 = finish(ra[rr][1]);
      csum[0] += x0.x;
      csum[1] += x0.y;
      csum[2] += x0.z;
      csum[3] += x0.w;
      csum[4] += x1.x;
      csum[5] += x1.y;
      csum[6] += x1.z;
      csum[7] += x1.w;
      uint4 h, m, lo;
      if constexpr (DBG == 1) {  // timing probe: no split (wrong numerics)
        h = make_uint4(pk_bf16(x0.x, x0.y), pk_bf16(x0.z, x0.w), pk_bf16(x1.x, x1.y),
                       pk_bf16(x1.z, x1.w));
        m = h;
        lo = h;
      } else {
        split3(x0.x, x0.y, h.x, m.x, lo.x);
        split3(x0.z, x0.w, h.y, m.y, lo.y);
        split3(x1.x, x1.y, h.z, m.z, lo.z);
        split3(x1.z, x1.w, h.w, m.w, lo.w);
      }
      const int off = k * kX3RowBytes + 16 * (c16 ^ (4 * (k & 3)));
      *reinterpret_cast<uint4*>(s + off) = h;
      *reinterpret_cast<uint4*>(s + kX3Part + off) = m;
      *reinterpret_cast<uint4*>(s + 2 * kX3Part + off) = lo;
    }
  };

  const int sa = G.wa[wave], sb = G.wb[wave];
  const bool idle = sa < 0 || DBG == 2;  // DBG 2: timing probe without MFMAs
  const int ib = idle ? 0 : G.base[sa];  // row slabs are P slabs: column == row index
  const int jb = idle ? 0 : G.base[sb];
  const bool do_cs = !idle && ib == 0;
  // transposed-read address of lane l inside a 32-column block: group g =
  // (l>>4)&1 -> columns 16g.., lane 4q+p -> k-row 8h+q, columns 4p..4p+3 (one
  // 8-byte slot), swizzled like the commit (8-byte slot ^ 8q)
  const int q = (lane >> 2) & 3, p = lane & 3, g = (lane >> 4) & 1, kh = lane >> 5;
  auto slot_off = [&](int colblock) {  // colblock: first staged column (multiple of 32)
    const int slot = (colblock >> 2) + 4 * g + p;
    return (8 * kh + q) * kX3RowBytes + 8 * (slot ^ (8 * q));
  };
  const int aoff0 = slot_off(64 * (idle ? 0 : sa)), aoff1 = slot_off(64 * (idle ? 0 : sa) + 32);
  const int boff0 = slot_off(64 * (idle ? 0 : sb)), boff1 = slot_off(64 * (idle ? 0 : sb) + 32);

  f32x16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[x][y][r] = 0.f;

  if (nk > 0) {
    fetch(kbeg);
    commit(0);
  }
  __syncthreads();

  auto step = [&](int kt, int cur, auto MF, auto NTc) {
    constexpr bool mf = decltype(MF)::value;
    constexpr int NT = decltype(NTc)::value;
    fetch(kbeg + (kt + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (mf) {
      const char* s = lds + cur * kX3Buf;
      bf16x8 a[2][3], bb[2][3];
#pragma unroll
      for (int pt = 0; pt < 3; ++pt) {
        const char* sp = s + pt * kX3Part;
        a[0][pt] = cat8(ds_tr16(sp + aoff0), ds_tr16(sp + aoff0 + 4 * kX3RowBytes));
        a[1][pt] = cat8(ds_tr16(sp + aoff1), ds_tr16(sp + aoff1 + 4 * kX3RowBytes));
        bb[0][pt] = cat8(ds_tr16(sp + boff0), ds_tr16(sp + boff0 + 4 * kX3RowBytes));
        if constexpr (NT == 2)
          bb[1][pt] = cat8(ds_tr16(sp + boff1), ds_tr16(sp + boff1 + 4 * kX3RowBytes));
      }
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < NT; ++tn) acc[tm][tn] = mfma_x3(a[tm], bb[tn], acc[tm][tn]);
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
  if (idle) {
    for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, F{}, N2{});
  } else if (half) {
    for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, T{}, N1{});
  } else {
    for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, T{}, N2{});
  }

  // column sums: [8 k-row threads][256 columns] through the (now free) LDS
  float* cs = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[(tid >> 5) * 256 + scol + e] = csum[e];
  __syncthreads();
  if (idle) return;
  store_tile<2, 2>(epi, acc, ib, jb, lane, I, J);
  if (do_cs) {
    const int col = 64 * sb + lane;
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) t += cs[r * 256 + col];
    if (jb + lane < J) epi.colsum(jb + lane, t);
  }
}

// Interleaved variant: loads run two K-tiles ahead, and the three-way split
// and LDS commit of tile kt+1 (already in registers) are issued between the
// MFMAs of tile kt (sched_group_barrier: the split VALU fills the MFMA gaps of
// the same wave instead of a separate commit phase after them).  One barrier
// per K-tile as before: buffer cur^1 was last read in step kt-1.
template <class Op, class Epi>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
void symred3i_kernel(Op op, Epi epi, SymPlan plan, int I, int J, int K, int k_chunk) {
  constexpr int BK = kX3Rows;
  constexpr int NR = BK / 8;
  __shared__ __attribute__((aligned(16))) char lds[2 * kX3Buf];

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
  const int c16 = tid & 31;
  const int scol = c16 * 8;
  const int sbase = G.base[scol >> 6];
  const int jcol = sbase >= 0 ? sbase + (scol & 63) : J;
  const typename Op::CB c0 = op.col_base(jcol), c1 = op.col_base(jcol + 4);
  typename Op::St ra[2][NR][2];
  float csum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) csum[e] = 0.f;
  typename Op::It it[NR];
#pragma unroll
  for (int rr = 0; rr < NR; ++rr) it[rr] = op.iter(kbeg + (tid >> 5) + 8 * rr);

  auto fetch = [&](int k0, auto S) {
    constexpr int set = decltype(S)::value;
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int k = k0 + (tid >> 5) + 8 * rr;
      ra[set][rr][0] = op.stage_it(it[rr], c0, k < kend);
      ra[set][rr][1] = op.stage_it(it[rr], c1, k < kend);
      op.template advance<BK>(it[rr]);
    }
  };
  auto commit = [&](int buf, auto S) {
    constexpr int set = decltype(S)::value;
    char* s = lds + buf * kX3Buf;
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int k = (tid >> 5) + 8 * rr;
      const float4 x0 = finish(ra[set][rr][0]);
      const float4 x1 = finish(ra[set][rr][1]);
      csum[0] += x0.x;
      csum[1] += x0.y;
      csum[2] += x0.z;
      csum[3] += x0.w;
      csum[4] += x1.x;
      csum[5] += x1.y;
      csum[6] += x1.z;
      csum[7] += x1.w;
      uint4 h, m, lo;
      split3(x0.x, x0.y, h.x, m.x, lo.x);
      split3(x0.z, x0.w, h.y, m.y, lo.y);
      split3(x1.x, x1.y, h.z, m.z, lo.z);
      split3(x1.z, x1.w, h.w, m.w, lo.w);
      const int off = k * kX3RowBytes + 16 * (c16 ^ (4 * (k & 3)));
      *reinterpret_cast<uint4*>(s + off) = h;
      *reinterpret_cast<uint4*>(s + kX3Part + off) = m;
      *reinterpret_cast<uint4*>(s + 2 * kX3Part + off) = lo;
    }
  };

  const int sa = G.wa[wave], sb = G.wb[wave];
  const bool idle = sa < 0;
  const int ib = idle ? 0 : G.base[sa];
  const int jb = idle ? 0 : G.base[sb];
  const bool do_cs = !idle && ib == 0;
  const int q = (lane >> 2) & 3, p = lane & 3, g = (lane >> 4) & 1, kh = lane >> 5;
  auto slot_off = [&](int colblock) {
    const int slot = (colblock >> 2) + 4 * g + p;
    return (8 * kh + q) * kX3RowBytes + 8 * (slot ^ (8 * q));
  };
  const int aoff0 = slot_off(64 * (idle ? 0 : sa)), aoff1 = slot_off(64 * (idle ? 0 : sa) + 32);
  const int boff0 = slot_off(64 * (idle ? 0 : sb)), boff1 = slot_off(64 * (idle ? 0 : sb) + 32);

  f32x16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[x][y][r] = 0.f;

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if (nk > 0) {
    fetch(kbeg, S0{});
    fetch(kbeg + BK, S1{});
    commit(0, S0{});
  }
  __syncthreads();

  // step kt: MFMAs on buffer cur; tile kt+1 (register set SN) split + written
  // to buffer cur^1 in the MFMA gaps; tile kt+2's loads into set SN^1
  auto step = [&](int kt, int cur, auto MF, auto NTc, auto SN) {
    constexpr bool mf = decltype(MF)::value;
    constexpr int NT = decltype(NTc)::value;
    constexpr int sn = decltype(SN)::value;
    fetch(kbeg + (kt + 2) * BK, std::integral_constant<int, sn ^ 1>{});
    if constexpr (mf) {
      const char* s = lds + cur * kX3Buf;
      bf16x8 a[2][3], bb[2][3];
#pragma unroll
      for (int pt = 0; pt < 3; ++pt) {
        const char* sp = s + pt * kX3Part;
        a[0][pt] = cat8(ds_tr16(sp + aoff0), ds_tr16(sp + aoff0 + 4 * kX3RowBytes));
        a[1][pt] = cat8(ds_tr16(sp + aoff1), ds_tr16(sp + aoff1 + 4 * kX3RowBytes));
        bb[0][pt] = cat8(ds_tr16(sp + boff0), ds_tr16(sp + boff0 + 4 * kX3RowBytes));
        if constexpr (NT == 2)
          bb[1][pt] = cat8(ds_tr16(sp + boff1), ds_tr16(sp + boff1 + 4 * kX3RowBytes));
      }
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < NT; ++tn) acc[tm][tn] = mfma_x3(a[tm], bb[tn], acc[tm][tn]);
      if (kt + 1 < nk) commit(cur ^ 1, SN);
      // interleave: loads, fragment reads, then one MFMA per 5 VALU
      __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 6 * (2 + NT), 0);
#pragma unroll
      for (int i = 0; i < 6 * 2 * NT; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
      }
    } else {
      if (kt + 1 < nk) commit(cur ^ 1, SN);
    }
    __syncthreads();
  };
  using T = std::integral_constant<bool, true>;
  using F = std::integral_constant<bool, false>;
  using N2 = std::integral_constant<int, 2>;
  using N1 = std::integral_constant<int, 1>;
  const bool half = jb + 32 >= J;
  auto run = [&](auto MF, auto NTc) {
    for (int kt = 0; kt < nk; kt += 2) {
      step(kt, 0, MF, NTc, S1{});
      if (kt + 1 < nk) step(kt + 1, 1, MF, NTc, S0{});
    }
  };
  if (idle) run(F{}, N2{});
  else if (half) run(T{}, N1{});
  else run(T{}, N2{});

  float* cs = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[(tid >> 5) * 256 + scol + e] = csum[e];
  __syncthreads();
  if (idle) return;
  store_tile<2, 2>(epi, acc, ib, jb, lane, I, J);
  if (do_cs) {
    const int col = 64 * sb + lane;
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) t += cs[r * 256 + col];
    if (jb + lane < J) epi.colsum(jb + lane, t);
  }
}

// ACMI_SYMRED=i selects symred3i_kernel (A/B timing); =n / =m the no-split /
// no-MFMA timing probes of symred3_kernel (wrong results)
inline int symred_variant() {
  static const int v = [] {
    const char* e = getenv("ACMI_SYMRED");
    return !e ? 0 : e[0] == 'i' ? 1 : e[0] == 'n' ? 2 : e[0] == 'm' ? 3 : 0;
  }();
  return v;
}

template <class Op, class Epi>
inline void launch_symred3(const Op& op, const Epi& e, const SymPlan& plan, int I, int J, int K,
                           int nchunk, int k_chunk, hipStream_t s) {
  const int v = symred_variant();
  if (v == 1)
    hipLaunchKernelGGL((symred3i_kernel<Op, Epi>), dim3(plan.ngroups * nchunk), dim3(256), 0, s, op,
                       e, plan, I, J, K, k_chunk);
  else if (v == 2)
    hipLaunchKernelGGL((symred3_kernel<Op, Epi, 1>), dim3(plan.ngroups * nchunk), dim3(256), 0, s, op,
                       e, plan, I, J, K, k_chunk);
  else if (v == 3)
    hipLaunchKernelGGL((symred3_kernel<Op, Epi, 2>), dim3(plan.ngroups * nchunk), dim3(256), 0, s, op,
                       e, plan, I, J, K, k_chunk);
  else
    hipLaunchKernelGGL((symred3_kernel<Op, Epi>), dim3(plan.ngroups * nchunk), dim3(256), 0, s, op,
                       e, plan, I, J, K, k_chunk);
}

}  // namespace acmi
