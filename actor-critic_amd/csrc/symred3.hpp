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

#include <algorithm>
#include <functional>
#include <map>
#include <mutex>
#include <random>
#include <vector>

#include "f16x2.hpp"  // split3, mfma_x3, ds_tr16, cat8 (split16.hpp); split2, mfma_x2
#include "symred.hpp"

namespace acmi {

constexpr int kX3Rows = 16;                 // k-rows per stage
constexpr int kX3RowBytes = 512;            // 256 bf16 columns
constexpr int kX3Part = kX3Rows * kX3RowBytes;
constexpr int kX3Buf = 3 * kX3Part;         // h, m, l
constexpr int symred3_lds_bytes() { return 2 * kX3Buf; }

template <class Op, class Epi>
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

// ---------------------------------------------------------------------------
// Six-slab groups: 8 waves (512 threads), two 64x64 sub-tiles per wave, six
// staged slabs (384 columns) per block.  The no-MFMA probe of symred3_kernel
// (ACMI_SYMRED=m: 0.87 of 1.50 ms at conv2's shape) shows the staging gather
// alone is as long as the MFMA work: with one sub-tile per staged slab the
// loads would need ~10 TB/s from L2 to keep the matrix cores busy.  Covering
// the needed sub-tiles with 6-slab groups of <= 16 sub-tiles takes 3 groups
// for conv2 / the heads (8 P slabs + dY; 11 groups of 4 slabs before) and 4
// for conv3 (9 P slabs + dY; 14 before): ~2.4x fewer staged bytes per MFMA.
// 72 KB of LDS and 2 x 64 accumulator registers per wave: one block per CU.
// The slab sets are fixed coverings of the slab pairs (found offline by a
// local search over 6-subsets: every pair of slabs, the dY slab included, lies
// in some set); sym_plan6 assigns the sub-tiles to them by bipartite matching
// with a balanced per-group capacity.
// ---------------------------------------------------------------------------
constexpr int kSixSlabs = 6;
constexpr int kSixRowBytes = kSixSlabs * 64 * 2;      // 768
constexpr int kSixPart = kX3Rows * kSixRowBytes;      // 12 KB
constexpr int kSixBuf = 3 * kSixPart;                 // 36 KB
constexpr int symred6_lds_bytes() { return 2 * kSixBuf; }

struct SymGroup6 {
  int16_t base[kSixSlabs];  // first [P | dY] column of each staged slab
  int8_t ra[8][2];          // per wave and tile: staged slab of the rows (-1: no tile)
  int8_t cb[8][2];          // per wave and tile: staged slab of the columns
};
constexpr int kSym6MaxGroups = 48;
struct SymPlan6 {
  int ngroups;
  SymGroup6 g[kSym6MaxGroups];
};

inline bool sym_plan6(int K, int cout_pad, SymPlan6* p) {
  if (cout_pad > 64 || cout_pad <= 0 || (K != 512 && K != 576)) return false;
  static const int8_t sets8[3][6] = {{0, 1, 2, 4, 6, 8}, {1, 2, 3, 5, 7, 8}, {0, 3, 4, 5, 6, 7}};
  static const int8_t sets9[4][6] = {
      {0, 1, 2, 5, 7, 9}, {1, 3, 4, 6, 7, 8}, {0, 2, 3, 4, 6, 8}, {3, 4, 5, 6, 8, 9}};
  const int nb = K / 64, ng = nb == 8 ? 3 : 4;
  const int8_t(*sets)[6] = nb == 8 ? sets8 : sets9;
  // sub-tiles (a, b), a <= b <= nb (b == nb: the dY slab)
  int ta[64], tb[64], nt = 0;
  for (int a = 0; a < nb; ++a)
    for (int b = a; b <= nb; ++b) ta[nt] = a, tb[nt] = b, ++nt;
  auto in = [&](int g, int x) {
    for (int i = 0; i < 6; ++i)
      if (sets[g][i] == x) return i;
    return -1;
  };
  int owner[64];
  for (int cap = (nt + ng - 1) / ng; cap <= 16; ++cap) {
    int load[8] = {0};
    for (int t = 0; t < nt; ++t) owner[t] = -1;
    // augmenting paths (Kuhn) with capacity cap per group
    bool ok = true;
    for (int t = 0; t < nt && ok; ++t) {
      int seen[8];
      std::function<bool(int)> aug = [&](int u) -> bool {
        for (int g = 0; g < ng; ++g) {
          if (seen[g] || in(g, ta[u]) < 0 || in(g, tb[u]) < 0) continue;
          seen[g] = 1;
          if (load[g] < cap) {
            owner[u] = g;
            ++load[g];
            return true;
          }
          for (int v = 0; v < nt; ++v)
            if (owner[v] == g && aug(v)) {
              owner[u] = g;
              return true;
            }
        }
        return false;
      };
      for (int g = 0; g < 8; ++g) seen[g] = 0;
      ok = aug(t);
    }
    if (!ok) continue;
    p->ngroups = ng;
    for (int g = 0; g < ng; ++g) {
      SymGroup6& G = p->g[g];
      for (int i = 0; i < 6; ++i) G.base[i] = (int16_t)(sets[g][i] == nb ? K : 64 * sets[g][i]);
      for (int w = 0; w < 8; ++w) G.ra[w][0] = G.ra[w][1] = G.cb[w][0] = G.cb[w][1] = -1;
      int n = 0;
      for (int pass = 0; pass < 2; ++pass)  // P x P sub-tiles first, dY sub-tiles last
        for (int t = 0; t < nt; ++t) {
          if (owner[t] != g || (tb[t] == nb) != (pass == 1)) continue;
          const int w = n % 8, s = n / 8;
          G.ra[w][s] = (int8_t)in(g, ta[t]);
          G.cb[w][s] = (int8_t)in(g, tb[t]);
          ++n;
        }
    }
    return true;
  }
  return false;
}

// Six-slab groups for any K (fc4: K = 1568, dY 512 wide): the [P | dY] column
// space is cut into 64-column slabs at multiples of 64 (a slab may straddle the
// P/dY boundary; rows >= K of a row slab are computed and dropped by the store
// mask).  Needed sub-tiles: (a, b), b >= a, a a slab holding P rows.  Groups are
// built greedily: every slab seeds a candidate six-set grown by the slab adding
// the most uncovered sub-tiles; the candidate with the most (capped at 16) wins
// and takes its 16 hardest sub-tiles (those whose slabs have the fewest other
// uncovered ones), full-width first so a half-width tile never sits in slot 0
// under a full one.  Five seeded restarts (shuffled tie order), the fewest
// groups kept: fc4 (1568 | 512) gets ~43 groups for its 525 sub-tiles.  Coverage
// is checked by acmi_selftest_plans; plans are cached per (K, cout_pad).
inline bool sym_plan6_greedy_build(int K, int cout_pad, SymPlan6* out) {
  const int J = K + cout_pad;
  const int ns = (J + 63) / 64, nbp = (K + 63) / 64;
  if (ns > 64 || nbp < 1) return false;
  bool found = false;
  for (int rs = 0; rs < 5; ++rs) {
    std::mt19937 rng(12345u + rs);
    std::vector<char> need((size_t)ns * ns, 0);
    int remaining = 0;
    for (int a = 0; a < nbp; ++a)
      for (int b = a; b < ns; ++b) need[(size_t)a * ns + b] = 1, ++remaining;
    auto nd = [&](int x, int y) -> int {
      return x <= y ? need[(size_t)x * ns + y] : need[(size_t)y * ns + x];
    };
    SymPlan6 p;
    int ng = 0;
    bool ok = true;
    std::vector<int> order(ns), xs(ns);
    while (remaining > 0) {
      if (ng == kSym6MaxGroups) {
        ok = false;
        break;
      }
      int best_set[6] = {0, 0, 0, 0, 0, 0}, best_key = -1, best_tot = -1;
      for (int i = 0; i < ns; ++i) order[i] = i;
      std::shuffle(order.begin(), order.end(), rng);
      for (int s0 : order) {
        int set[6] = {s0, 0, 0, 0, 0, 0}, n = 1;
        while (n < 6) {
          int bx = -1, bg = -1;
          xs = order;
          std::shuffle(xs.begin(), xs.end(), rng);
          for (int x : xs) {
            bool in = false;
            for (int i = 0; i < n; ++i) in |= set[i] == x;
            if (in) continue;
            int g = nd(x, x);
            for (int i = 0; i < n; ++i) g += nd(x, set[i]);
            if (g > bg) bg = g, bx = x;
          }
          set[n++] = bx;
        }
        int tot = 0;
        for (int i = 0; i < 6; ++i)
          for (int j = i; j < 6; ++j) tot += nd(set[i], set[j]);
        const int key = std::min(16, tot);
        if (key > best_key || (key == best_key && tot < best_tot)) {
          best_key = key, best_tot = tot;
          for (int i = 0; i < 6; ++i) best_set[i] = set[i];
        }
      }
      std::sort(best_set, best_set + 6);
      // the set's uncovered sub-tiles, hardest first (fewest other uncovered tiles on their slabs)
      int deg[6];
      for (int i = 0; i < 6; ++i) {
        deg[i] = 0;
        for (int y = 0; y < ns; ++y) deg[i] += nd(best_set[i], y);
      }
      struct T {
        int i, j, key;
        bool half;
      };
      std::vector<T> tiles;
      for (int i = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j)
          if (nd(best_set[i], best_set[j]))
            tiles.push_back({i, j, deg[i] + deg[j], 64 * best_set[j] + 32 >= J});
      std::stable_sort(tiles.begin(), tiles.end(), [](const T& x, const T& y) { return x.key < y.key; });
      if (tiles.size() > 16) tiles.resize(16);
      std::stable_sort(tiles.begin(), tiles.end(), [](const T& x, const T& y) { return !x.half && y.half; });
      SymGroup6& G = p.g[ng];
      for (int i = 0; i < 6; ++i) G.base[i] = (int16_t)(64 * best_set[i]);
      for (int w = 0; w < 8; ++w) G.ra[w][0] = G.ra[w][1] = G.cb[w][0] = G.cb[w][1] = -1;
      for (int m = 0; m < (int)tiles.size(); ++m) {
        need[(size_t)best_set[tiles[m].i] * ns + best_set[tiles[m].j]] = 0;
        --remaining;
        G.ra[m % 8][m / 8] = (int8_t)tiles[m].i;
        G.cb[m % 8][m / 8] = (int8_t)tiles[m].j;
      }
      ++ng;
    }
    if (ok && (!found || ng < out->ngroups)) {
      p.ngroups = ng;
      *out = p;
      found = true;
    }
  }
  return found;
}

inline bool sym_plan6_greedy(int K, int cout_pad, SymPlan6* p) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, std::pair<bool, SymPlan6>> cache;
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_pair(K, cout_pad);
  auto it = cache.find(key);
  if (it == cache.end()) {
    SymPlan6 q;
    const bool ok = sym_plan6_greedy_build(K, cout_pad, &q);
    it = cache.emplace(key, std::make_pair(ok, q)).first;
  }
  if (it->second.first) *p = it->second.second;
  return it->second.first;
}

// PIPE: the K-tile loads run two tiles ahead, and tile kt+1's split + LDS
// commit is issued between tile kt's first sub-tile MFMAs (sched_group_barrier)
// instead of after both sub-tiles.  With one 512-thread block per CU the two
// waves of a SIMD share the block's barrier phase, so without this a SIMD's
// MFMA pipe idles through every commit.
// The plan (by value) covers the upper triangle with groups; dense partials
// [chunk][I+1][J] through store_tile.
// F16: f16x2 split operands (f16x2.hpp, three MFMAs per product): the P columns
// [0, kp) scaled by the power of two of the published bound pmax, the dY
// columns by ymax's; parts h, l in the first two thirds of each LDS buffer; the
// accumulators unscaled per column before the store (rows are P columns).
template <class Op, class Epi, bool PIPE = false, bool F16 = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
void symred6_kernel(Op op, Epi epi, SymPlan6 plan, int I, int J, int K, int k_chunk,
                    const unsigned* pmax = nullptr, const unsigned* ymax = nullptr, int kp = 0) {
  constexpr int BK = kX3Rows;
  constexpr int NP = F16 ? 2 : 3;
  __shared__ __attribute__((aligned(16))) char lds[2 * kSixBuf];
  float sp = 1.f, sy = 1.f;
  if constexpr (F16) {
    sp = f16x2_scale_of_bits(pmax);
    sy = f16x2_scale_of_bits(ymax);
  }

  const int total = gridDim.x;
  const int b = blockIdx.x;
  const int xcd = b & 7, base8 = total >> 3, rem = total & 7;
  const int l = xcd * base8 + min(xcd, rem) + (b >> 3);
  const int ng = plan.ngroups;
  const int bz = l / ng;
  const auto& G = plan.g[l - bz * ng];
  set_z(epi, bz);
  const int kbeg = bz * k_chunk;
  const int kend = min(K, kbeg + k_chunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  // staging: thread -> k-row tid/32 (16 rows), 12 consecutive staged columns
  // 12*(tid&31) .. +11 = three float4 runs (a run never crosses a slab)
  const int srow = tid >> 5;
  const int scol = 12 * (tid & 31);
  typename Op::CB cbs[3];
  float scu[3];  // F16: the scale of each staged run's columns
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int c = scol + 4 * u;
    const int base = G.base[c >> 6];
    cbs[u] = op.col_base(base >= 0 ? base + (c & 63) : J);
    scu[u] = base + (c & 63) < kp ? sp : sy;
  }
  typename Op::It it = op.iter(kbeg + srow);
  typename Op::St ra[PIPE ? 2 : 1][3];
  float csum[12];
#pragma unroll
  for (int e = 0; e < 12; ++e) csum[e] = 0.f;

  auto fetch = [&](int k0, auto S) {
    constexpr int set = decltype(S)::value;
    const int k = k0 + srow;
#pragma unroll
    for (int u = 0; u < 3; ++u) ra[set][u] = op.stage_it(it, cbs[u], k < kend);
    op.template advance<BK>(it);
  };
  auto commit = [&](int buf, auto S) {
    constexpr int set = decltype(S)::value;
    char* s = lds + buf * kSixBuf + srow * kSixRowBytes;
    const int q8 = 8 * (srow & 3);
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const float4 x = finish(ra[set][u]);
      csum[4 * u] += x.x;
      csum[4 * u + 1] += x.y;
      csum[4 * u + 2] += x.z;
      csum[4 * u + 3] += x.w;
      uint2 h, m, lo;
      if constexpr (F16) {
        split2(x.x, x.y, scu[u], h.x, m.x);
        split2(x.z, x.w, scu[u], h.y, m.y);
      } else {
        split3(x.x, x.y, h.x, m.x, lo.x);
        split3(x.z, x.w, h.y, m.y, lo.y);
      }
      const int off = 8 * (((scol >> 2) + u) ^ q8);
      *reinterpret_cast<uint2*>(s + off) = h;
      *reinterpret_cast<uint2*>(s + kSixPart + off) = m;
      if constexpr (!F16) *reinterpret_cast<uint2*>(s + 2 * kSixPart + off) = lo;
    }
  };

  const int q = (lane >> 2) & 3, p = lane & 3, g = (lane >> 4) & 1, kh = lane >> 5;
  auto slot_off = [&](int colblock) {
    const int slot = (colblock >> 2) + 4 * g + p;
    return (8 * kh + q) * kSixRowBytes + 8 * (slot ^ (8 * q));
  };
  int ib[2], jb[2], aoff[2][2], boff[2][2];
  bool half[2];
  const int ntile = (G.ra[wave][0] >= 0) + (G.ra[wave][1] >= 0);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int sa = G.ra[wave][t] < 0 ? 0 : G.ra[wave][t];
    const int sb = G.cb[wave][t] < 0 ? 0 : G.cb[wave][t];
    ib[t] = G.base[sa];
    jb[t] = G.base[sb];
    half[t] = jb[t] + 32 >= J;
    aoff[t][0] = slot_off(64 * sa);
    aoff[t][1] = slot_off(64 * sa + 32);
    boff[t][0] = slot_off(64 * sb);
    boff[t][1] = slot_off(64 * sb + 32);
  }

  f32x16 acc[2][2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][x][y][r] = 0.f;

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if (nk > 0) {
    fetch(kbeg, S0{});
    if constexpr (PIPE) fetch(kbeg + BK, S1{});
    commit(0, S0{});
  }
  __syncthreads();

  auto tile = [&](const char* s, int t, auto NTc) {
    constexpr int NT = decltype(NTc)::value;
    bf16x8 a[2][3], bb[2][3];
#pragma unroll
    for (int pt = 0; pt < NP; ++pt) {
      const char* sp = s + pt * kSixPart;
      a[0][pt] = cat8(ds_tr16(sp + aoff[t][0]), ds_tr16(sp + aoff[t][0] + 4 * kSixRowBytes));
      a[1][pt] = cat8(ds_tr16(sp + aoff[t][1]), ds_tr16(sp + aoff[t][1] + 4 * kSixRowBytes));
      bb[0][pt] = cat8(ds_tr16(sp + boff[t][0]), ds_tr16(sp + boff[t][0] + 4 * kSixRowBytes));
      if constexpr (NT == 2)
        bb[1][pt] = cat8(ds_tr16(sp + boff[t][1]), ds_tr16(sp + boff[t][1] + 4 * kSixRowBytes));
    }
#pragma unroll
    for (int tm = 0; tm < 2; ++tm)
#pragma unroll
      for (int tn = 0; tn < NT; ++tn) {
        if constexpr (F16) {
          const f16x8 ah[2] = {__builtin_bit_cast(f16x8, a[tm][0]), __builtin_bit_cast(f16x8, a[tm][1])};
          const f16x8 bh[2] = {__builtin_bit_cast(f16x8, bb[tn][0]), __builtin_bit_cast(f16x8, bb[tn][1])};
          acc[t][tm][tn] = mfma_x2(ah, bh, acc[t][tm][tn]);
        } else {
          acc[t][tm][tn] = mfma_x3(a[tm], bb[tn], acc[t][tm][tn]);
        }
      }
  };
  // SN: register set holding tile kt+1 (PIPE) / receiving it (plain)
  auto step = [&](int kt, int cur, auto NTILE, auto N0, auto N1, auto SN) {
    constexpr int nt = decltype(NTILE)::value;
    constexpr int sn = decltype(SN)::value;
    const char* s = lds + cur * kSixBuf;
    if constexpr (PIPE) {
      fetch(kbeg + (kt + 2) * BK, std::integral_constant<int, sn ^ 1>{});
      if constexpr (nt >= 1) {
        tile(s, 0, N0);
        if (kt + 1 < nk) commit(cur ^ 1, SN);
        constexpr int nm = (F16 ? 3 : 6) * 2 * decltype(N0)::value;
        __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);             // the loads
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * NP * (2 + decltype(N0)::value), 0);  // fragments
#pragma unroll
        for (int i = 0; i < nm; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      } else {
        if (kt + 1 < nk) commit(cur ^ 1, SN);
      }
      if constexpr (nt >= 2) tile(s, 1, N1);
    } else {
      fetch(kbeg + (kt + 1) * BK, S0{});
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (nt >= 1) tile(s, 0, N0);
      if constexpr (nt >= 2) tile(s, 1, N1);
      __builtin_amdgcn_sched_barrier(0);
      commit(cur ^ 1, S0{});
    }
    __syncthreads();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  auto run = [&](auto NTILE, auto N0, auto N1) {
    if constexpr (PIPE) {
      for (int kt = 0; kt < nk; kt += 2) {
        step(kt, 0, NTILE, N0, N1, S1{});
        if (kt + 1 < nk) step(kt + 1, 1, NTILE, N0, N1, S0{});
      }
    } else {
      for (int kt = 0; kt < nk; ++kt) step(kt, kt & 1, NTILE, N0, N1, S0{});
    }
  };
  if (ntile == 0) run(I0{}, I2{}, I2{});
  else if (ntile == 1) {
    if (half[0]) run(I1{}, I1{}, I2{});
    else run(I1{}, I2{}, I2{});
  } else {
    if (half[0]) run(I2{}, I1{}, I1{});
    else if (half[1]) run(I2{}, I2{}, I1{});
    else run(I2{}, I2{}, I2{});
  }

  // column sums: [16 k-row threads][384 staged columns] through the free LDS
  float* cs = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int e = 0; e < 12; ++e) cs[srow * 384 + scol + e] = csum[e];
  __syncthreads();
  {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (t >= ntile) break;
      if constexpr (F16) {  // unscale: rows are P columns (sp), column j by its own scale
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
          const float inv = 1.f / (sp * (jb[t] + 32 * tn + (lane & 31) < kp ? sp : sy));
#pragma unroll
          for (int tm = 0; tm < 2; ++tm)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][tm][tn][r] *= inv;
        }
      }
      store_tile<2, 2>(epi, acc[t], ib[t], jb[t], lane, I, J);
      if (ib[t] == 0) {  // the (0, b) sub-tile is unique: its wave writes slab b's column sums
        const int col = 64 * G.cb[wave][t] + lane;
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) v += cs[r * 384 + col];
        if (jb[t] + lane < J) epi.colsum(jb[t] + lane, v);
      }
    }
  }
}

// pmax / ymax (both or neither): the f16x2 form, P columns [0, kp) and dY
// columns bounded by the published maxima
template <class Op, class Epi>
inline void launch_symred6(const Op& op, const Epi& e, const SymPlan6& plan, int I, int J, int K,
                           int nchunk, int k_chunk, hipStream_t s, const unsigned* pmax = nullptr,
                           const unsigned* ymax = nullptr, int kp = 0) {
  if (pmax && ymax)
    hipLaunchKernelGGL((symred6_kernel<Op, Epi, true, true>), dim3(plan.ngroups * nchunk), dim3(512), 0, s, op,
                       e, plan, I, J, K, k_chunk, pmax, ymax, kp);
  else
    hipLaunchKernelGGL((symred6_kernel<Op, Epi, true>), dim3(plan.ngroups * nchunk), dim3(512), 0, s, op, e,
                       plan, I, J, K, k_chunk, nullptr, nullptr, 0);
}

// Six-slab groups (symred6_kernel, loads two K-tiles ahead) where sym_plan6 has
// a covering, else four-slab groups (symred3_kernel).  Measured at the bench
// shape (conv2 patch rows, M = 10240): six 1.27 ms, six without the two-ahead
// loads 1.36, four 1.52, four with interleaved tiles 1.50; timing probes of the
// four-slab kernel without the operand split 1.43, without MFMAs 0.87.
template <class Op, class Epi>
inline void launch_symred3(const Op& op, const Epi& e, const SymPlan& plan, int I, int J, int K,
                           int nchunk, int k_chunk, hipStream_t s) {
  hipLaunchKernelGGL((symred3_kernel<Op, Epi>), dim3(plan.ngroups * nchunk), dim3(256), 0, s, op, e, plan, I, J,
                     K, k_chunk);
}

}  // namespace acmi
