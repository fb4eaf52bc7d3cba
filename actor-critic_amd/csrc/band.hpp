// Pixel-pair ("band") conv weight gradient + K-FAC A factor (plan: bandplan.hpp).
//
// One conv layer's [P;1]^T [P | dY] over the M*L patch rows is computed as
//   1. symred6_kernel over the DENSE rows [X | dY] of the M images (X the layer
//      input [M][H*W*C], dY its output gradient [M][L*CO]): only the 64x64
//      sub-tiles whose slabs share a patch, six slabs per block, bf16x3 split
//      operands (f32-accurate, symred3.hpp), per-chunk partials in compact
//      tile slots [chunk][tile][64][64] + column sums [chunk][ns*64];
//   2. band_reduce_kernel: the chunks summed in chunk order (in place, chunk 0);
//   3. band_fold_kernel: every output element sums its L pixel-pair entries in
//      location order -- the A factor's upper triangle (written to both halves,
//      so it is exactly symmetric), the homogeneous row/column, [dW; db].
// Fixed summation orders throughout: deterministic, no atomics.
// Reference: kfac's conv input factor over extract_image_patches rows
// (registration envs/atari/model.py:227-238) and tf.gradients' conv2d filter
// gradient (objectives.py:78) -- the same sums, reassociated.
#pragma once

#include <map>
#include <mutex>
#include <tuple>

#include "bandplan.hpp"
#include "symred3.hpp"

namespace acmi {

// launch-site profiling (net.hip)
static void prof_begin(int site, hipStream_t s);
static void prof_end(int site, hipStream_t s);

struct BandPlanDev {
  const BandGroup* g;
  int ngroups;
  int xcd_remap;  // 1: blocks XCD-contiguous (symred6's default map); 0: dispatch order
};

// ACMI_BAND_MAP=1: XCD-contiguous block map (each XCD's L2 sees neighbouring
// groups); default 0: dispatch order, so all XCDs work on the same chunk of
// images and its rows stay in the MALL while the groups re-read them
inline int band_xcd_remap() {
  static const int v = getenv("ACMI_BAND_MAP") ? atoi(getenv("ACMI_BAND_MAP")) : 0;
  return v;
}

struct EpiBand {
  float* part;  // [chunk][ntiles][64][64]
  float* cs;    // [chunk][ncols]
  int ntiles;
  int ncols;
  int z = 0;
};

// host plan per layer shape (no device needed: workspace sizing), and its
// device copy per device (built on first use, kept for the process)
inline const BandPlan* band_host_plan(int H, int W, int C, int KH, int KW, int S, int CO) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int, int, int, int>, BandPlan*> cache;
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_tuple(H, W, C, KH, KW, S, CO);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  BandGeom g;
  BandPlan* p = new BandPlan();
  if (!band_geom(H, W, C, KH, KW, S, CO, &g) || !band_plan_build(g, p) || band_plan_check(*p) != 0) {
    delete p;
    p = nullptr;
  }
  cache[key] = p;
  return p;
}

struct BandDev {
  const BandPlan* plan = nullptr;
  BandGroup* groups = nullptr;
  int* tabs = nullptr;  // pairs | atab | wtab | ctab | dtab
  int o_pairs = 0, o_atab = 0, o_wtab = 0, o_ctab = 0, o_dtab = 0;
  std::vector<int> host_tabs;  // source of the stream-ordered upload
};

inline const BandDev* band_dev(int H, int W, int C, int KH, int KW, int S, int CO, hipStream_t s) {
  const BandPlan* p = band_host_plan(H, W, C, KH, KW, S, CO);
  int dev = 0;
  if (!p || hipGetDevice(&dev) != hipSuccess) return nullptr;
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int, int, int, int, int>, BandDev*> cache;
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_tuple(H, W, C, KH, KW, S, CO, dev);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  std::vector<int> tabs;
  auto put = [&](const std::vector<int>& v) {
    const int o = (int)tabs.size();
    tabs.insert(tabs.end(), v.begin(), v.end());
    return o;
  };
  BandDev* d = new BandDev();
  d->plan = p;
  d->o_pairs = put(p->pairs);
  d->o_atab = put(p->atab);
  d->o_wtab = put(p->wtab);
  d->o_ctab = put(p->ctab);
  d->o_dtab = put(p->dtab);
  const size_t gb = p->groups.size() * sizeof(BandGroup), tb = tabs.size() * sizeof(int);
  // the upload is ordered on the caller's stream (no null-stream serialisation);
  // the host copies it reads must outlive it: the plan's groups are cached for the
  // process, the tables are staged into a host buffer kept beside the plan
  d->host_tabs = std::move(tabs);
  if (hipMalloc(&d->groups, gb) != hipSuccess || hipMalloc(&d->tabs, tb) != hipSuccess ||
      hipMemcpyAsync(d->groups, p->groups.data(), gb, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d->tabs, d->host_tabs.data(), tb, hipMemcpyHostToDevice, s) != hipSuccess) {
    // a failed allocation or copy is retried at the next call: release what was taken
    if (d->groups) (void)hipFree(d->groups);
    if (d->tabs) (void)hipFree(d->tabs);
    delete d;
    return nullptr;
  }
  cache[key] = d;
  return d;
}

// Chunks of the M image rows: ACMI_BAND_CHUNKS forces the count; by default
// about four dynamic rounds of one-block-per-CU blocks (groups differ in their
// tile counts, so many shorter blocks balance the CUs), chunks >= 512 rows.
inline void band_chunks(long long rows, int ngroups, int* nc, int* ch) {
  static const int forced = getenv("ACMI_BAND_CHUNKS") ? atoi(getenv("ACMI_BAND_CHUNKS")) : 0;
  long long n = forced > 0 ? forced : std::max(1, (4 * 256 + ngroups / 2) / std::max(1, ngroups));
  n = std::max(1LL, std::min(n, rows / 512 > 0 ? rows / 512 : 1));
  long long c = (rows + n - 1) / n;
  c = (c + 15) / 16 * 16;
  *ch = (int)c;
  *nc = (int)((rows + c - 1) / c);
}

inline long long band_ws_floats(const BandPlan* p, long long rows) {
  if (!p) return 0;
  int nc, ch;
  band_chunks(rows, (int)p->groups.size(), &nc, &ch);
  return (long long)nc * ((long long)p->ntiles * 4096 + (long long)p->geom.ns * 64);
}

// chunk sums in chunk order, in place into chunk 0 (float4 runs; the tile
// partials then the column sums)
__global__ __launch_bounds__(256) void band_reduce_kernel(float* part, long long n4t, float* cs,
                                                          long long n4c, int nc) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  float4* p;
  long long stride;
  if (i < n4t) {
    p = reinterpret_cast<float4*>(part) + i;
    stride = n4t;
  } else if (i < n4t + n4c) {
    p = reinterpret_cast<float4*>(cs) + (i - n4t);
    stride = n4c;
  } else {
    return;
  }
  float4 s = p[0];
  for (int c0 = 1; c0 < nc; c0 += 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p[(c0 + u < nc ? c0 + u : 0) * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (c0 + u < nc) s.x += v[u].x, s.y += v[u].y, s.z += v[u].z, s.w += v[u].w;
  }
  p[0] = s;
}

struct BandFold {
  const float* T;   // [ntiles][64][64], chunk-reduced
  const float* cs;  // [ns * 64]
  const int* pairs;
  const int* atab;
  const int* wtab;
  const int* ctab;
  const int* dtab;
  int L, C, CO, K;  // K = KK * C
  long long nA, nW, nH;
  float* astat;  // (K+1)^2
  float* grad;   // (K+1) x CO, [W; b]
  float rows;    // M * L
  float wscale;
};

// sum_l src[tab[l]] in location order, 8 table entries and 8 values in flight
__device__ __forceinline__ float band_gather_sum(const float* src, const int* tab, int L) {
  float s = 0.f;
  for (int l0 = 0; l0 < L; l0 += 8) {
    int o[8];
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) o[u] = tab[l0 + u < L ? l0 + u : L - 1];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[o[u]];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (l0 + u < L) s += v[u];
  }
  return s;
}

__global__ __launch_bounds__(256) void band_fold_kernel(BandFold f) {
  long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const int K1 = f.K + 1;
  const float inv = 1.0f / f.rows;
  if (idx < f.nA) {  // A-factor block of kernel positions (ka, kb), element (i, j)
    const int CC = f.C * f.C;
    const int P = (int)(idx / CC);
    const int e = (int)(idx - (long long)P * CC);
    const int i = e / f.C, j = e - (e / f.C) * f.C;
    const int pr = f.pairs[P], ka = pr >> 8, kb = pr & 255;
    if (ka == kb && i > j) return;  // diagonal block: the upper triangle, mirrored
    const float s = band_gather_sum(f.T + i * 64 + j, f.atab + (long long)P * f.L, f.L) * inv;
    const long long a = (long long)ka * f.C + i, b = (long long)kb * f.C + j;
    f.astat[a * K1 + b] = s;
    f.astat[b * K1 + a] = s;
    return;
  }
  idx -= f.nA;
  if (idx < f.nW) {  // weight gradient row (k, ci), column co
    const int per = f.C * f.CO;
    const int k = (int)(idx / per);
    const int rem = (int)(idx - (long long)k * per);
    const int ci = rem / f.CO, co = rem - (rem / f.CO) * f.CO;
    const float s = band_gather_sum(f.T + ci * 64 + co, f.wtab + (long long)k * f.L, f.L);
    f.grad[((long long)k * f.C + ci) * f.CO + co] = s * f.wscale;
    return;
  }
  idx -= f.nW;
  if (idx < f.nH) {  // homogeneous column of the A factor: patch column sums
    const int k = (int)(idx / f.C), ci = (int)(idx - (idx / f.C) * f.C);
    const float s = band_gather_sum(f.cs + ci, f.ctab + (long long)k * f.L, f.L) * inv;
    const long long a = (long long)k * f.C + ci;
    f.astat[a * K1 + f.K] = s;
    f.astat[(long long)f.K * K1 + a] = s;
    return;
  }
  idx -= f.nH;
  if (idx < f.CO) {  // bias gradient: dY column sums
    const int co = (int)idx;
    f.grad[(long long)f.K * f.CO + co] = band_gather_sum(f.cs + co, f.dtab, f.L);
    if (co == 0) f.astat[(long long)f.K * K1 + f.K] = f.rows * inv;
  }
}

// [dW; db] of one conv layer and its A factor ((K+1)^2, / (M*L)) from the layer
// input X [M][H][W][C] (f32, dense) and output gradient dY [M][OH][OW][CO].
inline int band_layer(const float* X, int H, int W, int C, int KH, int KW, int S, const float* dy,
                      int CO, int M, float* ws, long long ws_cap, float* grad, float* astat,
                      float wscale, hipStream_t s, int site = 0) {
  const BandDev* d = band_dev(H, W, C, KH, KW, S, CO, s);
  ACMI_REQUIRE(d, ACMI_ERR_ARG, "band plan unavailable for %dx%dx%d k%dx%d s%d -> %d", H, W, C, KH, KW, S,
               CO);
  const BandPlan& p = *d->plan;
  const BandGeom& g = p.geom;
  const int ng = (int)p.groups.size();
  int nc, ch;
  band_chunks(M, ng, &nc, &ch);
  const long long tile_f = (long long)p.ntiles * 4096, ncols = (long long)g.ns * 64;
  ACMI_REQUIRE((long long)nc * (tile_f + ncols) <= ws_cap, ACMI_ERR_WS,
               "band workspace too small (%lld > %lld)", (long long)nc * (tile_f + ncols), ws_cap);
  float* part = ws;
  float* cs = ws + (long long)nc * tile_f;
  CatRowsI<DenseRows> op{DenseRows{X, g.kp, M, g.kp}, g.kp, dy, g.L * CO, g.L * CO, g.L * CO, M};
  EpiBand epi{part, cs, p.ntiles, (int)ncols};
  BandPlanDev pd{d->groups, ng, band_xcd_remap()};
  prof_begin(site, s);
  hipLaunchKernelGGL((symred6_kernel<CatRowsI<DenseRows>, EpiBand, true, BandPlanDev>), dim3(ng * nc),
                     dim3(512), 0, s, op, epi, pd, g.nxs * 64, g.J, M, ch);
  prof_end(site, s);
  if (nc > 1) {
    const long long n4 = (tile_f + ncols) / 4;
    hipLaunchKernelGGL(band_reduce_kernel, dim3(cdiv(n4, 256)), dim3(256), 0, s, part, tile_f / 4, cs,
                       ncols / 4, nc);
  }
  BandFold f;
  f.T = part;
  f.cs = cs;
  f.pairs = d->tabs + d->o_pairs;
  f.atab = d->tabs + d->o_atab;
  f.wtab = d->tabs + d->o_wtab;
  f.ctab = d->tabs + d->o_ctab;
  f.dtab = d->tabs + d->o_dtab;
  f.L = g.L;
  f.C = C;
  f.CO = CO;
  f.K = g.KK * C;
  f.nA = (long long)p.pairs.size() * C * C;
  f.nW = (long long)g.KK * C * CO;
  f.nH = (long long)g.KK * C;
  f.astat = astat;
  f.grad = grad;
  f.rows = (float)((long long)M * g.L);
  f.wscale = wscale;
  hipLaunchKernelGGL(band_fold_kernel, dim3(cdiv(f.nA + f.nW + f.nH + CO, 256)), dim3(256), 0, s, f);
  ACMI_LAUNCH_CHECK("band_layer");
  return ACMI_OK;
}

}  // namespace acmi
