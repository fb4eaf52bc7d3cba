// Pixel-pair ("band") conv weight gradient + K-FAC A factor (plan: bandplan.hpp).
//
// One conv layer's [P;1]^T [P | dY] over the M*L patch rows is computed as
//   1. band_kernel over the DENSE rows [X | dY] of the M images (X the layer
//      input [M][H*W*C], dY its output gradient [M][L*CO]): only the 64x64
//      sub-tiles whose slabs share a patch, up to 8 staged slabs and 16 sub-tiles
//      per work item, per-chunk partials in compact tile slots
//      [chunk][tile][64][64] + column sums [chunk][ns*64];
//   2. band_reduce_kernel: the chunks summed in chunk order (in place, chunk 0);
//   3. band_fold_kernel: every output element sums its L pixel-pair entries in
//      location order -- the A factor's upper triangle (written to both halves,
//      so it is exactly symmetric), the homogeneous row/column, [dW; db].
// Fixed summation orders throughout: deterministic, no atomics on data.
// Reference: kfac's conv input factor over extract_image_patches rows
// (registration envs/atari/model.py:227-238) and tf.gradients' conv2d filter
// gradient (objectives.py:78) -- the same sums, reassociated.
//
// Arithmetic: "f16x2" split operands.  Every f32 operand x of a slab is scaled
// by a power of two s (one per tensor: X or dY) and split at the LDS commit into
//   h = f16_rn(x s),  l = f16_rn(x s - h)        (the subtraction is exact)
// so x s = h + l to 2^-22 relative, and each 32x32x16 tile takes the three
// v_mfma_f32_32x32x16_f16 of l*h + h*l + h*h into one f32 accumulator (every
// f16 x f16 product is exact in f32; the dropped l*l is <= 2^-22 |a||b|); the
// tile is multiplied by 1/(s_a s_b) (exact) when it is stored.  The scales put
// each tensor's bound at 2^14 < 65504: X from the layer's weights (a1, a2 are
// ReLU outputs of [0,1] pixels, bounded by the positive weight mass,
// band_bounds_kernel), dY from its exact max (published by the dX epilogues that
// produce it, gemm.hpp has_amax).  Elements far
// below the bound lose relative precision only where their absolute error
// (<= 2^-25 in scaled units) is < 2^-30 of the bound.  Three MFMAs per product
// instead of bf16x3's six: the same f32-class sums (accumulation error,
// ~sqrt(K) 2^-24, dominates the 2^-22 operand error) at twice the matrix rate.
//
// Work distribution: one 512-thread block per (group, chunk) item; block b runs
// item b >> 3 of XCD b & 7's list.  A list holds the groups of one spatial region
// of the image, chunk-major, so the blocks of one XCD stream the same image rows
// over the columns of one region: the region's slabs are fetched into that XCD's
// L2 once and re-read from there by the other groups of the region.
#pragma once

#include <map>
#include <mutex>
#include <tuple>

#include "bandplan.hpp"
#include "f16x2.hpp"  // split2, f16x2_scale, ds_tr16, stage_f4, zero_run

namespace acmi {

// launch-site profiling (net.hip)
static void prof_begin(int site, hipStream_t s);
static void prof_end(int site, hipStream_t s);

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
  int* tabs = nullptr;  // pairs | atab | wtab | ctab | dtab | xlist
  int o_pairs = 0, o_atab = 0, o_wtab = 0, o_ctab = 0, o_dtab = 0, o_xlist = 0;
  int xoff[9] = {};
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
  std::vector<int> xl;
  for (int x = 0; x < 8; ++x) {
    d->xoff[x] = (int)xl.size();
    xl.insert(xl.end(), p->xcd_groups[x].begin(), p->xcd_groups[x].end());
  }
  d->xoff[8] = (int)xl.size();
  d->o_xlist = put(xl);
  const size_t gb = p->groups.size() * sizeof(BandGroup), tb = tabs.size() * sizeof(int);
  // the upload is ordered on the caller's stream (no null-stream serialisation);
  // the host copies it reads outlive it: the plan's groups are cached for the
  // process, the tables are kept beside the device pointers
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

// Chunks of the M image rows: about three items per CU over the whole grid (the
// groups differ in work, so shorter items late in the grid fill the CUs), chunks
// >= 512 rows (2 / 3 / 5 / 6 / 8 chunks measured slower than 4 at conv2, M = 10240)
inline void band_chunks(long long rows, int ngroups, int* nc, int* ch) {
  long long n = std::max(1, (3 * 256 + ngroups / 2) / std::max(1, ngroups));
  n = std::max(1LL, std::min(n, rows / 512 > 0 ? rows / 512 : 1));
  long long c = (rows + n - 1) / n;
  c = (c + 15) / 16 * 16;
  *ch = (int)c;
  *nc = (int)((rows + c - 1) / c);
}

// band scratch (kBandScratch words at the end of the backward's partial region,
// zeroed before the dX chain): the bit patterns of max |d3|, |d2| (published by
// the dX epilogues, gemm.hpp has_amax) and of the a1 / a2 bounds
// (band_bounds_kernel); the kernels turn them into their operand scales
// published maxima (kAmaxSlots words each, common.hpp)
enum {
  kBsMaxA1 = 0 * kAmaxWords, kBsMaxA2 = 1 * kAmaxWords, kBsMaxD2 = 2 * kAmaxWords, kBsMaxD3 = 3 * kAmaxWords,
  kBsMaxW3 = 4 * kAmaxWords, kBsMaxD4 = 5 * kAmaxWords, kBsMaxW4 = 6 * kAmaxWords, kBsMaxD1 = 7 * kAmaxWords
};
constexpr int kBandScratch = 8 * kAmaxWords;

inline long long band_ws_floats(const BandPlan* p, long long rows) {
  if (!p) return 0;
  int nc, ch;
  band_chunks(rows, (int)p->groups.size(), &nc, &ch);
  return (long long)nc * ((long long)p->ntiles * 4096 + (long long)p->geom.ns * 64);
}

// The X bounds from the weights: a1 = relu(W1 x + b1) with x in [0, 1], so
// a1[c] <= B1[c] = sum_k max(W1[k][c], 0) + max(b1[c], 0); a2 = relu(W2 a1 + b2)
// with a1 >= 0, so a2[c'] <= sum_{k,c} max(W2[k][c][c'], 0) B1[c] + max(b2[c'], 0).
// Block c' (64 blocks) recomputes B1 (8192 weights) and sums conv2's column c'
// (512 rows); both maxima atomicMax-ed into the zeroed scratch.
__global__ __launch_bounds__(256) void band_bounds_kernel(const float* w1, const float* b1, const float* w2,
                                                         const float* b2, unsigned* scr) {
  __shared__ float part[8][32];
  __shared__ float B1[32];
  __shared__ float red[4];
  const int t = threadIdx.x, co = blockIdx.x;
  {  // B1: thread (q = t / 32, c = t % 32) sums taps q, q + 8, ... (coalesced rows of 32)
    const int c = t & 31, q = t >> 5;
    float acc = 0.f;
#pragma unroll 8
    for (int k = q; k < 256; k += 8) acc += fmaxf(w1[k * 32 + c], 0.f);
    part[q][c] = acc;
  }
  __syncthreads();
  if (t < 32) {
    float acc = fmaxf(b1[t], 0.f);
    for (int q = 0; q < 8; ++q) acc += part[q][t];
    B1[t] = acc;
  }
  __syncthreads();
  // conv2 column co: rows r = (kh, kw, c) of W2 [512][64]
  const float v = fmaxf(w2[t * 64 + co], 0.f) * B1[t & 31] + fmaxf(w2[(t + 256) * 64 + co], 0.f) * B1[t & 31];
  const float sum = wave_sum(v);
  if ((t & 63) == 0) red[t >> 6] = sum;
  __syncthreads();
  if (t == 0) {
    const float b2c = red[0] + red[1] + red[2] + red[3] + fmaxf(b2[co], 0.f);
    amax_update(scr + kBsMaxA2, b2c);
    if (co == 0) {
      float m = 0.f;
      for (int c = 0; c < 32; ++c) m = fmaxf(m, B1[c]);
      amax_update(scr + kBsMaxA1, m);
    }
  }
}

// ---------------------------------------------------------------------------
// the band kernel
// ---------------------------------------------------------------------------
constexpr int kBandRows = 16;                         // k-rows (images) per stage
constexpr int kBandRowBytes = kBandSlabs * 64 * 2;    // 1024: one f16 row of the staged columns
constexpr int kBandPart = kBandRows * kBandRowBytes;  // 16 KB
constexpr int kBandBuf = 2 * kBandPart;               // h, l

struct BandArgs {
  const float* X;    // [M][kp]
  const float* dy;   // [M][ldy]
  int kp, ldy, J, M;
  int k_chunk, nc;
  const BandGroup* groups;
  const int* xlist;  // groups of XCD x: xlist[xoff[x] .. xoff[x + 1])
  int xoff[9];
  const unsigned* xmax;  // bit patterns of the X bound and of max |dY| (band scratch)
  const unsigned* ymax;
  float* part;       // [nc][ntiles][64][64]
  float* cs;         // [nc][ncols]
  int ntiles, ncols;
};

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void band_kernel(BandArgs p) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kBandBuf];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  // staging: thread -> rows 2*rp, 2*rp + 1 of the stage; columns 4*lane .. +3
  // (staged slab lane / 16) and 256 + 4*lane .. +3 (slab 4 + lane / 16)
  const int rp = wave;
  const int q = (lane >> 2) & 3, pl = lane & 3, g = (lane >> 4) & 1, kh = lane >> 5;
  const float sx = f16x2_scale_of_bits(p.xmax), sy = f16x2_scale_of_bits(p.ymax);
  {
    // item: XCD x = b & 7 (the blocks b, b + 8, ... share an XCD under the
    // round-robin dispatch), its j-th (group, chunk) in the region's list
    const int x = blockIdx.x & 7;
    const int it = blockIdx.x >> 3;
    if (it >= (p.xoff[x + 1] - p.xoff[x]) * p.nc) return;
    const int ngx = p.xoff[x + 1] - p.xoff[x];
    const int chunk = it / ngx;
    const BandGroup& G = p.groups[p.xlist[p.xoff[x] + (it - chunk * ngx)]];
    const int kbeg = chunk * p.k_chunk;
    const int kend = min(p.M, kbeg + p.k_chunk);
    const int nk = (kend - kbeg + kBandRows - 1) / kBandRows;
    const int nslab = G.nslab;

    // this thread's two staged column runs: base pointer, row stride, scale
    const float* cptr[2];
    uint32_t cld[2];
    bool cok[2];
    float cscale[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int si = 4 * u + (lane >> 4);
      const int col = (si < nslab ? G.base[si] : p.J) + 4 * (lane & 15);
      cok[u] = si < nslab && col < p.J;
      const bool isx = col < p.kp;
      cptr[u] = isx ? p.X + col : p.dy + (col - p.kp);
      cld[u] = isx ? (uint32_t)p.kp : (uint32_t)p.ldy;
      cscale[u] = ((G.xmask >> (si & 7)) & 1) ? sx : sy;
    }
    float4 ra[1][4];  // one register set of staged loads
    float csum[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
    // element offsets of this thread's first row in the next stage to fetch
    // (stages are fetched in order: advanced by 16 rows per fetch)
    uint32_t foff[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) foff[u] = (uint32_t)(kbeg + 2 * rp) * cld[u];

    auto fetch = [&](int k0, auto S) {
      constexpr int set = decltype(S)::value;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const bool rok = k0 + 2 * rp + r < kend;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          ra[set][2 * r + u] = stage_f4(cptr[u] + foff[u] + r * cld[u], rok && cok[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) foff[u] += (uint32_t)kBandRows * cld[u];
    };
    // one staged float4 (row 2 rp + r, run u) of register set `set` into LDS buffer buf
    auto commit1 = [&](int buf, auto S, int r, int u) {
      constexpr int set = decltype(S)::value;
      {
        const int krow = 2 * rp + r;
        char* s = lds + buf * kBandBuf + krow * kBandRowBytes;
        const int q8 = 8 * (krow & 3);
        {
          const float4 v = ra[set][2 * r + u];
          csum[4 * u] += v.x;
          csum[4 * u + 1] += v.y;
          csum[4 * u + 2] += v.z;
          csum[4 * u + 3] += v.w;
          uint2 h, l;
          split2(v.x, v.y, cscale[u], h.x, l.x);
          split2(v.z, v.w, cscale[u], h.y, l.y);
          const int off = 8 * ((64 * u + lane) ^ q8);  // 8-byte slot (4 columns) of column 4*(64u + lane)
          *reinterpret_cast<uint2*>(s + off) = h;
          *reinterpret_cast<uint2*>(s + kBandPart + off) = l;
        }
      }
    };
    auto commit = [&](int buf, auto S) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int u = 0; u < 2; ++u) commit1(buf, S, r, u);
    };

    auto slot_off = [&](int colblock) {
      const int slot = (colblock >> 2) + 4 * g + pl;
      return (8 * kh + q) * kBandRowBytes + 8 * (slot ^ (8 * q));
    };
    int aoff[2][2], boff[2][2];
    float inv[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int sa = G.ra[wave][t] < 0 ? 0 : G.ra[wave][t];
      const int sb = G.cb[wave][t] < 0 ? 0 : G.cb[wave][t];
      aoff[t][0] = slot_off(64 * sa);
      aoff[t][1] = slot_off(64 * sa + 32);
      boff[t][0] = slot_off(64 * sb);
      boff[t][1] = slot_off(64 * sb + 32);
      const float s_a = ((G.xmask >> sa) & 1) ? sx : sy, s_b = ((G.xmask >> sb) & 1) ? sx : sy;
      inv[t] = 1.f / (s_a * s_b);  // powers of two: exact
    }
    const int ntile = (G.ra[wave][0] >= 0) + (G.ra[wave][1] >= 0);

    f32x16 acc[2][2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[t][a][b][r] = 0.f;

    using S0 = std::integral_constant<int, 0>;
    // Software-pipelined fragment reads.  Each wave's sub-tiles of stage kt are
    // read from LDS one sub-tile AHEAD of their MFMAs, and the last sub-tile of a
    // stage is multiplied after the barrier, while the next stage's first
    // fragments are in flight:
    //   barrier(kt-1) | read (kt,0) | mma (kt-1,last) + commit of stage kt+1
    //   (VALU split and LDS stores interleaved with those MFMAs) | fetch kt+2 |
    //   read (kt,1) | mma (kt,0) | barrier(kt) | read (kt+1,0) | ...
    // so no MFMA block waits for a burst of LDS reads issued right before it (in
    // the plain order every wave of the CU reads at the same time after each
    // barrier and the matrix pipes idle until the fragments return).  Fragment
    // sets: F[t] for tile t when a wave has two sub-tiles; by stage parity when
    // it has one.  Stages past the chunk end stage zeros (masked loads), so the
    // commit is unconditional and the trailing read is harmless.
    // (Measured and removed: two 16-row stages per barrier over a ring of four
    // LDS buffers -- half the barriers, bit-identical -- 0.66 vs 0.635 ms per
    // conv2 launch; no stage prefetch depth or plain-order variant did better.)
    struct Frag {
      f16x8 a[2][2], b[2][2];  // [32-column block][part h, l]
    };
    Frag F[2];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) F[f].a[x][y] = F[f].b[x][y] = f16x8{0, 0, 0, 0, 0, 0, 0, 0};
    auto fread = [&](const char* s, int t, Frag& f) {
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        const char* sp = s + pt * kBandPart;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          f.a[cb][pt] = cat8h(ds_tr16(sp + aoff[t][cb]), ds_tr16(sp + aoff[t][cb] + 4 * kBandRowBytes));
          f.b[cb][pt] = cat8h(ds_tr16(sp + boff[t][cb]), ds_tr16(sp + boff[t][cb] + 4 * kBandRowBytes));
        }
      }
    };
    // one 32x32 block (tm, tn) of sub-tile t: the three f16x2 MFMAs
    auto fmma1 = [&](auto T, const Frag& f, int tm, int tn) {
      constexpr int t = decltype(T)::value;
      f32x16 c = acc[t][tm][tn];
      c = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.a[tm][1], f.b[tn][0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.a[tm][0], f.b[tn][1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.a[tm][0], f.b[tn][0], c, 0, 0, 0);
      acc[t][tm][tn] = c;
    };
    auto fmma = [&](auto T, const Frag& f) {
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) fmma1(T, f, tm, tn);
    };
    // sub-tile t's MFMAs with the commit of LDS buffer buf interleaved: block
    // (tm, tn) = p's three MFMAs, then staged float4 p's split + stores (they
    // issue while the third MFMA runs)
    auto fmma_commit = [&](auto T, const Frag& f, int buf) {
#pragma unroll
      for (int p4 = 0; p4 < 4; ++p4) {
        fmma1(T, f, p4 >> 1, p4 & 1);
        commit1(buf, S0{}, p4 >> 1, p4 & 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    using T0 = std::integral_constant<int, 0>;
    using T1 = std::integral_constant<int, 1>;
    // one register set of staged loads: stage kt+1 is committed at the start of
    // step kt and stage kt+2 fetched into the same registers right after (one
    // stage of latency, as with two sets committed mid-step)
    if (nk > 0) {
      fetch(kbeg, S0{});
      commit(0, S0{});
      fetch(kbeg + kBandRows, S0{});
    }
    __syncthreads();
    if (ntile > 0) fread(lds, 0, F[0]);
    auto pstep = [&](int kt, auto I, auto NT) {
      constexpr int nt = decltype(NT)::value;
      constexpr int i = decltype(I)::value;
      const int cur = i & 1;
      const char* s = lds + cur * kBandBuf;
      // the previous stage's last sub-tile (zero fragments before the first
      // stage) with the commit of stage kt+1 interleaved
      if constexpr (nt == 2) fmma_commit(T1{}, F[1], cur ^ 1);
      if constexpr (nt == 1) fmma_commit(T0{}, F[(i + 1) & 1], cur ^ 1);
      if constexpr (nt == 0) commit(cur ^ 1, S0{});
      fetch(kbeg + (kt + 2) * kBandRows, S0{});
      if constexpr (nt == 2) {
        fread(s, 1, F[1]);
        fmma(T0{}, F[0]);
      }
      // (the MFMAs stay before the barrier: sunk past it, they would leave the
      // tile-1 reads just issued exposed at the barrier's wait)
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      const char* sn = lds + (cur ^ 1) * kBandBuf;
      if constexpr (nt == 2) fread(sn, 0, F[0]);
      if constexpr (nt == 1) fread(sn, 0, F[(i + 1) & 1]);
    };
    auto prun = [&](auto NT) {
      for (int kt = 0; kt < nk; kt += 2) {
        pstep(kt, std::integral_constant<int, 0>{}, NT);
        if (kt + 1 < nk) pstep(kt + 1, std::integral_constant<int, 1>{}, NT);
      }
      // the last stage's deferred sub-tile
      constexpr int nt = decltype(NT)::value;
      if constexpr (nt == 2) fmma(T1{}, F[1]);
      if constexpr (nt == 1) {
        if (nk > 0) {
          if ((nk - 1) & 1) fmma(T0{}, F[1]);
          else fmma(T0{}, F[0]);
        }
      }
    };
    if (ntile == 0) prun(std::integral_constant<int, 0>{});
    else if (ntile == 1) prun(std::integral_constant<int, 1>{});
    else prun(std::integral_constant<int, 2>{});

    // tiles, unscaled, into their compact slots of this chunk
    const int khalf = lane >> 5;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (t >= ntile) break;
      float* dst = p.part + ((long long)chunk * p.ntiles + G.tile[wave][t]) * 4096;
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < 2; ++tn)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            dst[(32 * tm + (r & 3) + 8 * (r >> 2) + 4 * khalf) * 64 + 32 * tn + (lane & 31)] =
                acc[t][tm][tn][r] * inv[t];
    }
    // column sums: [8 row-pair threads][512 staged columns] through the free LDS
    float* cl = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) cl[rp * 512 + 256 * u + 4 * lane + e] = csum[4 * u + e];
    __syncthreads();
    {
      const int col = tid, si = col >> 6;
      if (si < nslab && ((G.csown >> si) & 1)) {
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) v += cl[r * 512 + col];
        const int j = G.base[si] + (col & 63);
        if (j < p.J) p.cs[(long long)chunk * p.ncols + j] = v;
      }
    }
  }
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
// input X [M][H][W][C] (f32, dense) and output gradient dY [M][OH][OW][CO];
// xmax / ymax: device bit patterns of the X bound and of max |dY| (the operand
// scales, f16x2_scale).
inline int band_layer(const float* X, int H, int W, int C, int KH, int KW, int S, const float* dy,
                      int CO, int M, float* ws, long long ws_cap, float* grad, float* astat,
                      float wscale, const unsigned* xmax, const unsigned* ymax, hipStream_t s,
                      int site = 0) {
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
  // 32-bit element offsets inside the kernel
  ACMI_REQUIRE((long long)M * g.kp < (1LL << 31) && (long long)M * g.L * CO < (1LL << 31), ACMI_ERR_ARG,
               "band_layer: %d images exceed 32-bit offsets", M);
  float* part = ws;
  float* cs = ws + (long long)nc * tile_f;
  BandArgs a;
  a.X = X;
  a.dy = dy;
  a.kp = g.kp;
  a.ldy = g.L * CO;
  a.J = g.J;
  a.M = M;
  a.k_chunk = ch;
  a.nc = nc;
  a.groups = d->groups;
  a.xlist = d->tabs + d->o_xlist;
  for (int x = 0; x < 9; ++x) a.xoff[x] = d->xoff[x];
  a.xmax = xmax;
  a.ymax = ymax;
  a.part = part;
  a.cs = cs;
  a.ntiles = p.ntiles;
  a.ncols = (int)ncols;
  prof_begin(site, s);
  // one block per item (512 threads, 64 KB of LDS, two waves per SIMD): 8 x the
  // longest XCD list; the blocks past a shorter list's end exit at once
  int maxg = 0;
  for (int x = 0; x < 8; ++x) maxg = std::max(maxg, d->xoff[x + 1] - d->xoff[x]);
  hipLaunchKernelGGL(band_kernel, dim3(8 * maxg * nc), dim3(512), 0, s, a);
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
