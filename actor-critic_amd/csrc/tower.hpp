// Fused conv tower of the forward: conv1 -> conv2 -> conv3 of ONE image per
// block, the activations passing through LDS (envs/atari/model.py:177-195).
//
// At the rollout batch (512 images per launch) the per-layer kernels are
// latency-bound: each walks its K loop one staged K-tile at a time (conv1 8,
// conv2 16, conv3 36 k16-steps behind one global load each), 27 + 31 + 19 us
// for ~6 us of MFMA work each.  Here a block loads its u8 image once (28 KB),
// keeps a1 (51 KB) in LDS for conv2 and a2 (21 KB, over the image) for conv3,
// and streams only the weights: every lane loads its B fragment (8 k of one
// output column) straight from global/L2 one k-step ahead -- already split into
// bf16 h/m/l when the caller prepared the weights (acmi_conv_prepare, once per
// parameter version), else split here -- no weight staging, so 79 KB of LDS and
// two blocks (8 waves) per CU hold all 512 images of a rollout step at once.
//
// Arithmetic: conv1 as conv1_fwd_x3 (u8 pixels exact in bf16, three MFMAs per
// k16 against the weights' h/m/l, scale 1/255 and bias in one fmaf); conv2 /
// conv3 bf16x3 on both operands (mfma_x3, symred3.hpp) -- f32-accurate.  The
// a1 / a2 LDS images use convfwd3.hpp's 16-byte chunk swizzle by pixel x, so
// the lanes of a fragment read (consecutive output columns) hit distinct banks.
// Work per block: conv1 three row tiles per wave + the 13th by K halves on two
// waves (roles rotated by block parity: equal per-SIMD load); conv2 the 3x2
// tiles as one full tile + half the K of row tile 2 per wave (the halves summed
// in wave order through LDS); conv3 (C3 = 32) two row tiles x two K halves.
// Activations are also written to global memory (strided rows, like EpiAct) for
// the update's backward and K-FAC statistics.
#pragma once

#include "conv1u8.hpp"
#include "symred3.hpp"

namespace acmi {

constexpr int kTowObs = 84 * 84 * 4;       // u8 image, later a2 [81][64] f32 + scratch
constexpr int kTowA1 = 400 * 32 * 4;       // a1 [400][32] f32
constexpr int kTowLds = kTowObs + kTowA1;  // 79,424 B
constexpr int kTowScr = 16 * 32 * 4;       // conv1's 13th row tile, second K half
static_assert(2 * (kTowLds + kTowScr) <= 160 * 1024, "two blocks per CU");
static_assert(81 * 64 * 4 + 2 * 17 * 32 * 4 <= kTowObs, "a2 + conv2 scratch fit the image region");

// byte offset of 16-byte channel chunk `ch` of pixel p (x = its column) in an
// f32 [pixel][C] LDS image read with stride S (convfwd3.hpp chunk_pos)
template <int C, int S>
__device__ __forceinline__ int tow_pos(int p, int x, int ch) {
  return p * C * 4 + 16 * (ch ^ ((x / S) & (C / 4 - 1)));
}

__device__ __forceinline__ bf16x8 tow_bf16x8(const float4& x0, const float4& x1) {
  uint4 h;
  h.x = pk_bf16(x0.x, x0.y);
  h.y = pk_bf16(x0.z, x0.w);
  h.z = pk_bf16(x1.x, x1.y);
  h.w = pk_bf16(x1.z, x1.w);
  return __builtin_bit_cast(bf16x8, h);
}

__device__ __forceinline__ void tow_split8(const float4& x0, const float4& x1, bf16x8 (&o)[3]) {
  uint4 h, m, l;
  split3(x0.x, x0.y, h.x, m.x, l.x);
  split3(x0.z, x0.w, h.y, m.y, l.y);
  split3(x1.x, x1.y, h.z, m.z, l.z);
  split3(x1.z, x1.w, h.w, m.w, l.w);
  o[0] = __builtin_bit_cast(bf16x8, h);
  o[1] = __builtin_bit_cast(bf16x8, m);
  o[2] = __builtin_bit_cast(bf16x8, l);
}

// lane's B fragment of k16-step s, output columns c0 .. c0+31 of W [K][N]:
// B[16s + 8(lane>>5) + e][c0 + (lane & 31)], e = 0..7
template <int N>
__device__ __forceinline__ void tow_bload(const float* w, int s, int c0, int lane, float4 (&x)[2]) {
  const float* p = w + (16 * s + 8 * (lane >> 5)) * N + c0 + (lane & 31);
  x[0] = make_float4(p[0], p[N], p[2 * N], p[3 * N]);
  x[1] = make_float4(p[4 * N], p[5 * N], p[6 * N], p[7 * N]);
}

// Prepared weights (acmi_conv_prepare): conv1/conv2/conv3 weights split once
// per parameter version into the bf16x3 parts of every lane's B fragment,
// fragment-major -- [k16 step][32-col tile][part h,m,l][lane] x 16 B -- so the
// tower loads them with one 16-byte load per part instead of 8 scalar loads and
// a split per k-step and wave (the split of each weight done once, not by every
// wave of every block).
template <int C3>
struct TowerPrep {
  static constexpr long long FRAG = 3 * 64 * 16;  // bytes per (k-step, col tile)
  static constexpr long long O1 = 0, N1 = 16 * 1;             // conv1: 16 steps x 1 tile
  static constexpr long long O2 = O1 + N1 * FRAG, N2 = 32 * 2;  // conv2: 32 x 2
  static constexpr long long O3 = O2 + N2 * FRAG, N3 = 36 * (C3 / 32);
  static constexpr long long BYTES = O3 + N3 * FRAG;
};

__global__ void tower_prep_kernel(const float* w1, const float* w2, const float* w3, int C3, char* out) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;  // (layer, step, tile, lane)
  const int lane = g & 63;
  int f = g >> 6;  // fragment index over the three layers
  const int n3 = 36 * (C3 / 32);
  const float* w;
  int N, s, ct;
  long long o;
  if (f < 16) {
    w = w1, N = 32, s = f, ct = 0, o = 0;
  } else if ((f -= 16) < 64) {
    w = w2, N = 64, s = f >> 1, ct = f & 1, o = 16LL * 3 * 1024;
  } else if ((f -= 64) < n3) {
    w = w3, N = C3, s = f / (C3 / 32), ct = f % (C3 / 32), o = (16LL + 64) * 3 * 1024;
  } else {
    return;
  }
  const float* p = w + (16 * s + 8 * (lane >> 5)) * N + 32 * ct + (lane & 31);
  uint4 h, m, l;
  split3(p[0], p[N], h.x, m.x, l.x);
  split3(p[2 * N], p[3 * N], h.y, m.y, l.y);
  split3(p[4 * N], p[5 * N], h.z, m.z, l.z);
  split3(p[6 * N], p[7 * N], h.w, m.w, l.w);
  uint4* d = reinterpret_cast<uint4*>(out + o + ((long long)(s * (N / 32) + ct) * 3) * 1024) + lane;
  d[0] = h;
  d[64] = m;
  d[128] = l;
}

// B fragment of k16-step s, column tile ct from the prepared weights
__device__ __forceinline__ void tow_bprep(const char* base, int s, int nct, int ct, int lane, uint4 (&x)[3]) {
  const uint4* p = reinterpret_cast<const uint4*>(base + ((long long)(s * nct + ct) * 3) * 1024) + lane;
  x[0] = p[0];
  x[1] = p[64];
  x[2] = p[128];
}

// row of the 32x32 C/D fragment element r of `lane`
__device__ __forceinline__ int tow_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// a layer's B fragments, two k-steps in flight (slot = k-step parity, always a
// compile-time index): prepared bf16 parts (PREP) or f32 weights split here
template <bool PREP, int N, bool BF16 = false>
struct TowB {
  const float* w;
  const char* prep;
  uint4 q[2][3];
  float4 f[2][2];
  __device__ __forceinline__ void fetch(int s, int ct, int lane, int slot) {
    if constexpr (PREP && BF16) {  // the h part only
      q[slot][0] = reinterpret_cast<const uint4*>(prep + ((long long)(s * (N / 32) + ct) * 3) * 1024)[lane];
    } else if constexpr (PREP) {
      tow_bprep(prep, s, N / 32, ct, lane, q[slot]);
    } else {
      tow_bload<N>(w, s, 32 * ct, lane, f[slot]);
    }
  }
  __device__ __forceinline__ void get(int slot, bf16x8 (&b)[3]) {
    if constexpr (PREP) {
#pragma unroll
      for (int i = 0; i < 3; ++i) b[i] = __builtin_bit_cast(bf16x8, q[slot][i]);
    } else {
      tow_split8(f[slot][0], f[slot][1], b);
    }
  }
};

// BF16 (acmi_set_forward_mode ACMI_FWD_BF16): one bf16 MFMA per product -- the
// weights' h part and conv2/conv3 inputs rounded to bf16 (u8 pixels exact).
template <int C3, bool PREP, bool BF16 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void tower_kernel(const uint8_t* obs, long long img_stride, const float* w1, const float* b1,
                  const float* w2, const float* b2, const float* w3, const float* b3, float* a1g,
                  float* a2g, float* a3g, long long st, const char* prep) {
  using P = TowerPrep<C3>;
  __shared__ __attribute__((aligned(16))) char lds[kTowLds + kTowScr];
  char* const imgL = lds;           // u8 image; later a2
  char* const a1L = lds + kTowObs;  // a1; later conv3 scratch
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, kh8 = lane >> 5;
  const long long img = blockIdx.x;

  {  // the u8 image: all of a thread's 16-byte loads before its LDS stores
    constexpr int N16 = kTowObs / 16, NPT = (N16 + 255) / 256;
    const uint4* src = reinterpret_cast<const uint4*>(obs + img * img_stride);
    uint4 v[NPT];
#pragma unroll
    for (int q = 0; q < NPT; ++q) v[q] = src[min(tid + 256 * q, N16 - 1)];
#pragma unroll
    for (int q = 0; q < NPT; ++q)
      if (tid + 256 * q < N16) reinterpret_cast<uint4*>(imgL)[tid + 256 * q] = v[q];
  }

  // ---- conv1: [84][84][4] u8 -> a1 [20][20][32] -------------------------------
  {
    // row tiles w, w+4, w+8 of 13 for logical wave w; the 13th tile (rows
    // 384-399) by K halves on waves 2 (k-steps 0-7) and 3 (8-15), added through
    // LDS.  Odd blocks rotate the roles by two, so the two blocks of a CU give
    // every SIMD the same conv1 load: 3 + 3.5 tiles.
    const int w = (wave + 2 * (blockIdx.x & 1)) & 3;
    auto tile_of = [&](int u) { return u < 3 ? w + 4 * u : 12; };
    int abase[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = min(32 * tile_of(u) + col, 399);
      const int oh = p / 20, ow = p - oh * 20;
      abase[u] = (4 * oh * 84 + 4 * ow) * 4 + 8 * kh8;
    }
    f32x16 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
    TowB<PREP, 32, BF16> bw{w1, prep + P::O1};
    bw.fetch(0, 0, lane, 0);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s + 1 < 16) bw.fetch(s + 1, 0, lane, (s + 1) & 1);
      bf16x8 b[3];
      bw.get(s & 1, b);
      const int koff = (s >> 1) * 336 + 16 * (s & 1);  // kernel row kh = s/2, kw half
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u == 3 && (w < 2 || (s >> 3) != w - 2)) continue;
        const bf16x8 a = u8x8_to_bf16(*reinterpret_cast<const uint2*>(imgL + abase[u] + koff));
        if constexpr (!BF16) {
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[2], acc[u], 0, 0, 0);
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[1], acc[u], 0, 0, 0);
        }
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[0], acc[u], 0, 0, 0);
      }
    }
    const float bias = b1[col];
    float* g = a1g + img * st * 12800;
    auto emit1 = [&](int p, float v) {
      v = fmaxf(__builtin_fmaf(v, 1.0f / 255.0f, bias), 0.f);
      *reinterpret_cast<float*>(a1L + tow_pos<32, 2>(p, p % 20, col >> 2) + 4 * (col & 3)) = v;
      g[p * 32 + col] = v;
    };
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) emit1(32 * tile_of(u) + tow_row(r, lane), acc[u][r]);  // rows < 384
    float* scr12 = reinterpret_cast<float*>(lds + kTowLds);  // [16 rows][32]
    if (w == 3) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (tow_row(r, lane) < 16) scr12[tow_row(r, lane) * 32 + col] = acc[3][r];
    }
    __syncthreads();
    if (w == 2) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = tow_row(r, lane);
        if (m < 16) emit1(384 + m, acc[3][r] + scr12[m * 32 + col]);
      }
    }
  }
  __syncthreads();

  // ---- conv2: a1 -> a2 [9][9][64] ------------------------------------------------
  {
    const int ct = wave & 1, rtf = wave >> 1, hk0 = 16 * (wave >> 1);
    int pin[2], px[2];  // tile 0: row tile rtf (full K); tile 1: row tile 2 (k16 steps hk0..hk0+15)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = min(32 * (u ? 2 : rtf) + col, 80);
      const int oh = p / 9, ow = p - oh * 9;
      pin[u] = 2 * oh * 20 + 2 * ow;
      px[u] = 2 * ow;
    }
    f32x16 accF, accH;
#pragma unroll
    for (int r = 0; r < 16; ++r) accF[r] = accH[r] = 0.f;
    TowB<PREP, 64, BF16> bw{w2, prep + P::O2};
    bw.fetch(0, ct, lane, 0);
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      if (s + 1 < 32) bw.fetch(s + 1, ct, lane, (s + 1) & 1);
      bf16x8 b[3];
      bw.get(s & 1, b);
      const int tap = s >> 1, kh = tap >> 2, kw = tap & 3;
      const int ch = 4 * (s & 1) + 2 * kh8;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && (s < hk0 || s >= hk0 + 16)) continue;
        const int p = pin[u] + kh * 20 + kw, x = px[u] + kw;
        const float4 x0 = *reinterpret_cast<const float4*>(a1L + tow_pos<32, 2>(p, x, ch));
        const float4 x1 = *reinterpret_cast<const float4*>(a1L + tow_pos<32, 2>(p, x, ch + 1));
        bf16x8 a[3];
        if constexpr (BF16) {
          a[0] = tow_bf16x8(x0, x1);
          if (u == 0) accF = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], accF, 0, 0, 0);
          else accH = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], accH, 0, 0, 0);
          continue;
        }
        tow_split8(x0, x1, a);
        if (u == 0) accF = mfma_x3(a, b, accF);
        else accH = mfma_x3(a, b, accH);
      }
    }
    // row tile 2: the second K half (waves 2, 3) through LDS to the first
    float* scr = reinterpret_cast<float*>(imgL + 81 * 64 * 4);  // [ct][17 rows][32]
    if (wave >= 2) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = tow_row(r, lane);
        if (m < 17) scr[(ct * 17 + m) * 32 + col] = accH[r];
      }
    }
    __syncthreads();
    const int c = 32 * ct + col;
    const float bias = b2[c];
    float* g = a2g + img * st * 5184;
    auto emit = [&](int p, float v) {
      v = fmaxf(__builtin_fmaf(v, 1.0f, bias), 0.f);
      *reinterpret_cast<float*>(imgL + tow_pos<64, 1>(p, p % 9, c >> 2) + 4 * (c & 3)) = v;
      g[p * 64 + c] = v;
    };
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int p = 32 * rtf + tow_row(r, lane);
      emit(p, accF[r]);  // rows 0..63 are all valid
    }
    if (wave < 2) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = tow_row(r, lane);
        if (m < 17) emit(64 + m, accH[r] + scr[(ct * 17 + m) * 32 + col]);
      }
    }
  }
  __syncthreads();

  // ---- conv3: a2 -> a3 [7][7][C3] -------------------------------------------------
  {
    constexpr int NS = 36;  // k16 steps (576 / 16)
    const int rt = wave & 1;
    const int ct = C3 == 64 ? (wave >> 1) : 0;
    const int s0 = C3 == 64 ? 0 : 18 * (wave >> 1), s1 = C3 == 64 ? NS : s0 + 18;
    const int p0 = min(32 * rt + col, 48);
    const int oh = p0 / 7, ow = p0 - oh * 7;
    const int pin = oh * 9 + ow;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    TowB<PREP, C3, BF16> bw{w3, prep + P::O3};
    bw.fetch(s0, ct, lane, 0);
    for (int s = s0; s < s1; s += 2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ss = s + h;
        if (ss + 1 < s1) bw.fetch(ss + 1, ct, lane, h ^ 1);
        bf16x8 b[3];
        bw.get(h, b);
        const int tap = ss >> 2, kh = tap / 3, kw = tap - kh * 3;
        const int ch = 4 * (ss & 3) + 2 * kh8;
        const int p = pin + kh * 9 + kw, x = ow + kw;
        const float4 x0 = *reinterpret_cast<const float4*>(imgL + tow_pos<64, 1>(p, x, ch));
        const float4 x1 = *reinterpret_cast<const float4*>(imgL + tow_pos<64, 1>(p, x, ch + 1));
        bf16x8 a[3];
        if constexpr (BF16) {
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tow_bf16x8(x0, x1), b[0], acc, 0, 0, 0);
          continue;
        }
        tow_split8(x0, x1, a);
        acc = mfma_x3(a, b, acc);
      }
    }
    const int c = 32 * ct + col;
    const float bias = b3[c];
    float* g = a3g + img * st * (49 * C3);
    if constexpr (C3 == 32) {  // the second K half (waves 2, 3) through LDS to the first
      float* scr = reinterpret_cast<float*>(a1L);  // [rt][32 rows][32]
      if (wave >= 2) {
#pragma unroll
        for (int r = 0; r < 16; ++r) scr[(rt * 32 + tow_row(r, lane)) * 32 + col] = acc[r];
      }
      __syncthreads();
      if (wave < 2) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int p = 32 * rt + tow_row(r, lane);
          if (p < 49)
            g[p * C3 + c] = fmaxf(__builtin_fmaf(acc[r] + scr[(rt * 32 + tow_row(r, lane)) * 32 + col], 1.0f,
                                                 bias), 0.f);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = 32 * rt + tow_row(r, lane);
        if (p < 49) g[p * C3 + c] = fmaxf(__builtin_fmaf(acc[r], 1.0f, bias), 0.f);
      }
    }
  }
}

template <int C3>
inline void launch_tower(const uint8_t* obs, long long img_stride, int B, const float* P,
                         const long long* off, float* a1, float* a2, float* a3, long long st,
                         const void* prep, hipStream_t s, bool bf16 = false) {
#define ACMI_TOWER(PR, BF)                                                                            \
  hipLaunchKernelGGL((tower_kernel<C3, PR, BF>), dim3(B), dim3(256), 0, s, obs, img_stride, P + off[0], \
                     P + off[1], P + off[2], P + off[3], P + off[4], P + off[5], a1, a2, a3, st,       \
                     static_cast<const char*>(prep))
  if (prep && bf16) ACMI_TOWER(true, true);
  else if (prep) ACMI_TOWER(true, false);
  else if (bf16) ACMI_TOWER(false, true);
  else ACMI_TOWER(false, false);
#undef ACMI_TOWER
}

inline void launch_tower_prep(const float* P, const long long* off, int C3, void* prep, hipStream_t s) {
  const int frags = 16 + 64 + 36 * (C3 / 32);
  hipLaunchKernelGGL(tower_prep_kernel, dim3(frags * 64 / 256 + 1), dim3(256), 0, s, P + off[0], P + off[2],
                     P + off[4], C3, static_cast<char*>(prep));
}

}  // namespace acmi
