// The conv tower of ONE image split over kSplitParts workgroups (small rollout
// batches): part j computes conv3's output row j and, redundantly, the conv1 /
// conv2 rows that row needs -- no data passes between the parts.
//
// At B <= kSplitMaxB images a rollout step puts one workgroup per image on a
// 256-CU chip: the tower (tower.hpp) then runs one image's 13.7 MFLOP on one
// CU while most of the chip idles (configs[2], 32 envs: 21.6 us per fused
// tail + tower, ~14 of it the tower).  Part j of image n:
//   conv3 row j (7 pixels)        <- a2 rows j .. j+2 (27 pixels)
//                                 <- a1 rows 2j .. 2j+7 (160 pixels = 5 tiles)
//                                 <- input rows 8j .. 8j+35
// Each activation row is WRITTEN (a1 / a2 / a3 and their ReLU' words) by
// exactly one part (split_a1_lo/hi, split_a2_lo/hi), the others keep theirs in LDS.
//
// Bit-identical to the one-block tower (tower.hpp): every output pixel of every
// layer is the sum (K half 0) + (K half 1) of two MFMA chains from zero there and
// here, with the tower's f16x2 operands, scales, epilogue and LDS images
// (tow_pos / tow_put).  Per part: conv1 tiles 0-3 both halves on waves 0-3, tile
// 4's halves on waves 0 and 1; conv2 column tile x K half per wave; conv3 K half
// (x column tile at C3 = 64) per wave -- the critical wave issues 24 + 16 + 18
// k-steps against the one-block tower's ~90.
#pragma once

#include "tower.hpp"

namespace acmi {

constexpr int kSplitParts = 7;   // = conv3's output rows
#ifndef ACMI_SPLIT_DEPTH  // k-steps of B fragments in flight per wave (tower.hpp TowB)
#define ACMI_SPLIT_DEPTH 2
#endif
constexpr int kSpDepth = ACMI_SPLIT_DEPTH, kSpSlots = kSpDepth + 1;
constexpr int kSplitMaxB = 64;   // images per launch the split path takes (7 x 64 = 448 workgroups)
constexpr int kSpA1Rows = 8;     // a1 rows per part
constexpr int kSpA1Px = kSpA1Rows * 20;  // 160 = 5 tiles of 32
constexpr int kSpA2Px = 27;      // a2 rows j .. j+2
// LDS: the u8 image (only input rows 8j .. 8j+35 are filled) | a1 image (160 px x
// 32 ch, h / l f16) | a2 image (27 px x 64 ch) | partial-tile scratch
constexpr int kSpImg = 84 * 84 * 4;
constexpr int kSpA1 = kSpA1Px * 32 * 4;
constexpr int kSpA2 = 32 * 64 * 4;
constexpr int kSpScr = 4 * 32 * 32 * 4;
constexpr int kSpLds = kSpImg + kSpA1 + kSpA2 + kSpScr;
static_assert(2 * kSpLds <= 160 * 1024, "two blocks per CU");

// the a1 / a2 rows part j writes (a partition of each layer's rows; every part
// computes a superset of its own)
__host__ __device__ constexpr int split_a1_lo(int j) { return j == 0 ? 0 : 2 * j + 2; }
__host__ __device__ constexpr int split_a1_hi(int j) { return j == 6 ? 19 : 2 * j + 3; }  // inclusive
__host__ __device__ constexpr int split_a2_lo(int j) { return j == 0 ? 0 : j + 2; }
__host__ __device__ constexpr int split_a2_hi(int j) { return j == 6 ? 8 : (j == 0 ? 2 : j + 2); }
// the input rows part j's conv1 reads, as 16-byte stack words [g0, g1)
__host__ __device__ constexpr int split_word_lo(int j) { return 8 * j * 21; }
__host__ __device__ constexpr int split_word_hi(int j) { return (8 * j + 36) * 21 < 1764 ? (8 * j + 36) * 21 : 1764; }
// the stack words part j files into obs_out (rows 12j .. 12j+11)
__host__ __device__ constexpr int split_own_lo(int j) { return 12 * j * 21; }
__host__ __device__ constexpr int split_own_hi(int j) { return 12 * (j + 1) * 21; }

// Part j of image img over the caller's LDS (kSpLds bytes; the u8 image's input
// rows 8j .. 8j+35 already in place).  256 threads.
template <int C3, bool H16>
__device__ __forceinline__ void tower_part_body(int j, const float* b1, const float* b2, const float* b3,
                                                float* a1g, float* a2g, float* a3g, long long st, const char* prep,
                                                uint32_t* m1g, uint32_t* m2g, uint32_t* m3g, char* lds, long long img) {
  using P = TowerPrep<C3>;
  const unsigned* hdr = reinterpret_cast<const unsigned*>(prep + P::HDR);
  const float sw1 = f16x2_scale_of_bits(hdr + kTowMaxW1), sw2 = f16x2_scale_of_bits(hdr + kTowMaxW2);
  const float sw3 = f16x2_scale_of_bits(hdr + kTowMaxW3), sa1 = f16x2_scale_of_bits(hdr + kTowMaxA1);
  const float sa2 = f16x2_scale_of_bits(hdr + kTowMaxA2);
  char* const imgL = lds;
  char* const a1L = lds + kSpImg;
  char* const a2L = a1L + kSpA1;
  float* const scr = reinterpret_cast<float*>(a2L + kSpA2);  // [4][32][32]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, kh8 = lane >> 5;

  // ---- conv1: a1 rows 2j .. 2j+7 (local pixel q = global pixel - 40 j) ---------
  {
    // wave w: tile w (both K halves, the first kept at the midpoint); tile 4:
    // K half 0 on wave 0, half 1 on wave 1
    int abase[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = 32 * (u ? 4 : wave) + col;
      const int pg = 40 * j + q;
      const int oh = pg / 20, ow = pg - oh * 20;
      abase[u] = (4 * oh * 84 + 4 * ow) * 4 + 8 * kh8;
    }
    f32x16 acc[2], h0;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
    TowB<32, H16, kSpDepth> bw{prep + P::O1};
#pragma unroll
    for (int i = 0; i < kSpDepth; ++i) bw.fetch(i, 0, lane, i);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s + kSpDepth < 16) bw.fetch(s + kSpDepth, 0, lane, (s + kSpDepth) % kSpSlots);
      f16x8 b[2];
      bw.get(s % kSpSlots, b);
      const int koff = (s >> 1) * 336 + 16 * (s & 1);
      if (s == 8) {
        h0 = acc[0];
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[0][r] = 0.f;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && wave != (s >> 3)) continue;
        const f16x8 a = u8x8_to_f16(*reinterpret_cast<const uint2*>(imgL + abase[u] + koff));
        if constexpr (!H16) acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b[1], acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b[0], acc[u], 0, 0, 0);
      }
    }
    const float bias = b1[col], inv1 = 16777216.0f / sw1 * (1.0f / 255.0f);
    const TowOut g(a1g + img * st * 12800, 12800);
    uint32_t* mg = m1g ? m1g + img * st * 400 : nullptr;
    const int own_lo = 20 * split_a1_lo(j) - 40 * j, own_hi = 20 * (split_a1_hi(j) + 1) - 40 * j;  // local [lo, hi)
    const Tow1Addr ad(lane);
    // row R of local row tile u (local pixel q = 32 u + tow_row(R, lane))
    auto emit1 = [&](auto RC, int u, float v) -> unsigned long long {
      constexpr int R = decltype(RC)::value;
      const int q = 32 * u + tow_row(R, lane);
      v = fmaxf(__builtin_fmaf(v, inv1, bias), 0.f);
      tow1_put<R>(a1L, u, ad, v, sa1);
      if ((unsigned)(q - own_lo) < (unsigned)(own_hi - own_lo))
        g.store_imm<tow1_roff<R>()>((40 * j + 32 * u) * 128 + ad.go, v);
      return __ballot(v > 0.f);
    };
    auto tile_out = [&](int u, auto get) {
      uint32_t mw = 0;
      tow_static_for<0, 16>([&](auto R) {
        constexpr int r = decltype(R)::value;
        mw = tow_mword<r>(mw, emit1(R, u, get(r)));
      });
      const int q = 32 * u + lane;
      if (mg && lane < 32 && q >= own_lo && q < own_hi) mg[40 * j + q] = mw;
    };
    tile_out(wave, [&](int r) { return h0[r] + acc[0][r]; });
    // tile 4: half 1 (wave 1) through LDS to half 0 (wave 0)
    if (wave == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) scr[tow_row(r, lane) * 32 + col] = acc[1][r];
    }
    __syncthreads();
    if (wave == 0) tile_out(4, [&](int r) { return acc[1][r] + scr[tow_row(r, lane) * 32 + col]; });
  }
  __syncthreads();

  // ---- conv2: a2 rows j .. j+2 (local pixel q2 = global - 9 j) -----------------
  {
    const int ct = wave & 1, kq = wave >> 1;  // column tile, K half (k-steps 16 kq ..)
    const int q2 = min(col, kSpA2Px - 1);
    const int pin = 2 * (q2 / 9) * 20 + 2 * (q2 % 9);  // local a1 pixel of tap (0, 0)
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    TowB<64, H16, kSpDepth> bw{prep + P::O2};
#pragma unroll
    for (int i = 0; i < kSpDepth; ++i) bw.fetch(16 * kq + i, ct, lane, i);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int s = 16 * kq + i;
      if (i + kSpDepth < 16) bw.fetch(s + kSpDepth, ct, lane, (i + kSpDepth) % kSpSlots);
      f16x8 b[2];
      bw.get(i % kSpSlots, b);
      const int tap = s >> 1, kh = tap >> 2, kw = tap & 3;
      const int c8 = 2 * (s & 1) + kh8;
      const int p = pin + kh * 20 + kw, x = 2 * (q2 % 9) + kw;
      f16x8 a[2];
      a[0] = *reinterpret_cast<const f16x8*>(a1L + tow_pos<32, 2>(p, x, c8));
      if constexpr (!H16) a[1] = *reinterpret_cast<const f16x8*>(a1L + tow_pos<32, 2>(p, x, 4 + c8));
      if constexpr (H16) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], acc, 0, 0, 0);
      else acc = mfma_x2(a, b, acc);
    }
    // the second K half (waves 2, 3) through LDS to the first
    if (kq == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) scr[(ct * 32 + tow_row(r, lane)) * 32 + col] = acc[r];
    }
    __syncthreads();
    if (kq == 0) {
      const int c = 32 * ct + col;
      const float bias = b2[c], inv2 = 1.0f / (sa1 * sw2);
      const TowOut g(a2g + img * st * 5184, 5184);
      uint32_t* mg = m2g ? m2g + img * st * 162 : nullptr;
      const int own_lo = 9 * split_a2_lo(j) - 9 * j, own_hi = 9 * (split_a2_hi(j) + 1) - 9 * j;
      const Tow2Addr ad(lane, c);
      uint32_t mw = 0;
      tow_static_for<0, 16>([&](auto R) {
        constexpr int r = decltype(R)::value;
        const int m = tow_row(r, lane);
        const bool act = m < kSpA2Px;
        float v = acc[r] + scr[(ct * 32 + m) * 32 + col];
        v = fmaxf(__builtin_fmaf(v, inv2, bias), 0.f);
        if (act) {
          tow2_put<r>(a2L, 0, ad, v, sa2);
          if ((unsigned)(m - own_lo) < (unsigned)(own_hi - own_lo))
            g.store_imm<tow2_roff<r>()>(9 * j * 256 + ad.go, v);
        }
        mw = tow_mword<r>(mw, __ballot(act && v > 0.f));
      });
      if (mg && lane >= own_lo && lane < own_hi) mg[2 * (9 * j + lane) + ct] = mw;
    }
  }
  __syncthreads();

  // ---- conv3: a3 row j (7 pixels) ------------------------------------------------
  {
    // wave: column tile ct = wave & 1 (C3 = 64), K half kh (k-steps 18 kh ..)
    constexpr int NCT = C3 / 32;
    const int ct = C3 == 64 ? (wave & 1) : 0;
    const int kh = C3 == 64 ? (wave >> 1) : wave;
    const int q3 = min(col, 6);
    if (wave < 2 * NCT) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      TowB<C3, H16, kSpDepth> bw{prep + P::O3};
      const int s0 = 18 * kh;
#pragma unroll
      for (int i = 0; i < kSpDepth; ++i) bw.fetch(s0 + i, ct, lane, i);
#pragma unroll
      for (int i = 0; i < 18; ++i) {
        const int ss = s0 + i;
        if (i + kSpDepth < 18) bw.fetch(ss + kSpDepth, ct, lane, (i + kSpDepth) % kSpSlots);
        f16x8 b[2];
        bw.get(i % kSpSlots, b);
        const int tap = ss >> 2, kr = tap / 3, kc = tap - kr * 3;
        const int c8 = 2 * (ss & 3) + kh8;
        const int p = kr * 9 + q3 + kc, x = q3 + kc;
        f16x8 a[2];
        a[0] = *reinterpret_cast<const f16x8*>(a2L + tow_pos<64, 1>(p, x, c8));
        if constexpr (!H16) a[1] = *reinterpret_cast<const f16x8*>(a2L + tow_pos<64, 1>(p, x, 8 + c8));
        if constexpr (H16) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], acc, 0, 0, 0);
        else acc = mfma_x2(a, b, acc);
      }
      // rows 0..6 only (tow_row(r, lane) < 7): slot (kh, ct) = wave
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = tow_row(r, lane);
        if (m < 7) scr[(wave * 8 + m) * 32 + col] = acc[r];
      }
    }
    __syncthreads();
    // thread (pixel m = tid / 32 < 7, column c = tid % 32) of each column tile:
    // half 0 + half 1 (waves t and NCT + t)
    if (tid < 7 * 32) {
      const int m = tid >> 5, cc = tid & 31;
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        float v = scr[(t * 8 + m) * 32 + cc] + scr[((NCT + t) * 8 + m) * 32 + cc];
        const int c = 32 * t + cc;
        const float bias = b3[c], inv3 = 1.0f / (sa2 * sw3);
        v = fmaxf(__builtin_fmaf(v, inv3, bias), 0.f);
        a3g[img * st * (49 * C3) + (7 * j + m) * C3 + c] = v;
        const unsigned long long bal = __ballot(v > 0.f);  // lanes 0-31: pixel 2 mh, 32-63: 2 mh + 1
        if (m3g && (lane & 31) == 0)
          m3g[img * st * (49 * C3 / 32) + (7 * j + m) * NCT + t] = (uint32_t)(bal >> (lane & 32));
      }
    }
  }
}

}  // namespace acmi
