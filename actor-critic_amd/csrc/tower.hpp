// Fused conv tower of the forward: conv1 -> conv2 -> conv3 of ONE image per
// block, the activations passing through LDS (envs/atari/model.py:177-195).
//
// At the rollout batch (512 images per launch) the per-layer kernels are
// latency-bound: each walks its K loop one staged K-tile at a time (conv1 8,
// conv2 16, conv3 36 k16-steps behind one global load each), 27 + 31 + 19 us
// for ~6 us of MFMA work each.  Here a block loads its u8 image once (28 KB),
// keeps a1 (51 KB) in LDS for conv2 and a2 (21 KB, over the image) for conv3,
// and streams only the weights: every lane loads its B fragment (8 k of one
// output column) straight from global/L2 one k-step ahead, already split into
// f16 h/l by acmi_conv_prepare (once per parameter version) -- no weight
// staging, so 79 KB of LDS and two blocks (8 waves) per CU hold all 512 images
// of a rollout step at once.  (Without prepared weights the forward runs the
// per-layer kernels instead.)
//
// Arithmetic: f16x2 split operands (f16x2.hpp), each tensor scaled by a power of
// two from a bound the prepare step computes (tower_stats_body, in acmi_conv_prepare's first launch): the weights'
// max |W|, and the a1 / a2 bounds of band.hpp (ReLU outputs of [0,1] pixels
// under the positive weight mass).  conv1: u8 pixels exact as f16 subnormals
// (one byte permute per two), two MFMAs per k16 against the weights' h/l (bf16x3
// took three); conv2 / conv3: the a1 / a2 images in LDS hold the activations
// already split (h, l written once by the producing epilogue, tow_put), three
// MFMAs per product (bf16x3: six); the accumulators unscaled in the epilogue's
// bias fma -- f32-accurate.  The LDS images use convfwd3.hpp's 16-byte chunk
// swizzle by pixel x, so the lanes of a fragment read hit distinct banks.
// Work per block: conv1 three row tiles per wave + the 13th by K halves on two
// waves (roles rotated by block parity: equal per-SIMD load); conv2 the 3x2
// tiles as one full tile + half the K of row tile 2 per wave (the halves summed
// in wave order through LDS); conv3 (C3 = 32) two row tiles x two K halves.
// Every output pixel of every layer is the sum of two K halves, (first) +
// (second), each an MFMA chain from zero: a wave running a tile's whole K keeps
// the first half's accumulator and restarts at the midpoint.  That is the
// partition towersplit.hpp (one image over 7 workgroups, small batches) can run
// in parallel, so the two towers agree bit for bit.
// Activations are also written to global memory (strided rows, like EpiAct) for
// the update's backward and K-FAC statistics.
#pragma once

#include "conv1u8.hpp"
#include "f16x2.hpp"

namespace acmi {

constexpr int kTowObs = 84 * 84 * 4;       // u8 image, later a2 [81][64] f32 + scratch
constexpr int kTowA1 = 400 * 32 * 4;       // a1 [400][32] f32
constexpr int kTowLds = kTowObs + kTowA1;  // 79,424 B
constexpr int kTowScr = 16 * 32 * 4;       // conv1's 13th row tile, second K half
static_assert(2 * (kTowLds + kTowScr) <= 160 * 1024, "two blocks per CU");
static_assert(81 * 64 * 4 + 2 * 17 * 32 * 4 <= kTowObs, "a2 + conv2 scratch fit the image region");

// The a1 / a2 LDS images hold each activation already split (h, l f16 parts of
// the scaled value, written once by the producing layer's epilogue) instead of
// the f32 value split again by every wave that reads it (a1 pixels feed up to 4
// conv2 taps x 4 waves, a2 pixels up to 9 conv3 taps): per pixel [part][C] f16
// = C * 4 bytes, the 16-byte chunk c (8 channels of one part; c < C/8: h, else
// l) at chunk position c ^ (p / S) % (C/4) -- the fragment reads of one
// instruction (consecutive output pixels, input pixel p stepping by S within an
// output row) land on distinct chunk positions.  (Swizzling by the column x = p
// mod W instead, as convfwd3.hpp chunk_pos does, costs the producing epilogue a
// mod per row: ~5 of its ~21 VALU per stored row.)
#ifndef ACMI_TOW_PSWZ  // 1: swizzle by p / S (no p mod W in the producing epilogues); 0: by x / S
#define ACMI_TOW_PSWZ 1
#endif
template <int C, int S>
__device__ __forceinline__ int tow_pos(int p, int x, int c) {
  if constexpr (ACMI_TOW_PSWZ) return p * C * 4 + 16 * (c ^ ((p / S) & (C / 4 - 1)));
  return p * C * 4 + 16 * (c ^ ((x / S) & (C / 4 - 1)));
}
// byte offset of channel ch's part (0: h, 1: l) of pixel p
template <int C, int S>
__device__ __forceinline__ int tow_elem(int p, int x, int ch, int part) {
  return tow_pos<C, S>(p, x, part * (C / 8) + (ch >> 3)) + 2 * (ch & 7);
}
// the split of v (scaled by s) into the image
template <int C, int S>
__device__ __forceinline__ void tow_put(char* img, int p, int x, int ch, float v, float s) {
  const _Float16 h = (_Float16)(v * s);
  const _Float16 l = (_Float16)fmaf(v, s, -(float)h);
  // the l chunk's position is the h chunk's XOR C/8 (h chunks c < C/8, a power of
  // two, so (c + C/8) ^ sw == (c ^ sw) ^ C/8), and the pixel base p*4C keeps that
  // address bit clear: one XOR instead of a second swizzle
  const int eh = tow_elem<C, S>(p, x, ch, 0);
  *reinterpret_cast<_Float16*>(img + eh) = h;
  *reinterpret_cast<_Float16*>(img + (eh ^ (2 * C))) = l;
}

// conv1's epilogue addressing (C = 32, S = 2, swizzle by pixel index): for the
// row p = 32 T + tow_row(R, lane) of row tile T, the h element of channel col
// lies at T * 4096 + 128 (R & 3) + 1024 (R >> 2) + lv[k(R)] with the lane part
// lv[k] = 512 hl + 2 (col & 7) + (16 ((col >> 3) ^ 2 hl) ^ 16 kb(k)), because
// (p / 2) & 7 = ((R >> 1) & 1) | hl << 1 | ((R >> 2) & 1) << 2 for every T; the
// l element XOR 64.  So a row costs no address arithmetic: the four XOR variants
// are formed once, the row's constant lands in the ds_write offset field (and in
// the buffer store's for the global copy: 128 (R & 3) + 1024 (R >> 2) < 4096).
static_assert(ACMI_TOW_PSWZ == 1, "Tow1Addr assumes the pixel-index swizzle");
struct Tow1Addr {
  int lh[4], ll[4];  // h / l lane parts of the 4 XOR variants
  int go;            // lane part of the global byte offset: 512 hl + 4 col
  __device__ explicit Tow1Addr(int lane) {
    const int col = lane & 31, hl = lane >> 5;
    const int x = 512 * hl + 2 * (col & 7) + 16 * ((col >> 3) ^ (hl << 1));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      lh[k] = x ^ (16 * ((k & 1) | ((k >> 1) << 2)));
      ll[k] = lh[k] ^ 64;
    }
    go = 512 * hl + 4 * col;
  }
};
template <int R>
constexpr int tow1_roff() { return 128 * (R & 3) + 1024 * (R >> 2); }  // bytes, the lane-independent row part
template <int R>
constexpr int tow1_k() { return ((R >> 1) & 1) | (((R >> 2) & 1) << 1); }
// tow_put<32, 2> of row tile T's element R (img: the a1 image)
template <int R>
__device__ __forceinline__ void tow1_put(char* img, int T, const Tow1Addr& ad, float v, float s) {
  const _Float16 h = (_Float16)(v * s);
  const _Float16 l = (_Float16)fmaf(v, s, -(float)h);
  char* base = img + T * 4096;
  *reinterpret_cast<_Float16*>(base + ad.lh[tow1_k<R>()] + tow1_roff<R>()) = h;
  *reinterpret_cast<_Float16*>(base + ad.ll[tow1_k<R>()] + tow1_roff<R>()) = l;
}

// conv2's epilogue addressing (C = 64, S = 1): row p = 32 T + tow_row(R, lane),
// column c: (p & 15) = (R & 3) | hl << 2 | ((R >> 2) & 1) << 3, so the h element
// lies at T * 8192 + 256 (R & 3) + 2048 (R >> 2) + lh[k(R)] with lh[k] =
// 1024 hl + 2 (c & 7) + (16 ((c >> 3) ^ 4 hl) ^ 16 kr(k)); the l element (XOR
// 128) is the variant with kr's bit 3 flipped, lh[k ^ 4].
struct Tow2Addr {
  int lh[8];
  int go;  // lane part of the global byte offset: 1024 hl + 4 c
  __device__ Tow2Addr(int lane, int c) {
    const int hl = lane >> 5;
    const int x = 1024 * hl + 2 * (c & 7) + 16 * ((c >> 3) ^ (hl << 2));
#pragma unroll
    for (int k = 0; k < 8; ++k) lh[k] = x ^ (16 * ((k & 3) | ((k >> 2) << 3)));
    go = 1024 * hl + 4 * c;
  }
};
template <int R>
constexpr int tow2_roff() { return 256 * (R & 3) + 2048 * (R >> 2); }
template <int R>
constexpr int tow2_k() { return (R & 3) | (((R >> 2) & 1) << 2); }
template <int R>
__device__ __forceinline__ void tow2_put(char* img, int T, const Tow2Addr& ad, float v, float s) {
  const _Float16 h = (_Float16)(v * s);
  const _Float16 l = (_Float16)fmaf(v, s, -(float)h);
  char* base = img + T * 8192;
  *reinterpret_cast<_Float16*>(base + ad.lh[tow2_k<R>()] + tow2_roff<R>()) = h;
  *reinterpret_cast<_Float16*>(base + ad.lh[tow2_k<R>() ^ 4] + tow2_roff<R>()) = l;
}

// a1 / a2 to global memory: read again only by the update, after the rollout
#ifndef ACMI_TOW_NT
#define ACMI_TOW_NT 1
#endif
struct TowOut {  // one image's a1 / a2 in global memory as a buffer (SGPR base, 32-bit lane offsets)
  __amdgpu_buffer_rsrc_t rs;
  __device__ TowOut(float* base, int nfloats)
      : rs(__builtin_amdgcn_make_buffer_rsrc(base, (short)0, nfloats * 4, 0x00020000)) {}
  __device__ __forceinline__ void store(int i, float v) const {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, 4 * i, 0, ACMI_TOW_NT ? 2 : 0);  // aux 2: nt
  }
  // at byte offset vo (lane part) + IMM (compile time, as the scalar offset: a
  // vo + IMM sum was formed by VALU ORs per row instead of the offset field)
  template <int IMM>
  __device__ __forceinline__ void store_imm(int vo, float v) const {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, vo, IMM, ACMI_TOW_NT ? 2 : 0);
  }
};
// Prepared weights (acmi_conv_prepare): conv1/conv2/conv3 weights split once
// per parameter version into the f16 h/l parts of every lane's B fragment,
// fragment-major -- [k16 step][32-col tile][part h,l][lane] x 16 B -- so the
// tower loads them with one 16-byte load per part instead of 8 scalar loads and
// a split per k-step and wave; then a header of bounds (bit patterns, for the
// atomicMax of tower_stats_body): max |W1|, |W2|, |W3|, the a1, a2 and a3
// bounds, max |W4| (fc4roll.hpp's prepared fc4 reads the last two).
template <int C3>
struct TowerPrep {
  static constexpr long long FRAG = 2 * 64 * 16;  // bytes per (k-step, col tile)
  static constexpr long long O1 = 0, N1 = 16 * 1;             // conv1: 16 steps x 1 tile
  static constexpr long long O2 = O1 + N1 * FRAG, N2 = 32 * 2;  // conv2: 32 x 2
  static constexpr long long O3 = O2 + N2 * FRAG, N3 = 36 * (C3 / 32);
  static constexpr long long HDR = O3 + N3 * FRAG;  // 8 published bounds (common.hpp)
  static constexpr long long HDR_BYTES = 8 * 4 * kAmaxWords;
  static constexpr long long BYTES = HDR + HDR_BYTES;
};
enum {
  kTowMaxW1 = 0 * kAmaxWords, kTowMaxW2 = 1 * kAmaxWords, kTowMaxW3 = 2 * kAmaxWords, kTowMaxA1 = 3 * kAmaxWords,
  kTowMaxA2 = 4 * kAmaxWords, kTowMaxA3 = 5 * kAmaxWords, kTowMaxW4 = 6 * kAmaxWords
};

// the header's bounds (zeroed by the caller): 64 blocks of band.hpp's a1 / a2
// bounds (block c' takes conv2's column c') plus max |W| over all four layers
// (block co of 64; 256 threads)
__device__ __forceinline__ void tower_stats_body(const float* w1, const float* b1, const float* w2, const float* b2,
                                                 const float* w3, int n3, const float* w4, int n4, unsigned* hdr,
                                                 int co) {
  __shared__ float part[8][32];
  __shared__ float B1[32];
  __shared__ float red[4];
  const int t = threadIdx.x;
  {
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
  const float v = fmaxf(w2[t * 64 + co], 0.f) * B1[t & 31] + fmaxf(w2[(t + 256) * 64 + co], 0.f) * B1[t & 31];
  const float sum = wave_sum(v);
  if ((t & 63) == 0) red[t >> 6] = sum;
  // max |W| of the four layers over the grid: float4 runs, four loads in flight
  // per thread (one dependent load per element of fc4's 49*C3*512 was 16 us)
  auto absmax = [&](const float* w, int n) {
    float m = 0.f;
    if (((uintptr_t)w & 15) == 0 && n % 4 == 0) {
      const float4* w4v = reinterpret_cast<const float4*>(w);
      const int n4v = n / 4;
      int i = co * 256 + t;
      for (; i + 3 * 64 * 256 < n4v; i += 4 * 64 * 256) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = w4v[i + u * 64 * 256];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
      }
      for (; i < n4v; i += 64 * 256) {
        const float4 v = w4v[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
    } else {
      for (int i = co * 256 + t; i < n; i += 64 * 256) m = fmaxf(m, fabsf(w[i]));
    }
    return m;
  };
  float m1 = absmax(w1, 8192), m2 = absmax(w2, 32768), m3 = absmax(w3, n3), m4 = absmax(w4, n4);
  m1 = wave_max(m1);
  m2 = wave_max(m2);
  m3 = wave_max(m3);
  m4 = wave_max(m4);
  if ((t & 63) == 0) {
    amax_update(hdr + kTowMaxW1, m1);
    amax_update(hdr + kTowMaxW2, m2);
    amax_update(hdr + kTowMaxW3, m3);
    amax_update(hdr + kTowMaxW4, m4);
  }
  __syncthreads();
  if (t == 0) {
    amax_update(hdr + kTowMaxA2, red[0] + red[1] + red[2] + red[3] + fmaxf(b2[co], 0.f));
    if (co == 0) {
      float m = 0.f;
      for (int c = 0; c < 32; ++c) m = fmaxf(m, B1[c]);
      amax_update(hdr + kTowMaxA1, m);
    }
  }
}

// the a3 bound from the final a2 bound: block co takes conv3's column co,
// a3 <= sum_k max(W3[k][co], 0) * max a2 + max(b3[co], 0)  (one wave per column)
__device__ __forceinline__ void tower_stats3_body(const float* w3, const float* b3, int C3, unsigned* hdr, int co) {
  const int t = threadIdx.x & 63;
  float acc = 0.f;
  for (int k = t; k < 576; k += 64) acc += fmaxf(w3[k * C3 + co], 0.f);
  acc = wave_sum(acc);
  const float a2 = amax_read(hdr + kTowMaxA2);
  if (t == 0) amax_update(hdr + kTowMaxA3, acc * a2 + fmaxf(b3[co], 0.f));
}

// (block b; 256 threads: four fragments)
__device__ __forceinline__ void tower_prep_body(const float* w1, const float* w2, const float* w3, int C3, char* out,
                                                const unsigned* hdr, int b) {
  const int g = b * 256 + threadIdx.x;  // (layer, step, tile, lane)
  const int lane = g & 63;
  int f = g >> 6;  // fragment index over the three layers
  const int n3 = 36 * (C3 / 32);
  const float* w;
  int N, s, ct, layer;
  long long o;
  if (f < 16) {
    w = w1, N = 32, s = f, ct = 0, o = 0, layer = 0;
  } else if ((f -= 16) < 64) {
    w = w2, N = 64, s = f >> 1, ct = f & 1, o = 16LL * 2 * 1024, layer = 1;
  } else if ((f -= 64) < n3) {
    w = w3, N = C3, s = f / (C3 / 32), ct = f % (C3 / 32), o = (16LL + 64) * 2 * 1024, layer = 2;
  } else {
    return;
  }
  const float sw = f16x2_scale_of_bits(hdr + layer * kAmaxWords);  // (f, so layer, is wave-uniform)
  const float* p = w + (16 * s + 8 * (lane >> 5)) * N + 32 * ct + (lane & 31);
  uint4 h, l;
  split2(p[0], p[N], sw, h.x, l.x);
  split2(p[2 * N], p[3 * N], sw, h.y, l.y);
  split2(p[4 * N], p[5 * N], sw, h.z, l.z);
  split2(p[6 * N], p[7 * N], sw, h.w, l.w);
  uint4* d = reinterpret_cast<uint4*>(out + o + ((long long)(s * (N / 32) + ct) * 2) * 1024) + lane;
  d[0] = h;
  d[64] = l;
}

// row of the 32x32 C/D fragment element r of `lane`
__device__ __forceinline__ int tow_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }
// llvm.amdgcn.writelane (no clang builtin in this toolchain): v_writelane that
// hipcc schedules and pads -- a VALU-written SGPR (the ballot, often vcc) needs 2
// wait states before a writelane reads it, which hipcc inserts (s_nop 1) or fills
__device__ int acmi_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
// the ReLU' words of element R's two rows (ballot halves: rows tow_row(R, 0) and
// tow_row(R, 32)) written into the lanes of the same index of mw
template <int R>
__device__ __forceinline__ uint32_t tow_mword(uint32_t mw, unsigned long long bal) {
  constexpr int rr = (R & 3) + 8 * (R >> 2);
  const uint32_t lo = (uint32_t)bal, hi = (uint32_t)(bal >> 32);
  // (an unpadded asm-string writelane straight after the v_cmp read a stale vcc_lo)
  mw = (uint32_t)acmi_writelane((int)lo, rr, (int)mw);
  mw = (uint32_t)acmi_writelane((int)hi, rr + 4, (int)mw);
  return mw;
}
// f(std::integral_constant<int, I>) for I = B .. E-1
template <int B, int E, class F>
__device__ __forceinline__ void tow_static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    tow_static_for<B + 1, E>(f);
  }
}

// a layer's B fragments from the prepared weights, kTowDepth k-steps ahead of
// the one computed (slot = k-step mod kTowDepth + 1, a compile-time index in the
// unrolled loops); H16: the h part only
#ifndef ACMI_TOW_DEPTH
#define ACMI_TOW_DEPTH 2
#endif
constexpr int kTowDepth = ACMI_TOW_DEPTH, kTowSlots = kTowDepth + 1;
template <int N, bool H16 = false, int D = kTowDepth>
struct TowB {
  static constexpr int SLOTS = D + 1;
  const char* prep;
  uint4 q[SLOTS][2];
  __device__ __forceinline__ void fetch(int s, int ct, int lane, int slot) {
    const uint4* p = reinterpret_cast<const uint4*>(prep + ((long long)(s * (N / 32) + ct) * 2) * 1024) + lane;
    q[slot][0] = p[0];
    if constexpr (!H16) q[slot][1] = p[64];
  }
  __device__ __forceinline__ void get(int slot, f16x8 (&b)[2]) {
    b[0] = as_f16x8(q[slot][0]);
    if constexpr (!H16) b[1] = as_f16x8(q[slot][1]);
  }
};


// The tower of image `img` by one 256-thread block over the caller's LDS
// (kTowLds + kTowScr bytes).  IMG_IN_LDS: the u8 image is already in the
// image region (written there by the fused rollout tail's env step, which
// also stored it to obs) and is not loaded again.
template <int C3, bool H16, bool IMG_IN_LDS>
__device__ __forceinline__ void tower_body(const uint8_t* obs, long long img_stride, const float* b1,
                                           const float* b2, const float* b3, float* a1g, float* a2g, float* a3g,
                                           long long st, const char* prep, uint32_t* m1g, uint32_t* m2g,
                                           uint32_t* m3g, char* lds, long long img) {
  using P = TowerPrep<C3>;
  const unsigned* hdr = reinterpret_cast<const unsigned*>(prep + P::HDR);
  const float sw1 = f16x2_scale_of_bits(hdr + kTowMaxW1), sw2 = f16x2_scale_of_bits(hdr + kTowMaxW2);
  const float sw3 = f16x2_scale_of_bits(hdr + kTowMaxW3), sa1 = f16x2_scale_of_bits(hdr + kTowMaxA1);
  const float sa2 = f16x2_scale_of_bits(hdr + kTowMaxA2);
  char* const imgL = lds;           // u8 image; later a2
  char* const a1L = lds + kTowObs;  // a1; later conv3 scratch
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, kh8 = lane >> 5;

  if constexpr (!IMG_IN_LDS) {  // the u8 image: all of a thread's 16-byte loads before its LDS stores
    constexpr int NT = 256;
    constexpr int N16 = kTowObs / 16, NPT = (N16 + NT - 1) / NT;
    const uint4* src = reinterpret_cast<const uint4*>(obs + img * img_stride);
    uint4 v[NPT];
#pragma unroll
    for (int q = 0; q < NPT; ++q) v[q] = src[min(tid + NT * q, N16 - 1)];
#pragma unroll
    for (int q = 0; q < NPT; ++q)
      if (tid + NT * q < N16) reinterpret_cast<uint4*>(imgL)[tid + NT * q] = v[q];
  }
  // ---- conv1: [84][84][4] u8 -> a1 [20][20][32] -------------------------------
  {
    // row tiles w, w+4, w+8 of 13 for logical wave w; the 13th tile (rows
    // 384-399) by K halves on waves 2 (k-steps 0-7) and 3 (8-15), added through
    // LDS.  Odd blocks rotate the roles by two, so the two blocks of a CU give
    // every SIMD the same conv1 load: 3 + 3.5 tiles.
    const int w = (wave + 2 * (int)(img & 1)) & 3;
    auto tile_of = [&](int u) { return u < 3 ? w + 4 * u : 12; };
    int abase[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = min(32 * tile_of(u) + col, 399);
      const int oh = p / 20, ow = p - oh * 20;
      abase[u] = (4 * oh * 84 + 4 * ow) * 4 + 8 * kh8;
    }
    f32x16 acc[4], h0[3];  // h0: tiles u < 3, K half 0 (k-steps 0-7)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
    TowB<32, H16> bw{prep + P::O1};
#pragma unroll
    for (int i = 0; i < kTowDepth; ++i) bw.fetch(i, 0, lane, i);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s + kTowDepth < 16) bw.fetch(s + kTowDepth, 0, lane, (s + kTowDepth) % kTowSlots);
      f16x8 b[2];
      bw.get(s % kTowSlots, b);
      const int koff = (s >> 1) * 336 + 16 * (s & 1);  // kernel row kh = s/2, kw half
      if (s == 8) {  // every pixel sums its K halves (k-steps 0-7) + (8-15): the split tower's partition
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          h0[u] = acc[u];
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u == 3 && (w < 2 || (s >> 3) != w - 2)) continue;
        const f16x8 a = u8x8_to_f16(*reinterpret_cast<const uint2*>(imgL + abase[u] + koff));
        if constexpr (!H16) acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b[1], acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b[0], acc[u], 0, 0, 0);
      }
    }
    // 2^24 (subnormal pixels) / scale / 255: a power of two times f32(1/255), so
    // fma(v, inv1, bias) == fma(v * 2^24 / sw1, f32(1/255), bias) bit for bit
    const float bias = b1[col], inv1 = 16777216.0f / sw1 * (1.0f / 255.0f);
    const TowOut g(a1g + img * st * 12800, 12800);
    uint32_t* mg = m1g ? m1g + img * st * 400 : nullptr;
    // one row of the tile: returns the ReLU' ballot (bit = lane: the low word row
    // p of the lower half's pixel, the high word the upper half's)
    const Tow1Addr ad(lane);
    // row R of row tile T (pixel 32 T + tow_row(R, lane))
    auto emit1 = [&](auto RC, int T, float v) -> unsigned long long {
      constexpr int R = decltype(RC)::value;
      v = fmaxf(__builtin_fmaf(v, inv1, bias), 0.f);
      tow1_put<R>(a1L, T, ad, v, sa1);
      g.store_imm<tow1_roff<R>()>(T * 4096 + ad.go, v);
      return __ballot(v > 0.f);
    };
    // the tile's ReLU' words gathered by v_writelane (lane j: the tile's row j) and
    // stored by one instruction per tile instead of a masked store per row
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      uint32_t mw = 0;
      tow_static_for<0, 16>([&](auto R) {  // rows < 384
        constexpr int r = decltype(R)::value;
        mw = tow_mword<r>(mw, emit1(R, tile_of(u), h0[u][r] + acc[u][r]));
      });
      if (mg && lane < 32) mg[32 * tile_of(u) + lane] = mw;
    }
    float* scr12 = reinterpret_cast<float*>(lds + kTowLds);  // [16 rows][32]
    if (w == 3) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (tow_row(r, lane) < 16) scr12[tow_row(r, lane) * 32 + col] = acc[3][r];
    }
    __syncthreads();
    if (w == 2) {  // rows 384..399: r < 8 (tow_row(r, .) < 16 on every lane)
      uint32_t mw = 0;
      tow_static_for<0, 8>([&](auto R) {
        constexpr int r = decltype(R)::value;
        const int m = tow_row(r, lane);
        mw = tow_mword<r>(mw, emit1(R, 12, acc[3][r] + scr12[m * 32 + col]));
      });
      if (mg && lane < 16) mg[384 + lane] = mw;
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
    f32x16 accF, accH, hF;  // hF: row tile rtf, K half 0 (k-steps 0-15)
#pragma unroll
    for (int r = 0; r < 16; ++r) accF[r] = accH[r] = 0.f;
    TowB<64, H16> bw{prep + P::O2};
#pragma unroll
    for (int i = 0; i < kTowDepth; ++i) bw.fetch(i, ct, lane, i);
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      if (s + kTowDepth < 32) bw.fetch(s + kTowDepth, ct, lane, (s + kTowDepth) % kTowSlots);
      f16x8 b[2];
      bw.get(s % kTowSlots, b);
      const int tap = s >> 1, kh = tap >> 2, kw = tap & 3;
      const int c8 = 2 * (s & 1) + kh8;  // the 8 channels of this k-step and lane half
      if (s == 16) {  // every pixel sums its K halves (0-15) + (16-31)
        hF = accF;
#pragma unroll
        for (int r = 0; r < 16; ++r) accF[r] = 0.f;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && (s < hk0 || s >= hk0 + 16)) continue;
        const int p = pin[u] + kh * 20 + kw, x = px[u] + kw;
        f16x8 a[2];
        a[0] = *reinterpret_cast<const f16x8*>(a1L + tow_pos<32, 2>(p, x, c8));
        if constexpr (!H16) a[1] = *reinterpret_cast<const f16x8*>(a1L + tow_pos<32, 2>(p, x, 4 + c8));
        if constexpr (H16) {
          if (u == 0) accF = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], accF, 0, 0, 0);
          else accH = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], accH, 0, 0, 0);
          continue;
        }
        if (u == 0) accF = mfma_x2(a, b, accF);
        else accH = mfma_x2(a, b, accH);
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
    const float bias = b2[c], inv2 = 1.0f / (sa1 * sw2);  // exact: powers of two
    const TowOut g(a2g + img * st * 5184, 5184);
    uint32_t* mg = m2g ? m2g + img * st * 162 : nullptr;
    // (act: the lane's row exists; the ballot runs on every lane)
    const Tow2Addr ad(lane, c);
    // row R of row tile T (pixel 32 T + tow_row(R, lane))
    auto emit = [&](auto RC, int T, float v, bool act) -> unsigned long long {
      constexpr int R = decltype(RC)::value;
      v = fmaxf(__builtin_fmaf(v, inv2, bias), 0.f);
      if (act) {
        tow2_put<R>(imgL, T, ad, v, sa2);
        g.store_imm<tow2_roff<R>()>(T * 8192 + ad.go, v);
      }
      return __ballot(act && v > 0.f);
    };
    {
      uint32_t mw = 0;
      tow_static_for<0, 16>([&](auto R) {  // rows 0..63 are all valid
        constexpr int r = decltype(R)::value;
        mw = tow_mword<r>(mw, emit(R, rtf, hF[r] + accF[r], true));
      });
      if (mg && lane < 32) mg[2 * (32 * rtf + lane) + ct] = mw;
    }
    if (wave < 2) {  // rows 64..80: r < 8 on every lane, r = 8 (row 80) on the lower half
      uint32_t mw = 0;
      tow_static_for<0, 9>([&](auto R) {
        constexpr int r = decltype(R)::value;
        const int m = tow_row(r, lane);
        const bool act = m < 17;
        mw = tow_mword<r>(mw, emit(R, 2, act ? accH[r] + scr[(ct * 17 + m) * 32 + col] : 0.f, act));
      });
      if (mg && lane < 17) mg[2 * (64 + lane) + ct] = mw;
    }
  }
  __syncthreads();

  // ---- conv3: a2 -> a3 [7][7][C3] -------------------------------------------------
  {
    constexpr int NS = 36;  // k16 steps (576 / 16)
    const int rt = wave & 1;
    const int ct = C3 == 64 ? (wave >> 1) : 0;
    const int s0 = C3 == 64 ? 0 : 18 * (wave >> 1);
    const int p0 = min(32 * rt + col, 48);
    const int oh = p0 / 7, ow = p0 - oh * 7;
    const int pin = oh * 9 + ow;
    f32x16 acc, h3;  // h3 (C3 = 64): K half 0 (k-steps 0-17)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    TowB<C3, H16> bw{prep + P::O3};
    constexpr int NK = C3 == 64 ? NS : NS / 2;  // k-steps per wave: [s0, s0 + NK)
#pragma unroll
    for (int i = 0; i < kTowDepth; ++i) bw.fetch(s0 + i, ct, lane, i);
#pragma unroll
    for (int i = 0; i < NK; ++i) {
      const int ss = s0 + i;
      if (C3 == 64 && i == NS / 2) {  // every pixel sums its K halves (0-17) + (18-35)
        h3 = acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      }
      if (i + kTowDepth < NK) bw.fetch(ss + kTowDepth, ct, lane, (i + kTowDepth) % kTowSlots);
      f16x8 b[2];
      bw.get(i % kTowSlots, b);
      const int tap = ss >> 2, kh = tap / 3, kw = tap - kh * 3;
      const int c8 = 2 * (ss & 3) + kh8;
      const int p = pin + kh * 9 + kw, x = ow + kw;
      f16x8 a[2];
      a[0] = *reinterpret_cast<const f16x8*>(imgL + tow_pos<64, 1>(p, x, c8));
      if constexpr (!H16) a[1] = *reinterpret_cast<const f16x8*>(imgL + tow_pos<64, 1>(p, x, 8 + c8));
      if constexpr (H16) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], acc, 0, 0, 0);
        continue;
      }
      acc = mfma_x2(a, b, acc);
    }
    const int c = 32 * ct + col;
    const float bias = b3[c], inv3 = 1.0f / (sa2 * sw3);
    float* g = a3g + img * st * (49 * C3);
    uint32_t* mg = m3g ? m3g + img * st * (49 * C3 / 32) : nullptr;
    // (act: the lane's row exists; the ballot runs on every lane)
    auto emit3 = [&](int p, float v, bool act) -> unsigned long long {
      v = fmaxf(__builtin_fmaf(v, inv3, bias), 0.f);
      if (act) g[p * C3 + c] = v;
      return __ballot(act && v > 0.f);
    };
    // rows 32 rt + tow_row(r, lane) < 49: row tile 0 all 16 r; row tile 1 r < 8 on
    // every lane and r = 8 (row 48) on the lower half; the ReLU' words gathered by
    // v_writelane and stored once per tile
    auto emit_tile = [&](auto get) {
      uint32_t mw = 0;
      if (rt == 0) {
        tow_static_for<0, 16>([&](auto R) {
          constexpr int r = decltype(R)::value;
          mw = tow_mword<r>(mw, emit3(tow_row(r, lane), get(r), true));
        });
      } else {
        tow_static_for<0, 9>([&](auto R) {
          constexpr int r = decltype(R)::value;
          const int p = 32 + tow_row(r, lane);
          const bool act = p < 49;
          mw = tow_mword<r>(mw, emit3(p, act ? get(r) : 0.f, act));
        });
      }
      if (mg && lane < (rt ? 17 : 32)) mg[(32 * rt + lane) * (C3 / 32) + ct] = mw;
    };
    if constexpr (C3 == 32) {  // the second K half (waves 2, 3) through LDS to the first
      float* scr = reinterpret_cast<float*>(a1L);  // [rt][32 rows][32]
      if (wave >= 2) {
#pragma unroll
        for (int r = 0; r < 16; ++r) scr[(rt * 32 + tow_row(r, lane)) * 32 + col] = acc[r];
      }
      __syncthreads();
      if (wave < 2) emit_tile([&](int r) { return acc[r] + scr[(rt * 32 + tow_row(r, lane)) * 32 + col]; });
    } else {
      emit_tile([&](int r) { return h3[r] + acc[r]; });
    }
  }
}

template <int C3, bool H16 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void tower_kernel(const uint8_t* obs, long long img_stride, const float* b1, const float* b2,
                  const float* b3, float* a1g, float* a2g, float* a3g, long long st, const char* prep,
                  uint32_t* m1g, uint32_t* m2g, uint32_t* m3g) {
  __shared__ __attribute__((aligned(16))) char lds[kTowLds + kTowScr];
  tower_body<C3, H16, false>(obs, img_stride, b1, b2, b3, a1g, a2g, a3g, st, prep, m1g, m2g, m3g, lds,
                             blockIdx.x);
}
// prep: acmi_conv_prepare's fragments + bounds (required)
template <int C3>
inline void launch_tower(const uint8_t* obs, long long img_stride, int B, const float* P,
                         const long long* off, float* a1, float* a2, float* a3, long long st,
                         const void* prep, hipStream_t s, bool h16, uint32_t* m1, uint32_t* m2, uint32_t* m3) {
  const char* pp = static_cast<const char*>(prep);
  if (h16)
    hipLaunchKernelGGL((tower_kernel<C3, true>), dim3(B), dim3(256), 0, s, obs, img_stride, P + off[1],
                       P + off[3], P + off[5], a1, a2, a3, st, pp, m1, m2, m3);
  else
    hipLaunchKernelGGL((tower_kernel<C3, false>), dim3(B), dim3(256), 0, s, obs, img_stride, P + off[1],
                       P + off[3], P + off[5], a1, a2, a3, st, pp, m1, m2, m3);
}

}  // namespace acmi
