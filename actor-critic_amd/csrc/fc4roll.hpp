// fc4 at the rollout batch (envs/atari/model.py:200-204 -> nn.py:37-52 at
// B = N images): the split-K partial slabs [nz][B+1][512] that
// rollout_tail_kernel / heads_kernel reduce, computed without LDS.
//
// At B = 512 the staged gemm3 launch (64x128 tiles, 8 K chunks, 256 blocks) is
// a chain of 13 dependent K-tiles, each behind one global load round trip and
// a barrier: 15 us for 2.4 GFLOP.  Here W4 comes pre-split into the f16 h/l
// parts of every lane's B fragment (acmi_conv_prepare, once per parameter
// version, fragment-major like the tower's weights), each wave loads its own
// A fragments (8 consecutive k of one row per lane: two float4) and its B
// fragments straight from L2, kFc4Depth k-steps ahead in registers, and owns a
// 32-row x 64-column tile of one K chunk -- no LDS, no barrier.  Blocks map K
// chunk z to XCD z (b % nz), so an XCD's L2 holds only its chunk's W4 columns
// (590 KB) and a3 columns (400 KB at B = 512).
//
// Arithmetic: f16x2 (f16x2.hpp) -- W4 scaled by its max |W4|, a3 by the weight-
// derived a3 bound of the tower's header (tower_stats3_body), three MFMAs per
// k16-step and tile, the slabs unscaled before they are stored: f32-class like
// the staged bf16x3 launch (test_fc4_rollout_matches_gemm3), not bit-identical.
#pragma once

#include "stepper.hpp"  // PendState, env_commit_pending
#include "tower.hpp"

namespace acmi {

#ifndef ACMI_FC4_DEPTH
#define ACMI_FC4_DEPTH 3
#endif
constexpr int kFc4Depth = ACMI_FC4_DEPTH;  // k-steps in flight ahead of the one computed

// W4 [K][512] -> [K/16 steps][16 col tiles][part h, l][64 lanes] x 16 B, scaled
// by the power of two of hdr[kTowMaxW4] (the tower's header)
// (block b; 256 threads)
__device__ __forceinline__ void fc4_prep_body(const float* w4, int K, char* out, const unsigned* hdr, int b) {
  const int g = b * 256 + threadIdx.x;
  const int lane = g & 63, f = g >> 6;  // f = step * 16 + col tile
  if (f >= (K / 16) * 16) return;
  const float sw = f16x2_scale_of_bits(hdr + kTowMaxW4);
  const int s = f >> 4, ct = f & 15;
  const float* p = w4 + (16 * s + 8 * (lane >> 5)) * 512 + 32 * ct + (lane & 31);
  uint4 h, l;
  split2(p[0], p[512], sw, h.x, l.x);
  split2(p[2 * 512], p[3 * 512], sw, h.y, l.y);
  split2(p[4 * 512], p[5 * 512], sw, h.z, l.z);
  split2(p[6 * 512], p[7 * 512], sw, h.w, l.w);
  uint4* d = reinterpret_cast<uint4*>(out) + (long long)f * 128 + lane;
  d[0] = h;
  d[64] = l;
}

inline long long fc4_prep_bytes(int K) { return (long long)(K / 16) * 16 * 2 * 1024; }

// block b: K chunk z = b % nz, then (row tile, column half); wave w: column
// group 4 * half + w (64 columns).
// commit: the split rollout step's pending env states (towersplit.hpp), written
// into the env state by block 0 before this step's tail reads them (commitB = 0:
// none).
struct Fc4Commit {
  PendState* pend;
  acmi_env_state_t st;
  int B;
};
// CT: 32-column tiles per wave (2; 1 at small batches: twice the blocks, half
// the MFMA chain per wave)
template <int CT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
void fc4_roll_kernel(const float* a3, long long lda, int B, int K, const char* w4p, int nz, int chunk_steps,
                     float* part, const unsigned* hdr, Fc4Commit cm) {
  if (cm.B > 0 && blockIdx.x == 0) env_commit_pending(cm.st, cm.pend, cm.B);
  constexpr int D = kFc4Depth, NSLOT = D + 1;
  constexpr int NG = 512 / (128 * CT);  // column groups of 4 waves
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int z = blockIdx.x % nz, rest = blockIdx.x / nz;
  const int rt = rest / NG, cg = 4 * (rest % NG) + wave;  // the wave's columns 32 CT cg ..
  const int s0 = z * chunk_steps;
  const int ns = min(K / 16, s0 + chunk_steps) - s0;
  const int col = lane & 31;
  const int row = min(32 * rt + col, B - 1);
  const float* ap = a3 + (long long)row * lda + 16 * s0 + 8 * (lane >> 5);
  // fragment (step s, col tile ct, part pt): uint4 index (s * 16 + ct) * 128 + 64 pt + lane
  const uint4* bp = reinterpret_cast<const uint4*>(w4p) + ((long long)s0 * 16 + CT * cg) * 128 + lane;
  const float sa = f16x2_scale_of_bits(hdr + kTowMaxA3);
  const float inv = 1.0f / (sa * f16x2_scale_of_bits(hdr + kTowMaxW4));  // exact

  float4 av[NSLOT][2];
  uint4 bv[NSLOT][CT][2];
  auto load = [&](int i, int slot) {
    const float4* a = reinterpret_cast<const float4*>(ap + 16 * i);
    av[slot][0] = a[0];
    av[slot][1] = a[1];
    const uint4* b = bp + (long long)i * 16 * 128;
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        bv[slot][t][pt] = b[t * 128 + 64 * pt];
      }
  };
  f32x16 acc[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (i < ns) load(i, i);
  // step i lives in slot i % NSLOT: a runtime loop over whole slot rounds with
  // the slots unrolled, so every register-array index is a constant
  for (int i0 = 0; i0 < ns; i0 += NSLOT) {
#pragma unroll
    for (int sl = 0; sl < NSLOT; ++sl) {
      const int i = i0 + sl;
      if (i < ns) {
        if (i + D < ns) load(i + D, (sl + D) % NSLOT);
        f16x8 a[2];
        split2x8(av[sl][0], av[sl][1], sa, a[0], a[1]);
#pragma unroll
        for (int t = 0; t < CT; ++t) {
          const f16x8 b[2] = {as_f16x8(bv[sl][t][0]), as_f16x8(bv[sl][t][1])};
          acc[t] = mfma_x2(a, b, acc[t]);
        }
      }
    }
  }
  float* out = part + (long long)z * (B + 1) * 512 + 32 * CT * cg + col;
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = 32 * rt + tow_row(r, lane);
      if (rr < B) out[(long long)rr * 512 + 32 * t] = acc[t][r] * inv;
    }
}

// false when the shape is not one this kernel covers (the caller then uses gemm3)
// hdr: the tower's bounds header (TowerPrep::HDR of the same prep)
// the shapes fc4_roll_kernel takes (launch_fc4_roll returns false otherwise)
inline bool fc4_roll_ok(const float* a3, long long lda, int K, int chunk) {
  return !(chunk % 16 || K % 16 || (lda % 4) || ((uintptr_t)a3 % 16));
}
inline bool launch_fc4_roll(const float* a3, long long lda, int B, int K, const char* w4p, int nz, int chunk,
                            float* part, const unsigned* hdr, hipStream_t s, Fc4Commit cm = Fc4Commit{}) {
  if (!fc4_roll_ok(a3, lda, K, chunk)) return false;
  const int cs = chunk / 16;
#ifndef ACMI_FC4_SMALL_CT  // column tiles per wave at batches <= 64
#define ACMI_FC4_SMALL_CT 1
#endif
#ifndef ACMI_FC4_CT1_MAXB  // largest batch with one column tile per wave
#define ACMI_FC4_CT1_MAXB 64
#endif
  if (B <= ACMI_FC4_CT1_MAXB && ACMI_FC4_SMALL_CT == 1) {
    const dim3 grid(nz * ((B + 31) / 32) * 4), blk(256);
    hipLaunchKernelGGL(fc4_roll_kernel<1>, grid, blk, 0, s, a3, lda, B, K, w4p, nz, cs, part, hdr, cm);
  } else {
    const dim3 grid(nz * ((B + 31) / 32) * 2), blk(256);
    hipLaunchKernelGGL(fc4_roll_kernel<2>, grid, blk, 0, s, a3, lda, B, K, w4p, nz, cs, part, hdr, cm);
  }
  return true;
}

}  // namespace acmi
