// conv2's input gradient (d1 = conv2^T d2 * relu'(a1)) on f16x2 split operands
// (f16x2.hpp) with the weights split ONCE per parameter version, and the
// sampled-loss variant that reduces d1 to the K-FAC G factor of conv1's output
// without storing it.
//
// gemm3_kernel / convt_x3_kernel run this product with every block splitting
// the 128 x 256 weight matrix into h/m/l again (8000 blocks at the bench shape)
// and two row tiles per wave: ~10 VALU instructions per MFMA, more issue time
// than the matrix cores need (rocprofv3: SQ_INSTS_VALU 1.24e8 against 12.3 M
// MFMAs, 43 % MFMA-busy at 424 us).  Here
//   * the weights come pre-split from acmi_conv_prepare ([k16 step][phase]
//     [part h,l][lane] x 16 B, the A fragments of v_mfma_f32_32x32x16_f16, scaled
//     by the power of two of max |W2|), staged per k-step into LDS by a straight
//     16-byte copy (8 KB, read back lane-contiguous: conflict-free ds_read_b128);
//   * a wave owns 32 super-pixel columns and ALL FOUR stride phases (rows
//     (phase, ci)): the four phases of a super-pixel gather the same dY pixels
//     (tap (a, b) of phase (py, px) is kernel position (py + 2a, px + 2b)), so
//     one B fragment -- 8 channels of one dY pixel, two float4 loads from L2,
//     one split by the scale of max |d2| (published by the conv3 dX epilogue) --
//     feeds 4 x 3 MFMAs; the accumulators are unscaled before the epilogue;
//   * epilogue STORE: the ReLU'-masked d1 as float4 channel runs; epilogue
//     GRAM: the masked tile goes through LDS ([ci][super-pixel], stride 36:
//     conflict-free) and its Gram D D^T accumulates on bf16x3 MFMAs (d1 has no
//     bound yet) across the wave's tiles; blocks write part[block][33][32] for
//     finalize_cov_kernel (the layout gcov_layer's partials use).
// k runs in gemm3's order (tap-major, channel-minor); d1 is f32-accurate.
// (Measured on bf16x3, six MFMAs per product: 392 / 411 us per launch at
// M = 10240.)
// Reference: tf.gradients of the conv2d at envs/atari/model.py:184-189
// (objectives.py:78) and kfac's G factor of conv1's output (registration
// envs/atari/model.py:227-231) -- the same sums.
#pragma once

#include "f16x2.hpp"
#include "gemm.hpp"

namespace acmi {

// conv2 geometry: a1 [20][20][32] -> d2 [9][9][64], 4x4 stride 2
struct CT2 {
  static constexpr int CIN = 32, COUT = 64, OH = 9, OW = 9, PW = 10, L = 100;
  static constexpr int NKS = 16;                    // k16 steps: 4 taps x 64 channels
  static constexpr int STEP_BYTES = 4 * 2 * 1024;   // 4 phases x 2 parts x 64 lanes x 16 B
  static constexpr int FRAG_BYTES = NKS * STEP_BYTES;  // 131,072 B of prepared weights
  static constexpr int BYTES = FRAG_BYTES + 4 * kAmaxWords;  // + max |W2| (published, common.hpp)
  static constexpr int TILE = 128;                  // columns per block tile (4 waves x 32)
};

// max |W2| into the prepared block's scale word (zeroed by the caller)
// (block b of nb; 256 threads)
__device__ __forceinline__ void convt2_wmax_body(const float* w2, char* out, int b, int nb) {
  float m = 0.f;
  for (int i = b * 256 + threadIdx.x; i < 16 * CT2::CIN * CT2::COUT; i += nb * 256)
    m = fmaxf(m, fabsf(w2[i]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) amax_update(reinterpret_cast<unsigned*>(out + CT2::FRAG_BYTES), m);
}

// prepared weights: fragment (ks, phase) lane l holds W[py+2a][px+2b][ci][co..co+7],
// ci = l & 31, tap t = ks >> 2 = (a, b), co = 16 (ks & 3) + 8 (l >> 5)
// (block b; 256 threads)
__device__ __forceinline__ void convt2_prep_body(const float* w2, char* out, int blk) {
  const int g = blk * 256 + threadIdx.x;  // (ks, phase, lane)
  if (g >= CT2::NKS * 4 * 64) return;
  const int lane = g & 63, ph = (g >> 6) & 3, ks = g >> 8;
  const int py = ph >> 1, px = ph & 1, t = ks >> 2, a = t >> 1, b = t & 1;
  const int kh = py + 2 * a, kw = px + 2 * b;
  const int ci = lane & 31, co = 16 * (ks & 3) + 8 * (lane >> 5);
  const float* p = w2 + ((kh * 4 + kw) * CT2::CIN + ci) * CT2::COUT + co;
  const float sw = f16x2_scale_of_bits(reinterpret_cast<const unsigned*>(out + CT2::FRAG_BYTES));
  uint4 h, l;
  split2(p[0], p[1], sw, h.x, l.x);
  split2(p[2], p[3], sw, h.y, l.y);
  split2(p[4], p[5], sw, h.z, l.z);
  split2(p[6], p[7], sw, h.w, l.w);
  uint4* d = reinterpret_cast<uint4*>(out + (long long)ks * CT2::STEP_BYTES + ph * 2 * 1024) + lane;
  d[0] = h;
  d[64] = l;
}

// MASK: a1 is the ReLU' bit words (acmi_acts_t m1) instead of the f32 activation.
// MIX ("stacked"): the loss chain's and the sampled-loss chain's products as one
// launch over both chains' tiles -- tiles [0, T) are the loss chain's (d2 scaled
// by d2max, the STORE epilogue into d1), tiles [T, 2T) the sampled chain's (d2b
// by d2bmax, the GRAM epilogue): one W2^T stream and one accumulator set per
// wave, the epilogue chosen per tile; grid-stride over convt2_gram_blocks blocks.
template <bool GRAM, bool MASK = false, bool MIX = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
void convt2_kernel(const char* prep, const float* __restrict__ d2, const float* __restrict__ a1,
                   float* __restrict__ d1, int B, float* __restrict__ gpart, const unsigned* d2max,
                   unsigned* d1max, const float* __restrict__ d2b = nullptr, const unsigned* d2bmax = nullptr) {
  // 16 KB ring; the epilogue's transpose scratch (4 x 32 x 36 floats) reuses it
  __shared__ __attribute__((aligned(16))) char lds[std::max(2 * CT2::STEP_BYTES, 4 * 32 * 36 * 4)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int J = B * CT2::L;
  const int ctiles = (J + CT2::TILE - 1) / CT2::TILE;  // tiles of one chain
  // MIX: the sampled chain's tiles start at a multiple of the grid, so block b
  // takes the same Gram tiles in the same order as the Gram launch (bit-identical
  // partials); the slots [ctiles, gbase) are empty and skipped
  const int G = gridDim.x;
  const int gbase = MIX ? (ctiles + G - 1) / G * G : ctiles;
  const int ntiles = MIX ? gbase + ctiles : ctiles;
  auto valid_from = [&](int t) { return MIX && t >= ctiles && t < gbase ? t + G : t; };  // (gap < G)
  const int hl = lane >> 5;  // k half of the fragment; row offset 4 of the accumulator
  const float* zero = zero_run();
  const float sd_a = f16x2_scale_of_bits(d2max);
  const float sw = f16x2_scale_of_bits(reinterpret_cast<const unsigned*>(prep + CT2::FRAG_BYTES));
  const float inv_a = 1.f / (sw * sd_a);
  float sd_b = sd_a, inv_b = inv_a;
  if constexpr (MIX) {
    sd_b = f16x2_scale_of_bits(d2bmax);
    inv_b = 1.f / (sw * sd_b);
  }
  // a tile of the sampled chain (GRAM epilogue), its index within its chain
  auto gram_tile = [&](int tile) { return MIX ? tile >= gbase : GRAM; };
  auto local_tile = [&](int tile) { return MIX && tile >= gbase ? tile - gbase : tile; };

  float d1am = 0.f;  // !GRAM: max |d1| over the lane's stores, published once at the end
  f32x16 gacc;  // GRAM: this wave's D D^T over its tiles
#pragma unroll
  for (int r = 0; r < 16; ++r) gacc[r] = 0.f;

  // super-pixel column of this lane in a tile, and its dY image
  struct Col {
    bool ok;
    int n, Y, X;
    const float* dimg;
  };
  auto col_of = [&](int tile) {
    Col c;
    const int j = local_tile(tile) * CT2::TILE + 32 * wave + (lane & 31);
    c.ok = j < J;
    const int jj = c.ok ? j : 0;
    c.n = jj / CT2::L;
    const int sp = jj - c.n * CT2::L;
    c.Y = sp / CT2::PW;
    c.X = sp - c.Y * CT2::PW;
    c.dimg = (MIX && gram_tile(tile) ? d2b : d2) + (long long)c.n * (CT2::OH * CT2::OW * CT2::COUT);
    return c;
  };
  // lane's B fragment for k-step ks: dY pixel (Y - a, X - b), channels co..co+7.
  // Out-of-image taps load the zero run, selected on the ADDRESS (no branch:
  // a load under a branch makes the waitcnt pass drain vmcnt at the join)
  auto bload = [&](int ks, const Col& c, float4 (&x)[2]) {
    const int t = ks >> 2, a = t >> 1, b = t & 1;
    const int oy = c.Y - a, ox = c.X - b;
    const bool ok = c.ok & (oy >= 0) & (oy < CT2::OH) & (ox >= 0) & (ox < CT2::OW);
    const int oyc = max(oy, 0), oxc = max(ox, 0);  // (in range whenever ok)
    const float* p = c.dimg + (oyc * CT2::OW + oxc) * CT2::COUT + 16 * (ks & 3) + 8 * hl;
    x[0] = *reinterpret_cast<const float4*>(ok ? p : zero);
    x[1] = *reinterpret_cast<const float4*>(ok ? p + 4 : zero);
  };
  // A staging: 8 KB per k-step, two 16-byte runs per thread (named
  // registers: an array captured by the lambdas below was put in scratch)
  uint4 ra0, ra1;
  auto afetch = [&](int ks) {
    const uint4* src = reinterpret_cast<const uint4*>(prep + (long long)ks * CT2::STEP_BYTES) + tid;
    ra0 = src[0];
    ra1 = src[256];
  };
  auto acommit = [&](int buf) {
    uint4* dst = reinterpret_cast<uint4*>(lds + buf * CT2::STEP_BYTES) + tid;
    dst[0] = ra0;
    dst[256] = ra1;
  };
  // two B register sets, alternating by k-step parity (named, never indexed at
  // run time: a dynamically indexed register array lands in scratch)
  float4 bx0[2], bx1[2];
  const int first = valid_from(blockIdx.x);
  Col cur = col_of(min(first, ntiles - 1));
  afetch(0);
  bload(0, cur, bx0);

  for (int tile = first; tile < ntiles; tile = valid_from(tile + G)) {
    // step 0's operands were loaded before the loop or during the previous
    // tile's last k-step (its A is the same for every tile)
    const Col nextc = col_of(min(valid_from(tile + G), ntiles - 1));
    const bool jok = cur.ok;
    const int n = cur.n, Y = cur.Y, X = cur.X;
    const bool gt = gram_tile(tile);
    const float sd = MIX && gt ? sd_b : sd_a, inv = MIX && gt ? inv_b : inv_a;
    acommit(0);
    __syncthreads();

    f32x16 acc[4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[p][r] = 0.f;

    auto step = [&](int ks, float4 (&cb)[2], float4 (&nb)[2]) {
      const int buf = ks & 1;
      // the last k-step loads step 0 of the next tile (selected, not branched:
      // no load under a run-time branch, whose join would drain vmcnt)
      const bool last = ks + 1 == CT2::NKS;
      afetch(last ? 0 : ks + 1);
      Col c;
      c.ok = last ? nextc.ok : cur.ok;
      c.Y = last ? nextc.Y : cur.Y;
      c.X = last ? nextc.X : cur.X;
      c.dimg = last ? nextc.dimg : cur.dimg;
      bload(last ? 0 : ks + 1, c, nb);
      __builtin_amdgcn_sched_barrier(0);
      f16x8 b[2];
      split2x8(cb[0], cb[1], sd, b[0], b[1]);
      const char* As = lds + buf * CT2::STEP_BYTES + lane * 16;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        f16x8 a[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) a[q] = as_f16x8(*reinterpret_cast<const uint4*>(As + (p * 2 + q) * 1024));
        acc[p] = mfma_x2(a, b, acc[p]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (!last) acommit(buf ^ 1);  // (step 0's A is committed after the epilogue)
      __syncthreads();
    };
    // two steps per iteration, not unrolled further (a full unroll keeps every
    // step's addresses live and spills)
    for (int ks = 0; ks < CT2::NKS; ks += 2) {
      step(ks, bx0, bx1);
      step(ks + 1, bx1, bx0);
    }
    cur = nextc;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[p][r] *= inv;  // unscale (exact: powers of two)

    // epilogue: rows (phase p, ci) x this wave's 32 super-pixel columns
    float* scr = reinterpret_cast<float*>(lds) + wave * 32 * 36;  // [32][36] per wave
    if (!gt) {
      // ReLU'-masked d1 through the LDS transpose (each store instruction writes 8
      // whole 128-byte pixel rows): after it, lane (ri = 4 (lane & 7), cj = lane >> 3)
      // holds channels ri .. ri+3 of super-pixel columns cj + 8 q (q < 4) of each
      // phase.  Its four super-pixels are decoded once per tile (not per phase and
      // element, as EpiConvT's generic offset() does), a phase adds (py, px) to the
      // pixel, and the ReLU' bits come from one mask word per pixel.
      const int ri = 4 * (lane & 7), cj = lane >> 3;
      int pix[4];
      bool jok[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = local_tile(tile) * CT2::TILE + 32 * wave + cj + 8 * q;
        jok[q] = j < J;
        const int jj = jok[q] ? j : 0;
        const int nn = jj / CT2::L, sp = jj - nn * CT2::L;
        const int yy = sp / CT2::PW, xx = sp - yy * CT2::PW;
        pix[q] = (nn * 20 + 2 * yy) * 20 + 2 * xx;
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(scr + (lane & 31) * 36 + 8 * g + 4 * hl) =
              make_float4(acc[p][4 * g], acc[p][4 * g + 1], acc[p][4 * g + 2], acc[p][4 * g + 3]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int dp = (p >> 1) * 20 + (p & 1);
        float4 v[4];
        uint32_t bits[4];
        float4 xa[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = *reinterpret_cast<const float4*>(scr + (cj + 8 * q) * 36 + ri);
          const int px = pix[q] + dp;
          if constexpr (MASK) bits[q] = reinterpret_cast<const uint32_t*>(jok[q] ? a1 + px : zero)[0] >> ri;
          else xa[q] = *reinterpret_cast<const float4*>(jok[q] ? a1 + px * CT2::CIN + ri : zero);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 o;
          if constexpr (MASK) {
            o.x = (bits[q] & 1u) ? v[q].x : 0.f;
            o.y = (bits[q] & 2u) ? v[q].y : 0.f;
            o.z = (bits[q] & 4u) ? v[q].z : 0.f;
            o.w = (bits[q] & 8u) ? v[q].w : 0.f;
          } else {
            o.x = xa[q].x > 0.f ? v[q].x : 0.f;
            o.y = xa[q].y > 0.f ? v[q].y : 0.f;
            o.z = xa[q].z > 0.f ? v[q].z : 0.f;
            o.w = xa[q].w > 0.f ? v[q].w : 0.f;
          }
          if (jok[q]) {
            *reinterpret_cast<float4*>(d1 + (long long)(pix[q] + dp) * CT2::CIN + ri) = o;
            d1am = absmax4(d1am, o);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    } else {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int py = p >> 1, px = p & 1;
        const long long pix = ((long long)n * 20 + 2 * Y + py) * 20 + 2 * X + px;
        // masked tile as [ci][super-pixel] (rows ci = (r & 3) + 8 (r >> 2) + 4 hl)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ci = 8 * g + 4 * hl;
          float4 x;
          if constexpr (MASK) {  // ReLU' bits: word pix, channels ci .. ci + 3 (zero run past the end)
            const uint32_t b = *reinterpret_cast<const uint32_t*>(jok ? a1 + pix : zero) >> ci;
            x = make_float4((float)(b & 1u), (float)((b >> 1) & 1u), (float)((b >> 2) & 1u), (float)((b >> 3) & 1u));
          } else {
            x = *reinterpret_cast<const float4*>(jok ? a1 + pix * CT2::CIN + ci : zero);
          }
          const int c = lane & 31;
          scr[(ci + 0) * 36 + c] = x.x > 0.f ? acc[p][4 * g + 0] : 0.f;
          scr[(ci + 1) * 36 + c] = x.y > 0.f ? acc[p][4 * g + 1] : 0.f;
          scr[(ci + 2) * 36 + c] = x.z > 0.f ? acc[p][4 * g + 2] : 0.f;
          scr[(ci + 3) * 36 + c] = x.w > 0.f ? acc[p][4 * g + 3] : 0.f;
        }
        // G += D D^T, k = the 32 super-pixels (two k16 steps); the lane's fragment
        // D[ci = lane & 31][k = 16 h + 8 hl .. +7] serves as A and as B.  (LDS ops
        // of one wave execute in issue order: the reads see all lanes' stores.)
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float* rp = scr + (lane & 31) * 36 + 16 * h + 8 * hl;
          const float4 x0 = *reinterpret_cast<const float4*>(rp);
          const float4 x1 = *reinterpret_cast<const float4*>(rp + 4);
          uint4 hh, mm, ll;
          split3(x0.x, x0.y, hh.x, mm.x, ll.x);
          split3(x0.z, x0.w, hh.y, mm.y, ll.y);
          split3(x1.x, x1.y, hh.z, mm.z, ll.z);
          split3(x1.z, x1.w, hh.w, mm.w, ll.w);
          const bf16x8 f[3] = {__builtin_bit_cast(bf16x8, hh), __builtin_bit_cast(bf16x8, mm),
                               __builtin_bit_cast(bf16x8, ll)};
          gacc = mfma_x3(f, f, gacc);
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();  // the ring / scratch is reused by the next tile
  }

  if constexpr (MIX || !GRAM) amax_publish(d1max, d1am, lane);
  if constexpr (MIX || GRAM) {
    // the 4 waves' Grams summed in wave order through LDS, then part[block][33][32]
    float* red = reinterpret_cast<float*>(lds);  // [32][32]
    for (int w = 0; w < 4; ++w) {
      if (wave == w) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int i = (r & 3) + 8 * (r >> 2) + 4 * hl, jc = lane & 31;
          red[i * 32 + jc] = (w ? red[i * 32 + jc] : 0.f) + gacc[r];
        }
      }
      __syncthreads();
    }
    float* out = gpart + (long long)blockIdx.x * 33 * 32;
    for (int e = tid; e < 32 * 32; e += 256) out[e] = red[e];
  }
}

#ifndef ACMI_CT2_STORE_BLOCKS  // 0: one block per tile; else at most this many blocks (grid-stride)
#define ACMI_CT2_STORE_BLOCKS 0
#endif
inline int convt2_store_blocks(int B) {
  const int ntiles = (B * CT2::L + CT2::TILE - 1) / CT2::TILE;
  return ACMI_CT2_STORE_BLOCKS > 0 ? std::max(1, std::min(ntiles, ACMI_CT2_STORE_BLOCKS)) : ntiles;
}
// blocks of the Gram variant (per-block partials, finalize_cov_kernel sums them)
inline int convt2_gram_blocks(int B) {
  const int ntiles = (B * CT2::L + CT2::TILE - 1) / CT2::TILE;
  return std::max(1, std::min(ntiles, 768));
}

}  // namespace acmi
