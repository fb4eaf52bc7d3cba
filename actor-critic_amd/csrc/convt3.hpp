// Conv input gradient (transposed conv over all stride phases) on f16x2 split
// operands (f16x2.hpp) with the dY im2col served from LDS.
//
// gemm3_kernel runs dX as C[(phase, ci)][super-pixel] = sum_k W(k, i) dY(k, j)
// with B = RowsAsK<ConvTRows>: every column re-gathers its KHP x KWP dY pixels
// from L2 (conv3: 9 taps -> each dY value read 9 times) and every 128-column
// tile re-reads all the weights -- 1.4-2 GB of L2 traffic per launch, gather
// bound at ~5 TB/s.  Here a block takes all NI rows and NJ super-pixel columns:
//   * the dY of the (at most NIMG) images its columns touch is copied ONCE into
//     LDS as f32 ([pixel][COUT], 16-byte chunks XOR-swizzled by pixel so the
//     fragment reads of 16 lanes at different pixels are bank-conflict free),
//     plus one zero pixel for taps that fall outside the image;
//   * the K loop streams only the weights (split into f16 h/l by the scale of
//     max |W| at the commit into gemm3's k-contiguous image layout, ds_read_b128
//     fragments);
//   * the dY image is split into f16 h / l (scale of max |dY|, published by the
//     dY producer's epilogue) once, as it is staged; a lane's B fragment (8
//     consecutive k = 8 channels of one tap of its column) is then two
//     ds_read_b128 of its dY pixel (h chunk, l chunk), no per-read split;
//   * three f16 MFMAs per 32x32x16 (bf16x3 took six: 183 us per launch at
//     M = 10240), accumulators unscaled before the epilogue (EpiConvT through
//     the LDS transpose; it publishes max |dX| in turn).
#pragma once

#include "f16x2.hpp"
#include "gemm3.hpp"

namespace acmi {

// gemm3's k-contiguous LDS image (X3Image<true, BX, BK>) with two f16 parts
template <int BX, int BK>
struct X2ImageKC {
  static constexpr int PART = BX * BK * 2;  // bytes per part
  static constexpr int BYTES = 2 * PART;
  static constexpr int RB = BK * 2;         // bytes per LDS row
  // commit of 4 consecutive k of row x, scaled by s
  __device__ __forceinline__ static void write(char* sm, int k, int x, const float4& f, float s) {
    uint2 h, l;
    split2(f.x, f.y, s, h.x, l.x);
    split2(f.z, f.w, s, h.y, l.y);
    const int off = x * RB + 16 * sw_kc<BK>(k >> 3, x) + 8 * ((k >> 2) & 1);
    *reinterpret_cast<uint2*>(sm + off) = h;
    *reinterpret_cast<uint2*>(sm + PART + off) = l;
  }
  __device__ __forceinline__ static int frag_off(int lane, int ks, int x0) {
    const int x = x0 + (lane & 31);
    return x * RB + 16 * sw_kc<BK>(2 * ks + (lane >> 5), x);
  }
  __device__ __forceinline__ static f16x8 frag(const char* part, int off) {
    return as_f16x8(*reinterpret_cast<const uint4*>(part + off));
  }
};

template <int IH, int IW, int KH, int KW, int S, int CIN, int COUT, int NJ, int NWAVES = 4>
struct ConvTX3 {
  static constexpr int NTHR = 64 * NWAVES;
  static constexpr int PH = IH / S, PW = IW / S, L = PH * PW;
  static constexpr int OH = (IH - KH) / S + 1, OW = (IW - KW) / S + 1, OP = OH * OW;
  static constexpr int KHP = KH / S, KWP = KW / S;
  static constexpr int K = KHP * KWP * COUT;
  static constexpr int NI = S * S * CIN;
  static constexpr int WM = NI / 64, WN = NWAVES / WM;  // waves over rows / columns
  static constexpr int WCOLS = NJ / WN;            // columns per wave
  static constexpr int TN = WCOLS / 32;            // 32-column blocks per wave
  static constexpr int NIMG = (NJ - 1) / L + 2;    // images a block's columns can touch
  static constexpr int CH = COUT / 4;              // 16-byte chunks per dY pixel
  static constexpr int PIXW = 256 / (COUT * 4) > 0 ? 256 / (COUT * 4) : 1;  // pixels per bank window
  static constexpr int ZP = NIMG * OP;             // the zero pixel
  static constexpr int DY_BYTES = (ZP + 1) * COUT * 4;
  using IA = X2ImageKC<NI, 16>;
  static constexpr int LDS_BYTES = DY_BYTES + 2 * IA::BYTES;
  static_assert(NI % 64 == 0 && NWAVES % WM == 0 && NJ % (32 * WN) == 0 && COUT % 16 == 0, "shape");
  static_assert(IH % S == 0 && IW % S == 0 && KH % S == 0 && KW % S == 0, "phases");
  __device__ __forceinline__ static int chunk_pos(int p, int c) {
    return p * (COUT * 4) + 16 * (c ^ ((p / PIXW) & (CH - 1)));
  }
};

// conv3's input-gradient weights pre-split once per parameter version (acmi_conv_prepare):
// the A fragments of v_mfma_f32_32x32x16_f16, [k16 step][row tile][part h, l][lane]
// x 16 B, lane l of (ks, rt): W3[tap][ci = 32 rt + (l & 31)][co .. co + 7] with k0 =
// 16 ks + 8 (l >> 5) = (tap, co), scaled by the power of two of max |W3| (the
// tower's header) -- a k-step's 4 KB then stages as one 16-byte copy per thread
template <int COUT>
struct CT3Prep {
  static constexpr int CIN = 64, KSTEPS = 9 * COUT / 16;
  static constexpr int STEP_BYTES = 2 * 2 * 1024;  // 2 row tiles x 2 parts x 64 lanes x 16 B
  static constexpr long long BYTES = (long long)KSTEPS * STEP_BYTES;
};
// (block b; 256 threads = four fragments (rt, part-pair lanes))
template <int COUT>
__device__ __forceinline__ void convt3_prep_body(const float* w3, char* out, const unsigned* w3max, int b) {
  using P = CT3Prep<COUT>;
  const int g = b * 256 + threadIdx.x;  // (ks, rt, lane)
  if (g >= P::KSTEPS * 2 * 64) return;
  const int lane = g & 63, rt = (g >> 6) & 1, ks = g >> 7;
  const int ci = 32 * rt + (lane & 31), k0 = 16 * ks + 8 * (lane >> 5);
  const int tap = k0 / COUT, co = k0 - tap * COUT;
  const float* p = w3 + ((long long)tap * P::CIN + ci) * COUT + co;
  const float sw = f16x2_scale_of_bits(w3max);
  const float4 x0 = *reinterpret_cast<const float4*>(p), x1 = *reinterpret_cast<const float4*>(p + 4);
  uint4 h, l;
  split2(x0.x, x0.y, sw, h.x, l.x);
  split2(x0.z, x0.w, sw, h.y, l.y);
  split2(x1.x, x1.y, sw, h.z, l.z);
  split2(x1.z, x1.w, sw, h.w, l.w);
  uint4* d = reinterpret_cast<uint4*>(out + (long long)ks * P::STEP_BYTES + rt * 2 * 1024) + lane;
  d[0] = h;
  d[64] = l;
}

template <class CT>
constexpr int convt_x3_blocks_per_cu() {
  return std::min(8, 160 * 1024 / CT::LDS_BYTES);
}

// PA: the weights come pre-split from acmi_conv_prepare (CT3Prep, S = 1 only): a
// k-step's A staging is a 16-byte copy per thread; else they are staged from the
// f32 weights and split at the commit.
template <int IH, int IW, int KH, int KW, int S, int CIN, int COUT, int NJ, int NWAVES, class Epi, bool PA>
__global__ __launch_bounds__(64 * NWAVES) __attribute__((amdgpu_waves_per_eu(
    convt_x3_blocks_per_cu<ConvTX3<IH, IW, KH, KW, S, CIN, COUT, NJ, NWAVES>>() * NWAVES / 4)))
void convt_x3_kernel(const float* w, const char* wprep, const float* dy, int B, Epi epi, const unsigned* wmax,
                     const unsigned* dymax) {
  using CT = ConvTX3<IH, IW, KH, KW, S, CIN, COUT, NJ, NWAVES>;
  using IA = typename CT::IA;
  using W = ConvTWeights<KH, KW, S, CIN, COUT>;
  constexpr int NI = CT::NI, K = CT::K, L = CT::L, NTHR = CT::NTHR;
  constexpr int NA = NI * 16 / 4 / NTHR;  // weight float4 runs per thread per K-tile
  static_assert(NA >= 1 && NI * 16 / 4 == NA * NTHR, "weight staging map");
  static_assert(!PA || (S == 1 && NI == 64 && NTHR == 256 && IA::BYTES == CT3Prep<COUT>::STEP_BYTES),
                "prepared weights: conv3's shape");
  __shared__ __attribute__((aligned(16))) char lds[CT::LDS_BYTES];
  char* dimg = lds;
  char* abuf = lds + CT::DY_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / CT::WN, wn = wave - wm * CT::WN;
  const float sw = f16x2_scale_of_bits(wmax), sd = f16x2_scale_of_bits(dymax);
  const float inv = 1.f / (sw * sd);
  const int J = B * L;
  const int j0 = blockIdx.x * NJ;
  const int img_lo = j0 / L;
  const int img_hi = min(B - 1, (j0 + NJ - 1) / L);

  // weights: prepared fragments (one 16-byte copy per thread and k-step), or
  // gemm3's k-contiguous staging (one ConvTWeights run per thread)
  const W opA{w};
  typename W::R rowA[NA];
  if constexpr (!PA) {
#pragma unroll
    for (int v = 0; v < NA; ++v) rowA[v] = opA.row((tid + NTHR * v) / 4);
  }
  StF4 ra[NA];
  uint4 rp;
  auto fetch = [&](int ks) {
    if constexpr (PA) {
      rp = reinterpret_cast<const uint4*>(wprep + (long long)min(ks, K / 16 - 1) * IA::BYTES)[tid];
    } else {
      const int k = 16 * ks + (tid % 4) * 4;
      const auto c = opA.col(k);
#pragma unroll
      for (int v = 0; v < NA; ++v) ra[v] = opA.stage(rowA[v], c, k < K);
    }
  };
  auto commit = [&](int buf) {
    char* As = abuf + buf * IA::BYTES;
    if constexpr (PA) {
      reinterpret_cast<uint4*>(As)[tid] = rp;
    } else {
#pragma unroll
      for (int v = 0; v < NA; ++v) {
        const int idx = tid + NTHR * v;
        const int i = idx / 4;
        IA::write(As, (idx - i * 4) * 4, i, finish(ra[v]), sw);
      }
    }
  };

  fetch(0);
  // dY of images img_lo..img_hi (contiguous [img][OH][OW][COUT]) + the zero pixel,
  // split ONCE into its f16 h / l parts (scale of max |dY|) as it is staged: a
  // pixel's 16-byte chunks c < CH/2 hold h of channels 8c .. 8c+7, chunks CH/2 + c
  // their l -- every B fragment is then two plain reads (each dY value feeds up to
  // KHP x KWP taps: split per read it cost 12 VALU per fragment)
  {
    // all of a thread's loads issued before its stores (one latency, not one per load)
    const int n4 = (img_hi - img_lo + 1) * CT::OP * CT::CH;
    const float4* src = reinterpret_cast<const float4*>(dy + (long long)img_lo * CT::OP * COUT);
    constexpr int NPT = (CT::NIMG * CT::OP * CT::CH + NTHR - 1) / NTHR;
    float4 v[NPT];
#pragma unroll
    for (int q = 0; q < NPT; ++q) {
      const int e = tid + NTHR * q;
      v[q] = src[e < n4 ? e : 0];
    }
#pragma unroll
    for (int q = 0; q < NPT; ++q) {
      const int e = tid + NTHR * q;
      if (e >= n4) break;
      const int p = e / CT::CH, c = e - p * CT::CH;  // f32 chunk c: channels 4c .. 4c+3
      uint2 h, l;
      split2(v[q].x, v[q].y, sd, h.x, l.x);
      split2(v[q].z, v[q].w, sd, h.y, l.y);
      *reinterpret_cast<uint2*>(dimg + CT::chunk_pos(p, c >> 1) + 8 * (c & 1)) = h;
      *reinterpret_cast<uint2*>(dimg + CT::chunk_pos(p, CT::CH / 2 + (c >> 1)) + 8 * (c & 1)) = l;
    }
    for (int c = tid; c < CT::CH; c += NTHR)
      *reinterpret_cast<float4*>(dimg + CT::ZP * COUT * 4 + 16 * c) = f4zero();
  }
  commit(0);

  // per column block: the lane's super-pixel (image relative to img_lo, ih', iw')
  int cimg[CT::TN], cih[CT::TN], ciw[CT::TN];
  bool cok[CT::TN];
#pragma unroll
  for (int t = 0; t < CT::TN; ++t) {
    const int j = j0 + wn * CT::WCOLS + 32 * t + (lane & 31);
    cok[t] = j < J;
    const int jj = cok[t] ? j : j0;
    const int img = jj / L, p = jj - img * L;
    cimg[t] = img - img_lo;
    cih[t] = p / CT::PW;
    ciw[t] = p - cih[t] * CT::PW;
  }
  const int hl = lane >> 5;
  int aoff[2];
#pragma unroll
  for (int tm = 0; tm < 2; ++tm)
    aoff[tm] = PA ? ((2 * (2 * wm + tm)) * 64 + lane) * 16 : IA::frag_off(lane, 0, wm * 64 + 32 * tm);
  const int apart = PA ? 64 * 16 : IA::PART;  // bytes from a fragment's h part to its l part

  f32x16 acc[2][CT::TN];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < CT::TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  __syncthreads();

  // taps outer (the lane's dY pixel and its chunk swizzle computed once per tap),
  // the tap's COUT/16 k-steps inner; k-step ks = tap * NCS + cs
  constexpr int NCS = COUT / 16, NTAP = CT::KHP * CT::KWP;
  static_assert(NCS % 2 == 0, "k-steps per tap even: the LDS buffer is cs's parity");
  for (int tap = 0; tap < NTAP; ++tap) {
    const int khp = tap / CT::KWP, kwp = tap - khp * CT::KWP;
    int pb[CT::TN], psw[CT::TN];
#pragma unroll
    for (int tn = 0; tn < CT::TN; ++tn) {
      const int oh = cih[tn] - khp, ow = ciw[tn] - kwp;
      const bool ok = cok[tn] & (oh >= 0) & (ow >= 0) & (oh < CT::OH) & (ow < CT::OW);
      const int p = ok ? cimg[tn] * CT::OP + oh * CT::OW + ow : CT::ZP;
      pb[tn] = p * (COUT * 4);
      psw[tn] = (p / CT::PIXW) & (CT::CH - 1);
    }
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) {
      const int ks = tap * NCS + cs;
      const int cur = cs & 1;
      fetch(ks + 1);
      __builtin_amdgcn_sched_barrier(0);
      const char* As = abuf + cur * IA::BYTES;
      f16x8 a[2][2];
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int tm = 0; tm < 2; ++tm) a[tm][pt] = IA::frag(As + pt * apart, aoff[tm]);
      // this lane's 8 k: channels co .. co+7, co = 16 cs + 8 hl: h chunk co / 8
      const int ch = 2 * cs + hl;
#pragma unroll
      for (int tn = 0; tn < CT::TN; ++tn) {
        f16x8 b[2];
        b[0] = as_f16x8(*reinterpret_cast<const uint4*>(dimg + pb[tn] + 16 * (ch ^ psw[tn])));
        b[1] = as_f16x8(*reinterpret_cast<const uint4*>(dimg + pb[tn] + 16 * ((CT::CH / 2 + ch) ^ psw[tn])));
#pragma unroll
        for (int tm = 0; tm < 2; ++tm) acc[tm][tn] = mfma_x2(a[tm], b, acc[tm][tn]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < K / 16) commit(cur ^ 1);
      __syncthreads();
    }
  }
  // epilogue through the LDS transpose (the dY image is free now)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < CT::TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] *= inv;  // unscale (exact: powers of two)
  store_tile_lds<2, CT::TN>(epi, acc, wm * 64, j0 + wn * CT::WCOLS, lane,
                            reinterpret_cast<float*>(lds) + wave * 32 * 36, NI, J);
}

template <int IH, int IW, int KH, int KW, int S, int CIN, int COUT, int NJ, int NWAVES = 4,
          class Epi>
inline void launch_convt_x3(const float* w, const char* wprep, const float* dy, int B, const Epi& e,
                            const unsigned* wmax, const unsigned* dymax, hipStream_t s) {
  using CT = ConvTX3<IH, IW, KH, KW, S, CIN, COUT, NJ, NWAVES>;
  static_assert(CT::DY_BYTES >= NWAVES * 32 * 36 * 4, "epilogue transpose needs the dY region");
  if (wprep)
    hipLaunchKernelGGL((convt_x3_kernel<IH, IW, KH, KW, S, CIN, COUT, NJ, NWAVES, Epi, true>),
                       dim3(cdiv(B * CT::L, NJ)), dim3(CT::NTHR), 0, s, w, wprep, dy, B, e, wmax, dymax);
  else
    hipLaunchKernelGGL((convt_x3_kernel<IH, IW, KH, KW, S, CIN, COUT, NJ, NWAVES, Epi, false>),
                       dim3(cdiv(B * CT::L, NJ)), dim3(CT::NTHR), 0, s, w, wprep, dy, B, e, wmax, dymax);
}

}  // namespace acmi
