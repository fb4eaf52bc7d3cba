// Rollout-batch conv forward on bf16x3 with the im2col served from LDS.
//
// gemm3_kernel over RowsAsK<ConvRows> gathers every patch row from L2: each
// input pixel is re-read by every output position whose window covers it
// (conv1 8x8/4: 4x, conv2 4x4/2: 4x, conv3 3x3/1: 9x) and at 512 images the
// launch is a few hundred latency-bound tiles.  Here a block takes IMGS whole
// images: their input activations are copied ONCE into LDS ([img][y][x][C],
// 16-byte chunks XOR-swizzled by pixel for f32 inputs), the K loop streams only
// the weights (three-way split at the commit into gemm3's [part][k][j] image,
// ds_read_b64_tr_b16 fragments), and a lane's A fragment -- 8 consecutive k of
// its output pixel's patch -- is read straight from the image:
//   * f32 inputs (conv2, conv3): 8 channels of one tap = two ds_read_b128,
//     split into h/m/l on the fly (six MFMAs per 32x32x16);
//   * u8 inputs (conv1, C = 4): 2 horizontally adjacent pixels x 4 channels =
//     one ds_read_b64, exact in bf16 (three MFMAs: pixel x w_l, w_m, w_h).
// The block's 32-row x 32-column tiles are dealt to the 4 waves in contiguous
// row-major runs (consecutive tiles share the row block's A fragment).  Same
// epilogue (EpiAct: bias, ReLU, u8 scale, strided rows) as the GEMM paths.
#pragma once

#include "conv1u8.hpp"
#include "gemm3.hpp"

namespace acmi {

template <typename T, int H, int W, int C, int KH, int KW, int S, int COUT, int IMGS, int BKS = 64>
struct ConvFX3 {
  static constexpr bool U8 = sizeof(T) == 1;
  static constexpr int OH = (H - KH) / S + 1, OW = (W - KW) / S + 1, L = OH * OW;
  static constexpr int K = KH * KW * C, NK = K / 16, NS = K / BKS;  // k16 steps, stages
  static constexpr int ROWS = IMGS * L;
  static constexpr int RB = (ROWS + 31) / 32, CB = COUT / 32, NT = RB * CB;
  static constexpr int TW = (NT + 3) / 4;  // tiles per wave (at most)
  static constexpr int PIX = C * (int)sizeof(T);  // bytes per input pixel
  static constexpr int CH = PIX / 16;             // 16-byte chunks per pixel (f32)
  static constexpr int IMG_BYTES = H * W * PIX;
  using IB = X3Image<false, COUT, BKS>;  // weights, BKS k-rows per stage
  static constexpr int LDS_BYTES = IMGS * IMG_BYTES + 2 * IB::BYTES;
  static_assert(K % BKS == 0 && BKS % 16 == 0 && COUT % 32 == 0, "shape");
  static_assert(U8 ? (C == 4 && (KW * C) % 8 == 0) : (C % 8 == 0 && PIX % 16 == 0), "input layout");
  // f32 image: chunk c of pixel p (p = img*H*W + y*W + x) at a position XORed
  // by the pixel's x so the 16 lanes of a ds_read_b128 group (consecutive
  // output columns, i.e. x stepping by S) land on distinct 16-byte slots
  __device__ __forceinline__ static int chunk_pos(int p, int x, int c) {
    return p * PIX + 16 * (c ^ ((x / S) & (CH - 1)));
  }
};

template <class CF>
constexpr int convf_x3_blocks_per_cu() {
  return std::min(8, 160 * 1024 / CF::LDS_BYTES);
}

template <typename T, int H, int W, int C, int KH, int KW, int S, int COUT, int IMGS, int BKS, class Epi>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    convf_x3_blocks_per_cu<ConvFX3<T, H, W, C, KH, KW, S, COUT, IMGS, BKS>>())))
void convf_x3_kernel(const T* x, long long img_stride, int B, const float* w, Epi epi) {
  using CF = ConvFX3<T, H, W, C, KH, KW, S, COUT, IMGS, BKS>;
  using IB = typename CF::IB;
  constexpr int L = CF::L, K = CF::K;
  constexpr int NB = BKS * COUT / 4;        // weight float4 runs per stage
  constexpr int NBT = (NB + 255) / 256;     // per thread
  __shared__ __attribute__((aligned(16))) char lds[CF::LDS_BYTES];
  char* img = lds;
  char* bbuf = lds + IMGS * CF::IMG_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int img0 = blockIdx.x * IMGS;
  const int nimg = min(IMGS, B - img0);

  // weights [K][COUT] f32 row-major: run r -> k-row r / (COUT/4), 4 columns
  // the weight loads of a whole stage (BKS k-rows) are in flight together:
  // at rollout batch each stage's global-load latency is paid once per BKS k
  const MatI<true> opB{w, COUT, K, COUT};
  StF4 rb[NBT];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int q = 0; q < NBT; ++q) {
      const int r = tid + 256 * q;
      const int k = k0 + r / (COUT / 4), j = (r % (COUT / 4)) * 4;
      const bool on = r < NB;
      rb[q] = opB.stage(opB.row(on ? k : K), j, on && k < K);
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NBT; ++q) {
      const int r = tid + 256 * q;
      if (r < NB) IB::write(bbuf + buf * IB::BYTES, r / (COUT / 4), (r % (COUT / 4)) * 4, finish(rb[q]));
    }
  };
  fetch(0);
  // input images (each contiguous, images img_stride elements apart): all of a
  // thread's 16-byte loads are issued before its LDS stores (one latency, not
  // one per load); missing images (batch end) read image img0 and are not used
  {
    constexpr int N16 = CF::IMG_BYTES / 16;
    constexpr int NPT = (IMGS * N16 + 255) / 256;
    float4 v[NPT];
#pragma unroll
    for (int q = 0; q < NPT; ++q) {
      const int g = tid + 256 * q;
      const int i = min(g / N16, IMGS - 1), e = g - (g / N16) * N16;
      const int ii = i < nimg ? i : 0;
      const float4* src = reinterpret_cast<const float4*>(x + (long long)(img0 + ii) * img_stride);
      v[q] = src[g < IMGS * N16 ? e : 0];
    }
#pragma unroll
    for (int q = 0; q < NPT; ++q) {
      const int g = tid + 256 * q;
      if (g >= IMGS * N16) break;
      const int i = g / N16, e = g - i * N16;
      if constexpr (CF::U8) {
        *reinterpret_cast<float4*>(img + i * CF::IMG_BYTES + 16 * e) = v[q];
      } else {
        const int p = e / CF::CH, c = e - p * CF::CH;
        *reinterpret_cast<float4*>(img + CF::chunk_pos(i * H * W + p, p % W, c)) = v[q];
      }
    }
  }
  commit(0);

  // this wave's tiles: a contiguous run of the row-major (row block, col block) list
  const int t_lo = (wave * CF::NT) / 4, t_hi = ((wave + 1) * CF::NT) / 4;
  const int nt = t_hi - t_lo;
  int pix0[CF::TW];  // lane's output pixel: top-left input pixel (image-local index)
  int px0[CF::TW];   // its x
  bool rok[CF::TW];
#pragma unroll
  for (int u = 0; u < CF::TW; ++u) {
    const int t = min(t_lo + u, CF::NT - 1);
    const int i = (t / CF::CB) * 32 + (lane & 31);
    rok[u] = i < nimg * L;
    const int ii = rok[u] ? i : 0;
    const int im = ii / L, p = ii - im * L;
    const int oh = p / CF::OW, ow = p - oh * CF::OW;
    pix0[u] = im * H * W + oh * S * W + ow * S;
    px0[u] = ow * S;
  }
  constexpr int KS = BKS / 16;  // k16 steps per stage
  int boff[KS][CF::CB];
#pragma unroll
  for (int q = 0; q < KS; ++q)
#pragma unroll
    for (int cb = 0; cb < CF::CB; ++cb) boff[q][cb] = IB::frag_off(lane, q, 32 * cb);
  const int kh8 = 8 * (lane >> 5);

  f32x16 acc[CF::TW];
#pragma unroll
  for (int u = 0; u < CF::TW; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
  __syncthreads();

  for (int st = 0; st < CF::NS; ++st) {
    const int cur = st & 1;
    fetch((st + 1) * BKS);
    __builtin_amdgcn_sched_barrier(0);
    const char* Bs = bbuf + cur * IB::BYTES;
#pragma unroll
    for (int q = 0; q < KS; ++q) {
    const int ks = st * KS + q;
    bf16x8 bf[CF::CB][3];
#pragma unroll
    for (int cb = 0; cb < CF::CB; ++cb)
#pragma unroll
      for (int pt = 0; pt < 3; ++pt) bf[cb][pt] = IB::frag(Bs + pt * IB::PART, boff[q][cb]);
    // the lane's 8 k within this K-tile: tap (kh, kw), channels ci .. ci+7
    const int k0 = 16 * ks + kh8;
    int kh, kw, ci;
    if constexpr (CF::U8) {  // 8 k = pixels kw, kw+1 of row kh, 4 channels each
      kh = k0 / (KW * C);
      kw = (k0 - kh * KW * C) / C;
      ci = 0;
    } else {
      const int tap = k0 / C;
      kh = tap / KW;
      kw = tap - kh * KW;
      ci = k0 - tap * C;
    }
    const int doff = kh * W + kw;
#pragma unroll
    for (int u = 0; u < CF::TW; ++u) {
      if (u >= nt) break;
      const int t = t_lo + u, cb = t % CF::CB;
      const int p = pix0[u] + doff;
      // (cb is wave-uniform; a runtime index into bf would put it in scratch)
      if constexpr (CF::U8) {
        const uint2 v = *reinterpret_cast<const uint2*>(img + p * CF::PIX);
        const bf16x8 a = u8x8_to_bf16(v);
#pragma unroll
        for (int c = 0; c < CF::CB; ++c)
          if (c == cb) {
            acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bf[c][2], acc[u], 0, 0, 0);
            acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bf[c][1], acc[u], 0, 0, 0);
            acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bf[c][0], acc[u], 0, 0, 0);
          }
      } else {
        const int xx = px0[u] + kw;
        const float4 x0 = *reinterpret_cast<const float4*>(img + CF::chunk_pos(p, xx, ci / 4));
        const float4 x1 = *reinterpret_cast<const float4*>(img + CF::chunk_pos(p, xx, ci / 4 + 1));
        uint4 h, m, l;
        split3(x0.x, x0.y, h.x, m.x, l.x);
        split3(x0.z, x0.w, h.y, m.y, l.y);
        split3(x1.x, x1.y, h.z, m.z, l.z);
        split3(x1.z, x1.w, h.w, m.w, l.w);
        const bf16x8 a[3] = {__builtin_bit_cast(bf16x8, h), __builtin_bit_cast(bf16x8, m),
                             __builtin_bit_cast(bf16x8, l)};
#pragma unroll
        for (int c = 0; c < CF::CB; ++c)
          if (c == cb) acc[u] = mfma_x3(a, bf[c], acc[u]);
      }
    }
    }  // k16 steps of the stage
    __builtin_amdgcn_sched_barrier(0);
    if (st + 1 < CF::NS) commit(cur ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < CF::TW; ++u) {
    if (u >= nt) break;
    const int t = t_lo + u;
    f32x16 out[1][1];
    out[0][0] = acc[u];
    store_tile<1, 1>(epi, out, img0 * L + (t / CF::CB) * 32, (t % CF::CB) * 32, lane,
                     min(B * L, (img0 + nimg) * L), COUT);
  }
}

template <typename T, int H, int W, int C, int KH, int KW, int S, int COUT, int IMGS, int BKS,
          class Epi>
inline void launch_convf_x3(const T* x, long long img_stride, int B, const float* w, const Epi& e,
                            hipStream_t s) {
  hipLaunchKernelGGL((convf_x3_kernel<T, H, W, C, KH, KW, S, COUT, IMGS, BKS, Epi>),
                     dim3(cdiv(B, IMGS)), dim3(256), 0, s, x, img_stride, B, w, e);
}

}  // namespace acmi
