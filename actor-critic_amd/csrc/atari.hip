// Atari frame preprocessing on the device: the frame half of
// the reference's wrapper chain, batched over envs.
//
//   AtariFrameskipWrapper.step      envs/atari/wrappers.py:54-67   max of the last two raw
//                                                                  RGB frames (np.amax)
//   AtariPreprocessFrameWrapper     envs/atari/wrappers.py:30-33   cv2.cvtColor RGB2GRAY,
//                                                                  cv2.resize INTER_AREA 84x84
//   FrameStackWrapper.step/reset    envs/atari/wrappers.py:224-235 roll, zero on terminal,
//                                                                  insert; reset repeats
//
// cv2 (opencv-python, unpinned in requirements.txt:4) is not in this image; its
// published algorithms are restated (oracle/oracle.py `atari_gray`, `area_tables`,
// `area_resize`):
//   * RGB2GRAY on u8 is fixed point: Y = (4899 R + 9617 G + 1868 B + 8192) >> 14;
//   * INTER_AREA with a non-integer ratio (210x160 -> 84x84: 2.5 and 1.905) is the
//     generic area resampler: per destination coordinate a short run of source
//     coordinates with float weights (the cv2 DecimateAlpha tables, computed in
//     double); a destination pixel is sum_j beta_j * (sum_k S[sy_j][sx_k] * alpha_k)
//     accumulated in float in table order with separate multiply and add, rounded
//     half-to-even and saturated.  The kernel uses __fmul_rn/__fadd_rn so that no
//     product is contracted into an FMA: bit-exact with the restatement.
//
// Four workgroups per env, one per band of 21 output rows: the band's source rows of
// both frames are max-pooled and converted to gray straight from 3-dword loads into
// LDS (55 x 160 B for 210x160); then a thread owns one output column (its resampling
// run in registers, zero-padded to 3 entries) and walks the band's rows.
// Measured (scripts/atari_bench.py, 512 envs): 26.5 us per step = 5.0 TB/s of
// algorithmic bytes (0.62 of 8 TB/s); without the resampling the loads alone take 22 us.  HBM traffic
// per env-step: the raw frames (2 x 100,800 B) + the 4-frame stack word read and
// write (2 x 28,224 B) -- HBM bound.
#include <algorithm>

#include "common.hpp"

namespace acmi {
namespace {

constexpr int kOut = 84;       // output side (wrappers.py:32)
constexpr int kMaxTab = 8;     // table entries per destination coordinate (scale <= 6)
constexpr int kAtariThreads = 256;

struct AreaRun {
  int first, count;
  float alpha[kMaxTab];
};

// cv2 computeResizeAreaTab for one destination coordinate d (scale = 1 / (dsize / ssize))
__host__ __device__ void area_run(int ssize, int d, double scale, AreaRun* r) {
  const double f1 = d * scale, f2 = f1 + scale;
  const double cell = fmin(scale, (double)ssize - f1);
  int s1 = (int)ceil(f1), s2 = (int)floor(f2);
  s2 = min(s2, ssize - 1);
  s1 = min(s1, s2);
  int n = 0;
  r->first = s1;
  if ((double)s1 - f1 > 1e-3) {
    r->first = s1 - 1;
    r->alpha[n++] = (float)(((double)s1 - f1) / cell);
  }
  for (int s = s1; s < s2; ++s) r->alpha[n++] = (float)(1.0 / cell);
  if (f2 - (double)s2 > 1e-3) r->alpha[n++] = (float)(fmin(fmin(f2 - (double)s2, 1.0), cell) / cell);
  r->count = n;
  // zero weights past the run: S * 0 = +0 and x + +0 = x, so a fixed-length loop over
  // the padded run gives the same float sums as cv2's variable-length one
  for (int k = n; k < kMaxTab; ++k) r->alpha[k] = 0.f;
}

// longest run over the destination coordinates (host side, same double arithmetic)
int area_max_run(int ssize) {
  const double scale = 1.0 / ((double)kOut / ssize);
  int m = 0;
  for (int d = 0; d < kOut; ++d) {
    AreaRun r;
    area_run(ssize, d, scale, &r);
    m = std::max(m, r.count);
  }
  return m;
}

__device__ __forceinline__ uint32_t max_u8x4(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 32; k += 8) r |= max((a >> k) & 255u, (b >> k) & 255u) << k;
  return r;
}

__device__ __forceinline__ uint32_t gray_rgb(uint32_t r, uint32_t g, uint32_t b) {
  return (r * 4899u + g * 9617u + b * 1868u + 8192u) >> 14;
}

// 4 pixels from 3 RGB dwords: R0 G0 B0 R1 | G1 B1 R2 G2 | B2 R3 G3 B3
__device__ __forceinline__ uint32_t gray4(uint32_t w0, uint32_t w1, uint32_t w2) {
  const uint32_t y0 = gray_rgb(w0 & 255u, (w0 >> 8) & 255u, (w0 >> 16) & 255u);
  const uint32_t y1 = gray_rgb(w0 >> 24, w1 & 255u, (w1 >> 8) & 255u);
  const uint32_t y2 = gray_rgb((w1 >> 16) & 255u, w1 >> 24, w2 & 255u);
  const uint32_t y3 = gray_rgb((w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24);
  return y0 | (y1 << 8) | (y2 << 16) | (y3 << 24);
}

// mode 0: gray frame out ([84][84] u8 at out + e*out_stride)
// mode 1: stack step   (out word = terminal ? f<<24 : (in>>8) | f<<24)
// mode 2: stack reset  (out word = f * 0x01010101)
// grid (kBands, N): a workgroup makes 84/kBands output rows of env blockIdx.y from the
// source rows they cover (4 bands -> 4x the workgroups in flight of one per env).
constexpr int kBands = 4, kBandRows = kOut / kBands;  // 6/7/12 bands measured no faster
constexpr int kUnroll = 4;  // 4-pixel groups whose loads a thread issues together

// NY / NX: fixed (zero-padded) run lengths of the resampling, 0 = the run's own count
template <int NY, int NX>
__global__ __launch_bounds__(kAtariThreads) void atari_frames_kernel(
    const uint8_t* raw, long long env_stride, long long frame_stride, const uint8_t* nframes,
    int H, int W, double scale_y, double scale_x, int mode, const uint8_t* terminals,
    const uint8_t* stack_in, uint8_t* out, long long out_stride) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  AreaRun* ytab = reinterpret_cast<AreaRun*>(smem);  // this band's rows
  AreaRun* xtab = ytab + kBandRows;
  uint8_t* gray = reinterpret_cast<uint8_t*>(xtab + kOut);
  const int band = blockIdx.x, e = blockIdx.y, tid = threadIdx.x;
  const int dy0 = band * kBandRows;

  if (tid < kBandRows) area_run(H, dy0 + tid, scale_y, &ytab[tid]);
  else if (tid >= 64 && tid < 64 + kOut) area_run(W, tid - 64, scale_x, &xtab[tid - 64]);
  // source rows of the band (the same double arithmetic as area_run)
  int r0, r1;
  {
    AreaRun ra, rb;
    area_run(H, dy0, scale_y, &ra);
    area_run(H, dy0 + kBandRows - 1, scale_y, &rb);
    r0 = ra.first;
    r1 = rb.first + rb.count - 1;
  }

  // max-pooled gray rows r0..r1 straight from global memory, 4 pixels (3 dwords) per
  // group, kUnroll groups' loads in flight per thread
  const uint32_t* f0 = reinterpret_cast<const uint32_t*>(raw + e * env_stride);
  const bool two = frame_stride != 0 && (nframes == nullptr || nframes[e] >= 2);
  const uint32_t* f1 = reinterpret_cast<const uint32_t*>(raw + e * env_stride + (two ? frame_stride : 0));
  const int g0 = r0 * W / 4, ng = (r1 - r0 + 1) * W / 4;
  for (int base = 0; base < ng; base += kAtariThreads * kUnroll) {
    uint32_t a[kUnroll][3], b[kUnroll][3];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int g = base + tid + u * kAtariThreads;
      const int gs = g0 + (g < ng ? g : 0);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        a[u][q] = f0[3 * gs + q];
        b[u][q] = f1[3 * gs + q];
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int g = base + tid + u * kAtariThreads;
      if (g >= ng) break;
      const uint32_t w0 = max_u8x4(a[u][0], b[u][0]), w1 = max_u8x4(a[u][1], b[u][1]),
                     w2 = max_u8x4(a[u][2], b[u][2]);
      reinterpret_cast<uint32_t*>(gray)[g] = gray4(w0, w1, w2);
    }
  }
  __syncthreads();

  const bool term = mode == 1 && terminals != nullptr && terminals[e] != 0;
  uint8_t* dst = out + e * out_stride;
  const uint32_t* sin = mode == 1 ? reinterpret_cast<const uint32_t*>(stack_in + e * out_stride) : nullptr;
  // 3. resampling: a thread owns one destination column dx (its x run in registers,
  //    padded to NX) and walks the band's rows ly = ly0, ly0 + kRowGroups, ...
  constexpr int kRowGroups = kAtariThreads / kOut;
  const int dx = tid % kOut, ly0 = tid / kOut;
  if (ly0 >= kRowGroups) return;
  constexpr int KX = NX ? NX : kMaxTab, KY = NY ? NY : kMaxTab;
  const AreaRun& rx = xtab[dx];
  const int nx = NX ? NX : rx.count;
  int xo[KX];
  float xa[KX];
#pragma unroll
  for (int k = 0; k < KX; ++k) {
    xo[k] = min(rx.first + k, W - 1);  // padded entries (weight 0) stay inside the row
    xa[k] = rx.alpha[k];
  }
  const int nrows = r1 - r0 + 1;
  for (int ly = ly0; ly < kBandRows; ly += kRowGroups) {
    const AreaRun& ry = ytab[ly];
    const int ny = NY ? NY : ry.count;
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < KY; ++j) {
      if (j >= ny) break;
      const uint8_t* row = gray + min(ry.first + j - r0, nrows - 1) * W;
      float buf = 0.f;
#pragma unroll
      for (int k = 0; k < KX; ++k) {
        if (k >= nx) break;
        buf = __fadd_rn(buf, __fmul_rn((float)row[xo[k]], xa[k]));
      }
      sum = __fadd_rn(sum, __fmul_rn(ry.alpha[j], buf));
    }
    const uint32_t y = (uint32_t)min(255, max(0, __float2int_rn(sum)));
    const int p = (dy0 + ly) * kOut + dx;
    if (mode == 0) {
      dst[p] = (uint8_t)y;
    } else {
      uint32_t word;
      if (mode == 2) word = y * 0x01010101u;
      else word = (term ? 0u : (sin[p] >> 8)) | (y << 24);
      reinterpret_cast<uint32_t*>(dst)[p] = word;
    }
  }
}

int atari_launch(const char* what, const uint8_t* raw, int64_t env_stride, int64_t frame_stride,
                 const uint8_t* nframes, int N, int H, int W, int mode, const uint8_t* terminals,
                 const uint8_t* stack_in, uint8_t* out, int64_t out_stride, hipStream_t s) {
  const bool aligned = ((uintptr_t)raw % 4 == 0) && env_stride % 4 == 0 && frame_stride % 4 == 0 &&
                       (mode == 0 || ((uintptr_t)out % 4 == 0 && out_stride % 4 == 0 &&
                                      (mode != 1 || (uintptr_t)stack_in % 4 == 0)));
  // cv2 takes its integer-ratio fast path when both ratios are integers: not restated here
  const bool int_ratio = H % kOut == 0 && W % kOut == 0;
  ACMI_REQUIRE(raw && out && N >= 0 && H >= kOut && W >= kOut && H <= 6 * kOut && W <= 6 * kOut &&
                   W % 4 == 0 && H * W <= 40960 && !int_ratio && aligned &&
                   (mode != 1 || stack_in) && frame_stride >= 0 &&
                   out_stride >= (mode == 0 ? kOut * kOut : 4 * kOut * kOut),
               ACMI_ERR_ARG, "%s: bad arguments", what);
  if (N == 0) return ACMI_OK;
  const double sy = 1.0 / ((double)kOut / H), sx = 1.0 / ((double)kOut / W);
  // a band's source rows: at most kBandRows * scale + 2 of them
  const int band_rows = std::min(H, (int)(kBandRows * sy) + 3);
  const size_t lds = (kBandRows + kOut) * sizeof(AreaRun) + (size_t)band_rows * W;
  // 210x160: runs of at most 3 source rows / columns -> fixed 3x3 products per pixel
  const bool fixed3 = area_max_run(H) <= 3 && area_max_run(W) <= 3;
  auto kern = fixed3 ? atari_frames_kernel<3, 3> : atari_frames_kernel<0, 0>;
  hipLaunchKernelGGL(kern, dim3(kBands, N), dim3(kAtariThreads), lds, s, raw, (long long)env_stride,
                     (long long)frame_stride, nframes, H, W, sy, sx, mode, terminals, stack_in, out,
                     (long long)out_stride);
  ACMI_LAUNCH_CHECK(what);
  return ACMI_OK;
}

}  // namespace
}  // namespace acmi

extern "C" {

int acmi_atari_preprocess(const uint8_t* raw, int64_t env_stride, int64_t frame_stride,
                          const uint8_t* nframes, int N, int H, int W, uint8_t* gray_out,
                          int64_t out_stride, acmi_stream_t stream) {
  return acmi::atari_launch("acmi_atari_preprocess", raw, env_stride, frame_stride, nframes, N, H,
                            W, 0, nullptr, nullptr, gray_out, out_stride, (hipStream_t)stream);
}

int acmi_atari_stack(const uint8_t* raw, int64_t env_stride, int64_t frame_stride,
                     const uint8_t* nframes, int N, int H, int W, const uint8_t* terminals,
                     int reset, const uint8_t* stack_in, uint8_t* stack_out, int64_t stack_stride,
                     acmi_stream_t stream) {
  return acmi::atari_launch("acmi_atari_stack", raw, env_stride, frame_stride, nframes, N, H, W,
                            reset ? 2 : 1, terminals, stack_in, stack_out, stack_stride,
                            (hipStream_t)stream);
}

}  // extern "C"
