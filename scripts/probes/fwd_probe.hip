// Tile-shape probe for the rollout-size (M = 512 images) forward convolutions.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize \
//     scripts/probes/fwd_probe.hip -o scripts/probes/fwd_probe
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <algorithm>

#include "gemm_stream.hpp"
#include "wsgemm.hpp"
#include "../../actor-critic_amd/csrc/conv1u8.hpp"

namespace acmi {
void set_error(const char*, ...) {}
}  // namespace acmi
using namespace acmi;

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

__global__ void fill(float* p, long long n, uint32_t seed) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = (float)(mix32((uint32_t)i ^ seed) >> 8) * (1.0f / 16777216.0f) - 0.5f;
}
__global__ void fill8(uint8_t* p, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (long long)gridDim.x * blockDim.x) p[i] = (uint8_t)mix32((uint32_t)i);
}

template <class F>
static float timeit(F f, int reps = 50) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < 5; ++r) f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps * 1e3f;  // us
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 512;
  uint8_t* obs;
  float *a1, *a2, *a3, *w1, *w2, *w3, *b, *part;
  CK(hipMalloc(&obs, (long long)M * 28224));
  CK(hipMalloc(&a1, (long long)M * 12800 * 4));
  CK(hipMalloc(&a2, (long long)M * 5184 * 4));
  CK(hipMalloc(&a3, (long long)M * 1568 * 4));
  CK(hipMalloc(&w1, 256 * 32 * 4));
  CK(hipMalloc(&w2, 512 * 64 * 4));
  CK(hipMalloc(&w3, 576 * 32 * 4));
  CK(hipMalloc(&b, 64 * 4));
  CK(hipMalloc(&part, 8LL * M * 49 * 32 * 4));
  fill8<<<1024, 256>>>(obs, (long long)M * 28224);
  fill<<<1024, 256>>>(a1, (long long)M * 12800, 1);
  fill<<<1024, 256>>>(a2, (long long)M * 5184, 2);
  fill<<<64, 256>>>(w1, 256 * 32, 3);
  fill<<<64, 256>>>(w2, 512 * 64, 4);
  fill<<<64, 256>>>(w3, 576 * 32, 5);
  fill<<<1, 64>>>(b, 64, 6);
  CK(hipDeviceSynchronize());

  using S1 = ConvRows<uint8_t, 84, 84, 4, 8, 8, 4>;
  using S2 = ConvRows<float, 20, 20, 32, 4, 4, 2>;
  using S3 = ConvRows<float, 9, 9, 64, 3, 3, 1>;
  RowsAsK<S1> A1{S1{obs, 28224, M * 400}};
  RowsAsK<S2> A2{S2{a1, 12800, M * 81}};
  RowsAsK<S3> A3{S3{a2, 5184, M * 49}};
  MatI<true> B1{w1, 32, 256, 32}, B2{w2, 64, 512, 64}, B3{w3, 32, 576, 32};
  EpiBiasAct E1{a1, 32, b, 1}, E2{a2, 64, b, 1}, E3{a3, 32, b, 1};
  const double f1 = 2.0 * M * 400 * 256 * 32, f2 = 2.0 * M * 81 * 512 * 64, f3 = 2.0 * M * 49 * 576 * 32;
#define RUN(name, fl, ...)                                            \
  {                                                                   \
    float us = timeit([&] { __VA_ARGS__; });                          \
    printf("%-34s %7.1f us  %6.1f TF\n", name, us, (fl) / us / 1e6); \
  }
  printf("M=%d\n", M);
  {  // correctness of the wave-split kernel against gemm_kernel (same epilogue)
    auto cmp = [&](const char* name, float* out, long long n, auto ref, auto test) {
      float* r;
      CK(hipMalloc(&r, n * 4));
      ref();
      CK(hipMemcpy(r, out, n * 4, hipMemcpyDeviceToDevice));
      CK(hipMemset(out, 0, n * 4));
      test();
      CK(hipDeviceSynchronize());
      std::vector<float> h1(n), h2(n);
      CK(hipMemcpy(h1.data(), r, n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), out, n * 4, hipMemcpyDeviceToHost));
      double md = 0, mx = 0;
      for (long long i = 0; i < n; ++i) {
        md = std::max(md, (double)std::fabs(h1[i] - h2[i]));
        mx = std::max(mx, (double)std::fabs(h1[i]));
      }
      printf("check %-10s max|diff| %.3g (max|ref| %.3g)\n", name, md, mx);
      CK(hipFree(r));
    };
    cmp("conv1", a1, (long long)M * 12800,
        [&] { launch_gemm<128, 32, 32, 1, 1, false, false>(A1, B1, E1, M * 400, 32, 256, 1, 0, 0); },
        [&] { launch_gemm_ws<2, 2, 1, 32>(A1, B1, E1, M * 400, 32, 256, 0); });
    cmp("conv1 u8img", a1, (long long)M * 12800,
        [&] { launch_gemm<128, 32, 32, 1, 1, false, false>(A1, B1, E1, M * 400, 32, 256, 1, 0, 0); },
        [&] { launch_conv1_fwd_u8<32>(S1{obs, 28224, M * 400}, B1, E1, M * 400, 256, 0); });
    cmp("conv2", a2, (long long)M * 5184,
        [&] { launch_gemm<64, 64, 32, 1, 1, false, false>(A2, B2, E2, M * 81, 64, 512, 1, 0, 0); },
        [&] { launch_gemm_ws<1, 4, 2, 16>(A2, B2, E2, M * 81, 64, 512, 0); });
    cmp("conv3", a3, (long long)M * 1568,
        [&] { launch_gemm<128, 32, 32, 1, 1, false, false>(A3, B3, E3, M * 49, 32, 576, 1, 0, 0); },
        [&] { launch_gemm_ws<1, 4, 1, 32>(A3, B3, E3, M * 49, 32, 576, 0); });
  }
  RUN("conv1 256x32x32", f1, (launch_gemm<256, 32, 32, 2, 1, false, false>(A1, B1, E1, M * 400, 32, 256, 1, 0, 0)));
  RUN("conv1 128x32x32", f1, (launch_gemm<128, 32, 32, 1, 1, false, false>(A1, B1, E1, M * 400, 32, 256, 1, 0, 0)));
  RUN("conv1 128x32x32 depth2", f1, (launch_gemm<128, 32, 32, 1, 1, false, false, 2>(A1, B1, E1, M * 400, 32, 256, 1, 0, 0)));
  RUN("conv2 64x64x32 depth2", f2, (launch_gemm<64, 64, 32, 1, 1, false, false, 2>(A2, B2, E2, M * 81, 64, 512, 1, 0, 0)));
  RUN("conv3 128x32x32 depth2", f3, (launch_gemm<128, 32, 32, 1, 1, false, false, 2>(A3, B3, E3, M * 49, 32, 576, 1, 0, 0)));
  RUN("conv1 128x32x32 stream", f1, (launch_gemm_stream<128, 32, 32, 1, 1>(A1, B1, E1, M * 400, 32, 256, 1, 0)));
  RUN("conv1 256x32x32 stream", f1, (launch_gemm_stream<256, 32, 32, 2, 1>(A1, B1, E1, M * 400, 32, 256, 1, 0)));
  RUN("conv2 64x64x32 stream", f2, (launch_gemm_stream<64, 64, 32, 1, 1>(A2, B2, E2, M * 81, 64, 512, 1, 0)));
  RUN("conv2 128x64x32 stream", f2, (launch_gemm_stream<128, 64, 32, 2, 1>(A2, B2, E2, M * 81, 64, 512, 1, 0)));
  RUN("conv3 128x32x32 stream", f3, (launch_gemm_stream<128, 32, 32, 1, 1>(A3, B3, E3, M * 49, 32, 576, 1, 0)));
  RUN("conv2 128x64x32", f2, (launch_gemm<128, 64, 32, 2, 1, false, false>(A2, B2, E2, M * 81, 64, 512, 1, 0, 0)));
  RUN("conv2 64x64x32", f2, (launch_gemm<64, 64, 32, 1, 1, false, false>(A2, B2, E2, M * 81, 64, 512, 1, 0, 0)));
  RUN("conv2 128x32x32", f2, (launch_gemm<128, 32, 32, 1, 1, false, false>(A2, B2, E2, M * 81, 64, 512, 1, 0, 0)));
  RUN("conv2 64x64x16", f2, (launch_gemm<64, 64, 16, 1, 1, false, false>(A2, B2, E2, M * 81, 64, 512, 1, 0, 0)));
  RUN("conv3 128x32x32", f3, (launch_gemm<128, 32, 32, 1, 1, false, false>(A3, B3, E3, M * 49, 32, 576, 1, 0, 0)));
  RUN("conv1 u8 image BK32", f1, (launch_conv1_fwd_u8<32>(S1{obs, 28224, M * 400}, B1, E1, M * 400, 256, 0)));
  RUN("conv1 u8 image BK64", f1, (launch_conv1_fwd_u8<64>(S1{obs, 28224, M * 400}, B1, E1, M * 400, 256, 0)));
  RUN("conv1 u8 image BK16", f1, (launch_conv1_fwd_u8<16>(S1{obs, 28224, M * 400}, B1, E1, M * 400, 256, 0)));
  RUN("conv1 ws 2x2 BK32", f1, (launch_gemm_ws<2, 2, 1, 32>(A1, B1, E1, M * 400, 32, 256, 0)));
  RUN("conv1 ws 1x4 BK32", f1, (launch_gemm_ws<1, 4, 1, 32>(A1, B1, E1, M * 400, 32, 256, 0)));
  RUN("conv1 ws 4x1 BK32", f1, (launch_gemm_ws<4, 1, 1, 32>(A1, B1, E1, M * 400, 32, 256, 0)));
  RUN("conv2 ws 1x4 n64 BK32", f2, (launch_gemm_ws<1, 4, 2, 32>(A2, B2, E2, M * 81, 64, 512, 0)));
  RUN("conv2 ws 1x4 n64 BK16", f2, (launch_gemm_ws<1, 4, 2, 16>(A2, B2, E2, M * 81, 64, 512, 0)));
  RUN("conv2 ws 2x2 n64 BK32", f2, (launch_gemm_ws<2, 2, 2, 32>(A2, B2, E2, M * 81, 64, 512, 0)));
  RUN("conv2 ws 1x4 n32 BK32", f2, (launch_gemm_ws<1, 4, 1, 32>(A2, B2, E2, M * 81, 64, 512, 0)));
  RUN("conv3 ws 1x4 BK32", f3, (launch_gemm_ws<1, 4, 1, 32>(A3, B3, E3, M * 49, 32, 576, 0)));
  RUN("conv3 ws 1x4 BK16", f3, (launch_gemm_ws<1, 4, 1, 16>(A3, B3, E3, M * 49, 32, 576, 0)));
  RUN("conv3 ws 2x2 BK32", f3, (launch_gemm_ws<2, 2, 1, 32>(A3, B3, E3, M * 49, 32, 576, 0)));
  {
    // conv3 split-K into 3 (partials only; the reduce is a separate small kernel)
    EpiPartial P{part, M * 49, 32};
    RUN("conv3 128x32x32 splitK3 (no reduce)", f3,
        (launch_gemm<128, 32, 32, 1, 1, true, false>(A3, B3, P, M * 49, 32, 576, 3, 192, 0)));
    RUN("conv3 128x32x32 splitK6 (no reduce)", f3,
        (launch_gemm<128, 32, 32, 1, 1, true, false>(A3, B3, P, M * 49, 32, 576, 6, 96, 0)));
  }
  {  // one full-batch chain vs two half-batch chains on two streams
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const int H = M / 2;
    auto chain = [&](int n, int off, hipStream_t st) {
      RowsAsK<S1> a1_{S1{obs + (long long)off * 28224, 28224, n * 400}};
      EpiBiasAct e1_{a1 + (long long)off * 12800, 32, b, 1};
      launch_gemm<128, 32, 32, 1, 1, false, false>(a1_, B1, e1_, n * 400, 32, 256, 1, 0, st);
      RowsAsK<S2> a2_{S2{a1 + (long long)off * 12800, 12800, n * 81}};
      EpiBiasAct e2_{a2 + (long long)off * 5184, 64, b, 1};
      launch_gemm<64, 64, 32, 1, 1, false, false>(a2_, B2, e2_, n * 81, 64, 512, 1, 0, st);
      RowsAsK<S3> a3_{S3{a2 + (long long)off * 5184, 5184, n * 49}};
      EpiBiasAct e3_{a3 + (long long)off * 1568, 32, b, 1};
      launch_gemm<128, 32, 32, 1, 1, false, false>(a3_, B3, e3_, n * 49, 32, 576, 1, 0, st);
    };
    hipEvent_t ev0, ev1, j1, j2;
    CK(hipEventCreate(&ev0)); CK(hipEventCreate(&ev1)); CK(hipEventCreate(&j1)); CK(hipEventCreate(&j2));
    for (int pass = 0; pass < 2; ++pass) {
      const int reps = 50;
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(ev0, s1));
      for (int r = 0; r < reps; ++r) {
        if (pass == 0) {
          chain(M, 0, s1);
        } else {
          CK(hipEventRecord(j1, s1));
          CK(hipStreamWaitEvent(s2, j1, 0));
          chain(H, 0, s1);
          chain(M - H, H, s2);
          CK(hipEventRecord(j2, s2));
          CK(hipStreamWaitEvent(s1, j2, 0));
        }
      }
      CK(hipEventRecord(ev1, s1));
      CK(hipEventSynchronize(ev1));
      float ms;
      CK(hipEventElapsedTime(&ms, ev0, ev1));
      printf("conv1-3 chain %s: %.1f us per forward\n", pass ? "2 streams x M/2" : "1 stream x M", ms / reps * 1e3f);
    }
  }
  CK(hipGetLastError());
  return 0;
}
