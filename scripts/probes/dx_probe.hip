// Timing probe for the conv2 input-gradient GEMM (all stride phases as
// columns) and what its epilogue costs.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize \
//     scripts/probes/dx_probe.hip -o scripts/probes/dx_probe && ./scripts/probes/dx_probe
#include <cstdio>
#include <cstdlib>

#include "../../actor-critic_amd/csrc/gemm.hpp"

namespace acmi {

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

template <class F>
static float timeit(F f, int reps = 10) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

// same scatter as EpiConvT without the ReLU' read
template <int IH, int IW, int S, int CIN>
struct EpiNoMask {
  static constexpr bool VEC4 = true;
  EpiConvT<IH, IW, S, CIN> e;
  __device__ __forceinline__ float4 aux4(int, int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ void store4(int i0, int j, float4 v, float4) const {
    *reinterpret_cast<float4*>(e.out + e.offset(i0, j)) = v;
  }
};
// GEMM + gather only (a store that never happens but cannot be proven dead)
struct EpiNone {
  float* out;
  float never;
  __device__ __forceinline__ float aux(int, int) const { return 0.f; }
  __device__ __forceinline__ void store(int i, int j, float v, float) const {
    if (v == never) out[(long long)i * 128 + j] = v;
  }
};

}  // namespace acmi

using namespace acmi;

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 10240;
  using Src = ConvTRows<20, 20, 4, 4, 2, 64>;
  using W = ConvTWeights<4, 4, 2, 32, 64>;
  float *a1, *dy, *w2, *d1;
  const long long a1n = (long long)M * 400 * 32, dyn = (long long)M * 81 * 64;
  CK(hipMalloc(&a1, a1n * 4));
  CK(hipMalloc(&d1, a1n * 4));
  CK(hipMalloc(&dy, dyn * 4));
  CK(hipMalloc(&w2, 4 * 4 * 32 * 64 * 4));
  fill<<<4096, 256>>>(a1, a1n, 1);
  fill<<<4096, 256>>>(dy, dyn, 2);
  fill<<<64, 256>>>(w2, 4 * 4 * 32 * 64, 9);
  W opA{w2};
  RowsAsK<Src> opB{Src{dy, M * Src::L}};
  const int I = W::N, J = M * Src::L;
  const double fl = 2.0 * I * J * Src::COLS;
  EpiConvT<20, 20, 2, 32> em{d1, a1};
  EpiNoMask<20, 20, 2, 32> en{em};
  EpiNone e0{d1, 12345.f};
#define RUN(NAME, EPI, ...)                                                                  \
  {                                                                                         \
    float ms = timeit([&] { launch_gemm<__VA_ARGS__, false, false>(opA, opB, EPI, I, J,    \
                                                                   Src::COLS, 1, 0, 0); }); \
    printf("%-10s %-14s %.3f ms  %.1f TF\n", NAME, #__VA_ARGS__, ms, fl / ms / 1e9);       \
  }
#define ALL(NAME, EPI)                   \
  RUN(NAME, EPI, 128, 64, 32, 2, 1)      \
  RUN(NAME, EPI, 128, 64, 16, 2, 1)      \
  RUN(NAME, EPI, 128, 128, 32, 2, 2)     \
  RUN(NAME, EPI, 128, 128, 16, 2, 2)     \
  RUN(NAME, EPI, 128, 256, 16, 2, 4)     \
  RUN(NAME, EPI, 64, 128, 32, 1, 2)
  RUN("warmup", em, 128, 128, 16, 2, 2)
  ALL("mask", em)
  ALL("nomask", en)
  ALL("none", e0)
  {  // conv3 (stride 1): I = 64 channels, J = 81 pixels per image, K = 9 taps x 32
    using Src3 = ConvTRows<9, 9, 3, 3, 1, 32>;
    using W3 = ConvTWeights<3, 3, 1, 64, 32>;
    float *a2, *d2, *dy3, *w3;
    CK(hipMalloc(&a2, (long long)M * 81 * 64 * 4));
    CK(hipMalloc(&d2, (long long)M * 81 * 64 * 4));
    CK(hipMalloc(&dy3, (long long)M * 49 * 32 * 4));
    CK(hipMalloc(&w3, 9 * 64 * 32 * 4));
    fill<<<4096, 256>>>(a2, (long long)M * 81 * 64, 4);
    fill<<<4096, 256>>>(dy3, (long long)M * 49 * 32, 5);
    fill<<<64, 256>>>(w3, 9 * 64 * 32, 6);
    W3 oA{w3};
    RowsAsK<Src3> oB{Src3{dy3, M * Src3::L}};
    EpiConvT<9, 9, 1, 64> e3{d2, a2};
    const int I3 = W3::N, J3 = M * Src3::L;
    const double fl3 = 2.0 * I3 * J3 * Src3::COLS;
#define RUN3(...)                                                                                \
  {                                                                                               \
    float ms = timeit([&] { launch_gemm<__VA_ARGS__, false, false>(oA, oB, e3, I3, J3, Src3::COLS, \
                                                                   1, 0, 0); });                  \
    printf("conv3 dX %-14s %.3f ms  %.1f TF\n", #__VA_ARGS__, ms, fl3 / ms / 1e9);                \
  }
    RUN3(64, 128, 32, 1, 2)
    RUN3(64, 128, 32, 1, 2)
    RUN3(64, 128, 16, 1, 2)
    RUN3(64, 256, 16, 1, 4)
    RUN3(64, 256, 32, 1, 4)
    RUN3(64, 64, 32, 1, 1)
    RUN3(64, 64, 16, 1, 1)
  }
  return 0;
}
