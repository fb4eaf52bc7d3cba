// Standalone timing probe for the GEMM engine's reduction shapes (no torch).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize \
//     scripts/probes/gemm_probe.hip -o scripts/probes/gemm_probe && ./scripts/probes/gemm_probe
// Times the conv2 [P|dY|1]^T[P|dY|1] reduction (implicit im2col) against the
// same reduction over a dense, materialised patch matrix, and a square GEMM.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gemm_stream.hpp"

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

template <class F>
static float timeit(F f, int reps = 5) {
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

static void check_nc(int nc) {
  if (nc > 1024) {
    fprintf(stderr, "too many chunks %d\n", nc);
    exit(1);
  }
}
static void plan(long long rows, int tiles, int target, int* nc, int* ch) {
  long long n = target / tiles;
  if (n < 1) n = 1;
  long long c = (rows + n - 1) / n;
  if (c < 256) c = 256;
  c = (c + 31) / 32 * 32;
  *nc = (int)((rows + c - 1) / c);
  *ch = (int)c;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 10240;
  const long long R = (long long)M * 81;  // conv2 output pixels
  const int K = 512, COUT = 64;
  const int I = K, J = K + COUT + 1;
  float *a1, *dy, *dense, *part;
  const long long a1n = (long long)M * 400 * 32;
  CK(hipMalloc(&a1, a1n * 4));
  CK(hipMalloc(&dy, R * COUT * 4));
  CK(hipMalloc(&dense, R * K * 4));
  fill<<<4096, 256>>>(a1, a1n, 1);
  fill<<<4096, 256>>>(dy, R * COUT, 2);
  fill<<<4096, 256>>>(dense, R * K, 3);
  int live = 0;
  for (int x = 0; x < 4; ++x)
    for (int y = 0; y < 5; ++y)
      if (!(y < x && (y + 1) * 128 <= K)) ++live;
  int nc, ch;
  plan_rounds(R, live, 512, &nc, &ch); check_nc(nc);
  const int max_chunks = 1024;  // every plan below stays under this (checked)
  CK(hipMalloc(&part, (long long)max_chunks * (I + 1) * J * 4));
  const double flops = 2.0 * R * 128.0 * 128.0 * live;  // computed tiles
  printf("M=%d rows=%lld chunks=%d x %d, live tiles %d\n", M, R, nc, ch, live);

  using Conv2 = ConvRows<float, 20, 20, 32, 4, 4, 2>;
  {
    RowsAsI<Conv2> opA{Conv2{a1, 400 * 32, (int)R}};
    CatRowsI<Conv2> opB{Conv2{a1, 400 * 32, (int)R}, K, dy, COUT, COUT, COUT, (int)R};
    EpiPartial epi{part, I, J};
    float ms = timeit([&] {
      launch_gemm<128, 128, 32, 2, 2, true, true>(opA, opB, epi, I, J, (int)R, nc, ch, 0, K);
    });
    printf("conv2 implicit  128x128x32: %.3f ms  %.1f TF (computed tiles)\n", ms, flops / ms / 1e9);
    float ms2 = timeit([&] {
      launch_gemm<128, 128, 16, 2, 2, true, true>(opA, opB, epi, I, J, (int)R, nc, ch, 0, K);
    });
    printf("conv2 implicit  128x128x16: %.3f ms  %.1f TF (computed tiles)\n", ms2, flops / ms2 / 1e9);
    {
      int ncq, chq;
      plan_rounds(R, live, 1024, &ncq, &chq);
      check_nc(ncq);
      float msq = timeit([&] {
        launch_gemm<128, 128, 16, 2, 2, true, true, 2>(opA, opB, epi, I, J, (int)R, ncq, chq, 0, K);
      });
      printf("conv2 implicit  128x128x16 depth2 (1024 slots): %.3f ms  %.1f TF\n", msq, flops / msq / 1e9);
    }
    int nc3, ch3;
    plan_rounds(R, 8, 256, &nc3, &ch3); check_nc(nc3);
    float ms3 = timeit([&] {
      launch_gemm<256, 128, 32, 4, 2, true, true>(opA, opB, epi, I, J, (int)R, nc3, ch3, 0, K);
    });
    printf("conv2 implicit  256x128x32 (8 live): %.3f ms  %.1f TF (computed tiles)\n", ms3,
           2.0 * R * 256 * 128 * 8 / ms3 / 1e9);
    plan_rounds(R, 8, 512, &nc3, &ch3); check_nc(nc3);
    float ms4 = timeit([&] {
      launch_gemm<256, 128, 32, 4, 2, true, true>(opA, opB, epi, I, J, (int)R, nc3, ch3, 0, K);
    });
    printf("conv2 implicit  256x128x32 (8 live, planned for 512 slots): %.3f ms  %.1f TF (computed tiles)\n", ms4,
           2.0 * R * 256 * 128 * 8 / ms4 / 1e9);
  }
  {
    RowsAsI<DenseRows> opA{DenseRows{dense, K, (int)R, K}};
    CatRowsI<DenseRows> opB{DenseRows{dense, K, (int)R, K}, K, dy, COUT, COUT, COUT, (int)R};
    EpiPartial epi{part, I, J};
    float ms = timeit([&] {
      launch_gemm<128, 128, 32, 2, 2, true, true>(opA, opB, epi, I, J, (int)R, nc, ch, 0, K);
    });
    printf("dense reduction 128x128x32: %.3f ms  %.1f TF\n", ms, flops / ms / 1e9);
    float ms2 = timeit([&] {
      launch_gemm<128, 128, 16, 2, 2, true, true>(opA, opB, epi, I, J, (int)R, nc, ch, 0, K);
    });
    printf("dense reduction 128x128x16: %.3f ms  %.1f TF\n", ms2, flops / ms2 / 1e9);
    // the same over a 1/8 slice that stays resident in the Infinity Cache
    const long long R8 = R / 8;
    int nc8, ch8;
    plan_rounds(R8, live, 512, &nc8, &ch8); check_nc(nc8);
    RowsAsI<DenseRows> opA8{DenseRows{dense, K, (int)R8, K}};
    CatRowsI<DenseRows> opB8{DenseRows{dense, K, (int)R8, K}, K, dy, COUT, COUT, COUT, (int)R8};
    float ms3 = timeit([&] {
      launch_gemm<128, 128, 32, 2, 2, true, true>(opA8, opB8, epi, I, J, (int)R8, nc8, ch8, 0, K);
    }, 20);
    printf("dense reduction R/8 (resident) 128x128x32: %.3f ms  %.1f TF\n", ms3, flops / 8 / ms3 / 1e9);
    // plain operands (no [P|dY|1] segment logic) on the same rows
    RowsAsI<DenseRows> opB9{DenseRows{dense, K, (int)R, K}};
    EpiPartial epi9{part, I, K};
    const double fl9 = 2.0 * R * 128.0 * 128.0 * 10;
    float ms4 = timeit([&] {
      launch_gemm<128, 128, 32, 2, 2, true, false>(opA, opB9, epi9, I, K, (int)R, nc, ch, 0, K);
    });
    printf("dense P^T P (sym, plain ops) 128x128x32: %.3f ms  %.1f TF\n", ms4, fl9 / ms4 / 1e9);
    // same 14 live tiles as [P|dY|1] but B is a plain row source (cols >= 512 read as 0)
    RowsAsI<DenseRows> opB10{DenseRows{dense, K, (int)R, K}};
    float ms5 = timeit([&] {
      launch_gemm<128, 128, 32, 2, 2, true, true>(opA, opB10, epi, I, J, (int)R, nc, ch, 0, K);
    });
    printf("dense, plain B, J=577      128x128x32: %.3f ms  %.1f TF\n", ms5, flops / ms5 / 1e9);
    float ms6 = timeit([&] {
      launch_gemm<128, 128, 32, 2, 2, true, false>(opA, opB10, epi, I, J, (int)R, nc, ch, 0, K);
    });
    printf("dense, plain B, no colsum  128x128x32: %.3f ms  %.1f TF\n", ms6, flops / ms6 / 1e9);
    // padded row stride (544 floats) instead of 2 KB
    const int LDP = 544;
    float* dp;
    CK(hipMalloc(&dp, R * LDP * 4));
    fill<<<4096, 256>>>(dp, R * LDP, 7);
    RowsAsI<DenseRows> opAp{DenseRows{dp, LDP, (int)R, K}};
    CatRowsI<DenseRows> opBp{DenseRows{dp, LDP, (int)R, K}, K, dy, COUT, COUT, COUT, (int)R};
    float ms7 = timeit([&] {
      launch_gemm<128, 128, 32, 2, 2, true, true>(opAp, opBp, epi, I, J, (int)R, nc, ch, 0, K);
    });
    printf("dense reduction ld=544     128x128x32: %.3f ms  %.1f TF\n", ms7, flops / ms7 / 1e9);
    CK(hipFree(dp));
    // every row aliases row 0..7 (ld = 0 and a 8-row period via 'rows' trick is not
    // available): ld = 0 -> the whole reduction reads one 2 KB row (all L2 hits)
    RowsAsI<DenseRows> opAz{DenseRows{dense, 0, (int)R, K}};
    CatRowsI<DenseRows> opBz{DenseRows{dense, 0, (int)R, K}, K, dy, 0, COUT, COUT, (int)R};
    float ms9 = timeit([&] {
      launch_gemm<128, 128, 32, 2, 2, true, true>(opAz, opBz, epi, I, J, (int)R, nc, ch, 0, K);
    });
    printf("dense reduction ld=0 (L2)  128x128x32: %.3f ms  %.1f TF\n", ms9, flops / ms9 / 1e9);
    // exactly one round: 16 tiles x 32 chunks = 512 blocks, plain operands, no sym
    {
      const int ncx = 32;
      const int chx = (int)((R / ncx + 31) / 32 * 32);
      EpiPartial epx{part, K, K};
      const double fx = 2.0 * R * K * K;
      float msx = timeit([&] {
        launch_gemm<128, 128, 32, 2, 2, true, false>(opA, opB9, epx, K, K, (int)R, ncx, chx, 0, 0);
      });
      printf("P^T P 512 blocks (1 round) : %.3f ms  %.1f TF\n", msx, fx / msx / 1e9);
      const int ncy = 64;
      const int chy = (int)((R / ncy + 31) / 32 * 32);
      float msy = timeit([&] {
        launch_gemm<128, 128, 32, 2, 2, true, false>(opA, opB9, epx, K, K, (int)R, ncy, chy, 0, 0);
      });
      printf("P^T P 1024 blocks (2 rounds): %.3f ms  %.1f TF\n", msy, fx / msy / 1e9);
    }
    // 256x128 tiles (1 block/CU), same work
    int live2 = 0;
    for (int x = 0; x < 2; ++x)
      for (int y = 0; y < 5; ++y)
        if (!(2 * y + 1 < 2 * x)) ++live2;  // approx; timing only
    int nc2, ch2;
    plan_rounds(R, 10, 256, &nc2, &ch2); check_nc(nc2);
    float ms8 = timeit([&] {
      launch_gemm<256, 128, 32, 4, 2, true, true>(opA, opB, epi, I, J, (int)R, nc2, ch2, 0, 0);
    });
    printf("dense reduction 256x128x32 (no sym skip, 10 tiles): %.3f ms  %.1f TF\n", ms8,
           2.0 * R * 256.0 * 128.0 * 10 / ms8 / 1e9);
    (void)live2;
  }
  {  // conv2 input gradient: the 4 stride phases as 4 x 32 columns, K = 4 taps x 64
    using Src = ConvTRows<20, 20, 4, 4, 2, 64>;
    using W = ConvTWeights<4, 4, 2, 32, 64>;
    float *w2, *d1;
    CK(hipMalloc(&w2, 4 * 4 * 32 * 64 * 4));
    CK(hipMalloc(&d1, a1n * 4));
    fill<<<64, 256>>>(w2, 4 * 4 * 32 * 64, 9);
    RowsAsK<Src> opA{Src{dy, M * Src::L}};
    W opB{w2};
    EpiConvT<20, 20, 2, 32> epi{d1, a1};
    const double fl = 2.0 * M * Src::L * W::N * Src::COLS;
    float m1 = timeit([&] {
      launch_gemm<128, 128, 16, 2, 2, false, false>(opA, opB, epi, M * Src::L, W::N, Src::COLS, 1, 0, 0);
    });
    printf("conv2 dX 128x128x16: %.3f ms  %.1f TF\n", m1, fl / m1 / 1e9);
    float m2 = timeit([&] {
      launch_gemm<128, 128, 32, 2, 2, false, false>(opA, opB, epi, M * Src::L, W::N, Src::COLS, 1, 0, 0);
    });
    printf("conv2 dX 128x128x32: %.3f ms  %.1f TF\n", m2, fl / m2 / 1e9);
    float m3 = timeit([&] {
      launch_gemm<128, 64, 32, 2, 1, false, false>(opA, opB, epi, M * Src::L, W::N, Src::COLS, 1, 0, 0);
    });
    printf("conv2 dX 128x64x32: %.3f ms  %.1f TF\n", m3, fl / m3 / 1e9);
    float m4 = timeit([&] {
      launch_gemm<64, 128, 32, 1, 2, false, false>(opA, opB, epi, M * Src::L, W::N, Src::COLS, 1, 0, 0);
    });
    printf("conv2 dX 64x128x32: %.3f ms  %.1f TF\n", m4, fl / m4 / 1e9);
    float m5 = timeit([&] {
      launch_gemm<256, 128, 16, 4, 2, false, false>(opA, opB, epi, M * Src::L, W::N, Src::COLS, 1, 0, 0);
    });
    printf("conv2 dX 256x128x16: %.3f ms  %.1f TF\n", m5, fl / m5 / 1e9);
    CK(hipFree(w2));
    CK(hipFree(d1));
  }
  {
    const int N = 4096;
    float *A, *B, *C;
    CK(hipMalloc(&A, (long long)N * N * 4));
    CK(hipMalloc(&B, (long long)N * N * 4));
    CK(hipMalloc(&C, (long long)N * N * 4));
    fill<<<4096, 256>>>(A, (long long)N * N, 4);
    fill<<<4096, 256>>>(B, (long long)N * N, 5);
    RowsAsK<DenseRows> opA{DenseRows{A, N, N, N}};
    MatI<true> opB{B, N, N, N};
    EpiStore epi{C, N};
    float ms = timeit([&] { launch_gemm<128, 128, 32, 2, 2, false, false>(opA, opB, epi, N, N, N, 1, 0, 0); });
    printf("square 4096 KCONTIG-A     : %.3f ms  %.1f TF\n", ms, 2.0 * N * N * N / ms / 1e9);
    // both operands i-contiguous: C = A^T B with A stored [k][i]
    RowsAsI<DenseRows> opT{DenseRows{A, N, N, N}};
    float ms2 = timeit([&] { launch_gemm<128, 128, 32, 2, 2, false, false>(opT, opB, epi, N, N, N, 1, 0, 0); });
    printf("square 4096 both i-contig : %.3f ms  %.1f TF\n", ms2, 2.0 * N * N * N / ms2 / 1e9);
    float* P;
    CK(hipMalloc(&P, (long long)N * (N + 1) * 4 * 2));
    EpiPartial ep{P, N, N};
    float ms3 = timeit([&] { launch_gemm<128, 128, 32, 2, 2, true, false>(opT, opB, ep, N, N, N, 1, N, 0); });
    printf("square 4096 i-contig SPLITK(1 chunk, remap): %.3f ms  %.1f TF\n", ms3, 2.0 * N * N * N / ms3 / 1e9);
    float ms4 = timeit([&] { launch_gemm<128, 128, 32, 2, 2, true, false>(opT, opB, ep, N, N, N, 2, N / 2, 0); });
    printf("square 4096 i-contig SPLITK(2 chunks, remap): %.3f ms  %.1f TF\n", ms4, 2.0 * N * N * N / ms4 / 1e9);
  }
  CK(hipGetLastError());
  return 0;
}
