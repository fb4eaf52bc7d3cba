// Timing probe: publishing max |x| of a streamed tensor from every wave / block
// of a launch into device memory (the f16x2 operand scales, f16x2.hpp) -- which
// publication pattern stays off the kernel's critical path.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/probes/amax_probe.hip -o scripts/probes/amax_probe
//   ./scripts/probes/amax_probe
// The streamed kernel is heads_dx4-shaped: 10240 x 512 f32 read + written as
// float4, 20480 waves.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ void upd(unsigned* q, float m, bool check) {
  const unsigned v = __float_as_uint(m);
  if (!check || v > __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(q, v);
}

// V: 0 none, 1 wave atomic 1 word, 2 wave check 1 word, 3 block check 1 word,
// 4 wave check 64 slots x 4 B, 5 wave check 64 slots x 256 B, 6 wave check 64
// slots x 4 KB, 7 block plain store into pmax[block], 8 block check 64 slots x 256 B
template <int V>
__global__ __launch_bounds__(256) void stream_kernel(const float4* x, float4* y, long long n4, unsigned* w,
                                                     float* pmax) {
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  float m = 0.f;
  if (q < n4) {
    float4 v = x[q];
    v.x *= 1.5f, v.y *= 1.5f, v.z *= 1.5f, v.w *= 1.5f;
    y[q] = v;
    m = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
  }
  if constexpr (V == 0) return;
  m = wmax(m);
  const int lane = threadIdx.x & 63;
  if constexpr (V == 3 || V == 7 || V == 8) {
    __shared__ float red[4];
    if (lane == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      if constexpr (V == 3) upd(w, m, true);
      if constexpr (V == 7) pmax[blockIdx.x] = m;
      if constexpr (V == 8) upd(w + 64 * (blockIdx.x & 63), m, true);
    }
    return;
  }
  if (lane != 0) return;
  if constexpr (V == 1) upd(w, m, false);
  if constexpr (V == 2) upd(w, m, true);
  if constexpr (V == 4) upd(w + (blockIdx.x & 63), m, true);
  if constexpr (V == 5) upd(w + 64 * (blockIdx.x & 63), m, true);
  if constexpr (V == 6) upd(w + 1024 * (blockIdx.x & 63), m, true);
}

// readers: 2048 blocks, every wave derives a scale before a short body
template <int R>
__global__ __launch_bounds__(256) void read_kernel(const unsigned* w, float* out) {
  const int lane = threadIdx.x & 63;
  float m;
  if constexpr (R == 0) m = __uint_as_float(*w);                         // one word
  if constexpr (R == 1) m = wmax(__uint_as_float(w[64 * lane]));          // 64 slots, lane-parallel
  if constexpr (R == 2) {                                                // 64 slots, serial
    unsigned u = 0;
    for (int i = 0; i < 64; ++i) u = max(u, w[64 * i]);
    m = __uint_as_float(u);
  }
  out[(long long)blockIdx.x * 256 + threadIdx.x] = m * (float)threadIdx.x;
}

__global__ void fill(float* p, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = (float)(h >> 8) * (1.0f / 16777216.0f) - 0.5f;
  }
}

template <class F>
static float timeit(F f, int reps = 20) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return 1e3f * ms / reps;
}

template <int V>
static void run(const float4* x, float4* y, long long n4, unsigned* w, float* pmax) {
  const int blocks = (int)((n4 + 255) / 256);
  const float us = timeit([&] {
    CK(hipMemsetAsync(w, 0, 64 * 1024 * 4));
    hipLaunchKernelGGL(stream_kernel<V>, dim3(blocks), dim3(256), 0, 0, x, y, n4, w, pmax);
  });
  const float base = timeit([&] { CK(hipMemsetAsync(w, 0, 64 * 1024 * 4)); });
  printf("publish V%d: %.1f us (memset alone %.1f)\n", V, us, base);
}

template <int R>
static void runr(const unsigned* w, float* out) {
  const float us = timeit([&] { hipLaunchKernelGGL(read_kernel<R>, dim3(2048), dim3(256), 0, 0, w, out); });
  printf("read R%d: %.1f us\n", R, us);
}

int main() {
  const long long n = 10240LL * 512, n4 = n / 4;
  float *x, *y, *pmax, *out;
  unsigned* w;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&pmax, 65536 * 4));
  CK(hipMalloc(&out, 2048 * 256 * 4));
  CK(hipMalloc(&w, 64 * 1024 * 4));
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, x, n);
  CK(hipDeviceSynchronize());
  const float4* x4 = reinterpret_cast<const float4*>(x);
  float4* y4 = reinterpret_cast<float4*>(y);
  run<0>(x4, y4, n4, w, pmax);
  run<1>(x4, y4, n4, w, pmax);
  run<2>(x4, y4, n4, w, pmax);
  run<3>(x4, y4, n4, w, pmax);
  run<4>(x4, y4, n4, w, pmax);
  run<5>(x4, y4, n4, w, pmax);
  run<6>(x4, y4, n4, w, pmax);
  run<7>(x4, y4, n4, w, pmax);
  run<8>(x4, y4, n4, w, pmax);
  run<0>(x4, y4, n4, w, pmax);
  runr<0>(w, out);
  runr<1>(w, out);
  runr<2>(w, out);
  runr<0>(w, out);
  CK(hipDeviceSynchronize());
  return 0;
}
