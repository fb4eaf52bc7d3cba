// Probe: operand/result lane maps of v_mfma_i32_32x32x32_i8 on gfx950.
// Hypothesis: lane l holds A[row l&31][k = 16*(l>>5) + j] (j=0..15, 16 bytes),
// B[k = 16*(l>>5) + j][col l&31]; D[row][col], col = l&31,
// row = (r&3) + 8*(r>>2) + 4*(l>>5).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void probe(const signed char* A, const signed char* B, int* D) {
  const int l = threadIdx.x;
  signed char a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    a[j] = A[(l & 31) * 32 + 16 * (l >> 5) + j];   // A is 32x32 row-major [row][k]
    b[j] = B[(16 * (l >> 5) + j) * 32 + (l & 31)];  // B is 32x32 row-major [k][col]
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v16i c = {0};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    D[row * 32 + (l & 31)] = c[r];
  }
}

int main() {
  signed char hA[1024], hB[1024];
  int hD[1024], ref[1024];
  srand(1);
  for (int i = 0; i < 1024; ++i) { hA[i] = (signed char)(rand() % 256 - 128); hB[i] = (signed char)(rand() % 256 - 128); }
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
    int s = 0; for (int k = 0; k < 32; ++k) s += hA[i * 32 + k] * hB[k * 32 + j]; ref[i * 32 + j] = s; }
  signed char *dA, *dB; int* dD;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dD, 4096);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 1024; ++i) bad += hD[i] != ref[i];
  printf("i8 32x32x32 layout hypothesis: %d / 1024 mismatches (D[0]=%d ref=%d)\n", bad, hD[0], ref[0]);
  return bad != 0;
}
