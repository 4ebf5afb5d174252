// Probe the operand/result lane layout of v_mfma_i32_32x32x32_i8 with exact integers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void probe(const int8_t* A, const int8_t* B, int* C) {
  // A: 32x32 row-major (row r, k), B: 32x32 row-major (k, col c); hypothesis:
  // lane l holds A[l&31][16*(l>>5) + j] and B[16*(l>>5) + j][l&31], j = 0..15
  int l = threadIdx.x;
  int r = l & 31, h = l >> 5;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) { a[j] = A[r * 32 + 16 * h + j]; b[j] = B[(16 * h + j) * 32 + r]; }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16); __builtin_memcpy(&bv, b, 16);
  v16i acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc, 0, 0, 0);
  for (int reg = 0; reg < 16; ++reg) {
    int row = (reg & 3) + 8 * (reg >> 2) + 4 * h, col = r;
    C[row * 32 + col] = acc[reg];
  }
}
int main() {
  int8_t hA[1024], hB[1024]; int hC[1024], ref[1024];
  for (int i = 0; i < 1024; ++i) { hA[i] = (int8_t)((i * 7 + 3) % 11 - 5); hB[i] = (int8_t)((i * 13 + 1) % 9 - 4); }
  for (int r = 0; r < 32; ++r) for (int c = 0; c < 32; ++c) { int s = 0; for (int k = 0; k < 32; ++k) s += hA[r*32+k]*hB[k*32+c]; ref[r*32+c] = s; }
  int8_t *dA, *dB; int* dC;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 4096);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 1024; ++i) bad += hC[i] != ref[i];
  printf("i8 32x32x32 layout mismatches: %d of 1024 (hypothesis k = 16*(lane>>5) + j)\n", bad);
  return bad != 0;
}
