// Verifies the v_mfma_f64_16x16x4_f64 operand / result lane maps used by the
// predictor's block GEMM with exact integer data: A lane l = A[l&15][l>>4],
// B lane l = B[l>>4][l&15], D reg q of lane l = C[(l>>4) + 4q][l&15].
#include <hip/hip_runtime.h>
#include <cstdio>

using d4 = __attribute__((ext_vector_type(4))) double;

__global__ void probe(const double* A, const double* B, double* C) {
    const int l = threadIdx.x;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
    for (int q = 0; q < 4; ++q) C[((l >> 4) + 4 * q) * 16 + (l & 15)] = acc[q];
}

int main() {
    double hA[64], hB[64], hC[256], ref[256];
    for (int i = 0; i < 64; ++i) { hA[i] = (i * 7) % 11 - 5; hB[i] = (i * 5) % 13 - 6; }
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += hA[r * 4 + k] * hB[k * 16 + c];
            ref[r * 16 + c] = s;
        }
    double *dA, *dB, *dC;
    hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += hC[i] != ref[i];
    printf("mfma_f64_16x16x4 layout mismatches: %d / 256\n", bad);
    return bad != 0;
}
