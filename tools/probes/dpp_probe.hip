// Semantics probe for the CDNA4 cross-lane moves the systolic Jacobi levels rely on
// (cf_eigen.hip: lane_next, pair_sum_strided).  Prints OK / MISMATCH lines.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
    const int l = threadIdx.x;
    const int shl = __builtin_amdgcn_update_dpp(-1, l, 0x130, 0xF, 0xF, false);   // wave_shl:1
    const int ror8 = __builtin_amdgcn_update_dpp(-1, l, 0x128, 0xF, 0xF, false);  // row_ror:8
    const auto p16 = __builtin_amdgcn_permlane16_swap(l, l, false, false);
    const auto p32 = __builtin_amdgcn_permlane32_swap(l, l, false, false);
    float x = (float)(1 << (l >> 3));   // strided group sum: lanes {s + 8m} -> sum_m 2^m = 255
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));
    const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_int(x), __float_as_int(x), false, false);
    x = __int_as_float(r16[0]) + __int_as_float(r16[1]);
    const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_int(x), __float_as_int(x), false, false);
    x = __int_as_float(r32[0]) + __int_as_float(r32[1]);
    out[l * 8 + 0] = shl;
    out[l * 8 + 1] = ror8;
    out[l * 8 + 2] = p16[0];
    out[l * 8 + 3] = p16[1];
    out[l * 8 + 4] = p32[0];
    out[l * 8 + 5] = p32[1];
    out[l * 8 + 6] = (int)x;
}

int main() {
    int* d;
    int h[64 * 8];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad_shl = 0, bad_ror = 0, bad_sum = 0;
    for (int l = 0; l < 64; ++l) {
        if (l < 63 && h[l * 8] != l + 1) ++bad_shl;
        if (h[l * 8 + 1] != ((l & ~15) | ((l + 8) & 15))) ++bad_ror;
        if (h[l * 8 + 6] != 255) ++bad_sum;
    }
    printf("wave_shl:1 lane i <- i+1: %s (lane 63 -> %d)\n", bad_shl ? "MISMATCH" : "OK", h[63 * 8]);
    printf("row_ror:8: %s\n", bad_ror ? "MISMATCH" : "OK");
    printf("strided pair sum: %s\n", bad_sum ? "MISMATCH" : "OK");
    printf("permlane16_swap lanes 0,16,32,48: r0 %d %d %d %d r1 %d %d %d %d\n", h[2], h[16 * 8 + 2], h[32 * 8 + 2],
           h[48 * 8 + 2], h[3], h[16 * 8 + 3], h[32 * 8 + 3], h[48 * 8 + 3]);
    printf("permlane32_swap lanes 0,32: r0 %d %d r1 %d %d\n", h[4], h[32 * 8 + 4], h[5], h[32 * 8 + 5]);
    hipFree(d);
    return (bad_shl || bad_ror || bad_sum) ? 1 : 0;
}
