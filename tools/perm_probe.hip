#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
    unsigned v = threadIdx.x;
    auto r16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    auto r32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    unsigned d8 = __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, false);
    out[threadIdx.x * 5 + 0] = r16[0];
    out[threadIdx.x * 5 + 1] = r16[1];
    out[threadIdx.x * 5 + 2] = r32[0];
    out[threadIdx.x * 5 + 3] = r32[1];
    out[threadIdx.x * 5 + 4] = d8;
}
int main() {
    unsigned* d; hipMalloc(&d, 64 * 5 * 4);
    k<<<1, 64>>>(d);
    unsigned h[320]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) printf("%2d: p16 %2u %2u  p32 %2u %2u  dpp8 %2u\n", l, h[l*5], h[l*5+1], h[l*5+2], h[l*5+3], h[l*5+4]);
    return 0;
}
