// probe_sort.hip -- which rocprim radix-sort configurations run on this gfx950 for 64-bit keys
// with 32-bit values at ~10M items (the default onesweep dispatch returned invalid argument).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <vector>

template <class Cfg>
void run(const char* name, uint64_t* ka, uint64_t* kb, uint32_t* va, uint32_t* vb, int n, int bits) {
    size_t need = 0;
    hipError_t e = rocprim::radix_sort_pairs<Cfg>(nullptr, need, ka, kb, va, vb, n, 0, bits, 0);
    void* tmp = nullptr;
    if (e == hipSuccess) e = hipMalloc(&tmp, need);
    hipEvent_t t0, t1;
    hipEventCreate(&t0);
    hipEventCreate(&t1);
    hipEventRecord(t0, 0);
    if (e == hipSuccess) e = rocprim::radix_sort_pairs<Cfg>(tmp, need, ka, kb, va, vb, n, 0, bits, 0);
    hipEventRecord(t1, 0);
    hipError_t e2 = hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, t0, t1);
    std::vector<uint64_t> h(n);
    hipMemcpy(h.data(), kb, 8ull * n, hipMemcpyDeviceToHost);
    bool sorted = true;
    for (int i = 1; i < n; ++i) sorted &= h[i - 1] <= h[i];
    std::printf("%-28s err %s / %s  temp %zu  %.2f ms  sorted %d\n", name, hipGetErrorString(e), hipGetErrorString(e2),
                need, ms, (int)sorted);
    (void)hipGetLastError();
    if (tmp) hipFree(tmp);
}

__global__ void fill(uint64_t* k, uint32_t* v, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        x ^= x >> 29;
        k[i] = x & ((1ull << 47) - 1);
        v[i] = i;
    }
}

int main() {
    const int n = 10670686, bits = 47;
    uint64_t *ka, *kb;
    uint32_t *va, *vb;
    hipMalloc(&ka, 8ull * n);
    hipMalloc(&kb, 8ull * n);
    hipMalloc(&va, 4ull * n);
    hipMalloc(&vb, 4ull * n);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    std::printf("%s sharedMemPerBlock %zu maxSharedPerMP %zu\n", p.gcnArchName, p.sharedMemPerBlock,
                p.maxSharedMemoryPerMultiProcessor);
    auto refill = [&] { hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, 0, ka, va, n); };
    refill();
    run<rocprim::default_config>("default", ka, kb, va, vb, n, bits);
    refill();
    using os4 = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                           rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>,
                                                                               rocprim::kernel_config<256, 12>, 4>>;
    run<os4>("onesweep 256x12 4b", ka, kb, va, vb, n, bits);
    refill();
    using os8 = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                           rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 8>,
                                                                               rocprim::kernel_config<256, 8>, 8>>;
    run<os8>("onesweep 256x8 8b", ka, kb, va, vb, n, bits);
    refill();
    using ms = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config,
                                          (size_t)1 << 40>;
    run<ms>("merge sort", ka, kb, va, vb, n, bits);
    return 0;
}
