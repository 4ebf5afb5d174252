// eig2_probe.hip -- timing probe: what would a second resident user per CU buy the k = 180 Jacobi
// sweeps?  Two kernels run the same recursive-halving step (8 lanes per pair, float2 LDS columns,
// barrier per step, every pair rotated) for a fixed number of sweeps on synthetic users:
//   full : the whole k x k matrix in LDS (the production narrow layout), 1024 threads, 1 user/CU;
//   half : only SLOTS = 96 column slots in LDS (column c at slot c % 96: wrong math, same access
//          pattern and work), 768 threads, 2 users/CU.
// Output: microseconds per user and cycles per step for each.  Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

using f2 = __attribute__((ext_vector_type(2))) float;
constexpr int kGroup = 8;
constexpr int NR = 192, E2 = NR / 16, LD = 208;

__device__ __forceinline__ f2 lds_ld(const f2* p) { return *(const volatile __attribute__((address_space(3))) f2*)(p); }
__device__ __forceinline__ void lds_st(f2* p, f2 v) { *(volatile __attribute__((address_space(3))) f2*)(p) = v; }
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float pair_sum(float x) {
    x += dpp_mov<0xB1>(x);
    x += dpp_mov<0x4E>(x);
    x += dpp_mov<0x141>(x);
    return x;
}

template <int NT, int SLOTS, int WPE>
__global__ __launch_bounds__(NT, WPE) void sweeps(const float* Bg, float* out, int k, int nsweeps, unsigned long long* cyc) {
    extern __shared__ float smem[];
    float* B = smem;
    float* s_nrm = B + SLOTS * LD;
    float* s_dev = s_nrm + NR;
    const int tid = threadIdx.x;
    const float* src = Bg + (size_t)blockIdx.x * k * k;
    for (int idx = tid; idx < SLOTS * LD; idx += NT) B[idx] = 0.0f;
    __syncthreads();
    for (int c = 0; c < k; ++c)
        for (int i = tid; i < k; i += NT) B[(c % SLOTS) * LD + i] = src[(size_t)c * k + i];
    for (int i = tid; i < NR; i += NT) {
        s_nrm[i] = 1.0f;
        s_dev[i] = 0.0f;
    }
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const int n = (k + 1) & ~1;
    const int g = tid / kGroup, lig = tid % kGroup;
    constexpr int NG = NT / kGroup;
    int steps = 0;
    for (int sweep = 0; sweep < nsweeps; ++sweep) {
        for (int L = 0;; ++L) {
            const int segmax = (n + (1 << L) - 1) >> L;
            if (segmax < 2) break;
            const int FL = (segmax + 1) >> 1;
            steps += FL;
            const int sigma = g / FL, fi = g - sigma * FL;
            int s0 = 0, s1 = n;
            for (int bit = L - 1; bit >= 0; --bit) {
                const int half = (s1 - s0 + 1) >> 1;
                if ((sigma >> bit) & 1) s0 += half;
                else s1 = s0 + half;
            }
            const int f = (s1 - s0 + 1) >> 1, t = (s1 - s0) - f;
            const int p = s0 + fi;
            const bool fixed = g < NG && sigma < (1 << L) && fi < f && p < k;
            f2* bp = reinterpret_cast<f2*>(B + (fixed ? p % SLOTS : 0) * LD);
            f2 xp[E2];
            float devp = 0.0f, al = 0.0f;
            if (fixed) {
                f2 al2 = {0.f, 0.f};
#pragma unroll
                for (int e = 0; e < E2; ++e) {
                    xp[e] = lds_ld(bp + kGroup * e + lig);
                    al2 = __builtin_elementwise_fma(xp[e], xp[e], al2);
                }
                devp = s_dev[p];
                al = pair_sum(al2.x + al2.y);
            }
            const int tv = fixed ? min(t, k - s0 - f) : 0;
            const int nlive = fixed ? f : 0;
            int ti = fi;
            for (int step = 0; step < FL; ++step) {
                const int q = s0 + f + ti;
                if (step < nlive && ti < tv) {
                    f2* bq = reinterpret_cast<f2*>(B + (q % SLOTS) * LD);
                    const float dq = s_dev[q];
                    const float be = s_nrm[q];
                    f2 xq[E2];
                    f2 ga2[2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
                    for (int e = 0; e < E2; ++e) xq[e] = lds_ld(bq + kGroup * e + lig);
#pragma unroll
                    for (int e = 0; e < E2; ++e) ga2[e & 1] = __builtin_elementwise_fma(xp[e], xq[e], ga2[e & 1]);
                    const f2 gs = ga2[0] + ga2[1];
                    const float ga = pair_sum(gs.x + gs.y);
                    const float dd = be - al;
                    const float r = __builtin_amdgcn_sqrtf(fmaf(dd, dd, 4.0f * ga * ga));
                    const float tt = (dd < 0.0f ? -2.0f * ga : 2.0f * ga) * __builtin_amdgcn_rcpf(fabsf(dd) + r + 1e-30f);
                    const float c = __builtin_amdgcn_rsqf(fmaf(tt, tt, 1.0f));
                    const float sn = c * tt;
                    const f2 c2 = {c, c}, s2 = {sn, sn}, ns2 = {-sn, -sn};
#pragma unroll
                    for (int e = 0; e < E2; ++e) {
                        const f2 np = __builtin_elementwise_fma(ns2, xq[e], c2 * xp[e]);
                        lds_st(bq + kGroup * e + lig, __builtin_elementwise_fma(s2, xp[e], c2 * xq[e]));
                        xp[e] = np;
                    }
                    const float delta = fmaf(sn, sn, fmaf(c, c, -1.0f));
                    const float cc = c * c, ss = sn * sn;
                    const float ndp = delta + fmaf(cc, devp, ss * dq);
                    const float csg = 2.0f * c * sn * ga;
                    const float nal = fmaf(cc, al, fmaf(ss, be, -csg));
                    if (lig == 0) {
                        s_dev[q] = delta + fmaf(ss, devp, cc * dq);
                        s_nrm[q] = fmaf(ss, al, fmaf(cc, be, csg));
                    }
                    devp = ndp;
                    al = nal;
                }
                __syncthreads();
                if (++ti == f) ti = 0;
            }
            if (fixed) {
#pragma unroll
                for (int e = 0; e < E2; ++e) lds_st(bp + kGroup * e + lig, xp[e]);
                if (lig == 0) {
                    s_dev[p] = devp;
                    s_nrm[p] = al;
                }
            }
            __syncthreads();
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) {
        atomicAdd(&cyc[0], t1 - t0);
        atomicAdd(&cyc[1], (unsigned long long)steps);
    }
    for (int i = tid; i < k; i += NT) out[(size_t)blockIdx.x * k + i] = s_nrm[i] + B[(i % SLOTS) * LD + i];
}

template <int NT, int SLOTS, int WPE>
void run(const char* name, const float* dB, float* dout, int users, int k, int nsweeps, unsigned long long* dcyc,
         size_t lds_min = 0) {
    const size_t lds = std::max(lds_min, sizeof(float) * ((size_t)SLOTS * LD + 2 * NR));
    hipFuncSetAttribute((const void*)sweeps<NT, SLOTS, WPE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipMemset(dcyc, 0, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((sweeps<NT, SLOTS, WPE>), dim3(users), dim3(NT), lds, 0, dB, dout, k, nsweeps, dcyc);   // warm
    hipMemset(dcyc, 0, 16);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((sweeps<NT, SLOTS, WPE>), dim3(users), dim3(NT), lds, 0, dB, dout, k, nsweeps, dcyc);
    hipEventRecord(e1, 0);
    hipError_t err = hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    hipMemcpy(c, dcyc, 16, hipMemcpyDeviceToHost);
    // s_memtime runs at 100 MHz on gfx950: wall cycles of the shader clock = ticks * (sclk / 100 MHz)
    std::printf("%-6s k=%d users=%d sweeps=%d lds=%zu: %s  %.2f ms  %.3f us/user  %.1f memtime ticks/step\n", name, k,
                users, nsweeps, lds, hipGetErrorString(err), ms, 1000.0 * ms / users, (double)c[0] / (double)c[1]);
}

int main(int argc, char** argv) {
    const int users = argc > 1 ? atoi(argv[1]) : 20480;
    const int k = argc > 2 ? atoi(argv[2]) : 180;
    const int nsweeps = argc > 3 ? atoi(argv[3]) : 7;
    std::vector<float> h((size_t)users * k * k);
    unsigned s = 12345;
    for (int u = 0; u < users; ++u)
        for (int j = 0; j < k; ++j)
            for (int i = 0; i < k; ++i) {
                s = s * 1664525u + 1013904223u;
                h[((size_t)u * k + j) * k + i] = (i == j) ? 1.0f : ((s >> 8) * (1.0f / 16777216.0f) - 0.5f) * 0.02f;
            }
    float *dB, *dout;
    unsigned long long* dcyc;
    hipMalloc(&dB, h.size() * 4);
    hipMalloc(&dout, (size_t)users * k * 4);
    hipMalloc(&dcyc, 16);
    hipMemcpy(dB, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    run<1024, 188, 4>("full", dB, dout, users, k, nsweeps, dcyc);
    run<768, 96, 6>("half", dB, dout, users, k, nsweeps, dcyc);
    run<1024, 188, 4>("full", dB, dout, users, k, nsweeps, dcyc);
    run<768, 96, 6>("half", dB, dout, users, k, nsweeps, dcyc);
    run<768, 96, 6>("half1", dB, dout, users, k, nsweeps, dcyc, 100000);   // same kernel, 1 user/CU
    return 0;
}
