// Latency of dependent fp64 VALU chains on gfx950 and the accuracy of v_rsq_f64 (planning data
// for the spill solver's QL generator).  One wave; s_memtime around 4096-step chains.
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/fp64_chain_probe.hip -o /tmp/fp64_chain_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

constexpr int N = 4096;

__global__ void chains(const double* in, double* out, unsigned long long* cyc) {
    double x = in[threadIdx.x], y = in[threadIdx.x + 64];
    unsigned long long t0, t1;
    // 0: dependent fma
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) x = fma(x, 0.999999, 1e-7);
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
    // 1: dependent mul
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) y = y * 1.0000001;
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[1] = t1 - t0;
    // 2: dependent rsq (x -> rsq(x) stays in [~0.5, 2])
    double z = 1.5 + 0.1 * x;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) z = __builtin_amdgcn_rsq(z) + 0.5;
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[2] = t1 - t0;
    // 3: the QL generator's rotation chain (one lane's recurrence, as in eigen_spill_kernel)
    double p = 0.3 + 0.01 * y, c = 1.0, sn = 0.0;
    const double di = 0.7, ei = 0.2;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        const double g = c * ei;
        const double x2 = fma(p, p, ei * ei);
        double inv = __builtin_amdgcn_rsq(x2);
        const double hx = 0.5 * x2;
        inv = inv * fma(-hx, inv * inv, 1.5);
        inv = inv * fma(-hx, inv * inv, 1.5);
        sn = ei * inv;
        c = p * inv;
        p = c * di - sn * g;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[3] = t1 - t0;
    // 4: the same with p' = inv (p di - ei g) and one Newton step
    double p2 = 0.3 + 0.01 * y, c2 = 1.0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        const double g = c2 * ei;
        const double x2 = fma(p2, p2, ei * ei);
        const double tt = fma(p2, di, -ei * g);
        double inv = __builtin_amdgcn_rsq(x2);
        const double hx = 0.5 * x2;
        inv = inv * fma(-hx, inv * inv, 1.5);
        c2 = p2 * inv;
        p2 = inv * tt;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[4] = t1 - t0;
    out[threadIdx.x] = x + y + z + p + c + sn + p2 + c2;
}


// 5: the generator's block loop as eigen_spill_kernel runs it (readlane broadcasts, lane-0
// LDS + global stores under exec masking), over `len` positions; wave 0 times it, waves
// 1.. (if any) spin on dependent-free fp64 FMAs while `spin` is set (SIMD sharing)
template <int V>
__global__ void gen_loop(double2* gbuf, unsigned long long* cyc, int len, int spin_waves) {
    __shared__ double e[8192], d[8192];
    __shared__ int stop;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 8192; i += blockDim.x) {
        e[i] = 0.2 + 1e-6 * i;
        d[i] = 0.7 - 1e-6 * i;
    }
    if (tid == 0) stop = 0;
    __syncthreads();
    if (wave == 0) {
        double p = 0.3, c = 1.0, sn = 0.0, acc = 0.0;
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        for (int ib = len - 1; ib >= 0; ib -= 64) {
            const int cnt = min(64, ib + 1);
            const int pos = ib - lane;
            double eL = lane < cnt ? e[pos] : 0.0;
            double dL = lane < cnt ? d[pos] : 0.0;
            asm volatile("" : "+v"(eL), "+v"(dL));
            for (int t = 0; t < cnt; ++t) {
                double ei, di;
                if (V == 2) {   // no readlane: positions' values from arithmetic
                    ei = 0.2 + 1e-6 * (double)t;
                    di = 0.7 - 1e-6 * (double)t;
                } else {
                    ei = __builtin_bit_cast(double, ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(__builtin_bit_cast(unsigned long long, eL) >> 32), t) << 32) |
                                                          (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned long long, eL), t));
                    di = __builtin_bit_cast(double, ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(__builtin_bit_cast(unsigned long long, dL) >> 32), t) << 32) |
                                                          (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned long long, dL), t));
                }
                const double g = c * ei;
                const double h = c * p;
                const double x2 = fma(p, p, ei * ei);
                const double tt = fma(p, di, -(ei * g));
                double inv = __builtin_amdgcn_rsq(x2);
                const double hx = 0.5 * x2;
                inv = fma(inv, fma(-hx, inv * inv, 0.5), inv);
                inv = fma(inv, fma(-hx, inv * inv, 0.5), inv);
                const double r = x2 * inv;
                const double en = sn * r;
                sn = ei * inv;
                c = p * inv;
                p = inv * tt;
                const double dn = h + sn * (c * g + sn * di);
                if (V == 1) {   // no stores
                    acc += en + dn + c + sn;
                } else if (V == 3) {   // global stores only
                    if (lane == 0) {
                        const int i = ib - t;
                        gbuf[(size_t)i * 16] = make_double2(c, sn);
                        gbuf[(size_t)i * 16 + 1] = make_double2(en, dn);
                    }
                } else if (V == 4) {   // LDS stores only
                    if (lane == 0) {
                        const int i = ib - t;
                        e[i + 1] = en;
                        d[i + 1] = dn;
                    }
                } else if (lane == 0) {
                    const int i = ib - t;
                    e[i + 1] = en;
                    d[i + 1] = dn;
                    gbuf[(size_t)i * 16] = make_double2(c, sn);
                }
            }
        }
        if (acc == 12345.0) cyc[2] = 1;
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        if (tid == 0) {
            cyc[0] = t1 - t0;
            stop = 1;
        }
        __threadfence_block();
    } else if (wave <= spin_waves) {
        double a0 = 1.0 + lane, a1 = 2.0, a2 = 3.0, a3 = 4.0, a4 = 5.0, a5 = 6.0, a6 = 7.0, a7 = 8.0;
        while (!__atomic_load_n(&stop, __ATOMIC_RELAXED)) {
            for (int i = 0; i < 256; ++i) {
                a0 = fma(a0, 0.999, 1e-3); a1 = fma(a1, 0.999, 1e-3); a2 = fma(a2, 0.999, 1e-3); a3 = fma(a3, 0.999, 1e-3);
                a4 = fma(a4, 0.999, 1e-3); a5 = fma(a5, 0.999, 1e-3); a6 = fma(a6, 0.999, 1e-3); a7 = fma(a7, 0.999, 1e-3);
            }
        }
        if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 12345.0) cyc[1] = 1;
    }
}


// 6: two-phase generator: the serial chain alone (p, 1/r stashed in lane t by v_cndmask),
// then the per-position outputs vectorised over the block's 64 lanes
__global__ void gen_split(double2* gbuf, unsigned long long* cyc, int len) {
    __shared__ double e[8192], d[8192];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 8192; i += blockDim.x) {
        e[i] = 0.2 + 1e-6 * i;
        d[i] = 0.7 - 1e-6 * i;
    }
    __syncthreads();
    double p = 0.3, c = 1.0, sn = 0.0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int ib = len - 1; ib >= 0; ib -= 64) {
        const int cnt = min(64, ib + 1);
        const int pos = ib - lane;
        double eL = lane < cnt ? e[pos] : 0.0;
        double dL = lane < cnt ? d[pos] : 0.0;
        asm volatile("" : "+v"(eL), "+v"(dL));
        const double e2L = eL * eL;
        const double c0 = c, s0 = sn;
        double pT = 0.0, iT = 0.0;
        for (int t = 0; t < cnt; ++t) {
            const double ei2 = __builtin_bit_cast(double, ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(__builtin_bit_cast(unsigned long long, e2L) >> 32), t) << 32) |
                                                      (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned long long, e2L), t));
            const double di = __builtin_bit_cast(double, ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(__builtin_bit_cast(unsigned long long, dL) >> 32), t) << 32) |
                                                      (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned long long, dL), t));
            const double x2 = fma(p, p, ei2);
            const double tt = fma(p, di, -(c * ei2));
            double inv = __builtin_amdgcn_rsq(x2);
            const double hx = 0.5 * x2;
            inv = fma(inv, fma(-hx, inv * inv, 0.5), inv);
            inv = fma(inv, fma(-hx, inv * inv, 0.5), inv);
            const bool mine = lane == t;
            pT = mine ? p : pT;
            iT = mine ? inv : iT;
            c = p * inv;
            p = inv * tt;
        }
        // phase B: lane t = rotation t of the block
        const double cT = pT * iT, sT = eL * iT;
        const double x2T = fma(pT, pT, e2L);
        const double rT = x2T * iT;
        double cP = __shfl_up(cT, 1), sP = __shfl_up(sT, 1);
        if (lane == 0) {
            cP = c0;
            sP = s0;
        }
        const double g = cP * eL, h = cP * pT;
        const double en = sP * rT;
        const double dn = h + sT * (cT * g + sT * dL);
        if (lane < cnt) {
            e[pos + 1] = en;
            d[pos + 1] = dn;
            gbuf[(size_t)pos * 16] = make_double2(cT, sT);
        }
        sn = __shfl(sT, cnt - 1);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[0] = t1 - t0;
    if (p + c + sn == 12345.0) cyc[2] = 1;
}

__global__ void rsq_err(const double* v, double* r0, double* r1, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = v[i];
    const double a = __builtin_amdgcn_rsq(x);
    const double hx = 0.5 * x;
    const double b = a * fma(-hx, a * a, 1.5);
    r0[i] = a;
    r1[i] = b;
}

int main() {
    std::vector<double> h(128);
    for (int i = 0; i < 128; ++i) h[i] = 0.5 + 0.001 * i;
    double *din, *dout;
    unsigned long long* dc;
    hipMalloc(&din, 128 * 8);
    hipMalloc(&dout, 64 * 8);
    hipMalloc(&dc, 8 * 8);
    hipMemcpy(din, h.data(), 128 * 8, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) chains<<<1, 64>>>(din, dout, dc);
    unsigned long long c[8];
    hipMemcpy(c, dc, 5 * 8, hipMemcpyDeviceToHost);
    const char* nm[5] = {"fma chain", "mul chain", "rsq+add chain", "QL rotation (2 NR, 11 deep)", "QL rotation (1 NR, p'=inv*t)"};
    for (int i = 0; i < 5; ++i) printf("%-32s %8.1f cycles per step\n", nm[i], (double)c[i] / N);

    {
        double2* gb;
        hipMalloc(&gb, 8192 * 16 * 16);
        const int lens[2] = {8000, 8000};
        const int cfg[4][2] = {{64, 0}, {320, 0}, {320, 4}, {512, 7}};
        for (auto& cf : cfg) {
            gen_loop<0><<<1, cf[0]>>>(gb, dc, lens[0], cf[1]);
            hipMemcpy(c, dc, 8, hipMemcpyDeviceToHost);
            printf("gen loop, %3d threads, %d spinning waves: %8.1f cycles per rotation\n", cf[0], cf[1], (double)c[0] / lens[0]);
        }
        const char* vn[5] = {"as in the kernel", "no stores", "no readlane", "global stores only", "LDS stores only"};
        for (int v = 0; v < 5; ++v) {
            if (v == 0) gen_loop<0><<<1, 64>>>(gb, dc, lens[0], 0);
            if (v == 1) gen_loop<1><<<1, 64>>>(gb, dc, lens[0], 0);
            if (v == 2) gen_loop<2><<<1, 64>>>(gb, dc, lens[0], 0);
            if (v == 3) gen_loop<3><<<1, 64>>>(gb, dc, lens[0], 0);
            if (v == 4) gen_loop<4><<<1, 64>>>(gb, dc, lens[0], 0);
            hipMemcpy(c, dc, 8, hipMemcpyDeviceToHost);
            printf("gen loop variant %-20s %8.1f cycles per rotation\n", vn[v], (double)c[0] / lens[0]);
        }
        gen_split<<<1, 64>>>(gb, dc, lens[0]);
        hipMemcpy(c, dc, 8, hipMemcpyDeviceToHost);
        printf("gen two-phase (chain + vector outputs) %8.1f cycles per rotation\n", (double)c[0] / lens[0]);
    }
    const int n = 1 << 20;
    std::vector<double> v(n);
    for (int i = 0; i < n; ++i) v[i] = std::ldexp(1.0 + (double)i / n, (i % 40) - 20);
    double *dv, *d0, *d1;
    hipMalloc(&dv, n * 8);
    hipMalloc(&d0, n * 8);
    hipMalloc(&d1, n * 8);
    hipMemcpy(dv, v.data(), n * 8, hipMemcpyHostToDevice);
    rsq_err<<<n / 256, 256>>>(dv, d0, d1, n);
    std::vector<double> a(n), b(n);
    hipMemcpy(a.data(), d0, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), d1, n * 8, hipMemcpyDeviceToHost);
    double e0 = 0, e1 = 0;
    for (int i = 0; i < n; ++i) {
        const long double ref = 1.0L / std::sqrt((long double)v[i]);
        e0 = std::fmax(e0, (double)std::fabs((a[i] - ref) / ref));
        e1 = std::fmax(e1, (double)std::fabs((b[i] - ref) / ref));
    }
    printf("v_rsq_f64 max rel err %.3e (2^%.1f); after one Newton step %.3e (2^%.1f)\n", e0, std::log2(e0), e1,
           std::log2(e1));
    return 0;
}
