// cf_eigen.hip -- batched per-user normalized-Laplacian eigendecomposition on gfx950.
//
// Replaces compute_eigens() of precompute_local_threads.cpp:100-213 (same math as
// precompute_local.cpp:165-281).  One 256-thread workgroup owns one user:
//
//   1. gather W_u(i,j) = graph[item_i][item_j] from the HBM-resident dense graph
//      straight into LDS (k x k fp32, column-major, odd leading dimension);
//   2. d_i = row sum (fp64) with the 0 -> 1 rule (:129-141), s_i = sqrt(1/d_i)
//      (:149-153), L2(i,j) = (s_i * L(i,j)) * s_j (:155), sig_min_i from the FULL
//      row (:169-177);
//   3. B = sym_lower(L2) + I in place.  Eigen reads only the lower triangle of L2
//      (:164); the shift makes B positive definite (spectrum of L2 is in [0,2]) so
//      its singular values are its eigenvalues and the rotated columns of B are the
//      eigenvectors scaled by (lambda + 1);
//   4. one-sided (Hestenes) Jacobi sweeps in LDS: each step of a round-robin
//      tournament rotates k/2 disjoint column pairs; a pair is owned by one DPP row
//      (16 lanes), whose three dot products are reduced with DPP row ops;
//   5. lambda_j = ||b_j|| / ||v_j|| - 1 (||v_j|| tracks the fp32 rotation drift),
//      rank sort ascending, lim (:184-191), write the k x m row-major block, sigs,
//      evals and m.
//
// No MFMA: the matrices are tiny and the work is rotation-shaped, not GEMM-shaped.

#include "cf_internal.h"

namespace {

constexpr int kThreads = 256;
constexpr int kGroup = 16;                   // lanes per column pair = one DPP row
constexpr int kGroups = kThreads / kGroup;   // column pairs in flight per workgroup

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// All-reduce (sum) over the 16 lanes of a DPP row; every lane receives the total.
__device__ __forceinline__ float row16_sum(float x) {
    x += dpp_mov<0xB1>(x);   // quad_perm [1,0,3,2]
    x += dpp_mov<0x4E>(x);   // quad_perm [2,3,0,1]
    x += dpp_mov<0x141>(x);  // row_half_mirror
    x += dpp_mov<0x140>(x);  // row_mirror
    return x;
}

struct EigenArgs {
    const uint32_t* order;
    uint32_t first;
    const uint64_t* item_off;
    const uint32_t* items;
    const float* graph;
    uint64_t n_items;
    const uint64_t* evec_off;
    int32_t* m_out;
    float* sigs;
    float* evals;
    float* evecs;
    float tol_scale;
    int max_sweeps;
};

template <int EMAX>
struct EigenLds {
    static constexpr int NR = kGroup * EMAX;  // padded row count (>= k)
    static constexpr int LD = NR + 1;         // odd: column-parallel LDS access is conflict-free
    static constexpr size_t bytes() {
        return sizeof(float) * (size_t)NR * LD     // B
               + sizeof(uint32_t) * NR             // items
               + sizeof(float) * NR * 5            // s, l2 diagonal, sig, mu, scale drift
               + sizeof(int) * NR                  // perm
               + sizeof(int) * 4;                  // flags
    }
};

template <int EMAX>
__global__ __launch_bounds__(kThreads) void eigen_kernel(EigenArgs a) {
    using Lds = EigenLds<EMAX>;
    constexpr int NR = Lds::NR;
    constexpr int LD = Lds::LD;
    extern __shared__ float smem[];
    float* B = smem;
    uint32_t* s_item = reinterpret_cast<uint32_t*>(B + (size_t)NR * LD);
    float* s_s = reinterpret_cast<float*>(s_item + NR);
    float* s_l2d = s_s + NR;
    float* s_sig = s_l2d + NR;
    float* s_mu = s_sig + NR;
    float* s_dev = s_mu + NR;   // d_j = ||v_j||^2 - 1 of the implicit rotation product
    int* s_perm = reinterpret_cast<int*>(s_dev + NR);
    int* s_flag = s_perm + NR;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const uint32_t u = a.order[a.first + blockIdx.x];
    const uint64_t base = a.item_off[u];
    const int k = (int)(a.item_off[u + 1] - base);
    if (k <= 0 || k > NR) {
        if (tid == 0) a.m_out[u] = (k <= 0) ? 0 : -1;
        return;
    }

    // ---- 1. gather W_u (column-major, B[j*LD + i] = W(i,j)) ----------------------
    for (int i = tid; i < k; i += kThreads) s_item[i] = a.items[base + i];
    for (int idx = tid; idx < NR * LD; idx += kThreads) B[idx] = 0.0f;
    __syncthreads();
    for (int i = wave; i < k; i += kThreads / 64) {
        const float* row = a.graph + (size_t)s_item[i] * a.n_items;
        for (int j = lane; j < k; j += 64) B[j * LD + i] = row[s_item[j]];
    }
    __syncthreads();

    // ---- 2. degrees, D^-1/2, diagonal of L2, sig_min -------------------------------
    for (int i = tid; i < k; i += kThreads) {
        double d = 0.0;
        for (int j = 0; j < k; ++j) d += (double)B[j * LD + i];
        if (d == 0.0) d = 1.0;                      // (:137-140)
        const double s = sqrt(1.0 / d);             // inverse, then sqrt (:149-153)
        s_s[i] = (float)s;
        s_l2d[i] = (float)((s * (d - (double)B[i * LD + i])) * s);
    }
    __syncthreads();
    for (int i = tid; i < k; i += kThreads) {
        const float si = s_s[i];
        float acc = 0.0f;
        for (int j = 0; j < k; ++j) {
            const float l2 = (j == i) ? s_l2d[i] : -(si * B[j * LD + i]) * s_s[j];
            acc = fmaf(l2, l2, acc);
        }
        s_sig[i] = sqrtf(acc);                      // (:172-176)
    }
    __syncthreads();

    // ---- 3. B = sym_lower(L2) + I, in place ------------------------------------------
    for (int i = wave; i < k; i += kThreads / 64) {
        const float si = s_s[i];
        for (int j = lane; j < i; j += 64) {
            const float v = -(si * B[j * LD + i]) * s_s[j];
            B[j * LD + i] = v;   // (i,j), lower
            B[i * LD + j] = v;   // (j,i), mirrored
        }
        if (lane == 0) B[i * LD + i] = s_l2d[i] + 1.0f;
    }
    for (int i = tid; i < k; i += kThreads) s_dev[i] = 0.0f;
    if (tid == 0) s_flag[0] = 0;
    __syncthreads();

    // ---- 4. one-sided Jacobi --------------------------------------------------------
    const int n = (k + 1) & ~1;          // players in the round-robin tournament
    const int npairs = n >> 1;
    const int g = tid / kGroup;
    const int lig = tid % kGroup;
    const float tol = a.tol_scale * sqrtf((float)k) * 2.384185791015625e-07f;  // sqrt(k) * 2^-22
    for (int sweep = 0; sweep < a.max_sweeps && k > 1; ++sweep) {
        for (int step = 0; step < n - 1; ++step) {
            for (int pi = g; pi < npairs; pi += kGroups) {
                int p, q;
                if (pi == 0) {
                    p = n - 1;
                    q = step;
                } else {
                    p = (step + pi) % (n - 1);
                    q = (step - pi + n - 1) % (n - 1);
                }
                if (p >= k || q >= k) continue;
                float* bp = B + p * LD + lig;
                float* bq = B + q * LD + lig;
                float xp[EMAX], xq[EMAX];
                float al = 0.f, be = 0.f, ga = 0.f;
#pragma unroll
                for (int t = 0; t < EMAX; ++t) {
                    xp[t] = bp[kGroup * t];
                    xq[t] = bq[kGroup * t];
                    al = fmaf(xp[t], xp[t], al);
                    be = fmaf(xq[t], xq[t], be);
                    ga = fmaf(xp[t], xq[t], ga);
                }
                al = row16_sum(al);
                be = row16_sum(be);
                ga = row16_sum(ga);
                if (fabsf(ga) > tol * sqrtf(al * be)) {
                    const float zeta = (be - al) / (2.0f * ga);
                    const float t = copysignf(1.0f, zeta) / (fabsf(zeta) + sqrtf(1.0f + zeta * zeta));
                    const float c = 1.0f / sqrtf(1.0f + t * t);
                    const float s = c * t;
#pragma unroll
                    for (int e = 0; e < EMAX; ++e) {
                        bp[kGroup * e] = c * xp[e] - s * xq[e];
                        bq[kGroup * e] = s * xp[e] + c * xq[e];
                    }
                    // fp32 (c, s) are not exactly orthonormal: c^2 + s^2 = 1 + delta.
                    // Track each column's accumulated scale so lambda is not biased by
                    // ~k * sweeps * delta (2.4e-5 at k = 128 without this).
                    const float delta = fmaf(s, s, fmaf(c, c, -1.0f));
                    const float dp = s_dev[p], dq = s_dev[q];
                    const float cc = c * c, ss = s * s;
                    if (lig == 0) {
                        s_dev[p] = delta + fmaf(cc, dp, ss * dq);
                        s_dev[q] = delta + fmaf(ss, dp, cc * dq);
                        s_flag[0] = 1;
                    }
                }
            }
            __syncthreads();
        }
        const int rotated = s_flag[0];
        __syncthreads();
        if (!rotated) break;
        if (tid == 0) s_flag[0] = 0;
        __syncthreads();
    }

    // ---- 5. eigenvalues, ordering, lim, output ----------------------------------------
    // ||b_j|| accumulated in fp64: a k-term fp32 sum would cost ~k ulps (3e-5 at k=192).
    for (int j = tid; j < k; j += kThreads) {
        double acc = 0.0;
        for (int i = 0; i < k; ++i) {
            const double v = (double)B[j * LD + i];
            acc = fma(v, v, acc);
        }
        const double nrm = sqrt(acc);
        s_mu[j] = (float)(nrm / sqrt(1.0 + (double)s_dev[j]));   // lambda_j + 1
        s_s[j] = (float)(1.0 / nrm);                             // unit-normalises v_j
    }
    __syncthreads();
    for (int j = tid; j < k; j += kThreads) {
        const float mj = s_mu[j];
        int rank = 0;
        for (int i = 0; i < k; ++i) {
            const float mi = s_mu[i];
            rank += (mi < mj) || (mi == mj && i < j);
        }
        s_perm[rank] = j;
    }
    __syncthreads();
    if (tid == 0) {
        float smm = 0.0f;
        for (int i = 0; i < k; ++i)
            if (smm < s_sig[i]) smm = s_sig[i];
        smm = (float)((double)smm + 0.01);          // (:182)
        int lim = 0;
        for (; lim < k; ++lim)
            if ((double)(s_mu[s_perm[lim]] - 1.0f) > (double)smm) break;  // (:186-188)
        if (lim < 2) lim = 2;                        // (:190-191)
        s_flag[1] = lim;
        a.m_out[u] = lim;
    }
    __syncthreads();
    const int m = s_flag[1];
    for (int i = tid; i < k; i += kThreads) a.sigs[base + i] = (float)((double)s_sig[i] + 0.01);
    for (int r = tid; r < m && r < k; r += kThreads) a.evals[base + r] = s_mu[s_perm[r]] - 1.0f;
    float* out = a.evecs + a.evec_off[u];
    for (int idx = tid; idx < k * m; idx += kThreads) {
        const int i = idx / m;
        const int r = idx - i * m;
        float v = 0.0f;
        if (r < k) {
            const int j = s_perm[r];
            v = B[j * LD + i] * s_s[j];
        }
        out[idx] = v;
    }
}

template <int EMAX>
int launch_bucket(cf_ctx* ctx, const EigenArgs& args, uint32_t count, hipStream_t stream) {
    const size_t lds = EigenLds<EMAX>::bytes();
    static bool configured = false;
    if (!configured) {
        CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)eigen_kernel<EMAX>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        configured = true;
    }
    hipLaunchKernelGGL(eigen_kernel<EMAX>, dim3(count), dim3(kThreads), lds, stream, args);
    CF_HIP_CHECK(ctx, hipGetLastError());
    return CF_OK;
}

}  // namespace

int cf_launch_eigen(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                    const uint32_t* d_items, const uint64_t* d_evec_off, int32_t* d_m,
                    float* d_sigs, float* d_evals, float* d_evecs, hipStream_t stream) {
    EigenArgs args{};
    args.order = plan->d_order;
    args.item_off = d_item_off;
    args.items = d_items;
    args.graph = ctx->d_graph;
    args.n_items = ctx->n_items;
    args.evec_off = d_evec_off;
    args.m_out = d_m;
    args.sigs = d_sigs;
    args.evals = d_evals;
    args.evecs = d_evecs;
    args.tol_scale = ctx->tol_scale;
    args.max_sweeps = ctx->max_sweeps;
    for (const cf_bucket& b : plan->buckets) {
        if (b.count == 0) continue;
        args.first = b.first;
        int rc;
        switch (b.emax) {
            case 1: rc = launch_bucket<1>(ctx, args, b.count, stream); break;
            case 2: rc = launch_bucket<2>(ctx, args, b.count, stream); break;
            case 3: rc = launch_bucket<3>(ctx, args, b.count, stream); break;
            case 4: rc = launch_bucket<4>(ctx, args, b.count, stream); break;
            case 5: rc = launch_bucket<5>(ctx, args, b.count, stream); break;
            case 6: rc = launch_bucket<6>(ctx, args, b.count, stream); break;
            case 7: rc = launch_bucket<7>(ctx, args, b.count, stream); break;
            case 8: rc = launch_bucket<8>(ctx, args, b.count, stream); break;
            case 9: rc = launch_bucket<9>(ctx, args, b.count, stream); break;
            case 10: rc = launch_bucket<10>(ctx, args, b.count, stream); break;
            case 11: rc = launch_bucket<11>(ctx, args, b.count, stream); break;
            case 12: rc = launch_bucket<12>(ctx, args, b.count, stream); break;
            default: return cf_set_error(ctx, CF_ERANGE, "eigen bucket out of range (k > 192)");
        }
        if (rc != CF_OK) return rc;
    }
    return CF_OK;
}
