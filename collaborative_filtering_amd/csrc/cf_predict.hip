// cf_predict.hip -- graph-signal rating predictor on precomputed eigenvectors.
//
// Replaces neigh_program::apply of local_calc_precomp.cpp:217-380.  The reference
// partitions by movie and copies the whole user block per rating (:234,242); here the
// test ratings are regrouped BY USER: one 256-thread workgroup walks one user's k
// test movies against that user's k x m eigen block (L2-resident while it works),
// so every block is read from HBM once.  For test movie r of user u:
//
//   C    = the user's items j with w(movie_r -> item_j) > 0.1        (:132,254-265)
//   lim  = first eigenvalue index above w_lim, >= 2                   (:271-282)
//   S    = columns j < lim with some U(C, j) >= 1e-4                  (:284-304)
//   pred = v_S . (U_CS^T U_CS)^-1 U_CS^T (r_C - mean) + mean          (:308-315)
//   mse  = (float)(r - clamp(pred, 1, 5))^2, kk = |C|                 (:318-359)
//
// All arithmetic after the gather is fp64 (the reference's double path), the Gram
// matrix lives in LDS and is solved by LU with partial pivoting (Eigen's
// PartialPivLU class) followed by one wave's back substitution.

#include "cf_internal.h"

namespace {

constexpr int kThreads = 256;
constexpr size_t kMaxLdsGram = 128u * 128u * sizeof(double);

template <typename T>
struct PredArgs {
    const uint32_t* order;
    uint32_t first;
    const uint64_t* item_off;
    const uint32_t* items;
    const float* ratings;
    const int32_t* m;
    const T* evals;
    const uint64_t* evec_off;
    const T* evecs;
    const T* sigtab;
    int sig_mode;
    const float* graph;
    uint64_t n_items;
    float* mse;
    int32_t* kk;
    double* pred;
    double* scratch;       // per-block Gram storage when it does not fit in LDS
    int lmax;              // Gram dimension bound of the launch
    int gram_in_lds;
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Block-wide ordered compaction of flags[0..n): writes the indices with flag set to
// out[] in ascending order and returns their count.  n <= 256.
__device__ int block_compact(bool flag, int idx, int* out, int* s_cnt) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const unsigned long long bal = __ballot(flag);
    if (lane == 0) s_cnt[wave] = __popcll(bal);
    __syncthreads();
    int off = 0;
    for (int w = 0; w < wave; ++w) off += s_cnt[w];
    if (flag) out[off + __popcll(bal & ((1ull << lane) - 1ull))] = idx;
    const int total = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    __syncthreads();
    return total;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void predict_kernel(PredArgs<T> a, uint32_t count) {
    extern __shared__ double dsm[];
    const int lmax = a.lmax;
    double* M_lds = dsm;                                   // lmax*lmax (if gram_in_lds)
    double* tv = dsm + (a.gram_in_lds ? (size_t)lmax * lmax : 0);
    double* s_misc = tv + lmax;                            // [0] mean
    uint32_t* s_item = reinterpret_cast<uint32_t*>(s_misc + 4);
    float* s_rat = reinterpret_cast<float*>(s_item + CF_MAX_K);
    int* s_conn = reinterpret_cast<int*>(s_rat + CF_MAX_K);
    int* s_keep = s_conn + CF_MAX_K;
    int* s_rowp = s_keep + CF_MAX_K;
    int* s_cnt = s_rowp + CF_MAX_K;                        // [0..3] compaction, [4] lim, [5] piv
    double* M = a.gram_in_lds ? M_lds : a.scratch + (size_t)blockIdx.x * lmax * lmax;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    for (uint32_t ub = blockIdx.x; ub < count; ub += gridDim.x) {
        const uint32_t u = a.order[a.first + ub];
        const uint64_t base = a.item_off[u];
        const int k = (int)(a.item_off[u + 1] - base);
        const int m = a.m[u];
        const T* U = a.evecs + a.evec_off[u];
        const T* ev = a.evals + base;
        __syncthreads();
        for (int i = tid; i < k; i += kThreads) {
            s_item[i] = a.items[base + i];
            s_rat[i] = a.ratings[base + i];
        }
        __syncthreads();

        for (int r = 0; r < k; ++r) {
            // --- connected set C (ascending row order) ---
            const float* nrow = a.graph + (size_t)s_item[r] * a.n_items;
            const bool conn = tid < k && (double)nrow[s_item[tid < k ? tid : 0]] > 0.1;
            const int c = block_compact(conn, tid, s_conn, s_cnt);

            // --- lim from w_lim ---
            if (tid == 0) {
                const double w_lim = (double)a.sigtab[a.sig_mode == CF_SIGS_COMPAT ? (uint64_t)r : base + r];
                int lim = 0;
                for (; lim < m; ++lim) {
                    const double e = lim < k ? (double)ev[lim] : 0.0;
                    if (e > w_lim) break;
                }
                if (lim < 2) lim = 2;
                if (lim > m) lim = m;
                s_cnt[4] = lim;
            }
            __syncthreads();
            const int lim = s_cnt[4];

            // --- zero-column filter (signed, >= 1e-4) ---
            bool keep = false;
            if (tid < lim) {
                for (int i = 0; i < c; ++i)
                    if ((double)U[(size_t)s_conn[i] * m + tid] >= 0.0001) {
                        keep = true;
                        break;
                    }
            }
            const int L = block_compact(keep, tid, s_keep, s_cnt);

            // --- centred ratings mean ---
            if (wave == 0) {
                double sum = 0.0;
                for (int i = lane; i < c; i += 64) sum += (double)s_rat[s_conn[i]];
                sum = wave_sum(sum);
                if (lane == 0) s_misc[0] = sum / (double)c;
            }
            __syncthreads();
            const double mean = s_misc[0];

            // --- Gram M = G^T G and rhs t = G^T (r - mean), G = U(C, S) ---
            for (int e = tid; e < L * L; e += kThreads) {
                const int ia = e / L, ib = e - ia * L;
                if (ib < ia) continue;
                const int ca = s_keep[ia], cb = s_keep[ib];
                double acc = 0.0;
                for (int i = 0; i < c; ++i) {
                    const T* row = U + (size_t)s_conn[i] * m;
                    acc = fma((double)row[ca], (double)row[cb], acc);
                }
                M[ia * L + ib] = acc;
                M[ib * L + ia] = acc;
            }
            for (int ia = tid; ia < L; ia += kThreads) {
                const int ca = s_keep[ia];
                double acc = 0.0;
                for (int i = 0; i < c; ++i)
                    acc = fma((double)U[(size_t)s_conn[i] * m + ca], (double)s_rat[s_conn[i]] - mean, acc);
                tv[ia] = acc;
                s_rowp[ia] = ia;
            }
            __syncthreads();

            // --- LU with partial pivoting (row permutation kept in s_rowp) ---
            for (int kc = 0; kc < L; ++kc) {
                if (wave == 0) {
                    double best = -1.0;
                    int bi = 0x7fffffff;
                    for (int i = kc + lane; i < L; i += 64) {
                        const double v = fabs(M[s_rowp[i] * L + kc]);
                        if (v > best) {
                            best = v;
                            bi = i;
                        }
                    }
#pragma unroll
                    for (int off = 32; off >= 1; off >>= 1) {
                        const double ob = __shfl_xor(best, off);
                        const int oi = __shfl_xor(bi, off);
                        if (ob > best || (ob == best && oi < bi)) {
                            best = ob;
                            bi = oi;
                        }
                    }
                    if (lane == 0) {
                        if (best > 0.0 && bi != kc) {
                            const int t = s_rowp[kc];
                            s_rowp[kc] = s_rowp[bi];
                            s_rowp[bi] = t;
                        }
                        s_cnt[5] = best > 0.0;
                    }
                }
                __syncthreads();
                if (s_cnt[5]) {
                    const int pr = s_rowp[kc];
                    const double pinv = 1.0 / M[pr * L + kc];
                    const int rows = L - kc - 1;
                    const int cols = L - kc;  // column kc carries the multiplier
                    for (int e = tid; e < rows * cols; e += kThreads) {
                        const int ri = e / cols;
                        const int cj = e - ri * cols;
                        const int row = s_rowp[kc + 1 + ri];
                        const double l = M[row * L + kc] * pinv;
                        if (cj == 0) {
                            tv[row] -= l * tv[pr];
                        } else {
                            M[row * L + kc + cj] -= l * M[pr * L + kc + cj];
                        }
                    }
                }
                __syncthreads();
            }

            // --- back substitution (one wave) and prediction ---
            if (wave == 0) {
                // x_j lives in lane (j & 63), slot (j >> 6): L <= CF_MAX_K = 3 * 64.
                double x0 = 0.0, x1 = 0.0, x2 = 0.0;
                for (int i = L - 1; i >= 0; --i) {
                    const int row = s_rowp[i];
                    const double* Mr = M + (size_t)row * L;
                    double s = 0.0;
                    if (lane > i && lane < L) s = fma(Mr[lane], x0, s);
                    if (lane + 64 > i && lane + 64 < L) s = fma(Mr[lane + 64], x1, s);
                    if (lane + 128 > i && lane + 128 < L) s = fma(Mr[lane + 128], x2, s);
                    s = wave_sum(s);
                    const double xi = (tv[row] - s) / Mr[i];
                    if (lane == (i & 63)) {
                        if (i < 64) x0 = xi;
                        else if (i < 128) x1 = xi;
                        else x2 = xi;
                    }
                }
                double dot = 0.0;
                const T* vrow = U + (size_t)r * m;
                if (lane < L) dot = fma((double)vrow[s_keep[lane]], x0, dot);
                if (lane + 64 < L) dot = fma((double)vrow[s_keep[lane + 64]], x1, dot);
                if (lane + 128 < L) dot = fma((double)vrow[s_keep[lane + 128]], x2, dot);
                dot = wave_sum(dot);
                if (lane == 0) {
                    double pred = dot + mean;
                    if (pred > 5) pred = 5;
                    if (pred < 1) pred = 1;
                    const double d = (double)s_rat[r] - pred;
                    a.mse[base + r] = (float)(d * d);
                    a.kk[base + r] = c;
                    if (a.pred) a.pred[base + r] = pred;
                }
            }
            __syncthreads();
        }
    }
}

template <typename T>
int launch_predict_bucket(cf_ctx* ctx, PredArgs<T> args, uint32_t count, int lmax,
                          double** scratch, size_t* scratch_bytes, hipStream_t stream) {
    const size_t gram = (size_t)lmax * lmax * sizeof(double);
    args.lmax = lmax;
    args.gram_in_lds = gram <= kMaxLdsGram;
    const size_t lds = (args.gram_in_lds ? gram : 0) + lmax * sizeof(double) + 4 * sizeof(double) +
                       CF_MAX_K * (sizeof(uint32_t) + sizeof(float) + 3 * sizeof(int)) + 8 * sizeof(int);
    int blocks = (int)std::min<uint32_t>(count, 2048u);
    if (!args.gram_in_lds) {
        const size_t need = (size_t)blocks * gram;
        if (need > *scratch_bytes) {
            if (*scratch) (void)hipFree(*scratch);
            *scratch = nullptr;
            *scratch_bytes = 0;
            CF_HIP_CHECK(ctx, hipMalloc(scratch, need));
            *scratch_bytes = need;
        }
        args.scratch = *scratch;
    }
    CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)predict_kernel<T>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(predict_kernel<T>, dim3(blocks), dim3(kThreads), lds, stream, args, count);
    CF_HIP_CHECK(ctx, hipGetLastError());
    return CF_OK;
}

}  // namespace

template <typename T>
int cf_launch_predict(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                      const uint32_t* d_items, const float* d_ratings, const int32_t* d_m,
                      const T* d_evals, const uint64_t* d_evec_off, const T* d_evecs,
                      const T* d_sigtab, int sig_mode, float* d_mse, int32_t* d_kk,
                      double* d_pred, hipStream_t stream) {
    PredArgs<T> args{};
    args.order = plan->d_order;
    args.item_off = d_item_off;
    args.items = d_items;
    args.ratings = d_ratings;
    args.m = d_m;
    args.evals = d_evals;
    args.evec_off = d_evec_off;
    args.evecs = d_evecs;
    args.sigtab = d_sigtab;
    args.sig_mode = sig_mode;
    args.graph = ctx->d_graph;
    args.n_items = ctx->n_items;
    args.mse = d_mse;
    args.kk = d_kk;
    args.pred = d_pred;
    double* scratch = nullptr;
    size_t scratch_bytes = 0;
    int rc = CF_OK;
    for (const cf_bucket& b : plan->buckets) {
        if (b.count == 0) continue;
        args.first = b.first;
        const int lmax = std::max<int>(2, 16 * b.emax);
        rc = launch_predict_bucket<T>(ctx, args, b.count, lmax, &scratch, &scratch_bytes, stream);
        if (rc != CF_OK) break;
    }
    if (scratch) {
        (void)hipStreamSynchronize(stream);
        (void)hipFree(scratch);
    }
    return rc;
}

template int cf_launch_predict<float>(cf_ctx*, const cf_plan*, const uint64_t*, const uint32_t*,
                                      const float*, const int32_t*, const float*, const uint64_t*,
                                      const float*, const float*, int, float*, int32_t*, double*,
                                      hipStream_t);
template int cf_launch_predict<double>(cf_ctx*, const cf_plan*, const uint64_t*, const uint32_t*,
                                       const float*, const int32_t*, const double*,
                                       const uint64_t*, const double*, const double*, int, float*,
                                       int32_t*, double*, hipStream_t);
