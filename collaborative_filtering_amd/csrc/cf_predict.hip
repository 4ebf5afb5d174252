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
// All arithmetic after the gather is fp64 (the reference's double path).  The
// reference forms mm = U_CS^T U_CS and multiplies by its PartialPivLU inverse.  Here
// the symmetric Gram matrix is factored M = L D L^T (blocked, right-looking, packed
// lower triangle in LDS), bordered by t^T and v^T so the factorisation itself yields
// L^-1 t and L^-1 v and pred = sum_j (L^-1 v)_j (L^-1 t)_j / D_j + mean.  For a
// well-conditioned M this agrees with the inverse-based formula to cond(M) * eps.
// Like Gaussian elimination (and unlike Cholesky) LDL^T carries on through negative
// pivots, so a numerically indefinite, near-singular M gives the same kind of
// finite, clamped garbage as the reference instead of a NaN.

#include "cf_internal.h"

namespace {

constexpr int kThreads = 256;

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
    unsigned long long* phase_cycles;  // diagnostics: per-phase s_memtime totals (or null)
    int lmax;              // Gram dimension bound of the launch
    double* gbar;          // per-block scratch: Gbar = U^T U (lmax x lmax, full), fp64
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

// Packed lower-triangular index (row-major rows of increasing length).
__device__ __forceinline__ int tri(int i, int j) { return (i * (i + 1)) / 2 + j; }

#define WAVE_SYNC()                                              \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
    } while (0)

constexpr int kNB = 16;   // Cholesky panel width

template <typename T>
__global__ __launch_bounds__(kThreads) void predict_kernel(PredArgs<T> a, uint32_t count) {
    extern __shared__ double dsm[];
    const int lmax = a.lmax;
    // A: packed lower triangle of the bordered matrix [[M, .], [t^T, .], [v^T, .]],
    //    (lmax + 2) rows; rows L and L+1 hold t and v and become y = L^-1 t, z = L^-1 v.
    double* A = dsm;
    double* s_misc = A + (size_t)(lmax + 2) * (lmax + 3) / 2;   // [0] mean, [1] pred sum
    uint32_t* s_item = reinterpret_cast<uint32_t*>(s_misc + 4);
    float* s_rat = reinterpret_cast<float*>(s_item + CF_MAX_K);
    int* s_conn = reinterpret_cast<int*>(s_rat + CF_MAX_K);
    int* s_keep = s_conn + CF_MAX_K;
    int* s_nconn = s_keep + CF_MAX_K;                      // rows NOT in C (complement)
    int* s_cnt = s_nconn + CF_MAX_K;                       // [0..3] compaction, [4] lim
    double* Gb = a.gbar + (size_t)blockIdx.x * lmax * lmax;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    // Diagnostic phase stamps (thread 0 only; no effect on outputs).
    unsigned long long ph_acc[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long ph_t = 0;
#define PHASE_STAMP(ph)                                                   \
    if (a.phase_cycles && tid == 0) {                                     \
        const unsigned long long now = __builtin_amdgcn_s_memtime();      \
        if ((ph) >= 0) ph_acc[(ph) < 0 ? 0 : (ph)] += now - ph_t;         \
        ph_t = now;                                                       \
    }

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
        // Gbar = U^T U over all k rows (fp64, full m x m), once per user: a prediction
        // whose connected set C covers most rows forms its Gram matrix as
        // Gbar_SS - sum_{i not in C} u_i u_i^T, which is the same sum with O(eps)
        // cancellation error instead of c * L^2 work.
        {
            const int nt4 = (m + 3) >> 2;
            const int ntile = nt4 * (nt4 + 1) / 2;
            for (int tix = tid; tix < ntile; tix += kThreads) {
                int ta = 0, rem = tix;
                while (rem > ta) {
                    rem -= ta + 1;
                    ++ta;
                }
                const int tb = rem;
                double acc[4][4];
#pragma unroll
                for (int x = 0; x < 4; ++x)
#pragma unroll
                    for (int y = 0; y < 4; ++y) acc[x][y] = 0.0;
                const int a0 = min(4 * ta, m - 4 > 0 ? m - 4 : 0), b0 = 4 * tb;
                for (int i = 0; i < k; ++i) {
                    const T* row = U + (size_t)i * m;
                    double va[4], vb[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        va[q] = (double)row[min(4 * ta + q, m - 1)];
                        vb[q] = (double)row[min(b0 + q, m - 1)];
                    }
#pragma unroll
                    for (int x = 0; x < 4; ++x)
#pragma unroll
                        for (int y = 0; y < 4; ++y) acc[x][y] = fma(va[x], vb[y], acc[x][y]);
                }
                (void)a0;
#pragma unroll
                for (int x = 0; x < 4; ++x)
#pragma unroll
                    for (int y = 0; y < 4; ++y) {
                        const int ia = 4 * ta + x, ib = b0 + y;
                        if (ia < m && ib < m && ib <= ia) {
                            Gb[(size_t)ia * lmax + ib] = acc[x][y];
                            Gb[(size_t)ib * lmax + ia] = acc[x][y];
                        }
                    }
            }
        }
        __syncthreads();

        for (int r = 0; r < k; ++r) {
            PHASE_STAMP(-1);
            // --- connected set C: the user's items that are out-neighbours of movie r (:254-265)
            const float* nrow = a.graph + (size_t)s_item[r] * a.n_items;
            const bool conn = tid < k && (double)nrow[s_item[tid < k ? tid : 0]] > 0.1;
            const int c = block_compact(conn, tid, s_conn, s_cnt);
            const int nc = block_compact(tid < k && !conn, tid, s_nconn, s_cnt);
            const bool use_complement = nc < c;
            PHASE_STAMP(0);

            // --- lim = first eigenvalue index above w_lim, >= 2 (:271-282) ---
            {
                const double w_lim =
                    (double)a.sigtab[a.sig_mode == CF_SIGS_COMPAT ? (uint64_t)r : base + r];
                const bool above = tid < m && (double)(tid < k ? ev[tid] : (T)0) > w_lim;
                const unsigned long long bal = __ballot(above);
                if (lane == 0) s_cnt[wave] = bal ? (__ffsll((long long)bal) - 1 + 64 * wave) : 0x7fffffff;
                __syncthreads();
                int lim = min(min(s_cnt[0], s_cnt[1]), min(s_cnt[2], s_cnt[3]));
                lim = min(lim, m);
                if (lim < 2) lim = 2;
                if (lim > m) lim = m;
                __syncthreads();
                s_cnt[4] = lim;   // every thread writes the same value
            }
            const int lim = s_cnt[4];

            // --- zero-column filter: keep column j < lim iff some U(C, j) >= 1e-4 (:284-304)
            bool keep = false;
            if (tid < lim) {
                for (int i = 0; i < c; ++i)
                    if ((double)U[(size_t)s_conn[i] * m + tid] >= 0.0001) {
                        keep = true;
                        break;
                    }
            }
            const int L = block_compact(keep, tid, s_keep, s_cnt);
            PHASE_STAMP(1);

            // --- mean of the connected ratings (:311) ---
            if (wave == 0) {
                double sum = 0.0;
                for (int i = lane; i < c; i += 64) sum += (double)s_rat[s_conn[i]];
                sum = wave_sum(sum);
                if (lane == 0) s_misc[0] = sum / (double)c;
            }
            __syncthreads();
            const double mean = s_misc[0];
            PHASE_STAMP(2);

            // --- bordered Gram: A[i][j] = (G^T G)_ij (j <= i < L), A[L][j] = t_j, A[L+1][j] = v_j
            // 4x4 register tiles of the lower triangle, 8 independent loads per row of G.
            {
                const int nt4 = (L + 3) >> 2;
                const int ntile = nt4 * (nt4 + 1) / 2;
                for (int tix = tid; tix < ntile; tix += kThreads) {
                    int ta = 0, rem = tix;   // tix -> (ta >= tb), row-major over the lower triangle
                    while (rem > ta) {
                        rem -= ta + 1;
                        ++ta;
                    }
                    const int tb = rem;
                    int ca[4], cb[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int ia = 4 * ta + q, ib = 4 * tb + q;
                        ca[q] = s_keep[ia < L ? ia : L - 1];
                        cb[q] = s_keep[ib < L ? ib : L - 1];
                    }
                    double acc[4][4];
#pragma unroll
                    for (int x = 0; x < 4; ++x)
#pragma unroll
                        for (int y = 0; y < 4; ++y) acc[x][y] = 0.0;
                    const int nrows = use_complement ? nc : c;
                    const int* rows = use_complement ? s_nconn : s_conn;
                    int i = 0;
                    for (; i + 1 < nrows; i += 2) {   // two rows in flight: 16 independent loads
                        const T* row0 = U + (size_t)rows[i] * m;
                        const T* row1 = U + (size_t)rows[i + 1] * m;
                        double va0[4], vb0[4], va1[4], vb1[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            va0[q] = (double)row0[ca[q]];
                            vb0[q] = (double)row0[cb[q]];
                            va1[q] = (double)row1[ca[q]];
                            vb1[q] = (double)row1[cb[q]];
                        }
#pragma unroll
                        for (int x = 0; x < 4; ++x)
#pragma unroll
                            for (int y = 0; y < 4; ++y)
                                acc[x][y] = fma(va1[x], vb1[y], fma(va0[x], vb0[y], acc[x][y]));
                    }
                    for (; i < nrows; ++i) {
                        const T* row = U + (size_t)rows[i] * m;
                        double va[4], vb[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            va[q] = (double)row[ca[q]];
                            vb[q] = (double)row[cb[q]];
                        }
#pragma unroll
                        for (int x = 0; x < 4; ++x)
#pragma unroll
                            for (int y = 0; y < 4; ++y) acc[x][y] = fma(va[x], vb[y], acc[x][y]);
                    }
#pragma unroll
                    for (int x = 0; x < 4; ++x)
#pragma unroll
                        for (int y = 0; y < 4; ++y) {
                            const int ia = 4 * ta + x, ib = 4 * tb + y;
                            if (ia < L && ib <= ia)
                                A[tri(ia, ib)] = use_complement
                                                     ? Gb[(size_t)ca[x] * lmax + cb[y]] - acc[x][y]
                                                     : acc[x][y];
                        }
                }
                // t = G^T (r - mean): 4 lanes per column, each a strided quarter of C,
                // combined with two DPP-free shuffles; v = U(r, S).
                for (int e = tid; e < 4 * L; e += kThreads) {
                    const int j = e >> 2, part = e & 3;
                    const int cj = s_keep[j];
                    double acc0 = 0.0, acc1 = 0.0;
                    int i = part;
                    for (; i + 4 < c; i += 8) {
                        const int r0 = s_conn[i], r1 = s_conn[i + 4];
                        acc0 = fma((double)U[(size_t)r0 * m + cj], (double)s_rat[r0] - mean, acc0);
                        acc1 = fma((double)U[(size_t)r1 * m + cj], (double)s_rat[r1] - mean, acc1);
                    }
                    for (; i < c; i += 4) {
                        const int r0 = s_conn[i];
                        acc0 = fma((double)U[(size_t)r0 * m + cj], (double)s_rat[r0] - mean, acc0);
                    }
                    double acc = acc0 + acc1;
                    acc += __shfl_xor(acc, 1);
                    acc += __shfl_xor(acc, 2);
                    if (part == 0) {
                        A[tri(L, j)] = acc;
                        A[tri(L + 1, j)] = (double)U[(size_t)r * m + cj];
                    }
                }
            }
            __syncthreads();
            PHASE_STAMP(3);

            // --- blocked right-looking LDL^T of M, carrying the two border rows ---
            for (int kb = 0; kb < L; kb += kNB) {
                const int b = min(kNB, L - kb);
                // (1) diagonal block, unblocked LDL^T, in wave 0's registers: lane i < b
                //     holds row kb + i; column j is broadcast by shuffles.  D_j stays on
                //     the diagonal, L_ij (unit lower) below it.
                if (wave == 0) {
                    double rowv[kNB];
                    const int i = lane;
                    const bool live = i < b;
#pragma unroll
                    for (int q = 0; q < kNB; ++q)
                        rowv[q] = (live && q <= i) ? A[tri(kb + i, kb + q)] : 0.0;
#pragma unroll
                    for (int j = 0; j < kNB; ++j) {
                        if (j < b) {
                            const double dj = __shfl(rowv[j], j);
                            const double w = (i > j) ? rowv[j] : 0.0;   // unscaled a_ij
                            const double lij = w / dj;
                            // a_iq -= L_ij * a_qj, j < q <= i
#pragma unroll
                            for (int q = j + 1; q < kNB; ++q) {
                                const double wq = __shfl(w, q);
                                if (q <= i) rowv[q] = fma(-lij, wq, rowv[q]);
                            }
                            if (i > j) rowv[j] = lij;
                        }
                    }
#pragma unroll
                    for (int q = 0; q < kNB; ++q)
                        if (live && q <= i) A[tri(kb + i, kb + q)] = rowv[q];
                }
                __syncthreads();
                // (2) panel: rows below the block (incl. the border rows) solve against L11^T
                for (int i = kb + b + tid; i < L + 2; i += kThreads) {
                    double* Ai = A + tri(i, kb);
                    double x[kNB];
#pragma unroll
                    for (int jj = 0; jj < kNB; ++jj) x[jj] = jj < b ? Ai[jj] : 0.0;
#pragma unroll
                    for (int jj = 0; jj < kNB; ++jj) {
                        if (jj < b) {
                            // L_ij = (a_ij - sum_q L_iq D_q L_jq) / D_j   (broadcast reads of L11, D)
                            const double* Aj = A + tri(kb + jj, kb);
                            double sacc = x[jj];
#pragma unroll
                            for (int q = 0; q < jj; ++q)
                                sacc = fma(-x[q] * A[tri(kb + q, kb + q)], Aj[q], sacc);
                            x[jj] = sacc / Aj[jj];
                        }
                    }
#pragma unroll
                    for (int jj = 0; jj < kNB; ++jj)
                        if (jj < b) Ai[jj] = x[jj];
                }
                __syncthreads();
                // (3) trailing update A22 -= L21 L21^T over rows [kb+b, L+2), columns [kb+b, min(i, L-1)]
                {
                    const int r0 = kb + b;
                    const int nr = L + 2 - r0;   // rows
                    const int nc = L - r0;       // columns
                    if (nc > 0) {
                        const int tr = (nr + 3) >> 2, tcn = (nc + 3) >> 2;
                        for (int tix = tid; tix < tr * tcn; tix += kThreads) {
                            const int ti = tix / tcn, tq = tix - ti * tcn;
                            if (tq > ti) continue;   // strictly above the diagonal tiles
                            double acc[4][4];
#pragma unroll
                            for (int x = 0; x < 4; ++x)
#pragma unroll
                                for (int y = 0; y < 4; ++y) acc[x][y] = 0.0;
                            const double* Ar[4];
                            const double* Aq[4];
#pragma unroll
                            for (int x = 0; x < 4; ++x) {
                                const int gi = min(r0 + 4 * ti + x, L + 1);
                                const int gq = min(r0 + 4 * tq + x, L - 1);
                                Ar[x] = A + tri(gi, 0);
                                Aq[x] = A + tri(gq, 0);
                            }
                            for (int j = kb; j < kb + b; ++j) {
                                double vr[4], vq[4];
                                const double dj = A[tri(j, j)];
#pragma unroll
                                for (int x = 0; x < 4; ++x) {
                                    vr[x] = Ar[x][j] * dj;
                                    vq[x] = Aq[x][j];
                                }
#pragma unroll
                                for (int x = 0; x < 4; ++x)
#pragma unroll
                                    for (int y = 0; y < 4; ++y) acc[x][y] = fma(vr[x], vq[y], acc[x][y]);
                            }
#pragma unroll
                            for (int x = 0; x < 4; ++x)
#pragma unroll
                                for (int y = 0; y < 4; ++y) {
                                    const int gi = r0 + 4 * ti + x, gq = r0 + 4 * tq + y;
                                    if (gi < L + 2 && gq < L && gq <= gi) A[tri(gi, gq)] -= acc[x][y];
                                }
                        }
                    }
                }
                __syncthreads();
            }
            PHASE_STAMP(4);

            // --- pred = v^T M^-1 t + mean = sum_j (L^-1 v)_j (L^-1 t)_j / D_j + mean (:314-327)
            //     (the border rows hold (L^-1 t)_j / D_j and (L^-1 v)_j / D_j)
            if (wave == 0) {
                double dot = 0.0;
                const double* y = A + tri(L, 0);
                const double* z = A + tri(L + 1, 0);
                for (int j = lane; j < L; j += 64) dot = fma(y[j] * z[j], A[tri(j, j)], dot);
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
            PHASE_STAMP(5);
        }
    }
    if (a.phase_cycles && tid == 0)
        for (int ph = 0; ph < 6; ++ph) atomicAdd(&a.phase_cycles[ph], ph_acc[ph]);
}

template <typename T>
int launch_predict_bucket(cf_ctx* ctx, PredArgs<T> args, uint32_t count, int lmax, hipStream_t stream) {
    args.lmax = lmax;
    const size_t lds = sizeof(double) * ((size_t)(lmax + 2) * (lmax + 3) / 2 + 4) +
                       CF_MAX_K * (sizeof(uint32_t) + sizeof(float) + 3 * sizeof(int)) + 8 * sizeof(int);
    if (lds > 163840) return cf_set_error(ctx, CF_ERANGE, "predict bucket exceeds LDS");
    int blocks = (int)std::min<uint32_t>(count, 2048u);
    const size_t need = (size_t)blocks * lmax * lmax * sizeof(double);
    if (need > ctx->scratch_bytes) {
        if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
        ctx->d_scratch = nullptr;
        ctx->scratch_bytes = 0;
        CF_HIP_CHECK(ctx, hipMalloc(&ctx->d_scratch, need));
        ctx->scratch_bytes = need;
    }
    args.gbar = reinterpret_cast<double*>(ctx->d_scratch);
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
    args.phase_cycles = ctx->d_phase;
    int rc = CF_OK;
    for (const cf_bucket& b : plan->buckets) {
        if (b.count == 0) continue;
        args.first = b.first;
        const int lmax = std::max<int>(2, 16 * b.emax);
        rc = launch_predict_bucket<T>(ctx, args, b.count, lmax, stream);
        if (rc != CF_OK) break;
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
