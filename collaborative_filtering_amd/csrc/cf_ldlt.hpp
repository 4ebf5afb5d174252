// cf_ldlt.hpp -- blocked, bordered LDL^T of a packed lower triangle in LDS (fp64),
// shared by the precomp predictor (cf_predict.hip) and local_calc (cf_local.hip).
#pragma once

#include <hip/hip_runtime.h>

// Packed lower-triangular index (row-major rows of increasing length).
inline __device__ int tri(int i, int j) { return (i * (i + 1)) / 2 + j; }

#define WAVE_SYNC()                                              \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
    } while (0)

constexpr int kNB = 16;   // default LDL^T panel width

// Blocked right-looking LDL^T of the leading L x L block of the packed lower triangle
// A (rows [0, nrows), nrows >= L), carrying rows [L, nrows) as border rows: on return
// A holds unit-lower L below the diagonal, D on it, and border row i holds
// (L^-1 a_i)_j / D_j.  An exactly zero pivot is skipped (its column of L is 0), as
// Eigen's LU skips a zero pivot column: a structurally singular matrix whose trailing
// block has cancelled to exact zeros gives finite, clamped garbage like the
// reference's, not inf - inf = NaN.  Called by the whole block; starts and ends
// synchronised.
//
// ldlt_bordered_range factors only the columns [k0, k1) (all rows below them, trailing
// updates confined to columns < k1): a caller blocking the factorisation in wider panels
// applies the update of columns >= k1 itself.  ldlt_bordered = the full range.
// TAG: distinct instantiations for callers compiled to different register budgets
template <int kThreads, int NB = kNB, int TAG = 0>
__device__ void ldlt_bordered_range(double* A, int L, int nrows, int k0, int k1) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    for (int kb = k0; kb < k1; kb += NB) {
        const int b = min(NB, k1 - kb);
        // (1) diagonal block, unblocked LDL^T, in wave 0's registers: lane i < b holds
        //     row kb + i; column j is broadcast by shuffles.
        if (wave == 0) {
            double rowv[NB];
            const int i = lane;
            const bool live = i < b;
#pragma unroll
            for (int q = 0; q < NB; ++q) rowv[q] = (live && q <= i) ? A[tri(kb + i, kb + q)] : 0.0;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                if (j < b) {
                    const double dj = __shfl(rowv[j], j);
                    const double w = (i > j) ? rowv[j] : 0.0;   // unscaled a_ij
                    const double lij = dj != 0.0 ? w / dj : 0.0;   // exact-zero pivot: skipped
#pragma unroll
                    for (int q = j + 1; q < NB; ++q) {
                        const double wq = __shfl(w, q);
                        if (q <= i) rowv[q] = fma(-lij, wq, rowv[q]);
                    }
                    if (i > j) rowv[j] = lij;
                }
            }
#pragma unroll
            for (int q = 0; q < NB; ++q)
                if (live && q <= i) A[tri(kb + i, kb + q)] = rowv[q];
        }
        __syncthreads();
        // (2) panel: rows below the block (incl. the border rows) solve against L11^T
        for (int i = kb + b + tid; i < nrows; i += kThreads) {
            double* Ai = A + tri(i, kb);
            double x[NB];
#pragma unroll
            for (int jj = 0; jj < NB; ++jj) x[jj] = jj < b ? Ai[jj] : 0.0;
#pragma unroll
            for (int jj = 0; jj < NB; ++jj) {
                if (jj < b) {
                    const double* Aj = A + tri(kb + jj, kb);
                    double sacc = x[jj];
#pragma unroll
                    for (int q = 0; q < jj; ++q) sacc = fma(-x[q] * A[tri(kb + q, kb + q)], Aj[q], sacc);
                    x[jj] = Aj[jj] != 0.0 ? sacc / Aj[jj] : 0.0;
                }
            }
#pragma unroll
            for (int jj = 0; jj < NB; ++jj)
                if (jj < b) Ai[jj] = x[jj];
        }
        __syncthreads();
        // (3) trailing update A22 -= L21 D L21^T over rows [kb+b, nrows), columns [kb+b, L)
        {
            const int r0 = kb + b;
            const int nr = nrows - r0;
            const int nc = k1 - r0;
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
                        Ar[x] = A + tri(min(r0 + 4 * ti + x, nrows - 1), 0);
                        Aq[x] = A + tri(min(r0 + 4 * tq + x, k1 - 1), 0);
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
                            if (gi < nrows && gq < k1 && gq <= gi) A[tri(gi, gq)] -= acc[x][y];
                        }
                }
            }
        }
        __syncthreads();
    }
}

template <int kThreads, int NB = kNB>
__device__ void ldlt_bordered(double* A, int L, int nrows) {
    ldlt_bordered_range<kThreads, NB>(A, L, nrows, 0, L);
}
