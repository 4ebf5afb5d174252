// cf_predict_spill.hip -- neigh_program::apply (local_calc_precomp.cpp:217-380) for the
// users of the eigen spill path (CF_MAX_K < k <= CF_SPILL_MAX_K, BASELINE config 5).
//
// Same contract and the same algebra as predict_kernel (cf_predict.hip), re-laid out for
// k x k blocks that no longer fit in LDS: the per-user tables live in an HBM workspace
// slot, the per-rating factorisation in a per-workgroup HBM region (LDS when small).
// Two kernels per chunk of spill users:
//
//   spill_basis_kernel   one workgroup per user: lim of every row (:271-282); per column,
//                        the number of rows with U(i, j) >= 1e-4 (so the zero-column
//                        filter of :284-304 can be evaluated from the complement);
//                        Gbar = U^T U over [0, Lu), Lu = max lim; the orthonormal basis
//                        Q = U T1 T2 ... of U's leading Lu columns, T = I - su(G - I) -
//                        diag(G - I)/2 (upper triangular: Q's leading lim columns span
//                        U's for every row; each step squares the orthogonality error);
//                        g = Q^T r, h = Q^T 1.  Products are 64 x 64-tiled fp64 GEMMs.
//   spill_predict_kernel persistent workgroups claim (user, test movie) items, heaviest
//                        users first.  C = the user's items that are out-neighbours of
//                        the movie with w > 0.1 (:132,254-265), Cbar = the rest (it holds
//                        the movie's own row r), y = r - mean(r_C) (:311), P = Q_S Q_S^T
//                        over S = [0, lim):
//                          pred - mean = a_r + P_{r,Cbar} K^-1 b,   K = I - P_{Cbar,Cbar},
//                          a_r = (P y)_r - P_{r,Cbar} y_Cbar,  b = (P y)_Cbar - P_{Cbar,Cbar} y_Cbar
//                        (Woodbury on U_CS^T U_CS = I - Q_CbarS^T Q_CbarS in the Q basis),
//                        (P y)_a = Q_aS (g - mean h)_S.  Ratings this form does not take --
//                        a column dropped by the filter, no basis, c = 0, or a pivot of K
//                        below kPivMin while c >= lim -- solve the rating's own bordered
//                        Gram matrix M = U_CS^T U_CS (complement form Gbar_SS -
//                        sum_{i in Cbar} u_i u_i^T when smaller), as the dense path of
//                        cf_predict.hip does.
//
// Output per rating (row r of user u, entry base + r): mse = (float)(r - clamp(pred))^2,
// kk = |C|, pred (:318-359).
#include "cf_internal.h"
#include "cf_ldlt.hpp"

namespace {

constexpr int kT = 256;
constexpr int kW = kT / 64;
constexpr double kPivMin = 1e-10;    // as cf_predict.hip
constexpr float kOrthoMax = 1e-2f;   // as cf_predict.hip
constexpr float kOrthoDone = 1e-8f;  // as cf_predict.hip
constexpr int kMaxSteps = 4;
constexpr int kLdsA = 1920;          // doubles of the LDS factorisation region
constexpr int kSmallNp = 16;         // Woodbury rows up to which P entries are wave dots

template <typename T>
struct SpArgs {
    const uint32_t* order;   // plan order; slot s of the chunk is user order[first + s]
    uint32_t first;
    uint32_t nu;             // users in the chunk (slots used)
    int kmax;                // largest k of the bucket (slot sizing)
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
    double* ws;              // per slot: Q0, Q1, Gbar, Gt (kmax^2 each), g, h, diag (kmax each)
    size_t slot_d;
    int* wsi;                // per slot: lim[kmax], cpos[kmax], hdr[4] = {Lu, basis, qsel, -}
    size_t slot_i;
    double* fa;              // per workgroup factorisation region
    size_t fa_d;
    unsigned int* counter;   // work-item counter of the predict kernel
};

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// out(i, j, C(i, j)) over the 64 x 64 output tiles (i0, j0) of an M x N product with
// want(i0, j0), depth kend(j0) (triangular operands end early), operands staged in LDS
// 16 deep; thread (ty, tx) owns rows 4ty + x, columns 4tx + y of the tile.  A_LFAST: the
// depth index is A's contiguous one (staging walks it fastest so loads coalesce).
// Called by the whole block; ends synchronised.
template <bool A_LFAST, class FA, class FB, class FK, class FW, class FO>
__device__ void tile_gemm(int M, int N, FA ldA, FB ldB, FK kend, FW want, FO out, double* sA, double* sB) {
    const int tid = threadIdx.x;
    const int ty = tid >> 4, tx = tid & 15;
    const int ti = (M + 63) >> 6, tj = (N + 63) >> 6;
    for (int t = 0; t < ti * tj; ++t) {
        const int i0 = (t / tj) << 6, j0 = (t % tj) << 6;
        if (!want(i0, j0)) continue;
        const int K = kend(j0);
        double acc[4][4];
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) acc[x][y] = 0.0;
        for (int l0 = 0; l0 < K; l0 += 16) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e = tid + q * kT;
                const int ii = A_LFAST ? (e >> 4) : (e & 63);
                const int ll = A_LFAST ? (e & 15) : (e >> 6);
                const int gi = i0 + ii, gl = l0 + ll;
                sA[ll * 64 + ii] = (gi < M && gl < K) ? ldA(gi, gl) : 0.0;
                const int jj = e & 63, lb = e >> 6;
                const int gj = j0 + jj, glb = l0 + lb;
                sB[lb * 64 + jj] = (gj < N && glb < K) ? ldB(glb, gj) : 0.0;
            }
            __syncthreads();
#pragma unroll 4
            for (int ll = 0; ll < 16; ++ll) {
                double va[4], vb[4];
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    va[x] = sA[ll * 64 + 4 * ty + x];
                    vb[x] = sB[ll * 64 + 4 * tx + x];
                }
#pragma unroll
                for (int x = 0; x < 4; ++x)
#pragma unroll
                    for (int y = 0; y < 4; ++y) acc[x][y] = fma(va[x], vb[y], acc[x][y]);
            }
            __syncthreads();
        }
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) {
                const int gi = i0 + 4 * ty + x, gj = j0 + 4 * tx + y;
                if (gi < M && gj < N) out(gi, gj, acc[x][y]);
            }
    }
    __syncthreads();
}

// Block-wide ordered compaction over [0, n): out[] receives the indices with f(i) set,
// ascending; returns the count.  s_tmp: kW ints.
template <class F>
__device__ int compact(int n, F f, int* out, int* s_tmp) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int total = 0;
    for (int b0 = 0; b0 < n; b0 += kT) {
        const int i = b0 + tid;
        const bool fl = i < n && f(i);
        const unsigned long long bal = __ballot(fl);
        if (lane == 0) s_tmp[wave] = __popcll(bal);
        __syncthreads();
        int off = total, all = 0;
        for (int w = 0; w < kW; ++w) {
            if (w < wave) off += s_tmp[w];
            all += s_tmp[w];
        }
        if (fl) out[off + __popcll(bal & ((1ull << lane) - 1ull))] = i;
        total += all;
        __syncthreads();
    }
    return total;
}

// ---- per-user tables ---------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kT) void spill_basis_kernel(SpArgs<T> a) {
    __shared__ double sA[16 * 64], sB[16 * 64];
    __shared__ double s_ev[CF_SPILL_MAX_K];
    __shared__ int s_hdr[4];
    __shared__ float s_dev[kW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t s = blockIdx.x;
    const uint32_t u = a.order[a.first + s];
    const uint64_t base = a.item_off[u];
    const int k = (int)(a.item_off[u + 1] - base);
    const int m = a.m[u];
    const T* U = a.evecs + a.evec_off[u];
    const size_t kk2 = (size_t)a.kmax * a.kmax;
    double* slot = a.ws + s * a.slot_d;
    double* Qb[2] = {slot, slot + kk2};
    double* Gb = slot + 2 * kk2;   // Gbar = U^T U over [0, Lu), full, ld Lu
    double* Gt = slot + 3 * kk2;   // Gram of the current Q (steps > 0)
    double* gh = slot + 4 * kk2;   // g[Lu], h[Lu], diag[Lu]
    int* lim = a.wsi + s * a.slot_i;
    int* cpos = lim + a.kmax;
    int* hdr = cpos + a.kmax;

    for (int j = tid; j < m; j += kT) s_ev[j] = (double)a.evals[base + j];
    if (tid == 0) s_hdr[0] = 2;
    __syncthreads();
    // lim = first eigenvalue index above w_lim, clamped to [2, m] (:271-282)
    for (int i = tid; i < k; i += kT) {
        const double w_lim = (double)a.sigtab[a.sig_mode == CF_SIGS_COMPAT ? (uint64_t)i : base + i];
        int l = m;
        for (int j = 0; j < m; ++j)
            if (s_ev[j] > w_lim) {
                l = j;
                break;
            }
        l = min(max(l, 2), m);
        lim[i] = l;
        atomicMax(&s_hdr[0], l);
    }
    __syncthreads();
    const int Lu = s_hdr[0];
    // rows with U(i, j) >= 1e-4 per column j < Lu; Q0 = U(:, 0:Lu) in fp64
    for (int j = tid; j < Lu; j += kT) {
        int cnt = 0;
        for (int i = 0; i < k; ++i) {
            const double v = (double)U[(size_t)i * m + j];
            cnt += v >= 0.0001;
            Qb[0][(size_t)i * Lu + j] = v;
        }
        cpos[j] = cnt;
    }
    __syncthreads();
    int cur = 0, basis = 1;
    for (int step = 0; step < kMaxSteps; ++step) {
        const double* Q = Qb[cur];
        double* G = step == 0 ? Gb : Gt;
        float dev = 0.0f;
        tile_gemm<false>(
            Lu, Lu, [=](int i, int l) { return Q[(size_t)l * Lu + i]; },
            [=](int l, int j) { return Q[(size_t)l * Lu + j]; }, [=](int) { return k; },
            [](int, int) { return true; },
            [&](int i, int j, double v) {
                G[(size_t)i * Lu + j] = v;
                dev = fmaxf(dev, (float)fabs(v - (i == j ? 1.0 : 0.0)));
            },
            sA, sB);
        for (int off = 32; off >= 1; off >>= 1) dev = fmaxf(dev, __shfl_xor(dev, off));
        if (lane == 0) s_dev[wave] = dev;
        __syncthreads();
        dev = fmaxf(fmaxf(s_dev[0], s_dev[1]), fmaxf(s_dev[2], s_dev[3]));
        __syncthreads();
        if (step == 0 && !(dev <= kOrthoMax)) {   // U far from orthonormal: dense path only
            basis = 0;
            break;
        }
        // Q' = Q T,  T(l, j) = -G(l, j) (l < j), 1.5 - G(j, j)/2 (l = j), 0 (l > j)
        const double* Gr = G;
        double* Qn = Qb[cur ^ 1];
        tile_gemm<true>(
            k, Lu, [=](int i, int l) { return Q[(size_t)i * Lu + l]; },
            [=](int l, int j) {
                const double gv = Gr[(size_t)l * Lu + j];
                return l < j ? -gv : (l == j ? 1.5 - 0.5 * gv : 0.0);
            },
            [=](int j0) { return min(Lu, j0 + 64); }, [](int, int) { return true; },
            [=](int i, int j, double v) { Qn[(size_t)i * Lu + j] = v; }, sA, sB);
        cur ^= 1;
        if (dev <= kOrthoDone) break;
    }
    // g = Q^T r, h = Q^T 1
    if (basis) {
        const double* Q = Qb[cur];
        for (int j = tid; j < Lu; j += kT) {
            double g = 0.0, h = 0.0;
            for (int i = 0; i < k; ++i) {
                const double q = Q[(size_t)i * Lu + j];
                g = fma(q, (double)a.ratings[base + i], g);
                h += q;
            }
            gh[j] = g;
            gh[Lu + j] = h;
        }
    }
    if (tid == 0) {
        hdr[0] = Lu;
        hdr[1] = basis;
        hdr[2] = cur;
    }
}

// ---- per-rating predictions --------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kT) void spill_predict_kernel(SpArgs<T> a) {
    __shared__ double sA[16 * 64], sB[16 * 64];   // GEMM staging
    __shared__ double s_la[kLdsA];
    __shared__ float s_rat[CF_SPILL_MAX_K];
    __shared__ int s_conn[CF_SPILL_MAX_K];
    __shared__ int s_ncon[CF_SPILL_MAX_K];
    __shared__ int s_keep[CF_SPILL_MAX_K];
    __shared__ double s_misc[4];
    __shared__ int s_tmp[kW];
    __shared__ unsigned int s_item;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double* fa = a.fa + (size_t)blockIdx.x * a.fa_d;
    const uint32_t total = a.nu * (uint32_t)a.kmax;
    for (;;) {
        if (tid == 0) s_item = atomicAdd(a.counter, 1u);
        __syncthreads();
        const uint32_t w = s_item;
        __syncthreads();
        if (w >= total) break;   // every wave of every block reaches this exit
        const uint32_t s = w / (uint32_t)a.kmax;
        const int r = (int)(w - s * (uint32_t)a.kmax);
        const uint32_t u = a.order[a.first + s];
        const uint64_t base = a.item_off[u];
        const int k = (int)(a.item_off[u + 1] - base);
        if (r >= k) continue;   // block-uniform
        const int m = a.m[u];
        const T* U = a.evecs + a.evec_off[u];
        const size_t kk2 = (size_t)a.kmax * a.kmax;
        const double* slot = a.ws + s * a.slot_d;
        const int* lim_t = a.wsi + s * a.slot_i;
        const int* cpos = lim_t + a.kmax;
        const int* hdr = cpos + a.kmax;
        const int Lu = hdr[0];
        const bool basis = hdr[1] != 0;
        const double* Q = slot + (hdr[2] ? kk2 : 0);
        const double* Gb = slot + 2 * kk2;
        const double* gvec = slot + 4 * kk2;
        const double* hvec = gvec + Lu;
        const int lim = lim_t[r];

        // connected set C (:254-265); Cbar = the rest, the movie's own row r included
        const float* nrow = a.graph + (size_t)a.items[base + r] * a.n_items;
        for (int i = tid; i < k; i += kT) s_rat[i] = a.ratings[base + i];
        const int c = compact(k, [&](int i) { return (double)nrow[a.items[base + i]] > 0.1; }, s_conn, s_tmp);
        const int nc = compact(k, [&](int i) { return !((double)nrow[a.items[base + i]] > 0.1); }, s_ncon, s_tmp);
        // mean of the connected ratings (:311); c = 0 gives 0/0 = NaN, as in the reference
        if (wave == 0) {
            double sum = 0.0;
            for (int i = lane; i < c; i += 64) sum += (double)s_rat[s_conn[i]];
            sum = wsum(sum);
            if (lane == 0) s_misc[0] = sum / (double)c;
        }
        __syncthreads();
        const double mu = s_misc[0];
        bool fast = basis && c > 0;
        if (fast) {
            // zero-column filter from the complement: column j < lim is dropped iff every
            // row with U(i, j) >= 1e-4 lies in Cbar
            bool drop = false;
            for (int j = tid; j < lim; j += kT)
                if (cpos[j] <= nc) {
                    int hit = 0;
                    for (int q = 0; q < nc; ++q) hit += (double)U[(size_t)s_ncon[q] * m + j] >= 0.0001;
                    drop |= hit == cpos[j];
                }
            fast = !__syncthreads_or(drop);
        }
        if (fast) {
            const int np = nc + 1;   // rows Cbar..., then r
            const size_t need = (size_t)(nc + 2) * (nc + 3) / 2;
            double* A = need <= (size_t)kLdsA ? s_la : fa;
            const auto rowid = [&](int q) { return q < np - 1 ? s_ncon[q] : r; };
            // E = P_S over rows [Cbar, r] into packed rows 0..nc; (P y)_a into row nc + 1
            const int ne = np * (np + 1) / 2;
            const int nd = np <= kSmallNp ? ne + np : np;   // wave dots
            for (int e = wave; e < nd; e += kW) {
                const bool isE = np <= kSmallNp && e < ne;
                const int pa = isE ? 0 : (np <= kSmallNp ? e - ne : e);
                int ra = pa, rb = 0;
                if (isE) {
                    ra = 0;
                    while ((ra + 1) * (ra + 2) / 2 <= e) ++ra;
                    rb = e - ra * (ra + 1) / 2;
                }
                const double* xa = Q + (size_t)rowid(ra) * Lu;
                const double* xb = Q + (size_t)rowid(rb) * Lu;
                double acc = 0.0;
                if (isE)
                    for (int j = lane; j < lim; j += 64) acc = fma(xa[j], xb[j], acc);
                else
                    for (int j = lane; j < lim; j += 64) acc = fma(xa[j], gvec[j] - mu * hvec[j], acc);
                acc = wsum(acc);
                if (lane == 0) A[isE ? e : tri(np, pa)] = acc;
            }
            if (np > kSmallNp)
                tile_gemm<true>(
                    np, np, [&](int i, int l) { return Q[(size_t)rowid(i) * Lu + l]; },
                    [&](int l, int j) { return Q[(size_t)rowid(j) * Lu + l]; }, [=](int) { return lim; },
                    [](int i0, int j0) { return j0 <= i0; },
                    [&](int i, int j, double v) {
                        if (j <= i) A[tri(i, j)] = v;
                    },
                    sA, sB);
            __syncthreads();
            // b_a = (P y)_a - sum_q E_aq y_q (in place of (P y)_a), a_r likewise
            for (int pa = tid; pa < np; pa += kT) {
                double v = A[tri(np, pa)];
                for (int q = 0; q < np - 1; ++q) {
                    const double eq = q <= pa ? A[tri(pa, q)] : A[tri(q, pa)];
                    v = fma(-eq, (double)s_rat[s_ncon[q]] - mu, v);
                }
                if (pa < np - 1)
                    A[tri(np, pa)] = v;
                else
                    s_misc[1] = v;
            }
            __syncthreads();
            // K = I - P_CbarCbar
            for (int e = tid; e < nc * (nc + 1) / 2; e += kT) {
                int ra = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
                while (ra * (ra + 1) / 2 > e) --ra;
                while ((ra + 1) * (ra + 2) / 2 <= e) ++ra;
                A[e] = (e == tri(ra, ra) ? 1.0 : 0.0) - A[e];
            }
            __syncthreads();
            ldlt_bordered<kT>(A, nc, nc + 2);
            if (wave == 0) {
                double minpiv = 1.0, dot = 0.0;
                for (int j = lane; j < nc; j += 64) {
                    const double dj = A[tri(j, j)];
                    minpiv = fmin(minpiv, dj);
                    dot = fma(A[tri(nc, j)] * A[tri(nc + 1, j)], dj, dot);
                }
                dot = wsum(dot);
                for (int off = 32; off >= 1; off >>= 1) minpiv = fmin(minpiv, __shfl_xor(minpiv, off));
                if (lane == 0) {
                    s_misc[2] = dot;
                    s_misc[3] = minpiv;
                }
            }
            __syncthreads();
            // full rank but ill-conditioned: the dense path, whose error matches the reference's
            fast = !(!(s_misc[3] >= kPivMin) && c >= lim);
            if (fast && tid == 0) {
                double pred = mu + s_misc[1] + s_misc[2];
                if (pred > 5) pred = 5;
                if (pred < 1) pred = 1;
                const double d = (double)s_rat[r] - pred;
                a.mse[base + r] = (float)(d * d);
                a.kk[base + r] = c;
                if (a.pred) a.pred[base + r] = pred;
            }
            __syncthreads();
            if (fast) continue;
        }

        // ---- dense path: the rating's own bordered Gram matrix ----------------------------
        // zero-column filter: keep column j < lim iff some U(C, j) >= 1e-4 (:284-304)
        const bool use_complement = nc < c;
        const int L = compact(
            lim,
            [&](int j) {
                int hit = 0;
                const int n = use_complement ? nc : c;
                const int* rows = use_complement ? s_ncon : s_conn;
                for (int q = 0; q < n; ++q) hit += (double)U[(size_t)rows[q] * m + j] >= 0.0001;
                return use_complement ? cpos[j] - hit > 0 : hit > 0;
            },
            s_keep, s_tmp);
        const size_t need = (size_t)(L + 2) * (L + 3) / 2;
        double* A = need <= (size_t)kLdsA ? s_la : fa;
        const int nrows = use_complement ? nc : c;
        const int* rows = use_complement ? s_ncon : s_conn;
        // A(i, j) = (U_CS^T U_CS)_ij (j <= i < L), A(L, j) = t_j, A(L + 1, j) = v_j
        tile_gemm<false>(
            L, L, [&](int i, int l) { return (double)U[(size_t)rows[l] * m + s_keep[i]]; },
            [&](int l, int j) { return (double)U[(size_t)rows[l] * m + s_keep[j]]; },
            [=](int) { return nrows; }, [](int i0, int j0) { return j0 <= i0; },
            [&](int i, int j, double v) {
                if (j <= i) A[tri(i, j)] = use_complement ? Gb[(size_t)s_keep[i] * Lu + s_keep[j]] - v : v;
            },
            sA, sB);
        for (int j = tid; j < L; j += kT) {
            const int cj = s_keep[j];
            double t = 0.0;
            for (int q = 0; q < c; ++q) t = fma((double)U[(size_t)s_conn[q] * m + cj], (double)s_rat[s_conn[q]] - mu, t);
            A[tri(L, j)] = t;
            A[tri(L + 1, j)] = (double)U[(size_t)r * m + cj];
        }
        __syncthreads();
        ldlt_bordered<kT>(A, L, L + 2);
        // pred = v^T M^-1 t + mean = sum_j (L^-1 v)_j (L^-1 t)_j / D_j + mean (:314-327)
        if (wave == 0) {
            double dot = 0.0;
            for (int j = lane; j < L; j += 64) dot = fma(A[tri(L, j)] * A[tri(L + 1, j)], A[tri(j, j)], dot);
            dot = wsum(dot);
            if (lane == 0) {
                double pred = dot + mu;
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

}  // namespace

template <typename T>
int cf_launch_predict_spill(cf_ctx* ctx, const cf_plan* plan, const cf_bucket& b, const uint64_t* d_item_off,
                            const uint32_t* d_items, const float* d_ratings, const int32_t* d_m,
                            const T* d_evals, const uint64_t* d_evec_off, const T* d_evecs, const T* d_sigtab,
                            int sig_mode, float* d_mse, int32_t* d_kk, double* d_pred, hipStream_t stream) {
    if (b.count == 0) return CF_OK;
    const int kmax = (int)b.kmax;
    if (kmax > CF_SPILL_MAX_K) return cf_set_error(ctx, CF_ERANGE, "predict spill: k above CF_SPILL_MAX_K");
    SpArgs<T> a{};
    a.order = plan->d_order;
    a.kmax = kmax;
    a.item_off = d_item_off;
    a.items = d_items;
    a.ratings = d_ratings;
    a.m = d_m;
    a.evals = d_evals;
    a.evec_off = d_evec_off;
    a.evecs = d_evecs;
    a.sigtab = d_sigtab;
    a.sig_mode = sig_mode;
    a.graph = ctx->d_graph;
    a.n_items = ctx->n_items;
    a.mse = d_mse;
    a.kk = d_kk;
    a.pred = d_pred;
    // workspace: counter | factorisation regions | user slots (doubles) | slot ints
    const size_t kk2 = (size_t)kmax * kmax;
    a.slot_d = 4 * kk2 + 3 * (size_t)kmax;
    a.slot_i = 2 * (size_t)kmax + 4;
    a.fa_d = (size_t)(kmax + 2) * (kmax + 3) / 2;
    const size_t kSlotBudget = (size_t)8 << 30, kFaBudget = (size_t)4 << 30;
    const uint32_t slots = (uint32_t)std::max<size_t>(1, std::min<size_t>(b.count, kSlotBudget / (a.slot_d * 8)));
    const int blocks = (int)std::max<size_t>(32, std::min<size_t>(512, kFaBudget / (a.fa_d * 8)));
    const size_t fa_bytes = (size_t)blocks * a.fa_d * sizeof(double);
    const size_t ws_bytes = (size_t)slots * a.slot_d * sizeof(double);
    const size_t need = 256 + fa_bytes + ws_bytes + (size_t)slots * a.slot_i * sizeof(int);
    if (need > ctx->pspill_bytes) {
        if (ctx->d_pspill) (void)hipFree(ctx->d_pspill);
        ctx->d_pspill = nullptr;
        ctx->pspill_bytes = 0;
        CF_HIP_CHECK(ctx, hipMalloc(&ctx->d_pspill, need));
        ctx->pspill_bytes = need;
    }
    char* p = reinterpret_cast<char*>(ctx->d_pspill);
    a.counter = reinterpret_cast<unsigned int*>(p);
    a.fa = reinterpret_cast<double*>(p + 256);
    a.ws = reinterpret_cast<double*>(p + 256 + fa_bytes);
    a.wsi = reinterpret_cast<int*>(p + 256 + fa_bytes + ws_bytes);
    for (uint32_t u0 = 0; u0 < b.count; u0 += slots) {
        a.first = b.first + u0;
        a.nu = std::min(slots, b.count - u0);
        CF_HIP_CHECK(ctx, hipMemsetAsync(a.counter, 0, sizeof(unsigned int), stream));
        hipLaunchKernelGGL(spill_basis_kernel<T>, dim3(a.nu), dim3(kT), 0, stream, a);
        CF_HIP_CHECK(ctx, hipGetLastError());
        const uint32_t items = a.nu * (uint32_t)kmax;
        hipLaunchKernelGGL(spill_predict_kernel<T>, dim3((unsigned)std::min<uint32_t>(blocks, items)), dim3(kT), 0,
                           stream, a);
        CF_HIP_CHECK(ctx, hipGetLastError());
    }
    return CF_OK;
}

template int cf_launch_predict_spill<float>(cf_ctx*, const cf_plan*, const cf_bucket&, const uint64_t*,
                                            const uint32_t*, const float*, const int32_t*, const float*,
                                            const uint64_t*, const float*, const float*, int, float*, int32_t*,
                                            double*, hipStream_t);
template int cf_launch_predict_spill<double>(cf_ctx*, const cf_plan*, const cf_bucket&, const uint64_t*,
                                             const uint32_t*, const float*, const int32_t*, const double*,
                                             const uint64_t*, const double*, const double*, int, float*,
                                             int32_t*, double*, hipStream_t);
