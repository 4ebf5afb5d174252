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
//                        g = Q^T r, h = Q^T 1, P = Q Q^T (k x k), Q g and Q h.  Products
//                        are 64 x 64-tiled fp64 GEMMs.
//   spill_predict_kernel persistent workgroups claim (user, test movie) items, heaviest
//                        users first.  C = the user's items that are out-neighbours of
//                        the movie with w > 0.1 (:132,254-265), Cbar = the rest (it holds
//                        the movie's own row r), y = r - mean(r_C) (:311), P = Q_S Q_S^T
//                        over S = [0, lim):
//                          pred - mean = a_r + P_{r,Cbar} K^-1 b,   K = I - P_{Cbar,Cbar},
//                          a_r = (P y)_r - P_{r,Cbar} y_Cbar,  b = (P y)_Cbar - P_{Cbar,Cbar} y_Cbar
//                        (Woodbury on U_CS^T U_CS = I - Q_CbarS^T Q_CbarS in the Q basis),
//                        (P y)_a = Q_aS (g - mean h)_S; every entry is a gather from the
//                        per-user tables (columns [lim, Lu) subtracted when lim < Lu).  For
//                        c < lim (K singular) the minimum-norm least-squares prediction
//                        P_{r,C} P_CC^-1 y_C from the c x c block of P instead.  Ratings this form does not take --
//                        a column dropped by the filter, no basis, c = 0, or a pivot of K
//                        below kPivMin while c >= lim -- solve the rating's own bordered
//                        Gram matrix M = U_CS^T U_CS (complement form Gbar_SS -
//                        sum_{i in Cbar} u_i u_i^T when smaller), as the dense path of
//                        cf_predict.hip does.
//
// Output per rating (row r of user u, entry base + r): mse = (float)(r - clamp(pred))^2,
// kk = |C|, pred (:318-359).
#include <algorithm>
#include <cstring>

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

template <typename T>
struct SpArgs {
    const uint32_t* order;   // plan order; slot s of the chunk is user order[first + s]
    uint32_t first;
    uint32_t nu;             // users in the chunk (slots used)
    int kmax;                // largest k of the bucket (slot sizing)
    const uint64_t* item_off;
    const uint32_t* items;
    const float* ratings;
    const uint8_t* row_sel;   // rows to predict (null: all)
    const int32_t* m;
    const T* evals;
    const uint64_t* evec_off;
    const T* evecs;
    const T* sigtab;
    int sig_mode;
    GraphDev graph;
    uint64_t n_items;
    float* mse;
    int32_t* kk;
    double* pred;
    double* ws;              // per slot: Q0, Q1 (Q and P = Q Q^T), Gbar, Gt (k^2 each), g, h, PG, PH
    const uint64_t* soff;    // per slot s of the chunk (nu + 1): doubles offset of its slot in ws
    int* wsi;                // per slot: lim[k], cpos[k], hdr[8] = {Lu, basis, qsel, G-mode, spill_basis_mc state}
    const uint64_t* sioff;   // per slot (nu + 1): ints offset of its slot in wsi
    const uint64_t* roff;    // per slot (nu + 1): first work item (= row) of the slot; roff[nu] items
    double* fa;              // per workgroup factorisation region
    size_t fa_d;
    unsigned int* counter;   // work-item counter of the predict kernel
    uint32_t w0, w1;         // predict launch: the chunk's work items [w0, w1)
    unsigned long long* phase;   // diagnostics (cf_debug_phases) or null: see spill_predict_kernel
    // users with k > kSmallCap (the <T, 0, 2> predict kernel): per workgroup, the per-row
    // arrays (ratings, C, Cbar, kept columns) in HBM, 4 x rows_d words each
    uint32_t* rows;
    size_t rows_d;
    uint32_t s0;   // spill_basis_kernel: its first slot (the slots before it take spill_basis_mc)
    int G;         // spill_basis_mc: workgroups per user
};

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// out(i, j, C(i, j)) over the 64 x 64 output tiles (i0, j0) of an M x N product with
// want(i0, j0), depth kend(j0) (triangular operands end early); tiles t0, t0 + ts, ... only.  Operands are staged in
// LDS 16 deep (row stride kSt == 16 mod 32: the four 16-lane groups of a fragment read
// hit disjoint banks) with the next chunk's loads in flight while the current one is
// consumed; unconditional loads from clamped indices (a guarded load would become a
// branch with its own wait).  The products run on the fp64 matrix cores: wave w owns the
// 32 x 32 quadrant (w >> 1, w & 1) as 2 x 2 v_mfma_f64_16x16x4_f64 tiles (A lane l =
// A[l & 15][l >> 4], B lane l = B[l >> 4][l & 15], result q of lane l = C[(l >> 4) + 4q]
// [l & 15]; tools/mfma_f64_probe.hip).  A_LFAST / B_LFAST: the depth index is the
// operand's contiguous one (staging walks it fastest so loads coalesce).  Called by the
// whole block; ends synchronised.
using f64x4 = __attribute__((ext_vector_type(4))) double;
constexpr int kSt = 80;
// NBUF = 2 (the caller's sA / sB hold two chunks, 2 * 16 * kSt doubles each): two chunks of raw
// operands in flight in registers and the staged chunks alternating between the buffers, one
// barrier per chunk (cf_predict.hip's block_gemm scheme: the gathers of a 64-wide row block are
// ~2k cycles away, a chunk's MFMAs ~1k).  NBUF = 1 keeps the single-buffer LDS footprint for
// the two-workgroups-per-CU predictor.  LOWER: 16 x 16 tiles wholly above the diagonal skip
// their MFMAs (the callers keep j <= i only); tiles past M / N always do.
template <bool A_LFAST, bool B_LFAST, int NBUF = 1, bool LOWER = false, class FA, class FB, class FK, class FW,
          class FO>
__device__ void tile_gemm(int M, int N, FA ldA, FB ldB, FK kend, FW want, FO out, double* sA, double* sB, int t0 = 0,
                          int ts = 1) {
    static_assert(NBUF == 1 || NBUF == 2, "one or two staging buffers");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wr = (tid >> 6) >> 1, wc = (tid >> 6) & 1;
    const int ti = (M + 63) >> 6, tj = (N + 63) >> 6;
    for (int t = t0; t < ti * tj; t += ts) {   // tiles t0, t0 + ts, ... (spill_basis_mc: one workgroup's share)
        const int i0 = (t / tj) << 6, j0 = (t % tj) << 6;
        if (!want(i0, j0)) continue;
        const int K = kend(j0);
        bool live[2][2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
                const int r0 = i0 + 32 * wr + 16 * x, c0 = j0 + 32 * wc + 16 * y;
                live[x][y] = r0 < M && c0 < N && (!LOWER || c0 <= r0 + 15);
            }
        f64x4 acc[2][2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) acc[x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
        double ra0[4], rb0[4], ra1[4], rb1[4];
        auto fetch = [&](int l0, double (&ra)[4], double (&rb)[4]) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e = tid + q * kT;
                const int ii = A_LFAST ? (e >> 4) : (e & 63), la = A_LFAST ? (e & 15) : (e >> 6);
                const int jj = B_LFAST ? (e >> 4) : (e & 63), lb = B_LFAST ? (e & 15) : (e >> 6);
                ra[q] = ldA(min(i0 + ii, M - 1), min(l0 + la, K - 1));
                rb[q] = ldB(min(l0 + lb, K - 1), min(j0 + jj, N - 1));
            }
        };
        auto stage = [&](int l0, double (&ra)[4], double (&rb)[4], int b) {
            double* As = sA + (NBUF - 1) * b * 16 * kSt;
            double* Bs = sB + (NBUF - 1) * b * 16 * kSt;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e = tid + q * kT;
                const int ii = A_LFAST ? (e >> 4) : (e & 63), la = A_LFAST ? (e & 15) : (e >> 6);
                const int jj = B_LFAST ? (e >> 4) : (e & 63), lb = B_LFAST ? (e & 15) : (e >> 6);
                As[la * kSt + ii] = (i0 + ii < M && l0 + la < K) ? ra[q] : 0.0;
                Bs[lb * kSt + jj] = (j0 + jj < N && l0 + lb < K) ? rb[q] : 0.0;
            }
            __syncthreads();
        };
        auto mma = [&](int b) {
            const double* As = sA + (NBUF - 1) * b * 16 * kSt;
            const double* Bs = sB + (NBUF - 1) * b * 16 * kSt;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int row = (4 * ks + (lane >> 4)) * kSt + (lane & 15);
                double av[2], bv[2];
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    av[x] = As[row + 32 * wr + 16 * x];
                    bv[x] = Bs[row + 32 * wc + 16 * x];
                }
#pragma unroll
                for (int x = 0; x < 2; ++x)
#pragma unroll
                    for (int y = 0; y < 2; ++y)
                        if (live[x][y])
                            acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[x], bv[y], acc[x][y], 0, 0, 0);
            }
        };
        if (NBUF == 2) {
            if (K > 0) fetch(0, ra0, rb0);
            if (K > 16) fetch(16, ra1, rb1);
            for (int l0 = 0; l0 < K; l0 += 32) {
                // chunk c goes to buffer c & 1 after the barrier that published chunk c - 1,
                // which every wave reaches only after its MFMAs on chunk c - 2 (same buffer)
                stage(l0, ra0, rb0, 0);
                if (l0 + 32 < K) fetch(l0 + 32, ra0, rb0);
                mma(0);
                if (l0 + 16 < K) {
                    stage(l0 + 16, ra1, rb1, 1);
                    if (l0 + 48 < K) fetch(l0 + 48, ra1, rb1);
                    mma(1);
                }
            }
            __syncthreads();   // the next tile restarts at buffer 0, which slower waves may still read
        } else {
            if (K > 0) fetch(0, ra0, rb0);
            for (int l0 = 0; l0 < K; l0 += 16) {
                stage(l0, ra0, rb0, 0);
                if (l0 + 16 < K) fetch(l0 + 16, ra0, rb0);
                mma(0);
                __syncthreads();   // the chunk is consumed before the next one is staged
            }
        }
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int gi = i0 + 32 * wr + 16 * x + (lane >> 4) + 4 * q;
                    const int gj = j0 + 32 * wc + 16 * y + (lane & 15);
                    if (gi < M && gj < N) out(gi, gj, acc[x][y][q]);
                }
    }
    __syncthreads();
}

// C -= A B on the lower triangle of the output (tile_gemm's staging and MFMA layout), with the
// tile's C values loaded before its K loop so their latency hides behind the products instead
// of a load-then-store at the end.  cptr(i, j) = the address of C(i, j), used for j <= i only.
template <bool A_LFAST, bool B_LFAST, class FA, class FB, class FC>
__device__ void tile_gemm_sub(int M, int N, int K, FA ldA, FB ldB, FC cptr, double* sA, double* sB) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wr = (tid >> 6) >> 1, wc = (tid >> 6) & 1;
    const int ti = (M + 63) >> 6, tj = (N + 63) >> 6;
    for (int t = 0; t < ti * tj; ++t) {
        const int i0 = (t / tj) << 6, j0 = (t % tj) << 6;
        if (j0 > i0) continue;   // strictly above the diagonal tiles
        f64x4 acc[2][2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) acc[x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
        double ra[4], rb[4];
        auto fetch = [&](int l0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e = tid + q * kT;
                const int ii = A_LFAST ? (e >> 4) : (e & 63), la = A_LFAST ? (e & 15) : (e >> 6);
                const int jj = B_LFAST ? (e >> 4) : (e & 63), lb = B_LFAST ? (e & 15) : (e >> 6);
                ra[q] = ldA(min(i0 + ii, M - 1), min(l0 + la, K - 1));
                rb[q] = ldB(min(l0 + lb, K - 1), min(j0 + jj, N - 1));
            }
        };
        if (K > 0) fetch(0);
        double cv[2][2][4];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int gi = i0 + 32 * wr + 16 * x + (lane >> 4) + 4 * q;
                    const int gj = j0 + 32 * wc + 16 * y + (lane & 15);
                    cv[x][y][q] = (gi < M && gj < N && gj <= gi) ? *cptr(gi, gj) : 0.0;
                }
        for (int l0 = 0; l0 < K; l0 += 16) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e = tid + q * kT;
                const int ii = A_LFAST ? (e >> 4) : (e & 63), la = A_LFAST ? (e & 15) : (e >> 6);
                const int jj = B_LFAST ? (e >> 4) : (e & 63), lb = B_LFAST ? (e & 15) : (e >> 6);
                sA[la * kSt + ii] = (i0 + ii < M && l0 + la < K) ? ra[q] : 0.0;
                sB[lb * kSt + jj] = (j0 + jj < N && l0 + lb < K) ? rb[q] : 0.0;
            }
            __syncthreads();
            if (l0 + 16 < K) fetch(l0 + 16);
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int row = (4 * ks + (lane >> 4)) * kSt + (lane & 15);
                double av[2], bv[2];
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    av[x] = sA[row + 32 * wr + 16 * x];
                    bv[x] = sB[row + 32 * wc + 16 * x];
                }
#pragma unroll
                for (int x = 0; x < 2; ++x)
#pragma unroll
                    for (int y = 0; y < 2; ++y)
                        acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[x], bv[y], acc[x][y], 0, 0, 0);
            }
            __syncthreads();   // the chunk is consumed before the next one is staged
        }
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int gi = i0 + 32 * wr + 16 * x + (lane >> 4) + 4 * q;
                    const int gj = j0 + 32 * wc + 16 * y + (lane & 15);
                    if (gi < M && gj < N && gj <= gi) *cptr(gi, gj) = cv[x][y][q] - acc[x][y][q];
                }
    }
    __syncthreads();
}

// Fill the packed lower triangle of n rows, A[tri(ra, cb)] = f(ra, cb): wave w takes rows
// w, w + kW, ..., its lanes the columns of a row (contiguous in A; no per-element inversion
// of the triangular index).  Does not synchronise.
template <class F>
__device__ void fill_tri_rows(double* A, int n, F f) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int ra = wave; ra < n; ra += kW) {
        double* Arow = A + tri(ra, 0);
        for (int cb = lane; cb <= ra; cb += 64) Arow[cb] = f(ra, cb);
    }
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

// A[i][j] -= sum_{l in [d0, d1)} A[i][l] D_l A[j][l] over rows [c0, nrows), columns [c0, c1)
// (lower triangle), on the matrix cores: the rank-(d1 - d0) update of factored columns
// [d0, d1) into the packed lower triangle.
// OCC: the calling kernel's occupancy, so each gets its own copy compiled to its register budget
template <int OCC = 1>
__device__ void ldlt_rank_update(double* A, int nrows, int d0, int d1, int c0, int c1, double* sA, double* sB) {
#ifdef CF_SPILL_LDL_NOPRELOAD
    tile_gemm<true, true>(
        nrows - c0, c1 - c0, [=](int i, int l) { return A[tri(c0 + i, d0 + l)] * A[tri(d0 + l, d0 + l)]; },
        [=](int l, int j) { return A[tri(c0 + j, d0 + l)]; }, [=](int) { return d1 - d0; },
        [](int i0, int j0) { return j0 <= i0; },
        [=](int i, int j, double v) {
            if (j <= i) A[tri(c0 + i, c0 + j)] -= v;
        },
        sA, sB);
#else
    tile_gemm_sub<true, true>(
        nrows - c0, c1 - c0, d1 - d0, [=](int i, int l) { return A[tri(c0 + i, d0 + l)] * A[tri(d0 + l, d0 + l)]; },
        [=](int l, int j) { return A[tri(c0 + j, d0 + l)]; }, [=](int i, int j) { return A + tri(c0 + i, c0 + j); },
        sA, sB);
#endif
}

// LDL^T of the packed bordered matrix (as ldlt_bordered) in panels of kWidePanel columns,
// three levels: inside a panel, 64-column sub-panels; inside those, 16-column blocks factored
// by ldlt_bordered_range (diagonal block + row solves); every level updates the rest of its
// enclosing range on the matrix cores (ldlt_rank_update, C tile loaded ahead of the products)
// -- the trailing matrix (L2/HBM-resident for large systems) is read and written once per
// kWidePanel columns.  Measured on the C5 sample's 292 spill users, 185k ratings
// (profiles/r03/spill_ldl_panel/, tools/probe_pspill_c5.py): one level of 64 / 128 / 32
// columns 6.56 / 6.41 / 7.79 s (at 128 the VALU panel took 42% of the LDL^T cycles); two
// levels 128 without / with the C preload 5.92 / 5.51 s; 64 / 256 / 512 with it 5.75 / 5.44 /
// 5.50 s; three levels at 256: 5.27 s.
// tsplit (diagnostics, thread 0's s_memtime, or null): [0] += panel cycles, [1] += trailing.
#ifndef CF_SPILL_LDL_PANEL
#define CF_SPILL_LDL_PANEL 256
#endif
constexpr int kWidePanel = CF_SPILL_LDL_PANEL;   // columns per trailing update (a multiple of 64)
static_assert(kWidePanel % 64 == 0, "panels are whole 64-column sub-panels");
template <int OCC = 1>
__device__ void ldlt_bordered_wide(double* A, int L, int nrows, double* sA, double* sB,
                                   unsigned long long* tsplit = nullptr) {
    for (int k0 = 0; k0 < L; k0 += kWidePanel) {
        const int k1 = min(L, k0 + kWidePanel);
        const unsigned long long t0 = tsplit ? __builtin_amdgcn_s_memtime() : 0ull;
        for (int p0 = k0; p0 < k1; p0 += 64) {
            const int p1 = min(k1, p0 + 64);
#ifndef CF_SPILL_LDL_TWO_LEVEL   // third level: 16-column blocks, the rest of the sub-panel on the matrix cores
            for (int q0 = p0; q0 < p1; q0 += 16) {
                const int q1 = min(p1, q0 + 16);
                ldlt_bordered_range<kT, kNB, OCC>(A, L, nrows, q0, q1);
                if (q1 < p1) ldlt_rank_update<OCC>(A, nrows, q0, q1, q1, p1, sA, sB);
            }
#else
            ldlt_bordered_range<kT, kNB, OCC>(A, L, nrows, p0, p1);
#endif
            if (p1 < k1) ldlt_rank_update<OCC>(A, nrows, p0, p1, p1, k1, sA, sB);
        }
        const unsigned long long t1 = tsplit ? __builtin_amdgcn_s_memtime() : 0ull;
        if (tsplit && threadIdx.x == 0) tsplit[0] += t1 - t0;
        if (k1 < L) ldlt_rank_update<OCC>(A, nrows, k0, k1, k1, L, sA, sB);
        if (tsplit && threadIdx.x == 0) tsplit[1] += __builtin_amdgcn_s_memtime() - t1;
    }
}

// ---- per-user tables ---------------------------------------------------------------------
// the complement basis's +-1 test matrix Omega(i, j): a hash of the user's content (k and three
// item ids), i and j
__device__ __forceinline__ uint32_t omega_mix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    h *= 0x846CA68Bu;
    return h ^ (h >> 16);
}
__device__ __forceinline__ uint32_t omega_seed(const uint32_t* it, int k) {
    return omega_mix(omega_mix(omega_mix((uint32_t)k * 0x9E3779B1u + 0x7F4A7C15u) ^ it[0]) ^ it[k >> 1]) ^ it[k - 1];
}
__device__ __forceinline__ double omega_pm1(uint32_t seed, int i, int j) {
    return (omega_mix(seed ^ ((uint32_t)i * 0x85EBCA6Bu) ^ ((uint32_t)j * 0xC2B2AE35u)) & 1u) ? 1.0 : -1.0;
}

template <typename T>
__global__ __launch_bounds__(kT) void spill_basis_kernel(SpArgs<T> a) {
    __shared__ double sA[2 * 16 * kSt], sB[2 * 16 * kSt];   // tile_gemm<.., 2>: two staging buffers
    __shared__ double s_ev[CF_SPILL_MAX_K];
    __shared__ int s_hdr[4];
    __shared__ float s_dev[kW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t s = a.s0 + blockIdx.x;
    const uint32_t u = a.order[a.first + s];
    const uint64_t base = a.item_off[u];
    const int k = (int)(a.item_off[u + 1] - base);
    const int m = a.m[u];
    const T* U = a.evecs + a.evec_off[u];
    const size_t kk2 = (size_t)k * k;   // slots are sized by the user's own k (soff)
    double* slot = a.ws + a.soff[s];
    double* Qb[2] = {slot, slot + kk2};
    double* Gb = slot + 2 * kk2;   // Gbar = U^T U over [0, Lu), full, ld Lu
    double* Gt = slot + 3 * kk2;   // Gram of the current Q (steps > 0)
    double* gh = slot + 4 * kk2;   // g[Lu], h[Lu], PG[k], PH[k]
    int* lim = a.wsi + a.sioff[s];
    int* cpos = lim + k;
    int* hdr = cpos + k;

    // the eigenvalues staged in LDS (m > CF_SPILL_MAX_K, uncapped users: read from HBM)
    const bool ev_lds = m <= CF_SPILL_MAX_K;   // uniform
    if (ev_lds)
        for (int j = tid; j < m; j += kT) s_ev[j] = (double)a.evals[base + j];
    if (tid == 0) s_hdr[0] = 2;
    __syncthreads();
    // lim = first eigenvalue index above w_lim, clamped to [2, m] (:271-282)
    for (int i = tid; i < k; i += kT) {
        const double w_lim = (double)a.sigtab[a.sig_mode == CF_SIGS_COMPAT ? (uint64_t)i : base + i];
        int l = m;
        for (int j = 0; j < m; ++j)
            if ((ev_lds ? s_ev[j] : (double)a.evals[base + j]) > w_lim) {
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
        tile_gemm<false, false, 2>(
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
        tile_gemm<true, false, 2>(
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
        __syncthreads();
        // P = Q Q^T over [0, Lu) (k x k, ld k) into the spare Q buffer; PG = Q g, PH = Q h
        double* P = Qb[cur ^ 1];
        tile_gemm<true, true, 2, true>(
            k, k, [=](int i, int l) { return Q[(size_t)i * Lu + l]; },
            [=](int l, int j) { return Q[(size_t)j * Lu + l]; }, [=](int) { return Lu; },
            [](int i0, int j0) { return j0 <= i0; },
            [=](int i, int j, double v) {
                if (j <= i) {
                    P[(size_t)i * k + j] = v;
                    P[(size_t)j * k + i] = v;
                }
            },
            sA, sB);
        double* pg = gh + 2 * Lu;
        for (int i = wave; i < k; i += kW) {
            const double* qi = Q + (size_t)i * Lu;
            double x = 0.0, y = 0.0;
            for (int j = lane; j < Lu; j += 64) {
                x = fma(qi[j], gh[j], x);
                y = fma(qi[j], gh[Lu + j], y);
            }
            x = wsum(x);
            y = wsum(y);
            if (lane == 0) {
                pg[i] = x;
                pg[k + i] = y;
            }
        }
    }
    // ---- complement basis W (k x du, du = k - Lu) of span(Q), for the G-mode of the
    // rank-deficient ratings (spill_predict_kernel): Y = (I - Q Q^T) Omega for a +-1 test matrix,
    // W = Y L^-T D^-1/2 from Y^T Y = L D L^T (Cholesky-QR), then W^T r and W^T 1 -- the basis of
    // cf_predict.hip's G-mode, here beside P.  Regions: W in Gt (ld du), Q^T Omega and the packed
    // Y^T Y after Gbar's Lu x Lu in Gb, W^T r / W^T 1 after PG / PH.
    const int du = k - Lu;
    int gm = 0;
    if (basis && du > 0) {
        const double* Q = Qb[cur];
        double* Wm = Gt;
        double* QO = Gb + (size_t)Lu * Lu;
        double* YY = QO + (size_t)Lu * du;
        __shared__ int s_fail;
        // Omega(i, j) = +-1 from a hash of the user's content (k and three item ids), i and j
        const uint32_t seed = omega_seed(a.items + base, k);
        const auto omega = [seed](int i, int j) -> double { return omega_pm1(seed, i, j); };
        tile_gemm<false, false, 2>(
            Lu, du, [=](int i, int l) { return Q[(size_t)l * Lu + i]; }, [=](int l, int j) { return omega(l, j); },
            [=](int) { return k; }, [](int, int) { return true; },
            [=](int i, int j, double v) { QO[(size_t)i * du + j] = v; }, sA, sB);
        tile_gemm<true, false, 2>(
            k, du, [=](int i, int l) { return Q[(size_t)i * Lu + l]; }, [=](int l, int j) { return QO[(size_t)l * du + j]; },
            [=](int) { return Lu; }, [](int, int) { return true; },
            [=](int i, int j, double v) { Wm[(size_t)i * du + j] = omega(i, j) - v; }, sA, sB);
        tile_gemm<false, false, 2, true>(
            du, du, [=](int i, int l) { return Wm[(size_t)l * du + i]; }, [=](int l, int j) { return Wm[(size_t)l * du + j]; },
            [=](int) { return k; }, [](int i0, int j0) { return j0 <= i0; },
            [=](int i, int j, double v) {
                if (j <= i) YY[tri(i, j)] = v;
            },
            sA, sB);
        ldlt_bordered_wide(YY, du, du, sA, sB);
        if (tid == 0) s_fail = 0;
        __syncthreads();
        double dmax = 0.0;
        for (int j = 0; j < du; ++j) dmax = fmax(dmax, YY[tri(j, j)]);
        bool fail = false;
        for (int i = tid; i < k; i += kT) {
            double* xi = Wm + (size_t)i * du;
            // forward substitution in 16-column register panels (cf_predict.hip's W solve)
            for (int p0 = 0; p0 < du; p0 += 16) {
                const int bw = min(16, du - p0);
                double acc[16];
                int rb[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    acc[q] = q < bw ? xi[p0 + q] : 0.0;
                    rb[q] = tri(p0 + min(q, bw - 1), 0);
                }
                for (int t = 0; t < p0; ++t) {
                    const double xt = xi[t];
#pragma unroll
                    for (int q = 0; q < 16; ++q) acc[q] = fma(-YY[rb[q] + t], xt, acc[q]);
                }
#pragma unroll
                for (int q = 1; q < 16; ++q)
#pragma unroll
                    for (int t = 0; t < q; ++t) acc[q] = fma(-YY[rb[q] + p0 + t], acc[t], acc[q]);
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    if (q < bw) xi[p0 + q] = acc[q];
            }
            for (int j = 0; j < du; ++j) {
                const double dj = YY[tri(j, j)];
                fail |= !(dj > 1e-12 * dmax);
                xi[j] = dj > 0.0 ? xi[j] / sqrt(dj) : 0.0;
            }
        }
        if (fail) s_fail = 1;
        __syncthreads();
        gm = s_fail == 0;
        if (gm) {   // W^T r, W^T 1
            double* gw = gh + 2 * (size_t)Lu + 2 * (size_t)k;
            for (int j = tid; j < du; j += kT) {
                double g = 0.0, h = 0.0;
                for (int i = 0; i < k; ++i) {
                    const double w = Wm[(size_t)i * du + j];
                    g = fma(w, (double)a.ratings[base + i], g);
                    h += w;
                }
                gw[j] = g;
                gw[du + j] = h;
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        hdr[0] = Lu;
        hdr[1] = basis;
        hdr[2] = cur;
        hdr[3] = gm;   // complement basis W ready: G-mode for c < lim
    }
}

// Multi-workgroup form of spill_basis_kernel for the largest users (k > kSmallCap): one
// workgroup per user left most of the chip idle on the C5 sample's 19 users with k > 2816
// (the basis kernel was 8.0 of the 10.1 s of their prediction, profiles/r05/
// pbig_kernel_stats_x2.csv).  One launch per phase, a.G workgroups per user: the output tiles of
// every tile product go to workgroup t % G, the rows / columns of the vector phases likewise.
// Every value comes from the same code as in the one-workgroup kernel (the same tile, the same
// sequential dot product, the same one-workgroup LDL^T), so the tables are bit-identical.
// Cross-workgroup state, in the slot header: hdr[0] Lu (atomicMax), [1] basis, [2] current Q,
// [3] G-mode ready, [4] the step's max |Gram - I| (float bits, atomicMax), [5] stepping done,
// [6] a Cholesky-QR pivot failure (atomicOr).
enum : int { kBmInit, kBmLim, kBmCopy, kBmGram, kBmApply, kBmStep, kBmGh, kBmP, kBmQO, kBmW, kBmYY, kBmLdl, kBmFs, kBmGw };
template <typename T>
__global__ __launch_bounds__(kT) void spill_basis_mc(SpArgs<T> a, int phase, int step) {
    __shared__ double sA[2 * 16 * kSt], sB[2 * 16 * kSt];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = a.G;
    const uint32_t s = blockIdx.x / G;
    const int g = (int)(blockIdx.x % G);
    const uint32_t u = a.order[a.first + s];
    const uint64_t base = a.item_off[u];
    const int k = (int)(a.item_off[u + 1] - base);
    const int m = a.m[u];
    const T* U = a.evecs + a.evec_off[u];
    const size_t kk2 = (size_t)k * k;
    double* slot = a.ws + a.soff[s];
    double* Qb[2] = {slot, slot + kk2};
    double* Gb = slot + 2 * kk2;
    double* Gt = slot + 3 * kk2;
    double* gh = slot + 4 * kk2;
    int* lim = a.wsi + a.sioff[s];
    int* cpos = lim + k;
    int* hdr = cpos + k;
    const int gt = g * kT + tid, gs = G * kT;   // rows / columns gt, gt + gs, ... are this thread's
    if (phase == kBmInit) {
        if (g == 0 && tid < 8) hdr[tid] = tid == 0 ? 2 : (tid == 1 ? 1 : 0);
        return;
    }
    if (phase == kBmLim) {   // lim = first eigenvalue index above w_lim, clamped to [2, m] (:271-282)
        for (int i = gt; i < k; i += gs) {
            const double w_lim = (double)a.sigtab[a.sig_mode == CF_SIGS_COMPAT ? (uint64_t)i : base + i];
            int l = m;
            for (int j = 0; j < m; ++j)
                if ((double)a.evals[base + j] > w_lim) {
                    l = j;
                    break;
                }
            l = min(max(l, 2), m);
            lim[i] = l;
            atomicMax(&hdr[0], l);
        }
        return;
    }
    const int Lu = hdr[0];
    if (phase == kBmCopy) {   // rows with U(i, j) >= 1e-4 per column j < Lu; Q0 = U(:, 0:Lu) in fp64
        for (int j = gt; j < Lu; j += gs) {
            int cnt = 0;
            for (int i = 0; i < k; ++i) {
                const double v = (double)U[(size_t)i * m + j];
                cnt += v >= 0.0001;
                Qb[0][(size_t)i * Lu + j] = v;
            }
            cpos[j] = cnt;
        }
        return;
    }
    if (phase == kBmStep) {   // the step's outcome (grid: one workgroup per user)
        if (tid != 0 || hdr[5] || !hdr[1]) return;
        const float dev = __int_as_float(hdr[4]);
        if (step == 0 && !(dev <= kOrthoMax)) {   // U far from orthonormal: dense path only
            hdr[1] = 0;
            hdr[5] = 1;
            return;
        }
        hdr[2] ^= 1;
        if (dev <= kOrthoDone) hdr[5] = 1;
        hdr[4] = 0;
        return;
    }
    if (phase == kBmGram || phase == kBmApply) {
        if (hdr[5] || !hdr[1]) return;
        const double* Q = Qb[hdr[2]];
        double* Gm = step == 0 ? Gb : Gt;
        if (phase == kBmGram) {
            float dev = 0.0f;
            tile_gemm<false, false, 2>(
                Lu, Lu, [=](int i, int l) { return Q[(size_t)l * Lu + i]; },
                [=](int l, int j) { return Q[(size_t)l * Lu + j]; }, [=](int) { return k; },
                [](int, int) { return true; },
                [&](int i, int j, double v) {
                    Gm[(size_t)i * Lu + j] = v;
                    dev = fmaxf(dev, (float)fabs(v - (i == j ? 1.0 : 0.0)));
                },
                sA, sB, g, G);
            for (int off = 32; off >= 1; off >>= 1) dev = fmaxf(dev, __shfl_xor(dev, off));
            if (lane == 0) atomicMax(&hdr[4], __float_as_int(dev));   // dev >= 0: int order = float order
            return;
        }
        if (step == 0 && !(__int_as_float(hdr[4]) <= kOrthoMax)) return;
        const double* Gr = Gm;
        double* Qn = Qb[hdr[2] ^ 1];
        tile_gemm<true, false, 2>(
            k, Lu, [=](int i, int l) { return Q[(size_t)i * Lu + l]; },
            [=](int l, int j) {
                const double gv = Gr[(size_t)l * Lu + j];
                return l < j ? -gv : (l == j ? 1.5 - 0.5 * gv : 0.0);
            },
            [=](int j0) { return min(Lu, j0 + 64); }, [](int, int) { return true; },
            [=](int i, int j, double v) { Qn[(size_t)i * Lu + j] = v; }, sA, sB, g, G);
        return;
    }
    if (!hdr[1]) return;   // no basis: no tables, no complement
    const int cur = hdr[2];
    const double* Q = Qb[cur];
    if (phase == kBmGh) {   // g = Q^T r, h = Q^T 1
        for (int j = gt; j < Lu; j += gs) {
            double gg = 0.0, h = 0.0;
            for (int i = 0; i < k; ++i) {
                const double q = Q[(size_t)i * Lu + j];
                gg = fma(q, (double)a.ratings[base + i], gg);
                h += q;
            }
            gh[j] = gg;
            gh[Lu + j] = h;
        }
        return;
    }
    if (phase == kBmP) {   // P = Q Q^T over [0, Lu) (k x k) into the spare Q buffer; PG = Q g, PH = Q h
        double* P = Qb[cur ^ 1];
        tile_gemm<true, true, 2, true>(
            k, k, [=](int i, int l) { return Q[(size_t)i * Lu + l]; },
            [=](int l, int j) { return Q[(size_t)j * Lu + l]; }, [=](int) { return Lu; },
            [](int i0, int j0) { return j0 <= i0; },
            [=](int i, int j, double v) {
                if (j <= i) {
                    P[(size_t)i * k + j] = v;
                    P[(size_t)j * k + i] = v;
                }
            },
            sA, sB, g, G);
        double* pg = gh + 2 * Lu;
        for (int i = g * kW + wave; i < k; i += G * kW) {
            const double* qi = Q + (size_t)i * Lu;
            double x = 0.0, y = 0.0;
            for (int j = lane; j < Lu; j += 64) {
                x = fma(qi[j], gh[j], x);
                y = fma(qi[j], gh[Lu + j], y);
            }
            x = wsum(x);
            y = wsum(y);
            if (lane == 0) {
                pg[i] = x;
                pg[k + i] = y;
            }
        }
        return;
    }
    // complement basis W (spill_basis_kernel's regions and arithmetic)
    const int du = k - Lu;
    if (du <= 0) return;
    double* Wm = Gt;
    double* QO = Gb + (size_t)Lu * Lu;
    double* YY = QO + (size_t)Lu * du;
    const uint32_t seed = omega_seed(a.items + base, k);
    const auto omega = [seed](int i, int j) -> double { return omega_pm1(seed, i, j); };
    if (phase == kBmQO) {
        tile_gemm<false, false, 2>(
            Lu, du, [=](int i, int l) { return Q[(size_t)l * Lu + i]; }, [=](int l, int j) { return omega(l, j); },
            [=](int) { return k; }, [](int, int) { return true; },
            [=](int i, int j, double v) { QO[(size_t)i * du + j] = v; }, sA, sB, g, G);
    } else if (phase == kBmW) {
        tile_gemm<true, false, 2>(
            k, du, [=](int i, int l) { return Q[(size_t)i * Lu + l]; }, [=](int l, int j) { return QO[(size_t)l * du + j]; },
            [=](int) { return Lu; }, [](int, int) { return true; },
            [=](int i, int j, double v) { Wm[(size_t)i * du + j] = omega(i, j) - v; }, sA, sB, g, G);
    } else if (phase == kBmYY) {
        tile_gemm<false, false, 2, true>(
            du, du, [=](int i, int l) { return Wm[(size_t)l * du + i]; }, [=](int l, int j) { return Wm[(size_t)l * du + j]; },
            [=](int) { return k; }, [](int i0, int j0) { return j0 <= i0; },
            [=](int i, int j, double v) {
                if (j <= i) YY[tri(i, j)] = v;
            },
            sA, sB, g, G);
    } else if (phase == kBmLdl) {
        if (g == 0) ldlt_bordered_wide(YY, du, du, sA, sB);
    } else if (phase == kBmFs) {   // forward substitution in 16-column register panels, then the scaling
        double dmax = 0.0;
        for (int j = 0; j < du; ++j) dmax = fmax(dmax, YY[tri(j, j)]);
        bool fail = false;
        for (int i = gt; i < k; i += gs) {
            double* xi = Wm + (size_t)i * du;
            for (int p0 = 0; p0 < du; p0 += 16) {
                const int bw = min(16, du - p0);
                double acc[16];
                int rb[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    acc[q] = q < bw ? xi[p0 + q] : 0.0;
                    rb[q] = tri(p0 + min(q, bw - 1), 0);
                }
                for (int t = 0; t < p0; ++t) {
                    const double xt = xi[t];
#pragma unroll
                    for (int q = 0; q < 16; ++q) acc[q] = fma(-YY[rb[q] + t], xt, acc[q]);
                }
#pragma unroll
                for (int q = 1; q < 16; ++q)
#pragma unroll
                    for (int t = 0; t < q; ++t) acc[q] = fma(-YY[rb[q] + p0 + t], acc[t], acc[q]);
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    if (q < bw) xi[p0 + q] = acc[q];
            }
            for (int j = 0; j < du; ++j) {
                const double dj = YY[tri(j, j)];
                fail |= !(dj > 1e-12 * dmax);
                xi[j] = dj > 0.0 ? xi[j] / sqrt(dj) : 0.0;
            }
        }
        if (fail) atomicOr(&hdr[6], 1);
    } else if (phase == kBmGw) {   // W^T r, W^T 1 when the Cholesky-QR had no failed pivot
        const int gm = hdr[6] == 0;
        if (gm) {
            double* gw = gh + 2 * (size_t)Lu + 2 * (size_t)k;
            for (int j = gt; j < du; j += gs) {
                double gg = 0.0, h = 0.0;
                for (int i = 0; i < k; ++i) {
                    const double w = Wm[(size_t)i * du + j];
                    gg = fma(w, (double)a.ratings[base + i], gg);
                    h += w;
                }
                gw[j] = gg;
                gw[du + j] = h;
            }
        }
        if (g == 0 && tid == 0) hdr[3] = gm;
    }
}

// ---- per-rating predictions --------------------------------------------------------------
// CAP: the largest k the per-row LDS arrays hold (0: the arrays in the workgroup's HBM rows);
// OCC: workgroups per CU.  Users with k <= kSmallCap take <kSmallCap, 2> (81 KB of LDS, 256
// registers: two ratings per CU overlap their latency-bound phases; one GEMM staging buffer),
// larger ones <0, 2> (per-row arrays in HBM, any k; 57 KB of LDS with two staging buffers).
// The r04 <5000, 1> instantiation (every array in LDS, 116 KB, one per CU) measured 3% slower
// on the C5 sample's k > 2816 users than <0, 2>, bit-identical (profiles/r05/big2_r1.log).
constexpr int kSmallCap = 2816;
#ifndef CF_PSPILL_ROWS_LDS
#define CF_PSPILL_ROWS_LDS 1   // (A/B: 0 = the G-mode rows read from the HBM row arrays)
#endif
template <typename T, int CAP, int OCC>
__global__ __launch_bounds__(kT, OCC) void spill_predict_kernel(SpArgs<T> a) {
    constexpr int kNbuf = (CAP == 0 || CAP > kSmallCap) ? 2 : 1;
    __shared__ double sA[kNbuf * 16 * kSt], sB[kNbuf * 16 * kSt];
    __shared__ double s_la[kLdsA];
    __shared__ float s_rat_l[CAP ? CAP : 1];
    __shared__ int s_conn_l[CAP ? CAP : 1];
    __shared__ int s_ncon_l[CAP ? CAP : 1];
    __shared__ int s_keep_l[CAP ? CAP : 1];
    // CAP = 0: the G-mode Gram's row list staged in LDS when it fits (its gathers then start
    // from an LDS read instead of a dependent global one)
    constexpr int kRowsLds = 4096;
    __shared__ int s_rows_l[CAP ? 1 : kRowsLds];
    uint32_t* const rows_g = CAP ? nullptr : a.rows + (size_t)blockIdx.x * 4 * a.rows_d;
    float* const s_rat = CAP ? s_rat_l : reinterpret_cast<float*>(rows_g);
    int* const s_conn = CAP ? s_conn_l : reinterpret_cast<int*>(rows_g + a.rows_d);
    int* const s_ncon = CAP ? s_ncon_l : reinterpret_cast<int*>(rows_g + 2 * a.rows_d);
    int* const s_keep = CAP ? s_keep_l : reinterpret_cast<int*>(rows_g + 3 * a.rows_d);
    __shared__ double s_misc[4];
    __shared__ int s_tmp[kW];
    __shared__ unsigned int s_item;
    __shared__ unsigned int s_slot;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double* fa = a.fa + (size_t)blockIdx.x * a.fa_d;
    const uint64_t total = a.w1;   // one work item per (slot, row); this launch's are [w0, w1)
    // Diagnostic counters (thread 0, s_memtime; no effect on outputs): cycles of
    // {0 sets + mean, 1 column filter, 2 P entries, 3 b and K, 4 Woodbury LDL^T, 5 dense
    // path}, counts {6 Woodbury, 7 dense, 8 sum nc (Woodbury), 9 np > 64,
    // 10 dense by dropped column, 11 dense by pivot}.
    unsigned long long pc[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};   // 12, 13: wide LDL^T panel / trailing
    unsigned long long pt = 0;
#define SP_STAMP(ph)                                                        \
    if (a.phase && tid == 0) {                                              \
        const unsigned long long now = __builtin_amdgcn_s_memtime();        \
        if ((ph) >= 0) pc[(ph) < 0 ? 0 : (ph)] += now - pt;                 \
        pt = now;                                                           \
    }
    for (;;) {
        if (tid == 0) {
            // claim an item, and find its slot in the chunk's row prefix (binary search)
            const uint32_t w = a.w0 + atomicAdd(a.counter, 1u);
            uint32_t lo = 0, hi = a.nu;
            if (w < total)
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (a.roff[mid] <= w) lo = mid;
                    else hi = mid;
                }
            s_item = w;
            s_slot = lo;
        }
        __syncthreads();
        const uint32_t w = s_item;
        const uint32_t s = s_slot;
        __syncthreads();
        if (w >= total) break;   // every wave of every block reaches this exit
        const int r = (int)(w - a.roff[s]);
        const uint32_t u = a.order[a.first + s];
        const uint64_t base = a.item_off[u];
        const int k = (int)(a.item_off[u + 1] - base);
        if (a.row_sel && !a.row_sel[base + r]) continue;   // --pct: movie not sampled (block-uniform)
        const int m = a.m[u];
        const T* U = a.evecs + a.evec_off[u];
        const size_t kk2 = (size_t)k * k;
        const double* slot = a.ws + a.soff[s];
        const int* lim_t = a.wsi + a.sioff[s];
        const int* cpos = lim_t + k;
        const int* hdr = cpos + k;
        const int Lu = hdr[0];
        const bool basis = hdr[1] != 0;
        const double* Q = slot + (hdr[2] ? kk2 : 0);
        const double* Pm = slot + (hdr[2] ? 0 : kk2);   // P = Q Q^T over [0, Lu), k x k
        const double* Gb = slot + 2 * kk2;
        const double* gvec = slot + 4 * kk2;
        const double* hvec = gvec + Lu;
        const double* pgv = gvec + 2 * Lu;   // (Q g)_a, then (Q h)_a at + k
        const int lim = lim_t[r];
        SP_STAMP(-1);

        // connected set C (:254-265); Cbar = the rest, the movie's own row r included
        const GraphRow nrow = a.graph.row(a.items[base + r]);
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
        SP_STAMP(0);
        bool fast = basis && c > 0;
        if (fast) {
            // zero-column filter: column j < lim is dropped iff no row of C has U(i, j) >= 1e-4,
            // i.e. every such row lies in Cbar -- counted over the smaller of the two sets (on
            // the k > 3072 users c is ~60 against nc ~ k: lim x nc loads per rating were the
            // whole cost of their prediction)
            bool drop = false;
            const bool via_c = c < nc;
            for (int j = tid; j < lim; j += kT) {
                if (via_c) {
                    bool hit = false;
                    for (int q = 0; q < c && !hit; ++q) hit = (double)U[(size_t)s_conn[q] * m + j] >= 0.0001;
                    drop |= !hit;
                } else if (cpos[j] <= nc) {
                    int hit = 0;
                    for (int q = 0; q < nc; ++q) hit += (double)U[(size_t)s_ncon[q] * m + j] >= 0.0001;
                    drop |= hit == cpos[j];
                }
            }
            fast = !__syncthreads_or(drop);
            if (!fast && a.phase && tid == 0) pc[10] += 1;
        }
        SP_STAMP(1);
        if (fast && c < lim && hdr[3] && k - lim < c) {
            // G-mode (cf_predict.hip): in the complement coordinates X = [Q | W] of the user's
            // basis, B = X[Cbar, lim:k] (nc x d, d = k - lim < c), h = g - B^T y_Cbar with
            // g = (X^T r - mean X^T 1)[lim:k]:  pred - mean = -w_r^T (B^T B)^-1 h, w_r = X[r, lim:k]
            // -- the same minimum-norm prediction as P_{r,C} P_CC^-1 y_C below, from a d x d
            // system instead of c x c (the k > 3072 users: d ~ 600 against c ~ 2000)
            const int d = k - lim, du = k - Lu;
            const double* Wm = slot + 3 * kk2;
            const double* gW = gvec + 2 * Lu + 2 * k;
            const double* hW = gW + du;
            const auto X = [&](int i, int col) -> double {
                return col < Lu ? Q[(size_t)i * Lu + col] : Wm[(size_t)i * du + (col - Lu)];
            };
            const size_t need = (size_t)(d + 2) * (d + 3) / 2;
            double* A = need <= (size_t)kLdsA ? s_la : fa;
            // one Gram pass over the rows of [X[., lim:k] | y] of the smaller of C and Cbar
            // (X has orthonormal columns, so X_Cbar^T X_Cbar = I - X_C^T X_C and
            // h = X_C^T y_C = g - X_Cbar^T y_Cbar): B^T B and, in its last row, h, which goes to
            // the packed border row d + 1 (row d: w_r).  The subtraction costs ~eps cond(B^T B),
            // the conditioning of the minimum-norm problem itself.
            const bool via_c = c < nc;
            const int nrow = via_c ? c : nc;
            const int* rows = via_c ? s_conn : s_ncon;
            if (CAP == 0 && CF_PSPILL_ROWS_LDS && nrow <= kRowsLds) {
                for (int i = tid; i < nrow; i += kT) s_rows_l[i] = rows[i];
                __syncthreads();
                rows = s_rows_l;
            }
            const auto By = [&](int l, int i) -> double {
                return i < d ? X(rows[l], lim + i) : (double)s_rat[rows[l]] - mu;
            };
            tile_gemm<false, false, kNbuf, true>(
                d + 1, d + 1, [&](int i, int l) { return By(l, i); }, [&](int l, int j) { return By(l, j); },
                [=](int) { return nrow; }, [](int i0, int j0) { return j0 <= i0; },
                [&](int i, int j, double v) {
                    if (j > i) return;
                    if (i < d) {
                        A[tri(i, j)] = via_c ? (i == j ? 1.0 : 0.0) - v : v;
                    } else if (j < d) {
                        const int col = lim + j;
                        A[tri(d + 1, j)] = via_c ? v
                                                 : (col < Lu ? gvec[col] - mu * hvec[col] : gW[col - Lu] - mu * hW[col - Lu]) - v;
                    }
                },
                sA, sB);
            for (int j = tid; j < d; j += kT) A[tri(d, j)] = X(r, lim + j);
            __syncthreads();
            SP_STAMP(2);
            ldlt_bordered_wide<OCC>(A, d, d + 2, sA, sB, a.phase ? pc + 12 : nullptr);
            if (wave == 0) {
                double dot = 0.0;
                for (int j = lane; j < d; j += 64) dot = fma(A[tri(d, j)] * A[tri(d + 1, j)], A[tri(j, j)], dot);
                dot = wsum(dot);
                if (lane == 0) s_misc[2] = dot;
            }
            __syncthreads();
            if (tid == 0) {
                double pred = mu - s_misc[2];
                if (pred > 5) pred = 5;
                if (pred < 1) pred = 1;
                const double dd = (double)s_rat[r] - pred;
                a.mse[base + r] = (float)(dd * dd);
                a.kk[base + r] = c;
                if (a.pred) a.pred[base + r] = pred;
                if (a.phase) {
                    pc[6] += 1;
                    pc[8] += d;
                }
            }
            __syncthreads();
            SP_STAMP(4);
            continue;
        }
        if (fast && c < lim) {
            // Underdetermined (c < lim): K = I - P_CbarCbar is singular (rank <= k - lim < nc)
            // and U_CS^T U_CS too.  The prediction is the minimum-norm least-squares one, as
            // the G-mode of cf_predict.hip returns it for k <= 192:
            //   pred - mean = P_{r,C} P_CC^-1 y_C,  P_CC = Q_CS Q_CS^T  (c x c),
            // the projector's block on the connected rows (full rank when U_CS has full row
            // rank; the same value as -w_r^T G^-1 h in the complement coordinates).  Its size
            // is c, which is small exactly when K-mode's nc is large.
            const size_t need = (size_t)(c + 2) * (c + 3) / 2;
            double* A = need <= (size_t)kLdsA ? s_la : fa;
            const auto pent = [&](int ia, int ib) {   // P over S = [0, lim)
                double v = Pm[(size_t)ia * k + ib];
                const double* xa = Q + (size_t)ia * Lu;
                const double* xb = Q + (size_t)ib * Lu;
                for (int j = lim; j < Lu; ++j) v = fma(-xa[j], xb[j], v);
                return v;
            };
            fill_tri_rows(A, c, [&](int ra, int cb) { return pent(s_conn[ra], s_conn[cb]); });
            for (int e = tid; e < 2 * c; e += kT) {
                if (e < c) A[tri(c, e)] = pent(r, s_conn[e]);
                else A[tri(c + 1, e - c)] = (double)s_rat[s_conn[e - c]] - mu;
            }
            __syncthreads();
            SP_STAMP(2);
            ldlt_bordered_wide<OCC>(A, c, c + 2, sA, sB, a.phase ? pc + 12 : nullptr);
            if (wave == 0) {
                double dot = 0.0;
                for (int j = lane; j < c; j += 64) dot = fma(A[tri(c, j)] * A[tri(c + 1, j)], A[tri(j, j)], dot);
                dot = wsum(dot);
                if (lane == 0) s_misc[2] = dot;
            }
            __syncthreads();
            if (tid == 0) {
                double pred = mu + s_misc[2];
                if (pred > 5) pred = 5;
                if (pred < 1) pred = 1;
                const double d = (double)s_rat[r] - pred;
                a.mse[base + r] = (float)(d * d);
                a.kk[base + r] = c;
                if (a.pred) a.pred[base + r] = pred;
                if (a.phase) {
                    pc[6] += 1;
                    pc[8] += c;
                }
            }
            __syncthreads();
            SP_STAMP(4);
            continue;
        }
        if (fast) {
            const int np = nc + 1;   // rows Cbar..., then r
            const size_t need = (size_t)(nc + 2) * (nc + 3) / 2;
            double* A = need <= (size_t)kLdsA ? s_la : fa;
            const auto rowid = [&](int q) { return q < np - 1 ? s_ncon[q] : r; };
            // E = P_S over rows [Cbar, r] into packed rows 0..nc, (P y)_a into row nc + 1:
            // gathers from P and PG/PH, less the (usually empty) tail of columns [lim, Lu)
            fill_tri_rows(A, np, [&](int ra, int cb) {
                const int ia = rowid(ra), ib = rowid(cb);
                double v = Pm[(size_t)ia * k + ib];
                const double* xa = Q + (size_t)ia * Lu;
                const double* xb = Q + (size_t)ib * Lu;
                for (int j = lim; j < Lu; ++j) v = fma(-xa[j], xb[j], v);
                return v;
            });
            for (int pa = tid; pa < np; pa += kT) {
                const int ia = rowid(pa);
                double v = pgv[ia] - mu * pgv[k + ia];
                const double* xa = Q + (size_t)ia * Lu;
                for (int j = lim; j < Lu; ++j) v = fma(-xa[j], gvec[j] - mu * hvec[j], v);
                A[tri(np, pa)] = v;
            }
            __syncthreads();
            SP_STAMP(2);
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
            fill_tri_rows(A, nc, [&](int ra, int cb) { return (cb == ra ? 1.0 : 0.0) - A[tri(ra, cb)]; });
            __syncthreads();
            SP_STAMP(3);
            ldlt_bordered_wide<OCC>(A, nc, nc + 2, sA, sB, a.phase ? pc + 12 : nullptr);
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
            SP_STAMP(4);
            if (a.phase && tid == 0) {
                if (fast) {
                    pc[6] += 1;
                    pc[8] += nc;
                    pc[9] += np > 64;
                } else {
                    pc[11] += 1;
                }
            }
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
        tile_gemm<false, false, kNbuf, true>(
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
        ldlt_bordered_wide<OCC>(A, L, L + 2, sA, sB);
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
        SP_STAMP(5);
        if (a.phase && tid == 0) pc[7] += 1;
    }
    if (a.phase && tid == 0)
        for (int x = 0; x < 14; ++x) atomicAdd(&a.phase[x], pc[x]);
#undef SP_STAMP
}

// ---- a8: local_calc's predictor for units with n > CF_MAX_K ----------------------------
// local_predict_kernel (cf_local.hip) with the bordered Gram matrix in HBM: per (movie,
// test user) pair, the rated rows C of the movie's n x n eigenvector block (row 0 = the
// movie, its rating unknown, :400-405), lim = first eigenvalue > w_lim (>= 2, :444-451),
// M = U_CS^T U_CS over S = [0, lim) with no zero-column filter (:455-485), pred = v^T
// M^-1 U_CS^T (r - mean) + mean with v = U(0, S), clamp, mse (float), kk = |C| (:487-521).
struct LocSpArgs {
    const uint32_t* pair_movie;
    const uint32_t* pair_user;
    const uint64_t* pair_out;
    const uint64_t* item_off;
    const uint32_t* items;
    const float* evals;
    const uint64_t* evec_off;
    const float* evecs;
    const float* wlim;
    const uint64_t* test_off;
    const uint32_t* test_user;
    const float* test_rating;
    float* mse;
    int32_t* kk;
    double* pred;
    int32_t* lim_out;
    uint32_t n_pairs;
    double* fa;
    size_t fa_d;
    unsigned int* counter;
    // units with n > CF_SPILL_MAX_K (local_calc has no neighbourhood cap): per-workgroup HBM rows
    // for the ratings and the rated-row list, rows_d entries each (null when no unit needs them)
    float* rat_h;
    int* c_h;
    size_t rows_d;
};

__global__ __launch_bounds__(kT) void local_predict_spill_kernel(LocSpArgs a) {
    __shared__ double sA[16 * kSt], sB[16 * kSt];
    __shared__ double s_la[kLdsA];
    __shared__ float s_rat_lds[CF_SPILL_MAX_K];
    __shared__ int s_c_lds[CF_SPILL_MAX_K];
    __shared__ double s_misc[4];
    __shared__ int s_tmp[kW];
    __shared__ int s_lim;
    __shared__ unsigned int s_item;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double* fa = a.fa + (size_t)blockIdx.x * a.fa_d;
    for (;;) {
        if (tid == 0) s_item = atomicAdd(a.counter, 1u);
        __syncthreads();
        const uint32_t p = s_item;
        __syncthreads();
        if (p >= a.n_pairs) break;   // every wave of every block reaches this exit
        const uint32_t mv = a.pair_movie[p];
        const uint32_t user = a.pair_user[p];
        const uint64_t base = a.item_off[mv];
        const int n = (int)(a.item_off[mv + 1] - base);
        const float* U = a.evecs + a.evec_off[mv];
        const bool rows_lds = n <= CF_SPILL_MAX_K;   // uniform
        float* s_rat = rows_lds ? s_rat_lds : a.rat_h + blockIdx.x * a.rows_d;
        int* s_c = rows_lds ? s_c_lds : a.c_h + blockIdx.x * a.rows_d;
        // ratings of the local graph's rows by this user; row 0 is the unknown (:400-405)
        for (int i = tid; i < n; i += kT) {
            const uint32_t it = a.items[base + i];
            uint64_t lo = a.test_off[it];
            const uint64_t end = a.test_off[it + 1];
            uint64_t hi = end;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (a.test_user[mid] < user) lo = mid + 1;
                else hi = mid;
            }
            const float v = (lo < end && a.test_user[lo] == user) ? a.test_rating[lo] : 0.0f;
            if (i == 0) s_misc[1] = (double)v;
            s_rat[i] = i == 0 ? 0.0f : v;
        }
        if (tid == 0) {
            const double wl = (double)a.wlim[p];
            int lim = 0;
            for (; lim < n; ++lim)
                if ((double)a.evals[base + lim] > wl) break;
            s_lim = lim < 2 ? 2 : lim;
        }
        __syncthreads();
        const int c = compact(n, [&](int i) { return s_rat[i] != 0.0f; }, s_c, s_tmp);   // (:470-479)
        const int L = s_lim;
        if (wave == 0) {
            double sum = 0.0;
            for (int i = lane; i < c; i += 64) sum += (double)s_rat[s_c[i]];
            sum = wsum(sum);
            if (lane == 0) s_misc[0] = sum / (double)c;   // 0/0 = NaN when nothing is rated (:487)
        }
        __syncthreads();
        const double mean = s_misc[0];
        if (c > 0 && c < L) {
            // U_CS^T U_CS (L x L) has rank <= c < L: singular, and the reference's explicit
            // inverse returns rounding noise (:490).  As the predictor does for c < lim, this
            // returns the minimum-norm least-squares prediction, from the c x c system of the
            // same rows: pred - mean = (U_CS v_S)^T K^-1 y_C, K = U_CS U_CS^T -- O(c^2 L)
            // instead of O(L^3) (units of thousands of rows rated by tens)
            const size_t needc = (size_t)(c + 2) * (c + 3) / 2;
            double* Ac = needc <= (size_t)kLdsA ? s_la : fa;
            tile_gemm<true, true>(
                c, c, [&](int i, int l) { return (double)U[(size_t)s_c[i] * n + l]; },
                [&](int l, int j) { return (double)U[(size_t)s_c[j] * n + l]; }, [=](int) { return L; },
                [](int i0, int j0) { return j0 <= i0; },
                [&](int i, int j, double v) {
                    if (j <= i) Ac[tri(i, j)] = v;
                },
                sA, sB);
            for (int q = wave; q < c; q += kW) {
                const float* row = U + (size_t)s_c[q] * n;
                double t = 0.0;
                for (int j = lane; j < L; j += 64) t = fma((double)row[j], (double)U[j], t);   // v = row 0
                t = wsum(t);
                if (lane == 0) {
                    Ac[tri(c, q)] = t;
                    Ac[tri(c + 1, q)] = (double)s_rat[s_c[q]] - mean;
                }
            }
            __syncthreads();
            ldlt_bordered_wide(Ac, c, c + 2, sA, sB);
            if (wave == 0) {
                double dot = 0.0;
                for (int j = lane; j < c; j += 64) dot = fma(Ac[tri(c, j)] * Ac[tri(c + 1, j)], Ac[tri(j, j)], dot);
                dot = wsum(dot);
                if (lane == 0) {
                    double pred = dot + mean;
                    if (pred > 5) pred = 5;
                    if (pred < 1) pred = 1;
                    const double d = s_misc[1] - pred;
                    const uint64_t o = a.pair_out[p];
                    a.mse[o] = (float)(d * d);
                    a.kk[o] = c;
                    if (a.pred) a.pred[o] = pred;
                    if (a.lim_out) a.lim_out[o] = L;
                }
            }
            __syncthreads();
            continue;
        }
        const size_t need = (size_t)(L + 2) * (L + 3) / 2;
        double* A = need <= (size_t)kLdsA ? s_la : fa;
        // bordered Gram: A[i][j] = (U_C^T U_C)_ij (j <= i < L), A[L][j] = t_j, A[L+1][j] = v_j
        tile_gemm<false, false>(
            L, L, [&](int i, int l) { return (double)U[(size_t)s_c[l] * n + i]; },
            [&](int l, int j) { return (double)U[(size_t)s_c[l] * n + j]; }, [=](int) { return c; },
            [](int i0, int j0) { return j0 <= i0; },
            [&](int i, int j, double v) {
                if (j <= i) A[tri(i, j)] = v;
            },
            sA, sB);
        for (int b = tid; b < L; b += kT) {
            double t = 0.0;
            for (int q = 0; q < c; ++q) {
                const int ri = s_c[q];
                t = fma((double)U[(size_t)ri * n + b], (double)s_rat[ri] - mean, t);
            }
            A[tri(L, b)] = t;
            A[tri(L + 1, b)] = (double)U[b];   // vv = row 0 (:465-466)
        }
        __syncthreads();
        ldlt_bordered_wide(A, L, L + 2, sA, sB);
        if (wave == 0) {
            double dot = 0.0;
            for (int j = lane; j < L; j += 64) dot = fma(A[tri(L, j)] * A[tri(L + 1, j)], A[tri(j, j)], dot);
            dot = wsum(dot);
            if (lane == 0) {
                double pred = dot + mean;
                if (pred > 5) pred = 5;   // (:494-497)
                if (pred < 1) pred = 1;
                const double d = s_misc[1] - pred;
                const uint64_t o = a.pair_out[p];
                a.mse[o] = (float)(d * d);
                a.kk[o] = c;
                if (a.pred) a.pred[o] = pred;
                if (a.lim_out) a.lim_out[o] = L;
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
                            int sig_mode, float* d_mse, int32_t* d_kk, double* d_pred, const uint8_t* d_row_sel,
                            hipStream_t stream) {
    if (b.count == 0) return CF_OK;
    const int kmax = (int)b.kmax;
    // k > CF_SPILL_MAX_K (no cap, as the reference): those users' predict workgroups keep their
    // per-row arrays in HBM (the <T, 0, 1> kernel)
    SpArgs<T> a{};
    a.order = plan->d_order;
    a.kmax = kmax;
    a.item_off = d_item_off;
    a.items = d_items;
    a.ratings = d_ratings;
    a.row_sel = d_row_sel;
    a.m = d_m;
    a.evals = d_evals;
    a.evec_off = d_evec_off;
    a.evecs = d_evecs;
    a.sigtab = d_sigtab;
    a.sig_mode = sig_mode;
    a.graph = graph_dev(ctx);
    a.n_items = ctx->n_items;
    a.mse = d_mse;
    a.kk = d_kk;
    a.pred = d_pred;
    a.phase = ctx->d_phase;
    // workspace: counter | chunk tables | factorisation regions | user slots (doubles) | slot
    // ints.  Every user's slot is sized by its OWN k (4 k^2 + 4 k doubles, 2 k + 4 ints): a
    // config-5 bucket spans k = 193 .. 5000, and kmax-sized slots would hold ~100x fewer users.
    a.fa_d = (size_t)(kmax + 2) * (kmax + 3) / 2;
    // slots: as many users per chunk as a third of this context's share of the free HBM holds
    // (288 GB per GPU: all of a config-5 shard's spill users at once, so the basis launch fills
    // the chip), >= 8 GB; factorisation regions: a tenth of it (>= 4 GB), 32 .. 512 persistent
    // workgroups.  The floors never exceed half the share (cf_hbm_budget); if the allocation
    // still fails (another process or context took the memory meanwhile) both budgets halve
    // and the chunks are planned again.
    size_t kSlotBudget = cf_hbm_budget(ctx, ctx->pspill_bytes, 1.0 / 3.0, (size_t)8 << 30);
    // CF_PSPILL_BASIS_MC=0: every user's basis on the one-workgroup kernel (A/B)
    static const bool basis_mc = [] {
        const char* e = getenv("CF_PSPILL_BASIS_MC");
        return !(e && e[0] == '0');
    }();
    static const int basis_mc_min = [] {   // users above this k take spill_basis_mc (A/B: CF_PSPILL_BASIS_MC_MIN)
        const char* e = getenv("CF_PSPILL_BASIS_MC_MIN");
        return e ? atoi(e) : 768;
    }();
    static const uint32_t basis_mc_w = [] {   // its workgroups per CU over those users (A/B: CF_PSPILL_BASIS_MC_W)
        const char* e = getenv("CF_PSPILL_BASIS_MC_W");
        return e ? (uint32_t)std::max(1, atoi(e)) : 4u;
    }();
    int n_cu = 256;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, ctx->device);
    // (k > kSmallCap: a fifth, so that the two-per-CU kernel gets ~2 regions per CU at k = 5000)
    size_t kFaBudget = cf_hbm_budget(ctx, ctx->pspill_bytes, kmax > (uint64_t)kSmallCap ? 0.2 : 0.1, (size_t)4 << 30);
    // chunks over the bucket's users (plan order: largest k first), each within the budget
    struct Chunk {
        uint32_t u0, nu;
        size_t meta;   // index of its tables in `meta` (3 x (nu + 1))
    };
    std::vector<Chunk> chunks;
    std::vector<uint64_t> meta;
    int blocks = 0;
    size_t fa_bytes = 0, meta_bytes = 0, ws_bytes = 0, rows_bytes = 0;
    a.rows_d = kmax > (uint64_t)kSmallCap ? ((size_t)kmax + 63) / 64 * 64 : 0;
    // at least 32 regions (8 when one region is over 1 GB: k > ~16k)
    const size_t min_blocks = a.fa_d * sizeof(double) > ((size_t)1 << 30) ? 8 : 32;
    for (;;) {
        blocks = (int)std::max<size_t>(min_blocks, std::min<size_t>(512, kFaBudget / (a.fa_d * 8)));
        fa_bytes = (size_t)blocks * a.fa_d * sizeof(double);
        rows_bytes = (size_t)blocks * 4 * a.rows_d * sizeof(uint32_t);
        chunks.clear();
        meta.clear();
        size_t ws_max = 0, wsi_max = 0;
        for (uint32_t u0 = 0; u0 < b.count;) {
            Chunk c{u0, 0, meta.size()};
            uint64_t sd = 0, si = 0, rows = 0;
            std::vector<uint64_t> t_sd{0}, t_si{0}, t_r{0};
            while (u0 + c.nu < b.count) {
                const uint32_t u = plan->h_order[b.first + u0 + c.nu];
                const uint64_t k = plan->h_item_off[u + 1] - plan->h_item_off[u];
                const uint64_t d = 4 * k * k + 4 * k;
                if (c.nu > 0 && (sd + d) * sizeof(double) > kSlotBudget) break;
                sd += d;
                si += 2 * k + 8;
                rows += k;
                t_sd.push_back(sd);
                t_si.push_back(si);
                t_r.push_back(rows);
                ++c.nu;
            }
            meta.insert(meta.end(), t_sd.begin(), t_sd.end());
            meta.insert(meta.end(), t_si.begin(), t_si.end());
            meta.insert(meta.end(), t_r.begin(), t_r.end());
            ws_max = std::max(ws_max, (size_t)sd);
            wsi_max = std::max(wsi_max, (size_t)si);
            chunks.push_back(c);
            u0 += c.nu;
        }
        meta_bytes = ((meta.size() * sizeof(uint64_t) + 255) / 256) * 256;
        ws_bytes = ws_max * sizeof(double);
        const size_t need = 256 + meta_bytes + fa_bytes + rows_bytes + ws_bytes + wsi_max * sizeof(int);
        if (need <= ctx->pspill_bytes) break;
        if (ctx->d_pspill) {
            CF_HIP_CHECK(ctx, hipStreamSynchronize(stream));   // earlier launches may still read it
            (void)hipFree(ctx->d_pspill);
        }
        ctx->d_pspill = nullptr;
        ctx->pspill_bytes = 0;
        if (hipMalloc(&ctx->d_pspill, need) == hipSuccess) {
            ctx->pspill_bytes = need;
            break;
        }
        (void)hipGetLastError();
        ctx->d_pspill = nullptr;
        // one user per chunk and the fewest regions is the smallest plan there is
        if ((size_t)blocks == min_blocks && std::all_of(chunks.begin(), chunks.end(), [](const Chunk& c) { return c.nu == 1; }))
            return cf_set_error(ctx, CF_ENOMEM, "spill predictor workspace (" + std::to_string(need) + " bytes)");
        kSlotBudget /= 2;
        kFaBudget /= 2;
    }
    char* p = reinterpret_cast<char*>(ctx->d_pspill);
    a.counter = reinterpret_cast<unsigned int*>(p);
    uint64_t* d_meta = reinterpret_cast<uint64_t*>(p + 256);
    a.fa = reinterpret_cast<double*>(p + 256 + meta_bytes);
    a.rows = reinterpret_cast<uint32_t*>(p + 256 + meta_bytes + fa_bytes);
    a.ws = reinterpret_cast<double*>(p + 256 + meta_bytes + fa_bytes + rows_bytes);
    a.wsi = reinterpret_cast<int*>(p + 256 + meta_bytes + fa_bytes + rows_bytes + ws_bytes);
    // the tables go up in one asynchronous copy from the context's pinned staging buffer; the
    // previous call's copy out of it has completed before it is overwritten (its event)
    const size_t meta_n = meta.size() * sizeof(uint64_t);
    if (ctx->pspill_meta_ev) CF_HIP_CHECK(ctx, hipEventSynchronize(ctx->pspill_meta_ev));
    else CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&ctx->pspill_meta_ev, hipEventDisableTiming));
    if (meta_n > ctx->pspill_meta_bytes) {
        if (ctx->h_pspill_meta) (void)hipHostFree(ctx->h_pspill_meta);
        ctx->h_pspill_meta = nullptr;
        ctx->pspill_meta_bytes = 0;
        CF_HIP_CHECK(ctx, hipHostMalloc(&ctx->h_pspill_meta, meta_n));
        ctx->pspill_meta_bytes = meta_n;
    }
    std::memcpy(ctx->h_pspill_meta, meta.data(), meta_n);
    CF_HIP_CHECK(ctx, hipMemcpyAsync(d_meta, ctx->h_pspill_meta, meta_n, hipMemcpyHostToDevice, stream));
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->pspill_meta_ev, stream));
    for (const Chunk& c : chunks) {
        a.first = b.first + c.u0;
        a.nu = c.nu;
        a.soff = d_meta + c.meta;
        a.sioff = a.soff + (c.nu + 1);
        a.roff = a.sioff + (c.nu + 1);
        const uint64_t* roff_h = meta.data() + c.meta + 2 * (c.nu + 1);
        const uint64_t items = roff_h[c.nu];
        // users are largest k first: [0, nb) need the full-capacity kernel, [nb, nu) fit the small one
        const auto k_of = [&](uint32_t i) {
            const uint32_t u = plan->h_order[b.first + c.u0 + i];
            return plan->h_item_off[u + 1] - plan->h_item_off[u];
        };
        uint32_t nb = 0;
        while (nb < c.nu && k_of(nb) > (uint64_t)kSmallCap) ++nb;
        CF_HIP_CHECK(ctx, hipMemsetAsync(a.counter, 0, 256, stream));
        // the basis: the largest users on spill_basis_mc (about four workgroups per CU over them,
        // one launch per phase; 1 / 2 / 4 / 8 per CU: 2742 / 2670 / 2632 / 2643 ms on the C5
        // sample's k > 2816 users, 665 / 495 / 414 / 395 ms on its 192 < k <= 3072 ones,
        // profiles/r05/bw_*_ah{1,2}.log), the rest one workgroup each
        // (every k > kSmallCap user, and the largest users above basis_mc_min up to one per CU:
        // C5 sample's 192 < k <= 3072 group 1610 -> 496 ms at 768, profiles/r05/bmin_*_af1.log)
        uint32_t nbm = 0;
        if (basis_mc) {
            uint32_t n_min = 0;
            while (n_min < c.nu && k_of(n_min) > (uint64_t)basis_mc_min) ++n_min;
            nbm = std::max(nb, std::min(n_min, (uint32_t)n_cu));
        }
        if (nbm > 0) {
            SpArgs<T> am = a;
            am.G = (int)std::max<uint32_t>(1, std::min<uint32_t>(64, (basis_mc_w * (uint32_t)n_cu + nbm - 1) / nbm));
            SpArgs<T> a1 = a;
            a1.G = 1;
            const dim3 gm(nbm * (uint32_t)am.G), g1(nbm);
            hipLaunchKernelGGL(spill_basis_mc<T>, g1, dim3(kT), 0, stream, a1, (int)kBmInit, 0);
            hipLaunchKernelGGL(spill_basis_mc<T>, gm, dim3(kT), 0, stream, am, (int)kBmLim, 0);
            hipLaunchKernelGGL(spill_basis_mc<T>, gm, dim3(kT), 0, stream, am, (int)kBmCopy, 0);
            for (int step = 0; step < kMaxSteps; ++step) {
                hipLaunchKernelGGL(spill_basis_mc<T>, gm, dim3(kT), 0, stream, am, (int)kBmGram, step);
                hipLaunchKernelGGL(spill_basis_mc<T>, gm, dim3(kT), 0, stream, am, (int)kBmApply, step);
                hipLaunchKernelGGL(spill_basis_mc<T>, g1, dim3(kT), 0, stream, a1, (int)kBmStep, step);
            }
            for (int ph : {(int)kBmGh, (int)kBmP, (int)kBmQO, (int)kBmW, (int)kBmYY, (int)kBmLdl, (int)kBmFs, (int)kBmGw})
                if (ph == kBmLdl) hipLaunchKernelGGL(spill_basis_mc<T>, g1, dim3(kT), 0, stream, a1, ph, 0);
                else hipLaunchKernelGGL(spill_basis_mc<T>, gm, dim3(kT), 0, stream, am, ph, 0);
            CF_HIP_CHECK(ctx, hipGetLastError());
        }
        if (c.nu > nbm) {
            SpArgs<T> ab = a;
            ab.s0 = nbm;
            hipLaunchKernelGGL(spill_basis_kernel<T>, dim3(c.nu - nbm), dim3(kT), 0, stream, ab);
            CF_HIP_CHECK(ctx, hipGetLastError());
        }
        const uint64_t split = roff_h[nb];
        if (split > 0) {   // k > kSmallCap: per-row arrays in HBM, two workgroups per CU, heaviest first
            SpArgs<T> ab = a;
            ab.w0 = 0;
            ab.w1 = (uint32_t)split;
            hipLaunchKernelGGL((spill_predict_kernel<T, 0, 2>), dim3((unsigned)std::min<uint64_t>(blocks, split)),
                               dim3(kT), 0, stream, ab);
            CF_HIP_CHECK(ctx, hipGetLastError());
        }
        if (items > split) {
            SpArgs<T> as = a;
            as.counter = a.counter + 32;   // its own zeroed counter (another 128-byte line)
            as.w0 = (uint32_t)split;
            as.w1 = (uint32_t)items;
            hipLaunchKernelGGL((spill_predict_kernel<T, kSmallCap, 2>),
                               dim3((unsigned)std::min<uint64_t>(blocks, items - split)), dim3(kT), 0, stream, as);
            CF_HIP_CHECK(ctx, hipGetLastError());
        }
    }
    return CF_OK;
}

template int cf_launch_predict_spill<float>(cf_ctx*, const cf_plan*, const cf_bucket&, const uint64_t*,
                                            const uint32_t*, const float*, const int32_t*, const float*,
                                            const uint64_t*, const float*, const float*, int, float*, int32_t*,
                                            double*, const uint8_t*, hipStream_t);
template int cf_launch_predict_spill<double>(cf_ctx*, const cf_plan*, const cf_bucket&, const uint64_t*,
                                             const uint32_t*, const float*, const int32_t*, const double*,
                                             const uint64_t*, const double*, const double*, int, float*,
                                             int32_t*, double*, const uint8_t*, hipStream_t);

int cf_launch_local_predict_spill(cf_ctx* ctx, uint32_t n_pairs, int nmax, const uint32_t* d_pair_movie,
                                  const uint32_t* d_pair_user, const uint64_t* d_pair_out, const uint64_t* d_item_off,
                                  const uint32_t* d_items, const float* d_evals, const uint64_t* d_evec_off,
                                  const float* d_evecs, const float* d_wlim, const uint64_t* d_test_off,
                                  const uint32_t* d_test_user, const float* d_test_rating, float* d_mse,
                                  int32_t* d_kk, double* d_pred, int32_t* d_lim, hipStream_t stream) {
    if (n_pairs == 0) return CF_OK;
    LocSpArgs a{};
    a.pair_movie = d_pair_movie;
    a.pair_user = d_pair_user;
    a.pair_out = d_pair_out;
    a.item_off = d_item_off;
    a.items = d_items;
    a.evals = d_evals;
    a.evec_off = d_evec_off;
    a.evecs = d_evecs;
    a.wlim = d_wlim;
    a.test_off = d_test_off;
    a.test_user = d_test_user;
    a.test_rating = d_test_rating;
    a.mse = d_mse;
    a.kk = d_kk;
    a.pred = d_pred;
    a.lim_out = d_lim;
    a.n_pairs = n_pairs;
    a.fa_d = (size_t)(nmax + 2) * (nmax + 3) / 2;
    const int blocks = (int)std::min<size_t>(
        n_pairs, std::max<size_t>(32, std::min<size_t>(512, ((size_t)4 << 30) / (a.fa_d * 8))));
    a.rows_d = nmax > CF_SPILL_MAX_K ? ((size_t)nmax + 63) / 64 * 64 : 0;
    const size_t fa_bytes = (size_t)blocks * a.fa_d * sizeof(double);
    const size_t need = 256 + fa_bytes + (size_t)blocks * a.rows_d * (sizeof(float) + sizeof(int));
    if (need > ctx->pspill_bytes) {
        if (ctx->d_pspill) (void)hipFree(ctx->d_pspill);
        ctx->d_pspill = nullptr;
        ctx->pspill_bytes = 0;
        CF_HIP_CHECK(ctx, hipMalloc(&ctx->d_pspill, need));
        ctx->pspill_bytes = need;
    }
    a.counter = reinterpret_cast<unsigned int*>(ctx->d_pspill);
    a.fa = reinterpret_cast<double*>(static_cast<char*>(ctx->d_pspill) + 256);
    if (a.rows_d) {
        a.rat_h = reinterpret_cast<float*>(static_cast<char*>(ctx->d_pspill) + 256 + fa_bytes);
        a.c_h = reinterpret_cast<int*>(a.rat_h + (size_t)blocks * a.rows_d);
    }
    CF_HIP_CHECK(ctx, hipMemsetAsync(a.counter, 0, sizeof(unsigned int), stream));
    hipLaunchKernelGGL(local_predict_spill_kernel, dim3(blocks), dim3(kT), 0, stream, a);
    CF_HIP_CHECK(ctx, hipGetLastError());
    return CF_OK;
}
