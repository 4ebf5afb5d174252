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
// All arithmetic after the gather is fp64 (the reference's double path).
//
// Fast path (per user, then one wave per rating).  The prediction is the value at row
// r of the least-squares fit of r_C - mean on span(U_CS): it depends on U_S only
// through an orthonormal basis Q_S of its column span.  Once per user:
//   Gbar = U^T U over the columns [0, Lu), Lu = max_r lim_r;
//   Q = U T1 T2 with T = I - su(G - I) - diag(G - I) / 2 (su = strictly upper part),
//   T1 from Gbar and T2 from (U T1)^T (U T1).  U is near-orthonormal (eigenvectors:
//   |Gbar - I| ~ 1e-6), each step squares the orthogonality error (1e-6 -> 1e-12 ->
//   1e-24), and T1, T2 are upper triangular, so the leading lim columns of Q span the
//   leading lim columns of U and one Q serves every row's prefix S = [0, lim).  All
//   four products are tiled GEMM-shaped work (no sequential factorisation);
//   g = Q^T r, h = Q^T 1, the prefix tables PG(i, l) = sum_{j<l} Q_ij g_j,
//   PH(i, l) = sum_{j<l} Q_ij h_j, and the projector P = Q Q^T (k x k).
// With P = Q_S Q_S^T (the k x k projector), Cbar = rows not in C (nc of them),
// y = r - mean, and Q_S^T Q_S = I:
//   pred - mean = a_r + P_{r,Cbar} K^-1 b,   K = I - P_{Cbar,Cbar}  (nc x nc),
//   a_r = (P y)_r - P_{r,Cbar} y_Cbar,   b = (P y)_Cbar - P_{Cbar,Cbar} y_Cbar,
// (Woodbury on U_CS^T U_CS = Q_S^T Q_S - Q_CbarS^T Q_CbarS), where (P y)_i =
// PG(i, lim) - mean PH(i, lim).  lim is all but constant within a user (mean Lu - lim
// = 0.08 on the C2 workload), so the entries of P_S = P - sum_{j in [lim, Lu)} Q_j Q_j^T
// are gathers from P with a (usually empty) tail correction.  A rating therefore costs
// (nc + 1)(nc + 2) / 2 gathers and an nc x nc LDL^T instead of a lim x lim
// factorisation.
//
// Dense path (block-wide, the rating's own Gram matrix) for the ratings the fast path
// does not take: the column filter drops a column, nc > kNcMax, c = 0, a pivot of K
// below kPivMin while c >= lim (full rank but ill-conditioned: U_CS^T U_CS has an
// eigenvalue < kPivMin), or U is not near-orthonormal (max |Gbar - I| > kOrthoMax: no
// Q for this user).
// It factors M = U_CS^T U_CS = L D L^T (blocked, right-looking, packed lower triangle
// in LDS), bordered by t^T and v^T so the factorisation itself yields L^-1 t and
// L^-1 v and pred = sum_j (L^-1 v)_j (L^-1 t)_j / D_j + mean.  When the complement is
// smaller it forms M as Gbar_SS - sum_{i not in C} u_i u_i^T.  Like Gaussian
// elimination (and unlike Cholesky) LDL^T carries on through negative pivots, so a
// numerically indefinite, near-singular M gives the same kind of finite, clamped
// garbage as the reference's inverse (:314) instead of a NaN.

#include "cf_internal.h"
#include "cf_ldlt.hpp"   // block-wide systems here use 8-column panels (measured: 16 -> 8 is
                           // 164.3 -> 160.0 ms at C2; the spill paths keep 16)

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kNcMax = 62;            // fast path: complement rows (nc + 2 border rows <= 64 lanes)
// fast path: smallest pivot of K = I - P_CbarCbar (its pivots bound the smallest
// eigenvalue of U_CS^T U_CS in the Q basis, so this admits cond <~ 1e10, where the
// reference's own explicit inverse is accurate to ~cond * eps; parity is tested to 1e8)
constexpr double kPivMin = 1e-10;
// max |Gbar - I| for a basis: each correction step squares the orthogonality error, and
// steps repeat (up to 4) until the last Gram is within kOrthoDone, so Q is orthonormal to
// ~1e-16 for any U within kOrthoMax of orthonormal
constexpr double kOrthoMax = 1e-2;
constexpr float kOrthoDone = 1e-8f;

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
    int ncw;               // fast-path bound on nc for this launch
    int ew;                // doubles of per-wave fast-path matrix E / K
    int a_elems;           // doubles of the shared factorisation / scratch region
    double* gbar;          // per-block scratch: Gbar = U^T U (lmax x lmax, full), fp64
    double* qs;            // per-block scratch: Q ((lmax + 2) x lmax rows: Q, g, h), fp64
    double* q1;            // per-block scratch: U T1, then P = Q Q^T (lmax x lmax), fp64
    double* pgh;           // per-block scratch: {PG, PH}(i, l), lmax x (lmax + 1) pairs, fp64
    double* abig;          // per-block HBM region of the block-wide systems (when !big_lds)
    size_t abig_elems;     // (lmax + 2)(lmax + 3) / 2
    int big_lds;           // 1: the block-wide systems use the LDS region A
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

// Block-level GEMM on 64 x 64 output blocks: C(i, j) = sum_{l < kend(j0)} A(i, l) B(l, j)
// for i < M, j < N, over the blocks (i0, j0) with want(i0, j0).  A(i, l) =
// xA(i, l, loadA(i, l)) and likewise B: load* only reads memory, x* converts / applies
// a formula, so the loads of the next 16-deep chunk stay in flight (raw, in registers)
// while the current chunk -- staged in LDS as fp64 (`stage`: kStageElems doubles) with
// coalesced loads -- is consumed; the conversions run when the chunk is written to LDS.
// A_LFAST / B_LFAST say whether l is the operand's contiguous index in memory.  The
// products run on the fp64 matrix cores: wave w owns the 32 x 32 quadrant (w >> 1,
// w & 1) of the block as 2 x 2 v_mfma_f64_16x16x4_f64 tiles (A lane l = A[l&15][l>>4],
// B lane l = B[l>>4][l&15], result q of lane l = C[(l>>4) + 4q][l&15]; checked by
// tools/mfma_f64_probe.hip), so a 16-deep chunk costs each wave 16 LDS fragment reads for
// 16 MFMAs -- an eighth of the LDS traffic of 4 x 4 VALU register tiles.  Called by the
// whole block; the caller synchronises before reading C.
constexpr int kStageLd = 80;                       // == 16 (mod 32): the four 16-lane row
                                                   // groups of a fragment read hit disjoint banks
constexpr int kStageElems = 2 * 16 * kStageLd;
using f64x4 = __attribute__((ext_vector_type(4))) double;
template <bool A_LFAST, bool B_LFAST, class LA, class XA, class LB, class XB, class FK, class FW, class FO>
__device__ void block_gemm(int M, int N, LA loadA, XA xA, LB loadB, XB xB, FK kend, FW want, FO out,
                           double* stage) {
    double* As = stage;
    double* Bs = stage + 16 * kStageLd;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wr = (tid >> 6) >> 1, wc = (tid >> 6) & 1;   // this wave's 32 x 32 quadrant
    using RA = decltype(loadA(0, 0));
    using RB = decltype(loadB(0, 0));
    for (int i0 = 0; i0 < M; i0 += 64)
        for (int j0 = 0; j0 < N; j0 += 64) {
            if (!want(i0, j0)) continue;
            const int K = kend(j0);
            f64x4 acc[2][2];
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y) acc[x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
            RA ra[4];
            RB rb[4];
            // unconditional loads from clamped indices: a guarded load would become a
            // branch with its own wait (one full latency per load)
            auto fetch = [&](int l0) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int e = tid + kThreads * t;
                    const int ia = A_LFAST ? (e >> 4) : (e & 63), la = A_LFAST ? (e & 15) : (e >> 6);
                    const int jb = B_LFAST ? (e >> 4) : (e & 63), lb = B_LFAST ? (e & 15) : (e >> 6);
                    ra[t] = loadA(min(i0 + ia, M - 1), min(l0 + la, K - 1));
                    rb[t] = loadB(min(l0 + lb, K - 1), min(j0 + jb, N - 1));
                }
            };
            if (K > 0) fetch(0);
            for (int l0 = 0; l0 < K; l0 += 16) {
                __syncthreads();   // the previous chunk is consumed
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int e = tid + kThreads * t;
                    const int ia = A_LFAST ? (e >> 4) : (e & 63), la = A_LFAST ? (e & 15) : (e >> 6);
                    const int jb = B_LFAST ? (e >> 4) : (e & 63), lb = B_LFAST ? (e & 15) : (e >> 6);
                    const bool oka = i0 + ia < M && l0 + la < K;
                    const bool okb = j0 + jb < N && l0 + lb < K;
                    As[la * kStageLd + ia] = oka ? xA(i0 + ia, l0 + la, ra[t]) : 0.0;
                    Bs[lb * kStageLd + jb] = okb ? xB(l0 + lb, j0 + jb, rb[t]) : 0.0;
                }
                __syncthreads();
                if (l0 + 16 < K) fetch(l0 + 16);
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const int row = (4 * ks + (lane >> 4)) * kStageLd + (lane & 15);
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
                            acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[x], bv[y], acc[x][y], 0, 0, 0);
                }
            }
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int i = i0 + 32 * wr + 16 * x + (lane >> 4) + 4 * q;
                        const int j = j0 + 32 * wc + 16 * y + (lane & 15);
                        if (i < M && j < N) out(i, j, acc[x][y][q]);
                    }
        }
}

template <typename T>
__global__ __launch_bounds__(kThreads, 2) void predict_kernel(PredArgs<T> a, uint32_t count) {
    extern __shared__ double dsm[];
    const int lmax = a.lmax;
    // A: the factorisation region.  Per user it holds Gbar's LDL^T, then the per-wave
    //    fast-path scratch, then (dense path) the packed lower triangle of the bordered
    //    matrix [[M, .], [t^T, .], [v^T, .]] ((lmax + 2) rows).
    double* A = dsm;
    double* s_misc = A + a.a_elems;   // [0] mean (dense path), [1] sum of the user's ratings
    uint32_t* s_item = reinterpret_cast<uint32_t*>(s_misc + 4);
    float* s_rat = reinterpret_cast<float*>(s_item + CF_MAX_K);
    int* s_conn = reinterpret_cast<int*>(s_rat + CF_MAX_K);
    int* s_keep = s_conn + CF_MAX_K;
    int* s_nconn = s_keep + CF_MAX_K;                      // rows NOT in C (complement)
    int* s_lim = s_nconn + CF_MAX_K;                       // lim of every row
    int* s_cpos = s_lim + CF_MAX_K;                        // #rows with U(i, j) >= 1e-4
    int* s_slow = s_cpos + CF_MAX_K;                       // rows left to the dense path
    int* s_cnt = s_slow + CF_MAX_K;                        // [0..3] compaction, [4] lim,
                                                           // [5] Lu, [6] Lq, [7] #dense rows,
                                                           // [8] next fast-path rating
    // complement masks: bit i of word 3r + (i >> 6) = item i is NOT an out-neighbour of
    // item r with w > 0.1 (:254-265); fast-path rating order (largest nc first)
    uint64_t* s_cmask = reinterpret_cast<uint64_t*>(s_cnt + 12);
    int* s_order = reinterpret_cast<int*>(s_cmask + 3 * CF_MAX_K);
    int* s_cbar = s_conn;   // fast path: per-wave complement lists (kWaves x 64), aliases s_conn/s_keep
    double* Gb = a.gbar + (size_t)blockIdx.x * lmax * lmax;
    double* Qs = a.qs + (size_t)blockIdx.x * (lmax + 2) * lmax;
    double* PGH = a.pgh + (size_t)blockIdx.x * lmax * (lmax + 1) * 2;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    // Diagnostic phase stamps (thread 0 only; no effect on outputs):
    // {user setup, basis Q, fast ratings, block-wide ratings} cycles, {#fast, #block-wide}
    // ratings, {Gbar GEMM, block-wide K path} cycles.
    unsigned long long ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
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
        PHASE_STAMP(-1);
        if (tid == 0) {
            s_cnt[5] = 0;
            s_cnt[7] = 0;
            s_cnt[8] = 0;
        }
        for (int j = tid; j < m; j += kThreads) A[j] = (double)ev[j];   // evals staged in A
        __syncthreads();
        for (int i = tid; i < k; i += kThreads) {
            s_item[i] = a.items[base + i];
            s_rat[i] = a.ratings[base + i];
            // lim = first eigenvalue index above w_lim, clamped to [2, m] (:271-282)
            const double w_lim = (double)a.sigtab[a.sig_mode == CF_SIGS_COMPAT ? (uint64_t)i : base + i];
            int lim = m;
            for (int j = 0; j < m; ++j)
                if (A[j] > w_lim) {
                    lim = j;
                    break;
                }
            lim = min(max(lim, 2), m);
            s_lim[i] = lim;
            atomicMax(&s_cnt[5], lim);
        }
        if (wave == 0) {
            double sum = 0.0;
            for (int i = lane; i < k; i += 64) sum += (double)a.ratings[base + i];
            sum = wave_sum(sum);
            if (lane == 0) s_misc[1] = sum;
        }
        __syncthreads();
        const int Lu = s_cnt[5];
        // complement masks, four graph rows in flight per wave (unconditional clamped
        // loads, see block_gemm), then nc of every row in s_slow (free until the fast path)
        for (int r0 = 4 * wave; r0 < k; r0 += 4 * kWaves) {
            float gv[4][3];
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                const float* nrow = a.graph + (size_t)s_item[min(r0 + x, k - 1)] * a.n_items;
#pragma unroll
                for (int t = 0; t < 3; ++t) gv[x][t] = nrow[s_item[min(64 * t + lane, k - 1)]];
            }
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                int nc = 0;
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const int i = 64 * t + lane;
                    const unsigned long long bal = __ballot(i < k && !((double)gv[x][t] > 0.1));   // (:259)
                    nc += __popcll(bal);
                    if (lane == 0 && r0 + x < k) s_cmask[3 * (r0 + x) + t] = bal;
                }
                if (lane == 0 && r0 + x < k) s_slow[r0 + x] = nc;
            }
        }
        __syncthreads();
        // fast-path order: descending nc (ties by row), so the waves that claim ratings
        // dynamically finish together (longest first)
        for (int i = tid; i < k; i += kThreads) {
            const int ni = s_slow[i];
            int rank = 0;
            for (int j = 0; j < k; ++j) {
                const int nj = s_slow[j];
                rank += (nj > ni) || (nj == ni && j < i);
            }
            s_order[rank] = i;
        }

        // Gbar = U^T U over the columns [0, Lu), all k rows: full copy in Gb (the dense
        // path's complement form reads it); max |Gbar - I| (non-negative floats order
        // as their bit patterns) decides whether this user gets a basis.  All products
        // of this phase are block_gemm calls staged through A (free until the fast path).
        double* stage = A;
        if (tid == 0) s_cnt[6] = 0;
        __syncthreads();
        unsigned long long tg0 = (a.phase_cycles && tid == 0) ? __builtin_amdgcn_s_memtime() : 0ull;
        const auto all_blocks = [](int, int) { return true; };
        const auto lower_blocks = [](int i0, int j0) { return j0 <= i0; };
        float dev = 0.0f;   // this thread's max |Gbar - I|
        const auto as_double = [](int, int, auto v) { return (double)v; };
        // T(l, j) from a symmetric G: -G(l, j) (l < j), 1.5 - G(j, j) / 2 (l = j), 0 (l > j)
        const auto tri_T = [](int l, int j, double g) { return l < j ? -g : (l == j ? 1.5 - 0.5 * g : 0.0); };
        block_gemm<false, false>(
            Lu, Lu, [&](int i, int l) { return U[(size_t)l * m + i]; }, as_double,
            [&](int l, int j) { return U[(size_t)l * m + j]; }, as_double, [&](int) { return k; }, lower_blocks,
            [&](int i, int j, double v) {
                if (j > i) return;
                Gb[(size_t)i * lmax + j] = v;
                Gb[(size_t)j * lmax + i] = v;
                const float d = (float)fabs(v - (i == j ? 1.0 : 0.0));
                dev = fmaxf(dev, d == d ? d : 3.0e38f);
            },
            stage);
        for (int off = 32; off >= 1; off >>= 1) dev = fmaxf(dev, __shfl_xor(dev, off));
        if (lane == 0) atomicMax(&s_cnt[6], __float_as_int(dev));
        __syncthreads();
        if (a.phase_cycles && tid == 0) ph_acc[6] += __builtin_amdgcn_s_memtime() - tg0;
        for (int j = tid; j < Lu; j += kThreads) {
            int cnt = 0;
            for (int i0 = 0; i0 < k; i0 += 8) {
                double v[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) v[t] = (double)U[(size_t)min(i0 + t, k - 1) * m + j];
#pragma unroll
                for (int t = 0; t < 8; ++t) cnt += (i0 + t < k) && v[t] >= 0.0001;
            }
            s_cpos[j] = cnt;
        }
        __syncthreads();
        const int Lq = (__int_as_float(s_cnt[6]) <= (float)kOrthoMax) ? Lu : 0;
        PHASE_STAMP(0);

        // Q = U T1 T2 ..., T(l, j) = -G(l, j) (l < j), 1.5 - G(j, j) / 2 (l = j), 0 (l > j),
        // T1 from Gbar, each further T from the Gram of the previous product (held in the
        // PGH buffer until the prefix tables are built); stop once that Gram is within
        // kOrthoDone of I (two steps for eigenvectors, |Gbar - I| ~ 1e-6).
        double* Q1 = a.q1 + (size_t)blockIdx.x * lmax * lmax;
        double* G2 = PGH;
        if (Lq > 0) {
            const auto tri_end = [&](int j0) { return min(Lq, j0 + 64); };
            block_gemm<true, false>(
                k, Lq, [&](int i, int l) { return U[(size_t)i * m + l]; }, as_double,
                [&](int l, int j) { return Gb[(size_t)l * lmax + j]; }, tri_T, tri_end, all_blocks,
                [&](int i, int j, double v) { Q1[(size_t)i * Lq + j] = v; }, stage);
            double* X = Q1;
            double* Y = Qs;
            for (int it = 0; it < 3; ++it) {
                __syncthreads();
                if (tid == 0) s_cnt[6] = 0;
                __syncthreads();
                float dv = 0.0f;
                block_gemm<false, false>(
                    Lq, Lq, [&](int i, int l) { return X[(size_t)l * Lq + i]; }, as_double,
                    [&](int l, int j) { return X[(size_t)l * Lq + j]; }, as_double, [&](int) { return k; },
                    lower_blocks,
                    [&](int i, int j, double v) {
                        if (j > i) return;
                        G2[(size_t)i * Lq + j] = v;
                        G2[(size_t)j * Lq + i] = v;
                        const float d = (float)fabs(v - (i == j ? 1.0 : 0.0));
                        dv = fmaxf(dv, d == d ? d : 3.0e38f);
                    },
                    stage);
                for (int off = 32; off >= 1; off >>= 1) dv = fmaxf(dv, __shfl_xor(dv, off));
                if (lane == 0) atomicMax(&s_cnt[6], __float_as_int(dv));
                __syncthreads();
                const bool last = it == 2 || __int_as_float(s_cnt[6]) <= kOrthoDone;
                block_gemm<true, false>(
                    k, Lq, [&](int i, int l) { return X[(size_t)i * Lq + l]; }, as_double,
                    [&](int l, int j) { return G2[(size_t)l * Lq + j]; }, tri_T, tri_end, all_blocks,
                    [&](int i, int j, double v) { Y[(size_t)i * Lq + j] = v; }, stage);
                if (last) {
                    if (Y != Qs) {
                        __syncthreads();
                        for (int e = tid; e < k * Lq; e += kThreads) Qs[e] = Y[e];
                    }
                    break;
                }
                double* tmp = X;
                X = Y;
                Y = tmp;
            }
        }
        __syncthreads();
        // g, h (global rows k, k + 1 of Qs, and staged in A: T2 is no longer needed)
        double* s_g = A;
        double* s_h = A + Lq;
        for (int j = tid; j < Lq; j += kThreads) {
            double g = 0.0, h = 0.0;
            for (int i0 = 0; i0 < k; i0 += 8) {
                double v[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const double q = Qs[(size_t)min(i0 + t, k - 1) * Lq + j];
                    v[t] = i0 + t < k ? q : 0.0;
                }
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    g = fma(v[t], (double)s_rat[min(i0 + t, k - 1)], g);   // v[t] = 0 past k
                    h += v[t];
                }
            }
            Qs[(size_t)k * Lq + j] = g;
            Qs[(size_t)(k + 1) * Lq + j] = h;
            s_g[j] = g;
            s_h[j] = h;
        }
        __syncthreads();
        for (int i = tid; i < k; i += kThreads) {
            const double* qi = Qs + (size_t)i * Lq;
            double2* out = reinterpret_cast<double2*>(PGH) + (size_t)i * (Lq + 1);
            double pg = 0.0, ph = 0.0;
            out[0] = make_double2(0.0, 0.0);
            for (int j0 = 0; j0 < Lq; j0 += 8) {
                double v[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const double q = qi[min(j0 + t, Lq - 1)];
                    v[t] = j0 + t < Lq ? q : 0.0;
                }
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    if (j0 + t < Lq) {
                        pg = fma(v[t], s_g[j0 + t], pg);
                        ph = fma(v[t], s_h[j0 + t], ph);
                        out[j0 + t + 1] = make_double2(pg, ph);
                    }
            }
        }
        double* Pm = Q1;   // U T1 is consumed: P = Q Q^T takes its place
        if (Lq > 0)
            block_gemm<true, true>(
                k, k, [&](int i, int l) { return Qs[(size_t)i * Lq + l]; }, as_double,
                [&](int l, int j) { return Qs[(size_t)j * Lq + l]; }, as_double, [&](int) { return Lq; }, lower_blocks,
                [&](int i, int j, double v) {
                    if (j > i) return;
                    Pm[(size_t)i * k + j] = v;
                    Pm[(size_t)j * k + i] = v;
                },
                stage);
        __syncthreads();
        PHASE_STAMP(1);

        // ---- fast path: one wave per rating ------------------------------------------
        {
            double* Ew = A + (size_t)wave * a.ew;
            int* cb = s_cbar + wave * 64;
            const double sum_all = s_misc[1];
            // ratings are claimed from s_order one ahead (LDS counter)
            auto claim = [&]() {
                int v = 0;
                if (lane == 0) v = atomicAdd(&s_cnt[8], 1);
                return __shfl(v, 0);
            };
            const unsigned long long fw0 = a.phase_cycles ? __builtin_amdgcn_s_memtime() : 0ull;
            // diagnostics, summed over this wave's ratings of the user (wave-uniform)
            unsigned long long wacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            int idx = claim();
            while (idx < k) {
                const int r = s_order[idx];
                idx = claim();
                const unsigned long long rt0 = a.phase_cycles ? __builtin_amdgcn_s_memtime() : 0ull;
                int nc = 0;
                double sc = 0.0;
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const int i = 64 * t + lane;
                    const unsigned long long bal = s_cmask[3 * r + t];
                    const bool out = (bal >> lane) & 1ull;
                    if (out) {
                        const int pos = nc + __popcll(bal & ((1ull << lane) - 1ull));
                        if (pos < 64) cb[pos] = i;
                        sc += (double)s_rat[i];
                    }
                    nc += __popcll(bal);
                }
                sc = wave_sum(sc);
                const int c = k - nc;
                const int lim = s_lim[r];
                bool slow = c == 0 || nc > a.ncw || lim > Lq || m < 2;
                // too many complement rows for one wave: the block-wide K path (bit 16)
                const bool wide = !(c == 0 || lim > Lq || m < 2) && nc > a.ncw;
                WAVE_SYNC();
                if (!slow) {
                    // column j < lim is dropped (:284-304) iff every row with
                    // U(i, j) >= 1e-4 lies in Cbar
                    bool drop = false;
                    for (int j = lane; j < lim; j += 64) {
                        const int cp = s_cpos[j];
                        if (cp <= nc) {
                            int hit = 0;
                            for (int q = 0; q < nc; ++q) hit += (double)U[(size_t)cb[q] * m + j] >= 0.0001;
                            drop |= hit == cp;
                        }
                    }
                    slow = __ballot(drop) != 0ull;
                }
                if (slow) {
                    if (lane == 0) s_slow[atomicAdd(&s_cnt[7], 1)] = r | (wide ? 0x10000 : 0);
                    continue;
                }
                const double mu = (sum_all - sc) / (double)c;   // mean over C (:311)
                const unsigned long long sp0 = a.phase_cycles ? __builtin_amdgcn_s_memtime() : 0ull;

                // E = P_S over the rows [Cbar..., r] (np rows, packed lower): gathers
                // from P, minus the tail sum_{j in [lim, Lq)} Q_aj Q_bj when lim < Lq.
                const int np = nc + 1;
                const int nent = np * (np + 1) / 2;
                // border-row inputs, issued ahead of the P gathers: (PG, PH)(i, lim) of row
                // cb[lane] (lane < nc) or r (lane 63), and y_q = r_q - mu of the complement
                const double2* pgh_lim = reinterpret_cast<const double2*>(PGH) + lim;
                const double2 py = pgh_lim[(size_t)(lane < nc ? cb[lane] : r) * (Lq + 1)];
                double* sy = Ew + (a.ew - 64);
                if (lane < nc) sy[lane] = (double)s_rat[cb[lane]] - mu;
                auto entry_rows = [&](int e, int& ia, int& ib) {
                    int ra = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
                    while (ra * (ra + 1) / 2 > e) --ra;
                    while ((ra + 1) * (ra + 2) / 2 <= e) ++ra;
                    const int rb = e - ra * (ra + 1) / 2;
                    ia = ra < nc ? cb[ra] : r;
                    ib = rb < nc ? cb[rb] : r;
                };
                for (int e0 = 0; e0 < nent; e0 += 4 * 64) {   // four gathers in flight per lane
                    double v[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        int ia, ib;
                        entry_rows(min(e0 + 64 * t + lane, nent - 1), ia, ib);
                        v[t] = Pm[(size_t)ia * k + ib];
                    }
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        if (e0 + 64 * t + lane < nent) Ew[e0 + 64 * t + lane] = v[t];
                }
                if (lim < Lq) {   // rare (mean Lu - lim = 0.08): the tail of P_S
                    for (int e = lane; e < nent; e += 64) {
                        int ia, ib;
                        entry_rows(e, ia, ib);
                        const double* xa = Qs + (size_t)ia * Lq;
                        const double* xb = Qs + (size_t)ib * Lq;
                        double v = Ew[e];
                        for (int j = lim; j < Lq; ++j) v = fma(-xa[j], xb[j], v);
                        Ew[e] = v;
                    }
                }
                WAVE_SYNC();

                // Border rows: row nc = P_{r,Cbar} (already in place), row nc + 1 := b.
                // a_r on lane 63 (never a border lane's register).
                double bl = 0.0, ar = 0.0;
                if (lane < nc) {
                    bl = py.x - mu * py.y;
                    for (int q = 0; q < nc; ++q) {
                        const double eq = q <= lane ? Ew[tri(lane, q)] : Ew[tri(q, lane)];
                        bl = fma(-eq, sy[q], bl);
                    }
                }
                if (lane == 63) {
                    ar = py.x - mu * py.y;
                    for (int q = 0; q < nc; ++q) ar = fma(-Ew[tri(nc, q)], sy[q], ar);
                }
                WAVE_SYNC();
                if (lane < nc) {
                    Ew[tri(nc + 1, lane)] = bl;
                    for (int q = 0; q <= lane; ++q) Ew[tri(lane, q)] = (q == lane ? 1.0 : 0.0) - Ew[tri(lane, q)];
                }
                WAVE_SYNC();
                const unsigned long long sp1 = a.phase_cycles ? __builtin_amdgcn_s_memtime() : 0ull;
                if (a.phase_cycles) wacc[0] += sp1 - sp0;
                // LDL^T of K (nc columns), border rows nc (P_{r,Cbar}) and nc + 1 (b);
                // lane i owns row i.  Panels of 4 columns, no per-column sync:
                //  1. every lane factors the 4x4 diagonal block redundantly in registers;
                //  2. each row below it solves against that block (its 4 entries of L);
                //  3. the rank-4 trailing update A22 -= L21 D L21^T is one
                //     v_mfma_f64_16x16x4 per 16x16 lower tile (k = 4 = the panel width).
                // An exactly zero pivot is skipped (its column of L is 0), as in cf_ldlt.hpp.
                const int nrows = nc + 2;
                double minpiv = 1.0;
                const int li = lane & 15, lk = lane >> 4;
                for (int j0 = 0; j0 < nc; j0 += 4) {
                    const int pw = min(4, nc - j0);
                    double Lm[4][4], Dv[4], Di[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        // unconditional (clamped) broadcast reads, then select
                        double at[4];
#pragma unroll
                        for (int u = 0; u <= t; ++u)
                            at[u] = Ew[tri(j0 + min(t, pw - 1), j0 + min(u, pw - 1))];
#pragma unroll
                        for (int u = 0; u <= t; ++u)
                            at[u] = t < pw ? at[u] : (u == t ? 1.0 : 0.0);
                        // row t of the block against the rows above it (left-looking)
#pragma unroll
                        for (int u = 0; u < t; ++u) {
                            double x = at[u];
#pragma unroll
                            for (int s2 = 0; s2 < u; ++s2) x = fma(-Lm[t][s2] * Dv[s2], Lm[u][s2], x);
                            Lm[t][u] = x * Di[u];
                        }
                        double d = at[t];
#pragma unroll
                        for (int s2 = 0; s2 < t; ++s2) d = fma(-Lm[t][s2] * Dv[s2], Lm[t][s2], d);
                        Dv[t] = d;
                        Di[t] = d != 0.0 ? 1.0 / d : 0.0;   // exact-zero pivot: column skipped
                    }
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        if (t < pw) minpiv = fmin(minpiv, Dv[t]);
                    if (lane >= j0 && lane < nrows) {
                        if (lane < j0 + pw) {   // a row of the block: L and D from the factor
#pragma unroll
                            for (int t = 0; t < 4; ++t)
                                if (lane - j0 == t) {
#pragma unroll
                                    for (int u = 0; u < t; ++u) Ew[tri(lane, j0 + u)] = Lm[t][u];
                                    Ew[tri(lane, lane)] = Dv[t];
                                }
                        } else {   // a row below: z L11^T = a_i, l_i = z / D
                            double z[4];
#pragma unroll
                            for (int t = 0; t < 4; ++t) z[t] = Ew[tri(lane, j0 + min(t, pw - 1))];
#pragma unroll
                            for (int t = 0; t < 4; ++t) {
                                z[t] = t < pw ? z[t] : 0.0;
#pragma unroll
                                for (int s2 = 0; s2 < t; ++s2) z[t] = fma(-z[s2], Lm[t][s2], z[t]);
                            }
#pragma unroll
                            for (int t = 0; t < 4; ++t)
                                if (t < pw) Ew[tri(lane, j0 + t)] = z[t] * Di[t];
                        }
                    }
                    WAVE_SYNC();
                    const int r0 = j0 + pw;
                    if (r0 < nc) {
                        const int ntr = (nrows - r0 + 15) >> 4, ntc = (nc - r0 + 15) >> 4;
                        const double dk = lk == 0 ? Dv[0] : lk == 1 ? Dv[1] : lk == 2 ? Dv[2] : Dv[3];
                        const int kc = j0 + min(lk, pw - 1);
                        for (int ti = 0; ti < ntr; ++ti) {
                            const int arow = r0 + 16 * ti + li;
                            const double av = Ew[tri(min(arow, nrows - 1), kc)];
                            const double aop = (arow < nrows && lk < pw) ? -av * dk : 0.0;
                            const int tmax = min(ti, ntc - 1);
                            // two tiles of the row at a time: loads, then MFMAs, then stores
                            for (int tq0 = 0; tq0 <= tmax; tq0 += 2) {
                                f64x4 acc[2];
                                double bop[2];
#pragma unroll
                                for (int x = 0; x < 2; ++x) {
                                    const int col = r0 + 16 * (tq0 + x) + li;
                                    const double bv = Ew[tri(min(col, nc - 1), kc)];
                                    bop[x] = (col < nc && lk < pw) ? bv : 0.0;
#pragma unroll
                                    for (int q = 0; q < 4; ++q) {
                                        const int row = r0 + 16 * ti + lk + 4 * q;
                                        const int rc = min(row, nrows - 1);
                                        const double v = Ew[tri(rc, min(col, rc))];
                                        acc[x][q] = (tq0 + x <= tmax && row < nrows && col < nc && col <= row) ? v : 0.0;
                                    }
                                }
                                acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(aop, bop[0], acc[0], 0, 0, 0);
                                if (tq0 + 1 <= tmax) acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(aop, bop[1], acc[1], 0, 0, 0);
#pragma unroll
                                for (int x = 0; x < 2; ++x) {
                                    const int col = r0 + 16 * (tq0 + x) + li;
#pragma unroll
                                    for (int q = 0; q < 4; ++q) {
                                        const int row = r0 + 16 * ti + lk + 4 * q;
                                        if (tq0 + x <= tmax && row < nrows && col < nc && col <= row)
                                            Ew[tri(row, col)] = acc[x][q];
                                    }
                                }
                            }
                        }
                    }
                    WAVE_SYNC();
                }
                if (a.phase_cycles) wacc[1] += __builtin_amdgcn_s_memtime() - sp1;
                double dot = 0.0;
                if (lane < nc) dot = Ew[tri(nc, lane)] * Ew[tri(nc + 1, lane)] * Ew[tri(lane, lane)];
                dot = wave_sum(dot);
                ar = __shfl(ar, 63);
                WAVE_SYNC();
                // Full-rank but ill-conditioned (c >= lim): the dense path, whose error
                // matches the reference's.  Rank-deficient (c < lim: U_CS^T U_CS is
                // singular in exact arithmetic, the reference's inverse returns rounding
                // noise) stays here: b is orthogonal to null(K) exactly as t is to null(M),
                // so this is the same kind of noise-amplified value.
                if (!(minpiv >= kPivMin) && c >= lim) {
                    if (lane == 0) s_slow[atomicAdd(&s_cnt[7], 1)] = r;
                    continue;
                }
                if (lane == 0) {
                    double pred = mu + ar + dot;
                    if (pred > 5) pred = 5;
                    if (pred < 1) pred = 1;
                    const double d = (double)s_rat[r] - pred;
                    a.mse[base + r] = (float)(d * d);
                    a.kk[base + r] = c;
                    if (a.pred) a.pred[base + r] = pred;
                }
                if (a.phase_cycles) {   // per nc class: cycles, count (wave-uniform)
                    const unsigned long long dt = __builtin_amdgcn_s_memtime() - rt0;
                    if (nc <= 4) {
                        wacc[3] += dt;
                        wacc[6] += 1;
                    } else if (nc <= 16) {
                        wacc[4] += dt;
                        wacc[7] += 1;
                    } else {
                        wacc[5] += dt;
                    }
                }
            }
            if (a.phase_cycles) {
                wacc[2] += __builtin_amdgcn_s_memtime() - fw0;
                if (lane == 0)
                    for (int x = 0; x < 8; ++x) atomicAdd(&a.phase_cycles[8 + x], wacc[x]);
            }
        }
        __syncthreads();
        const int nslow = s_cnt[7];
        if (a.phase_cycles && tid == 0) {
            ph_acc[4] += (unsigned long long)(k - nslow);
            ph_acc[5] += (unsigned long long)nslow;
        }
        PHASE_STAMP(2);

        // The block-wide systems live in LDS when the bucket's full triangle fits beside two
        // resident blocks per CU, else in this block's HBM region (L2-resident while used).
        // (The per-wave fast-path scratch in A is dead by now: a system that fits in A --
        // (n + 2)(n + 3)/2 doubles for n rows -- uses it whatever big_lds says.)
        double* const Ahbm = a.abig + (size_t)blockIdx.x * a.abig_elems;
        // ---- block-wide paths: the K system of the fast path for large complements, and
        // the rating's own bordered Gram matrix (dense) for everything else ---------------
        for (int si = 0; si < nslow; ++si) {
            const int r = s_slow[si] & 0xffff;
            // connected set C: the user's items that are out-neighbours of movie r (:254-265)
            const float* nrow = a.graph + (size_t)s_item[r] * a.n_items;
            const bool conn = tid < k && (double)nrow[s_item[tid < k ? tid : 0]] > 0.1;
            const int c = block_compact(conn, tid, s_conn, s_cnt);
            const int nc = block_compact(tid < k && !conn, tid, s_nconn, s_cnt);
            const bool use_complement = nc < c;
            const int lim = s_lim[r];
            double* AW = (a.big_lds || (size_t)(nc + 2) * (nc + 3) / 2 <= (size_t)a.a_elems) ? A : Ahbm;

            bool wide = (s_slow[si] >> 16) != 0;
            const unsigned long long tw0 = (a.phase_cycles && tid == 0) ? __builtin_amdgcn_s_memtime() : 0ull;
            if (wide) {   // block-uniform
                bool drop = false;   // the column filter, as in the fast path
                if (tid < lim && s_cpos[tid] <= nc) {
                    int hit = 0;
                    for (int q = 0; q < nc; ++q) hit += (double)U[(size_t)s_nconn[q] * m + tid] >= 0.0001;
                    drop = hit == s_cpos[tid];
                }
                wide = !__syncthreads_or(drop);
            }
            if (wide) {
                // E = P_S over the rows [Cbar..., r] into AW (packed), then the bordered K
                // system exactly as in the fast path, factored by the blocked LDL^T.
                const int np = nc + 1;
                for (int e = tid; e < np * (np + 1) / 2; e += kThreads) {
                    int ra = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
                    while (ra * (ra + 1) / 2 > e) --ra;
                    while ((ra + 1) * (ra + 2) / 2 <= e) ++ra;
                    const int rb = e - ra * (ra + 1) / 2;
                    const int ia = ra < nc ? s_nconn[ra] : r;
                    const int ib = rb < nc ? s_nconn[rb] : r;
                    double v = Pm[(size_t)ia * k + ib];
                    const double* xa = Qs + (size_t)ia * Lq;
                    const double* xb = Qs + (size_t)ib * Lq;
                    for (int j = lim; j < Lq; ++j) v = fma(-xa[j], xb[j], v);
                    AW[e] = v;
                }
                if (wave == 0) {
                    double sc = 0.0;
                    for (int q = lane; q < nc; q += 64) sc += (double)s_rat[s_nconn[q]];
                    sc = wave_sum(sc);
                    if (lane == 0) s_misc[0] = (s_misc[1] - sc) / (double)c;
                }
                __syncthreads();
                const double mu = s_misc[0];
                const double2* pgh_lim = reinterpret_cast<const double2*>(PGH) + lim;
                // b_a = (Py)_a - sum_q E_aq y_q for the rows a of Cbar, a_r likewise as row nc:
                // g lanes per row (g = 4 / 2 / 1 as (nc + 1) g fits the block), shuffle-reduced
                {
                    const int nrw = nc + 1;
                    const int g = nrw * 4 <= kThreads ? 4 : (nrw * 2 <= kThreads ? 2 : 1);
                    const int ra = tid / g, part = tid - ra * g;
                    double v = 0.0;
                    if (ra < nrw)
                        for (int q = part; q < nc; q += g) {
                            const double eq = q <= ra ? AW[tri(ra, q)] : AW[tri(q, ra)];
                            v = fma(-eq, (double)s_rat[s_nconn[q]] - mu, v);
                        }
                    if (g >= 4) v += __shfl_xor(v, 2);
                    if (g >= 2) v += __shfl_xor(v, 1);
                    if (ra < nrw && part == 0) {
                        const double2 py = pgh_lim[(size_t)(ra < nc ? s_nconn[ra] : r) * (Lq + 1)];
                        v += py.x - mu * py.y;
                        if (ra < nc)
                            AW[tri(nc + 1, ra)] = v;   // row nc + 1 is read by nobody before the sync
                        else
                            s_misc[2] = v;
                    }
                }
                __syncthreads();
                for (int e = tid; e < nc * (nc + 1) / 2; e += kThreads) {
                    int ra = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
                    while (ra * (ra + 1) / 2 > e) --ra;
                    while ((ra + 1) * (ra + 2) / 2 <= e) ++ra;
                    AW[e] = (e == tri(ra, ra) ? 1.0 : 0.0) - AW[e];   // K = I - P_CbarCbar
                }
                __syncthreads();
                ldlt_bordered<kThreads, 8>(AW, nc, nc + 2);
                if (wave == 0) {
                    double minpiv = 1.0, dot = 0.0;
                    for (int j = lane; j < nc; j += 64) {
                        const double dj = AW[tri(j, j)];
                        minpiv = fmin(minpiv, dj);
                        dot = fma(AW[tri(nc, j)] * AW[tri(nc + 1, j)], dj, dot);
                    }
                    dot = wave_sum(dot);
                    for (int off = 32; off >= 1; off >>= 1) minpiv = fmin(minpiv, __shfl_xor(minpiv, off));
                    if (lane == 0) {
                        s_misc[3] = dot;
                        s_cnt[4] = minpiv >= kPivMin ? 1 : 0;
                    }
                }
                __syncthreads();
                wide = !(s_cnt[4] == 0 && c >= lim);   // ill-conditioned full rank: dense
                if (wide && tid == 0) {
                    double pred = mu + s_misc[2] + s_misc[3];
                    if (pred > 5) pred = 5;
                    if (pred < 1) pred = 1;
                    const double d = (double)s_rat[r] - pred;
                    a.mse[base + r] = (float)(d * d);
                    a.kk[base + r] = c;
                    if (a.pred) a.pred[base + r] = pred;
                }
                __syncthreads();
                if (a.phase_cycles && tid == 0) ph_acc[7] += __builtin_amdgcn_s_memtime() - tw0;
                if (wide) continue;
            }

            // zero-column filter: keep column j < lim iff some U(C, j) >= 1e-4 (:284-304)
            bool keep = false;
            if (tid < lim) {
                for (int i = 0; i < c; ++i)
                    if ((double)U[(size_t)s_conn[i] * m + tid] >= 0.0001) {
                        keep = true;
                        break;
                    }
            }
            const int L = block_compact(keep, tid, s_keep, s_cnt);
            AW = (a.big_lds || (size_t)(L + 2) * (L + 3) / 2 <= (size_t)a.a_elems) ? A : Ahbm;

            // mean of the connected ratings (:311)
            if (wave == 0) {
                double sum = 0.0;
                for (int i = lane; i < c; i += 64) sum += (double)s_rat[s_conn[i]];
                sum = wave_sum(sum);
                if (lane == 0) s_misc[0] = sum / (double)c;
            }
            __syncthreads();
            const double mean = s_misc[0];

            // bordered Gram: AW[i][j] = (G^T G)_ij (j <= i < L), AW[L][j] = t_j, AW[L+1][j] = v_j
            {
                const int nt4 = (L + 3) >> 2;
                const int ntile = nt4 * (nt4 + 1) / 2;
                for (int tix = tid; tix < ntile; tix += kThreads) {
                    int ta = 0, rem = tix;
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
                                AW[tri(ia, ib)] = use_complement
                                                     ? Gb[(size_t)ca[x] * lmax + cb[y]] - acc[x][y]
                                                     : acc[x][y];
                        }
                }
                // t = G^T (r - mean): 4 lanes per column, each a strided quarter of C;
                // v = U(r, S).
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
                        AW[tri(L, j)] = acc;
                        AW[tri(L + 1, j)] = (double)U[(size_t)r * m + cj];
                    }
                }
            }
            __syncthreads();

            ldlt_bordered<kThreads, 8>(AW, L, L + 2);

            // pred = v^T M^-1 t + mean = sum_j (L^-1 v)_j (L^-1 t)_j / D_j + mean (:314-327)
            if (wave == 0) {
                double dot = 0.0;
                const double* y = AW + tri(L, 0);
                const double* z = AW + tri(L + 1, 0);
                for (int j = lane; j < L; j += 64) dot = fma(y[j] * z[j], AW[tri(j, j)], dot);
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
        PHASE_STAMP(3);
    }
    // slots 0-7 (thread 0 of the block); 8-10 are added per rating / user by lane 0 of
    // every wave
    if (a.phase_cycles && tid == 0)
        for (int ph = 0; ph < 8; ++ph) atomicAdd(&a.phase_cycles[ph], ph_acc[ph]);
}

// Scratch doubles per workgroup and workgroups of a bucket launch (see launch_predict_bucket).
inline int predict_blocks(uint32_t count) { return (int)std::min<uint32_t>(count, 8192u); }
inline size_t predict_per_block(int lmax) {
    const size_t big = (size_t)(lmax + 2) * (lmax + 3) / 2;
    return (size_t)lmax * lmax + (size_t)(lmax + 2) * lmax + (size_t)lmax * (lmax + 1) * 2 +
           (size_t)lmax * lmax + big;
}

template <typename T>
int launch_predict_bucket(cf_ctx* ctx, PredArgs<T> args, uint32_t count, int lmax, double* scratch,
                          size_t scratch_bytes, hipStream_t stream) {
    args.lmax = lmax;
    const size_t lds_fixed = sizeof(double) * 4 + CF_MAX_K * (sizeof(uint32_t) + sizeof(float) + 6 * sizeof(int)) +
                             12 * sizeof(int) + CF_MAX_K * (3 * sizeof(uint64_t) + sizeof(int));   // s_cmask, s_order
    const int big = (lmax + 2) * (lmax + 3) / 2;
    // The full (lmax + 2)-row triangle of the block-wide systems in LDS would leave one
    // 4-wave block per CU for k > 128; there it moves to HBM and the LDS keeps only the
    // basis GEMM staging and the per-wave fast-path systems (nc <= 60), two blocks per CU.
    args.ncw = std::min(kNcMax, lmax);
    args.ew = (args.ncw + 2) * (args.ncw + 3) / 2 + 64;   // + y of the complement rows
    args.big_lds = sizeof(double) * (size_t)std::max({big, kWaves * args.ew, kStageElems}) + lds_fixed <= 81920;
    if (!args.big_lds) {
        args.ncw = std::min(60, lmax);
        args.ew = (args.ncw + 2) * (args.ncw + 3) / 2 + 64;
    }
    args.a_elems = std::max({args.big_lds ? big : 0, kWaves * args.ew, kStageElems, 2 * lmax});
    args.abig_elems = (size_t)big;
    const size_t lds = sizeof(double) * (size_t)args.a_elems + lds_fixed;
    if (lds > 163840) return cf_set_error(ctx, CF_ERANGE, "predict bucket exceeds LDS");
    // Up to 8192 workgroups (~one user each for most buckets): the hardware dispatcher then
    // balances the per-user cost (~k^3) dynamically.  Measured at C2: 2048 -> 160.2 ms,
    // 4096 -> 155.7, 8192 -> 152.3, 16384 / all users -> 152.5.  Scratch: ~1.6 MB per
    // workgroup at k <= 192 (13 GB of the 288 GB).
    int blocks = (int)std::min<uint32_t>(count, 8192u);
    const size_t per_block = (size_t)lmax * lmax + (size_t)(lmax + 2) * lmax + (size_t)lmax * (lmax + 1) * 2 +
                             (size_t)lmax * lmax + (args.big_lds ? 0 : (size_t)big);
    if ((size_t)blocks * per_block * sizeof(double) > scratch_bytes)
        return cf_set_error(ctx, CF_EINVAL, "predict scratch undersized");
    args.gbar = scratch;
    args.qs = args.gbar + (size_t)blocks * lmax * lmax;
    args.pgh = args.qs + (size_t)blocks * (lmax + 2) * lmax;
    args.q1 = args.pgh + (size_t)blocks * lmax * (lmax + 1) * 2;
    args.abig = args.q1 + (size_t)blocks * lmax * lmax;
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
    // Scratch for every LDS bucket, sized once (largest bucket) per stream; the bucket launches
    // alternate between two context-owned streams (fork/join by events with the caller's
    // stream) so one bucket's tail overlaps the next -- each stream has its own scratch copy.
    // Diagnostics (phase counters) keep one stream.
    size_t need = 0;
    for (const cf_bucket& b : plan->buckets)
        if (b.count && b.emax != kSpillBucket)
            need = std::max(need, (size_t)predict_blocks(b.count) *
                                      predict_per_block(std::max<int>(2, 16 * b.emax)) * sizeof(double));
    const bool overlap = !ctx->d_phase;
    const size_t copies = overlap ? cf_ctx::kAuxStreams : 1;
    if (need * copies > ctx->scratch_bytes) {
        if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
        ctx->d_scratch = nullptr;
        ctx->scratch_bytes = 0;
        CF_HIP_CHECK(ctx, hipMalloc(&ctx->d_scratch, need * copies));
        ctx->scratch_bytes = need * copies;
    }
    if (overlap) {
        if (!ctx->aux_stream[0]) {
            for (int i = 0; i < cf_ctx::kAuxStreams; ++i) {
                CF_HIP_CHECK(ctx, hipStreamCreateWithFlags(&ctx->aux_stream[i], hipStreamNonBlocking));
                CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&ctx->aux_event[i], hipEventDisableTiming));
            }
            CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&ctx->aux_event[cf_ctx::kAuxStreams], hipEventDisableTiming));
        }
        CF_HIP_CHECK(ctx, hipEventRecord(ctx->aux_event[cf_ctx::kAuxStreams], stream));
        for (int i = 0; i < cf_ctx::kAuxStreams; ++i) CF_HIP_CHECK(ctx, hipStreamWaitEvent(ctx->aux_stream[i], ctx->aux_event[cf_ctx::kAuxStreams], 0));
    }
    int nb = 0;
    for (const cf_bucket& b : plan->buckets) {
        if (b.count == 0) continue;
        if (b.emax == kSpillBucket) {   // k > CF_MAX_K: HBM-workspace predictor, alone, first
            hipStream_t st = overlap ? ctx->aux_stream[0] : stream;
            rc = cf_launch_predict_spill<T>(ctx, plan, b, d_item_off, d_items, d_ratings, d_m, d_evals, d_evec_off,
                                            d_evecs, d_sigtab, sig_mode, d_mse, d_kk, d_pred, st);
            if (rc != CF_OK) break;
            if (overlap) {
                CF_HIP_CHECK(ctx, hipEventRecord(ctx->aux_event[0], st));
                for (int i = 1; i < cf_ctx::kAuxStreams; ++i) CF_HIP_CHECK(ctx, hipStreamWaitEvent(ctx->aux_stream[i], ctx->aux_event[0], 0));
            }
            continue;
        }
        args.first = b.first;
        const int lmax = std::max<int>(2, 16 * b.emax);
        const int si = overlap ? (nb++ % cf_ctx::kAuxStreams) : 0;
        rc = launch_predict_bucket<T>(ctx, args, b.count, lmax,
                                      reinterpret_cast<double*>(static_cast<char*>(ctx->d_scratch) + si * need), need,
                                      overlap ? ctx->aux_stream[si] : stream);
        if (rc != CF_OK) break;
    }
    if (overlap)
        for (int i = 0; i < cf_ctx::kAuxStreams; ++i) {
            CF_HIP_CHECK(ctx, hipEventRecord(ctx->aux_event[i], ctx->aux_stream[i]));
            CF_HIP_CHECK(ctx, hipStreamWaitEvent(stream, ctx->aux_event[i], 0));
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
