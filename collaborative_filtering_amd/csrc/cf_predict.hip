// cf_predict.hip -- graph-signal rating predictor on precomputed eigenvectors.
//
// Replaces neigh_program::apply of local_calc_precomp.cpp:217-380.  The reference
// partitions by movie and copies the whole user block per rating (:234,242); here the
// test ratings are regrouped BY USER: one 256-thread workgroup walks one user's k
// test movies against that user's k x m eigen block, so every block is read from HBM
// once.  For test movie r of user u:
//
//   C    = the user's items j with w(movie_r -> item_j) > 0.1        (:132,254-265)
//   lim  = first eigenvalue index above w_lim, >= 2                   (:271-282)
//   S    = columns j < lim with some U(C, j) >= 1e-4                  (:284-304)
//   pred = v_S . (U_CS^T U_CS)^-1 U_CS^T (r_C - mean) + mean          (:308-315)
//   mse  = (float)(r - clamp(pred, 1, 5))^2, kk = |C|                 (:318-359)
//
// All arithmetic after the gather is fp64 (the reference's double path).
//
// Basis (per user, block-wide, fp64 MFMA GEMMs).  The prediction is the value at row r
// of the least-squares fit of r_C - mean on span(U_CS): it depends on U_S only through
// its column span.  With Lu = max_r lim_r:
//   Q = U T1, T1 = I - su(Gbar - I) - diag(Gbar - I) / 2 from Gbar = U^T U over [0, Lu):
//     upper triangular, so the leading lim columns of Q span those of U for every lim;
//   W = an orthonormal basis of the complement of span(Q) (k - Lu columns): Y = (I - Q Q^T)
//     Omega for a +-1 test matrix Omega, then Cholesky-QR (Y^T Y = L D L^T, W = Y L^-T
//     D^-1/2);
//   X = [Q | W] (k x k), then one joint step X <- X T(X^T X) (T upper triangular again:
//     prefix spans kept) squares the orthogonality error of the whole basis to ~1e-20.
//   For every lim, X[:, lim:k] is an orthonormal basis of the complement of
//   span(U[:, :lim]) -- the "tail" columns [lim, Lu) of Q included.
//
// Fast path (one wave per rating).  With Cbar = the rows not in C (nc of them, r among
// them), d = k - lim, B = X[Cbar, lim:k] (nc x d) and y = r - mean on C:
//   h = X[C, lim:k]^T y_C = (X^T r - mean X^T 1)[lim:k] - B^T y_Cbar
//   c >= lim (nc <= d, full rank):  pred - mean = -e_r^T K^-1 B h,  K = B B^T  (nc x nc)
//   c <  lim (nc >  d):             pred - mean = -w_r^T G^-1 h,    G = B^T B  (d x d)
// K = I - P_CbarCbar (P = X_S X_S^T) is the Woodbury form of U_CS^T U_CS (the same
// non-unit spectrum), and the first line is exactly the reference's solution.  For c < lim
// U_CS^T U_CS is singular: the reference's explicit inverse returns rounding noise of its
// Eigen build, and this kernel returns the minimum-norm least-squares prediction (the
// pseudo-inverse solution).  Either system has min(nc, d) rows and is the Gram
// matrix of gathered rows of X: fp64 MFMA on one wave (bordered by B h / e_r or w_r / h),
// then the wave's bordered LDL^T.  A rating costs ~nc d min(nc, d) MFMA flops instead of a
// lim x lim factorisation.
//
// Dense path (block-wide, the rating's own Gram matrix) for the ratings the fast path
// does not take: the column filter drops a column, min(nc, d) > nmax, c = 0, a pivot of
// K below kPivMin while c >= lim (full rank but ill-conditioned: U_CS^T U_CS has an
// eigenvalue < kPivMin), or U is not near-orthonormal (max |Gbar - I| > kOrthoMax: no
// basis for this user).
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
constexpr int kNsysMax = 62;          // fast path: system rows (n + 2 border rows <= 64 lanes)
// fast path: smallest pivot of K = I - P_CbarCbar (its pivots bound the smallest
// eigenvalue of U_CS^T U_CS in the Q basis, so this admits cond <~ 1e10, where the
// reference's own explicit inverse is accurate to ~cond * eps; parity is tested to 1e8)
constexpr double kPivMin = 1e-10;
// max |Gbar - I| for a basis: each correction step squares the orthogonality error, and
// steps repeat (up to 4) until the last Gram is within kOrthoDone, so Q is orthonormal to
// ~1e-16 for any U within kOrthoMax of orthonormal
constexpr double kOrthoMax = 1e-2;
constexpr float kOrthoDone = 1e-8f;
#ifndef CF_PRED_FS_PW
// columns of the complement's forward-substitution register panels: 8 halves the basis
// kernel's scratch (964 -> 516 B per lane; WRITE 241 -> 191 GB, predict 160.1 -> 152.7 ms on a
// 125k-user C4 shard, bit-identical outputs, profiles/r05/pred_fs{16,8}_e1.log); 16 is the r04 layout
#define CF_PRED_FS_PW 8
#endif
constexpr int kFsPw = CF_PRED_FS_PW;
#ifndef CF_PRED_BASIS_OCC
#define CF_PRED_BASIS_OCC 3    // basis-kernel blocks per CU: LDS ~50 KB each.  3 -> 168 VGPRs with
                               // spills still beats 2 (256, fewer spills): C4 shard predict 170.4
                               // -> 161.8 ms; 1 block: 214 ms (profiles/r04/pred_variants_v2, _v3)
#endif

// Per-user slot of a chunk (basis kernel -> rating kernel), offsets in doubles from the slot
// base; the int / u64 arrays live in double-sized cells.
struct SlotOff {
    size_t stride;   // doubles per slot
    int gb, x, q1, ap, gx, hx, misc, cmask, lim, order, cpos, pmask;
};

template <typename T>
struct PredArgs {
    const uint32_t* order;
    const uint64_t* item_off;
    const uint32_t* items;
    const float* ratings;
    const uint8_t* row_sel;   // rows to predict (null: all; bin/local_calc_precomp --pct)
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
    unsigned long long* phase_cycles;  // diagnostics: per-phase s_memtime totals (or null)
    int lmax;              // Gram dimension bound of the launch (row stride of the bases)
    int nmax;              // fast path: largest system min(nc, d) on one wave
    int ew;                // doubles of per-wave fast-path scratch (system + y + g)
    int a_elems;           // doubles of the rating kernel's shared factorisation region
    int big_lds;           // 1: the block-wide systems use the LDS region A
    int tail_basis;        // 1: the last joint step writes only X's columns from Lmin on
    const uint64_t* cmask_in;   // the eigen kernel's complement masks (fused step), or null
    uint64_t cmask_words;       // their extent (users beyond it gather the graph)
    const uint64_t* cmask_fp;   // per user: the fingerprint of the items they were built from
    uint32_t cmask_users;
    double* slots;         // per-user slots of the chunk
    SlotOff so;
    // block-wide ratings handed to pred_dense_kernel (null: the rating kernel's block runs its
    // user's own): dq[0] = count, dq[1] = claim counter, then 2 words per rating (plan
    // position, row | lim << 16); dense_ws: one factorisation region per dense workgroup
    uint32_t* dq;
    double* dense_ws;
};


// lane i's value exchanged with lane perm(i) inside its row of 16 (DPP: no LDS round trip)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
// Sum over each row of 16 lanes, the same bits in all 16 (quad permutes xor 1 and xor 2, then
// the half-row and row mirrors pair the quads and the halves; each pair adds the same two
// operands in both lanes).  Every lane of the row active.
__device__ __forceinline__ double row16_sum(double v) {
    v += dpp_f64<0xB1>(v);    // quad_perm [1, 0, 3, 2]
    v += dpp_f64<0x4E>(v);    // quad_perm [2, 3, 0, 1]
    v += dpp_f64<0x141>(v);   // row_half_mirror
    v += dpp_f64<0x140>(v);   // row_mirror
    return v;
}
#ifdef CF_PRED_SHFL_SUM   // A/B: the LDS-permute butterfly (six dependent ds_bpermute pairs)
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
#else
__device__ __forceinline__ double lane_f64(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
// Sum over the wave, the same bits in every lane: a butterfly inside each row of 16 (quad
// permutes xor 1 and xor 2, then the half-row and row mirrors pair the quads and the halves;
// each pair adds the same two operands in both lanes), then the four row sums in a fixed order.
// Called with every lane active.
__device__ __forceinline__ double wave_sum(double v) {
    v = row16_sum(v);
    return (lane_f64(v, 0) + lane_f64(v, 16)) + (lane_f64(v, 32) + lane_f64(v, 48));
}
#endif

// 1 / d for an LDL^T pivot: v_rcp_f64 and two Newton steps (5 dependent ops; the IEEE
// division is a ~10-op chain with scale / fixup steps) -- within an ulp or two of 1 / d for
// the normal pivots the fast path factors (|d| in [1e-300, 1e300]); CF_PRED_IEEE_DIV restores
// the division (A/B)
__device__ __forceinline__ double pivot_rcp(double d) {
#ifdef CF_PRED_IEEE_DIV
    return 1.0 / d;
#else
    double x = __builtin_amdgcn_rcp(d);
    double e = fma(-d, x, 1.0);
    x = fma(x, e, x);
    e = fma(-d, x, 1.0);
    return fma(x, e, x);
#endif
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
constexpr int kStageBuf = 2 * 16 * kStageLd;        // one chunk: A then B, 16 x kStageLd each
#ifdef CF_PRED_GEMM_SINGLE_BUFFER
constexpr int kStageNbuf = 1;
#else
constexpr int kStageNbuf = 2;                       // chunks alternate buffers: one barrier each
#endif
constexpr int kStageElems = kStageNbuf * kStageBuf;
using f64x4 = __attribute__((ext_vector_type(4))) double;
// MFMAs of 16 x 16 tiles that hold no output are skipped (wave-uniform): tiles past M or N,
// and with LOWER (callers that keep only j <= i) tiles wholly above the diagonal -- at k = 107
// that is 7 x 7 of the 8 x 8 tiles of a k x k product, and 6 of 16 in a diagonal block.
template <bool A_LFAST, bool B_LFAST, bool LOWER = false, class LA, class XA, class LB, class XB, class FK, class FW,
          class FO>
__device__ void block_gemm(int M, int N, LA loadA, XA xA, LB loadB, XB xB, FK kend, FW want, FO out,
                           double* stage) {
    int tid = threadIdx.x;
    __asm__ volatile("" : "+v"(tid));   // per call: keeps the index math out of the user loop
    const int lane = tid & 63;
    const int wr = (tid >> 6) >> 1, wc = (tid >> 6) & 1;   // this wave's 32 x 32 quadrant
    using RA = decltype(loadA(0, 0));
    using RB = decltype(loadB(0, 0));
    for (int i0 = 0; i0 < M; i0 += 64)
        for (int j0 = 0; j0 < N; j0 += 64) {
            if (!want(i0, j0)) continue;
            const int K = kend(j0);
            bool live[2][2];
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y) {
                    const int ti = i0 + 32 * wr + 16 * x, tj = j0 + 32 * wc + 16 * y;
#ifdef CF_PRED_GEMM_NOSKIP   // A/B: every tile of the block
                    live[x][y] = ti == ti && tj == tj;
#else
                    live[x][y] = ti < M && tj < N && (!LOWER || tj <= ti + 15);
#endif
                }
            f64x4 acc[2][2];
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y) acc[x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
            // two 16-deep chunks of raw operands in flight (registers) while a third is staged
            // in LDS and consumed: the operands come from HBM / the MALL (~2k cycles away),
            // a chunk's 16 MFMAs per wave take ~1k
            RA ra0[4], ra1[4];
            RB rb0[4], rb1[4];
            // unconditional loads from clamped indices: a guarded load would become a
            // branch with its own wait (one full latency per load)
            auto fetch = [&](int l0, RA (&ra)[4], RB (&rb)[4]) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int e = tid + kThreads * t;
                    const int ia = A_LFAST ? (e >> 4) : (e & 63), la = A_LFAST ? (e & 15) : (e >> 6);
                    const int jb = B_LFAST ? (e >> 4) : (e & 63), lb = B_LFAST ? (e & 15) : (e >> 6);
                    ra[t] = loadA(min(i0 + ia, M - 1), min(l0 + la, K - 1));
                    rb[t] = loadB(min(l0 + lb, K - 1), min(j0 + jb, N - 1));
                }
            };
            // with two buffers, chunk c is written to buffer c & 1 after the barrier that
            // published chunk c - 1, which every wave reaches only after its MFMAs on chunk
            // c - 2 (the same buffer): one barrier per chunk
            auto stage_chunk = [&](int l0, RA (&ra)[4], RB (&rb)[4], int b) {
                double* As = stage + (kStageNbuf - 1) * b * kStageBuf;
                double* Bs = As + 16 * kStageLd;
                if (kStageNbuf == 1) __syncthreads();   // the previous chunk is consumed
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
            };
            auto mma_chunk = [&](int b) {
                const double* As = stage + (kStageNbuf - 1) * b * kStageBuf;
                const double* Bs = As + 16 * kStageLd;
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
                            if (live[x][y])
                                acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[x], bv[y], acc[x][y], 0, 0, 0);
                }
            };
            if (K > 0) fetch(0, ra0, rb0);
            if (K > 16) fetch(16, ra1, rb1);
            for (int l0 = 0; l0 < K; l0 += 32) {
                stage_chunk(l0, ra0, rb0, 0);
                if (l0 + 32 < K) fetch(l0 + 32, ra0, rb0);
                mma_chunk(0);
                if (l0 + 16 < K) {
                    stage_chunk(l0 + 16, ra1, rb1, 1);
                    if (l0 + 48 < K) fetch(l0 + 48, ra1, rb1);
                    mma_chunk(1);
                }
            }
            // the next output block restarts at buffer 0, which slower waves may still read
            if (kStageNbuf == 2) __syncthreads();
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

// Lower triangle of a Gram matrix on ONE wave, fp64 MFMA: E[tri(i, j)] = sum_{s < inner}
// val(i, s) val(j, s) for j <= i < nt (nt <= 16 NS).  val(a, s) comes from load(a, s), which
// must return 0 outside a < nt, s < inner (callers clamp the address and select).  Operand
// strips of 16 rows x 4 terms: lane l of strip t holds val(16t + (l & 15), s0 + (l >> 4)),
// which is both the A fragment (A[l&15][l>>4]) of tile row t and the B fragment
// (B[l>>4][l&15]) of tile column t; the NS(NS+1)/2 lower tiles accumulate in registers.
// Operands are fetched PF steps (4 PF terms) at a time and the next batch is in flight while
// the current one's MFMAs issue, so a rating pays ~inner / (4 PF) load round trips.
template <int NS, int PF, class LOAD>
__device__ void wave_gram_t(int nt, int inner, LOAD load, double* E) {
    constexpr int NT = NS * (NS + 1) / 2;
    const int lane = threadIdx.x & 63;
    const int li = lane & 15, lk = lane >> 4;
    f64x4 acc[NT];
#pragma unroll
    for (int x = 0; x < NT; ++x) acc[x] = f64x4{0.0, 0.0, 0.0, 0.0};
    double v[PF][NS], w[PF][NS];
    auto fetch = [&](int s0) {
#pragma unroll
        for (int p = 0; p < PF; ++p)
#pragma unroll
            for (int t = 0; t < NS; ++t) w[p][t] = load(16 * t + li, s0 + 4 * p + lk);
    };
    fetch(0);
    for (int s0 = 0; s0 < inner; s0 += 4 * PF) {
#pragma unroll
        for (int p = 0; p < PF; ++p)
#pragma unroll
            for (int t = 0; t < NS; ++t) v[p][t] = w[p][t];
        if (s0 + 4 * PF < inner) fetch(s0 + 4 * PF);
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            if (s0 + 4 * p >= inner) break;   // wave-uniform
            int x = 0;
#pragma unroll
            for (int ti = 0; ti < NS; ++ti)
#pragma unroll
                for (int tj = 0; tj <= ti; ++tj, ++x)
                    acc[x] = __builtin_amdgcn_mfma_f64_16x16x4f64(v[p][ti], v[p][tj], acc[x], 0, 0, 0);
        }
    }
    int x = 0;
#pragma unroll
    for (int ti = 0; ti < NS; ++ti)
#pragma unroll
        for (int tj = 0; tj <= ti; ++tj, ++x)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 16 * ti + lk + 4 * q, col = 16 * tj + li;
                if (row < nt && col <= row) E[tri(row, col)] = acc[x][q];
            }
}

#ifndef CF_PRED_GRAM_PF4
#define CF_PRED_GRAM_PF4 2   // operand steps in flight of the 4 x 4-tile (nt > 48) Gram: 2 (was 4) halves its
// operand registers, so the rating kernel spills 76 instead of 156 B per lane (C4 shard predict 151.7 -> 149.6 ms,
// rating-kernel WRITE 14.4 -> 6.2 GB, bit-identical; profiles/r05/pv_*_m1.log)
#endif
template <class LOAD>
__device__ void wave_gram(int nt, int inner, LOAD load, double* E) {
    if (nt <= 16)
        wave_gram_t<1, 16>(nt, inner, load, E);
    else if (nt <= 32)
        wave_gram_t<2, 8>(nt, inner, load, E);
    else if (nt <= 48)
        wave_gram_t<3, 4>(nt, inner, load, E);
    else
        wave_gram_t<4, CF_PRED_GRAM_PF4>(nt, inner, load, E);
}

// Diagnostic phase stamps (thread 0 only; no effect on outputs): {user setup, basis,
// fast ratings, block-wide ratings} cycles, {#fast, #block-wide} ratings, {Gbar GEMM} cycles.
#define PHASE_STAMP(ph)                                                   \
    if (a.phase_cycles && tid == 0) {                                     \
        const unsigned long long now = __builtin_amdgcn_s_memtime();      \
        if ((ph) >= 0) ph_acc[(ph) < 0 ? 0 : (ph)] += now - ph_t;         \
        ph_t = now;                                                       \
    }

// ---- kernel 1: per user of a chunk, lim / complement masks / order of the ratings, Gbar,
// the basis X = [Q | W] and X^T r, X^T 1, into the user's slot ---------------------------
#ifndef CF_PRED_MASK_ROWS
#define CF_PRED_MASK_ROWS 8
#endif
constexpr int kMaskRows = CF_PRED_MASK_ROWS;   // graph rows gathered per wave at once
// One user (position uo of the plan's order) into `slot`: the body of pred_basis_kernel and
// the first half of pred_fused_kernel.
template <typename T>
__device__ __forceinline__ void basis_user(const PredArgs<T> a, uint32_t uo, double* slot, double* dsm,
                                           unsigned long long (&ph_acc)[8], unsigned long long& ph_t) {
    const int lmax = a.lmax;
    double* A = dsm;                                       // block_gemm staging
    double* s_misc = A + kStageElems;                      // [1] sum of the user's ratings
    uint32_t* s_item = reinterpret_cast<uint32_t*>(s_misc + 4);
    float* s_rat = reinterpret_cast<float*>(s_item + CF_MAX_K);
    int* s_lim = reinterpret_cast<int*>(s_rat + CF_MAX_K);   // lim of every row
    int* s_cpos = s_lim + CF_MAX_K;                        // #rows with U(i, j) >= 1e-4
    int* s_slow = s_cpos + CF_MAX_K;                       // nc of every row
    int* s_cnt = s_slow + CF_MAX_K;                        // [5] Lu, [6] orthogonality, [9] failure
    // complement masks: bit i of word 3r + (i >> 6) = item i is NOT an out-neighbour of
    // item r with w > 0.1 (:254-265); fast-path rating order (largest nc first)
    uint64_t* s_cmask = reinterpret_cast<uint64_t*>(s_cnt + 12);
    int* s_order = reinterpret_cast<int*>(s_cmask + 3 * CF_MAX_K);
    // per row: the smallest column j whose rows with U(i, j) >= 1e-4 are this row alone (a
    // single-complement rating of the row drops j if j < lim); -1 once the row is predicted here
    int* s_dmin = s_order + CF_MAX_K;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    {
        double* Gb = slot + a.so.gb;
        const uint32_t u = a.order[uo];
        const uint64_t base = a.item_off[u];
        const int k = (int)(a.item_off[u + 1] - base);
        const int m = a.m[u];
        const T* U = a.evecs + a.evec_off[u];
        const T* ev = a.evals + base;
        __syncthreads();
        PHASE_STAMP(-1);
        if (tid == 0) {
            s_cnt[5] = 0;
            s_cnt[10] = CF_MAX_K;
            s_cnt[11] = CF_MAX_K;   // first column with no U(i, j) >= 1e-4
        }
        for (int j = tid; j < m; j += kThreads) A[j] = (double)ev[j];   // evals staged in A
        __syncthreads();
        for (int i = tid; i < k; i += kThreads) {
            s_item[i] = a.items[base + i];
            s_rat[i] = a.ratings[base + i];
            // lim = first eigenvalue index above w_lim, clamped to [2, m] (:271-282)
            const double w_lim = (double)a.sigtab[a.sig_mode == CF_SIGS_COMPAT ? (uint64_t)i : base + i];
            // eight evals per probe, so the LDS reads of a probe are in flight together
            int lim = m;
            for (int j0 = 0; j0 < m; j0 += 8) {
                unsigned above = 0;
#pragma unroll
                for (int t = 0; t < 8; ++t) above |= (j0 + t < m && A[min(j0 + t, m - 1)] > w_lim) ? 1u << t : 0u;
                if (above) {
                    lim = j0 + __builtin_ctz(above);
                    break;
                }
            }
            lim = min(max(lim, 2), m);
            s_lim[i] = lim;
            s_dmin[i] = CF_MAX_K;
            atomicMax(&s_cnt[5], lim);
            atomicMin(&s_cnt[10], lim);
        }
        if (wave == 0) {
            double sum = 0.0;
            for (int i = lane; i < k; i += 64) sum += (double)a.ratings[base + i];
            sum = wave_sum(sum);
            if (lane == 0) s_misc[1] = sum;
        }
        __syncthreads();
        const int Lu = s_cnt[5];
        // complement masks: from the eigen kernel, which gathered the same graph entries (fused
        // step), else kMaskRows graph rows in flight per wave (unconditional clamped loads, see
        // block_gemm); nc of every row in s_slow (free until the fast path)
        // the masks only if the eigen run built them from this very item list (fingerprint;
        // s_cnt[7], uniform after the barrier)
        if (a.cmask_in && 3 * (base + (uint64_t)k) <= a.cmask_words && u < a.cmask_users && wave == 0) {
            const uint64_t fp = cf_items_fp(s_item, k, base, lane);
            if (lane == 0) s_cnt[7] = fp == a.cmask_fp[u];
        } else if (tid == 0) {
            s_cnt[7] = 0;
        }
        __syncthreads();
        if (s_cnt[7]) {
            const uint64_t* cm = a.cmask_in + 3 * base;
            for (int i = tid; i < 3 * k; i += kThreads) s_cmask[i] = cm[i];
            __syncthreads();
            for (int r = tid; r < k; r += kThreads)
                s_slow[r] = __popcll(s_cmask[3 * r]) + __popcll(s_cmask[3 * r + 1]) + __popcll(s_cmask[3 * r + 2]);
        } else
        for (int r0 = kMaskRows * wave; r0 < k; r0 += kMaskRows * kWaves) {
            float gv[kMaskRows][3];
#pragma unroll
            for (int x = 0; x < kMaskRows; ++x) {
                const GraphRow nrow = a.graph.row(s_item[min(r0 + x, k - 1)]);
#pragma unroll
                for (int t = 0; t < 3; ++t) gv[x][t] = nrow[s_item[min(64 * t + lane, k - 1)]];
            }
#pragma unroll
            for (int x = 0; x < kMaskRows; ++x) {
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

        // Gbar = U^T U over the columns [0, Lu), all k rows: its upper triangle in Gb (the
        // dense path's complement form reads it symmetrically); max |Gbar - I| (non-negative floats order
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
        block_gemm<false, false, true>(
            Lu, Lu, [&](int i, int l) { return U[(size_t)l * m + i]; }, as_double,
            [&](int l, int j) { return U[(size_t)l * m + j]; }, as_double, [&](int) { return k; }, lower_blocks,
            [&](int i, int j, double v) {
                if (j > i) return;
                Gb[(size_t)j * lmax + i] = v;   // upper triangle only: T1 reads G(l, j), l <= j
                const float d = (float)fabs(v - (i == j ? 1.0 : 0.0));
                dev = fmaxf(dev, d == d ? d : 3.0e38f);
            },
            stage);
        for (int off = 32; off >= 1; off >>= 1) dev = fmaxf(dev, __shfl_xor(dev, off));
        if (lane == 0) atomicMax(&s_cnt[6], __float_as_int(dev));
        __syncthreads();
#ifndef CF_PRED_BASIS_PROBE
        if (a.phase_cycles && tid == 0) ph_acc[6] += __builtin_amdgcn_s_memtime() - tg0;
#endif
        // per column j < Lu: the rows with U(i, j) >= 1e-4 as a 3-word mask (the rating
        // kernel's column filter is then P_j & ~Cbar == 0 per column) and their count
        {
            uint64_t* pm_g = reinterpret_cast<uint64_t*>(slot + a.so.pmask);
            for (int j = tid; j < Lu; j += kThreads) {
                int cnt = 0, sole = 0;
#pragma unroll
                for (int w = 0; w < 3; ++w) {
                    uint64_t bits = 0;
                    const int iend = min(k, 64 * w + 64);
                    for (int i0 = 64 * w; i0 < iend; i0 += 16) {
                        double v[16];
#pragma unroll
                        for (int t = 0; t < 16; ++t) v[t] = (double)U[(size_t)min(i0 + t, k - 1) * m + j];
#pragma unroll
                        for (int t = 0; t < 16; ++t)
                            if (i0 + t < iend && v[t] >= 0.0001) bits |= 1ull << (i0 + t - 64 * w);
                    }
                    pm_g[3 * j + w] = bits;
                    cnt += __popcll(bits);
                    if (bits) sole = 64 * w + __builtin_ctzll(bits);
                }
                s_cpos[j] = cnt;
                if (cnt == 0) atomicMin(&s_cnt[11], j);
                if (cnt == 1) atomicMin(&s_dmin[sole], j);
            }
        }
        __syncthreads();
        const int Lq = (__int_as_float(s_cnt[6]) <= (float)kOrthoMax) ? Lu : 0;
        PHASE_STAMP(0);

        // ---- basis X = [Q | W] (file header): Q = U T1, W by Cholesky-QR of (I - Q Q^T)
        // Omega, one joint T step on X; then X^T r and X^T 1 --------------------------------
        double* Q1 = slot + a.so.q1;
        double* Xb = slot + a.so.x;
        double* AP = slot + a.so.ap;
        const int ld = lmax;
        double* Xf = Xb;   // the final basis
        int Lx = 0;        // 0: no basis (every rating of the user takes the dense path)
        int jlo = 0;       // first column of Xf the last joint step wrote (a multiple of 64)
        if (Lq > 0) {
            // the W-failure flag is cleared before the barrier that ends the Q product, so every
            // thread reads it cleared below also when there is no complement (du == 0)
            if (tid == 0) s_cnt[9] = 0;
            const auto tri_end = [&](int j0) { return min(Lq, j0 + 64); };
            block_gemm<true, false>(
                k, Lq, [&](int i, int l) { return U[(size_t)i * m + l]; }, as_double,
                [&](int l, int j) { return Gb[(size_t)l * lmax + j]; }, tri_T, tri_end, all_blocks,
                [&](int i, int j, double v) { Xb[(size_t)i * ld + j] = v; }, stage);
            __syncthreads();
#ifdef CF_PRED_BASIS_PROBE
            const unsigned long long tw0 = (a.phase_cycles && tid == 0) ? __builtin_amdgcn_s_memtime() : 0ull;
#endif
            const int du = k - Lq;
            if (du > 0) {
                // Omega(i, j) = +-1 from a hash of (the user's content, i, j): the seed mixes k
                // and three of its item ids, never the user's position in the batch, so a user
                // gets the same basis bits in any batch or range split (multi-GPU runs equal
                // the one-GPU run)
                const auto mix = [](uint32_t h) {
                    h ^= h >> 16;
                    h *= 0x7FEB352Du;
                    h ^= h >> 15;
                    h *= 0x846CA68Bu;
                    return h ^ (h >> 16);
                };
                const uint32_t seed = mix(mix(mix((uint32_t)k * 0x9E3779B1u + 0x7F4A7C15u) ^ s_item[0]) ^
                                          s_item[k >> 1]) ^ s_item[k - 1];
                const auto omega = [seed](int i, int j) -> double {
                    uint32_t h = seed ^ ((uint32_t)i * 0x85EBCA6Bu) ^ ((uint32_t)j * 0xC2B2AE35u);
                    h ^= h >> 16;
                    h *= 0x7FEB352Du;
                    h ^= h >> 15;
                    h *= 0x846CA68Bu;
                    h ^= h >> 16;
                    return (h & 1u) ? 1.0 : -1.0;
                };
                const auto om = [&](int l, int j) { return omega(l, j); };
                // Q^T Omega (Lq x du) -> Q1
                block_gemm<false, false>(
                    Lq, du, [&](int i, int l) { return Xb[(size_t)l * ld + i]; }, as_double, om, as_double,
                    [&](int) { return k; }, all_blocks, [&](int i, int j, double v) { Q1[(size_t)i * ld + j] = v; },
                    stage);
                __syncthreads();
                // Y = Omega - Q (Q^T Omega) (k x du) -> Xb[:, Lq:k]
                block_gemm<true, false>(
                    k, du, [&](int i, int l) { return Xb[(size_t)i * ld + l]; }, as_double,
                    [&](int l, int j) { return Q1[(size_t)l * ld + j]; }, as_double, [&](int) { return Lq; },
                    all_blocks, [&](int i, int j, double v) { Xb[(size_t)i * ld + Lq + j] = omega(i, j) - v; }, stage);
                __syncthreads();
                // Y^T Y (du x du, packed lower) -> AP, L D L^T in place
                block_gemm<false, false, true>(
                    du, du, [&](int i, int l) { return Xb[(size_t)l * ld + Lq + i]; }, as_double,
                    [&](int l, int j) { return Xb[(size_t)l * ld + Lq + j]; }, as_double, [&](int) { return k; },
                    lower_blocks, [&](int i, int j, double v) { if (j <= i) AP[tri(i, j)] = v; }, stage);
                __syncthreads();
                // factor and solve with L in LDS when it fits the (now idle) GEMM staging
                double* LP = AP;
#ifndef CF_PRED_COMPLEMENT_GLOBAL
                if (tri(du, 0) <= kStageElems) {
                    LP = stage;
                    for (int i = tid; i < tri(du, 0); i += kThreads) LP[i] = AP[i];
                    __syncthreads();
                }
#endif
                ldlt_bordered<kThreads, 16>(LP, du, du);
                // W row i = D^-1/2 L^-1 y_i, in place (each thread its own rows)
                double dmax = 0.0;
                for (int j = 0; j < du; ++j) dmax = fmax(dmax, LP[tri(j, j)]);
                bool fail = false;
                for (int i = tid; i < k; i += kThreads) {
                    double* xi = Xb + (size_t)i * ld + Lq;
                    // forward substitution in 16-column panels held in registers: the solved
                    // entries t < p0 are read once per panel (independent loads, 16 independent
                    // accumulators) instead of once per column in one dependent chain; each
                    // entry still accumulates t = 0 .. j-1 in order (bit-identical results)
                    for (int p0 = 0; p0 < du; p0 += kFsPw) {
                        const int b = min(kFsPw, du - p0);
                        double acc[kFsPw];
                        int rb[kFsPw];
#pragma unroll
                        for (int q = 0; q < kFsPw; ++q) {
                            acc[q] = q < b ? xi[p0 + q] : 0.0;
                            rb[q] = tri(p0 + min(q, b - 1), 0);
                        }
#pragma unroll 2
                        for (int t = 0; t < p0; ++t) {
                            const double xt = xi[t];
#pragma unroll
                            for (int q = 0; q < kFsPw; ++q) acc[q] = fma(-LP[rb[q] + t], xt, acc[q]);
                        }
#pragma unroll
                        for (int q = 1; q < kFsPw; ++q)
#pragma unroll
                            for (int t = 0; t < q; ++t) acc[q] = fma(-LP[rb[q] + p0 + t], acc[t], acc[q]);
#pragma unroll
                        for (int q = 0; q < kFsPw; ++q)
                            if (q < b) xi[p0 + q] = acc[q];
                    }
                    for (int j = 0; j < du; ++j) {
                        const double dj = LP[tri(j, j)];
                        fail |= !(dj > 1e-12 * dmax);
                        xi[j] = dj > 0.0 ? xi[j] / sqrt(dj) : 0.0;
                    }
                }
                // a plain flag store, not __syncthreads_or: that one needs 256 B of static LDS,
                // which would push the fused kernel's LDS past two workgroups per CU
                if (fail) s_cnt[9] = 1;
                __syncthreads();
            }
#ifdef CF_PRED_BASIS_PROBE   // diagnostics: slot 7 = complement build, slot 6 = joint steps
            if (a.phase_cycles && tid == 0) ph_acc[7] += __builtin_amdgcn_s_memtime() - tw0;
            const unsigned long long tj0 = (a.phase_cycles && tid == 0) ? __builtin_amdgcn_s_memtime() : 0ull;
#endif
            // joint T steps on X (k columns): X^T X packed in AP, X <- X T (ping-pong Xb/Q1).
            // The ratings read only the columns [lim, k) of X, lim >= Lmin, and T is upper
            // triangular, so the last step needs only the column blocks from jlo = Lmin rounded
            // down to 64 on: the Gram rows i >= jlo (every G(l, j), l <= j, of those columns)
            // and the product columns j >= jlo.  A step that another one must follow needs the
            // whole X: its Gram is then redone in full (jlo = 0) before the product.
            double* Xs = Xb;
            double* Xd = Q1;
            jlo = a.tail_basis ? (min(s_cnt[10], k) & ~63) : 0;
            if (s_cnt[9] == 0) {
                for (int it = 0; it < 3; ++it) {
                    if (tid == 0) s_cnt[6] = 0;
                    __syncthreads();
                    float dv = 0.0f;
                    const int glo = jlo;
                    block_gemm<false, false, true>(
                        k, k, [&](int i, int l) { return Xs[(size_t)l * ld + i]; }, as_double,
                        [&](int l, int j) { return Xs[(size_t)l * ld + j]; }, as_double, [&](int) { return k; },
                        // (+ the leading block's diagonal tiles, so the convergence decision
                        // below also sees the deviation of those columns: ADVICE r4)
                        [glo](int i0, int j0) { return j0 <= i0 && (i0 >= glo || i0 == j0); },
                        [&](int i, int j, double v) {
                            if (j > i) return;
                            AP[tri(i, j)] = v;
                            const float dd = (float)fabs(v - (i == j ? 1.0 : 0.0));
                            dv = fmaxf(dv, dd == dd ? dd : 3.0e38f);
                        },
                        stage);
                    for (int off = 32; off >= 1; off >>= 1) dv = fmaxf(dv, __shfl_xor(dv, off));
                    if (lane == 0) atomicMax(&s_cnt[6], __float_as_int(dv));
                    __syncthreads();
                    const float dev_x = __int_as_float(s_cnt[6]);
                    if (!(dev_x <= (float)kOrthoMax)) break;   // no basis: Lx stays 0
                    if (glo > 0 && !(dev_x <= kOrthoDone)) {   // another step follows: full Gram
                        jlo = 0;
                        --it;
                        __syncthreads();   // every thread has read dev_x before s_cnt[6] is reset
                        continue;
                    }
                    const auto k_end = [&](int j0) { return min(k, j0 + 64); };
                    block_gemm<true, false>(
                        k, k, [&](int i, int l) { return Xs[(size_t)i * ld + l]; }, as_double,
                        [&](int l, int j) { return AP[tri(max(l, j), min(l, j))]; }, tri_T, k_end,
                        [glo](int, int j0) { return j0 >= glo; },
                        [&](int i, int j, double v) { Xd[(size_t)i * ld + j] = v; }, stage);
                    __syncthreads();
                    double* tmp = Xs;
                    Xs = Xd;
                    Xd = tmp;
                    if (dev_x <= kOrthoDone) {
                        Lx = k;
                        break;
                    }
                }
            }
            Xf = Xs;
#ifdef CF_PRED_BASIS_PROBE
            if (a.phase_cycles && tid == 0) ph_acc[6] += __builtin_amdgcn_s_memtime() - tj0;
#endif
        }
        // X^T r and X^T 1, the rating-level arrays and the flags into the slot
        double* s_gx = slot + a.so.gx;
        double* s_hx = slot + a.so.hx;
        double* gxl = A;                 // LDS copies for the closed form below (staging is idle)
        double* hxl = A + CF_MAX_K;
        int* s_list = reinterpret_cast<int*>(A + 2 * CF_MAX_K);
        if (Lx > 0)
            for (int j = jlo + tid; j < k; j += kThreads) {
                double g0 = 0.0, g1 = 0.0, h0 = 0.0, h1 = 0.0;
                int i = 0;
                for (; i + 1 < k; i += 2) {
                    const double x0 = Xf[(size_t)i * ld + j], x1 = Xf[(size_t)(i + 1) * ld + j];
                    g0 = fma(x0, (double)s_rat[i], g0);
                    g1 = fma(x1, (double)s_rat[i + 1], g1);
                    h0 += x0;
                    h1 += x1;
                }
                if (i < k) {
                    const double x0 = Xf[(size_t)i * ld + j];
                    g0 = fma(x0, (double)s_rat[i], g0);
                    h0 += x0;
                }
                s_gx[j] = gxl[j] = g0 + g1;
                s_hx[j] = hxl[j] = h0 + h1;
            }
        __syncthreads();
        // ---- single-complement ratings (Cbar = {r}, nc = 1: about a third of C4's) in closed
        // form here, instead of one rating-kernel wave each.  The fast path's K-mode at n = 1:
        // K = x.x with x = X[r, lim:k], b = x.g - K y_r (g = (X^T r - mu X^T 1)[lim:k], y_r = r_r -
        // mu), then its 1 x 1 LDL^T bordered by b and e_r: pred = mu - ((b / K)(1 / K)) K.  A row
        // whose column filter drops a column (P_j within {r}: s_cnt[11], s_dmin) or whose K is
        // below kPivMin stays with the rating kernel.  16 lanes per row, DPP row sums.
        int n_rate = k;   // ratings left to the rating kernel: s_order[0, n_rate)
#ifdef CF_PRED_NO_CLOSED   // A/B: every rating in the rating kernel
        if (false) {
#else
        if (Lx > 0 && m >= 2 && k >= 2) {
#endif
            const int zmin = s_cnt[11];
            const bool cand = tid < k && s_slow[tid] == 1 && ((s_cmask[3 * tid + (tid >> 6)] >> (tid & 63)) & 1ull) &&
                              s_lim[tid] < k && s_lim[tid] <= zmin && s_lim[tid] <= s_dmin[tid];
            const int ncand = block_compact(cand, tid, s_list, s_cnt);
            const double sum_all = s_misc[1];
            const int gl = tid & 15;
            for (int e = tid >> 4; e < ncand; e += kThreads / 16) {
                const int r = s_list[e];
                const int lim = s_lim[r];
                const int d = k - lim;
                const double rr = (double)s_rat[r];
                const double mu = (sum_all - rr) / (double)(k - 1);   // mean over C (:311)
                double kq = 0.0, bg = 0.0;
                for (int j = gl; j < d; j += 16) {
                    const double x = Xf[(size_t)r * ld + lim + j];
                    const double g = gxl[lim + j] - mu * hxl[lim + j];
                    kq = fma(x, x, kq);
                    bg = fma(x, g, bg);
                }
                kq = row16_sum(kq);
                bg = row16_sum(bg);
                if (gl == 0 && kq >= kPivMin) {
                    if (!a.row_sel || a.row_sel[base + r]) {
                        const double di = pivot_rcp(kq);
                        const double ba = fma(-kq, rr - mu, bg);
                        double pred = mu - ((ba * di) * di) * kq;
                        if (pred > 5) pred = 5;
                        if (pred < 1) pred = 1;
                        const double er = rr - pred;
                        a.mse[base + r] = (float)(er * er);
                        a.kk[base + r] = k - 1;
                        if (a.pred) a.pred[base + r] = pred;
                    }
                    s_dmin[r] = -1;
                }
            }
            __syncthreads();
            const int ord = tid < k ? s_order[tid] : 0;
            n_rate = block_compact(tid < k && s_dmin[ord] != -1, ord, s_order, s_cnt);
        }
        PHASE_STAMP(1);
        {
            int* lim_g = reinterpret_cast<int*>(slot + a.so.lim);
            int* ord_g = reinterpret_cast<int*>(slot + a.so.order);
            int* cpos_g = reinterpret_cast<int*>(slot + a.so.cpos);
            uint64_t* cm_g = reinterpret_cast<uint64_t*>(slot + a.so.cmask);
            for (int i = tid; i < k; i += kThreads) {
                lim_g[i] = s_lim[i];
                ord_g[i] = s_order[i];
            }
            for (int i = tid; i < 3 * k; i += kThreads) cm_g[i] = s_cmask[i];
            for (int j = tid; j < Lu; j += kThreads) cpos_g[j] = s_cpos[j];
            if (tid == 0) {
                double* misc = slot + a.so.misc;
                misc[0] = s_misc[1];
                misc[1] = (double)Lx;
                misc[2] = (double)Lq;
                misc[3] = Xf == Q1 ? 1.0 : 0.0;
                misc[4] = (double)n_rate;
            }
        }
    }
}

template <typename T>
__global__ __launch_bounds__(kThreads, CF_PRED_BASIS_OCC) void pred_basis_kernel(PredArgs<T> a, uint32_t first, uint32_t count) {
    extern __shared__ double dsm[];
    unsigned long long ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long ph_t = 0;
    // One user per workgroup: every launch uses grid = count.  Without a loop around the user
    // the values set up before it are not kept live across iterations: scratch 516 -> 308 B per
    // lane, C4 shard predict 149.7 -> 145.8 ms with the rating kernel's same change, bit-identical
    // (profiles/r05/pv_*_m2.log)
    const uint32_t ub = blockIdx.x;
    if (ub < count) basis_user(a, first + ub, a.slots + (size_t)ub * a.so.stride, dsm, ph_acc, ph_t);
    if (a.phase_cycles && threadIdx.x == 0)
        for (int ph = 0; ph < 8; ++ph) atomicAdd(&a.phase_cycles[ph], ph_acc[ph]);
}

// ---- kernel 2: per user of a chunk, every rating from the slot: the fast path (one wave per
// rating) and the dense path (block-wide) -------------------------------------------------
#ifndef CF_PRED_RATING_OCC
#define CF_PRED_RATING_OCC 2   // rating-kernel blocks per CU (registers and the LDS budget below)
#endif
constexpr size_t kRatingLds = 163840 / CF_PRED_RATING_OCC;
#ifndef CF_PRED_LDL_PW
// fast-path LDL^T panel width (4 or 8): columns per trailing update.  8 (two MFMA k-steps per
// trailing update, half the updates): C4 125k-user shard predict 163.1 -> 159.9 ms, 299 of
// 13.3M outputs differ by <= 1.3e-5 (rounding order; profiles/r04/pred_variants_v4/)
#define CF_PRED_LDL_PW 8
#endif
constexpr int kLdlPw = CF_PRED_LDL_PW;
static_assert(kLdlPw == 4 || kLdlPw == 8, "panel width: one or two MFMA k-steps");
// The dense path of one rating (row r, lim) of a user: the rating's own bordered Gram matrix
// M = U_CS^T U_CS, blocked LDL^T, block-wide (local_calc_precomp.cpp:254-327).  Called by the
// rating kernel's block for its user, or by pred_dense_kernel.  s_item / s_rat hold the user's
// items and ratings; A is the LDS factorisation region (a.a_elems doubles), Ahbm the HBM one.
template <typename T>
__device__ __forceinline__ void dense_rating(const PredArgs<T>& a, int r, int lim, int k, int m, uint64_t base,
                                             const T* U, const double* Gb, double* A, double* Ahbm,
                                             const uint32_t* s_item, const float* s_rat, int* s_conn, int* s_nconn,
                                             int* s_keep, int* s_cnt, double* s_misc) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int lmax = a.lmax;
    // connected set C: the user's items that are out-neighbours of movie r (:254-265)
    const GraphRow nrow = a.graph.row(s_item[r]);
    const bool conn = tid < k && (double)nrow[s_item[tid < k ? tid : 0]] > 0.1;
    const int c = block_compact(conn, tid, s_conn, s_cnt);
    const int nc = block_compact(tid < k && !conn, tid, s_nconn, s_cnt);
    const bool use_complement = nc < c;
    double* AW = (a.big_lds || (size_t)(nc + 2) * (nc + 3) / 2 <= (size_t)a.a_elems) ? A : Ahbm;

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
                                             ? Gb[(size_t)min(ca[x], cb[y]) * lmax + max(ca[x], cb[y])] -
                                                   acc[x][y]
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

// Every rating of one user (position uo of the plan's order) from `slot`: the body of
// pred_rating_kernel and the second half of pred_fused_kernel.
template <typename T>
__device__ __forceinline__ void rating_user(const PredArgs<T> a, uint32_t uo, double* slot, double* dsm,
                                            unsigned long long (&ph_acc)[8], unsigned long long& ph_t) {
    const int lmax = a.lmax;
    // A: the factorisation region: the per-wave fast-path scratch, then (dense path) the
    //    packed lower triangle of the bordered matrix [[M, .], [t^T, .], [v^T, .]].
    double* A = dsm;
    double* s_misc = A + a.a_elems;   // [0] mean (dense path), [1] sum of the user's ratings
    double* s_gx = s_misc + 4;                              // X^T r (k)
    double* s_hx = s_gx + CF_MAX_K;                         // X^T 1 (k)
    uint32_t* s_item = reinterpret_cast<uint32_t*>(s_hx + CF_MAX_K);
    float* s_rat = reinterpret_cast<float*>(s_item + CF_MAX_K);
    int* s_conn = reinterpret_cast<int*>(s_rat + CF_MAX_K);
    int* s_keep = s_conn + CF_MAX_K;
    int* s_nconn = s_keep + CF_MAX_K;                      // rows NOT in C (complement)
    int* s_lim = s_nconn + CF_MAX_K;                       // lim of every row
    int* s_cpos = s_lim + CF_MAX_K;                        // #rows with U(i, j) >= 1e-4
    int* s_slow = s_cpos + CF_MAX_K;                       // rows left to the dense path
    int* s_cnt = s_slow + CF_MAX_K;                        // [0..3] compaction, [4] flag,
                                                           // [7] #dense rows, [8] next rating
    uint64_t* s_cmask = reinterpret_cast<uint64_t*>(s_cnt + 12);
    int* s_order = reinterpret_cast<int*>(s_cmask + 3 * CF_MAX_K);
    int* s_cb = s_order + CF_MAX_K;                        // kWaves x CF_MAX_K
    uint64_t* s_pmask = reinterpret_cast<uint64_t*>(s_cb + kWaves * CF_MAX_K);   // 3 x CF_MAX_K

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    {
        const double* Gb = slot + a.so.gb;
        double* AP = slot + a.so.ap;
        const uint32_t u = a.order[uo];
        const uint64_t base = a.item_off[u];
        const int k = (int)(a.item_off[u + 1] - base);
        const int m = a.m[u];
        const T* U = a.evecs + a.evec_off[u];
        const double* misc = slot + a.so.misc;
        const int Lx = (int)misc[1];
        const int Lq = (int)misc[2];
        const double* Xf = slot + (misc[3] != 0.0 ? a.so.q1 : a.so.x);
        const int n_rate = (int)misc[4];   // the rest were predicted by the basis kernel
        const int ld = lmax;
        __syncthreads();
        {
            const int* lim_g = reinterpret_cast<const int*>(slot + a.so.lim);
            const int* ord_g = reinterpret_cast<const int*>(slot + a.so.order);
            const int* cpos_g = reinterpret_cast<const int*>(slot + a.so.cpos);
            const uint64_t* cm_g = reinterpret_cast<const uint64_t*>(slot + a.so.cmask);
            for (int i = tid; i < k; i += kThreads) {
                s_item[i] = a.items[base + i];
                s_rat[i] = a.ratings[base + i];
                s_lim[i] = lim_g[i];
                s_order[i] = ord_g[i];
                s_gx[i] = slot[a.so.gx + i];
                s_hx[i] = slot[a.so.hx + i];
            }
            for (int i = tid; i < 3 * k; i += kThreads) s_cmask[i] = cm_g[i];
            for (int j = tid; j < min(m, k + 2); j += kThreads) s_cpos[j] = j < Lq ? cpos_g[j] : 0;
            const uint64_t* pm_g = reinterpret_cast<const uint64_t*>(slot + a.so.pmask);
            for (int i = tid; i < 3 * min(m, k + 2); i += kThreads) s_pmask[i] = i < 3 * Lq ? pm_g[i] : 0ull;
            if (tid == 0) {
                s_misc[1] = misc[0];
                s_cnt[7] = 0;
                s_cnt[8] = 0;
            }
        }
        __syncthreads();
        PHASE_STAMP(-1);

        // ---- fast path: one wave per rating, in the complement coordinates of its prefix --
        {
            double* Ew = A + (size_t)wave * a.ew;
            int* cb = s_cb + wave * CF_MAX_K;
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
            while (idx < n_rate) {
                const int r = s_order[idx];
                idx = claim();
                if (a.row_sel && !a.row_sel[base + r]) continue;   // movie not sampled (wave-uniform)
                const unsigned long long rt0 = a.phase_cycles ? __builtin_amdgcn_s_memtime() : 0ull;
                // Cbar in ascending row order (the position of r in it), its rating sum
                int nc = 0, posr = 0;
                double sc = 0.0;
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const int i = 64 * t + lane;
                    const unsigned long long bal = s_cmask[3 * r + t];
                    if ((bal >> lane) & 1ull) {
                        cb[nc + __popcll(bal & ((1ull << lane) - 1ull))] = i;
                        sc += (double)s_rat[i];
                    }
                    if ((r >> 6) == t) posr = nc + __popcll(bal & ((1ull << (r & 63)) - 1ull));
                    nc += __popcll(bal);
                }
                sc = wave_sum(sc);
                const int c = k - nc;
                const int lim = s_lim[r];
                const int d = k - lim;
                const bool kmode = nc <= d;   // c >= lim: full rank
                const int n = kmode ? nc : d;
                const bool r_out = (s_cmask[3 * r + (r >> 6)] >> (r & 63)) & 1ull;   // r in Cbar (w(r,r) <= 0.1)
                bool slow = c == 0 || Lx == 0 || m < 2 || n > a.nmax || !r_out;
                WAVE_SYNC();
                if (!slow) {
                    // column j < lim is dropped (:284-304) iff every row with
                    // U(i, j) >= 1e-4 lies in Cbar
                    bool drop = false;
                    const uint64_t c0 = ~s_cmask[3 * r], c1 = ~s_cmask[3 * r + 1], c2 = ~s_cmask[3 * r + 2];
                    for (int j = lane; j < lim; j += 64)
                        drop |= ((s_pmask[3 * j] & c0) | (s_pmask[3 * j + 1] & c1) | (s_pmask[3 * j + 2] & c2)) == 0ull;
                    slow = __ballot(drop) != 0ull;
                }
                if (slow) {
                    if (lane == 0) s_slow[atomicAdd(&s_cnt[7], 1)] = r;
                    continue;
                }
                const double mu = (sum_all - sc) / (double)c;   // mean over C (:311)
                const unsigned long long sp0 = a.phase_cycles ? __builtin_amdgcn_s_memtime() : 0ull;
                // The system and its border rows come out of ONE Gram pass over gathered rows of
                // X (B = X[Cbar, lim:k]) with one extra operand (g = (X^T r - mu X^T 1)[lim:k],
                // y = r - mu on Cbar), so h = g - B^T y is never formed on its own:
                //   K-mode: Gram of the rows {B, g^T} -> K and B g; b = B h = B g - K y;
                //   G-mode: Gram of the columns {B, y} -> G and B^T y; h = g - B^T y.
                double* aux = Ew + (n + 2) * (n + 3) / 2;   // [0, nc): y; [nc, nc + d): g
                for (int q = lane; q < nc; q += 64) aux[q] = (double)s_rat[cb[q]] - mu;
                for (int j = lane; j < d; j += 64) aux[nc + j] = s_gx[lim + j] - mu * s_hx[lim + j];
                WAVE_SYNC();
                const double* yv = aux;
                const double* gv = aux + nc;
                if (kmode) {
                    wave_gram(nc + 1, d,
                              [&](int ar, int s) {
                                  const int s2 = min(s, d - 1);
                                  const double vg = Xf[(size_t)cb[min(ar, nc - 1)] * ld + lim + s2];
                                  const double vl = gv[s2];
                                  return s < d ? (ar < nc ? vg : (ar == nc ? vl : 0.0)) : 0.0;
                              },
                              Ew);
                    WAVE_SYNC();
                    // b_a = (B g)_a - sum_q K_aq y_q into border row n; row n + 1 = e_r
                    double ba = 0.0;
                    if (lane < n) {
                        ba = Ew[tri(n, lane)];
                        for (int q = 0; q < n; ++q) {
                            const double kq = q <= lane ? Ew[tri(lane, q)] : Ew[tri(q, lane)];
                            ba = fma(-kq, yv[q], ba);
                        }
                    }
                    WAVE_SYNC();
                    if (lane < n) {
                        Ew[tri(n, lane)] = ba;
                        Ew[tri(n + 1, lane)] = lane == posr ? 1.0 : 0.0;
                    }
                } else {
                    if (d > 0)
                        wave_gram(d + 1, nc,
                                  [&](int ar, int s) {
                                      const int s2 = min(s, nc - 1);
                                      const double vg = Xf[(size_t)cb[s2] * ld + lim + min(ar, d - 1)];
                                      const double vl = yv[s2];
                                      return s < nc ? (ar < d ? vg : (ar == d ? vl : 0.0)) : 0.0;
                                  },
                                  Ew);
                    WAVE_SYNC();
                    // row n = w_r, row n + 1 = h = g - B^T y (row d of the Gram)
                    if (lane < n) {
                        const double h = gv[lane] - Ew[tri(n, lane)];
                        Ew[tri(n + 1, lane)] = h;
                        Ew[tri(n, lane)] = Xf[(size_t)r * ld + lim + lane];
                    }
                }
                WAVE_SYNC();
                const unsigned long long sp1 = a.phase_cycles ? __builtin_amdgcn_s_memtime() : 0ull;
                if (a.phase_cycles) wacc[0] += sp1 - sp0;
                // LDL^T of the n x n system, border rows n and n + 1;
                // lane i owns row i.  Panels of 4 columns, no per-column sync:
                //  1. every lane factors the 4x4 diagonal block redundantly in registers;
                //  2. each row below it solves against that block (its 4 entries of L);
                //  3. the rank-4 trailing update A22 -= L21 D L21^T is one
                //     v_mfma_f64_16x16x4 per 16x16 lower tile (k = 4 = the panel width).
                // An exactly zero pivot is skipped (its column of L is 0), as in cf_ldlt.hpp.
                const int nrows = n + 2;
                double minpiv = 1.0;
                const int li = lane & 15, lk = lane >> 4;
                for (int j0 = 0; j0 < n; j0 += kLdlPw) {
                    const int pw = min(kLdlPw, n - j0);
                    double Lm[kLdlPw][kLdlPw], Dv[kLdlPw], Di[kLdlPw];
#pragma unroll
                    for (int t = 0; t < kLdlPw; ++t) {
                        // unconditional (clamped) broadcast reads, then select
                        double at[kLdlPw];
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
                        Di[t] = d != 0.0 ? pivot_rcp(d) : 0.0;   // exact-zero pivot: column skipped
                    }
#pragma unroll
                    for (int t = 0; t < kLdlPw; ++t)
                        if (t < pw) minpiv = fmin(minpiv, Dv[t]);
                    if (lane >= j0 && lane < nrows) {
                        if (lane < j0 + pw) {   // a row of the block: L and D from the factor
#pragma unroll
                            for (int t = 0; t < kLdlPw; ++t)
                                if (lane - j0 == t) {
#pragma unroll
                                    for (int u = 0; u < t; ++u) Ew[tri(lane, j0 + u)] = Lm[t][u];
                                    Ew[tri(lane, lane)] = Dv[t];
                                }
                        } else {   // a row below: z L11^T = a_i, l_i = z / D
                            double z[kLdlPw];
#pragma unroll
                            for (int t = 0; t < kLdlPw; ++t) z[t] = Ew[tri(lane, j0 + min(t, pw - 1))];
#pragma unroll
                            for (int t = 0; t < kLdlPw; ++t) {
                                z[t] = t < pw ? z[t] : 0.0;
#pragma unroll
                                for (int s2 = 0; s2 < t; ++s2) z[t] = fma(-z[s2], Lm[t][s2], z[t]);
                            }
#pragma unroll
                            for (int t = 0; t < kLdlPw; ++t)
                                if (t < pw) Ew[tri(lane, j0 + t)] = z[t] * Di[t];
                        }
                    }
                    WAVE_SYNC();
                    const int r0 = j0 + pw;
                    if (r0 < n) {
                        const int ntr = (nrows - r0 + 15) >> 4, ntc = (n - r0 + 15) >> 4;
                        // MFMA step s takes the panel's columns 4s .. 4s + 3 (lane group lk)
                        double dk[kLdlPw / 4];
                        int kc[kLdlPw / 4];
#pragma unroll
                        for (int s4 = 0; s4 < kLdlPw / 4; ++s4) {
                            double dsel = Dv[4 * s4];
#pragma unroll
                            for (int t = 1; t < 4; ++t) dsel = lk == t ? Dv[4 * s4 + t] : dsel;
                            dk[s4] = dsel;
                            kc[s4] = j0 + min(4 * s4 + lk, pw - 1);
                        }
                        for (int ti = 0; ti < ntr; ++ti) {
                            const int arow = r0 + 16 * ti + li;
                            double aop[kLdlPw / 4];
#pragma unroll
                            for (int s4 = 0; s4 < kLdlPw / 4; ++s4) {
                                const double av = Ew[tri(min(arow, nrows - 1), kc[s4])];
                                aop[s4] = (arow < nrows && 4 * s4 + lk < pw) ? -av * dk[s4] : 0.0;
                            }
                            const int tmax = min(ti, ntc - 1);
                            // two tiles of the row at a time: loads, then MFMAs, then stores
                            for (int tq0 = 0; tq0 <= tmax; tq0 += 2) {
                                f64x4 acc[2];
                                double bop[2][kLdlPw / 4];
#pragma unroll
                                for (int x = 0; x < 2; ++x) {
                                    const int col = r0 + 16 * (tq0 + x) + li;
#pragma unroll
                                    for (int s4 = 0; s4 < kLdlPw / 4; ++s4) {
                                        const double bv = Ew[tri(min(col, n - 1), kc[s4])];
                                        bop[x][s4] = (col < n && 4 * s4 + lk < pw) ? bv : 0.0;
                                    }
#pragma unroll
                                    for (int q = 0; q < 4; ++q) {
                                        const int row = r0 + 16 * ti + lk + 4 * q;
                                        const int rc = min(row, nrows - 1);
                                        const double v = Ew[tri(rc, min(col, rc))];
                                        acc[x][q] = (tq0 + x <= tmax && row < nrows && col < n && col <= row) ? v : 0.0;
                                    }
                                }
#pragma unroll
                                for (int s4 = 0; s4 < kLdlPw / 4; ++s4) {
                                    acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(aop[s4], bop[0][s4], acc[0], 0, 0, 0);
                                    if (tq0 + 1 <= tmax)
                                        acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(aop[s4], bop[1][s4], acc[1], 0, 0, 0);
                                }
#pragma unroll
                                for (int x = 0; x < 2; ++x) {
                                    const int col = r0 + 16 * (tq0 + x) + li;
#pragma unroll
                                    for (int q = 0; q < 4; ++q) {
                                        const int row = r0 + 16 * ti + lk + 4 * q;
                                        if (tq0 + x <= tmax && row < nrows && col < n && col <= row)
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
                if (lane < n) dot = Ew[tri(n, lane)] * Ew[tri(n + 1, lane)] * Ew[tri(lane, lane)];
                dot = wave_sum(dot);
                WAVE_SYNC();
                // Full rank but ill-conditioned (c >= lim, a pivot of K below kPivMin): the
                // dense path, whose error matches the reference's
                if (kmode && !(minpiv >= kPivMin)) {
                    if (lane == 0) s_slow[atomicAdd(&s_cnt[7], 1)] = r;
                    continue;
                }
                if (lane == 0) {
                    double pred = mu - dot;
                    if (pred > 5) pred = 5;
                    if (pred < 1) pred = 1;
                    const double e = (double)s_rat[r] - pred;
                    a.mse[base + r] = (float)(e * e);
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
        // resident blocks per CU, else in this block's HBM region AP (L2-resident while
        // used; the basis no longer needs it).  (The per-wave fast-path scratch in A is dead
        // by now: a system that fits in A -- (n + 2)(n + 3)/2 doubles for n rows -- uses it
        // whatever big_lds says.)  pred_dense_kernel uses a region of its own per workgroup.
        // ---- dense path: the rating's own bordered Gram matrix, block-wide -----------------
        // (queued for pred_dense_kernel when a.dq is set: a few users with many block-wide
        // ratings would otherwise run them one after another in one block, a tail of the launch)
        if (a.dq && nslow > 0) {
            if (tid < nslow) {
                const int r = s_slow[tid] & 0xffff;
                const uint32_t q = atomicAdd(a.dq, 1u);
                a.dq[4 + 2 * (size_t)q] = uo;
                a.dq[4 + 2 * (size_t)q + 1] = (uint32_t)r | ((uint32_t)s_lim[r] << 16);
            }
        } else {
            for (int si = 0; si < nslow; ++si) {
                const int r = s_slow[si] & 0xffff;
                dense_rating<T>(a, r, s_lim[r], k, m, base, U, Gb, A, AP, s_item, s_rat, s_conn, s_nconn, s_keep,
                                s_cnt, s_misc);
            }
        }
        PHASE_STAMP(3);
    }
}

template <typename T>
__global__ __launch_bounds__(kThreads, CF_PRED_RATING_OCC) void pred_rating_kernel(PredArgs<T> a, uint32_t first, uint32_t count) {
    extern __shared__ double dsm[];
    unsigned long long ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long ph_t = 0;
    // one user per workgroup, grid = count (as the basis kernel): scratch 76 -> 8 B per lane
    const uint32_t ub = blockIdx.x;
    if (ub < count) rating_user(a, first + ub, a.slots + (size_t)ub * a.so.stride, dsm, ph_acc, ph_t);
    // slots 0-7 (thread 0 of the block); 8-15 are added per rating / user by lane 0 of
    // every wave
    if (a.phase_cycles && threadIdx.x == 0)
        for (int ph = 0; ph < 8; ++ph) atomicAdd(&a.phase_cycles[ph], ph_acc[ph]);
}

// Block-wide ratings queued by pred_rating_kernel (a.dq), one rating per claim, persistent
// workgroups: the rating's user's items and ratings, its slot's Gbar (the launch's chunk starts
// at plan position `first`), and a factorisation region of its own in HBM.  Every workgroup
// leaves when the claims pass the count the rating kernel wrote.
template <typename T>
__global__ __launch_bounds__(kThreads) void pred_dense_kernel(PredArgs<T> a, uint32_t first) {
    extern __shared__ double dsm[];
    double* A = dsm;
    double* s_misc = A + a.a_elems;
    double* s_gx = s_misc + 4;
    double* s_hx = s_gx + CF_MAX_K;
    uint32_t* s_item = reinterpret_cast<uint32_t*>(s_hx + CF_MAX_K);
    float* s_rat = reinterpret_cast<float*>(s_item + CF_MAX_K);
    int* s_conn = reinterpret_cast<int*>(s_rat + CF_MAX_K);
    int* s_keep = s_conn + CF_MAX_K;
    int* s_nconn = s_keep + CF_MAX_K;
    int* s_lim = s_nconn + CF_MAX_K;
    int* s_cpos = s_lim + CF_MAX_K;
    int* s_slow = s_cpos + CF_MAX_K;
    int* s_cnt = s_slow + CF_MAX_K;
    const int tid = threadIdx.x;
    double* Ahbm = a.dense_ws + (size_t)blockIdx.x * ((size_t)(a.lmax + 2) * (a.lmax + 3) / 2);
    for (;;) {
        if (tid == 0) s_cnt[8] = (int)atomicAdd(a.dq + 1, 1u);
        __syncthreads();
        const uint32_t q = (uint32_t)s_cnt[8];
        __syncthreads();
        if (q >= a.dq[0]) break;   // uniform: every wave of every workgroup reaches this exit
        const uint32_t uo = a.dq[4 + 2 * (size_t)q];
        const uint32_t rl = a.dq[4 + 2 * (size_t)q + 1];
        const int r = (int)(rl & 0xffffu), lim = (int)(rl >> 16);
        const uint32_t u = a.order[uo];
        const uint64_t base = a.item_off[u];
        const int k = (int)(a.item_off[u + 1] - base);
        const int m = a.m[u];
        const T* U = a.evecs + a.evec_off[u];
        const double* Gb = a.slots + (size_t)(uo - first) * a.so.stride + a.so.gb;
        for (int i = tid; i < k; i += kThreads) {
            s_item[i] = a.items[base + i];
            s_rat[i] = a.ratings[base + i];
        }
        __syncthreads();
        dense_rating<T>(a, r, lim, k, m, base, U, Gb, A, Ahbm, s_item, s_rat, s_conn, s_nconn, s_keep, s_cnt,
                        s_misc);
    }
}

// ---- fused: basis then ratings of one user in the same workgroup, users claimed from a
// device counter; a workgroup reuses ONE slot for all its users, so the slot set is one
// slot per resident workgroup (~0.2-0.5 GB, within the 256 MiB Infinity Cache for k <~ 120)
// and the rating half reads the basis it has just written instead of a chunk of 8192 slots
// written a whole launch earlier.  Same arithmetic per user as the two kernels.  Measured
// slower on C4 (1.80 vs 1.66 s): the rating half is latency-bound on its dependent chains,
// not on where the slot lives, so it is an A/B option (CF_PRED_FUSED=1), not the default.
// The fused kernel calls the two halves as real functions: each keeps the register
// allocation of its own kernel instead of one allocation over both bodies (inlined, the
// fused body spilled 684 B per lane against 444 / 176).
#ifdef CF_PRED_FUSED_INLINE
#define CF_PRED_CALL __forceinline__
#else
#define CF_PRED_CALL __noinline__
#endif
template <typename T>
__device__ CF_PRED_CALL void basis_user_call(const PredArgs<T> a, uint32_t uo, double* slot, double* dsm,
                                             unsigned long long (&ph_acc)[8], unsigned long long& ph_t) {
    basis_user(a, uo, slot, dsm, ph_acc, ph_t);
}
template <typename T>
__device__ CF_PRED_CALL void rating_user_call(const PredArgs<T> a, uint32_t uo, double* slot, double* dsm,
                                              unsigned long long (&ph_acc)[8], unsigned long long& ph_t) {
    rating_user(a, uo, slot, dsm, ph_acc, ph_t);
}

template <typename T>
__global__ __launch_bounds__(kThreads, CF_PRED_RATING_OCC) void pred_fused_kernel(PredArgs<T> a, uint32_t first, uint32_t count,
                                                                                  uint32_t* next) {
    extern __shared__ double dsm[];
    unsigned long long ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long ph_t = 0;
    double* slot = a.slots + (size_t)blockIdx.x * a.so.stride;
    uint32_t* s_claim = reinterpret_cast<uint32_t*>(dsm);   // free between users (both halves open with a barrier)
    for (;;) {
        if (threadIdx.x == 0) s_claim[0] = atomicAdd(next, 1u);
        __syncthreads();
        const uint32_t ub = s_claim[0];
        if (ub >= count) break;   // uniform: every thread read the same claim
        basis_user_call(a, first + ub, slot, dsm, ph_acc, ph_t);
        __syncthreads();
        rating_user_call(a, first + ub, slot, dsm, ph_acc, ph_t);
        __syncthreads();
    }
}

// Chunks of up to kChunk users per (basis, rating) launch pair; each user of a chunk owns a
// slot (SlotOff) holding Gbar, X, Q1 (the basis's second buffer), the packed triangle AP and
// the per-row arrays, ~1 MB at lmax = 192.
constexpr uint32_t kChunkDefault = 32768;   // C4 predict: 2048 / 4096 / 8192 / 16384 / 32768 users
                                            // -> 1712 / 1668 / 1658 / 1649 / 1640 ms (profiles/r03/pred_chunk_ab/)
// CF_PRED_CHUNK overrides the users per launch pair (A/B runs); read once per process.
inline uint32_t pred_chunk() {
    static const uint32_t c = [] {
        const char* e = std::getenv("CF_PRED_CHUNK");
        const long v = e ? std::atol(e) : 0;
        return v >= 256 && v <= (1 << 20) ? (uint32_t)v : kChunkDefault;
    }();
    return c;
}
inline int fast_tri(int n) { return (n + 2) * (n + 3) / 2; }
inline SlotOff slot_layout(int lmax) {
    SlotOff so{};
    size_t o = 0;
    const size_t l2 = (size_t)lmax * lmax;
    so.gb = (int)o; o += l2;
    so.x = (int)o; o += l2;
    so.q1 = (int)o; o += l2;
    so.ap = (int)o; o += (size_t)(lmax + 2) * (lmax + 3) / 2;
    so.gx = (int)o; o += lmax;
    so.hx = (int)o; o += lmax;
    so.misc = (int)o; o += 8;
    so.cmask = (int)o; o += 3 * (size_t)lmax;                 // u64 per cell
    so.lim = (int)o; o += (lmax + 1) / 2;                    // ints, two per cell
    so.order = (int)o; o += (lmax + 1) / 2;
    so.cpos = (int)o; o += (lmax + 1) / 2;
    so.pmask = (int)o; o += 3 * (size_t)lmax;                 // u64 per cell
    so.stride = (o + 15) & ~(size_t)15;                      // 128-byte aligned slots
    return so;
}
// Slot bytes of one launch pair of up to `users` users, over the plan's LDS buckets.
inline size_t chunk_slot_bytes(const cf_plan* plan, uint32_t users) {
    size_t need = 0;
    for (const cf_bucket& b : plan->buckets)
        if (b.count && b.emax != kSpillBucket)
            need = std::max(need, (size_t)std::min(b.count, users) *
                                      slot_layout(std::max<int>(2, 16 * b.emax)).stride * sizeof(double));
    return need;
}
// Users per launch pair: pred_chunk(), halved while its slot copies would take more than a
// third of the HBM left (the context's own scratch counted as free), down to 2048.
inline uint32_t fit_chunk(cf_ctx* ctx, const cf_plan* plan, size_t copies) {
    uint32_t chunk = pred_chunk();
    const size_t budget = cf_hbm_budget(ctx, ctx->scratch_bytes, 1.0 / 3.0, 0);   // this context's share
    while (chunk > 2048 && chunk_slot_bytes(plan, chunk) * copies > budget) chunk /= 2;
    return chunk;
}
// Grow the context's slot scratch to `copies` chunks of `chunk` users; if the allocation fails
// (the HBM left is smaller than fit_chunk's estimate) the chunk halves, down to 256 users.
inline int ensure_slot_scratch(cf_ctx* ctx, const cf_plan* plan, size_t copies, uint32_t& chunk) {
    for (;;) {
        const size_t need = chunk_slot_bytes(plan, chunk) * copies;
        if (need <= ctx->scratch_bytes) return CF_OK;
        if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
        ctx->d_scratch = nullptr;
        ctx->scratch_bytes = 0;
        if (hipMalloc(&ctx->d_scratch, need) == hipSuccess) {
            ctx->scratch_bytes = need;
            return CF_OK;
        }
        (void)hipGetLastError();
        ctx->d_scratch = nullptr;
        if (chunk <= 256) return cf_set_error(ctx, CF_ENOMEM, "predictor slots (" + std::to_string(need) + " bytes)");
        chunk /= 2;
    }
}
inline size_t basis_lds() {
    return sizeof(double) * (kStageElems + 4) + CF_MAX_K * (sizeof(uint32_t) + sizeof(float) + 3 * sizeof(int)) +
           12 * sizeof(int) + CF_MAX_K * (3 * sizeof(uint64_t) + 2 * sizeof(int));   // ..., s_order, s_dmin
}
static_assert(2 * CF_MAX_K + CF_MAX_K / 2 <= kStageElems, "closed-form LDS copies exceed the staging area");
inline size_t rating_lds_fixed() {
    return sizeof(double) * (4 + 2 * CF_MAX_K) +                                      // s_misc, s_gx, s_hx
           CF_MAX_K * (sizeof(uint32_t) + sizeof(float) + 6 * sizeof(int)) + 12 * sizeof(int) +
           CF_MAX_K * (3 * sizeof(uint64_t) + sizeof(int)) + kWaves * CF_MAX_K * sizeof(int) +   // cmask, order, cb
           3 * CF_MAX_K * sizeof(uint64_t);                                                   // pmask
}

// Launch geometry of a bucket (everything but the chunk).
template <typename T>
int setup_bucket(cf_ctx* ctx, PredArgs<T>& args, int lmax, size_t& rating_lds) {
    args.lmax = lmax;
    const size_t lds_fixed = rating_lds_fixed();
    const int big = (lmax + 2) * (lmax + 3) / 2;
    // Per wave: the bordered system triangle of up to nmax rows plus y and g beside it.
    // nmax is the largest that keeps two 4-wave blocks per CU (<= 80 KiB each); the
    // block-wide systems use the LDS only where their full (lmax + 2)-row triangle fits as
    // well, else the slot's HBM region AP.
    const auto per_wave = [&](int n) { return fast_tri(n) + 2 * lmax; };   // + y (nc) and g (d)
    int nmax = std::min(kNsysMax, lmax);
    while (nmax > 8 && sizeof(double) * (size_t)(kWaves * per_wave(nmax)) + lds_fixed > kRatingLds) --nmax;
    args.nmax = nmax;
    args.ew = per_wave(nmax);
    args.big_lds = sizeof(double) * (size_t)std::max(big, kWaves * args.ew) + lds_fixed <= kRatingLds;
    args.a_elems = std::max({args.big_lds ? big : 0, kWaves * args.ew, 2 * lmax});
    args.so = slot_layout(lmax);
    rating_lds = sizeof(double) * (size_t)args.a_elems + lds_fixed;
    if (rating_lds > 163840) return cf_set_error(ctx, CF_ERANGE, "predict bucket exceeds LDS");
    CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)pred_dense_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)rating_lds));
    CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)pred_rating_kernel<T>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)rating_lds));
    CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)pred_basis_kernel<T>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)basis_lds()));
    return CF_OK;
}

// CF_PRED_FUSED=1 selects the fused persistent kernel; default: the two-kernel chunked path
// (C4 predict 1660 ms against 1803-1813 ms fused, profiles/r03/pred_fused_rejected/).
inline bool pred_fused_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("CF_PRED_FUSED");
        return e && e[0] == '1';
    }();
    return on;
}

// CF_PRED_TAIL=0 makes the last joint basis step write every column of X (A/B runs); default:
// only the column blocks the ratings read (from Lmin = min_r lim_r on).
inline int pred_tail_basis() {
    static const int on = [] {
        const char* e = std::getenv("CF_PRED_TAIL");
        return e && e[0] == '0' ? 0 : 1;
    }();
    return on;
}

// Fused launch of a bucket: dynamic LDS = the larger of the two halves, grid = the
// workgroups resident at once (capped by the launch bounds the slot set was sized for).
template <typename T>
int fused_geometry(cf_ctx* ctx, size_t rating_lds, uint32_t grid_cap, uint32_t& grid, size_t& lds) {
    lds = std::max(rating_lds, basis_lds());
    CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)pred_fused_kernel<T>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int per_cu = 0, cus = 0;
    CF_HIP_CHECK(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pred_fused_kernel<T>, kThreads, lds));
    CF_HIP_CHECK(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    grid = std::min<uint32_t>(grid_cap, (uint32_t)std::max(1, per_cu) * (uint32_t)std::max(1, cus));
    return CF_OK;
}

}  // namespace

template <typename T>
int cf_launch_predict(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                      const uint32_t* d_items, const float* d_ratings, const int32_t* d_m,
                      const T* d_evals, const uint64_t* d_evec_off, const T* d_evecs,
                      const T* d_sigtab, int sig_mode, float* d_mse, int32_t* d_kk,
                      double* d_pred, const uint8_t* d_row_sel, hipStream_t stream) {
    PredArgs<T> args{};
    args.order = plan->d_order;
    args.item_off = d_item_off;
    args.items = d_items;
    args.ratings = d_ratings;
    args.row_sel = d_row_sel;
    args.m = d_m;
    args.evals = d_evals;
    args.evec_off = d_evec_off;
    args.evecs = d_evecs;
    args.sigtab = d_sigtab;
    args.sig_mode = sig_mode;
    args.graph = graph_dev(ctx);
    args.n_items = ctx->n_items;
    args.mse = d_mse;
    args.kk = d_kk;
    args.pred = d_pred;
    args.phase_cycles = ctx->d_phase;
    args.tail_basis = pred_tail_basis();
    args.cmask_in = cf_cmask_lookup(ctx, plan, d_item_off, d_items);
    args.cmask_words = args.cmask_in ? ctx->cmask_bytes / sizeof(uint64_t) : 0;
    args.cmask_fp = args.cmask_in ? ctx->d_cmask_fp : nullptr;
    args.cmask_users = args.cmask_in ? ctx->cmask_users : 0;
    int rc = CF_OK;
    // Slots for one chunk of the largest LDS bucket, per stream; the chunks of every bucket
    // alternate between two context-owned streams (fork/join by events with the caller's
    // stream) so one chunk's tail overlaps the next.  Diagnostics keep one stream.
    const bool overlap = !ctx->d_phase;
    // fused (CF_PRED_FUSED=1): one slot per resident workgroup; the phase diagnostics keep the two kernels
    const bool fused = overlap && pred_fused_enabled();
    uint32_t fused_max = 0;
    if (fused) {
        int cus = 0;
        CF_HIP_CHECK(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
        fused_max = (uint32_t)std::max(1, cus) * CF_PRED_RATING_OCC;   // launch-bounds residency
        if (!ctx->d_pred_next)
            CF_HIP_CHECK(ctx, hipMalloc(&ctx->d_pred_next, 32 * sizeof(uint32_t) * cf_ctx::kAuxStreams));
    }
    const size_t copies = overlap ? cf_ctx::kAuxStreams : 1;
    uint32_t kChunk = fused ? fused_max : fit_chunk(ctx, plan, copies);
    CF_TRY(ensure_slot_scratch(ctx, plan, copies, kChunk));
    if (fused && kChunk != fused_max)   // one slot per resident workgroup is not negotiable
        return cf_set_error(ctx, CF_ENOMEM, "fused predictor slots");
    // block-wide ratings of the chunked path go to pred_dense_kernel: a queue per stream (every
    // rating of a chunk at most once) and one factorisation region per dense workgroup
    int n_cu = 0;
    CF_HIP_CHECK(ctx, hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, ctx->device));
    const uint32_t dense_grid = 2u * (uint32_t)std::max(1, n_cu);
    if (!fused) {
        // always kAuxStreams copies (the most any call uses): a buffer sized for one copy by a
        // call with the phase diagnostics on would otherwise be indexed past its end by the
        // second stream of a later overlapped call
        const size_t qw = 4 + 2 * (size_t)kChunk * (size_t)std::max<uint32_t>(plan->kmax, 2);
        const size_t ww = (size_t)dense_grid * ((size_t)(CF_MAX_K + 2) * (CF_MAX_K + 3) / 2);
        constexpr size_t kCopies = cf_ctx::kAuxStreams;
        if (qw > ctx->dense_q_words) {
            if (ctx->d_dense_q) (void)hipFree(ctx->d_dense_q);
            ctx->d_dense_q = nullptr;
            ctx->dense_q_words = 0;
            CF_TRY(cf_malloc_evict(ctx, reinterpret_cast<void**>(&ctx->d_dense_q), sizeof(uint32_t) * qw * kCopies,
                                   "dense rating queue"));
            ctx->dense_q_words = qw;
        }
        if (ww > ctx->dense_ws_doubles) {
            if (ctx->d_dense_ws) (void)hipFree(ctx->d_dense_ws);
            ctx->d_dense_ws = nullptr;
            ctx->dense_ws_doubles = 0;
            CF_TRY(cf_malloc_evict(ctx, reinterpret_cast<void**>(&ctx->d_dense_ws), sizeof(double) * ww * kCopies,
                                   "dense factorisation regions"));
            ctx->dense_ws_doubles = ww;
        }
    }
    const size_t need = chunk_slot_bytes(plan, kChunk);   // one copy
    if (fused) kChunk = 0;
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
                                            d_evecs, d_sigtab, sig_mode, d_mse, d_kk, d_pred, d_row_sel, st);
            if (rc != CF_OK) break;
            if (overlap) {
                CF_HIP_CHECK(ctx, hipEventRecord(ctx->aux_event[0], st));
                for (int i = 1; i < cf_ctx::kAuxStreams; ++i) CF_HIP_CHECK(ctx, hipStreamWaitEvent(ctx->aux_stream[i], ctx->aux_event[0], 0));
            }
            continue;
        }
        size_t rating_lds = 0;
        rc = setup_bucket<T>(ctx, args, std::max<int>(2, 16 * b.emax), rating_lds);
        if (rc != CF_OK) break;
        if (fused) {   // the whole bucket in one persistent launch, users claimed largest-k first
            uint32_t grid = 0;
            size_t lds = 0;
            rc = fused_geometry<T>(ctx, rating_lds, fused_max, grid, lds);
            if (rc != CF_OK) break;
            grid = std::min(grid, b.count);
            const int si = nb++ % cf_ctx::kAuxStreams;
            hipStream_t st = ctx->aux_stream[si];
            args.slots = reinterpret_cast<double*>(static_cast<char*>(ctx->d_scratch) + si * need);
            if ((size_t)grid * args.so.stride * sizeof(double) > need) {
                rc = cf_set_error(ctx, CF_EINVAL, "predict scratch undersized");
                break;
            }
            uint32_t* next = ctx->d_pred_next + 32 * si;
            if (hipMemsetAsync(next, 0, sizeof(uint32_t), st) != hipSuccess) {
                rc = cf_set_error(ctx, CF_EHIP, "predict counter reset failed");
                break;
            }
            hipLaunchKernelGGL(pred_fused_kernel<T>, dim3(grid), dim3(kThreads), lds, st, args, b.first, b.count, next);
            if (hipGetLastError() != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, "predict launch failed");
            continue;
        }
        for (uint32_t c0 = 0; c0 < b.count && rc == CF_OK; c0 += kChunk) {
            const uint32_t cnt = std::min(kChunk, b.count - c0);
            const int si = overlap ? (nb++ % cf_ctx::kAuxStreams) : 0;
            hipStream_t st = overlap ? ctx->aux_stream[si] : stream;
            args.slots = reinterpret_cast<double*>(static_cast<char*>(ctx->d_scratch) + si * need);
            if ((size_t)cnt * args.so.stride * sizeof(double) > need) {
                rc = cf_set_error(ctx, CF_EINVAL, "predict scratch undersized");
                break;
            }
            // one workgroup per user of the chunk: the hardware dispatcher balances the
            // per-user cost (~k^3) dynamically
            hipLaunchKernelGGL(pred_basis_kernel<T>, dim3(cnt), dim3(kThreads), basis_lds(), st, args, b.first + c0, cnt);
            args.dq = ctx->d_dense_q + si * ctx->dense_q_words;
            args.dense_ws = ctx->d_dense_ws + si * ctx->dense_ws_doubles;
            if (hipMemsetAsync(args.dq, 0, 4 * sizeof(uint32_t), st) != hipSuccess) {
                rc = cf_set_error(ctx, CF_EHIP, "dense queue reset failed");
                break;
            }
            hipLaunchKernelGGL(pred_rating_kernel<T>, dim3(cnt), dim3(kThreads), rating_lds, st, args, b.first + c0,
                               cnt);
            hipLaunchKernelGGL(pred_dense_kernel<T>, dim3(dense_grid), dim3(kThreads), rating_lds, st, args,
                               b.first + c0);
            args.dq = nullptr;
            if (hipGetLastError() != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, "predict launch failed");
        }
        if (rc != CF_OK) break;
    }
    if (overlap)
        for (int i = 0; i < cf_ctx::kAuxStreams; ++i) {
            CF_HIP_CHECK(ctx, hipEventRecord(ctx->aux_event[i], ctx->aux_stream[i]));
            CF_HIP_CHECK(ctx, hipStreamWaitEvent(stream, ctx->aux_event[i], 0));
        }
    return rc;
}

// Fused step: cf_eigen_run + cf_predict_run_f32 with per-bucket overlap.  Eigen buckets
// alternate between the context's two aux streams (as cf_eigen_run); each records an event,
// and the predictor chunks of that bucket start on the two predictor streams as soon as it
// fires, so a bucket's prediction (fp64 MFMA, latency-bound) runs beside the next buckets'
// Jacobi sweeps (fp32 VALU + LDS) instead of after all of them.  In compat mode every user's
// w_lim reads the global sig table (the sigs of the first users, local_calc_precomp.cpp:414,
// 437,440), so those users' eigen pass runs first on its own (a prefix plan; their bucket
// later rewrites the same bits).  Events: step_time_ev = {start, eigen done, end}.
int cf_launch_step(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items,
                   const float* d_ratings, const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs, float* d_evals,
                   float* d_evecs, int sig_mode, float* d_mse, int32_t* d_kk, double* d_pred, hipStream_t stream) {
    if (ctx->eigen_method != CF_EIGEN_JACOBI || ctx->d_stats || ctx->d_phase || plan->buckets.size() > 16) {
        // diagnostics / the tridiagonal solver: the two stages one after the other
        CF_TRY(cf_launch_eigen(ctx, plan, d_item_off, d_items, d_evec_off, d_m, d_sigs, d_evals, d_evecs, stream));
        return cf_launch_predict<float>(ctx, plan, d_item_off, d_items, d_ratings, d_m, d_evals, d_evec_off, d_evecs,
                                        d_sigs, sig_mode, d_mse, d_kk, d_pred, nullptr, stream);
    }
    if (!ctx->aux_stream[0])
        for (int i = 0; i < cf_ctx::kAuxStreams; ++i) {
            CF_HIP_CHECK(ctx, hipStreamCreateWithFlags(&ctx->aux_stream[i], hipStreamNonBlocking));
            CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&ctx->aux_event[i], hipEventDisableTiming));
        }
    if (!ctx->aux_event[cf_ctx::kAuxStreams])
        CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&ctx->aux_event[cf_ctx::kAuxStreams], hipEventDisableTiming));
    if (!ctx->step_stream[0]) {
        for (hipStream_t& st : ctx->step_stream) CF_HIP_CHECK(ctx, hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        for (hipEvent_t& e : ctx->step_bucket_ev) CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (hipEvent_t& e : ctx->step_sync_ev) CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (hipEvent_t& e : ctx->step_time_ev) CF_HIP_CHECK(ctx, hipEventCreate(&e));
    }
    hipStream_t* es = ctx->aux_stream;   // eigen
    hipStream_t* ps = ctx->step_stream;  // predict
    // compat prefix: the users whose sigs cover rows [0, kmax) of the concatenated table
    cf_plan* pre = nullptr;
    if (sig_mode == CF_SIGS_COMPAT && plan->n_users) {
        if (!plan->prefix) {
            uint32_t j = 0;
            while (j < plan->n_users && plan->h_item_off[j] < plan->kmax) ++j;
            CF_TRY(cf_plan_create(ctx, j, plan->h_item_off.data(), &const_cast<cf_plan*>(plan)->prefix));
        }
        pre = plan->prefix;
    }
    PredArgs<float> args{};
    args.order = plan->d_order;
    args.item_off = d_item_off;
    args.items = d_items;
    args.ratings = d_ratings;
    args.m = d_m;
    args.evals = d_evals;
    args.evec_off = d_evec_off;
    args.evecs = d_evecs;
    args.sigtab = d_sigs;
    args.sig_mode = sig_mode;
    args.graph = graph_dev(ctx);
    args.n_items = ctx->n_items;
    args.mse = d_mse;
    args.kk = d_kk;
    args.pred = d_pred;
    args.tail_basis = pred_tail_basis();
    // the eigen kernels hand the predictor its complement masks (24 B per rating); without the
    // buffer (CF_STEP_MASKS=0, or no HBM for it) the basis kernel gathers the graph itself
    uint64_t* d_cmask = cf_cmask_buffer(ctx, plan);
    cf_cmask_mark(ctx, plan, d_item_off, d_items, false);
    args.cmask_in = d_cmask;
    args.cmask_words = d_cmask ? ctx->cmask_bytes / sizeof(uint64_t) : 0;
    args.cmask_fp = d_cmask ? ctx->d_cmask_fp : nullptr;
    args.cmask_users = d_cmask ? ctx->cmask_users : 0;
    uint32_t kChunk = fit_chunk(ctx, plan, 2);
    CF_TRY(ensure_slot_scratch(ctx, plan, 2, kChunk));
    const size_t need = chunk_slot_bytes(plan, kChunk);   // one copy
    // fork every stream from the caller's
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->step_time_ev[0], stream));
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->aux_event[cf_ctx::kAuxStreams], stream));
    for (int i = 0; i < 2; ++i) {
        CF_HIP_CHECK(ctx, hipStreamWaitEvent(es[i], ctx->aux_event[cf_ctx::kAuxStreams], 0));
        CF_HIP_CHECK(ctx, hipStreamWaitEvent(ps[i], ctx->aux_event[cf_ctx::kAuxStreams], 0));
    }
    int rc = CF_OK;
    // after the fork a failed event call sets rc and skips the rest, so the join below always
    // orders the caller's stream after every kernel already queued on es / ps
#define CF_STEP_CHECK(expr)                                                                            \
    if (rc == CF_OK) {                                                                                 \
        const hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    }
    if (pre) {   // prefix users first, then every predictor stream waits for their sigs
        rc = cf_launch_eigen(ctx, pre, d_item_off, d_items, d_evec_off, d_m, d_sigs, d_evals, d_evecs, ps[0]);
        CF_STEP_CHECK(hipEventRecord(ctx->step_sync_ev[0], ps[0]));
        CF_STEP_CHECK(hipStreamWaitEvent(ps[1], ctx->step_sync_ev[0], 0));
    }
    int nb = 0, nc = 0;
    for (size_t bi = 0; bi < plan->buckets.size() && rc == CF_OK; ++bi) {
        const cf_bucket& b = plan->buckets[bi];
        if (b.count == 0) continue;
        hipStream_t est = es[nb++ % 2];
        if (b.emax == kSpillBucket) {   // spill eigen alone first (it fills the chip), as cf_launch_eigen
            rc = cf_launch_eigen_spill(ctx, plan, b, d_item_off, d_items, d_evec_off, d_m, d_sigs, d_evals, d_evecs,
                                       es[0]);
            if (rc != CF_OK) break;
            CF_STEP_CHECK(hipEventRecord(ctx->step_bucket_ev[bi], es[0]));
            CF_STEP_CHECK(hipStreamWaitEvent(es[1], ctx->step_bucket_ev[bi], 0));
            CF_STEP_CHECK(hipStreamWaitEvent(ps[0], ctx->step_bucket_ev[bi], 0));
            rc = cf_launch_predict_spill<float>(ctx, plan, b, d_item_off, d_items, d_ratings, d_m, d_evals, d_evec_off,
                                                d_evecs, d_sigs, sig_mode, d_mse, d_kk, d_pred, nullptr, ps[0]);
            continue;
        }
        rc = cf_launch_eigen_flagged(ctx, plan, b.emax, b.first, b.count, nullptr, d_item_off, d_items, d_evec_off,
                                     d_m, d_sigs, d_evals, d_evecs, est, d_cmask);
        if (rc != CF_OK) break;
        CF_STEP_CHECK(hipEventRecord(ctx->step_bucket_ev[bi], est));
        size_t rating_lds = 0;
        rc = setup_bucket<float>(ctx, args, std::max<int>(2, 16 * b.emax), rating_lds);
        if (rc != CF_OK) break;
        bool waited[2] = {false, false};
        for (uint32_t c0 = 0; c0 < b.count; c0 += kChunk) {
            const uint32_t cnt = std::min(kChunk, b.count - c0);
            const int si = nc++ % 2;
            if (!waited[si]) {
                CF_STEP_CHECK(hipStreamWaitEvent(ps[si], ctx->step_bucket_ev[bi], 0));
                waited[si] = true;
            }
            if (rc != CF_OK) break;
            args.slots = reinterpret_cast<double*>(static_cast<char*>(ctx->d_scratch) + si * need);
            hipLaunchKernelGGL(pred_basis_kernel<float>, dim3(cnt), dim3(kThreads), basis_lds(), ps[si], args,
                               b.first + c0, cnt);
            hipLaunchKernelGGL(pred_rating_kernel<float>, dim3(cnt), dim3(kThreads), rating_lds, ps[si], args,
                               b.first + c0, cnt);
            if (hipGetLastError() != hipSuccess) {
                rc = cf_set_error(ctx, CF_EHIP, "step predict launch failed");
                break;
            }
        }
    }
#undef CF_STEP_CHECK
    // join: eigen streams -> "eigen done" event on the caller, then the predictor streams
    for (int i = 0; i < 2; ++i) {
        CF_HIP_CHECK(ctx, hipEventRecord(ctx->aux_event[i], es[i]));
        CF_HIP_CHECK(ctx, hipStreamWaitEvent(stream, ctx->aux_event[i], 0));
    }
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->step_time_ev[1], stream));
    for (int i = 0; i < 2; ++i) {
        CF_HIP_CHECK(ctx, hipEventRecord(ctx->step_sync_ev[1 + i], ps[i]));
        CF_HIP_CHECK(ctx, hipStreamWaitEvent(stream, ctx->step_sync_ev[1 + i], 0));
    }
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->step_time_ev[2], stream));
    cf_cmask_mark(ctx, plan, d_item_off, d_items, rc == CF_OK && d_cmask);
    return rc;
}

uint64_t* cf_cmask_buffer(cf_ctx* ctx, const cf_plan* plan) {
    if (!ctx->step_masks || !plan->n_users) return nullptr;
    const size_t mb = 3 * sizeof(uint64_t) * (size_t)plan->h_item_off[plan->n_users];
    if (plan->n_users > ctx->cmask_users) {   // the fingerprints: a separate buffer, so plans of
        if (ctx->d_cmask_fp) (void)hipFree(ctx->d_cmask_fp);   // different sizes never overlap
        ctx->d_cmask_fp = nullptr;
        ctx->cmask_users = 0;
        ctx->cmask_gen = ~0ull;
        if (hipMalloc(&ctx->d_cmask_fp, sizeof(uint64_t) * plan->n_users) != hipSuccess) {
            (void)hipGetLastError();
            ctx->d_cmask_fp = nullptr;
            return nullptr;
        }
        ctx->cmask_users = plan->n_users;
    }
    if (mb > ctx->cmask_bytes) {
        if (ctx->d_cmask) (void)hipFree(ctx->d_cmask);
        ctx->d_cmask = nullptr;
        ctx->cmask_bytes = 0;
        ctx->cmask_gen = ~0ull;
        if (hipMalloc(&ctx->d_cmask, mb) != hipSuccess) {   // optional: the predictor gathers instead
            (void)hipGetLastError();
            ctx->d_cmask = nullptr;
            return nullptr;
        }
        ctx->cmask_bytes = mb;
    }
    return static_cast<uint64_t*>(ctx->d_cmask);
}

void cf_cmask_mark(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items, bool valid) {
    ctx->cmask_plan = plan->id;
    ctx->cmask_key[0] = d_item_off;
    ctx->cmask_key[1] = d_items;
    ctx->cmask_gen = valid ? ctx->graph_gen : ~0ull;
}

const uint64_t* cf_cmask_lookup(const cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                                const uint32_t* d_items) {
    const bool hit = ctx->d_cmask && ctx->cmask_gen == ctx->graph_gen && ctx->cmask_plan == plan->id &&
                     ctx->cmask_key[0] == d_item_off && ctx->cmask_key[1] == d_items;
    return hit ? static_cast<const uint64_t*>(ctx->d_cmask) : nullptr;
}

template int cf_launch_predict<float>(cf_ctx*, const cf_plan*, const uint64_t*, const uint32_t*,
                                      const float*, const int32_t*, const float*, const uint64_t*,
                                      const float*, const float*, int, float*, int32_t*, double*,
                                      const uint8_t*, hipStream_t);
template int cf_launch_predict<double>(cf_ctx*, const cf_plan*, const uint64_t*, const uint32_t*,
                                       const float*, const int32_t*, const double*,
                                       const uint64_t*, const double*, const double*, int, float*,
                                       int32_t*, double*, const uint8_t*, hipStream_t);

// The fast path's largest system (rows min(nc, d)) in a bucket of Gram bound lmax: the nmax
// setup_bucket derives from the LDS budget.  Ratings with a larger system take the block-wide
// path; the parity tests use it to tell which rank-deficient rows return the minimum-norm
// prediction.
extern "C" int cf_debug_predict_nmax(int lmax) {
    if (lmax < 2 || lmax > CF_MAX_K) return -1;
    const size_t lds_fixed = rating_lds_fixed();
    const auto per_wave = [&](int n) { return fast_tri(n) + 2 * lmax; };
    int nmax = std::min(kNsysMax, lmax);
    while (nmax > 8 && sizeof(double) * (size_t)(kWaves * per_wave(nmax)) + lds_fixed > kRatingLds) --nmax;
    return nmax;
}
