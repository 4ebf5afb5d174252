// cf_local.hip -- local_calc (a8) on gfx950: the per-movie graph-signal predictor.
//
// Replaces vertex_program::apply of local_calc.cpp:262-526.  For each movie vertex m
// with n = 1 + #out-neighbours >= 3 (:269-272):
//   1. eigen_kernel<kLocal>: the local graph's W (star-shaped, w > 0.1), L2 without the
//      0 -> 1 degree rule, all n eigenpairs, and the full L2 kept in HBM (:276-378);
//   2. eigen_kernel<kSigma>, one workgroup per (movie, test user): w_lim =
//      sqrt(lambda_min(L2_h L2_h^T)) = sigma_min(L2_h) over the user's unrated rows h,
//      by the same one-sided Jacobi on the columns L2_h^T (:402-436);
//   3. local_predict_kernel, one workgroup per pair: lim = first eigenvalue > w_lim (>= 2,
//      :444-451), the bordered Gram M = U_C^T U_C of the rated rows C (no zero-column
//      filter, :455-485) factored by the blocked LDL^T of cf_ldlt.hpp, pred = v^T M^-1
//      U_C^T (r - mean) + mean, clamp, mse (float), kk = |C| (:487-521).
// Test ratings are looked up in a CSR over compact item ids (users ascending).

#include <algorithm>
#include <vector>

#include "cf_internal.h"
#include "cf_ldlt.hpp"

namespace {

constexpr int kThreads = 256;

struct LocalPredArgs {
    const uint32_t* pair_movie;   // pair -> movie unit
    const uint32_t* pair_user;    // pair -> test user
    const uint64_t* pair_out;     // pair -> output slot (its test-rating entry)
    const uint64_t* item_off;     // movie unit -> [m, out-neighbours...]
    const uint32_t* items;
    const float* evals;           // per movie unit at item_off, n values ascending
    const uint64_t* evec_off;     // per movie unit, n x n row-major
    const float* evecs;
    const float* wlim;            // per pair
    const uint64_t* test_off;
    const uint32_t* test_user;
    const float* test_rating;
    float* mse;
    int32_t* kk;
    double* pred;
    int32_t* lim_out;
    int lmax;
};

__device__ float lookup_rating(const LocalPredArgs& a, uint32_t movie, uint32_t user) {
    uint64_t lo = a.test_off[movie];
    const uint64_t end = a.test_off[movie + 1];
    uint64_t hi = end;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a.test_user[mid] < user) lo = mid + 1;
        else hi = mid;
    }
    return (lo < end && a.test_user[lo] == user) ? a.test_rating[lo] : 0.0f;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__global__ __launch_bounds__(kThreads) void local_predict_kernel(LocalPredArgs a, uint32_t n_pairs) {
    extern __shared__ double dsm[];
    const int lmax = a.lmax;
    double* A = dsm;                                                   // (lmax+2)(lmax+3)/2
    double* s_misc = A + (size_t)(lmax + 2) * (lmax + 3) / 2;          // [0] mean [1] real
    float* s_rat = reinterpret_cast<float*>(s_misc + 4);
    int* s_c = reinterpret_cast<int*>(s_rat + CF_MAX_K);
    int* s_cnt = s_c + CF_MAX_K;                                       // [0..3] waves, [4] lim
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    for (uint32_t p = blockIdx.x; p < n_pairs; p += gridDim.x) {
        const uint32_t mv = a.pair_movie[p];
        const uint32_t user = a.pair_user[p];
        const uint64_t base = a.item_off[mv];
        const int n = (int)(a.item_off[mv + 1] - base);
        const float* U = a.evecs + a.evec_off[mv];
        __syncthreads();
        // ratings of the local graph's rows by this user; row 0 is the unknown (:400-405)
        float r = 0.0f;
        if (tid < n) {
            const float v = lookup_rating(a, a.items[base + tid], user);
            if (tid == 0) s_misc[1] = (double)v;
            r = tid == 0 ? 0.0f : v;
            s_rat[tid] = r;
        }
        // rated rows C in row order (:470-479), ordered ballot compaction
        const bool rated = tid < n && r != 0.0f;
        const unsigned long long bal = __ballot(rated);
        if (lane == 0) s_cnt[wave] = __popcll(bal);
        __syncthreads();
        int off = 0;
        for (int w = 0; w < wave; ++w) off += s_cnt[w];
        const int c = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        if (rated) s_c[off + __popcll(bal & ((1ull << lane) - 1ull))] = tid;
        if (tid == 0) {
            // lim = first eigenvalue above w_lim, >= 2 (:444-451)
            const double wl = (double)a.wlim[p];
            int lim = 0;
            for (; lim < n; ++lim)
                if ((double)a.evals[base + lim] > wl) break;
            if (lim < 2) lim = 2;
            s_cnt[4] = lim;
        }
        __syncthreads();
        const int L = s_cnt[4];
        if (wave == 0) {
            double sum = 0.0;
            for (int i = lane; i < c; i += 64) sum += (double)s_rat[s_c[i]];
            sum = wave_sum(sum);
            if (lane == 0) s_misc[0] = sum / (double)c;   // 0/0 = NaN when nothing is rated (:487)
        }
        __syncthreads();
        const double mean = s_misc[0];
        // bordered Gram: A[a][b] = (U_C^T U_C)_ab (b <= a < L), A[L][b] = t_b, A[L+1][b] = v_b
        for (int e = tid; e < L * (L + 1) / 2; e += kThreads) {
            int ra = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
            while (ra * (ra + 1) / 2 > e) --ra;
            while ((ra + 1) * (ra + 2) / 2 <= e) ++ra;
            const int rb = e - ra * (ra + 1) / 2;
            double g = 0.0;
            for (int i = 0; i < c; ++i) {
                const float* row = U + (size_t)s_c[i] * n;
                g = fma((double)row[ra], (double)row[rb], g);
            }
            A[e] = g;
        }
        for (int b = tid; b < L; b += kThreads) {
            double t = 0.0;
            for (int i = 0; i < c; ++i) {
                const int ri = s_c[i];
                t = fma((double)U[(size_t)ri * n + b], (double)s_rat[ri] - mean, t);
            }
            A[tri(L, b)] = t;
            A[tri(L + 1, b)] = (double)U[b];   // vv = row 0 (:465-466)
        }
        __syncthreads();
        ldlt_bordered<kThreads>(A, L, L + 2);
        if (wave == 0) {
            double dot = 0.0;
            for (int j = lane; j < L; j += 64) dot = fma(A[tri(L, j)] * A[tri(L + 1, j)], A[tri(j, j)], dot);
            dot = wave_sum(dot);
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
    }
}

// ---- w_lim of the pairs of units with n > CF_MAX_K, shared per movie ---------------------
// L2_h L2_h^T (:425-435) is the principal submatrix B_hh of B = L2 L2^T with the user's rated
// rows R deleted.  With B = W Theta W^T (spill eigen mode 3, once per movie) and mu not an
// eigenvalue, Haynsworth's inertia additivity on B - mu (whose inverse has the R-block
// F(mu) = W_R (Theta - mu)^-1 W_R^T, the inverse of the Schur complement of B_hh - mu) gives
//   #{eigenvalues of B_hh below mu} = #{theta_j < mu} - #{negative eigenvalues of F(mu)},
// and interlacing puts lambda_min(B_hh) in [theta_0, theta_c] (c = |R|).  The bracket shrinks
// on that count: per step one c x c F(mu) on the fp64 matrix cores and its LDL^T inertia
// (replacing the per-pair fp64 Gram + tridiagonalisation of n x n, mode 2 of
// eigen_spill_kernel, ~n^3 per pair).  Inside a bracket with no pole theta_j, F is smooth and
// exactly one of its eigenvalues crosses zero at lambda_min(B_hh) (dF/dmu = W_R (Theta -
// mu)^-2 W_R^T is positive definite, so they all increase), so det F changes sign there:
// the next mu is the Illinois regula-falsi point on det F (its log and sign from the LDL^T
// pivots) when both ends carry opposite signs, the midpoint otherwise -- ~10-15 steps to the
// fp32 result instead of 44 bisections.  One workgroup per pair; pairs with c > kWlimCmax
// keep mode 2 (solved = 0).
//
// F on v_mfma_f64_16x16x4_f64: F's 16 x 16 lower tiles (<= 78 at c = 184) are spread over the
// four waves (row tiles snake-assigned: at most 21 accumulator tiles per wave), W_R's columns
// staged through LDS kWlimKc at a time as fp64 (exact: fp32 values), the scaling d_j =
// 1 / (theta_j - mu) applied to the A operand in registers; the next chunk's loads are in
// flight while the current one is multiplied.  The accumulators then move to the packed
// lower triangle (which aliases the staging area) for the LDL^T.
// Three size classes of the kernel, by c: F's packed triangle is sized for the class's
// largest c, so the common small systems (c <= 64: 17 KB of LDS, 4 accumulator tiles per
// wave) run eight workgroups per CU instead of the one that a 184-row triangle (136 KB)
// leaves room for -- the iterations are latency chains (staged W_R chunks, one barrier per
// LDL^T pivot), and more resident pairs hide them (r05: one 29 s launch at one wave per SIMD).
constexpr int kWlimCmax = 184;   // largest class: every pair of a k <= 180 user
constexpr int kWlimIters = 64;
constexpr double kWlimTol = 1e-9;    // relative bracket width at exit (w_lim = sqrt, fp32: 5e-10 << 6e-8)
// accumulator tiles of the busiest wave under the snake row-tile map {w, 7 - w, 8 + w}
constexpr int wlim_slots(int T) {
    int best = 0;
    for (int w = 0; w < 4; ++w) {
        const int pr[3] = {w, 7 - w, 8 + w};
        int sl = 0;
        for (int x = 0; x < 3; ++x)
            if (pr[x] < T) sl += T - pr[x];
        best = sl > best ? sl : best;
    }
    return best;
}
template <int CMAX>
struct WlimGeom {
    static constexpr int kTiles = (CMAX + 15) / 16;                  // row tiles of F
    static constexpr int kLd = 16 * kTiles + 4;                      // staged row stride (doubles)
    static constexpr int kSlots = wlim_slots(kTiles);
    // columns of W_R staged per chunk (a barrier pair and a load round trip each): 32 for the
    // classes with room, 16 where F's registers fill the file (64 spilled)
    static constexpr int kKc = (kTiles > 4 && kTiles <= 8) ? 32 : 16;
    static constexpr int kLoads = (16 * kTiles * kKc + kThreads - 1) / kThreads;   // floats per thread
    static constexpr int kFElems = CMAX * (CMAX + 1) / 2;
    static constexpr int kStageElems = kKc * kLd + kKc;
    static constexpr int kSmem = kFElems > kStageElems ? kFElems : kStageElems;   // F aliases the staging
    static_assert(kTiles <= 12, "the snake row-tile map covers 12 row tiles");
};
static_assert(WlimGeom<184>::kSlots == 21 && WlimGeom<64>::kSlots == 4 && WlimGeom<128>::kSlots == 9, "slots");
struct WlimArgs {
    uint32_t n_pairs;
    const uint32_t* pair_movie;
    const uint32_t* pair_user;
    const uint64_t* item_off;
    const uint32_t* items;
    const float* theta;     // per movie unit at item_off: eigenvalues of B, ascending
    const uint64_t* w_off;  // per movie unit: its n x n eigenvector block, row-major
    const float* W;         // B's eigenvectors (spill eigen mode 3)
    const float* W_sym;     // units with sym[v] != 0: L2's own eigenvectors (mode 1), B = L2^2
    const uint8_t* sym;
    const uint64_t* test_off;
    const uint32_t* test_user;
    const float* test_rating;
    float* wlim;
    uint8_t* solved;
    int32_t* pair_c;        // rated rows per pair (-1: not counted yet), shared by the classes
    unsigned long long* stats;   // optional (CF_LOCAL_VERBOSE): per class {pairs, iterations, secant steps, c}
};

// #{theta_j < x} (or <= x) over the ascending eigenvalues
__device__ __forceinline__ int count_below(const float* th, int n, double x, bool le = false) {
    int l = 0, h = n;
    while (l < h) {
        const int md = (l + h) >> 1;
        const double t = (double)th[md];
        if (t < x || (le && t == x)) l = md + 1;
        else h = md;
    }
    return l;
}

// Pairs with CLO < c <= CMAX (c = rated rows of the unit); the others are left to their class.
// Waves per SIMD the class is held to (its registers): 2 for c <= 128 (two workgroups per CU; at
// 3 or 4 the c <= 64 class spills 0.6 KB per lane), 1 for the largest class (LDS for one).
constexpr int wlim_wpe(int cmax) { return cmax <= 64 ? 2 : (cmax <= 128 ? 2 : 1); }
template <int CMAX, int CLO>
__global__ __launch_bounds__(kThreads, wlim_wpe(CMAX)) void local_wlim_kernel(WlimArgs a) {
    using f64x4 = __attribute__((ext_vector_type(4))) double;
    using Geo = WlimGeom<CMAX>;
    constexpr int kWlimTiles = Geo::kTiles;
    constexpr int kWlimLd = Geo::kLd;
    constexpr int kWlimSlots = Geo::kSlots;
    constexpr int kWlimLoads = Geo::kLoads;
    constexpr int kWlimKc = Geo::kKc;
    __shared__ double s_F[Geo::kSmem];   // packed lower F; the staging tiles alias its start
    __shared__ int s_R[CMAX];
    __shared__ int s_c[kThreads / 64];
    __shared__ double s_x[4];
    __shared__ double s_red[2 * (kThreads / 64)];
    double* const Ws = s_F;                        // [kWlimKc][kWlimLd]
    double* const Ds = s_F + kWlimKc * kWlimLd;    // [kWlimKc]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    LocalPredArgs la{};   // lookup_rating's test arrays
    la.test_off = a.test_off;
    la.test_user = a.test_user;
    la.test_rating = a.test_rating;
    for (uint32_t p = blockIdx.x; p < a.n_pairs; p += gridDim.x) {
        const uint32_t v = a.pair_movie[p], user = a.pair_user[p];
        const uint64_t base = a.item_off[v];
        const int n = (int)(a.item_off[v + 1] - base);
        {   // another class's pair: skip before any work (its count is known after the first class)
            const int c0 = a.pair_c[p];
            if (c0 >= 0 && (c0 <= CLO || c0 > CMAX)) continue;   // uniform
        }
        if (n > 65535) continue;   // 32-bit offsets into the n x n block below: mode 2 (solved = 0)
        // rated rows, ascending (row 0, the movie itself, counts as unrated: :405-413)
        int c = 0;
        for (int b0 = 0; b0 < n; b0 += kThreads) {
            const int i = b0 + tid;
            const bool rated = i >= 1 && i < n && lookup_rating(la, a.items[base + i], user) != 0.0f;
            const unsigned long long bal = __ballot(rated);
            if (lane == 0) s_c[wave] = __popcll(bal);
            __syncthreads();
            int off = c, all = 0;
            for (int w = 0; w < kThreads / 64; ++w) {
                if (w < wave) off += s_c[w];
                all += s_c[w];
            }
            const int pos = off + __popcll(bal & ((1ull << lane) - 1ull));
            if (rated && pos < CMAX) s_R[pos] = i;
            c += all;
            __syncthreads();
        }
        if (tid == 0) a.pair_c[p] = c;
        if (c <= CLO || c > CMAX) continue;   // uniform: another class's (c > kWlimCmax: mode 2)
        const float* th = a.theta + base;
        const float* Wv = (a.sym && a.sym[v] ? a.W_sym : a.W) + a.w_off[v];
        // this wave's row tiles (snake order over the rows, largest first) and tile slots
        const int nt = (c + 15) >> 4;
        const int pr[3] = {wave, 7 - wave, 8 + wave};
        int rows[3], rstart[3], nslot = 0;
#pragma unroll
        for (int x = 0; x < 3; ++x) {
            rows[x] = pr[x] < nt ? nt - 1 - pr[x] : -1;
            rstart[x] = nslot;
            nslot += rows[x] >= 0 ? rows[x] + 1 : 0;
        }
        auto slot_ij = [&](int sl, int& I, int& J) {
            const int x = sl >= rstart[2] && rows[2] >= 0 ? 2 : (sl >= rstart[1] && rows[1] >= 0 ? 1 : 0);
            I = rows[x];
            J = sl - rstart[x];
        };
        // this thread's staged elements: column tid % kWlimKc of the chunk, rows tid / kWlimKc +
        // kRowStep q -- every row of the 16 nt row tiles, rows >= c staged as 0 (sR = -1), so no
        // tile row reads stale LDS
        static_assert(kThreads % kWlimKc == 0, "one staged column per thread");
        const int scol = tid % kWlimKc, srow0 = tid / kWlimKc;
        constexpr int kRowStep = kThreads / kWlimKc;
        static_assert(kRowStep * kWlimLoads >= 16 * kWlimTiles && 16 * kWlimTiles <= kWlimLd,
                      "the staged rows cover every row tile");
        // 32-bit element offsets of this thread's staged rows in the unit's n x n block (n <=
        // 65535 keeps them in range; ~0u: past c) -- 64-bit addresses per load were hoisted and
        // spilled
        uint32_t roff[kWlimLoads];
#pragma unroll
        for (int q = 0; q < kWlimLoads; ++q) {
            const int r = srow0 + kRowStep * q;
            roff[q] = r < c ? (uint32_t)s_R[r] * (uint32_t)n + (uint32_t)scol : ~0u;
        }
        double lo = (double)th[0], hi = (double)th[min(c, n - 1)];
        bool guess = false;   // hi is the Rayleigh bound: the first trial point sits just below it
        if (c > 0) {
            // A tighter upper end: lambda_min(B_hh) <= the Rayleigh quotient of x = w_0 with its
            // rated rows zeroed (B's lowest eigenvector, whose eigenvalue the deletion lifts the
            // least).  In B's eigenbasis z = W^T x = e_0 - s, s_j = sum_{r in R} W_rj W_r0, so
            // x^T B x / x^T x = sum_j theta_j z_j^2 / sum_j z_j^2: c n multiply-adds, about one
            // F-build's loads and no MFMA, against the ~5 bisections from theta_c it saves (r06:
            // 29-31 iterations per pair on the C2 leg).  The 1e-6 margin covers fp32 W's
            // departure from orthonormality.
            double* w0 = s_F;   // c <= CMAX doubles; F / the staging are not in use yet
            for (int r = tid; r < c; r += kThreads) w0[r] = (double)Wv[(uint32_t)s_R[r] * (uint32_t)n];
            __syncthreads();
            double num = 0.0, den = 0.0;
            for (int j = tid; j < n; j += kThreads) {
                double sj = 0.0;
                for (int r = 0; r < c; ++r) sj = fma((double)Wv[(uint32_t)s_R[r] * (uint32_t)n + (uint32_t)j], w0[r], sj);
                const double z = (j == 0 ? 1.0 : 0.0) - sj;
                num = fma((double)th[j] * z, z, num);
                den = fma(z, z, den);
            }
            num = wave_sum(num);
            den = wave_sum(den);
            if (lane == 0) {
                s_red[2 * wave] = num;
                s_red[2 * wave + 1] = den;
            }
            __syncthreads();
            num = den = 0.0;
            for (int w = 0; w < kThreads / 64; ++w) {
                num += s_red[2 * w];
                den += s_red[2 * w + 1];
            }
            if (den > 0.0) {
                const double rq = num / den * (1.0 + 1e-6);
                if (rq > lo && rq < hi) {
                    hi = rq;
                    guess = true;
                }
            }
            __syncthreads();   // w0 (s_F) is reused as the staging area below
        }
        double Llo = 0.0, Lhi = 0.0;      // log2 |det F| at the ends (valid when s*** != 0)
        int slo = 0, shi = 0;             // sign of det F at the ends (0: unknown)
        int kept = 0;                     // +1 / -1: which end the last two steps kept
        int last_secant = 0;
        double w_prev = hi - lo;
        int n_it = 0, n_sec = 0;
        for (int it = 0; it < kWlimIters && c > 0 && hi - lo > kWlimTol * fabs(hi); ++it) {
            ++n_it;
            // ---- next mu: Illinois regula falsi inside a pole-free bracket, else bisection
            // (the Rayleigh bound lies within ~0.4% above lambda_min on the test units: the first
            // trial 1% of the bracket below it usually lands under the root, a 1% bracket)
            double mu = it == 0 && guess ? lo + 0.99 * (hi - lo) : 0.5 * (lo + hi);
            const int poles = count_below(th, n, hi) - count_below(th, n, lo, true);   // theta_j in (lo, hi)
            const bool secant = slo != 0 && shi != 0 && slo != shi && poles <= 0 &&
                                !(last_secant && (hi - lo) > 0.5 * w_prev);
            if (secant) {
                // |f_lo| / (|f_lo| + |f_hi|), from log2 |det F| in fp32 hardware exp2 (the weight only
                // places mu inside the bracket; the inertia count decides which end moves)
                const float t = __frcp_rn(1.0f + exp2f(fminf(fmaxf((float)(Lhi - Llo), -120.0f), 120.0f)));
                const double m2 = lo + t * (hi - lo);
                if (m2 > lo && m2 < hi) mu = m2;
            }
            last_secant = secant;
            n_sec += secant;
            w_prev = hi - lo;
            // ---- F(mu) = W_R diag(1 / (theta - mu)) W_R^T on the matrix cores
            f64x4 acc[kWlimSlots];
#pragma unroll
            for (int sl = 0; sl < kWlimSlots; ++sl) acc[sl] = f64x4{0.0, 0.0, 0.0, 0.0};
            float nxt[kWlimLoads];
            auto fetch = [&](int j0) {
#pragma unroll
                for (int q = 0; q < kWlimLoads; ++q) {   // branch-free: an in-range load, then a select
                    const bool ok = roff[q] != ~0u && j0 + scol < n;
                    const float x = Wv[ok ? roff[q] + (uint32_t)j0 : 0u];
                    nxt[q] = ok ? x : 0.0f;
                }
            };
            fetch(0);
            for (int j0 = 0; j0 < n; j0 += kWlimKc) {
                __syncthreads();   // the previous chunk is consumed
#pragma unroll
                for (int q = 0; q < kWlimLoads; ++q) {
                    const int r = srow0 + kRowStep * q;
                    if (r < 16 * kWlimTiles) Ws[scol * kWlimLd + r] = (double)nxt[q];
                }
                for (int jj = tid; jj < kWlimKc; jj += kThreads)
                    Ds[jj] = j0 + jj < n ? 1.0 / ((double)th[j0 + jj] - mu) : 0.0;
                // rows c .. 16 nt - 1 of the tiles are zero (staged as 0.0 above: roff = ~0u)
                __syncthreads();
                if (j0 + kWlimKc < n) fetch(j0 + kWlimKc);
                // an offset the compiler cannot see through: the operand addresses below are
                // recomputed per chunk instead of hoisted out of the chunk loop (they were, for
                // every (ks, slot), and spilled)
                int opq = 0;
                asm volatile("" : "+v"(opq));
#pragma unroll
                for (int ks = 0; ks < kWlimKc / 4; ++ks) {
                    const int kk = 4 * ks + (lane >> 4);
                    const double dk = Ds[kk];
                    const double* wrow = Ws + opq + kk * kWlimLd + (lane & 15);
                    int pI = -1;
                    double av = 0.0;
#pragma unroll
                    for (int sl = 0; sl < kWlimSlots; ++sl) {
                        if (sl < nslot) {
                            int I, J;
                            slot_ij(sl, I, J);
                            if (I != pI) {
                                av = wrow[16 * I] * dk;
                                pI = I;
                            }
                            const double bv = wrow[16 * J];
                            acc[sl] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[sl], 0, 0, 0);
                        }
                    }
                }
            }
            __syncthreads();   // every wave is done with the staging area (F aliases it)
#pragma unroll
            for (int sl = 0; sl < kWlimSlots; ++sl) {
                if (sl < nslot) {
                    int I, J;
                    slot_ij(sl, I, J);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int ia = 16 * I + (lane >> 4) + 4 * q, ib = 16 * J + (lane & 15);
                        if (ia < c && ib <= ia) s_F[tri(ia, ib)] = acc[sl][q];
                    }
                }
            }
            __syncthreads();
            // ---- inertia and det of F: right-looking LDL^T, negative pivots counted
            int neg = 0, sgn = 1;
            double ldet = 0.0;
            for (int k = 0; k < c; ++k) {
                const double dk = s_F[tri(k, k)];
                neg += dk < 0.0;
                sgn = dk < 0.0 ? -sgn : (dk == 0.0 ? 0 : sgn);
                if (dk != 0.0) {
                    int ex;   // log2 |dk| = exponent + log2(mantissa): no fp64 log in the loop (its
                    const double mt = frexp(fabs(dk), &ex);   // constants were hoisted and spilled)
                    ldet += (double)ex + (double)__log2f((float)mt);
                    const double rdk = 1.0 / dk;
                    const int m = c - 1 - k;   // trailing rows k+1 .. c-1
                    for (int e = tid; e < m * (m + 1) / 2; e += kThreads) {
                        int ii = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
                        while (ii * (ii + 1) / 2 > e) --ii;
                        while ((ii + 1) * (ii + 2) / 2 <= e) ++ii;
                        const int i = k + 1 + ii, j = k + 1 + (e - ii * (ii + 1) / 2);
                        s_F[tri(i, j)] -= s_F[tri(i, k)] * rdk * s_F[tri(j, k)];
                    }
                }
                __syncthreads();
            }
            if (tid == 0) {
                const bool below = count_below(th, n, mu) - neg >= 1;   // lambda_min(B_hh) < mu
                // Illinois: an end kept twice in a row has its |f| halved
                if (below) {
                    hi = mu;
                    shi = sgn;
                    Lhi = ldet;
                    if (kept == -1 && slo != 0) Llo -= 1.0;   // halve |f| (log2)
                    kept = -1;
                } else {
                    lo = mu;
                    slo = sgn;
                    Llo = ldet;
                    if (kept == 1 && shi != 0) Lhi -= 1.0;
                    kept = 1;
                }
                s_x[0] = lo;
                s_x[1] = hi;
                s_x[2] = Llo;
                s_x[3] = Lhi;
                s_c[0] = slo;
                s_c[1] = shi;
                s_c[2] = kept;
            }
            __syncthreads();
            lo = s_x[0];
            hi = s_x[1];
            Llo = s_x[2];
            Lhi = s_x[3];
            slo = s_c[0];
            shi = s_c[1];
            kept = s_c[2];
            __syncthreads();
        }
        if (tid == 0) {
            a.wlim[p] = (float)sqrt(fmax(0.5 * (lo + hi), 0.0));   // as mode 2 (:435-436)
            a.solved[p] = 1;
            if (a.stats) {
                const int cls = CMAX <= 64 ? 0 : (CMAX <= 128 ? 1 : 2);
                atomicAdd(&a.stats[4 * cls + 0], 1ull);
                atomicAdd(&a.stats[4 * cls + 1], (unsigned long long)n_it);
                atomicAdd(&a.stats[4 * cls + 2], (unsigned long long)n_sec);
                atomicAdd(&a.stats[4 * cls + 3], (unsigned long long)c);
            }
        }
    }
}

// A unit whose local W is symmetric (every w(nb_i -> nb_j) > 0.1 equal to w(nb_j -> nb_i), the
// thresholded values bit for bit; row and column 0 are the movie's own row by construction,
// :326-334) has L2 = D^-1/2 (D - W) D^-1/2 symmetric up to the rounding of its two scalings,
// so B = L2 L2^T = L2^2 to that rounding: B's eigenpairs are (lambda_j^2, v_j) of the mode-1
// eigendecomposition the predictor already has, and mode 3 is not needed for it.  (On the
// knn2 graphs of integer ratings w(a, b) == w(b, a) bitwise; a numpy model of the C2-style
// spill units put the w_lim difference at 2e-8 relative.)  sym[v] starts at 1 for the spill
// units; one workgroup per (unit, row block) clears it on the first asymmetric pair.
__global__ __launch_bounds__(kThreads) void local_sym_kernel(const uint32_t* units, uint32_t n_units,
                                                             const uint64_t* item_off, const uint32_t* items,
                                                             GraphDev graph, uint8_t* sym) {
    constexpr int kRows = 8;
    for (uint32_t w = blockIdx.x; ; w += gridDim.x) {
        // work item w -> (unit, row block): units in order, ceil(n / kRows) blocks each
        uint32_t v = 0, rb = w;
        bool found = false;
        for (uint32_t x = 0; x < n_units; ++x) {
            const uint32_t u = units[x];
            const uint32_t nb = (uint32_t)((item_off[u + 1] - item_off[u] + kRows - 1) / kRows);
            if (rb < nb) {
                v = u;
                found = true;
                break;
            }
            rb -= nb;
        }
        if (!found) return;
        if (!sym[v]) continue;
        const uint64_t base = item_off[v];
        const int n = (int)(item_off[v + 1] - base);
        bool asym = false;
        for (int i = 1 + (int)rb * kRows; i < n && i < 1 + ((int)rb + 1) * kRows; ++i) {
            const uint32_t ai = items[base + i];
            const GraphRow ri = graph.row(ai);
            for (int j = i + 1 + (int)threadIdx.x; j < n; j += kThreads) {
                const uint32_t aj = items[base + j];
                float x = ri[aj], y = graph.row(aj)[ai];
                if (!((double)x > 0.1)) x = 0.0f;
                if (!((double)y > 0.1)) y = 0.0f;
                asym |= __float_as_uint(x) != __float_as_uint(y);
            }
        }
        if (__syncthreads_or(asym) && threadIdx.x == 0) sym[v] = 0;
    }
}

// theta_j = lambda_j^2 of a symmetric unit (its B = L2^2), from the mode-1 eigenvalues (fp32,
// ascending); a unit whose squares are not ascending (a negative lambda_0 of magnitude above
// lambda_1 -- not seen: lambda_0 = 0 to rounding for a connected unit) is handed back to mode 3.
__global__ __launch_bounds__(kThreads) void local_theta_kernel(const uint32_t* units, uint32_t n_units,
                                                               const uint64_t* item_off, const float* evals,
                                                               float* theta, uint8_t* sym) {
    for (uint32_t x = blockIdx.x; x < n_units; x += gridDim.x) {
        const uint32_t v = units[x];
        if (!sym[v]) continue;
        const uint64_t base = item_off[v];
        const int n = (int)(item_off[v + 1] - base);
        bool bad = false;
        for (int i = threadIdx.x; i < n; i += kThreads) {
            const double l = (double)evals[base + i];
            theta[base + i] = (float)(l * l);
            if (i > 0) {
                const double l0 = (double)evals[base + i - 1];
                bad |= (float)(l * l) < (float)(l0 * l0);
            }
        }
        if (__syncthreads_or(bad) && threadIdx.x == 0) sym[v] = 0;
    }
}

}  // namespace

extern "C" int cf_local_calc(cf_ctx* ctx, uint32_t n_movies, const uint64_t* movie_off,
                             const uint32_t* movie_items, const uint64_t* test_off,
                             const uint32_t* test_user, const float* test_rating, float* mse,
                             int32_t* kk, double* pred, float* wlim, int32_t* lim) {
    if (!ctx || (n_movies && (!movie_off || !movie_items)) || !test_off || !mse || !kk)
        return cf_set_error(ctx, CF_EINVAL, "cf_local_calc: null argument");
    if (!has_graph(ctx)) return cf_set_error(ctx, CF_ESTATE, "cf_local_calc: no item graph uploaded");
    CF_TRY(set_device(ctx));
    const uint32_t n_items = ctx->n_items;
    const uint64_t n_test = test_off[n_items];
    if (n_test && (!test_user || !test_rating)) return cf_set_error(ctx, CF_EINVAL, "cf_local_calc: null test arrays");
    // every id the kernels read must lie inside the uploaded graph, and lookup_rating
    // binary-searches each item's test users, so they must be strictly ascending
    if (n_movies && movie_off[0] != 0) return cf_set_error(ctx, CF_EINVAL, "cf_local_calc: movie_off[0] != 0");
    for (uint32_t v = 0; v < n_movies; ++v) {
        if (movie_off[v + 1] < movie_off[v]) return cf_set_error(ctx, CF_EINVAL, "cf_local_calc: movie_off not monotone");
        for (uint64_t i = movie_off[v]; i < movie_off[v + 1]; ++i)
            if (movie_items[i] >= n_items)
                return cf_set_error(ctx, CF_EINVAL, "cf_local_calc: unit " + std::to_string(v) + " names item " +
                                                        std::to_string(movie_items[i]) + " outside the graph");
    }
    if (test_off[0] != 0) return cf_set_error(ctx, CF_EINVAL, "cf_local_calc: test_off[0] != 0");
    for (uint32_t m = 0; m < n_items; ++m) {
        if (test_off[m + 1] < test_off[m]) return cf_set_error(ctx, CF_EINVAL, "cf_local_calc: test_off not monotone");
        for (uint64_t t = test_off[m] + 1; t < test_off[m + 1]; ++t)
            if (test_user[t] <= test_user[t - 1])
                return cf_set_error(ctx, CF_EINVAL, "cf_local_calc: test users of item " + std::to_string(m) +
                                                        " are not strictly ascending");
    }
    // units with n >= 3 and their (movie, test user) pairs (:269-272, :394)
    std::vector<uint64_t> sq_off(n_movies + 1, 0);
    std::vector<uint32_t> pair_movie, pair_user;
    std::vector<uint64_t> pair_out, pair_k;
    for (uint32_t v = 0; v < n_movies; ++v) {
        const uint64_t n = movie_off[v + 1] - movie_off[v];
        // no neighbourhood cap (local_calc.cpp:269-272 builds any unit): units with n >
        // CF_SPILL_MAX_K take the HUGE layout of the spill kernels (cf_eigen_spill.hip), bounded
        // only by HBM (CF_ENOMEM: the n x n blocks below and the solver's 2 n^2 fp64 slot)
        if (n > 0xFFFFFFFFull / 4)
            return cf_set_error(ctx, CF_ERANGE, "cf_local_calc: movie unit " + std::to_string(v) + " too large");
        sq_off[v + 1] = sq_off[v] + n * n;
        if (n < 3) continue;
        const uint32_t m = movie_items[movie_off[v]];
        if (m >= n_items) return cf_set_error(ctx, CF_EINVAL, "cf_local_calc: movie id out of range");
        for (uint64_t t = test_off[m]; t < test_off[m + 1]; ++t) {
            pair_movie.push_back(v);
            pair_user.push_back(test_user[t]);
            pair_out.push_back(t);
            pair_k.push_back(n);
        }
    }
    // pairs of units with n <= CF_MAX_K first (LDS predictor), then the rest (spill predictor)
    {
        std::vector<uint32_t> idx(pair_movie.size());
        for (uint32_t i = 0; i < idx.size(); ++i) idx[i] = i;
        std::stable_partition(idx.begin(), idx.end(), [&](uint32_t i) { return pair_k[i] <= CF_MAX_K; });
        std::vector<uint32_t> pm(idx.size()), pu(idx.size());
        std::vector<uint64_t> po(idx.size()), pk(idx.size());
        for (size_t i = 0; i < idx.size(); ++i) {
            pm[i] = pair_movie[idx[i]];
            pu[i] = pair_user[idx[i]];
            po[i] = pair_out[idx[i]];
            pk[i] = pair_k[idx[i]];
        }
        pair_movie.swap(pm);
        pair_user.swap(pu);
        pair_out.swap(po);
        pair_k.swap(pk);
    }
    const uint32_t n_pairs = (uint32_t)pair_movie.size();
    uint32_t n_small = 0;
    while (n_small < n_pairs && pair_k[n_small] <= CF_MAX_K) ++n_small;
    // movie plan (units with n < 3 are excluded by giving them k = 0)
    std::vector<uint64_t> plan_off(n_movies + 1, 0);
    for (uint32_t v = 0; v < n_movies; ++v) {
        const uint64_t n = movie_off[v + 1] - movie_off[v];
        plan_off[v + 1] = plan_off[v] + (n >= 3 ? n : 0);
    }
    std::vector<uint64_t> pplan_off(n_pairs + 1, 0);
    for (uint32_t p = 0; p < n_pairs; ++p) pplan_off[p + 1] = pplan_off[p] + pair_k[p];
    cf_plan* mplan = nullptr;
    cf_plan* pplan = nullptr;
    CF_TRY(cf_plan_create_cap(ctx, n_movies, plan_off.data(), ~0ull, &mplan));
    int rc = cf_plan_create_cap(ctx, n_pairs, pplan_off.data(), ~0ull, &pplan);
    if (rc != CF_OK) {
        cf_plan_destroy(mplan);
        return rc;
    }
    cf_plan* p3plan = nullptr;   // mode 3's plan: the asymmetric spill units
    auto cleanup = [&]() {
        cf_plan_destroy(mplan);
        cf_plan_destroy(pplan);
        cf_plan_destroy(p3plan);
    };
    const uint64_t n_entries = movie_off[n_movies];
    DevBuf d_moff, d_mitems, d_sqoff, d_evals, d_evecs, d_l2, d_nout, d_toff, d_tuser, d_trat, d_pm, d_pu,
        d_po, d_wlim, d_mse, d_kk, d_pred, d_lim, d_theta, d_bvec, d_solved, d_sym, d_units, d_pairc, d_wstats;
    uint32_t n_sym_units = 0;
    // spill pairs' w_lim by bisection on the movie's B = L2 L2^T (local_wlim_kernel), unless
    // cf_set_local_wlim(ctx, 0) keeps the per-pair tridiagonalisation for every one
    const bool use_bisect = ctx->local_wlim_bisect && n_pairs > n_small;
    bool all_solved = false;
    auto alloc_copy = [&](DevBuf& b, const void* h, size_t bytes) -> int {
        CF_TRY(dev_alloc(ctx, b, bytes));
        if (h && bytes) CF_HIP_CHECK(ctx, hipMemcpy(b.p, h, bytes, hipMemcpyHostToDevice));
        return CF_OK;
    };
    rc = CF_OK;
    do {
        if ((rc = alloc_copy(d_moff, movie_off, sizeof(uint64_t) * (n_movies + 1)))) break;
        if ((rc = alloc_copy(d_mitems, movie_items, sizeof(uint32_t) * n_entries))) break;
        if ((rc = alloc_copy(d_sqoff, sq_off.data(), sizeof(uint64_t) * (n_movies + 1)))) break;
        if ((rc = alloc_copy(d_evals, nullptr, sizeof(float) * n_entries))) break;
        if ((rc = alloc_copy(d_evecs, nullptr, sizeof(float) * sq_off[n_movies]))) break;
        if ((rc = alloc_copy(d_l2, nullptr, sizeof(float) * sq_off[n_movies]))) break;
        if ((rc = alloc_copy(d_nout, nullptr, sizeof(int32_t) * n_movies))) break;
        if ((rc = alloc_copy(d_toff, test_off, sizeof(uint64_t) * (n_items + 1)))) break;
        if ((rc = alloc_copy(d_tuser, test_user, sizeof(uint32_t) * n_test))) break;
        if ((rc = alloc_copy(d_trat, test_rating, sizeof(float) * n_test))) break;
        if ((rc = alloc_copy(d_pm, pair_movie.data(), sizeof(uint32_t) * n_pairs))) break;
        if ((rc = alloc_copy(d_pu, pair_user.data(), sizeof(uint32_t) * n_pairs))) break;
        if ((rc = alloc_copy(d_po, pair_out.data(), sizeof(uint64_t) * n_pairs))) break;
        if ((rc = alloc_copy(d_wlim, nullptr, sizeof(float) * n_pairs))) break;
        if ((rc = alloc_copy(d_mse, mse, sizeof(float) * n_test))) break;
        if ((rc = alloc_copy(d_kk, kk, sizeof(int32_t) * n_test))) break;
        if (pred && (rc = alloc_copy(d_pred, pred, sizeof(double) * n_test))) break;
        if (lim && (rc = alloc_copy(d_lim, lim, sizeof(int32_t) * n_test))) break;
        const auto* moff = static_cast<const uint64_t*>(d_moff.p);
        const auto* mit = static_cast<const uint32_t*>(d_mitems.p);
        const auto* sqo = static_cast<const uint64_t*>(d_sqoff.p);
        if ((rc = cf_launch_local_eigen(ctx, mplan, moff, mit, sqo, static_cast<float*>(d_evals.p),
                                        static_cast<float*>(d_evecs.p), static_cast<float*>(d_l2.p), sqo,
                                        static_cast<int32_t*>(d_nout.p), 0)))
            break;
        if (use_bisect) {
            // the eigenpairs of every large movie's B = L2 L2^T, then one bisection per spill
            // pair; the pairs it leaves (c > kWlimCmax) go to mode 2 below.  Units with a
            // symmetric W take B's eigenpairs from mode 1 (local_sym_kernel); the others run
            // spill eigen mode 3 (CF_LOCAL_SYM=0: every unit on mode 3, for A/B)
            static const bool sym_on = [] {
                const char* e = getenv("CF_LOCAL_SYM");
                return !(e && e[0] == '0');
            }();
            if ((rc = alloc_copy(d_theta, nullptr, sizeof(float) * n_entries))) break;
            if ((rc = alloc_copy(d_solved, nullptr, n_pairs))) break;
            CF_HIP_CHECK(ctx, hipMemset(d_solved.p, 0, n_pairs));
            std::vector<uint32_t> spill_units;
            for (uint32_t v = 0; v < n_movies; ++v)
                if (plan_off[v + 1] - plan_off[v] > (uint64_t)CF_MAX_K) spill_units.push_back(v);
            std::vector<uint8_t> sym(n_movies, 0);
            if ((rc = alloc_copy(d_sym, nullptr, n_movies))) break;
            CF_HIP_CHECK(ctx, hipMemset(d_sym.p, 0, n_movies));
            if (sym_on && !spill_units.empty()) {
                for (uint32_t v : spill_units) sym[v] = 1;
                if ((rc = alloc_copy(d_units, spill_units.data(), sizeof(uint32_t) * spill_units.size()))) break;
                CF_HIP_CHECK(ctx, hipMemcpy(d_sym.p, sym.data(), n_movies, hipMemcpyHostToDevice));
                const uint32_t nu = (uint32_t)spill_units.size();
                const auto* du = static_cast<const uint32_t*>(d_units.p);
                auto* ds = static_cast<uint8_t*>(d_sym.p);
                hipLaunchKernelGGL(local_sym_kernel, dim3(4096), dim3(kThreads), 0, 0, du, nu, moff, mit, graph_dev(ctx), ds);
                hipLaunchKernelGGL(local_theta_kernel, dim3(std::min<uint32_t>(nu, 1024u)), dim3(kThreads), 0, 0, du, nu,
                                   moff, static_cast<const float*>(d_evals.p), static_cast<float*>(d_theta.p), ds);
                if (hipGetLastError() != hipSuccess) {
                    rc = cf_set_error(ctx, CF_EHIP, "local symmetry kernels");
                    break;
                }
                CF_HIP_CHECK(ctx, hipMemcpy(sym.data(), d_sym.p, n_movies, hipMemcpyDeviceToHost));
            }
            // mode 3 over the asymmetric spill units only (symmetric ones get k = 0 in its plan)
            bool any_mode3 = false;
            std::vector<uint64_t> p3_off(n_movies + 1, 0);
            for (uint32_t v = 0; v < n_movies; ++v) {
                const uint64_t n = plan_off[v + 1] - plan_off[v];
                const bool m3 = n > (uint64_t)CF_MAX_K && !sym[v];
                any_mode3 |= m3;
                p3_off[v + 1] = p3_off[v] + (m3 ? n : 0);
            }
            n_sym_units = 0;
            for (uint32_t v : spill_units) n_sym_units += sym[v];
            if (getenv("CF_LOCAL_VERBOSE"))
                fprintf(stderr, "[local] %u of %zu spill units symmetric (mode 3 skipped)\n", n_sym_units,
                        spill_units.size());
            if (any_mode3) {
                if ((rc = alloc_copy(d_bvec, nullptr, sizeof(float) * sq_off[n_movies]))) break;
                if ((rc = cf_plan_create_cap(ctx, n_movies, p3_off.data(), ~0ull, &p3plan))) break;
                for (const cf_bucket& b : p3plan->buckets) {
                    if (b.emax != kSpillBucket || !b.count) continue;
                    cf_spill_local loc{};
                    loc.mode = 3;
                    loc.l2 = static_cast<float*>(d_l2.p);
                    loc.l2_off = sqo;
                    if ((rc = cf_launch_eigen_spill(ctx, p3plan, b, moff, mit, sqo, static_cast<int32_t*>(d_nout.p),
                                                    nullptr, static_cast<float*>(d_theta.p),
                                                    static_cast<float*>(d_bvec.p), 0, &loc)))
                        break;
                }
                if (rc != CF_OK) break;
            }
            WlimArgs wa{};
            wa.n_pairs = n_pairs - n_small;
            wa.pair_movie = static_cast<const uint32_t*>(d_pm.p) + n_small;
            wa.pair_user = static_cast<const uint32_t*>(d_pu.p) + n_small;
            wa.item_off = moff;
            wa.items = mit;
            wa.theta = static_cast<const float*>(d_theta.p);
            wa.w_off = sqo;
            wa.W = static_cast<const float*>(d_bvec.p);
            wa.W_sym = static_cast<const float*>(d_evecs.p);
            wa.sym = static_cast<const uint8_t*>(d_sym.p);
            wa.test_off = static_cast<const uint64_t*>(d_toff.p);
            wa.test_user = static_cast<const uint32_t*>(d_tuser.p);
            wa.test_rating = static_cast<const float*>(d_trat.p);
            wa.wlim = static_cast<float*>(d_wlim.p) + n_small;
            wa.solved = static_cast<uint8_t*>(d_solved.p) + n_small;
            if ((rc = alloc_copy(d_pairc, nullptr, sizeof(int32_t) * std::max<uint32_t>(wa.n_pairs, 1)))) break;
            CF_HIP_CHECK(ctx, hipMemset(d_pairc.p, 0xFF, sizeof(int32_t) * std::max<uint32_t>(wa.n_pairs, 1)));   // -1
            wa.pair_c = static_cast<int32_t*>(d_pairc.p);
            const bool verbose = getenv("CF_LOCAL_VERBOSE") != nullptr;
            if (verbose) {
                if ((rc = alloc_copy(d_wstats, nullptr, 12 * sizeof(unsigned long long)))) break;
                CF_HIP_CHECK(ctx, hipMemset(d_wstats.p, 0, 12 * sizeof(unsigned long long)));
                wa.stats = static_cast<unsigned long long*>(d_wstats.p);
            }
            int cus = 0;
            CF_HIP_CHECK(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
            // the small class first (it counts every pair's c), then the larger ones, which skip
            // the other classes' pairs at once; a grid of a few workgroups per resident slot
            const uint32_t cu = (uint32_t)std::max(1, cus);
            hipLaunchKernelGGL((local_wlim_kernel<64, -1>), dim3(std::min<uint32_t>(wa.n_pairs, cu * 32u)), dim3(kThreads),
                               0, 0, wa);
            hipLaunchKernelGGL((local_wlim_kernel<128, 64>), dim3(std::min<uint32_t>(wa.n_pairs, cu * 8u)),
                               dim3(kThreads), 0, 0, wa);
            hipLaunchKernelGGL((local_wlim_kernel<kWlimCmax, 128>), dim3(std::min<uint32_t>(wa.n_pairs, cu * 4u)),
                               dim3(kThreads), 0, 0, wa);
            if (hipGetLastError() != hipSuccess) {
                rc = cf_set_error(ctx, CF_EHIP, "local_wlim_kernel launch");
                break;
            }
            if (verbose) {
                unsigned long long st[12];
                CF_HIP_CHECK(ctx, hipMemcpy(st, d_wstats.p, sizeof(st), hipMemcpyDeviceToHost));
                for (int cl = 0; cl < 3; ++cl)
                    fprintf(stderr, "[local] w_lim class c <= %d: %llu pairs, %.2f iterations (%.2f secant), mean c %.1f\n",
                            cl == 0 ? 64 : (cl == 1 ? 128 : kWlimCmax), st[4 * cl],
                            st[4 * cl] ? (double)st[4 * cl + 1] / st[4 * cl] : 0.0,
                            st[4 * cl] ? (double)st[4 * cl + 2] / st[4 * cl] : 0.0,
                            st[4 * cl] ? (double)st[4 * cl + 3] / st[4 * cl] : 0.0);
            }
            // the per-pair solver's workspace is sized by the largest unit (2 n^2 fp64 per slot:
            // 1.6 GB at n = 10,000): skip its launch when the bisection solved every spill pair
            std::vector<uint8_t> sv(n_pairs - n_small);
            if (hipMemcpy(sv.data(), static_cast<uint8_t*>(d_solved.p) + n_small, sv.size(), hipMemcpyDeviceToHost) !=
                hipSuccess) {
                rc = cf_set_error(ctx, CF_EHIP, "cf_local_calc: copy solved flags");
                break;
            }
            all_solved = std::all_of(sv.begin(), sv.end(), [](uint8_t f) { return f != 0; });
        }
        if ((rc = cf_launch_local_sigma(ctx, pplan, moff, mit, static_cast<const uint32_t*>(d_pm.p),
                                        static_cast<const uint32_t*>(d_pu.p), static_cast<const float*>(d_l2.p),
                                        sqo, static_cast<const uint64_t*>(d_toff.p),
                                        static_cast<const uint32_t*>(d_tuser.p),
                                        static_cast<const float*>(d_trat.p), static_cast<float*>(d_wlim.p), 0,
                                        use_bisect ? static_cast<const uint8_t*>(d_solved.p) : nullptr,
                                        all_solved)))
            break;
        if (n_pairs > n_small) {
            int nbig = 3;
            for (uint32_t p = n_small; p < n_pairs; ++p) nbig = std::max<int>(nbig, (int)pair_k[p]);
            if ((rc = cf_launch_local_predict_spill(
                     ctx, n_pairs - n_small, nbig, static_cast<const uint32_t*>(d_pm.p) + n_small,
                     static_cast<const uint32_t*>(d_pu.p) + n_small, static_cast<const uint64_t*>(d_po.p) + n_small,
                     moff, mit, static_cast<const float*>(d_evals.p), sqo, static_cast<const float*>(d_evecs.p),
                     static_cast<const float*>(d_wlim.p) + n_small, static_cast<const uint64_t*>(d_toff.p),
                     static_cast<const uint32_t*>(d_tuser.p), static_cast<const float*>(d_trat.p),
                     static_cast<float*>(d_mse.p), static_cast<int32_t*>(d_kk.p),
                     pred ? static_cast<double*>(d_pred.p) : nullptr, lim ? static_cast<int32_t*>(d_lim.p) : nullptr,
                     0)))
                break;
        }
        if (n_small) {
            LocalPredArgs la{};
            la.pair_movie = static_cast<const uint32_t*>(d_pm.p);
            la.pair_user = static_cast<const uint32_t*>(d_pu.p);
            la.pair_out = static_cast<const uint64_t*>(d_po.p);
            la.item_off = moff;
            la.items = mit;
            la.evals = static_cast<const float*>(d_evals.p);
            la.evec_off = sqo;
            la.evecs = static_cast<const float*>(d_evecs.p);
            la.wlim = static_cast<const float*>(d_wlim.p);
            la.test_off = static_cast<const uint64_t*>(d_toff.p);
            la.test_user = static_cast<const uint32_t*>(d_tuser.p);
            la.test_rating = static_cast<const float*>(d_trat.p);
            la.mse = static_cast<float*>(d_mse.p);
            la.kk = static_cast<int32_t*>(d_kk.p);
            la.pred = pred ? static_cast<double*>(d_pred.p) : nullptr;
            la.lim_out = lim ? static_cast<int32_t*>(d_lim.p) : nullptr;
            uint64_t nmax = 3;
            for (uint32_t p = 0; p < n_small; ++p) nmax = std::max(nmax, pair_k[p]);
            la.lmax = (int)nmax;
            const size_t lds = sizeof(double) * ((size_t)(nmax + 2) * (nmax + 3) / 2 + 4) +
                               CF_MAX_K * (sizeof(float) + sizeof(int)) + 8 * sizeof(int);
            if (lds > 163840) {
                rc = cf_set_error(ctx, CF_ERANGE, "local predict exceeds LDS");
                break;
            }
            if (hipFuncSetAttribute((const void*)local_predict_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds) != hipSuccess) {
                rc = cf_set_error(ctx, CF_EHIP, "local predict LDS attribute");
                break;
            }
            const uint32_t blocks = std::min<uint32_t>(n_small, 65536u);   // ~one pair each: dispatcher-balanced
            hipLaunchKernelGGL(local_predict_kernel, dim3(blocks), dim3(kThreads), lds, 0, la, n_small);
            if (hipGetLastError() != hipSuccess) {
                rc = cf_set_error(ctx, CF_EHIP, "local_predict_kernel launch");
                break;
            }
        }
        if (hipDeviceSynchronize() != hipSuccess) {
            rc = cf_set_error(ctx, CF_EHIP, "cf_local_calc: device synchronize");
            break;
        }
        if (hipMemcpy(mse, d_mse.p, sizeof(float) * n_test, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(kk, d_kk.p, sizeof(int32_t) * n_test, hipMemcpyDeviceToHost) != hipSuccess ||
            (pred && hipMemcpy(pred, d_pred.p, sizeof(double) * n_test, hipMemcpyDeviceToHost) != hipSuccess) ||
            (lim && hipMemcpy(lim, d_lim.p, sizeof(int32_t) * n_test, hipMemcpyDeviceToHost) != hipSuccess)) {
            rc = cf_set_error(ctx, CF_EHIP, "cf_local_calc: copy out");
            break;
        }
        if (wlim) {
            std::vector<float> w(n_pairs);
            if (n_pairs && hipMemcpy(w.data(), d_wlim.p, sizeof(float) * n_pairs, hipMemcpyDeviceToHost) != hipSuccess) {
                rc = cf_set_error(ctx, CF_EHIP, "cf_local_calc: copy w_lim");
                break;
            }
            for (uint32_t p = 0; p < n_pairs; ++p) wlim[pair_out[p]] = w[p];
        }
    } while (false);
    cleanup();
    // the spill workspaces of a large call (HUGE units: up to half the free HBM) are released
    // here rather than held by the context for the next call (synchronous call: nothing reads
    // them any more)
    if (hipDeviceSynchronize() == hipSuccess) {
        if (ctx->d_spill) (void)hipFree(ctx->d_spill);
        ctx->d_spill = nullptr;
        ctx->spill_bytes = 0;
        if (ctx->d_pspill) (void)hipFree(ctx->d_pspill);
        ctx->d_pspill = nullptr;
        ctx->pspill_bytes = 0;
    }
    return rc;
}
