// cf_eigen_spill.hip -- compute_eigens for users with CF_MAX_K < k <= CF_SPILL_MAX_K.
//
// The LDS Jacobi kernel (cf_eigen.hip) keeps a user's k x k matrix in LDS, which holds
// k <= 192 in fp32.  Power-law degree mixes (BASELINE config 5: p95 k ~ 1.5k) need
// k x k matrices of up to 72 MB in fp64, so this path works on an HBM-resident
// workspace, one 512-thread workgroup per user (persistent over the spill users, an
// atomic counter hands them out largest-k first):
//
//   1. gather W_u from the dense graph into the user's own output slot (fp32 k x k),
//      d_i (fp64) with the 0 -> 1 rule (precompute_local_threads.cpp:129-141),
//      s_i = sqrt(1/d_i) (:149-153), L2(i,j) = (s_i L(i,j)) s_j (:155) in fp64 -- bit
//      identical to the oracle's L2 -- sig_min_i from the full row (:169-177), and
//      A = sym_lower(L2) (:164, Eigen reads the lower triangle) as a full symmetric
//      fp64 matrix, column-major, in the workspace;
//   2. blocked Householder tridiagonalisation (LAPACK dsytrd/dlatrd, lower): panels of
//      SP_NB = 32 reflectors, each panel's W built with symmetric matrix-vector products
//      against the not-yet-updated trailing matrix, then one rank-2*SP_NB update of the
//      trailing matrix (A -= V W^T + W V^T) with SP_CC columns staged per step;
//   3. implicit-shift QL (tql2, oracle tridiag_ql) on Z = I: a generator wave runs the
//      serial recurrence and publishes each iteration's rotation sequence (coefficients
//      broadcast with v_readlane) while seven applier waves apply the previous batch of
//      SP_QB = 16 iterations to Z in one lagged, branch-free pass (identity-padded
//      sequences), one read + one write per element per batch;
//   4a. eigenvectors of A = Q Z: the Householder panels applied to Z last to first in
//      compact-WY form (I - V T V^T, SP_RC rows of V staged per step);
//   4b. rank sort, sign convention sum_i v_ij >= 0 (as cf_eigen.hip), lim (:184-191),
//      and the k x m row-major block, sigs, evals, m -- the same record as the LDS path.
//
// Everything is fp64: the matrices are too large for the fp32 Jacobi tolerance argument
// of the LDS path, and the FP64 vector rate of MI355X equals its unpacked FP32 rate.
// Cost: tridiagonalisation 4k^3/3 flops (half in matrix-vector products), QL
// ~ (#rotations) x 6k flops over one Z pass per 16 iterations, back-transform 2k^3; see
// DESIGN.md 3.6.

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cf_internal.h"

namespace {

constexpr int SP_T = 512;
constexpr int SP_W = SP_T / 64;
constexpr int SP_QB = 16;                        // QL iterations applied per pass over Z
constexpr int SP_NB = 32;                        // Householder panel width (dlatrd block)
constexpr int SP_CC = 32;                        // columns staged per trailing-update step
constexpr int SP_RC = 64;                        // rows of V staged per back-transform step

struct SpillArgs {
    const uint32_t* order;
    uint32_t first;
    uint32_t count;
    const uint64_t* item_off;
    const uint32_t* items;
    GraphDev graph;
    uint64_t n_items;
    const uint64_t* evec_off;
    int32_t* m_out;
    float* sigs;
    float* evals;
    float* evecs;
    double* work;
    uint64_t work_stride;    // doubles per workgroup slot (>= kmax^2)
    uint64_t big_off;        // BIG launches: rc, rs, tau (kmax doubles each) at this slot offset
    unsigned int* counter;   // next spill user (zeroed before the launch)
    unsigned long long* phase;   // 8 counters (cf_debug_spill), summed by thread 0
    cf_spill_local loc;      // a8 modes (loc.mode = 0: compute_eigens of a user)
    // staged multi-CU path (BIG users of compute_eigens, see spill_mc_*): 0 = the whole user
    // here; 1 = assembly only, sig to the slot; 2 = QL on a block of Z's rows (d, e from the
    // slot after the multi-CU tridiagonalisation; part 0 stores the eigenvalues); 3 = Z to
    // row-major; 4 = back-transform and output of a block of Z's columns.  In stages >= 1 the
    // slot is the user's, not the workgroup's, and a claim is (user, part), mc_parts parts
    // per user.
    int mc_stage;
    int mc_parts;        // parts of each of the first mc_n2 users of the launch
    int mc_parts_rest;   // parts of each of the others
    int mc_n2;
    uint64_t vs;   // BIG / HUGE: stride of the slot's k-long vectors (McLayout), >= the launch's kmax
    const uint64_t* slot_off;   // staged stages: per unit of the wave, its slot's offset in `work`
    int de_lds;    // HUGE: QL's d / e in the dynamic LDS tail (else in the slot's per-part pair)
};

// Staged slots: after rc / rs / tau (big_off + 3 vs, vs = the launch's vector stride >= its
// largest k) the tridiagonal d, e, the sigs, the eigenvalues (QL's d), the panel's dot products
// xv, xw, then one QL coefficient buffer per row part (each part runs its own generator).  HUGE
// launches (k > CF_SPILL_MAX_K, whose per-row vectors no longer fit in LDS) add a private
// (d, e) pair per QL part, for parts whose d / e do not fit in LDS either, and the rank / row
// list `perm`.
constexpr int MC_QL_ROWS = 2 * (SP_T - 64);        // rows of one QL part, at least: one applier pass
constexpr int MC_BT_COLS = SP_T;                   // columns of one back-transform part, at least
struct McLayout {
    uint64_t vs, d, e, sig, df, xv, xw, gbuf, gsz, parts_max, pde, perm, extra_big, extra_huge;
    __host__ __device__ explicit McLayout(uint64_t v) : vs(v) {
        d = 3 * v;
        e = 4 * v;
        sig = 5 * v;
        df = 6 * v;
        xv = 7 * v;
        xw = 7 * v + 32;
        gbuf = 7 * v + 64;
        gsz = 4ull * SP_QB * (v + 2 * SP_QB + 4);   // doubles per coefficient buffer pair
        parts_max = (v + MC_QL_ROWS - 1) / MC_QL_ROWS;
        pde = gbuf + parts_max * gsz;
        perm = pde + 2 * parts_max * v;
        extra_big = pde;
        extra_huge = perm + v;
    }
};
// Slot of a staged unit of k rows: the k x k matrix, Z, the panel W, the QL coefficient buffers
// of stage 0, then (at this offset) the McLayout vectors.
__host__ __device__ constexpr uint64_t spill_base_stride(uint64_t k) {
    return 2ull * k * k + (uint64_t)SP_NB * k + 4ull * SP_QB * (k + 2 * SP_QB + 4) + 64;
}
// the symv's transposed partials z_k (one per row-block pair: <= ceil(vs / 64) rows of vs) share
// the QL buffers' space (gbuf): the tridiagonalisation is over before QL starts.  ceil(v/64) v <=
// ceil(v/896) 64 (v + 36) for every v >= 1, so they fit.

// LDS of one workgroup.  NL = the largest k of the launch's layout.  Up to SP_NL (3072) the
// per-row vectors rc / rs / tau live in LDS too; a BIG launch (SP_NL < k <= CF_SPILL_MAX_K)
// keeps d / e (the QL recurrence's operands) and sig / perm in LDS and moves rc / rs / tau to
// the user's HBM slot, with the 32-column staging tiles (which alias rc in the LDS layout) in
// a dedicated region.
constexpr int SP_NL = 3072;
constexpr int SP_STAGE = 2 * 32 * 33;             // the largest staging use: two 32 x 33 tiles
template <int NL, bool BIG>
struct SpillSmemT {
    double d[NL];
    double e[NL];
    double rc[BIG ? 1 : NL];
    double rs[BIG ? 1 : NL];
    double tau[BIG ? 1 : NL];
    double stage[BIG ? SP_STAGE : 1];
    double vj[SP_NB], wj[SP_NB], xv[SP_NB], xw[SP_NB];
    double part[8 * 64];
    float sig[NL];
    int perm[NL];
    double red[SP_W + 4];
    int flag[4];
};
static_assert(sizeof(SpillSmemT<SP_NL, false>) <= 163840, "spill LDS");
static_assert(sizeof(SpillSmemT<CF_SPILL_MAX_K, true>) <= 163840, "big spill LDS");

// LDS of a HUGE launch (k > CF_SPILL_MAX_K): every k-long vector lives in the user's slot,
// except QL's d / e, which take the dynamic tail of the workgroup's LDS when 16 k bytes fit
// beside the header (k <= ~10,100; the generator's serial chain reads them): then they overlay
// the staging tiles, which QL does not use.
struct SpillSmemHugeHdr {
    double vj[SP_NB], wj[SP_NB], xv[SP_NB], xw[SP_NB];
    double red[SP_W + 4];
    int seq[4 * SP_QB + 8];   // the generator's sequence ranges and flags (BIG: in perm)
    int flag[4];
};
struct SpillSmemHugeWork {
    double stage[SP_STAGE];
    double vsb[SP_RC * (SP_NB + 1)];   // back-transform V rows (BIG: in e)
    double part[8 * 64];
};
constexpr size_t kHugeHdr = (sizeof(SpillSmemHugeHdr) + 15) & ~(size_t)15;
constexpr size_t kLdsMax = 163840;
// dynamic LDS of a HUGE launch of largest k with d / e in LDS (de_lds) or not
inline size_t huge_lds_bytes(uint64_t kmax, bool de_lds) {
    return kHugeHdr + std::max<size_t>(sizeof(SpillSmemHugeWork), de_lds ? 16 * kmax : 0);
}
// largest k whose d / e fit in a HUGE launch's LDS
constexpr uint64_t kHugeDeLdsMax = (kLdsMax - kHugeHdr) / 16;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Lane l's double as a wave-uniform value (two v_readlane_b32 into SGPRs).
__device__ __forceinline__ double bcast_lane(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Sum over the workgroup, returned to every thread (two barriers).
__device__ __forceinline__ double block_sum(double v, double* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wave_sum(v);
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < SP_W; ++w) t += red[w];
    __syncthreads();
    return t;
}

template <int NL, bool BIG, bool HUGE = false>
__global__ __launch_bounds__(SP_T) void eigen_spill_kernel(SpillArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    // LDS views: SpillSmemT, or (HUGE) the header + the staging work area / the d-e tail
    using SmT = SpillSmemT<(HUGE ? 1 : NL), (BIG || HUGE)>;
    SmT& S = *reinterpret_cast<SmT*>(smem_raw);
    SpillSmemHugeHdr& H = *reinterpret_cast<SpillSmemHugeHdr*>(smem_raw);
    SpillSmemHugeWork& HW = *reinterpret_cast<SpillSmemHugeWork*>(smem_raw + kHugeHdr);
    double* const de_tail = reinterpret_cast<double*>(smem_raw + kHugeHdr);
    int* const s_flag = HUGE ? H.flag : S.flag;
    double* const s_red = HUGE ? H.red : S.red;
    double* const s_vj = HUGE ? H.vj : S.vj;
    double* const s_wj = HUGE ? H.wj : S.wj;
    double* const s_xv = HUGE ? H.xv : S.xv;
    double* const s_xw = HUGE ? H.xw : S.xw;
    double* const s_part = HUGE ? HW.part : S.part;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const McLayout Lo(a.vs);
    constexpr bool SLOTV = BIG || HUGE;   // rc / rs / tau in the slot
    double* M = a.mc_stage ? nullptr : a.work + (size_t)blockIdx.x * a.work_stride;
    uint64_t bo = a.big_off;   // offset of the McLayout vectors in the slot
    // per-row vectors and the staging tiles (see SpillSmemT)
    double* rc = SLOTV && M ? M + bo : S.rc;
    double* rs = SLOTV && M ? M + bo + Lo.vs : S.rs;
    double* tau = SLOTV && M ? M + bo + 2 * Lo.vs : S.tau;
    double* const stage = HUGE ? HW.stage : (BIG ? S.stage : S.rc);
    // QL's d / e, the rank / row list, the sigs: LDS (SpillSmemT) or the slot (HUGE, set per unit)
    double* Sd = S.d;
    double* Se = S.e;
    int* Sperm = S.perm;
    const double eps = 2.220446049250313e-16;   // 2^-52 (tql2)

    for (;;) {
        if (tid == 0) s_flag[0] = (int)atomicAdd(a.counter, 1u);
        __syncthreads();
        const int idx = s_flag[0];
        __syncthreads();
        const int st = a.mc_stage;
        // claims: the first n2 users in P0 parts each, the rest in P1 (stage 2 gives the largest
        // users of a batch smaller than the CU count one part more)
        const int P0 = st ? a.mc_parts : 1, P1 = st ? a.mc_parts_rest : 1, n2 = st ? a.mc_n2 : 0;
        if (idx >= n2 * P0 + ((int)a.count - n2) * P1) break;   // uniform: every wave leaves together
        int ui, part, P;
        if (idx < n2 * P0) {
            ui = idx / P0;
            part = idx - ui * P0;
            P = P0;
        } else {
            const int j = idx - n2 * P0;
            ui = n2 + j / P1;
            part = j - (j / P1) * P1;
            P = P1;
        }
        const int mode = a.loc.mode;
        const uint32_t unit = a.order[a.first + ui];
        const uint32_t u = mode == 2 ? a.loc.pair_movie[unit] : unit;   // the unit whose items index the graph
        if (mode == 2 && a.loc.solved && a.loc.solved[unit]) continue;   // w_lim by bisection already
        const uint64_t base = a.item_off[u];
        const int nrows = (int)(a.item_off[u + 1] - base);
        int n = nrows;
        if (st) {   // staged: the unit's own slot (sized for its k when slot_off is given)
            M = a.work + (a.slot_off ? a.slot_off[ui] : (uint64_t)ui * a.work_stride);
            bo = a.slot_off ? spill_base_stride((uint64_t)nrows) : a.big_off;
            if (SLOTV) {
                rc = M + bo;
                rs = M + bo + Lo.vs;
                tau = M + bo + 2 * Lo.vs;
            }
        }
        if constexpr (HUGE) {
            // the per-row vectors of this unit: QL parts take their own (d, e) copy, in the LDS
            // tail when it fits (de_lds) or in the part's pair of the slot; the back-transform
            // reads the eigenvalues where part 0 of QL left them; stage 0 (one workgroup per
            // unit) uses the slot's d / e
            double* mc = M + bo;
            Sperm = reinterpret_cast<int*>(mc + Lo.perm);
            if (st == 2) {
                Sd = a.de_lds ? de_tail : mc + Lo.pde + 2 * (uint64_t)part * Lo.vs;
                Se = Sd + Lo.vs;
            } else if (st == 4) {
                Sd = mc + Lo.df;
            } else {
                Sd = mc + Lo.d;
                Se = mc + Lo.e;
            }
        }
        if (mode == 2) {
            // w_lim pass (local_calc.cpp:402-436): the unrated rows h of the movie's L2 (row 0,
            // the movie itself, counts as unrated, :405-413), in row order, into Sperm
            const uint32_t user = a.loc.pair_user[unit];
            int h = 0;
            for (int b0 = 0; b0 < nrows; b0 += SP_T) {
                const int i = b0 + tid;
                bool unr = false;
                if (i < nrows) {
                    if (i == 0) {
                        unr = true;
                    } else {
                        const uint32_t mv = a.items[base + i];
                        uint64_t lo = a.loc.test_off[mv];
                        const uint64_t end = a.loc.test_off[mv + 1];
                        uint64_t hi = end;
                        while (lo < hi) {
                            const uint64_t mid = (lo + hi) >> 1;
                            if (a.loc.test_user[mid] < user) lo = mid + 1;
                            else hi = mid;
                        }
                        unr = !(lo < end && a.loc.test_user[lo] == user) || a.loc.test_rating[lo] == 0.0f;
                    }
                }
                const unsigned long long bal = __ballot(unr);
                if (lane == 0) s_red[wave] = (double)__popcll(bal);
                __syncthreads();
                int off = h, all = 0;
                for (int w = 0; w < SP_W; ++w) {
                    const int cw = (int)s_red[w];
                    if (w < wave) off += cw;
                    all += cw;
                }
                if (unr) Sperm[off + __popcll(bal & ((1ull << lane) - 1ull))] = i;
                h += all;
                __syncthreads();
            }
            n = h;
        }
        float* Wt = mode == 2 ? nullptr : a.evecs + a.evec_off[u];   // k x k scratch until the output is written
        auto Mat = [&](int r, int c) -> double& { return M[(size_t)c * n + r]; };
        double* Zb = M + (size_t)n * n;          // tridiagonal eigenvectors Z (column-major, then rows)
        double* Wp = Zb + (size_t)n * n;         // [SP_NB][n] panel W of the tridiagonalisation
        unsigned long long t0 = tid == 0 ? __builtin_amdgcn_s_memtime() : 0ull, t1 = 0, t2 = 0, t3 = 0, tgen = 0;
        unsigned long long n_iter = 0, n_rot = 0;
        // the sigs of the rows: LDS, or the slot (HUGE)
        auto sig_set = [&](int i, float v) {
            if constexpr (HUGE) M[bo + Lo.sig + i] = (double)v;
            else S.sig[i] = v;
        };
        auto sig_get = [&](int i) -> float {
            if constexpr (HUGE) return (float)M[bo + Lo.sig + i];
            else return S.sig[i];
        };

        if (st >= 2) {
            // resume: d, e from the slot (the multi-CU tridiagonalisation left them there) for
            // QL, the eigenvalues and sigs for the output
            const double* mc = M + bo;
            if constexpr (HUGE) {
                if (st == 2)   // this part's own copy (the generator updates it)
                    for (int i = tid; i < n; i += SP_T) {
                        Sd[i] = mc[Lo.d + i];
                        Se[i] = mc[Lo.e + i];
                    }
            } else {
                for (int i = tid; i < n; i += SP_T) {
                    Sd[i] = mc[(st == 4 ? Lo.df : Lo.d) + i];
                    Se[i] = mc[Lo.e + i];
                    S.sig[i] = (float)mc[Lo.sig + i];
                }
            }
            __syncthreads();
        } else if (mode == 2 || mode == 3) {
            // ---- 1s. A = L2_h L2_h^T (h x h, fp64 sums of the stored fp32 L2 rows, :425-435);
            // mode 3: every row, B = L2 L2^T of the movie, whose eigenpairs the bisection of
            // local_wlim_kernel (cf_local.hip) shares across the movie's pairs
            const float* L2m = a.loc.l2 + a.loc.l2_off[u];
            const int npk = n * (n + 1) / 2;
            for (int e = wave; e < npk; e += SP_W) {
                int p = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
                while (p * (p + 1) / 2 > e) --p;
                while ((p + 1) * (p + 2) / 2 <= e) ++p;
                const int q = e - p * (p + 1) / 2;
                const float* rp = L2m + (size_t)(mode == 3 ? p : Sperm[p]) * nrows;
                const float* rq = L2m + (size_t)(mode == 3 ? q : Sperm[q]) * nrows;
                double acc = 0.0;
                for (int j = lane; j < nrows; j += 64) acc = fma((double)rp[j], (double)rq[j], acc);
                acc = wave_sum(acc);
                if (lane == 0) {
                    Mat(p, q) = acc;
                    Mat(q, p) = acc;
                }
            }
            __syncthreads();
        } else {
        // ---- 1. W_u, degrees, s, L2, sig_min, A = sym_lower(L2) ------------------------
        // mode 1 (local graph, local_calc.cpp:326-360): W(i, j) = w(item_i -> item_j) if
        // > 0.1, column 0 mirrors row 0 (W(i, 0) = w(movie -> item_i), W(0, 0) = 0), and no
        // 0 -> 1 degree rule.
        for (int i = wave; i < n; i += SP_W) {
            const GraphRow grow = a.graph.row(a.items[base + i]);
            const GraphRow grow0 = a.graph.row(a.items[base]);
            double ds = 0.0;
            for (int j = lane; j < n; j += 64) {
                float w = grow[a.items[base + j]];
                if (mode == 1) {
                    if (j == 0) w = (i == 0) ? 0.0f : grow0[a.items[base + i]];
                    if (!((double)w > 0.1)) w = 0.0f;
                }
                Wt[(size_t)i * n + j] = w;
                ds += (double)w;
            }
            ds = wave_sum(ds);
            if (lane == 0) rs[i] = (ds == 0.0 && mode == 0) ? 1.0 : ds;   // (:137-140)
        }
        __syncthreads();
        for (int i = tid; i < n; i += SP_T) rc[i] = sqrt(1.0 / rs[i]);   // (:149-153)
        __syncthreads();
        float* L2out = mode == 1 ? a.loc.l2 + a.loc.l2_off[u] : nullptr;
        for (int i = wave; i < n; i += SP_W) {
            const double si = rc[i], di = rs[i];
            double sq = 0.0;
            for (int j = lane; j < n; j += 64) {
                const double l = (j == i ? di : 0.0) - (double)Wt[(size_t)i * n + j];
                const double l2 = (si * l) * rc[j];   // (:155)
                sq += l2 * l2;
                if (L2out) L2out[(size_t)i * n + j] = (float)l2;   // unsymmetrised, for the w_lim pass
                if (j <= i) {
                    Mat(i, j) = l2;
                    Mat(j, i) = l2;
                }
            }
            sq = wave_sum(sq);
            if (lane == 0) sig_set(i, sqrtf((float)sq));   // (:172-176)
        }
        __syncthreads();
        }   // mode != 2

        if (a.mc_stage == 1) {   // assembly only: sig to the slot, the next user
            if constexpr (!HUGE)   // (HUGE: written there already)
                for (int i = tid; i < n; i += SP_T) M[bo + Lo.sig + i] = (double)S.sig[i];
            __syncthreads();
            continue;
        }
        if (tid == 0) t1 = __builtin_amdgcn_s_memtime();
        // ---- 2. blocked Householder tridiagonalisation (LAPACK dsytrd/dlatrd, lower) ---------
        // Panels of SP_NB columns.  Inside a panel, column j is brought up to date with the
        // panel's earlier reflectors (A -= V W^T + W V^T restricted to column j), its
        // reflector H_j = I - tau_j v v^T (v[j+1] = 1) annihilates A(j+2:n, j), and
        //   w = tau (A v - V (W^T v) - W (V^T v)),  w += -tau/2 (w.v) v
        // uses the trailing matrix as of the panel start.  After the panel one rank-2*SP_NB
        // update A -= V W^T + W V^T refreshes the trailing square.  The symmetric
        // matrix-vector product is the only per-column pass over the trailing matrix, so the
        // workspace traffic is ~8 B per element-step instead of tred2's ~24 B.
        // v_j is stored in M(j+1:n, j); A = Q T Q^T with Q = H_0 H_1 ... H_{n-2},
        // T = tridiag(d, e) with e[j] = T(j+1, j).
        for (int p = 0; p < (st >= 2 ? 0 : n - 1); p += SP_NB) {   // stages >= 2: done by spill_mc_*
            const int jb = min(SP_NB, n - 1 - p);
            for (int jj = 0; jj < jb; ++jj) {
                const int j = p + jj;
                double* colj = M + (size_t)j * n;
                if (jj > 0) {
                    if (tid < jj) {
                        s_vj[tid] = M[(size_t)(p + tid) * n + j];
                        s_wj[tid] = Wp[(size_t)tid * n + j];
                    }
                    __syncthreads();
                    for (int r = j + tid; r < n; r += SP_T) {
                        double acc = colj[r];
                        for (int t = 0; t < jj; ++t)
                            acc -= M[(size_t)(p + t) * n + r] * s_wj[t] + Wp[(size_t)t * n + r] * s_vj[t];
                        colj[r] = acc;
                    }
                    __syncthreads();
                }
                // reflector of x = A(j+1:n, j) (dlarfg without the rescaling loop)
                const double alpha = colj[j + 1];
                const double ajj = colj[j];
                double part = 0.0;
                for (int r = j + 2 + tid; r < n; r += SP_T) {
                    const double x = colj[r];
                    part += x * x;
                }
                const double sigma = block_sum(part, s_red);   // barriers: alpha read before v is stored
                double tj = 0.0, beta = alpha, scal = 0.0;
                if (sigma != 0.0) {
                    beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
                    tj = (beta - alpha) / beta;
                    scal = 1.0 / (alpha - beta);
                }
                if (tid == 0) {
                    Sd[j] = ajj;
                    Se[j] = beta;
                    tau[j] = tj;
                }
                for (int r = j + 1 + tid; r < n; r += SP_T) {
                    const double vr = (r == j + 1) ? 1.0 : colj[r] * scal;
                    rc[r] = vr;
                    colj[r] = vr;
                }
                __syncthreads();
                const int r0 = j + 1;
                if (tj == 0.0) {   // H_j = I: w = 0
                    for (int r = tid; r < n; r += SP_T) Wp[(size_t)jj * n + r] = 0.0;
                    __syncthreads();
                    continue;
                }
                // x_v[t] = W(:,t).v and x_w[t] = V(:,t).v over rows r0..n-1, one wave per dot
                for (int q = wave; q < 2 * jj; q += SP_W) {
                    const int t = q >> 1;
                    const double* src = (q & 1) ? M + (size_t)(p + t) * n : Wp + (size_t)t * n;
                    double s = 0.0;
                    for (int r = r0 + lane; r < n; r += 64) s += src[r] * rc[r];
                    s = wave_sum(s);
                    if (lane == 0) {
                        if (q & 1)
                            s_xw[t] = s;
                        else
                            s_xv[t] = s;
                    }
                }
                // y = A(r0:n, r0:n) v: a wave per (64-row block, column segment), lane per row
                // (column-major reads coalesce); segments split the columns when there are
                // fewer row blocks than waves, partial sums combined in LDS in a fixed order.
                const int rows = n - r0;
                const int nrb = (rows + 63) >> 6;
                const int segs = nrb >= SP_W ? 1 : SP_W / nrb;
                const int seglen = (rows + segs - 1) / segs;
                for (int unit = wave; unit < nrb * segs; unit += SP_W) {
                    const int rb = unit % nrb, sg = unit / nrb;
                    const int r = r0 + rb * 64 + lane;
                    const int c_lo = r0 + sg * seglen, c_hi = min(n, c_lo + seglen);
                    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
                    if (r < n) {
                        const double* mr = M + r;
                        int c = c_lo;
                        // 16 column loads in flight per lane: the pass is bound by memory
                        // latency x bytes in flight as much as by HBM bandwidth
                        for (; c + 16 <= c_hi; c += 16) {
                            double x[16];
#pragma unroll
                            for (int t = 0; t < 16; ++t) x[t] = mr[(size_t)(c + t) * n];
#pragma unroll
                            for (int t = 0; t < 16; t += 4) {
                                p0 += x[t] * rc[c + t];
                                p1 += x[t + 1] * rc[c + t + 1];
                                p2 += x[t + 2] * rc[c + t + 2];
                                p3 += x[t + 3] * rc[c + t + 3];
                            }
                        }
                        for (; c < c_hi; ++c) p0 += mr[(size_t)c * n] * rc[c];
                    }
                    const double ps = (p0 + p1) + (p2 + p3);
                    if (segs == 1) {
                        if (r < n) rs[r] = ps;
                    } else {
                        s_part[sg * (nrb * 64) + rb * 64 + lane] = ps;
                    }
                }
                __syncthreads();
                double yv = 0.0;
                for (int r = r0 + tid; r < n; r += SP_T) {
                    double y;
                    if (segs == 1) {
                        y = rs[r];
                    } else {
                        y = 0.0;
                        for (int sg = 0; sg < segs; ++sg) y += s_part[sg * (nrb * 64) + (r - r0)];
                    }
                    for (int t = 0; t < jj; ++t)
                        y -= M[(size_t)(p + t) * n + r] * s_xv[t] + Wp[(size_t)t * n + r] * s_xw[t];
                    y *= tj;
                    rs[r] = y;
                    yv += y * rc[r];
                }
                const double a2 = -0.5 * tj * block_sum(yv, s_red);
                for (int r = tid; r < n; r += SP_T) Wp[(size_t)jj * n + r] = r >= r0 ? rs[r] + a2 * rc[r] : 0.0;
                __syncthreads();
            }
            // trailing update A(q:n, q:n) -= V W^T + W V^T (q = p + jb), full square so the
            // next panels' column-major symv stays coalesced.  Lane per row with that row's
            // V and W entries in registers; each column's V and W entries are broadcast from
            // LDS (SP_CC columns staged at a time).
            const int q = p + jb;
            const int mq = n - q;
            if (mq > 0) {
                const int nrb = (mq + 63) >> 6;
                double* stg = stage;   // [SP_CC][2 * SP_NB]: V(c, t) then W(c, t)
                for (int pass = 0; pass < nrb; pass += SP_W) {
                    const int rb = pass + wave;
                    const int r = q + rb * 64 + lane;
                    const bool act = rb < nrb && r < n;
                    double vr[SP_NB], wr[SP_NB];
#pragma unroll
                    for (int t = 0; t < SP_NB; ++t) {
                        vr[t] = (act && t < jb) ? M[(size_t)(p + t) * n + r] : 0.0;
                        wr[t] = (act && t < jb) ? Wp[(size_t)t * n + r] : 0.0;
                    }
                    for (int c0 = q; c0 < n; c0 += SP_CC) {
                        const int cn = min(SP_CC, n - c0);
                        __syncthreads();
                        for (int idx = tid; idx < SP_CC * 2 * SP_NB; idx += SP_T) {
                            const int cc = idx / (2 * SP_NB), t2 = idx - cc * (2 * SP_NB);
                            const int t = t2 & (SP_NB - 1);
                            double v = 0.0;
                            if (cc < cn && t < jb)
                                v = t2 < SP_NB ? M[(size_t)(p + t) * n + c0 + cc] : Wp[(size_t)t * n + c0 + cc];
                            stg[idx] = v;
                        }
                        __syncthreads();
                        if (!act) continue;
                        // software-pipelined: the next 8 columns' loads are in flight while
                        // the current 8 are updated; sched_barrier keeps the scheduler from
                        // hoisting every column's 64 LDS operands at once (VGPR spills)
                        double* mp = M + (size_t)c0 * n + r;
                        double cur[8];
#pragma unroll
                        for (int u8 = 0; u8 < 8; ++u8) cur[u8] = u8 < cn ? mp[(size_t)u8 * n] : 0.0;
                        for (int cc = 0; cc < cn; cc += 8) {
                            double nxt[8];
#pragma unroll
                            for (int u8 = 0; u8 < 8; ++u8)
                                nxt[u8] = cc + 8 + u8 < cn ? mp[(size_t)(cc + 8 + u8) * n] : 0.0;
#pragma unroll
                            for (int u8 = 0; u8 < 8; ++u8) {
                                __builtin_amdgcn_sched_barrier(0);
                                const double* sv = stg + (cc + u8) * 2 * SP_NB;
                                double acc0 = cur[u8], acc1 = 0.0;
#pragma unroll
                                for (int t = 0; t < SP_NB; t += 2) {
                                    if ((t & 7) == 0) __builtin_amdgcn_sched_barrier(0);
                                    acc0 -= vr[t] * sv[SP_NB + t] + wr[t] * sv[t];
                                    acc1 -= vr[t + 1] * sv[SP_NB + t + 1] + wr[t + 1] * sv[t + 1];
                                }
                                if (cc + u8 < cn) mp[(size_t)(cc + u8) * n] = acc0 + acc1;
                            }
#pragma unroll
                            for (int u8 = 0; u8 < 8; ++u8) cur[u8] = nxt[u8];
                        }
                    }
                }
                __syncthreads();
            }
        }
        if (tid == 0 && st < 2) {
            Sd[n - 1] = M[(size_t)(n - 1) * n + (n - 1)];
            Se[n - 1] = 0.0;
        }
        if (mode == 2) {
            // w_lim = sqrt(lambda_min(L2_h L2_h^T)) (:435-436): the smallest eigenvalue of
            // tridiag(d, e) by Sturm-count multisection, 65 sub-intervals per round over the
            // lanes of wave 0 (12 rounds shrink the Gershgorin interval by 65^12 ~ 5e21)
            __syncthreads();
            if (wave == 0) {
                double lo = 1e300, hi = -1e300;
                for (int i = lane; i < n; i += 64) {
                    const double rad = (i > 0 ? fabs(Se[i - 1]) : 0.0) + (i < n - 1 ? fabs(Se[i]) : 0.0);
                    lo = fmin(lo, Sd[i] - rad);
                    hi = fmax(hi, Sd[i] + rad);
                }
                for (int off = 32; off >= 1; off >>= 1) {
                    lo = fmin(lo, __shfl_xor(lo, off));
                    hi = fmax(hi, __shfl_xor(hi, off));
                }
                for (int it = 0; it < 12 && hi - lo > 4.0 * eps * fmax(fabs(lo), fabs(hi)); ++it) {
                    const double x = lo + (hi - lo) * (double)(lane + 1) / 65.0;
                    int cnt = 0;
                    double q = 1.0;
                    for (int i = 0; i < n; ++i) {
                        const double ei = i > 0 ? Se[i - 1] : 0.0;
                        q = (Sd[i] - x) - (i > 0 ? ei * ei / q : 0.0);
                        if (q == 0.0) q = -1e-300;   // x is an eigenvalue of the leading block
                        cnt += q < 0.0;
                    }
                    const unsigned long long hit = __ballot(cnt >= 1);   // lambda_min < x_lane
                    const int f = hit ? __ffsll((long long)hit) - 1 : 64;
                    const double xf = __shfl(x, f < 64 ? f : 63);
                    const double xp = __shfl(x, f > 0 ? f - 1 : 0);
                    const double nlo = f > 0 ? xp : lo;
                    const double nhi = f < 64 ? xf : hi;
                    lo = nlo;
                    hi = nhi;
                }
                if (lane == 0) a.loc.wlim[unit] = (float)sqrt(fmax(0.5 * (lo + hi), 0.0));
            }
            __syncthreads();
            continue;
        }
        // rows of Z this workgroup runs QL on (stage 2: the P-th part, 64-row aligned; the QL
        // recurrence is replicated, the rotations touch rows independently)
        const int part_len = ((n + P - 1) / P + 63) & ~63;
        const int row_lo = st == 2 ? min(n, part * part_len) : 0;
        const int row_hi = st == 2 ? min(n, row_lo + part_len) : n;
        if (st == 0 || (st == 2 && row_lo < row_hi)) {
        // Z = I: tql2 accumulates the tridiagonal eigenvectors, Q is applied afterwards
        {
            const int w = row_hi - row_lo;
            for (size_t idx = tid; idx < (size_t)n * w; idx += SP_T) {
                const int c = (int)(idx / w), r = row_lo + (int)(idx - (size_t)c * w);
                Zb[(size_t)c * n + r] = r == c ? 1.0 : 0.0;
            }
        }
        __syncthreads();
        if (tid == 0) t2 = __builtin_amdgcn_s_memtime();

        if (tid == 0) t3 = __builtin_amdgcn_s_memtime();
        // ---- 3. implicit QL (tql2) on Z: one generator wave, seven applier waves ------------
        // Wave 0 runs the QL recurrence on (d, e) -- which never reads Z -- and writes the
        // rotation sequences of up to SP_QB consecutive iterations (each on its own [l, m])
        // into one of two coefficient buffers; lane 0 carries the serial rotation chain, the
        // whole wave does the per-iteration shift of d and the buffer resets.  Meanwhile
        // waves 1..7 apply the previous batch in ONE pass over the touched columns of Z:
        // sequence t lags sequence t-1 by one position, so a row streams through all SP_QB
        // sweeps with one load and one store per column.  Positions outside a sequence's
        // range hold the identity rotation (c = 1, s = 0), which turns the carry into a plain
        // one-column delay, so the pass is branch-free.
        {
            constexpr int QB = SP_QB;
            // coefficient buffers, diagonal layout: row rw holds stage t's rotation at position
            // rw + t in column t, so the QB pairs one applier step needs are contiguous
            constexpr int OFF = QB + 4;
            static_assert(QB == 16, "applier: 64 lanes = 4 steps x 16 stages");
            const int gld = n + 2 * QB + 4;                 // rows -OFF .. n+QB-1
            double2* Gbuf = reinterpret_cast<double2*>(st == 2 ? M + bo + Lo.gbuf + (size_t)part * Lo.gsz
                                                               : Wp + (size_t)SP_NB * n);   // [2][gld][QB]
            int* const seqb = HUGE ? H.seq : Sperm;         // (BIG: perm is free until 4c)
            int* seq_l = seqb;                              // [2][QB]
            int* seq_m = seqb + 2 * QB;                     // [2][QB]
            int* bflag = seqb + 4 * QB;                     // [2] nseq, [2] generator done
            for (size_t idx = tid; idx < (size_t)2 * QB * gld; idx += SP_T) Gbuf[idx] = make_double2(1.0, 0.0);
            if (tid < 2 * QB) {
                seq_l[tid] = 0;
                seq_m[tid] = 0;
            }
            if (tid < 4) bflag[tid] = 0;
            __syncthreads();
            // generator state (wave 0, uniform across its lanes)
            int gl = 0, gm = 0, giter = 0, gphase = 0;
            double gf = 0.0, gtst1 = 0.0;
            auto gen_batch = [&](int buf) {
                const unsigned long long tg = lane == 0 ? __builtin_amdgcn_s_memtime() : 0ull;
                double2* G = Gbuf + (size_t)buf * QB * gld;
                // identity back into the ranges this buffer held two batches ago
                for (int t = 0; t < bflag[buf]; ++t) {
                    const int lo = seq_l[buf * QB + t], hi = seq_m[buf * QB + t];
                    for (int pp = lo + lane; pp < hi; pp += 64) G[(size_t)(pp - t + OFF) * QB + t] = make_double2(1.0, 0.0);
                }
                __threadfence_block();
                int nseq = 0;
                while (nseq < QB && gl < n) {
                    // HUGE with d / e in the slot: the lanes' stores of the previous iteration
                    // land before this one reads them (LDS accesses of a wave are in order)
                    if constexpr (HUGE) __threadfence_block();
                    if (gphase == 0) {
                        gtst1 = fmax(gtst1, fabs(Sd[gl]) + fabs(Se[gl]));
                        // m = first index >= l with a negligible e[m] (n if none): 64 at a time
                        int mfound = n;
                        for (int m0 = gl; m0 < n; m0 += 64) {
                            const int mi = m0 + lane;
                            const bool neg = mi < n && fabs(Se[mi]) <= eps * gtst1;
                            const unsigned long long bal = __ballot(neg);
                            if (bal) {
                                mfound = m0 + __builtin_ctzll(bal);
                                break;
                            }
                        }
                        gm = mfound;
                        if (gm == gl) {
                            if (lane == 0) {
                                Sd[gl] += gf;
                                Se[gl] = 0.0;
                            }
                            ++gl;
                            continue;
                        }
                        giter = 0;
                        gphase = 1;
                    }
                    const int l = gl, m = gm;
                    ++giter;
                    if (lane == 0) {
                        ++n_iter;
                        n_rot += (unsigned long long)(m - l);
                    }
                    double hsh = 0.0;
                    if (lane == 0) {
                        const double g0 = Sd[l];
                        double p = (Sd[l + 1] - g0) / (2.0 * Se[l]);
                        double r = hypot(p, 1.0);
                        if (p < 0) r = -r;
                        Sd[l] = Se[l] / (p + r);
                        Sd[l + 1] = Se[l] * (p + r);
                        hsh = g0 - Sd[l];
                    }
                    hsh = __shfl(hsh, 0);
                    for (int i = l + 2 + lane; i < n; i += 64) Sd[i] -= hsh;
                    gf += hsh;
                    if constexpr (HUGE) __threadfence_block();   // lane 0's d[l + 1], the shifted d
                    // the bulge chase, in two phases per 64 positions.  (A) the serial
                    // chain alone, on wave-uniform values: p and 1/r of each rotation, with
                    // e_i^2 and d_i broadcast from a per-lane block by v_readlane and the
                    // two results kept in the position's lane by v_cndmask -- ~24 VALU per
                    // rotation, no memory access.  (B) every output of the 64 rotations
                    // (c, s, e and d one place down) at once, lane t = rotation t.  The
                    // chain never reads a position it has written (writes go to i + 1).
                    // tools/probes/fp64_chain_probe.hip: 167 cycles per rotation against
                    // 272 for the one-phase loop (whose stores and extra VALU sat in the
                    // chain's issue stream).
                    const double dl1 = Sd[l + 1];
                    const double el1 = Se[l + 1];
                    double p = Sd[m];
                    double c = 1.0;
                    // c of the last three rotations and s of the last two (QL's c, c2, c3,
                    // s, s2 at the end of the chase)
                    double hc1 = 1.0, hc2 = 1.0, hc3 = 1.0, hs1 = 0.0, hs2 = 0.0;
                    for (int ib = m - 1; ib >= l; ib -= 64) {
                        const int cnt = min(64, ib - l + 1);
                        const int pos = ib - lane;
                        double eL = lane < cnt ? Se[pos] : 0.0;
                        double dL = lane < cnt ? Sd[pos] : 0.0;
                        // a register redefinition: the loads are waited for here, once
                        asm volatile("" : "+v"(eL), "+v"(dL));
                        const double e2L = eL * eL;
                        double pT = 0.0, iT = 0.0;   // lane t: p entering rotation t, its 1/r
                        for (int t = 0; t < cnt; ++t) {
                            const double ei2 = bcast_lane(e2L, t);
                            const double di = bcast_lane(dL, t);
                            // r = hypot(p, e_i); |p|, |e_i| <= ||T|| here, so the plain form
                            // neither overflows nor underflows.  1/r = rsq(x2) refined by two
                            // Newton steps (inv += inv (1/2 - x2/2 inv^2); 0.5 is an inline
                            // constant).  p' = c' d_i - s' c e_i = (p d_i - c e_i^2) / r.
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
                        // (B) lane t < cnt: rotation t at position i = ib - t
                        const double cT = pT * iT, sT = eL * iT;
                        const double rT = fma(pT, pT, e2L) * iT;
                        double cP = __shfl_up(cT, 1), sP = __shfl_up(sT, 1);   // rotation t - 1
                        if (lane == 0) {
                            cP = hc1;
                            sP = hs1;
                        }
                        const double g = cP * eL;
                        const double en = sP * rT;
                        const double dn = cP * pT + sT * (cT * g + sT * dL);
                        if (lane < cnt) {
                            Se[pos + 1] = en;
                            Sd[pos + 1] = dn;
                            G[(size_t)(pos - nseq + OFF) * QB + nseq] = make_double2(cT, sT);
                        }
                        const double b1 = __shfl(cT, cnt - 1), b2 = __shfl(cT, max(cnt - 2, 0)),
                                     b3 = __shfl(cT, max(cnt - 3, 0));
                        const double q1 = __shfl(sT, cnt - 1), q2 = __shfl(sT, max(cnt - 2, 0));
                        const double o1 = hc1, o2 = hc2, os1 = hs1;
                        hc1 = b1;
                        hc2 = cnt >= 2 ? b2 : o1;
                        hc3 = cnt >= 3 ? b3 : (cnt == 2 ? o1 : o2);
                        hs1 = q1;
                        hs2 = cnt >= 2 ? q2 : os1;
                    }
                    const double sn = hs1;
                    p = -sn * hs2 * hc3 * el1 * Se[l] / dl1;
                    c = hc1;
                    const double e_l = sn * p;
                    const int conv = !(fabs(e_l) > eps * gtst1 && giter < 60);
                    if (lane == 0) {
                        Se[l] = e_l;
                        Sd[l] = c * p;
                        seq_l[buf * QB + nseq] = l;
                        seq_m[buf * QB + nseq] = m;
                        if (conv) {
                            Sd[l] += gf;
                            Se[l] = 0.0;
                        }
                    }
                    ++nseq;
                    if (conv) {
                        ++gl;
                        gphase = 0;
                    }
                }
                if (lane == 0) {
                    bflag[buf] = nseq;
                    bflag[2 + buf] = gl >= n;
                    tgen += __builtin_amdgcn_s_memtime() - tg;
                }
            };
            if (wave == 0) gen_batch(0);
            __syncthreads();
            // appliers: waves 1..7, two rows per thread (rows r0 and r0 + NA share each
            // coefficient load)
            const bool applier = wave != 0;
            const int ta = tid - 64;
            constexpr int NA = SP_T - 64;
            for (int b = 0;; ++b) {
                const int buf = b & 1;
                const int nseq = bflag[buf];
                if (nseq == 0) break;                       // uniform
                const int gen_done = bflag[2 + buf];
                if (wave == 0) {
                    if (!gen_done) {
                        gen_batch(buf ^ 1);
                    } else if (lane == 0) {
                        bflag[buf ^ 1] = 0;
                    }
                } else if (applier) {
                    int L = n, Mx = 0;
                    for (int t = 0; t < nseq; ++t) {
                        L = min(L, seq_l[buf * QB + t]);
                        Mx = max(Mx, seq_m[buf * QB + t]);
                    }
                    const double2* G = Gbuf + (size_t)buf * QB * gld;
                    for (int rbase = row_lo; rbase < row_hi; rbase += 2 * NA) {
                        // every lane stays active (the coefficient pairs are read from all
                        // 64 lanes); rows past row_hi alias row_lo and do not store
                        const int r0 = rbase + ta, r1 = r0 + NA;
                        if (rbase + (wave - 1) * 64 >= row_hi) continue;   // the whole wave is past the rows
                        const bool a0 = r0 < row_hi, a1 = r1 < row_hi;
                        double c0[QB], c1[QB];
#pragma unroll
                        for (int t = 0; t < QB; ++t) {
                            c0[t] = 0.0;
                            c1[t] = 0.0;
                        }
                        double* z0 = Zb + (a0 ? r0 : row_lo);
                        double* z1 = Zb + (a1 ? r1 : row_lo);
                        // four steps per iteration: one coalesced load brings the 4 x 16
                        // coefficient pairs (lane 16u + t: step u, stage t), v_readlane puts
                        // each pair in SGPRs for the FMAs; the next four columns of both rows
                        // are loaded one iteration ahead
                        double n0[4], n1[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            n0[u] = Mx - u >= L ? z0[(size_t)(Mx - u) * n] : 0.0;
                            n1[u] = Mx - u >= L ? z1[(size_t)(Mx - u) * n] : 0.0;
                        }
                        for (int tau = Mx; tau >= L - QB; tau -= 4) {
                            const double2 csl = G[(size_t)(tau - (lane >> 4) + OFF) * QB + (lane & 15)];
                            double v0[4], v1[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                v0[u] = n0[u];
                                v1[u] = n1[u];
                                const int tn = tau - 4 - u;
                                n0[u] = tn >= L ? z0[(size_t)tn * n] : 0.0;
                                n1[u] = tn >= L ? z1[(size_t)tn * n] : 0.0;
                            }
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
#pragma unroll
                                for (int t = 0; t < QB; ++t) {
                                    const double cx = bcast_lane(csl.x, 16 * u + t);
                                    const double sy = bcast_lane(csl.y, 16 * u + t);
                                    const double o0 = sy * v0[u] + cx * c0[t];
                                    c0[t] = cx * v0[u] - sy * c0[t];
                                    v0[u] = o0;
                                    const double o1 = sy * v1[u] + cx * c1[t];
                                    c1[t] = cx * v1[u] - sy * c1[t];
                                    v1[u] = o1;
                                }
                                const int tc = tau - u + QB;
                                if (tc <= Mx && tc >= L) {
                                    if (a0) z0[(size_t)tc * n] = v0[u];
                                    if (a1) z1[(size_t)tc * n] = v1[u];
                                }
                            }
                        }
                    }
                }
                __syncthreads();
            }
        }
        }   // st == 0 || st == 2
        const unsigned long long t4 = tid == 0 ? __builtin_amdgcn_s_memtime() : 0ull;
        if (st == 2) {   // the eigenvalues (every part computed the same d) to the slot
            if (part == 0) {
                for (int i = tid; i < n; i += SP_T) M[bo + Lo.df + i] = Sd[i];
                if (a.phase && tid == 0) {
                    atomicAdd(&a.phase[4], t4 - t3);
                    atomicAdd(&a.phase[5], tgen);
                    atomicAdd(&a.phase[6], n_iter);
                    atomicAdd(&a.phase[1], n_rot);   // staged path: slot 1 (assembly) holds the rotation count
                }
            }
            __syncthreads();
            continue;
        }
        // ---- 4a. Z to row-major (in place, 32 x 32 tile pairs through LDS) ------------------
        if (st == 0 || st == 3) {
            double* buf = stage;   // two 32 x 33 tiles
            const int nt = (n + 31) >> 5;
            for (int I = 0; I < nt; ++I) {
                for (int J = I; J < nt; ++J) {
                    for (int idx = tid; idx < 2048; idx += SP_T) {
                        const int which = idx >> 10, el = idx & 1023, cc = el >> 5, rr = el & 31;
                        const int r = (which ? J : I) * 32 + rr, c = (which ? I : J) * 32 + cc;
                        buf[which * 1056 + cc * 33 + rr] = (r < n && c < n) ? Zb[(size_t)c * n + r] : 0.0;
                    }
                    __syncthreads();
                    for (int idx = tid; idx < 2048; idx += SP_T) {
                        const int which = idx >> 10, el = idx & 1023, cc = el >> 5, rr = el & 31;
                        // which 0: block (rows I, cols J) <- tile B transposed; 1: (rows J, cols I) <- A^T
                        const int r = (which ? J : I) * 32 + rr, c = (which ? I : J) * 32 + cc;
                        if (r < n && c < n) Zb[(size_t)c * n + r] = buf[(which ? 0 : 1056) + rr * 33 + cc];
                    }
                    __syncthreads();
                }
            }
        }
        if (st == 3) continue;
        // columns of Z this workgroup back-transforms and writes (stage 4: the P-th part)
        const int col_lo = st == 4 ? min(n, part * part_len) : 0;
        const int col_hi = st == 4 ? min(n, col_lo + part_len) : n;
        if (col_lo >= col_hi) continue;   // uniform
        // ---- 4b. eigenvectors of A = Q Z: compact-WY panels applied last to first --------------
        // P_b = H_p ... H_{p+jb-1} = I - V T V^T (dlarft forward/columnwise), Z(p+1:n, :) -=
        // V (T (V^T Z)).  Lane per column of the row-major Z; V rows staged in LDS and read as
        // wave-uniform broadcasts, the jb-vectors V^T z and T (V^T z) live in registers.
        {
            double* Tm = stage;              // [SP_NB][SP_NB]
            double* Gm = stage + SP_NB * SP_NB;
            double* Vs = HUGE ? HW.vsb : Se;   // [SP_RC][SP_NB + 1]
            constexpr int VLD = SP_NB + 1;
            for (int p = ((n - 2) / SP_NB) * SP_NB; p >= 0; p -= SP_NB) {
                const int jb = min(SP_NB, n - 1 - p);
                for (int q = wave; q < SP_NB * SP_NB; q += SP_W) {
                    const int t = q / SP_NB, i = q - t * SP_NB;
                    if (t < i && i < jb) {
                        const double* vt = M + (size_t)(p + t) * n;
                        const double* vi = M + (size_t)(p + i) * n;
                        double s = 0.0;
                        for (int r = p + i + 1 + lane; r < n; r += 64) s += vt[r] * vi[r];
                        s = wave_sum(s);
                        if (lane == 0) Gm[q] = s;
                    }
                }
                for (int idx = tid; idx < SP_NB * SP_NB; idx += SP_T) Tm[idx] = 0.0;
                __syncthreads();
                for (int i = 0; i < jb; ++i) {
                    const double ti = tau[p + i];
                    if (tid < i) {
                        double s = 0.0;
                        for (int s_ = tid; s_ < i; ++s_) s += Tm[tid * SP_NB + s_] * Gm[s_ * SP_NB + i];
                        Tm[tid * SP_NB + i] = -ti * s;
                    } else if (tid == i) {
                        Tm[i * SP_NB + i] = ti;
                    }
                    __syncthreads();
                }
                const int r_lo = p + 1;
                for (int cbase = col_lo; cbase < col_hi; cbase += SP_W * 64) {
                    const int c = cbase + wave * 64 + lane;
                    const bool cact = c < col_hi;
                    double x[SP_NB];
#pragma unroll
                    for (int t = 0; t < SP_NB; ++t) x[t] = 0.0;
                    for (int half = 0; half < 2; ++half) {
                        for (int rc0 = r_lo; rc0 < n; rc0 += SP_RC) {
                            const int rn = min(SP_RC, n - rc0);
                            __syncthreads();
                            for (int idx = tid; idx < SP_RC * SP_NB; idx += SP_T) {
                                const int t = idx / SP_RC, rr = idx - t * SP_RC;
                                const int r = rc0 + rr;
                                Vs[rr * VLD + t] = (rr < rn && t < jb && r >= p + t + 1) ? M[(size_t)(p + t) * n + r] : 0.0;
                            }
                            __syncthreads();
                            if (!cact) continue;
                            double* zc = Zb + (size_t)rc0 * n + c;
                            // software-pipelined rows: the next 8 rows' loads are in flight
                            // while the current 8 are used (the row loop is latency-bound
                            // otherwise); rows past rn read row rc0 and meet zero V entries
                            double cur[8];
#pragma unroll
                            for (int u8 = 0; u8 < 8; ++u8) cur[u8] = zc[(size_t)(u8 < rn ? u8 : 0) * n];
                            for (int rr = 0; rr < rn; rr += 8) {
                                double nxt[8];
#pragma unroll
                                for (int u8 = 0; u8 < 8; ++u8) {
                                    const int rq = rr + 8 + u8;
                                    nxt[u8] = zc[(size_t)(rq < rn ? rq : 0) * n];
                                }
#pragma unroll
                                for (int u8 = 0; u8 < 8; ++u8) {
                                    __builtin_amdgcn_sched_barrier(0);
                                    const double* vr = Vs + (rr + u8) * VLD;
                                    if (half == 0) {
#pragma unroll
                                        for (int t = 0; t < SP_NB; ++t) x[t] += vr[t] * cur[u8];
                                    } else {
                                        double s0 = 0.0, s1 = 0.0;
#pragma unroll
                                        for (int t = 0; t < SP_NB; t += 2) {
                                            s0 += vr[t] * x[t];
                                            s1 += vr[t + 1] * x[t + 1];
                                        }
                                        if (rr + u8 < rn) zc[(size_t)(rr + u8) * n] = cur[u8] - (s0 + s1);
                                    }
                                }
#pragma unroll
                                for (int u8 = 0; u8 < 8; ++u8) cur[u8] = nxt[u8];
                            }
                        }
                        if (half == 0) {   // x <- T x (T upper triangular)
#pragma unroll
                            for (int s_ = 0; s_ < SP_NB; ++s_) {
                                double acc = 0.0;
#pragma unroll
                                for (int t = s_; t < SP_NB; ++t) acc += Tm[s_ * SP_NB + t] * x[t];
                                x[s_] = acc;
                            }
                        }
                    }
                }
                __syncthreads();
            }
        }
        // ---- 4c. order, sign, lim, output --------------------------------------------------
        // (stage 4: every part ranks all eigenvalues; the sign and the output are its columns',
        // with each column's rank kept in the slot's rc)
        int* rank_of = st == 4 ? reinterpret_cast<int*>(rc) : nullptr;
        for (int j = tid; j < n; j += SP_T) {
            const double lj = Sd[j];
            int rank = 0;
            for (int i = 0; i < n; ++i) {
                const double li = Sd[i];
                rank += (li < lj) || (li == lj && i < j);
            }
            Sperm[rank] = j;
            if (rank_of) rank_of[j] = rank;
        }
        for (int cb = col_lo + wave * 64; cb < col_hi; cb += SP_W * 64) {
            const int c = cb + lane;
            if (c < col_hi) {
                double s0 = 0.0, s1 = 0.0;
                int r = 0;
                for (; r + 2 <= n; r += 2) {
                    s0 += Zb[(size_t)r * n + c];
                    s1 += Zb[(size_t)(r + 1) * n + c];
                }
                if (r < n) s0 += Zb[(size_t)r * n + c];
                rs[c] = (s0 + s1) < 0.0 ? -1.0 : 1.0;
            }
        }
        __syncthreads();
        if (tid == 0) {
            int lim = n;   // local_calc keeps every eigenpair (es(ll2), local_calc.cpp:378): modes 1, 3
            if (mode == 0) {
                float smm = 0.0f;
                for (int i = 0; i < n; ++i)
                    if (smm < sig_get(i)) smm = sig_get(i);
                smm = (float)((double)smm + 0.01);   // (:179-182)
                for (lim = 0; lim < n; ++lim)
                    if (Sd[Sperm[lim]] > (double)smm) break;   // (:186-188)
                if (lim < 2) lim = 2;                             // (:190-191)
            }
            s_flag[3] = lim;
            a.m_out[u] = lim;
        }
        __syncthreads();
        const int mm = s_flag[3];
        if (part == 0) {
            if (mode == 0)
                for (int i = tid; i < n; i += SP_T) a.sigs[base + i] = (float)((double)sig_get(i) + 0.01);
            for (int r = tid; r < mm; r += SP_T) a.evals[base + r] = (float)Sd[Sperm[r]];
        }
        if (st == 4) {
            const int w = col_hi - col_lo;
            for (size_t idx = tid; idx < (size_t)n * w; idx += SP_T) {
                const int i = (int)(idx / w), j = col_lo + (int)(idx - (size_t)i * w);
                const int r = rank_of[j];
                if (r < mm) Wt[(size_t)i * mm + r] = (float)(Zb[(size_t)i * n + j] * rs[j]);
            }
            __syncthreads();
            if (a.phase && tid == 0 && part == 0) {
                atomicAdd(&a.phase[0], 1ull);
                atomicAdd(&a.phase[7], __builtin_amdgcn_s_memtime() - t4);
            }
            continue;
        }
        for (size_t idx = tid; idx < (size_t)n * mm; idx += SP_T) {
            const int i = (int)(idx / mm), r = (int)(idx - (size_t)i * mm);
            const int j = Sperm[r];
            Wt[idx] = (float)(Zb[(size_t)i * n + j] * rs[j]);
        }
        __syncthreads();
        if (a.phase && tid == 0) {
            const unsigned long long t5 = __builtin_amdgcn_s_memtime();
            atomicAdd(&a.phase[0], 1ull);
            atomicAdd(&a.phase[1], t1 - t0);
            atomicAdd(&a.phase[2], t2 - t1);
            atomicAdd(&a.phase[3], t3 - t2);
            atomicAdd(&a.phase[4], t4 - t3);
            atomicAdd(&a.phase[5], tgen);
            atomicAdd(&a.phase[6], n_iter);
            atomicAdd(&a.phase[7], t5 - t4);
        }
    }
}

// ---- multi-CU tridiagonalisation of the BIG users (k > SP_NL), all of a launch at once ----------
// The single-workgroup solver spends ~54% of a k = 4000 user in the tridiagonalisation, and its
// per-reflector symmetric matrix-vector product reads the whole trailing matrix from HBM through
// ONE CU.  Here the same blocked algorithm (dlatrd panels of SP_NB, the stage-2 code of
// eigen_spill_kernel) runs as a sequence of launches over every BIG user of the batch: per
// reflector j, spill_mc_col (one workgroup per user: the column update, the reflector, the
// panel dot products), spill_mc_symv (G workgroups per user, each a block of the trailing rows)
// and spill_mc_fin (one per user: the panel corrections, w); per panel, spill_mc_trail (G2 per
// user, column blocks of the rank-2 SP_NB update).  Kernel boundaries order the steps, so no
// workgroup waits on another.  The QL and back-transform then resume in eigen_spill_kernel
// (mc_stage 2) from the slot's d, e, tau and the reflectors stored in M.
struct McArgs {
    const uint32_t* order;
    uint32_t first;
    uint32_t count;
    const uint64_t* item_off;
    double* work;
    const uint64_t* slot_off;   // per user of the wave: its slot's offset in `work` (doubles); the
                                // McLayout vectors start spill_base_stride(k) into the slot
    int G;               // workgroups per user of spill_mc_symv / spill_mc_trail
    uint64_t vs;         // McLayout vector stride
    // the multi-workgroup assembly (spill_mc_deg / spill_mc_l2 / spill_mc_gram)
    const uint32_t* items;
    GraphDev graph;
    int mode;            // cf_spill_local::mode (0: compute_eigens)
    float* l2;           // mode 1 writes the movie's L2, mode 3 reads it
    const uint64_t* l2_off;
};

__device__ __forceinline__ double* mc_slot(const McArgs& a, uint32_t u) { return a.work + a.slot_off[u]; }

__device__ __forceinline__ int mc_n(const McArgs& a, uint32_t u) {
    const uint32_t unit = a.order[a.first + u];
    return (int)(a.item_off[unit + 1] - a.item_off[unit]);
}

// column j of the panel at p: bring it up to date with the panel's earlier reflectors, form
// its reflector (v in M(j+1:n, j) and rc, tau, d, e), and the panel dot products xv, xw
__global__ __launch_bounds__(SP_T) void spill_mc_col(McArgs a, int j, int p) {
    __shared__ double vj[SP_NB], wj[SP_NB], red[SP_W + 4];
    const uint32_t u = blockIdx.x;
    const int n = mc_n(a, u);
    if (j >= n - 1) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, jj = j - p;
    double* M = mc_slot(a, u);
    const uint64_t bo = spill_base_stride((uint64_t)n);
    double* Wp = M + 2 * (size_t)n * n;
    const McLayout Lo(a.vs);
    double* rc = M + bo;
    double* tau = rc + 2 * Lo.vs;
    double* mc = M + bo;
    double* colj = M + (size_t)j * n;
    if (jj > 0) {
        if (tid < jj) {
            vj[tid] = M[(size_t)(p + tid) * n + j];
            wj[tid] = Wp[(size_t)tid * n + j];
        }
        __syncthreads();
        for (int r = j + tid; r < n; r += SP_T) {
            double acc = colj[r];
            for (int t = 0; t < jj; ++t) acc -= M[(size_t)(p + t) * n + r] * wj[t] + Wp[(size_t)t * n + r] * vj[t];
            colj[r] = acc;
        }
        __syncthreads();
    }
    const double alpha = colj[j + 1];
    const double ajj = colj[j];
    double part = 0.0;
    for (int r = j + 2 + tid; r < n; r += SP_T) {
        const double x = colj[r];
        part += x * x;
    }
    const double sigma = block_sum(part, red);
    double tj = 0.0, beta = alpha, scal = 0.0;
    if (sigma != 0.0) {
        beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
        tj = (beta - alpha) / beta;
        scal = 1.0 / (alpha - beta);
    }
    if (tid == 0) {
        mc[Lo.d + j] = ajj;
        mc[Lo.e + j] = beta;
        tau[j] = tj;
    }
    for (int r = j + 1 + tid; r < n; r += SP_T) {
        const double vr = (r == j + 1) ? 1.0 : colj[r] * scal;
        rc[r] = vr;
        colj[r] = vr;
    }
    __syncthreads();
    if (tj == 0.0) return;
    // x_v[t] = W(:,t).v and x_w[t] = V(:,t).v over rows j+1..n-1, one wave per dot
    const int r0 = j + 1;
    for (int q = wave; q < 2 * jj; q += SP_W) {
        const int t = q >> 1;
        const double* src = (q & 1) ? M + (size_t)(p + t) * n : Wp + (size_t)t * n;
        double sdot = 0.0;
        for (int r = r0 + lane; r < n; r += 64) sdot += src[r] * rc[r];
        sdot = wave_sum(sdot);
        if (lane == 0) mc[((q & 1) ? Lo.xw : Lo.xv) + t] = sdot;
    }
}

// y = A(r0:n, r0:n) v on G workgroups per user, each 64 x 64 tile of the lower triangle read
// once (the matrix is symmetric; spill_mc_trail keeps only the lower triangle and a 64-wide band
// above the diagonal up to date).  Tiles are anchored at r0.  Workgroup g takes the row-block
// pairs {k, nrb - 1 - k}, k = g, g + G, ... (nrb + 1 tiles a pair: balanced); wave w of it the
// column blocks C = w, w + 4, ... <= R.  A tile (R, C) adds
// A_RC v_C to the rows' partial y_R (lane = row, column-major loads coalesce) and, below the
// diagonal, A_RC^T v_R to the pair's partial z_k over C's columns (the 64 x 16 products of a
// slab transposed through the wave's LDS scratch, four 16-row sums per column).  z_k lives in
// the slot; a column block always belongs to the same wave, so its z entries are updated by one
// lane, R = k then nrb - 1 - k: deterministic, and independent of G.  spill_mc_fin forms y =
// y_R + sum_k z_k in pair order.
constexpr int MC_SYMV_T = 256;
#ifndef CF_SYMV_ZPRE
#define CF_SYMV_ZPRE 1   // (A/B: 0 = z loaded at the += itself)
#endif
constexpr int MC_TQ = 16 * 65;   // a wave's slab transposition scratch: 16 columns x 64 rows (+1 pad)
// HUGE (k > CF_SPILL_MAX_K): v is read from the slot (L2-resident) instead of an LDS copy.
template <bool HUGE>
__global__ __launch_bounds__(MC_SYMV_T) void spill_mc_symv(McArgs a, int j) {
    __shared__ double vs_lds[HUGE ? 1 : CF_SPILL_MAX_K];
    __shared__ double part[MC_SYMV_T / 64][64];
    __shared__ double tq[MC_SYMV_T / 64][MC_TQ];
    const uint32_t u = blockIdx.x / a.G;
    const int g = blockIdx.x % a.G;
    const int n = mc_n(a, u);
    if (j >= n - 1) return;
    double* M = mc_slot(a, u);
    const uint64_t bo = spill_base_stride((uint64_t)n);
    const McLayout Lo(a.vs);
    const double* rc = M + bo;
    double* rs = M + bo + Lo.vs;
    const double tj = rc[2 * Lo.vs + j];
    if (tj == 0.0) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const double* vs = HUGE ? rc : vs_lds;
    constexpr int NWV = MC_SYMV_T / 64;
    const int r0 = j + 1;
    const int nrb = (n - r0 + 63) >> 6;
    const int npair = (nrb + 1) >> 1;
    if (g >= npair) return;   // uniform; spill_mc_fin sums z over every pair
    if (!HUGE)
        for (int c = r0 + tid; c < n; c += MC_SYMV_T) vs_lds[c] = rc[c];
    // z_k = 0 for every pair k of this workgroup, on this wave's column blocks, by the lanes that
    // update them below.  One partial per row-block PAIR (not per workgroup): the sums are then
    // the same whatever G the launch uses (G depends on how many users share the wave, so a
    // per-workgroup partial made a user's records depend on the other users of its batch)
    for (int k = g; k < npair; k += a.G) {
        double* zk = M + bo + Lo.gbuf + (size_t)k * Lo.vs;
        for (int C = wave; C < nrb; C += NWV)
            for (int s16 = 0; s16 < 64; s16 += 16) {
                const int c = r0 + C * 64 + s16 + lane;
                if (lane < 16 && c < n) zk[c] = 0.0;
            }
    }
    __syncthreads();
    double* q = tq[wave];
    const int ci = lane & 15, qq = lane >> 4;
    for (int it = 0; it < 2 * ((npair - g + a.G - 1) / a.G); ++it) {
        const int k = g + (it >> 1) * a.G;
        const int R = (it & 1) ? nrb - 1 - k : k;
        if ((it & 1) && R == k) continue;   // the middle block of an odd count (uniform)
        double* z = M + bo + Lo.gbuf + (size_t)k * Lo.vs;
        const int r = r0 + R * 64 + lane;
        const bool ract = r < n;
        const double vr = ract ? vs[r] : 0.0;
        double y0 = 0.0, y1 = 0.0;
        for (int C = wave; C <= R; C += NWV) {
            const int cb0 = r0 + C * 64;
            const int cw = min(64, n - cb0);
            for (int s16 = 0; s16 < cw; s16 += 16) {
                const int c0 = cb0 + s16;
                double x[16];
                const double* mp = M + (size_t)c0 * n + r;
                // z's old value is loaded with the slab, so the += below waits on that batch of
                // loads instead of starting a round trip of its own per slab
                const bool zl = CF_SYMV_ZPRE && C < R && qq == 0 && s16 + ci < cw;
                const double zold = zl ? z[c0 + ci] : 0.0;
#pragma unroll
                for (int t = 0; t < 16; ++t) x[t] = (ract && s16 + t < cw) ? mp[(size_t)t * n] : 0.0;
#pragma unroll
                for (int t = 0; t < 16; t += 2) {
                    y0 = fma(x[t], s16 + t < cw ? vs[c0 + t] : 0.0, y0);
                    y1 = fma(x[t + 1], s16 + t + 1 < cw ? vs[c0 + t + 1] : 0.0, y1);
                }
                if (C < R) {
#pragma unroll
                    for (int t = 0; t < 16; ++t) q[t * 65 + lane] = x[t] * vr;
                    double sacc = 0.0;
#pragma unroll
                    for (int rr = 0; rr < 16; ++rr) sacc += q[ci * 65 + qq * 16 + rr];
                    sacc += __shfl_xor(sacc, 16);
                    sacc += __shfl_xor(sacc, 32);
                    if (qq == 0 && s16 + ci < cw) {
                        if (CF_SYMV_ZPRE) z[c0 + ci] = zold + sacc;
                        else z[c0 + ci] += sacc;
                    }
                }
            }
        }
        part[wave][lane] = y0 + y1;
        __syncthreads();
        if (wave == 0 && ract) {
            double y = 0.0;
#pragma unroll
            for (int w = 0; w < NWV; ++w) y += part[w][lane];
            rs[r] = y;
        }
        __syncthreads();
    }
}

// w_jj = tau (y - V xv - W xw) - tau/2 ((...) . v) v into W(:, jj) (0 above row j+1)
__global__ __launch_bounds__(SP_T) void spill_mc_fin(McArgs a, int j, int p) {
    __shared__ double xv[SP_NB], xw[SP_NB], red[SP_W + 4];
    const uint32_t u = blockIdx.x;
    const int n = mc_n(a, u);
    if (j >= n - 1) return;
    const int tid = threadIdx.x, jj = j - p;
    double* M = mc_slot(a, u);
    const uint64_t bo = spill_base_stride((uint64_t)n);
    double* Wp = M + 2 * (size_t)n * n;
    const McLayout Lo(a.vs);
    const double* rc = M + bo;
    double* rs = M + bo + Lo.vs;
    const double* mc = M + bo;
    const double tj = rc[2 * Lo.vs + j];
    const int r0 = j + 1;
    if (tj == 0.0) {
        for (int r = tid; r < n; r += SP_T) Wp[(size_t)jj * n + r] = 0.0;
        return;
    }
    if (tid < jj) {
        xv[tid] = mc[Lo.xv + tid];
        xw[tid] = mc[Lo.xw + tid];
    }
    __syncthreads();
    // y = the row-block partials + the transposed partials z_k of spill_mc_symv (one per
    // row-block pair), in pair order
    const int gz = (((n - r0 + 63) >> 6) + 1) >> 1;
    const double* z = mc + Lo.gbuf;
    double yv = 0.0;
    for (int r = r0 + tid; r < n; r += SP_T) {
        double y = rs[r];
        for (int g = 0; g < gz; ++g) y += z[(size_t)g * Lo.vs + r];
        for (int t = 0; t < jj; ++t) y -= M[(size_t)(p + t) * n + r] * xv[t] + Wp[(size_t)t * n + r] * xw[t];
        y *= tj;
        rs[r] = y;
        yv += y * rc[r];
    }
    const double a2 = -0.5 * tj * block_sum(yv, red);
    for (int r = tid; r < n; r += SP_T) Wp[(size_t)jj * n + r] = r >= r0 ? rs[r] + a2 * rc[r] : 0.0;
}

// trailing update A(q:n, q:n) -= V W^T + W V^T after the panel at p, q = p + jb, on the lower
// triangle and a band of at least 64 above the diagonal (what spill_mc_symv reads): G
// workgroups per user, workgroup g the SP_CC-column chunks g, g + G, ... (interleaved, so the
// triangle's work is balanced); lane per row with that row's V and W entries in registers, each
// column's entries broadcast from LDS (the stage-2 code of eigen_spill_kernel)
__global__ __launch_bounds__(SP_T) void spill_mc_trail(McArgs a, int p) {
    __shared__ double stg[SP_CC * 2 * SP_NB];
    const uint32_t u = blockIdx.x / a.G;
    const int g = blockIdx.x % a.G;
    const int n = mc_n(a, u);
    if (p >= n - 1) return;
    const int jb = min(SP_NB, n - 1 - p);
    const int q = p + jb, mq = n - q;
    if (mq <= 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double* M = mc_slot(a, u);
    const double* Wp = M + 2 * (size_t)n * n;
    const int nchunk = (mq + SP_CC - 1) / SP_CC;
    if (g >= nchunk) return;   // uniform
    const int nrb = (mq + 63) >> 6;
    // row block rb (rows q + 64 rb ..) is updated in chunk ch iff its last row is >= the
    // chunk's first column - 64, i.e. ch * SP_CC <= 64 rb + 127
    const int rb_first = max(0, (g * SP_CC - 127 + 63) / 64);   // first row block any chunk of g needs
    for (int pass = (rb_first / SP_W) * SP_W; pass < nrb; pass += SP_W) {
        const int rb = pass + wave;
        const int r = q + rb * 64 + lane;
        const bool act = rb < nrb && r < n;
        const int ch_top = (min(pass + SP_W - 1, nrb - 1) * 64 + 127) / SP_CC;   // the pass's last chunk
        double vr[SP_NB], wr[SP_NB];
#pragma unroll
        for (int t = 0; t < SP_NB; ++t) {
            vr[t] = (act && t < jb) ? M[(size_t)(p + t) * n + r] : 0.0;
            wr[t] = (act && t < jb) ? Wp[(size_t)t * n + r] : 0.0;
        }
        for (int ch = g; ch < nchunk && ch <= ch_top; ch += a.G) {
            const int c0 = q + ch * SP_CC;
            const int cn = min(SP_CC, n - c0);
            __syncthreads();
            for (int idx = tid; idx < SP_CC * 2 * SP_NB; idx += SP_T) {
                const int cc = idx / (2 * SP_NB), t2 = idx - cc * (2 * SP_NB);
                const int t = t2 & (SP_NB - 1);
                double v = 0.0;
                if (cc < cn && t < jb) v = t2 < SP_NB ? M[(size_t)(p + t) * n + c0 + cc] : Wp[(size_t)t * n + c0 + cc];
                stg[idx] = v;
            }
            __syncthreads();
            if (!act || ch * SP_CC > rb * 64 + 127) continue;
            double* mp = M + (size_t)c0 * n + r;
            double cur[8];
#pragma unroll
            for (int u8 = 0; u8 < 8; ++u8) cur[u8] = u8 < cn ? mp[(size_t)u8 * n] : 0.0;
            for (int cc = 0; cc < cn; cc += 8) {
                double nxt[8];
#pragma unroll
                for (int u8 = 0; u8 < 8; ++u8) nxt[u8] = cc + 8 + u8 < cn ? mp[(size_t)(cc + 8 + u8) * n] : 0.0;
#pragma unroll
                for (int u8 = 0; u8 < 8; ++u8) {
                    __builtin_amdgcn_sched_barrier(0);
                    const double* sv = stg + (cc + u8) * 2 * SP_NB;
                    double acc0 = cur[u8], acc1 = 0.0;
#pragma unroll
                    for (int t = 0; t < SP_NB; t += 2) {
                        if ((t & 7) == 0) __builtin_amdgcn_sched_barrier(0);
                        acc0 -= vr[t] * sv[SP_NB + t] + wr[t] * sv[t];
                        acc1 -= vr[t + 1] * sv[SP_NB + t + 1] + wr[t + 1] * sv[t + 1];
                    }
                    if (cc + u8 < cn) mp[(size_t)(cc + u8) * n] = acc0 + acc1;
                }
#pragma unroll
                for (int u8 = 0; u8 < 8; ++u8) cur[u8] = nxt[u8];
            }
        }
    }
}

// the last diagonal element and e[n-1] = 0
__global__ void spill_mc_end(McArgs a) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= a.count) return;
    const int n = mc_n(a, u);
    double* M = mc_slot(a, u);
    const uint64_t bo = spill_base_stride((uint64_t)n);
    double* mc = M + bo;
    const McLayout Lo(a.vs);
    mc[Lo.d + n - 1] = M[(size_t)(n - 1) * n + (n - 1)];
    mc[Lo.e + n - 1] = 0.0;
}

// ---- multi-workgroup assembly of the staged users (stage 1 of eigen_spill_kernel, spread) -----
// One wave per row over every CU instead of one workgroup per user: at k = 10,000 the
// assembly moves ~1.6 GB per unit, which one CU takes tens of seconds to stream.  Same
// arithmetic and summation order per row as the single-workgroup stage 1 (lane-strided partial
// sums, the xor butterfly), so the results are bit-identical.  grid = (blocks per unit, units).
__device__ __forceinline__ float mc_weight(const McArgs& a, uint64_t base, int i, int j, const GraphRow& grow,
                                           const GraphRow& grow0) {
    float w = grow[a.items[base + j]];
    if (a.mode == 1) {   // the star-shaped local graph (local_calc.cpp:326-334), w > 0.1
        if (j == 0) w = (i == 0) ? 0.0f : grow0[a.items[base + i]];
        if (!((double)w > 0.1)) w = 0.0f;
    }
    return w;
}

// d_i (fp64, with the 0 -> 1 rule for users only, precompute_local_threads.cpp:137-140 vs
// local_calc.cpp:354-360) into rs, s_i = sqrt(1/d_i) (:149-153) into rc
__global__ __launch_bounds__(256) void spill_mc_deg(McArgs a) {
    const uint32_t ui = blockIdx.y;
    const uint32_t unit = a.order[a.first + ui];
    const uint64_t base = a.item_off[unit];
    const int n = (int)(a.item_off[unit + 1] - base);
    double* M = mc_slot(a, ui);
    const uint64_t bo = spill_base_stride((uint64_t)n);
    double* rc = M + bo;
    double* rs = rc + McLayout(a.vs).vs;
    const int lane = threadIdx.x & 63;
    const GraphRow grow0 = a.graph.row(a.items[base]);
    for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += gridDim.x * 4) {
        const GraphRow grow = a.graph.row(a.items[base + i]);
        double ds = 0.0;
        for (int j = lane; j < n; j += 64) ds += (double)mc_weight(a, base, i, j, grow, grow0);
        ds = wave_sum(ds);
        if (lane == 0) {
            const double d = (ds == 0.0 && a.mode == 0) ? 1.0 : ds;
            rs[i] = d;
            rc[i] = sqrt(1.0 / d);
        }
    }
}

// L2(i, j) = (s_i L(i, j)) s_j (:155) in fp64, A = sym_lower(L2) full symmetric column-major in
// the slot, sig_i = |L2(i, :)| (:169-177) to the slot, and (mode 1) the unsymmetrised fp32 L2
// for the w_lim pass
__global__ __launch_bounds__(256) void spill_mc_l2(McArgs a) {
    const uint32_t ui = blockIdx.y;
    const uint32_t unit = a.order[a.first + ui];
    const uint64_t base = a.item_off[unit];
    const int n = (int)(a.item_off[unit + 1] - base);
    double* M = mc_slot(a, ui);
    const uint64_t bo = spill_base_stride((uint64_t)n);
    const McLayout Lo(a.vs);
    const double* rc = M + bo;
    const double* rs = rc + Lo.vs;
    double* sig = M + bo + Lo.sig;
    float* L2out = a.mode == 1 ? a.l2 + a.l2_off[unit] : nullptr;
    const int lane = threadIdx.x & 63;
    const GraphRow grow0 = a.graph.row(a.items[base]);
    for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += gridDim.x * 4) {
        const GraphRow grow = a.graph.row(a.items[base + i]);
        const double si = rc[i], di = rs[i];
        double sq = 0.0;
        for (int j = lane; j < n; j += 64) {
            const double l = (j == i ? di : 0.0) - (double)mc_weight(a, base, i, j, grow, grow0);
            const double l2 = (si * l) * rc[j];
            sq += l2 * l2;
            if (L2out) L2out[(size_t)i * n + j] = (float)l2;
            if (j <= i) {
                M[(size_t)j * n + i] = l2;
                M[(size_t)i * n + j] = l2;
            }
        }
        sq = wave_sum(sq);
        if (lane == 0) sig[i] = (double)sqrtf((float)sq);
    }
}

// mode 3: B = L2 L2^T of the movie (the w_lim bisection's matrix, local_calc.cpp:425-435 with
// every row), exact fp32 x fp32 products summed in fp64 on v_mfma_f64_16x16x4_f64: one 64 x 64
// tile of the lower triangle per workgroup (4 waves of 32 x 32, 2 x 2 MFMA tiles each), the
// depth staged 16 columns at a time through LDS, the next chunk's loads in flight; the tile and
// its mirror go to the slot's column-major A.  grid = (lower tiles of the wave's kmax, units).
constexpr int MC_GRAM_LD = 68;
__global__ __launch_bounds__(256) void spill_mc_gram(McArgs a) {
    using f64x4 = __attribute__((ext_vector_type(4))) double;
    __shared__ double As[16 * MC_GRAM_LD], Bs[16 * MC_GRAM_LD];
    const uint32_t ui = blockIdx.y;
    const uint32_t unit = a.order[a.first + ui];
    const int n = (int)(a.item_off[unit + 1] - a.item_off[unit]);
    const int nt = (n + 63) >> 6;
    // lower-triangle tile t -> (ti, tj), tj <= ti
    const int t = blockIdx.x;
    int ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (ti * (ti + 1) / 2 > t) --ti;
    while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
    const int tj = t - ti * (ti + 1) / 2;
    if (ti >= nt) return;   // uniform: a smaller unit of the wave
    const float* L2m = a.l2 + a.l2_off[unit];
    double* M = mc_slot(a, ui);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int i0 = ti * 64, j0 = tj * 64;
    // staging: thread e loads rows (e >> 2) of both operands, depth 4 (e & 3) .. + 3
    const int sr = tid >> 2, sd = (tid & 3) * 4;
    const bool ra_ok = i0 + sr < n, rb_ok = j0 + sr < n;
    const float* pa = L2m + (size_t)(ra_ok ? i0 + sr : 0) * n;
    const float* pb = L2m + (size_t)(rb_ok ? j0 + sr : 0) * n;
    float fa[4], fb[4];
    auto fetch = [&](int l0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int l = l0 + sd + q;
            fa[q] = (ra_ok && l < n) ? pa[l] : 0.0f;
            fb[q] = (rb_ok && l < n) ? pb[l] : 0.0f;
        }
    };
    f64x4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
    const bool diag = ti == tj;
    fetch(0);
    for (int l0 = 0; l0 < n; l0 += 16) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            As[(sd + q) * MC_GRAM_LD + sr] = (double)fa[q];
            Bs[(sd + q) * MC_GRAM_LD + sr] = (double)fb[q];
        }
        __syncthreads();
        if (l0 + 16 < n) fetch(l0 + 16);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int row = (4 * ks + (lane >> 4)) * MC_GRAM_LD + (lane & 15);
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
                    if (!diag || 32 * wc + 16 * y <= 32 * wr + 16 * x)   // uniform: tiles above the diagonal skip
                        acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[x], bv[y], acc[x][y], 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int gi = i0 + 32 * wr + 16 * x + (lane >> 4) + 4 * q;
                const int gj = j0 + 32 * wc + 16 * y + (lane & 15);
                if (gi < n && gj < n && gj <= gi) {
                    M[(size_t)gj * n + gi] = acc[x][y][q];
                    M[(size_t)gi * n + gj] = acc[x][y][q];
                }
            }
}

}  // namespace

// Staged multi-CU path for BIG users [first, first + count) (plan positions, k non-increasing),
// `slots` users at a time: stage 1 (assembly) on eigen_spill_kernel, the tridiagonalisation on
// the spill_mc_* launches, then eigen_spill_kernel again for QL (stage 2, MC_QL_ROWS-row parts,
// each with its own copy of the serial generator), Z to row-major (stage 3) and the
// back-transform + output (stage 4, MC_BT_COLS-column parts).
// d / e of a HUGE launch's QL parts in LDS when they fit (CF_SPILL_HUGE_DE=global forces the
// slot copies, for tests of that path at sizes that would fit)
static bool huge_de_lds(uint64_t vs) {
    static const bool force_global = [] {
        const char* e = getenv("CF_SPILL_HUGE_DE");
        return e && std::string(e) == "global";
    }();
    return !force_global && vs <= kHugeDeLdsMax;
}

template <bool HUGE>
// Waves: [wave_start[w], wave_start[w + 1]) of the range's users; d_off holds, per user of the
// range, its slot's offset from the start of its wave's region (slots sized for the user's own k).
static int spill_mc_launch(cf_ctx* ctx, const cf_plan* plan, SpillArgs a, uint32_t first,
                           const std::vector<uint32_t>& wave_start, const uint64_t* d_off, uint32_t n_cu,
                           hipStream_t st) {
    constexpr int NL = HUGE ? 1 : CF_SPILL_MAX_K;
    const auto kern = eigen_spill_kernel<NL, true, HUGE>;
    a.de_lds = HUGE && huge_de_lds(a.vs);
    const size_t lds = HUGE ? huge_lds_bytes(a.vs, a.de_lds) : sizeof(SpillSmemT<CF_SPILL_MAX_K, true>);
    CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (size_t w = 0; w + 1 < wave_start.size(); ++w) {
        const uint32_t w0 = wave_start[w], cnt = wave_start[w + 1] - w0;
        a.first = first + w0;
        a.count = cnt;
        a.slot_off = d_off + w0;
        McArgs m{};
        m.order = a.order;
        m.first = a.first;
        m.count = cnt;
        m.item_off = a.item_off;
        m.work = a.work;
        m.slot_off = a.slot_off;
        m.vs = a.vs;
        m.items = a.items;
        m.graph = a.graph;
        m.mode = a.loc.mode;
        m.l2 = a.loc.l2;
        m.l2_off = a.loc.l2_off;
        // the largest k of this wave (plan order: the wave's first user)
        const uint32_t unit0 = plan->h_order[a.first];
        const uint32_t kmax = (uint32_t)(plan->h_item_off[unit0 + 1] - plan->h_item_off[unit0]);
        // assembly over every CU: B = L2 L2^T on the matrix cores (mode 3), else degrees then L2
        if (m.mode == 3) {
            const uint32_t nt = (kmax + 63) / 64;
            hipLaunchKernelGGL(spill_mc_gram, dim3(nt * (nt + 1) / 2, cnt), dim3(256), 0, st, m);
        } else {
            const uint32_t rb = std::max<uint32_t>(1, std::min<uint32_t>((kmax + 3) / 4, (8 * n_cu + cnt - 1) / cnt));
            hipLaunchKernelGGL(spill_mc_deg, dim3(rb, cnt), dim3(256), 0, st, m);
            hipLaunchKernelGGL(spill_mc_l2, dim3(rb, cnt), dim3(256), 0, st, m);
        }
        CF_HIP_CHECK(ctx, hipGetLastError());
        // ~4 workgroups per CU over the batch for the memory-bound products, at least 64 rows each
        m.G = (int)std::max<uint32_t>(1, std::min<uint32_t>((4 * n_cu + cnt - 1) / cnt, (kmax + 63) / 64));
        for (int p = 0; p < (int)kmax - 1; p += SP_NB) {
            const int jbmax = std::min(SP_NB, (int)kmax - 1 - p);
            for (int jj = 0; jj < jbmax; ++jj) {
                const int j = p + jj;
                hipLaunchKernelGGL(spill_mc_col, dim3(cnt), dim3(SP_T), 0, st, m, j, p);
                hipLaunchKernelGGL(spill_mc_symv<HUGE>, dim3(cnt * m.G), dim3(MC_SYMV_T), 0, st, m, j);
                hipLaunchKernelGGL(spill_mc_fin, dim3(cnt), dim3(SP_T), 0, st, m, j, p);
            }
            hipLaunchKernelGGL(spill_mc_trail, dim3(cnt * m.G), dim3(SP_T), 0, st, m, p);
            CF_HIP_CHECK(ctx, hipGetLastError());
        }
        hipLaunchKernelGGL(spill_mc_end, dim3((cnt + 63) / 64), dim3(64), 0, st, m);
        CF_HIP_CHECK(ctx, hipGetLastError());
        // QL on row parts, Z to row-major, back-transform + output on column parts: only as
        // many parts as fit the CUs in one round (each QL part repeats the serial generator, so
        // a batch that fills the GPU on its own users runs one part per user, and a second
        // round of parts would double the stage)
        const uint32_t fill = std::max<uint32_t>(1, n_cu / cnt);   // every part in the first round
        // (the back-transform's parts split columns, nothing is repeated: as many as its
        // columns give, claimed dynamically over the CUs)
        const uint32_t qcap = (kmax + MC_QL_ROWS - 1) / MC_QL_ROWS;
        const int parts[3] = {(int)std::min<uint32_t>(fill, qcap), 1, (int)((kmax + MC_BT_COLS - 1) / MC_BT_COLS)};
        // the CUs the uniform QL split leaves idle give the batch's largest users (its critical
        // path) one more part each -- still one round
        static const bool ql_extra = [] {
            const char* e = getenv("CF_SPILL_QL_EXTRA");
            return !(e && e[0] == '0');
        }();
        const uint32_t used = cnt * (uint32_t)parts[0];
        const uint32_t n2 = (ql_extra && (uint32_t)parts[0] < qcap && used < n_cu) ? std::min(cnt, n_cu - used) : 0;
        for (int s = 0; s < 3; ++s) {
            a.mc_stage = 2 + s;
            a.mc_parts = s == 0 ? parts[0] + 1 : parts[s];
            a.mc_parts_rest = parts[s];
            a.mc_n2 = s == 0 ? (int)n2 : 0;
            const uint32_t items = (uint32_t)a.mc_n2 * (uint32_t)a.mc_parts + (cnt - (uint32_t)a.mc_n2) * (uint32_t)parts[s];
            const uint32_t g = std::min<uint32_t>(items, n_cu);
            CF_HIP_CHECK(ctx, hipMemsetAsync(a.counter, 0, sizeof(unsigned int), st));
            hipLaunchKernelGGL(kern, dim3(g), dim3(SP_T), lds, st, a);
            CF_HIP_CHECK(ctx, hipGetLastError());
        }
    }
    return CF_OK;
}

// The spill bucket (users sorted by k, largest first) in k ranges, each launch with slots sized
// for its own largest k, so a few k = 5000 users (400 MB slots) no longer cap the number of
// workgroups for the many smaller ones: k > CF_SPILL_MAX_K (HUGE: local_calc's units only; every
// k-long vector in the slot) and (3072, 5000] (BIG layout; for whole units from mc_min = 1536
// on) one after the other on ctx->spill_side, beside (192, 3072] on `stream`.  The two side
// ranges share one workspace region (same stream, in order); the rest has its own.
int cf_launch_eigen_spill(cf_ctx* ctx, const cf_plan* plan, const cf_bucket& b, const uint64_t* d_item_off,
                          const uint32_t* d_items, const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs,
                          float* d_evals, float* d_evecs, hipStream_t stream, const cf_spill_local* loc,
                          bool defer_join) {
    if (b.count == 0) return CF_OK;
    // no k cap (compute_eigens users and local_calc's units alike): k > CF_SPILL_MAX_K takes
    // the HUGE layout on the staged multi-CU path
    int n_cu = 256;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, ctx->device);
    // k ranges over the bucket's plan positions (k non-increasing)
    enum Kind { kRest = 0, kBig = 1, kHuge = 2 };
    struct Range {
        uint32_t first, count, kmax;
        int kind;
    };
    std::vector<Range> rs;
    {
        // (finer ranges run one after the other lost more to each range's tail than their
        // smaller slots gained: 4.88 vs 4.12 s on the config-5 sample's k <= 3072 users)
        // compute_eigens: users above mc_min take the staged multi-CU path in the BIG layout.
        // Default 1536: on the config-5 sample's 292 users with 192 < k <= 3072 the spill group
        // eigen went 4.08 -> 1.24 s (cut 3072 -> 1536; 1024: 1.41 s; profiles/r04/c5_mc_cut/);
        // CF_SPILL_MC_MIN overrides (A/B)
        static const uint32_t mc_min = [] {
            const char* e = getenv("CF_SPILL_MC_MIN");
            const long v = e ? atol(e) : 1536L;
            return (uint32_t)std::max<long>(CF_MAX_K, std::min<long>(v, SP_NL));
        }();
        // every whole-unit mode (a user; local_calc's movie graph and its B = L2 L2^T) may take the
        // staged multi-CU path; the per-pair w_lim mode (its n is the pair's unrated rows) may not
        const bool unit_mode = !loc || loc->mode != 2;
        // HUGE from CF_SPILL_MAX_K on (CF_SPILL_HUGE_MIN lowers the cut, for tests that run the
        // HUGE layout against the BIG one on the same units: the arithmetic is the same)
        static const uint32_t huge_min = [] {
            const char* e = getenv("CF_SPILL_HUGE_MIN");
            const long v = e ? atol(e) : (long)CF_SPILL_MAX_K;
            return (uint32_t)std::max<long>(CF_MAX_K, std::min<long>(v, CF_SPILL_MAX_K));
        }();
        const uint32_t cuts[3] = {huge_min, unit_mode ? std::min(mc_min, huge_min) : std::min<uint32_t>(SP_NL, huge_min), 0u};
        const int kinds[3] = {kHuge, kBig, kRest};
        uint32_t j = b.first;
        const uint32_t end = b.first + b.count;
        auto kof = [&](uint32_t pos) {
            const uint32_t u = plan->h_order[pos];
            return (uint32_t)(plan->h_item_off[u + 1] - plan->h_item_off[u]);
        };
        for (int c = 0; c < 3 && j < end; ++c) {
            const uint32_t j0 = j;
            while (j < end && kof(j) > cuts[c]) ++j;
            if (j > j0) rs.push_back({j0, j - j0, kof(j0), kinds[c]});
        }
        if (j < end) rs.push_back({j, end - j, kof(j), kRest});   // (degenerate: k <= 0)
    }
    auto base_stride = [](uint64_t kmax) { return spill_base_stride(kmax); };
    // the k-long vector stride of a range's slots (McLayout): BIG keeps CF_SPILL_MAX_K, HUGE its
    // own kmax rounded to 64
    auto vs_of = [](const Range& r) -> uint64_t {
        return r.kind == kHuge ? ((uint64_t)r.kmax + 63) / 64 * 64 : (uint64_t)CF_SPILL_MAX_K;
    };
    // BIG users of compute_eigens take the staged multi-CU path (CF_SPILL_MC=0: the
    // single-workgroup kernel); their slots carry d, e, sig and the panel dot products too
    static const bool mc_env = [] {
        const char* e = getenv("CF_SPILL_MC");
        return !(e && e[0] == '0');
    }();
    const bool mc_on = mc_env && (!loc || loc->mode != 2);
    auto stride_of = [&](const Range& r) {
        const McLayout lo(vs_of(r));
        const uint64_t extra = r.kind == kHuge ? lo.extra_huge : r.kind == kBig ? (mc_on ? lo.extra_big : 3ull * lo.vs) : 0ull;
        return base_stride(r.kmax) + extra;
    };
    // workspace cap: three quarters of this context's share of the free HBM (>= 24 GB, but at
    // most half the share: cf_hbm_budget); the side ranges get 60 % of it.  Staged users hold a
    // slot sized for their own k for the whole launch, as many per wave as the side region
    // holds: one wave lets every QL generator run at once (r04: 9 waves of 56 400-MB slots for
    // C5's 10k users; r05 per-user slots: 2 waves at a half (72 GB), 1 at three quarters (96 GB),
    // 27.7 -> 24.7 s, profiles/r05/budget_*_u1.log).  A failed allocation halves the cap (more
    // waves / fewer slots) down to one slot per range.
    static const double budget_frac = [] {   // (A/B: CF_SPILL_BUDGET)
        const char* e = getenv("CF_SPILL_BUDGET");
        return e ? atof(e) : 0.75;
    }();
    uint64_t budget = cf_hbm_budget(ctx, ctx->spill_bytes, budget_frac, 24ull << 30);
    const bool has_side = !rs.empty() && rs.front().kind != kRest;
    const bool has_rest = !rs.empty() && rs.back().kind == kRest;
    std::vector<uint32_t> grid(rs.size());
    uint64_t side_bytes = 0, rest_bytes = 0;
    auto user_slot = [&](const Range& r, uint32_t pos) {   // bytes of a staged user's own slot
        const McLayout lo(vs_of(r));
        const uint64_t k = (uint64_t)(plan->h_item_off[plan->h_order[pos] + 1] - plan->h_item_off[plan->h_order[pos]]);
        return (spill_base_stride(k) + (r.kind == kHuge ? lo.extra_huge : lo.extra_big)) * sizeof(double);
    };
    for (;;) {
        side_bytes = rest_bytes = 0;
        bool minimal = true;
        for (size_t i = 0; i < rs.size(); ++i) {
            const uint64_t slot = stride_of(rs[i]) * sizeof(double);
            const bool side = rs[i].kind != kRest;
            const uint64_t share = side ? (has_rest ? budget / 5 * 3 : budget) : (has_side ? budget / 5 * 2 : budget);
            if (side && mc_on) {   // staged: the whole range if it fits, else the share (>= its largest slot)
                uint64_t all = 0;
                for (uint32_t j = 0; j < rs[i].count; ++j) all += user_slot(rs[i], rs[i].first + j);
                const uint64_t region = std::max<uint64_t>(user_slot(rs[i], rs[i].first), std::min<uint64_t>(all, share));
                side_bytes = std::max<uint64_t>(side_bytes, region);
                minimal = minimal && region == user_slot(rs[i], rs[i].first);
                continue;
            }
            uint32_t g = std::min<uint32_t>(rs[i].count, (uint32_t)n_cu);
            g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(g, share / slot));
            grid[i] = g;
            minimal = minimal && g == 1;
            if (side) side_bytes = std::max<uint64_t>(side_bytes, (uint64_t)g * slot);
            else rest_bytes = std::max<uint64_t>(rest_bytes, (uint64_t)g * slot);
        }
        const size_t need = 256 + side_bytes + rest_bytes;
        if (need <= ctx->spill_bytes) break;
        // the previous launches on either stream may still read the old workspace
        CF_HIP_CHECK(ctx, hipStreamSynchronize(stream));
        if (ctx->spill_side) CF_HIP_CHECK(ctx, hipStreamSynchronize(ctx->spill_side));
        if (ctx->d_spill) (void)hipFree(ctx->d_spill);
        ctx->d_spill = nullptr;
        ctx->spill_bytes = 0;
        if (hipMalloc(&ctx->d_spill, need) == hipSuccess) {
            ctx->spill_bytes = need;
            CF_HIP_CHECK(ctx, hipMemsetAsync(ctx->d_spill, 0, 256, stream));
            break;
        }
        (void)hipGetLastError();
        ctx->d_spill = nullptr;
        if (minimal) return cf_set_error(ctx, CF_ENOMEM, "spill workspace (" + std::to_string(need) + " bytes)");
        budget /= 2;
    }
    if (has_side && !ctx->spill_side) {
        CF_HIP_CHECK(ctx, hipStreamCreateWithFlags(&ctx->spill_side, hipStreamNonBlocking));
        for (hipEvent_t& e : ctx->spill_side_ev) CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // staged ranges: waves filled greedily up to the side region (largest k first), and per user
    // its slot's offset from its wave's start, for every staged range in one table, uploaded once
    // (the side stream orders the copy after the previous call's kernels; the pinned staging
    // buffer is rewritten only after its previous copy has completed)
    std::vector<std::vector<uint32_t>> waves(rs.size());
    std::vector<size_t> off_base(rs.size(), 0);
    std::vector<uint64_t> offs;
    if (mc_on)
        for (size_t i = 0; i < rs.size(); ++i) {
            if (rs[i].kind == kRest) continue;
            off_base[i] = offs.size();
            uint64_t cur = 0;
            waves[i].push_back(0);
            for (uint32_t j = 0; j < rs[i].count; ++j) {
                const uint64_t sz = user_slot(rs[i], rs[i].first + j);
                if (cur > 0 && cur + sz > side_bytes) {
                    waves[i].push_back(j);
                    cur = 0;
                }
                offs.push_back(cur / sizeof(double));
                cur += sz;
            }
            waves[i].push_back(rs[i].count);
            if (getenv("CF_SPILL_VERBOSE"))
                fprintf(stderr, "[spill] range %zu: %u users k %u..%u, %zu waves in a %.1f GB side region\n", i,
                        rs[i].count, (unsigned)(plan->h_item_off[plan->h_order[rs[i].first + rs[i].count - 1] + 1] -
                                                plan->h_item_off[plan->h_order[rs[i].first + rs[i].count - 1]]),
                        (unsigned)rs[i].kmax, waves[i].size() - 1, side_bytes / 1e9);
        }
    if (!offs.empty()) {
        const size_t bytes = offs.size() * sizeof(uint64_t);
        if (!ctx->spill_off_ev) CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&ctx->spill_off_ev, hipEventDisableTiming));
        else CF_HIP_CHECK(ctx, hipEventSynchronize(ctx->spill_off_ev));
        if (bytes > ctx->spill_off_bytes) {
            if (ctx->h_spill_off) (void)hipHostFree(ctx->h_spill_off);
            if (ctx->d_spill_off) {
                CF_HIP_CHECK(ctx, hipStreamSynchronize(ctx->spill_side));   // its kernels may still read it
                (void)hipFree(ctx->d_spill_off);
            }
            ctx->h_spill_off = nullptr;
            ctx->d_spill_off = nullptr;
            ctx->spill_off_bytes = 0;
            CF_HIP_CHECK(ctx, hipHostMalloc(&ctx->h_spill_off, bytes));
            CF_HIP_CHECK(ctx, hipMalloc(&ctx->d_spill_off, bytes));
            ctx->spill_off_bytes = bytes;
        }
        std::memcpy(ctx->h_spill_off, offs.data(), bytes);
    }
    char* ws = static_cast<char*>(ctx->d_spill);
    SpillArgs a{};
    a.order = plan->d_order;
    a.item_off = d_item_off;
    a.items = d_items;
    a.graph = graph_dev(ctx);
    a.n_items = ctx->n_items;
    a.evec_off = d_evec_off;
    a.m_out = d_m;
    a.sigs = d_sigs;
    a.evals = d_evals;
    a.evecs = d_evecs;
    if (loc) a.loc = *loc;
    a.mc_parts = 1;
    a.mc_parts_rest = 1;
    a.mc_n2 = 0;
    a.phase = ctx->spill_debug ? ctx->d_dbg : nullptr;   // counters of their own (cf_debug_spill)
    bool side_started = false;
    for (size_t i = 0; i < rs.size(); ++i) {
        const Range& r = rs[i];
        const bool side = r.kind != kRest;
        hipStream_t st = side ? ctx->spill_side : stream;
        if (side && !side_started) {   // the side stream starts where `stream` is
            CF_HIP_CHECK(ctx, hipEventRecord(ctx->spill_side_ev[0], stream));
            CF_HIP_CHECK(ctx, hipStreamWaitEvent(st, ctx->spill_side_ev[0], 0));
            side_started = true;
            if (!offs.empty()) {
                CF_HIP_CHECK(ctx, hipMemcpyAsync(ctx->d_spill_off, ctx->h_spill_off, offs.size() * sizeof(uint64_t),
                                                 hipMemcpyHostToDevice, st));
                CF_HIP_CHECK(ctx, hipEventRecord(ctx->spill_off_ev, st));
            }
        }
        a.first = r.first;
        a.count = r.count;
        a.counter = reinterpret_cast<unsigned int*>(ws) + (side ? 0 : 1);   // one claim counter per stream
        a.work = reinterpret_cast<double*>(ws + 256 + (side ? 0 : side_bytes));
        a.work_stride = stride_of(r);
        a.big_off = base_stride(r.kmax);
        a.vs = vs_of(r);
        a.de_lds = 0;
        if (side && mc_on) {
            const uint64_t* d_off = ctx->d_spill_off + off_base[i];
            if (r.kind == kHuge) CF_TRY(spill_mc_launch<true>(ctx, plan, a, r.first, waves[i], d_off, (uint32_t)n_cu, st));
            else CF_TRY(spill_mc_launch<false>(ctx, plan, a, r.first, waves[i], d_off, (uint32_t)n_cu, st));
        } else if (r.kind == kHuge) {   // one workgroup per unit, every vector in the slot
            CF_HIP_CHECK(ctx, hipMemsetAsync(a.counter, 0, sizeof(unsigned int), st));
            const size_t lds = huge_lds_bytes(a.vs, false);
            CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)eigen_spill_kernel<1, true, true>,
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL((eigen_spill_kernel<1, true, true>), dim3(grid[i]), dim3(SP_T), lds, st, a);
        } else if (r.kind == kBig) {
            CF_HIP_CHECK(ctx, hipMemsetAsync(a.counter, 0, sizeof(unsigned int), st));
            const size_t lds = sizeof(SpillSmemT<CF_SPILL_MAX_K, true>);
            CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)eigen_spill_kernel<CF_SPILL_MAX_K, true>,
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL((eigen_spill_kernel<CF_SPILL_MAX_K, true>), dim3(grid[i]), dim3(SP_T), lds, st, a);
        } else {
            CF_HIP_CHECK(ctx, hipMemsetAsync(a.counter, 0, sizeof(unsigned int), st));
            const size_t lds = sizeof(SpillSmemT<SP_NL, false>);
            CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)eigen_spill_kernel<SP_NL, false>,
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL((eigen_spill_kernel<SP_NL, false>), dim3(grid[i]), dim3(SP_T), lds, st, a);
        }
        CF_HIP_CHECK(ctx, hipGetLastError());
        if (side) {
            CF_HIP_CHECK(ctx, hipEventRecord(ctx->spill_side_ev[1], st));
            ctx->spill_side_pending = true;
        }
    }
    if (!defer_join) return cf_spill_join(ctx, stream);
    return CF_OK;
}

int cf_spill_join(cf_ctx* ctx, hipStream_t stream) {
    if (!ctx->spill_side_pending) return CF_OK;
    CF_HIP_CHECK(ctx, hipStreamWaitEvent(stream, ctx->spill_side_ev[1], 0));
    ctx->spill_side_pending = false;
    return CF_OK;
}

int cf_debug_spill(cf_ctx* ctx, int enable, uint64_t* out8) {
    if (!ctx) return CF_EINVAL;
    CF_TRY(set_device(ctx));
    if (enable) CF_TRY(cf_debug_counters(ctx));
    ctx->spill_debug = enable != 0;
    if (out8) {
        for (int i = 0; i < 8; ++i) out8[i] = 0;
        if (ctx->d_dbg) {
            CF_HIP_CHECK(ctx, hipDeviceSynchronize());
            CF_HIP_CHECK(ctx, hipMemcpy(out8, ctx->d_dbg, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
            CF_HIP_CHECK(ctx, hipMemset(ctx->d_dbg, 0, 8 * sizeof(uint64_t)));
        }
    }
    return CF_OK;
}
