// cf_eigen_tri.hip -- compute_eigens (precompute_local_threads.cpp:100-213) for k <= 192 by
// Householder tridiagonalisation + implicit QL, the algorithm class of Eigen's
// SelfAdjointEigenSolver (:164) and of the oracle (tred2 / tql2), restructured for the GPU:
//
//   A  tri_reduce_kernel   one workgroup per user, everything in LDS:
//        gather W_u, d_i (fp64, 0 -> 1 rule, :129-141), s_i = sqrt(1/d_i) (:149-153),
//        L2(i,j) = (s_i L(i,j)) s_j in fp64 (:155, bit-identical to the oracle), sig_min_i
//        with the reference's float accumulation (:169-177, bit-identical), A =
//        sym_lower(L2) in fp32, Householder reduction to tridiagonal T (fp32 storage,
//        fp64 reductions), accumulation of Q with A = Q T Q^T.  Writes diag/off-diag of T
//        (fp64), Q (fp32, into the user's own evecs slot), sigs and the cut smm.
//   B  tri_ql_kernel       one LANE per user: the tql2 recurrence on (diag, off) in fp64,
//        recording every iteration's rotation sequence (c, s) and its [l, m].  The
//        recurrence is serial per user, so the batch runs it 64 users per wave instead of
//        one lane per workgroup.
//   C  tri_apply_kernel    one workgroup per user: Q into LDS, the recorded rotations
//        applied in batches of 8 QL iterations per pass (each row streams through the 8
//        sweeps with 8 carried values: a lagged pipeline, one LDS read + write per
//        element per batch), then the record of cf_eigen.hip: ascending order, sign
//        convention sum_i v_ij >= 0, lim (:184-191), k x m row-major block, evals, m.
//
// Work: ~4/3 k^3 (reduction) + 4/3 k^3 (Q) + ~6 k^3 (rotations) flops, against ~29 k^3 for
// the one-sided Jacobi kernel at its measured 9.7 sweeps.  Measured (C2 mix, 20k users):
// 90 ms against the Jacobi kernel's 54 ms -- every phase of a Householder step is a short
// latency chain (matrix-vector partials, one-wave reflector, rank-2 update) separated by
// barriers, with one or two workgroups per CU, so the flop saving does not show yet; the
// Jacobi kernel stays the default (cf_set_eigen_method) and DESIGN.md lists the next steps.  A user whose QL record
// overflows its budget (never seen: the budget is 3k^2 rotations, tql2 takes ~k^2) is
// flagged and recomputed by the Jacobi kernel.

#include "cf_internal.h"

namespace {

constexpr int TR_T = 256;          // threads of kernels A and C
constexpr int TR_W = TR_T / 64;
constexpr int TR_Q = 8;            // QL iterations per application pass
constexpr int TR_NMAX = CF_MAX_K;

struct TriArgs {
    const uint32_t* order;     // plan order; this launch covers order[first .. first + count)
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
    double* dd;                // per entry: diagonal of T, then eigenvalues (B)
    double* ee;                // per entry: off-diagonal of T
    float* smm;                // per user (plan index - first): cut (:179-182)
    int* flag;                 // per user (plan index - first): 1 = QL record overflow
    float2* rot;               // rotation records of the chunk
    const uint64_t* rot_off;   // per plan index j: [start, end) at 2j, 2j + 1 (chunk-relative)
    int2* hdr;                 // [l, m] per QL iteration
    const uint64_t* hdr_off;   // per plan index j: [start, end) at 2j, 2j + 1
    int* n_iter;               // per user: QL iterations recorded
    uint32_t group_first;      // plan index of the group start (smm / flag / n_iter index base)
    unsigned long long* stats; // cf_debug_tri: {rotations, QL iterations, overflows, users}
};

template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// Wave sum in fp64, uniform result: DPP inside each 16-lane row (quad perms, half-row and
// row mirrors), then the four row sums through readlane.  ~8x shorter latency than the
// ds_bpermute chain of __shfl_xor on doubles.
__device__ __forceinline__ double wsum(double v) {
    v += dpp_d<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_d<0x141>(v);   // row_half_mirror
    v += dpp_d<0x140>(v);   // row_mirror
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const double r0 = __hiloint2double(__builtin_amdgcn_readlane(hi, 0), __builtin_amdgcn_readlane(lo, 0));
    const double r1 = __hiloint2double(__builtin_amdgcn_readlane(hi, 16), __builtin_amdgcn_readlane(lo, 16));
    const double r2 = __hiloint2double(__builtin_amdgcn_readlane(hi, 32), __builtin_amdgcn_readlane(lo, 32));
    const double r3 = __hiloint2double(__builtin_amdgcn_readlane(hi, 48), __builtin_amdgcn_readlane(lo, 48));
    return (r0 + r1) + (r2 + r3);
}

__host__ __device__ constexpr int tri_ld(int n) { return n | 1; }   // odd row stride: conflict-free columns

// ---- A: assembly + tridiagonalisation + Q ---------------------------------------------------
// 1024 threads.  A is row-major with a row stride LD = n rounded up to a multiple of 4 and
// = 4 (mod 64): float4 rows for the rank-2 updates (lanes over columns), and only 2-way
// bank conflicts for the thread-per-row passes of the assembly.  Matrix-vector products use
// the symmetry (A u)_c = sum_q A[q][c] u_q: thread (c, part) sums a quarter of the rows.
constexpr int TA_T = 1024;
constexpr int TA_W = TA_T / 64;
constexpr int TR_SLOTS = (TR_NMAX + TA_W - 1) / TA_W;   // matrix rows per wave (12)

__host__ __device__ constexpr int tri_lda(int n) {
    return ((n + 3) & ~3) + ((4 - (((n + 3) & ~3) & 63)) & 63);
}

__global__ __launch_bounds__(TA_T) void tri_reduce_kernel(TriArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t jj = blockIdx.x;
    const uint32_t u = a.order[a.first + jj];
    const uint64_t base = a.item_off[u];
    const int n = (int)(a.item_off[u + 1] - base);
    const uint32_t js = a.first + jj - a.group_first;   // index into the group's per-user arrays
    if (n <= 0) {
        if (tid == 0) {
            a.m_out[u] = 0;
            a.smm[js] = 0.0f;
        }
        return;
    }
    const int LD = tri_lda(n);
    unsigned long long tA0 = (a.stats && tid == 0) ? __builtin_amdgcn_s_memtime() : 0ull, tA1 = 0, tA2 = 0;
    float* A = reinterpret_cast<float*>(smem_raw);                     // n x LD
    double* vu = reinterpret_cast<double*>(A + (size_t)n * LD);        // u (fp64); d_i in assembly
    double* hh = vu + TR_NMAX;                                         // h_i
    double* part = hh + TR_NMAX;                                       // [4][TR_NMAX] partial sums
    double* vp = part;                                                 // s_i during the assembly
    // part + 4N: the second fp64 u buffer.  During the assembly part[0, N) holds s_i,
    // part + 2N the item ids and part + 3N the per-wave sig maxima.
    double* red = part + 3 * TR_NMAX;
    uint32_t* s_item = reinterpret_cast<uint32_t*>(part + 2 * TR_NMAX);

    for (int i = tid; i < n; i += TA_T) s_item[i] = a.items[base + i];
    __syncthreads();
    for (int i = wave; i < n; i += TA_W) {
        const GraphRow grow = a.graph.row(s_item[i]);
        for (int j = lane; j < n; j += 64) A[i * LD + j] = grow[s_item[j]];
    }
    __syncthreads();
    for (int i = tid; i < n; i += TA_T) {
        const float* row = A + i * LD;
        double d = 0.0;
        for (int j = 0; j < n; ++j) d += (double)row[j];
        if (d == 0.0) d = 1.0;                       // (:137-140)
        vu[i] = d;
        vp[i] = sqrt(1.0 / d);                       // (:149-153)
    }
    __syncthreads();
    float sig_i = 0.0f;
    for (int i = tid; i < n; i += TA_T) {
        float* row = A + i * LD;
        const double si = vp[i], di = vu[i];
        float acc = 0.0f;
        for (int j = 0; j < n; ++j) {
            const double l = (j == i ? di : 0.0) - (double)row[j];
            const double l2 = (si * l) * vp[j];      // (:155)
            acc = (float)((double)acc + l2 * l2);    // (:172-176)
        }
        sig_i = sqrtf(acc);
        a.sigs[base + i] = (float)((double)sig_i + 0.01);   // (:177)
        for (int j = 0; j <= i; ++j) {
            const double l = (j == i ? di : 0.0) - (double)row[j];
            row[j] = (float)((si * l) * vp[j]);
        }
    }
    {   // cut smm = float(max sig + 0.01) (:179-182)
        float mx = (tid < n) ? sig_i : 0.0f;
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        if (lane == 0) reinterpret_cast<float*>(red)[wave] = mx;
        __syncthreads();
        if (tid == 0) {
            float m = 0.0f;
            for (int w = 0; w < TA_W; ++w) m = fmaxf(m, reinterpret_cast<float*>(red)[w]);
            a.smm[js] = (float)((double)m + 0.01);
        }
    }
    for (int i = wave; i < n; i += TA_W)
        for (int j = i + 1 + lane; j < n; j += 64) A[i * LD + j] = A[j * LD + i];
    __syncthreads();

    // ---- Householder reduction with the matrix in registers -------------------------------
    // Row r lives in wave r % 16, slot r / 16; lane holds columns lane, lane + 64, lane + 128:
    // ra[j][t] = A[16 j + wave][lane + 64 t] (36 registers; 16 waves x 12 slots x 192 columns
    // cover k <= 192).  A step is then: per-wave partials of A u from registers (LDS 16 x 192),
    // one wave reduces them to w = p - K u, every wave applies the rank-2 update to its own
    // registers, and the owner wave of the next row forms the next reflector straight from its
    // registers.  Three barriers per step and no LDS round trip of the matrix.
    float ra[TR_SLOTS][3];
#pragma unroll
    for (int j = 0; j < TR_SLOTS; ++j)
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int r = 16 * j + wave, c = lane + 64 * t;
            ra[j][t] = (r < n && c < n) ? A[r * LD + c] : 0.0f;
        }
    __syncthreads();   // A (LDS) is dead from here: the region is reused below
    float* P = reinterpret_cast<float*>(smem_raw);        // [16][TR_NMAX] partial sums
    float* Ub = P + TA_W * TR_NMAX;                        // [2][TR_NMAX] reflectors (fp32)
    float* Wv = Ub + 2 * TR_NMAX;                          // [TR_NMAX] w / t
    double* hh2 = reinterpret_cast<double*>(Wv + TR_NMAX); // [TR_NMAX] h_i
    double* Kw = hh2 + TR_NMAX;                            // [TA_W] per-wave u^T A u
    double* e2 = Kw + TA_W;                                // [TR_NMAX] off-diagonal of T
    // The reflector rows go to the evecs slot (global) and are read back for Q.  (Keeping them
    // packed in LDS failed the k = 15/16 parity cases and was not faster; not pursued.)
    double* dd = a.dd + base;
    double* ee = a.ee + base;
    float* slot = a.evecs + a.evec_off[u];
    if (a.stats && tid == 0) tA1 = __builtin_amdgcn_s_memtime();
    // reflector of row i by its owner wave: u (fp32, zero beyond i) into Ub[i & 1], the
    // reflector row into the evecs slot (for Q), h_i = |u|^2 / 2 of the rounded u, e_i
    auto reflector = [&](int i) {
        const int ji = i >> 4;
        double x[3];
        double sa = 0.0, sq = 0.0;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            float v = 0.0f;
#pragma unroll
            for (int j = 0; j < TR_SLOTS; ++j) v = (j == ji) ? ra[j][t] : v;
            const int c = lane + 64 * t;
            x[t] = c < i ? (double)v : 0.0;
            sa += fabs(x[t]);
            sq += x[t] * x[t];
        }
        const double scale = wsum(sa);
        const double ssq = wsum(sq);
        float* ub = Ub + (i & 1) * TR_NMAX;
        if (scale == 0.0) {
#pragma unroll
            for (int t = 0; t < 3; ++t) ub[lane + 64 * t] = 0.0f;
            if (lane == 0) {
                e2[i] = 0.0;
                hh2[i] = 0.0;
            }
            return;
        }
        const double inv = 1.0 / scale;
        const double hn = ssq * inv * inv;
        double xf = x[0];
        if (((i - 1) >> 6) == 1) xf = x[1];
        if (((i - 1) >> 6) == 2) xf = x[2];
        const double f = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(xf), (i - 1) & 63),
                                          __builtin_amdgcn_readlane(__double2loint(xf), (i - 1) & 63)) * inv;
        const double g = f > 0 ? -sqrt(hn) : sqrt(hn);
        double uu = 0.0;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int c = lane + 64 * t;
            float uf_ = 0.0f;
            if (c < i) uf_ = (float)(c == i - 1 ? f - g : x[t] * inv);
            ub[c] = uf_;
            uu += (double)uf_ * (double)uf_;
            if (c < i) slot[i * n + c] = uf_;
        }
        const double h = 0.5 * wsum(uu);
        if (lane == 0) {
            e2[i] = scale * g;
            hh2[i] = h;
        }
    };
    if (n > 1 && wave == ((n - 1) & (TA_W - 1))) reflector(n - 1);
    __syncthreads();
    for (int i = n - 1; i > 0; --i) {
        const double h = hh2[i];
        const float* ub = Ub + (i & 1) * TR_NMAX;
        if (h != 0.0) {
            // (1) per-wave partials of (A u)_c over this wave's rows, and the wave's share of
            // u^T A u (so that K needs no second reduction)
            float acc[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < TR_SLOTS; ++j) {
                const float ur = ub[16 * j + wave];
#pragma unroll
                for (int t = 0; t < 3; ++t) acc[t] = fmaf(ra[j][t], ur, acc[t]);
            }
            double kw = 0.0;
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                P[wave * TR_NMAX + lane + 64 * t] = acc[t];
                kw += (double)acc[t] * (double)ub[lane + 64 * t];
            }
            kw = wsum(kw);
            if (lane == 0) Kw[wave] = kw;
            __syncthreads();
            // (2) p = (A u) / h, K = u^T A u / 2h^2, w = p - K u (zero beyond i)
            if (tid < TR_NMAX) {
                double sum = 0.0, ks = 0.0;
#pragma unroll
                for (int w = 0; w < TA_W; ++w) {
                    sum += (double)P[w * TR_NMAX + tid];
                    ks += Kw[w];
                }
                const double K = ks / (2.0 * h * h);
                Wv[tid] = tid < i ? (float)(sum / h - K * (double)ub[tid]) : 0.0f;
            }
            __syncthreads();
            // (3) rank-2 update of this wave's rows
            float uc[3], wc[3];
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                uc[t] = ub[lane + 64 * t];
                wc[t] = Wv[lane + 64 * t];
            }
#pragma unroll
            for (int j = 0; j < TR_SLOTS; ++j) {
                const float ur = ub[16 * j + wave], wr = Wv[16 * j + wave];
#pragma unroll
                for (int t = 0; t < 3; ++t) ra[j][t] -= ur * wc[t] + wr * uc[t];
            }
        }
        if (i > 1 && wave == ((i - 1) & (TA_W - 1))) reflector(i - 1);
        __syncthreads();
    }
    // diagonal of T from the owners' registers
#pragma unroll
    for (int j = 0; j < TR_SLOTS; ++j)
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int r = 16 * j + wave, c = lane + 64 * t;
            if (r == c && r < n) dd[r] = (double)ra[j][t];
        }
    if (tid == 0) {
        e2[0] = 0.0;
        hh2[0] = 0.0;
    }
    if (a.stats && tid == 0) tA2 = __builtin_amdgcn_s_memtime();
    // ---- Q = H_{n-1} ... H_1 in registers (same distribution) ---------------------------------
#pragma unroll
    for (int j = 0; j < TR_SLOTS; ++j)
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int r = 16 * j + wave, c = lane + 64 * t;
            ra[j][t] = (r == c && r < n) ? 1.0f : 0.0f;
        }
    __syncthreads();   // e2, hh2 and the reflector rows visible
    for (int q = tid; q < n; q += TA_T) ee[q] = e2[q];
    if (n > 1 && tid < TR_NMAX) Ub[TR_NMAX + tid] = tid < 1 ? slot[1 * n + tid] : 0.0f;
    __syncthreads();
    for (int i = 1; i < n; ++i) {
        const double h = hh2[i];
        const float* ub = Ub + (i & 1) * TR_NMAX;
        const float unext = (i + 1 < n && tid < i + 1) ? slot[(i + 1) * n + tid] : 0.0f;
        if (h != 0.0) {
            float acc[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < TR_SLOTS; ++j) {
                const float ur = ub[16 * j + wave];
#pragma unroll
                for (int t = 0; t < 3; ++t) acc[t] = fmaf(ur, ra[j][t], acc[t]);
            }
#pragma unroll
            for (int t = 0; t < 3; ++t) P[wave * TR_NMAX + lane + 64 * t] = acc[t];
            __syncthreads();
            if (tid < TR_NMAX) {
                double sum = 0.0;
#pragma unroll
                for (int w = 0; w < TA_W; ++w) sum += (double)P[w * TR_NMAX + tid];
                Wv[tid] = (float)(sum / h);
            }
            __syncthreads();
            float tc[3];
#pragma unroll
            for (int t = 0; t < 3; ++t) tc[t] = Wv[lane + 64 * t];
#pragma unroll
            for (int j = 0; j < TR_SLOTS; ++j) {
                const float ur = ub[16 * j + wave];
#pragma unroll
                for (int t = 0; t < 3; ++t) ra[j][t] -= ur * tc[t];
            }
        }
        if (i + 1 < n && tid < TR_NMAX) Ub[((i + 1) & 1) * TR_NMAX + tid] = unext;
        __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < TR_SLOTS; ++j)
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int r = 16 * j + wave, c = lane + 64 * t;
            if (r < n && c < n) slot[r * n + c] = ra[j][t];
        }
    if (a.stats && tid == 0) {
        const unsigned long long t3 = __builtin_amdgcn_s_memtime();
        atomicAdd(&a.stats[4], tA1 - tA0);
        atomicAdd(&a.stats[5], tA2 - tA1);
        atomicAdd(&a.stats[6], t3 - tA2);
        atomicAdd(&a.stats[7], (unsigned long long)n);
    }
}

// ---- B: batched tql2 with rotation recording (one lane per user) ------------------------------
// d and e live in LDS, interleaved by lane ([i][lane]) so the lanes' same-index accesses are
// conflict-free.  JAMA's per-iteration shift d[i] -= h (i >= l + 2) is kept lazy: those
// entries are stored as d + f (f = the accumulated shift) and read as stored - f.
__global__ __launch_bounds__(64) void tri_ql_kernel(TriArgs a, int ub, int kmax) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    double* D = reinterpret_cast<double*>(smem_raw);   // [kmax][ub]
    double* E = D + (size_t)kmax * ub;
    const int lane = threadIdx.x;
    const uint32_t jj = blockIdx.x * ub + lane;   // group launch: first == group_first
    const bool act = lane < ub && jj < a.count;
    if (!act) return;
    const uint32_t u = a.order[a.first + jj];
    const uint64_t base = a.item_off[u];
    const int n = (int)(a.item_off[u + 1] - base);
    if (n <= 0) {
        a.flag[jj] = 0;
        a.n_iter[jj] = 0;
        return;
    }
    auto dR = [&](int i) -> double& { return D[(size_t)i * ub + lane]; };
    auto eR = [&](int i) -> double& { return E[(size_t)i * ub + lane]; };
    const double* gd = a.dd + base;
    const double* ge = a.ee + base;
    for (int i = 0; i < n; ++i) {
        dR(i) = gd[i];
        eR(i) = (i + 1 < n) ? ge[i + 1] : 0.0;   // tql2 entry shift e[i-1] = e[i]
    }
    const size_t pj = 2 * (size_t)(a.first + jj);
    float2* rot = a.rot + a.rot_off[pj];
    const uint64_t rot_cap = a.rot_off[pj + 1] - a.rot_off[pj];
    int2* hdr = a.hdr + a.hdr_off[pj];
    const uint64_t hdr_cap = a.hdr_off[pj + 1] - a.hdr_off[pj];
    uint64_t nrot = 0, nh = 0;
    bool overflow = false;
    double f = 0.0, tst1 = 0.0;   // f: JAMA's accumulated shift; D[i >= l+2] hold d + f
    const double eps = 2.220446049250313e-16;
    // entries are stored "lazy" (d + f) from the start (f = 0)
    for (int l = 0; l < n && !overflow; ++l) {
        // materialise d[l], d[l+1] (explicit while l is current)
        dR(l) -= f;
        if (l + 1 < n) dR(l + 1) -= f;
        tst1 = fmax(tst1, fabs(dR(l)) + fabs(eR(l)));
        int m = l;
        while (m < n && !(fabs(eR(m)) <= eps * tst1)) ++m;
        if (m > l) {
            int iter = 0;
            do {
                ++iter;
                if (nh >= hdr_cap || nrot + (uint64_t)(m - l) > rot_cap) {
                    overflow = true;
                    break;
                }
                const double g0 = dR(l);
                const double el = eR(l);
                double p = (dR(l + 1) - g0) / (2.0 * el);
                double r = sqrt(p * p + 1.0);
                if (p < 0) r = -r;
                const double dl = el / (p + r);
                dR(l) = dl;
                dR(l + 1) = el * (p + r);
                const double dl1 = dR(l + 1);
                const double h0 = g0 - dl;
                f += h0;   // d[i >= l+2] -= h0, lazily
                // d_at(i): explicit for i <= l+1, stored - f beyond
                p = (m >= l + 2) ? dR(m) - f : dR(m);
                double c = 1.0, c2 = 1.0, c3 = 1.0, s = 0.0, s2 = 0.0;
                const double el1 = eR(l + 1);
                for (int i = m - 1; i >= l; --i) {
                    const double ei = eR(i);
                    const double di = (i >= l + 2) ? dR(i) - f : dR(i);
                    c3 = c2;
                    c2 = c;
                    s2 = s;
                    const double g = c * ei;
                    const double h = c * p;
                    r = sqrt(p * p + ei * ei);
                    eR(i + 1) = s * r;
                    const double ri = 1.0 / r;
                    s = ei * ri;
                    c = p * ri;
                    p = c * di - s * g;
                    const double dn = h + s * (c * g + s * di);
                    dR(i + 1) = (i + 1 >= l + 2) ? dn + f : dn;
                    rot[nrot + (m - 1 - i)] = make_float2((float)c, (float)s);
                }
                hdr[nh++] = make_int2(l, m);
                nrot += (uint64_t)(m - l);
                p = -s * s2 * c3 * el1 * eR(l) / dl1;
                eR(l) = s * p;
                dR(l) = c * p;
            } while (fabs(eR(l)) > eps * tst1 && iter < 60);
        }
        dR(l) += f;   // eigenvalue l (JAMA: d[l] += f)
        eR(l) = 0.0;
        // d[l+1] goes back to lazy storage for the next l? It becomes the new d[l]
        // (explicit) -- re-lazify it so the materialisation at the loop head is uniform.
        if (l + 1 < n) dR(l + 1) += f;
    }
    double* od = a.dd + base;
    for (int i = 0; i < n; ++i) od[i] = dR(i);
    a.flag[jj] = overflow ? 1 : 0;
    a.n_iter[jj] = (int)nh;
    if (a.stats) {
        atomicAdd(&a.stats[0], (unsigned long long)nrot);
        atomicAdd(&a.stats[1], (unsigned long long)nh);
        atomicAdd(&a.stats[2], overflow ? 1ull : 0ull);
        atomicAdd(&a.stats[3], 1ull);
    }
}

// ---- C: rotations applied to Q, ordering, output ---------------------------------------------
__global__ __launch_bounds__(TR_T) void tri_apply_kernel(TriArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t jj = blockIdx.x;
    const uint32_t u = a.order[a.first + jj];
    const uint64_t base = a.item_off[u];
    const int n = (int)(a.item_off[u + 1] - base);
    const uint32_t js = a.first + jj - a.group_first;
    if (n <= 0 || a.flag[js]) return;
    const int LD = tri_ld(n);
    float* V = reinterpret_cast<float*>(smem_raw);                       // n x LD
    float2* cs = reinterpret_cast<float2*>(V + ((n * LD + 1) & ~1));    // [TR_Q][TR_NMAX]
    double* ev = reinterpret_cast<double*>(cs + TR_Q * TR_NMAX);        // eigenvalues
    int* perm = reinterpret_cast<int*>(ev + TR_NMAX);
    float* sgn = reinterpret_cast<float*>(perm + TR_NMAX);
    int* sh = reinterpret_cast<int*>(sgn + TR_NMAX);                    // [2 * TR_Q + 4]
    float* slot = a.evecs + a.evec_off[u];
    for (int i = wave; i < n; i += TR_W)
        for (int j = lane; j < n; j += 64) V[i * LD + j] = slot[i * n + j];
    for (int i = tid; i < n; i += TR_T) ev[i] = a.dd[base + i];
    const float2* rot = a.rot + a.rot_off[2 * (size_t)(a.first + jj)];
    const int2* hdr = a.hdr + a.hdr_off[2 * (size_t)(a.first + jj)];
    const int n_it = a.n_iter[js];
    uint64_t rpos = 0;
    for (int b0 = 0; b0 < n_it; b0 += TR_Q) {
        const int nseq = min(TR_Q, n_it - b0);
        __syncthreads();   // previous batch done with cs / sh
        if (tid < nseq) {
            const int2 lm = hdr[b0 + tid];
            sh[tid] = lm.x;
            sh[TR_Q + tid] = lm.y;
        }
        __syncthreads();
        int L = n, Mx = 0;
        uint64_t offs[TR_Q];
        {
            uint64_t off = rpos;
#pragma unroll
            for (int t = 0; t < TR_Q; ++t) {
                offs[t] = off;
                if (t < nseq) {
                    L = min(L, sh[t]);
                    Mx = max(Mx, sh[TR_Q + t]);
                    off += (uint64_t)(sh[TR_Q + t] - sh[t]);
                }
            }
            rpos = off;
        }
        // stage [t][pp]: rotation of sequence t at position pp, identity outside [l_t, m_t);
        // all 8 loads of a thread are issued before the LDS stores
        for (int pp = tid; pp < n; pp += TR_T) {
            float2 v[TR_Q];
#pragma unroll
            for (int t = 0; t < TR_Q; ++t) {
                const int l = t < nseq ? sh[t] : 0, m = t < nseq ? sh[TR_Q + t] : 0;
                v[t] = (pp >= l && pp < m) ? rot[offs[t] + (m - 1 - pp)] : make_float2(1.0f, 0.0f);
            }
#pragma unroll
            for (int t = 0; t < TR_Q; ++t) cs[t * TR_NMAX + pp] = v[t];
        }
        __syncthreads();
        const int r = tid;
        if (r < n) {
            float* row = V + r * LD;
            float carry[TR_Q];
            carry[0] = row[Mx];
#pragma unroll
            for (int t = 1; t < TR_Q; ++t) carry[t] = 0.0f;
            int tau = Mx - 1;
            // head: sequences t >= 1 pick up their first carry (pp == Mx)
            for (; tau >= L && tau > Mx - nseq; --tau) {
                float val = row[tau];
                bool ok = true;
#pragma unroll
                for (int t = 0; t < TR_Q; ++t) {
                    if (t < nseq) {
                        const int pp = tau + t;
                        if (pp > Mx) {
                            ok = false;
                        } else if (pp == Mx) {
                            if (ok) carry[t] = val;
                            ok = false;
                        } else {
                            const float2 q = cs[t * TR_NMAX + pp];
                            const float out = q.y * val + q.x * carry[t];
                            carry[t] = q.x * val - q.y * carry[t];
                            val = out;
                        }
                    }
                }
                if (ok) row[tau + nseq] = val;
            }
            // interior: every sequence rotates (L <= tau, tau + nseq - 1 < Mx)
            if (nseq == TR_Q) {
                // 4 positions per iteration: rotation (tau, t) depends on (tau, t-1) and
                // (tau+1, t) only, so the unrolled block runs as a wavefront
                for (; tau - 3 >= L; tau -= 4) {
                    float2 q[4][TR_Q];
                    float x[4];
#pragma unroll
                    for (int s4 = 0; s4 < 4; ++s4) {
                        x[s4] = row[tau - s4];
#pragma unroll
                        for (int t = 0; t < TR_Q; ++t) q[s4][t] = cs[t * TR_NMAX + tau - s4 + t];
                    }
#pragma unroll
                    for (int s4 = 0; s4 < 4; ++s4) {
                        float val = x[s4];
#pragma unroll
                        for (int t = 0; t < TR_Q; ++t) {
                            const float out = q[s4][t].y * val + q[s4][t].x * carry[t];
                            carry[t] = q[s4][t].x * val - q[s4][t].y * carry[t];
                            val = out;
                        }
                        row[tau - s4 + TR_Q] = val;
                    }
                }
                for (; tau >= L; --tau) {
                    float val = row[tau];
#pragma unroll
                    for (int t = 0; t < TR_Q; ++t) {
                        const float2 q = cs[t * TR_NMAX + tau + t];
                        const float out = q.y * val + q.x * carry[t];
                        carry[t] = q.x * val - q.y * carry[t];
                        val = out;
                    }
                    row[tau + TR_Q] = val;
                }
            } else {
                for (; tau >= L; --tau) {
                    float val = row[tau];
#pragma unroll
                    for (int t = 0; t < TR_Q; ++t) {
                        if (t < nseq) {
                            const float2 q = cs[t * TR_NMAX + tau + t];
                            const float out = q.y * val + q.x * carry[t];
                            carry[t] = q.x * val - q.y * carry[t];
                            val = out;
                        }
                    }
                    row[tau + nseq] = val;
                }
            }
            // tail: flush (pp == L - 1 emits the carry), tau = L-1 .. L-nseq
            for (; tau >= L - nseq; --tau) {
                float val = 0.0f;
                bool ok = false;
#pragma unroll
                for (int t = 0; t < TR_Q; ++t) {
                    if (t < nseq) {
                        const int pp = tau + t;
                        if (pp > Mx) {
                            ok = false;
                        } else if (pp == Mx) {
                            if (ok) carry[t] = val;
                            ok = false;
                        } else if (pp >= L) {
                            const float2 q = cs[t * TR_NMAX + pp];
                            const float out = q.y * val + q.x * carry[t];
                            carry[t] = q.x * val - q.y * carry[t];
                            val = out;
                        } else if (pp == L - 1) {
                            val = carry[t];
                            ok = true;
                        } else {
                            ok = false;
                        }
                    }
                }
                if (ok) row[tau + nseq] = val;
            }
        }
    }
    __syncthreads();
    // ascending order of the eigenvalues (ties by index), signs, lim, output
    for (int j = tid; j < n; j += TR_T) {
        const double lj = ev[j];
        int rank = 0;
        double s = 0.0;
        for (int i = 0; i < n; ++i) {
            const double li = ev[i];
            rank += (li < lj) || (li == lj && i < j);
            s += (double)V[i * LD + j];
        }
        perm[rank] = j;
        sgn[j] = s < 0.0 ? -1.0f : 1.0f;
    }
    __syncthreads();
    if (tid == 0) {
        const float smm = a.smm[js];
        int lim;
        for (lim = 0; lim < n; ++lim)
            if (ev[perm[lim]] > (double)smm) break;   // (:186-188)
        if (lim < 2) lim = 2;                          // (:190-191)
        sh[2 * TR_Q] = lim;
        a.m_out[u] = lim;
    }
    __syncthreads();
    const int m = sh[2 * TR_Q];
    for (int r = tid; r < m && r < n; r += TR_T) a.evals[base + r] = (float)ev[perm[r]];
    for (int i = wave; i < n; i += TR_W)
        for (int r = lane; r < m; r += 64) {
            float v = 0.0f;
            if (r < n) {
                const int j = perm[r];
                v = V[i * LD + j] * sgn[j];
            }
            slot[i * m + r] = v;
        }
}

size_t tri_lds_a(int kmax) {
    const size_t assembly = sizeof(float) * (size_t)kmax * tri_lda(kmax) + sizeof(double) * 7 * TR_NMAX +
                            sizeof(float) * 3 * TR_NMAX;
    const size_t reduction = sizeof(float) * (TA_W + 3) * TR_NMAX + sizeof(double) * TR_NMAX;
    return std::max(assembly, reduction);
}
size_t tri_lds_c(int kmax) {
    return sizeof(float) * (size_t)((kmax * tri_ld(kmax) + 1) & ~1) + sizeof(float2) * TR_Q * TR_NMAX +
           sizeof(double) * TR_NMAX + sizeof(int) * TR_NMAX + sizeof(float) * TR_NMAX + sizeof(int) * (2 * TR_Q + 4);
}
// kernel B: users per 64-lane block so that D and E ([kmax][ub] fp64 each) fit 150 KB
int tri_ql_ub(int kmax) { return std::max(1, std::min(64, (int)(150 * 1024 / (16 * std::max(kmax, 1))))); }

}  // namespace

// Rotation-record budget per user (float2 units) and header budget (QL iterations).
static inline uint64_t tri_rot_cap(uint64_t k) { return (3 * k * k) / 2 + 64; }
static inline uint64_t tri_hdr_cap(uint64_t k) { return 3 * k + 16; }

int cf_tri_prepare(cf_ctx* ctx, cf_plan* plan, const uint64_t* item_off) {
    // Groups: plan-order ranges (across LDS buckets) whose QL records fit the budget; kernel
    // B runs once per group.  Parts: a group's sub-range inside one bucket (kernels A, C and
    // the Jacobi fallback are per bucket).  Per plan index j: [start, end) of its records,
    // group-relative, at 2j and 2j + 1.
    const uint64_t budget = (uint64_t)8 << 30;   // bytes of rotation records per group
    plan->tri_chunks.clear();
    plan->tri_groups.clear();
    plan->n_entries = plan->n_users ? item_off[plan->n_users] : 0;
    std::vector<uint64_t> r2(2 * (size_t)plan->n_users + 2, 0), h2(2 * (size_t)plan->n_users + 2, 0);
    uint64_t acc = 0, acch = 0;
    bool open = false;
    for (const cf_bucket& b : plan->buckets) {
        if (b.emax == kSpillBucket || b.count == 0) continue;
        uint32_t start = b.first;
        open = false;   // a group never spans buckets (cf_launch_eigen_tri's emax_min runs whole groups)
        for (uint32_t j = b.first; j < b.first + b.count; ++j) {
            const uint32_t u = plan->h_order[j];
            const uint64_t k = item_off[u + 1] - item_off[u];
            const uint64_t rc = tri_rot_cap(k), hc = tri_hdr_cap(k);
            if (!open || (acc + rc) * sizeof(float2) > budget) {
                if (open && j > start) {
                    plan->tri_chunks.push_back({b.emax, start, j - start, b.kmax, (uint32_t)plan->tri_groups.size() - 1});
                    start = j;
                }
                plan->tri_groups.push_back({j, 0, 0});
                acc = 0;
                acch = 0;
                open = true;
            }
            cf_tri_group& g = plan->tri_groups.back();
            g.count = j + 1 - g.first;
            g.kmax = std::max<uint32_t>(g.kmax, (uint32_t)k);
            r2[2 * (size_t)j] = acc;
            h2[2 * (size_t)j] = acch;
            acc += rc;
            acch += hc;
            r2[2 * (size_t)j + 1] = acc;
            h2[2 * (size_t)j + 1] = acch;
            plan->tri_rot_max = std::max(plan->tri_rot_max, acc);
            plan->tri_hdr_max = std::max(plan->tri_hdr_max, acch);
        }
        plan->tri_chunks.push_back({b.emax, start, b.first + b.count - start, b.kmax,
                                    (uint32_t)plan->tri_groups.size() - 1});
    }
    for (const auto& g : plan->tri_groups) plan->tri_users_max = std::max(plan->tri_users_max, g.count);
    if (plan->n_users) {
        CF_HIP_CHECK(ctx, hipMalloc(&plan->d_tri_roff, sizeof(uint64_t) * r2.size()));
        CF_HIP_CHECK(ctx, hipMalloc(&plan->d_tri_hoff, sizeof(uint64_t) * h2.size()));
        CF_HIP_CHECK(ctx, hipMemcpy(plan->d_tri_roff, r2.data(), sizeof(uint64_t) * r2.size(), hipMemcpyHostToDevice));
        CF_HIP_CHECK(ctx, hipMemcpy(plan->d_tri_hoff, h2.data(), sizeof(uint64_t) * h2.size(), hipMemcpyHostToDevice));
    }
    return CF_OK;
}

static int tri_scratch(cf_ctx* ctx, const cf_plan* plan, TriArgs& a) {
    const size_t ne = std::max<uint64_t>(plan->n_entries, 1), nu = std::max<uint32_t>(plan->tri_users_max, 1);
    const size_t need = 2 * ne * sizeof(double) + nu * (sizeof(float) + 2 * sizeof(int)) + 256 +
                        (plan->tri_rot_max + 1) * sizeof(float2) + (plan->tri_hdr_max + 1) * sizeof(int2) +
                        8 * sizeof(unsigned long long);
    if (need > ctx->tri_bytes) {
        if (ctx->d_tri) (void)hipFree(ctx->d_tri);
        ctx->d_tri = nullptr;
        ctx->tri_bytes = 0;
        CF_TRY(cf_malloc_evict(ctx, &ctx->d_tri, need, "tridiagonal eigen scratch"));
        ctx->tri_bytes = need;
    }
    char* p = static_cast<char*>(ctx->d_tri);
    a.stats = ctx->tri_debug ? ctx->d_dbg + 8 : nullptr;   // counters of their own (cf_debug_tri)
    p += 8 * sizeof(unsigned long long);
    a.dd = reinterpret_cast<double*>(p);
    p += ne * sizeof(double);
    a.ee = reinterpret_cast<double*>(p);
    p += ne * sizeof(double);
    a.rot = reinterpret_cast<float2*>(p);
    p += (plan->tri_rot_max + 1) * sizeof(float2);
    a.hdr = reinterpret_cast<int2*>(p);
    p += (plan->tri_hdr_max + 1) * sizeof(int2);
    a.smm = reinterpret_cast<float*>(p);
    p += nu * sizeof(float);
    a.flag = reinterpret_cast<int*>(p);
    p += nu * sizeof(int);
    a.n_iter = reinterpret_cast<int*>(p);
    return CF_OK;
}

int cf_launch_eigen_tri(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items,
                        const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs, float* d_evals, float* d_evecs,
                        hipStream_t stream, int emax_min) {
    if (plan->tri_groups.empty()) return CF_OK;
    TriArgs a{};
    CF_TRY(tri_scratch(ctx, plan, a));
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
    a.rot_off = plan->d_tri_roff;
    a.hdr_off = plan->d_tri_hoff;
    static bool configured = false;
    if (!configured) {
        CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)tri_reduce_kernel,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)tri_lds_a(TR_NMAX)));
        CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)tri_apply_kernel,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)tri_lds_c(TR_NMAX)));
        CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)tri_ql_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                              150 * 1024));
        configured = true;
    }
    for (uint32_t gi = 0; gi < plan->tri_groups.size(); ++gi) {
        const cf_tri_group& g = plan->tri_groups[gi];
        bool wanted = false;   // groups lie inside one bucket: its chunks share one emax
        for (const cf_tri_chunk& c : plan->tri_chunks)
            if (c.group == gi) wanted = c.emax >= emax_min;
        if (!wanted) continue;
        a.group_first = g.first;
        for (const cf_tri_chunk& c : plan->tri_chunks) {
            if (c.group != gi) continue;
            a.first = c.first;
            a.count = c.count;
            hipLaunchKernelGGL(tri_reduce_kernel, dim3(c.count), dim3(TA_T), tri_lds_a(std::max<int>(1, c.kmax)),
                               stream, a);
            CF_HIP_CHECK(ctx, hipGetLastError());
        }
        a.first = g.first;
        a.count = g.count;
        const int kmax = std::max<int>(1, (int)g.kmax);
        const int ub = tri_ql_ub(kmax);
        hipLaunchKernelGGL(tri_ql_kernel, dim3((g.count + ub - 1) / ub), dim3(64), (size_t)16 * kmax * ub, stream, a,
                           ub, kmax);
        CF_HIP_CHECK(ctx, hipGetLastError());
        for (const cf_tri_chunk& c : plan->tri_chunks) {
            if (c.group != gi) continue;
            a.first = c.first;
            a.count = c.count;
            hipLaunchKernelGGL(tri_apply_kernel, dim3(c.count), dim3(TR_T), tri_lds_c(std::max<int>(1, c.kmax)),
                               stream, a);
            CF_HIP_CHECK(ctx, hipGetLastError());
            // users whose QL record overflowed: recomputed by the Jacobi kernel
            CF_TRY(cf_launch_eigen_flagged(ctx, plan, c.emax, c.first, c.count, a.flag + (c.first - g.first),
                                           d_item_off, d_items, d_evec_off, d_m, d_sigs, d_evals, d_evecs, stream));
        }
    }
    return CF_OK;
}

int cf_debug_tri(cf_ctx* ctx, int enable, uint64_t* out4) {   // out4: 8 slots
    if (!ctx) return CF_EINVAL;
    CF_TRY(set_device(ctx));
    if (enable) CF_TRY(cf_debug_counters(ctx));
    ctx->tri_debug = enable != 0;
    if (out4) {
        for (int i = 0; i < 8; ++i) out4[i] = 0;
        if (ctx->d_dbg) {
            CF_HIP_CHECK(ctx, hipDeviceSynchronize());
            CF_HIP_CHECK(ctx, hipMemcpy(out4, ctx->d_dbg + 8, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
            CF_HIP_CHECK(ctx, hipMemset(ctx->d_dbg + 8, 0, 8 * sizeof(uint64_t)));
        }
    }
    return CF_OK;
}
