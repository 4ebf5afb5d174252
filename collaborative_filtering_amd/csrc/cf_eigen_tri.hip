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
// the one-sided Jacobi kernel at its measured 9.7 sweeps.  A user whose QL record
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
    const float* graph;
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
};

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ double bsum(double v, double* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wsum(v);
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < TR_W; ++w) t += red[w];
    return t;
}

__host__ __device__ constexpr int tri_ld(int n) { return n | 1; }   // odd row stride: conflict-free columns

// ---- A: assembly + tridiagonalisation + Q ---------------------------------------------------
__global__ __launch_bounds__(TR_T) void tri_reduce_kernel(TriArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t jj = blockIdx.x;
    const uint32_t u = a.order[a.first + jj];
    const uint64_t base = a.item_off[u];
    const int n = (int)(a.item_off[u + 1] - base);
    if (n <= 0) {
        if (tid == 0) a.m_out[u] = 0;
        return;
    }
    const int LD = tri_ld(n);
    float* A = reinterpret_cast<float*>(smem_raw);                 // n x LD, row-major
    double* vu = reinterpret_cast<double*>(A + ((n * LD + 1) & ~1));  // u of the step
    double* vp = vu + TR_NMAX;                                     // p / w of the step
    double* hh = vp + TR_NMAX;                                     // h_i of every step
    double* red = hh + TR_NMAX;                                    // reductions (8)
    uint32_t* s_item = reinterpret_cast<uint32_t*>(red + 8);

    for (int i = tid; i < n; i += TR_T) s_item[i] = a.items[base + i];
    __syncthreads();
    // W_u: wave per row, lanes over columns
    for (int i = wave; i < n; i += TR_W) {
        const float* grow = a.graph + (size_t)s_item[i] * a.n_items;
        for (int j = lane; j < n; j += 64) A[i * LD + j] = grow[s_item[j]];
    }
    __syncthreads();
    // degrees and scales, thread per row, sequential j (the oracle's summation order)
    for (int i = tid; i < n; i += TR_T) {
        double d = 0.0;
        for (int j = 0; j < n; ++j) d += (double)A[i * LD + j];
        if (d == 0.0) d = 1.0;                       // (:137-140)
        vu[i] = d;
        vp[i] = sqrt(1.0 / d);                       // (:149-153)
    }
    __syncthreads();
    // sig_min (float accumulation of double squares, :172-176) and L2 rows kept in registers?
    // No: L2(i,j) is recomputed where needed; each thread owns row i.
    float sig_i = 0.0f;
    for (int i = tid; i < n; i += TR_T) {
        const double si = vp[i], di = vu[i];
        float acc = 0.0f;
        for (int j = 0; j < n; ++j) {
            const double l = (j == i ? di : 0.0) - (double)A[i * LD + j];
            const double l2 = (si * l) * vp[j];      // (:155)
            acc = (float)((double)acc + l2 * l2);
        }
        sig_i = sqrtf(acc);
        a.sigs[base + i] = (float)((double)sig_i + 0.01);   // (:177)
    }
    // cut smm = float(max sig + 0.01) (:179-182)
    {
        float mx = (tid < n) ? sig_i : 0.0f;
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        __syncthreads();
        if (lane == 0) reinterpret_cast<float*>(red)[wave] = mx;
        __syncthreads();
        if (tid == 0) {
            float m = 0.0f;
            for (int w = 0; w < TR_W; ++w) m = fmaxf(m, reinterpret_cast<float*>(red)[w]);
            a.smm[jj] = (float)((double)m + 0.01);
        }
        __syncthreads();
    }
    // A = sym_lower(L2) in place (row i owned by thread i; column writes go to rows j > i
    // of the upper part, which no thread reads W from any more: W_ij for j < i only)
    // Two passes so that no W value is overwritten before it is read.
    for (int i = tid; i < n; i += TR_T) {
        const double si = vp[i], di = vu[i];
        for (int j = 0; j <= i; ++j) {
            const double l = (j == i ? di : 0.0) - (double)A[i * LD + j];
            A[i * LD + j] = (float)((si * l) * vp[j]);
        }
    }
    __syncthreads();
    for (int idx = tid; idx < n * n; idx += TR_T) {
        const int i = idx / n, j = idx - i * n;
        if (j > i) A[i * LD + j] = A[j * LD + i];
    }
    __syncthreads();

    // ---- Householder reduction: step i annihilates A[i][0 .. i-2] --------------------------
    double* dd = a.dd + base;
    double* ee = a.ee + base;
    for (int i = n - 1; i > 0; --i) {
        double part = 0.0;
        for (int q = tid; q < i; q += TR_T) part += fabs((double)A[i * LD + q]);
        const double scale = bsum(part, red);
        if (scale == 0.0) {
            if (tid == 0) {
                ee[i] = 0.0;
                hh[i] = 0.0;
            }
            for (int q = tid; q < i; q += TR_T) A[i * LD + q] = 0.0f;   // u = 0
            __syncthreads();
            continue;
        }
        double hp = 0.0;
        for (int q = tid; q < i; q += TR_T) {
            const double v = (double)A[i * LD + q] / scale;
            vu[q] = v;
            hp += v * v;
        }
        double h = bsum(hp, red);
        if (tid == 0) {
            const double f = vu[i - 1];
            const double g = f > 0 ? -sqrt(h) : sqrt(h);
            ee[i] = scale * g;
            h -= f * g;
            vu[i - 1] = f - g;
            red[7] = h;
        }
        __syncthreads();
        h = red[7];
        // p = A[0:i, 0:i] u / h, thread per row
        for (int j = tid; j < i; j += TR_T) {
            const float* row = A + j * LD;
            double p0 = 0.0, p1 = 0.0;
            int q = 0;
            for (; q + 2 <= i; q += 2) {
                p0 += (double)row[q] * vu[q];
                p1 += (double)row[q + 1] * vu[q + 1];
            }
            if (q < i) p0 += (double)row[q] * vu[q];
            vp[j] = (p0 + p1) / h;
        }
        __syncthreads();
        double kp = 0.0;
        for (int j = tid; j < i; j += TR_T) kp += vu[j] * vp[j];
        const double K = bsum(kp, red) / (h + h);
        for (int j = tid; j < i; j += TR_T) vp[j] -= K * vu[j];
        __syncthreads();
        // rank-2 update of the active block; reflector u into row i (dead from now on)
        for (int idx = tid; idx < i * i; idx += TR_T) {
            const int r = idx / i, c = idx - r * i;
            A[r * LD + c] = (float)((double)A[r * LD + c] - (vu[r] * vp[c] + vp[r] * vu[c]));
        }
        for (int q = tid; q < i; q += TR_T) A[i * LD + q] = (float)vu[q];
        if (tid == 0) hh[i] = h;
        __syncthreads();
    }
    for (int i = tid; i < n; i += TR_T) dd[i] = (double)A[i * LD + i];
    if (tid == 0) {
        ee[0] = 0.0;
        hh[0] = 0.0;
    }
    __syncthreads();
    // reflectors (strict lower triangle) to the evecs slot, then Q in LDS
    float* slot = a.evecs + a.evec_off[u];
    for (int idx = tid; idx < n * n; idx += TR_T) {
        const int i = idx / n, j = idx - i * n;
        if (j < i) slot[idx] = A[i * LD + j];
    }
    __syncthreads();
    for (int idx = tid; idx < n * n; idx += TR_T) {
        const int i = idx / n, j = idx - i * n;
        A[i * LD + j] = (i == j) ? 1.0f : 0.0f;
    }
    __syncthreads();
    // Q = H_{n-1} ... H_1: for i = 1 .. n-1, Q[0:i, 0:i] -= u (u^T Q[0:i, 0:i]) / h_i
    for (int i = 1; i < n; ++i) {
        const double h = hh[i];
        if (h == 0.0) continue;   // uniform
        for (int q = tid; q < i; q += TR_T) vu[q] = (double)slot[i * n + q];
        __syncthreads();
        for (int c = tid; c < i; c += TR_T) {
            double t0 = 0.0, t1 = 0.0;
            int r = 0;
            for (; r + 2 <= i; r += 2) {
                t0 += vu[r] * (double)A[r * LD + c];
                t1 += vu[r + 1] * (double)A[(r + 1) * LD + c];
            }
            if (r < i) t0 += vu[r] * (double)A[r * LD + c];
            vp[c] = (t0 + t1) / h;
        }
        __syncthreads();
        for (int idx = tid; idx < i * i; idx += TR_T) {
            const int r = idx / i, c = idx - r * i;
            A[r * LD + c] = (float)((double)A[r * LD + c] - vu[r] * vp[c]);
        }
        __syncthreads();
    }
    // Q to the slot (row-major n x n)
    for (int idx = tid; idx < n * n; idx += TR_T) {
        const int i = idx / n, j = idx - i * n;
        slot[idx] = A[i * LD + j];
    }
}

// ---- B: batched tql2 with rotation recording (one lane per user) ------------------------------
__global__ __launch_bounds__(64) void tri_ql_kernel(TriArgs a) {
    const uint32_t jj = blockIdx.x * 64 + threadIdx.x;
    if (jj >= a.count) return;
    const uint32_t u = a.order[a.first + jj];
    const uint64_t base = a.item_off[u];
    const int n = (int)(a.item_off[u + 1] - base);
    if (n <= 0) return;
    double* d = a.dd + base;
    double* e = a.ee + base;
    const size_t pj = 2 * (size_t)(a.first + jj);
    float2* rot = a.rot + a.rot_off[pj];
    const uint64_t rot_cap = a.rot_off[pj + 1] - a.rot_off[pj];
    int2* hdr = a.hdr + a.hdr_off[pj];
    const uint64_t hdr_cap = a.hdr_off[pj + 1] - a.hdr_off[pj];
    uint64_t nrot = 0, nh = 0;
    bool overflow = false;
    for (int i = 1; i < n; ++i) e[i - 1] = e[i];
    e[n - 1] = 0.0;
    double f = 0.0, tst1 = 0.0;
    const double eps = 2.220446049250313e-16;
    for (int l = 0; l < n && !overflow; ++l) {
        tst1 = fmax(tst1, fabs(d[l]) + fabs(e[l]));
        int m = l;
        while (m < n && !(fabs(e[m]) <= eps * tst1)) ++m;
        if (m > l) {
            int iter = 0;
            do {
                ++iter;
                if (nh >= hdr_cap || nrot + (uint64_t)(m - l) > rot_cap) {
                    overflow = true;
                    break;
                }
                const double g0 = d[l];
                double p = (d[l + 1] - g0) / (2.0 * e[l]);
                double r = sqrt(p * p + 1.0);
                if (p < 0) r = -r;
                d[l] = e[l] / (p + r);
                d[l + 1] = e[l] * (p + r);
                const double dl1 = d[l + 1];
                const double h0 = g0 - d[l];
                for (int i = l + 2; i < n; ++i) d[i] -= h0;
                f += h0;
                p = d[m];
                double c = 1.0, c2 = 1.0, c3 = 1.0, s = 0.0, s2 = 0.0;
                const double el1 = e[l + 1];
                double di = d[m - 1 >= 0 ? m - 1 : 0], ei = e[m - 1 >= 0 ? m - 1 : 0];
                for (int i = m - 1; i >= l; --i) {
                    const double di_n = i > l ? d[i - 1] : 0.0, ei_n = i > l ? e[i - 1] : 0.0;  // prefetch
                    c3 = c2;
                    c2 = c;
                    s2 = s;
                    const double g = c * ei;
                    const double h = c * p;
                    r = sqrt(p * p + ei * ei);
                    e[i + 1] = s * r;
                    const double ri = 1.0 / r;
                    s = ei * ri;
                    c = p * ri;
                    p = c * di - s * g;
                    d[i + 1] = h + s * (c * g + s * di);
                    rot[nrot + (m - 1 - i)] = make_float2((float)c, (float)s);
                    di = di_n;
                    ei = ei_n;
                }
                hdr[nh++] = make_int2(l, m);
                nrot += (uint64_t)(m - l);
                p = -s * s2 * c3 * el1 * e[l] / dl1;
                e[l] = s * p;
                d[l] = c * p;
            } while (fabs(e[l]) > eps * tst1 && iter < 60);
        }
        d[l] += f;
        e[l] = 0.0;
    }
    a.flag[jj] = overflow ? 1 : 0;
    a.n_iter[jj] = (int)nh;
}

// ---- C: rotations applied to Q, ordering, output ---------------------------------------------
__global__ __launch_bounds__(TR_T) void tri_apply_kernel(TriArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t jj = blockIdx.x;
    const uint32_t u = a.order[a.first + jj];
    const uint64_t base = a.item_off[u];
    const int n = (int)(a.item_off[u + 1] - base);
    if (n <= 0 || a.flag[jj]) return;
    const int LD = tri_ld(n);
    float* V = reinterpret_cast<float*>(smem_raw);                       // n x LD
    float2* cs = reinterpret_cast<float2*>(V + ((n * LD + 1) & ~1));    // [TR_Q][n]
    int* perm = reinterpret_cast<int*>(cs + TR_Q * TR_NMAX);
    float* sgn = reinterpret_cast<float*>(perm + TR_NMAX);
    int* sh = reinterpret_cast<int*>(sgn + TR_NMAX);                    // [2 * TR_Q + 4]
    float* slot = a.evecs + a.evec_off[u];
    for (int idx = tid; idx < n * n; idx += TR_T) {
        const int i = idx / n, j = idx - i * n;
        V[i * LD + j] = slot[idx];
    }
    const float2* rot = a.rot + a.rot_off[2 * (size_t)(a.first + jj)];
    const int2* hdr = a.hdr + a.hdr_off[2 * (size_t)(a.first + jj)];
    const int n_it = a.n_iter[jj];
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
        // stage: sequence t covers positions [l_t, m_t - 1], stored from m_t - 1 down
        {
            uint64_t off = rpos;
            for (int t = 0; t < nseq; ++t) {
                const int l = sh[t], m = sh[TR_Q + t];
                for (int p = tid; p < n; p += TR_T) {
                    float2 v = make_float2(1.0f, 0.0f);
                    if (p >= l && p < m) v = rot[off + (m - 1 - p)];
                    cs[t * TR_NMAX + p] = v;
                }
                off += (uint64_t)(m - l);
            }
            rpos = off;
        }
        __syncthreads();
        int L = n, Mx = 0;
        for (int t = 0; t < nseq; ++t) {
            L = min(L, sh[t]);
            Mx = max(Mx, sh[TR_Q + t]);
        }
        const int r = tid;
        if (r < n) {
            float* row = V + r * LD;
            float carry[TR_Q];
            carry[0] = row[Mx];
#pragma unroll
            for (int t = 1; t < TR_Q; ++t) carry[t] = 0.0f;
            for (int tau = Mx - 1; tau >= L - nseq; --tau) {
                float val = tau >= L ? row[tau] : 0.0f;
                bool ok = tau >= L;
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
    const double* ev = a.dd + base;
    for (int j = tid; j < n; j += TR_T) {
        const double lj = ev[j];
        int rank = 0;
        for (int i = 0; i < n; ++i) {
            const double li = ev[i];
            rank += (li < lj) || (li == lj && i < j);
        }
        perm[rank] = j;
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += (double)V[i * LD + j];
        sgn[j] = s < 0.0 ? -1.0f : 1.0f;
    }
    __syncthreads();
    if (tid == 0) {
        const float smm = a.smm[jj];
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
    for (int idx = tid; idx < n * m; idx += TR_T) {
        const int i = idx / m, r = idx - i * m;
        float v = 0.0f;
        if (r < n) {
            const int j = perm[r];
            v = V[i * LD + j] * sgn[j];
        }
        slot[idx] = v;
    }
    (void)lane;
    (void)wave;
}

size_t tri_lds_a(int kmax) {
    return sizeof(float) * (size_t)((kmax * tri_ld(kmax) + 1) & ~1) + sizeof(double) * (3 * TR_NMAX + 8) +
           sizeof(uint32_t) * TR_NMAX;
}
size_t tri_lds_c(int kmax) {
    return sizeof(float) * (size_t)((kmax * tri_ld(kmax) + 1) & ~1) + sizeof(float2) * TR_Q * TR_NMAX +
           sizeof(int) * TR_NMAX + sizeof(float) * TR_NMAX + sizeof(int) * (2 * TR_Q + 4);
}

}  // namespace

// Rotation-record budget per user (float2 units) and header budget (QL iterations).
static inline uint64_t tri_rot_cap(uint64_t k) { return 3 * k * k + 64; }
static inline uint64_t tri_hdr_cap(uint64_t k) { return 4 * k + 16; }

int cf_tri_prepare(cf_ctx* ctx, cf_plan* plan, const uint64_t* item_off) {
    // Chunks: plan-order ranges inside one LDS bucket whose QL records fit the budget.
    // Per plan index j: [start, end) of its rotation / header records, chunk-relative,
    // stored at 2j and 2j + 1.
    const uint64_t budget = (uint64_t)1536 << 20;   // bytes of rotation records per chunk
    plan->tri_chunks.clear();
    plan->n_entries = plan->n_users ? item_off[plan->n_users] : 0;
    std::vector<uint64_t> r2(2 * (size_t)plan->n_users + 2, 0), h2(2 * (size_t)plan->n_users + 2, 0);
    for (const cf_bucket& b : plan->buckets) {
        if (b.emax == kSpillBucket || b.count == 0) continue;
        uint32_t start = b.first;
        uint64_t acc = 0, acch = 0;
        for (uint32_t j = b.first; j < b.first + b.count; ++j) {
            const uint32_t u = plan->h_order[j];
            const uint64_t k = item_off[u + 1] - item_off[u];
            const uint64_t rc = tri_rot_cap(k), hc = tri_hdr_cap(k);
            if (j > start && (acc + rc) * sizeof(float2) > budget) {
                plan->tri_chunks.push_back({b.emax, start, j - start, b.kmax});
                start = j;
                acc = 0;
                acch = 0;
            }
            r2[2 * (size_t)j] = acc;
            h2[2 * (size_t)j] = acch;
            acc += rc;
            acch += hc;
            r2[2 * (size_t)j + 1] = acc;
            h2[2 * (size_t)j + 1] = acch;
            plan->tri_rot_max = std::max(plan->tri_rot_max, acc);
            plan->tri_hdr_max = std::max(plan->tri_hdr_max, acch);
        }
        plan->tri_chunks.push_back({b.emax, start, b.first + b.count - start, b.kmax});
    }
    for (const auto& c : plan->tri_chunks) plan->tri_users_max = std::max(plan->tri_users_max, c.count);
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
                        (plan->tri_rot_max + 1) * sizeof(float2) + (plan->tri_hdr_max + 1) * sizeof(int2);
    if (need > ctx->tri_bytes) {
        if (ctx->d_tri) (void)hipFree(ctx->d_tri);
        ctx->d_tri = nullptr;
        ctx->tri_bytes = 0;
        if (hipMalloc(&ctx->d_tri, need) != hipSuccess)
            return cf_set_error(ctx, CF_ENOMEM, "tridiagonal eigen scratch (" + std::to_string(need) + " bytes)");
        ctx->tri_bytes = need;
    }
    char* p = static_cast<char*>(ctx->d_tri);
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
                        hipStream_t stream) {
    if (plan->tri_chunks.empty()) return CF_OK;
    TriArgs a{};
    CF_TRY(tri_scratch(ctx, plan, a));
    a.order = plan->d_order;
    a.item_off = d_item_off;
    a.items = d_items;
    a.graph = ctx->d_graph;
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
        configured = true;
    }
    for (const cf_tri_chunk& c : plan->tri_chunks) {
        a.first = c.first;
        a.count = c.count;
        const int kmax = std::max<int>(1, (int)c.kmax);
        hipLaunchKernelGGL(tri_reduce_kernel, dim3(c.count), dim3(TR_T), tri_lds_a(kmax), stream, a);
        CF_HIP_CHECK(ctx, hipGetLastError());
        hipLaunchKernelGGL(tri_ql_kernel, dim3((c.count + 63) / 64), dim3(64), 0, stream, a);
        CF_HIP_CHECK(ctx, hipGetLastError());
        hipLaunchKernelGGL(tri_apply_kernel, dim3(c.count), dim3(TR_T), tri_lds_c(kmax), stream, a);
        CF_HIP_CHECK(ctx, hipGetLastError());
        // users whose QL record overflowed: recomputed by the Jacobi kernel
        CF_TRY(cf_launch_eigen_flagged(ctx, plan, c.emax, c.first, c.count, a.flag, d_item_off, d_items, d_evec_off,
                                       d_m, d_sigs, d_evals, d_evecs, stream));
    }
    return CF_OK;
}
