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
//   2. Householder tridiagonalisation and accumulation of Q (the EISPACK tred2 order
//      that the oracle restates, oracle/cf_oracle.cpp tridiag_householder), with the
//      symmetric matrix-vector product thread-per-row (coalesced column reads) and the
//      rank-2 update wave-per-column;
//   3. implicit-shift QL (tql2, oracle tridiag_ql): one lane generates the rotation
//      sequence of an iteration into LDS, then every thread applies it to its own rows
//      of Q, carrying one value across the sequence (one read + one write per element);
//   4. rank sort, sign convention sum_i v_ij >= 0 (as cf_eigen.hip), lim (:184-191),
//      and the k x m row-major block, sigs, evals, m -- the same record as the LDS path.
//
// Everything is fp64: the matrices are too large for the fp32 Jacobi tolerance argument
// of the LDS path, and the FP64 vector rate of MI355X equals its unpacked FP32 rate.
// The path is bound by workspace traffic (tridiagonalisation ~k^3/3 elements read and
// 2k^3/3 read+written, QL ~ (#rotations) x k x 16 B), see DESIGN.md.

#include "cf_internal.h"

namespace {

constexpr int SP_T = 512;
constexpr int SP_W = SP_T / 64;
constexpr int SP_N = CF_SPILL_MAX_K;
constexpr int SP_Q = 8;                          // QL iterations applied per pass over Q
constexpr int SP_TB = 64;                        // positions per staged coefficient block

struct SpillArgs {
    const uint32_t* order;
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
    double* work;
    uint64_t work_stride;    // doubles per workgroup slot (>= kmax^2)
    unsigned int* counter;   // next spill user (zeroed before the launch)
    unsigned long long* phase;   // 8 counters (cf_debug_spill), summed by thread 0
};

struct SpillSmem {
    double d[SP_N];
    double e[SP_N];
    double rc[SP_N];
    double rs[SP_N];
    float sig[SP_N];
    int perm[SP_N];
    double red[SP_W + 4];
    int flag[4];
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
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

__global__ __launch_bounds__(SP_T) void eigen_spill_kernel(SpillArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SpillSmem& S = *reinterpret_cast<SpillSmem*>(smem_raw);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double* M = a.work + (size_t)blockIdx.x * a.work_stride;
    const double eps = 2.220446049250313e-16;   // 2^-52 (tql2)

    for (;;) {
        if (tid == 0) S.flag[0] = (int)atomicAdd(a.counter, 1u);
        __syncthreads();
        const int idx = S.flag[0];
        __syncthreads();
        if (idx >= (int)a.count) break;   // uniform: every wave leaves together
        const uint32_t u = a.order[a.first + idx];
        const uint64_t base = a.item_off[u];
        const int n = (int)(a.item_off[u + 1] - base);
        float* Wt = a.evecs + a.evec_off[u];   // k x k scratch until the output is written
        auto Mat = [&](int r, int c) -> double& { return M[(size_t)c * n + r]; };
        unsigned long long t0 = tid == 0 ? __builtin_amdgcn_s_memtime() : 0ull, t1 = 0, t2 = 0, t3 = 0, tgen = 0;
        unsigned long long n_iter = 0;

        // ---- 1. W_u, degrees, s, L2, sig_min, A = sym_lower(L2) ------------------------
        for (int i = wave; i < n; i += SP_W) {
            const float* grow = a.graph + (size_t)a.items[base + i] * a.n_items;
            double ds = 0.0;
            for (int j = lane; j < n; j += 64) {
                const float w = grow[a.items[base + j]];
                Wt[(size_t)i * n + j] = w;
                ds += (double)w;
            }
            ds = wave_sum(ds);
            if (lane == 0) S.rs[i] = (ds == 0.0) ? 1.0 : ds;   // (:137-140)
        }
        __syncthreads();
        for (int i = tid; i < n; i += SP_T) S.rc[i] = sqrt(1.0 / S.rs[i]);   // (:149-153)
        __syncthreads();
        for (int i = wave; i < n; i += SP_W) {
            const double si = S.rc[i], di = S.rs[i];
            double sq = 0.0;
            for (int j = lane; j < n; j += 64) {
                const double l = (j == i ? di : 0.0) - (double)Wt[(size_t)i * n + j];
                const double l2 = (si * l) * S.rc[j];   // (:155)
                sq += l2 * l2;
                if (j <= i) {
                    Mat(i, j) = l2;
                    Mat(j, i) = l2;
                }
            }
            sq = wave_sum(sq);
            if (lane == 0) S.sig[i] = sqrtf((float)sq);   // (:172-176)
        }
        __syncthreads();

        if (tid == 0) t1 = __builtin_amdgcn_s_memtime();
        // ---- 2a. tridiagonalisation (tred2) ---------------------------------------------
        for (int j = tid; j < n; j += SP_T) S.d[j] = Mat(n - 1, j);
        __syncthreads();
        for (int i = n - 1; i > 0; --i) {
            double part = 0.0;
            for (int q = tid; q < i; q += SP_T) part += fabs(S.d[q]);
            const double scale = block_sum(part, S.red);
            double h = 0.0;
            if (scale == 0.0) {
                if (tid == 0) S.e[i] = S.d[i - 1];
                __syncthreads();
                for (int j = tid; j < i; j += SP_T) {
                    S.d[j] = Mat(i - 1, j);
                    Mat(i, j) = 0.0;
                    Mat(j, i) = 0.0;
                }
            } else {
                double hp = 0.0;
                for (int q = tid; q < i; q += SP_T) {
                    const double v = S.d[q] / scale;
                    S.d[q] = v;
                    hp += v * v;
                }
                h = block_sum(hp, S.red);
                if (tid == 0) {
                    const double f = S.d[i - 1];
                    double g = sqrt(h);
                    if (f > 0) g = -g;
                    S.e[i] = scale * g;
                    h -= f * g;
                    S.d[i - 1] = f - g;
                    S.red[SP_W] = h;
                }
                __syncthreads();
                h = S.red[SP_W];
                // u into column i; p = A[0:i, 0:i] u, thread per row (column reads coalesce)
                for (int j = tid; j < i; j += SP_T) {
                    Mat(j, i) = S.d[j];
                    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
                    int q = 0;
                    for (; q + 8 <= i; q += 8) {
                        double x[8];
#pragma unroll
                        for (int t = 0; t < 8; ++t) x[t] = Mat(j, q + t);
                        p0 += x[0] * S.d[q] + x[4] * S.d[q + 4];
                        p1 += x[1] * S.d[q + 1] + x[5] * S.d[q + 5];
                        p2 += x[2] * S.d[q + 2] + x[6] * S.d[q + 6];
                        p3 += x[3] * S.d[q + 3] + x[7] * S.d[q + 7];
                    }
                    for (; q < i; ++q) p0 += Mat(j, q) * S.d[q];
                    S.e[j] = ((p0 + p1) + (p2 + p3)) / h;
                }
                __syncthreads();
                double fp = 0.0;
                for (int j = tid; j < i; j += SP_T) fp += S.e[j] * S.d[j];
                const double hh = block_sum(fp, S.red) / (h + h);
                for (int j = tid; j < i; j += SP_T) S.e[j] -= hh * S.d[j];
                __syncthreads();
                // rank-2 update of the active block, wave per column
                for (int j = wave; j < i; j += SP_W) {
                    const double dj = S.d[j], ej = S.e[j];
                    double* col = M + (size_t)j * n;
                    for (int q0 = 0; q0 < i; q0 += 256) {
                        double x[4];
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int q = q0 + 64 * t + lane;
                            x[t] = q < i ? col[q] : 0.0;
                        }
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int q = q0 + 64 * t + lane;
                            if (q < i) col[q] = x[t] - (dj * S.e[q] + ej * S.d[q]);
                        }
                    }
                }
                __syncthreads();
                for (int j = tid; j < i; j += SP_T) {
                    S.d[j] = Mat(i - 1, j);
                    Mat(i, j) = 0.0;
                }
            }
            __syncthreads();
            if (tid == 0) S.d[i] = h;
            __syncthreads();
        }
        if (tid == 0) t2 = __builtin_amdgcn_s_memtime();
        // ---- 2b. accumulate Q --------------------------------------------------------------
        for (int i = 0; i < n - 1; ++i) {
            if (tid == 0) {
                Mat(n - 1, i) = Mat(i, i);
                Mat(i, i) = 1.0;
            }
            __syncthreads();
            const double h = S.d[i + 1];
            if (h != 0.0) {
                const double* uc = M + (size_t)(i + 1) * n;
                for (int q = tid; q <= i; q += SP_T) S.rc[q] = uc[q];   // u of this step, staged in LDS
                __syncthreads();
                for (int j = wave; j <= i; j += SP_W) {
                    double* col = M + (size_t)j * n;
                    double g0 = 0.0, g1 = 0.0;
                    for (int q0 = 0; q0 <= i; q0 += 256) {
                        double x[4];
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int q = q0 + 64 * t + lane;
                            x[t] = q <= i ? col[q] : 0.0;
                        }
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int q = q0 + 64 * t + lane;
                            if (q <= i) (t & 1 ? g1 : g0) += S.rc[q] * x[t];
                        }
                    }
                    const double g = wave_sum(g0 + g1);
                    for (int q0 = 0; q0 <= i; q0 += 256) {
                        double x[4];
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int q = q0 + 64 * t + lane;
                            x[t] = q <= i ? col[q] : 0.0;
                        }
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int q = q0 + 64 * t + lane;
                            if (q <= i) col[q] = x[t] - g * (S.rc[q] / h);
                        }
                    }
                }
            }
            __syncthreads();
            for (int q = tid; q <= i; q += SP_T) Mat(q, i + 1) = 0.0;
            __syncthreads();
        }
        for (int j = tid; j < n; j += SP_T) {
            S.d[j] = Mat(n - 1, j);
            Mat(n - 1, j) = 0.0;
        }
        __syncthreads();
        if (tid == 0) {
            Mat(n - 1, n - 1) = 1.0;
            for (int i = 1; i < n; ++i) S.e[i - 1] = S.e[i];   // tql2 entry shift
            S.e[n - 1] = 0.0;
        }
        __syncthreads();

        if (tid == 0) t3 = __builtin_amdgcn_s_memtime();
        // ---- 3. implicit QL (tql2) -----------------------------------------------------------
        // Thread 0 runs the QL recurrence on (d, e) -- which never reads Q -- and records the
        // rotation sequences of up to SP_Q consecutive iterations (each on its own [l, m]).
        // All threads then apply the batch in ONE pass over the touched columns of Q:
        // sequence t lags sequence t-1 by one position, so a row streams through all SP_Q
        // sweeps with one load and one store per column (SP_Q carried values per row).
        {
            double* Gc = M + (size_t)n * n;      // [SP_Q][n] cosines
            double* Gs = Gc + (size_t)SP_Q * n;  // [SP_Q][n] sines
            int* seq_l = S.perm;                 // perm is free until section 4
            int* seq_m = S.perm + SP_Q;
            int gl = 0, gm = 0, giter = 0, gphase = 0;   // thread 0's generator state
            double gf = 0.0, gtst1 = 0.0;
            for (;;) {
                if (tid == 0) {
                    const unsigned long long tg = __builtin_amdgcn_s_memtime();
                    int nseq = 0;
                    while (nseq < SP_Q && gl < n) {
                        if (gphase == 0) {
                            gtst1 = fmax(gtst1, fabs(S.d[gl]) + fabs(S.e[gl]));
                            gm = gl;
                            while (gm < n && !(fabs(S.e[gm]) <= eps * gtst1)) ++gm;
                            if (gm == gl) {
                                S.d[gl] += gf;
                                S.e[gl] = 0.0;
                                ++gl;
                                continue;
                            }
                            giter = 0;
                            gphase = 1;
                        }
                        const int l = gl, m = gm;
                        ++giter;
                        ++n_iter;
                        const double g0 = S.d[l];
                        double p = (S.d[l + 1] - g0) / (2.0 * S.e[l]);
                        double r = hypot(p, 1.0);
                        if (p < 0) r = -r;
                        S.d[l] = S.e[l] / (p + r);
                        S.d[l + 1] = S.e[l] * (p + r);
                        const double dl1 = S.d[l + 1];
                        const double hsh = g0 - S.d[l];
                        for (int i = l + 2; i < n; ++i) S.d[i] -= hsh;
                        gf += hsh;
                        p = S.d[m];
                        double c = 1.0, c2 = 1.0, c3 = 1.0, sn = 0.0, s2 = 0.0;
                        const double el1 = S.e[l + 1];
                        double* gc = Gc + (size_t)nseq * n;
                        double* gs = Gs + (size_t)nseq * n;
                        for (int i = m - 1; i >= l; --i) {
                            c3 = c2;
                            c2 = c;
                            s2 = sn;
                            const double g = c * S.e[i];
                            const double h = c * p;
                            r = hypot(p, S.e[i]);
                            S.e[i + 1] = sn * r;
                            sn = S.e[i] / r;
                            c = p / r;
                            p = c * S.d[i] - sn * g;
                            S.d[i + 1] = h + sn * (c * g + sn * S.d[i]);
                            gc[i] = c;
                            gs[i] = sn;
                        }
                        p = -sn * s2 * c3 * el1 * S.e[l] / dl1;
                        S.e[l] = sn * p;
                        S.d[l] = c * p;
                        seq_l[nseq] = l;
                        seq_m[nseq] = m;
                        ++nseq;
                        if (!(fabs(S.e[l]) > eps * gtst1 && giter < 60)) {
                            S.d[l] += gf;
                            S.e[l] = 0.0;
                            ++gl;
                            gphase = 0;
                        }
                    }
                    S.flag[1] = nseq;
                    S.flag[2] = gl >= n;
                    tgen += __builtin_amdgcn_s_memtime() - tg;
                }
                __syncthreads();
                const int nseq = S.flag[1];
                const int done = S.flag[2];
                if (nseq > 0) {
                    int L = n, Mx = 0;
                    for (int t = 0; t < nseq; ++t) {
                        L = min(L, seq_l[t]);
                        Mx = max(Mx, seq_m[t]);
                    }
                    // one row of Q per thread and pass (rows rbase + tid)
                    for (int rbase = 0; rbase < n; rbase += SP_T) {
                        const int r = rbase + tid;
                        const bool act = r < n;
                        double carry[SP_Q];
                        carry[0] = act ? Mat(r, Mx) : 0.0;
#pragma unroll
                        for (int t = 1; t < SP_Q; ++t) carry[t] = 0.0;
                        const int tau_hi = Mx - 1, tau_lo = L - nseq;
                        for (int tb = tau_hi; tb >= tau_lo; tb -= SP_TB) {
                            // stage the coefficients of this block: [t][j] for tau = tb - j
                            __syncthreads();
                            for (int idx = tid; idx < SP_Q * SP_TB; idx += SP_T) {
                                const int t = idx / SP_TB, j = idx - t * SP_TB;
                                const int pp = tb - j + t;
                                double cv = 1.0, sv = 0.0;
                                if (t < nseq && pp >= seq_l[t] && pp < seq_m[t]) {
                                    cv = Gc[(size_t)t * n + pp];
                                    sv = Gs[(size_t)t * n + pp];
                                }
                                S.rc[idx] = cv;
                                S.rs[idx] = sv;
                            }
                            __syncthreads();
                            if (!act) continue;
                            const int jn = min(SP_TB, tb - tau_lo + 1);
                            for (int j0 = 0; j0 < jn; j0 += 8) {
                                double xin[8];
#pragma unroll
                                for (int u8 = 0; u8 < 8; ++u8) {
                                    const int tau = tb - j0 - u8;
                                    xin[u8] = (j0 + u8 < jn && tau >= L) ? Mat(r, tau) : 0.0;
                                }
#pragma unroll
                                for (int u8 = 0; u8 < 8; ++u8) {
                                    const int j = j0 + u8;
                                    if (j < jn) {
                                        const int tau = tb - j;
                                        double val = xin[u8];
                                        bool ok = tau >= L;
#pragma unroll
                                        for (int t = 0; t < SP_Q; ++t) {
                                            const int pp = tau + t;
                                            if (t >= nseq) {
                                                // sequences past the batch: pass through
                                            } else if (pp > Mx) {
                                                ok = false;
                                            } else if (pp == Mx) {
                                                if (ok) carry[t] = val;
                                                ok = false;
                                            } else if (pp >= L) {
                                                const double cv = S.rc[t * SP_TB + j], sv = S.rs[t * SP_TB + j];
                                                const double out = sv * val + cv * carry[t];
                                                carry[t] = cv * val - sv * carry[t];
                                                val = out;
                                            } else if (pp == L - 1) {
                                                val = carry[t];
                                                ok = true;
                                            } else {
                                                ok = false;
                                            }
                                        }
                                        if (ok) Mat(r, tau + nseq) = val;
                                    }
                                }
                            }
                        }
                    }
                }
                __syncthreads();
                if (done) break;
            }
        }

        const unsigned long long t4 = tid == 0 ? __builtin_amdgcn_s_memtime() : 0ull;
        // ---- 4. order, sign, lim, output --------------------------------------------------
        for (int j = tid; j < n; j += SP_T) {
            const double lj = S.d[j];
            int rank = 0;
            for (int i = 0; i < n; ++i) {
                const double li = S.d[i];
                rank += (li < lj) || (li == lj && i < j);
            }
            S.perm[rank] = j;
        }
        for (int j = wave; j < n; j += SP_W) {
            const double* col = M + (size_t)j * n;
            double sum = 0.0;
            for (int q = lane; q < n; q += 64) sum += col[q];
            sum = wave_sum(sum);
            if (lane == 0) S.rs[j] = sum < 0.0 ? -1.0 : 1.0;
        }
        __syncthreads();
        if (tid == 0) {
            float smm = 0.0f;
            for (int i = 0; i < n; ++i)
                if (smm < S.sig[i]) smm = S.sig[i];
            smm = (float)((double)smm + 0.01);   // (:179-182)
            int lim;
            for (lim = 0; lim < n; ++lim)
                if (S.d[S.perm[lim]] > (double)smm) break;   // (:186-188)
            if (lim < 2) lim = 2;                             // (:190-191)
            S.flag[3] = lim;
            a.m_out[u] = lim;
        }
        __syncthreads();
        const int mm = S.flag[3];
        for (int i = tid; i < n; i += SP_T) a.sigs[base + i] = (float)((double)S.sig[i] + 0.01);
        for (int r = tid; r < mm; r += SP_T) a.evals[base + r] = (float)S.d[S.perm[r]];
        for (int r = wave; r < mm; r += SP_W) {
            const int j = S.perm[r];
            const double sg = S.rs[j];
            const double* col = M + (size_t)j * n;
            for (int i = lane; i < n; i += 64) Wt[(size_t)i * mm + r] = (float)(col[i] * sg);
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

}  // namespace

int cf_launch_eigen_spill(cf_ctx* ctx, const cf_plan* plan, const cf_bucket& b, const uint64_t* d_item_off,
                          const uint32_t* d_items, const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs,
                          float* d_evals, float* d_evecs, hipStream_t stream) {
    if (b.count == 0) return CF_OK;
    int n_cu = 256;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, ctx->device);
    const uint64_t stride = (uint64_t)b.kmax * b.kmax + 2ull * SP_Q * b.kmax + 64;
    const uint64_t slot_bytes = stride * sizeof(double);
    const uint64_t budget = 8ull << 30;   // workspace cap; fewer resident users beyond it
    uint32_t grid = std::min<uint32_t>(b.count, (uint32_t)n_cu);
    grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(grid, budget / slot_bytes));
    const size_t need = (size_t)grid * slot_bytes + 256;
    if (need > ctx->spill_bytes) {
        if (ctx->d_spill && ctx->spill_debug) {   // keep the diagnostic counters across the regrowth
            CF_HIP_CHECK(ctx, hipStreamSynchronize(stream));
        }
        if (ctx->d_spill) (void)hipFree(ctx->d_spill);
        ctx->d_spill = nullptr;
        ctx->spill_bytes = 0;
        if (hipMalloc(&ctx->d_spill, need) != hipSuccess)
            return cf_set_error(ctx, CF_ENOMEM, "spill workspace (" + std::to_string(need) + " bytes)");
        ctx->spill_bytes = need;
        CF_HIP_CHECK(ctx, hipMemsetAsync(ctx->d_spill, 0, 256, stream));
    }
    SpillArgs a{};
    a.order = plan->d_order;
    a.first = b.first;
    a.count = b.count;
    a.item_off = d_item_off;
    a.items = d_items;
    a.graph = ctx->d_graph;
    a.n_items = ctx->n_items;
    a.evec_off = d_evec_off;
    a.m_out = d_m;
    a.sigs = d_sigs;
    a.evals = d_evals;
    a.evecs = d_evecs;
    a.counter = reinterpret_cast<unsigned int*>(ctx->d_spill);
    a.work = reinterpret_cast<double*>(static_cast<char*>(ctx->d_spill) + 256);
    a.work_stride = stride;
    a.phase = ctx->spill_debug ? reinterpret_cast<unsigned long long*>(static_cast<char*>(ctx->d_spill) + 64) : nullptr;
    CF_HIP_CHECK(ctx, hipMemsetAsync(a.counter, 0, sizeof(unsigned int), stream));
    const size_t lds = sizeof(SpillSmem);
    static_assert(sizeof(SpillSmem) <= 163840, "spill LDS");
    CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)eigen_spill_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)lds));
    hipLaunchKernelGGL(eigen_spill_kernel, dim3(grid), dim3(SP_T), lds, stream, a);
    CF_HIP_CHECK(ctx, hipGetLastError());
    return CF_OK;
}

int cf_debug_spill(cf_ctx* ctx, int enable, uint64_t* out8) {
    if (!ctx) return CF_EINVAL;
    CF_TRY(set_device(ctx));
    ctx->spill_debug = enable != 0;
    if (out8) {
        for (int i = 0; i < 8; ++i) out8[i] = 0;
        if (ctx->d_spill) {
            CF_HIP_CHECK(ctx, hipDeviceSynchronize());
            CF_HIP_CHECK(ctx, hipMemcpy(out8, static_cast<char*>(ctx->d_spill) + 64, 8 * sizeof(uint64_t),
                                        hipMemcpyDeviceToHost));
            CF_HIP_CHECK(ctx, hipMemset(static_cast<char*>(ctx->d_spill) + 64, 0, 8 * sizeof(uint64_t)));
        }
    }
    return CF_OK;
}
