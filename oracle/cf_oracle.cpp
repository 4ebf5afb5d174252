// cf_oracle.cpp -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
//
// This file is the parity oracle for the MI355X rebuild.  Only tests/, the
// __graft_entry__.smoke() check and bench.py's cpu_baseline leg may load it.
// The product library (collaborative_filtering_amd/libcf_mi355x.so) never
// links or calls it.
//
// PARITY STATUS: "parity unpinned" with respect to the reference binaries.
// The reference cannot be built here (graphlab.hpp, Eigen/Dense, boost and
// boost/threadpool.hpp are absent) and it ships no tests,
// fixtures or golden vectors.  The arithmetic the reference delegates to the
// third-party Eigen library (Eigen 3.x, GraphLab-2.1 era, version not pinned by
// the reference: SelfAdjointEigenSolver = Householder tridiagonalisation +
// implicit symmetric QR; MatrixXd::inverse = PartialPivLU) is restated below
// from the published algorithms and pinned against numpy/LAPACK (eigh, inv) via
// the fixtures in tests/golden/ and against closed-form spectra.
//
// Every function cites the reference file:line it follows.  Double precision
// throughout, with the reference's float roundings reproduced where they occur.

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <thread>
#include <utility>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// Symmetric eigensolver: Householder reduction to tridiagonal form followed by
// the implicit-shift QL iteration (EISPACK tred2/tql2 algorithm class, the same
// class as Eigen's SelfAdjointEigenSolver).  Reads ONLY the lower triangle of
// a (row-major n x n), like Eigen (precompute_local_threads.cpp:164).
// On return: d = eigenvalues ascending, V (row-major n x n) columns = vectors.
// ---------------------------------------------------------------------------
void tridiag_householder(int n, std::vector<double>& V, std::vector<double>& d,
                         std::vector<double>& e) {
    auto at = [&](int r, int c) -> double& { return V[(size_t)r * n + c]; };
    for (int j = 0; j < n; ++j) d[j] = at(n - 1, j);
    for (int i = n - 1; i > 0; --i) {
        double scale = 0.0, h = 0.0;
        for (int k = 0; k < i; ++k) scale += std::fabs(d[k]);
        if (scale == 0.0) {
            e[i] = d[i - 1];
            for (int j = 0; j < i; ++j) {
                d[j] = at(i - 1, j);
                at(i, j) = 0.0;
                at(j, i) = 0.0;
            }
        } else {
            for (int k = 0; k < i; ++k) {
                d[k] /= scale;
                h += d[k] * d[k];
            }
            double f = d[i - 1];
            double g = std::sqrt(h);
            if (f > 0) g = -g;
            e[i] = scale * g;
            h -= f * g;
            d[i - 1] = f - g;
            for (int j = 0; j < i; ++j) e[j] = 0.0;
            for (int j = 0; j < i; ++j) {
                f = d[j];
                at(j, i) = f;
                g = e[j] + at(j, j) * f;
                for (int k = j + 1; k <= i - 1; ++k) {
                    g += at(k, j) * d[k];
                    e[k] += at(k, j) * f;
                }
                e[j] = g;
            }
            f = 0.0;
            for (int j = 0; j < i; ++j) {
                e[j] /= h;
                f += e[j] * d[j];
            }
            double hh = f / (h + h);
            for (int j = 0; j < i; ++j) e[j] -= hh * d[j];
            for (int j = 0; j < i; ++j) {
                f = d[j];
                g = e[j];
                for (int k = j; k <= i - 1; ++k) at(k, j) -= (f * e[k] + g * d[k]);
                d[j] = at(i - 1, j);
                at(i, j) = 0.0;
            }
        }
        d[i] = h;
    }
    // Accumulate the orthogonal transformation.
    for (int i = 0; i < n - 1; ++i) {
        at(n - 1, i) = at(i, i);
        at(i, i) = 1.0;
        double h = d[i + 1];
        if (h != 0.0) {
            for (int k = 0; k <= i; ++k) d[k] = at(k, i + 1) / h;
            for (int j = 0; j <= i; ++j) {
                double g = 0.0;
                for (int k = 0; k <= i; ++k) g += at(k, i + 1) * at(k, j);
                for (int k = 0; k <= i; ++k) at(k, j) -= g * d[k];
            }
        }
        for (int k = 0; k <= i; ++k) at(k, i + 1) = 0.0;
    }
    for (int j = 0; j < n; ++j) {
        d[j] = at(n - 1, j);
        at(n - 1, j) = 0.0;
    }
    at(n - 1, n - 1) = 1.0;
    e[0] = 0.0;
}

// V is passed TRANSPOSED here (VT[col*n + row]) so the rotation sweeps are contiguous.
void tridiag_ql(int n, std::vector<double>& VT, std::vector<double>& d, std::vector<double>& e) {
    auto at = [&](int r, int c) -> double& { return VT[(size_t)c * n + r]; };
    for (int i = 1; i < n; ++i) e[i - 1] = e[i];
    e[n - 1] = 0.0;
    double f = 0.0, tst1 = 0.0;
    const double eps = std::ldexp(1.0, -52);
    for (int l = 0; l < n; ++l) {
        tst1 = std::max(tst1, std::fabs(d[l]) + std::fabs(e[l]));
        int m = l;
        while (m < n) {
            if (std::fabs(e[m]) <= eps * tst1) break;
            ++m;
        }
        if (m > l) {
            int iter = 0;
            do {
                ++iter;
                double g = d[l];
                double p = (d[l + 1] - g) / (2.0 * e[l]);
                double r = std::hypot(p, 1.0);
                if (p < 0) r = -r;
                d[l] = e[l] / (p + r);
                d[l + 1] = e[l] * (p + r);
                double dl1 = d[l + 1];
                double h = g - d[l];
                for (int i = l + 2; i < n; ++i) d[i] -= h;
                f += h;
                p = d[m];
                double c = 1.0, c2 = c, c3 = c;
                double el1 = e[l + 1];
                double s = 0.0, s2 = 0.0;
                for (int i = m - 1; i >= l; --i) {
                    c3 = c2;
                    c2 = c;
                    s2 = s;
                    g = c * e[i];
                    h = c * p;
                    r = std::hypot(p, e[i]);
                    e[i + 1] = s * r;
                    s = e[i] / r;
                    c = p / r;
                    p = c * d[i] - s * g;
                    d[i + 1] = h + s * (c * g + s * d[i]);
                    double* vi = &at(0, i);
                    double* vi1 = &at(0, i + 1);
                    for (int k = 0; k < n; ++k) {
                        h = vi1[k];
                        vi1[k] = s * vi[k] + c * h;
                        vi[k] = c * vi[k] - s * h;
                    }
                }
                p = -s * s2 * c3 * el1 * e[l] / dl1;
                e[l] = s * p;
                d[l] = c * p;
            } while (std::fabs(e[l]) > eps * tst1 && iter < 60);
        }
        d[l] += f;
        e[l] = 0.0;
    }
    // Ascending selection sort of values with their vectors (Eigen sorts the same way).
    for (int i = 0; i < n - 1; ++i) {
        int k = i;
        double p = d[i];
        for (int j = i + 1; j < n; ++j)
            if (d[j] < p) {
                k = j;
                p = d[j];
            }
        if (k != i) {
            d[k] = d[i];
            d[i] = p;
            for (int j = 0; j < n; ++j) std::swap(at(j, i), at(j, k));  // contiguous columns
        }
    }
}

// Eigen-class PartialPivLU, in place on row-major a (n x n); perm[i] = source row.
// Zero pivots are skipped like Eigen's unblocked_lu (no division, no error).
void lu_partial_pivot(int n, double* a, std::vector<int>& perm) {
    perm.resize(n);
    for (int i = 0; i < n; ++i) perm[i] = i;
    for (int k = 0; k < n; ++k) {
        int piv = k;
        double best = std::fabs(a[(size_t)k * n + k]);
        for (int i = k + 1; i < n; ++i) {
            double v = std::fabs(a[(size_t)i * n + k]);
            if (v > best) {
                best = v;
                piv = i;
            }
        }
        if (best != 0.0) {
            if (piv != k) {
                for (int j = 0; j < n; ++j) std::swap(a[(size_t)k * n + j], a[(size_t)piv * n + j]);
                std::swap(perm[k], perm[piv]);
            }
            const double pv = a[(size_t)k * n + k];
            for (int i = k + 1; i < n; ++i) a[(size_t)i * n + k] /= pv;
        }
        for (int i = k + 1; i < n; ++i) {
            const double lik = a[(size_t)i * n + k];
            for (int j = k + 1; j < n; ++j) a[(size_t)i * n + j] -= lik * a[(size_t)k * n + j];
        }
    }
}

// MatrixXd::inverse() for dynamic sizes = PartialPivLU(a).solve(Identity).
void lu_inverse(int n, const double* a_in, double* inv) {
    std::vector<double> lu(a_in, a_in + (size_t)n * n);
    std::vector<int> perm;
    lu_partial_pivot(n, lu.data(), perm);
    std::vector<double> col(n);
    for (int c = 0; c < n; ++c) {
        for (int i = 0; i < n; ++i) col[i] = (perm[i] == c) ? 1.0 : 0.0;
        for (int i = 0; i < n; ++i) {  // unit lower
            double s = col[i];
            for (int j = 0; j < i; ++j) s -= lu[(size_t)i * n + j] * col[j];
            col[i] = s;
        }
        for (int i = n - 1; i >= 0; --i) {  // upper
            double s = col[i];
            for (int j = i + 1; j < n; ++j) s -= lu[(size_t)i * n + j] * col[j];
            col[i] = s / lu[(size_t)i * n + i];
        }
        for (int i = 0; i < n; ++i) inv[(size_t)i * n + c] = col[i];
    }
}

}  // namespace

extern "C" {

// Symmetric eigendecomposition (lower triangle of a, row-major n x n).
// evals ascending; evecs row-major n x n with eigenvector j in column j.
int cfo_eigh(int n, const double* a, double* evals, double* evecs) {
    if (n <= 0) return 0;
    std::vector<double> V((size_t)n * n), d(n), e(n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            const int r = std::max(i, j), c = std::min(i, j);
            V[(size_t)i * n + j] = a[(size_t)r * n + c];
        }
    tridiag_householder(n, V, d, e);
    std::vector<double> VT((size_t)n * n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) VT[(size_t)j * n + i] = V[(size_t)i * n + j];
    tridiag_ql(n, VT, d, e);
    std::memcpy(evals, d.data(), sizeof(double) * n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) evecs[(size_t)i * n + j] = VT[(size_t)j * n + i];
    return 0;
}

int cfo_inverse(int n, const double* a, double* inv) {
    lu_inverse(n, a, inv);
    return 0;
}

// a2-a4: compute_eigens (precompute_local_threads.cpp:100-194).
//   Wu     : k x k row-major directed weights, Wu[i*k+j] = weights(item_i, item_j) (:118-125)
//   faithful: 1 = perform the reference's dense LU inverse of D and the two dense
//             GEMMs (:149-155); 0 = the algebraically identical O(k^2) form.
//             Both give bit-identical L2 (checked by tests).
//   L2_out : optional k x k row-major normalized Laplacian (full, unsymmetrised)
//   sigs   : k values, sigs[i] = (double)sig_min_i + 0.01 (:172-177)
//   evals  : k slots; first m written (ascending), rest zero
//   evecs  : k*k slots; first k*m written row-major (k rows, m columns) (:205-209)
// Returns m (= lim, >= 2).  For k == 1 the reference pads with uninitialised
// memory (:193-194); the oracle pads with 0.
int cfo_compute_eigens(int k, const double* Wu, int faithful, double* L2_out, double* sigs,
                       double* evals, double* evecs) {
    if (k <= 0) return 0;
    const size_t kk = (size_t)k * k;
    std::vector<double> L(kk), L2(kk), dvec(k);
    // D with the 0 -> 1 rule (:129-141)
    for (int i = 0; i < k; ++i) {
        double count = 0;
        for (int j = 0; j < k; ++j) count += Wu[(size_t)i * k + j];
        dvec[i] = (count == 0) ? 1.0 : count;
    }
    // L = D - W (:144-145)
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j)
            L[(size_t)i * k + j] = (i == j ? dvec[i] : 0.0) - Wu[(size_t)i * k + j];
    if (faithful) {
        // dd2 = sqrt(inverse(D)) elementwise, L2 = dd2 * L * dd2 (:148-155)
        std::vector<double> D(kk, 0.0), Di(kk), T(kk);
        for (int i = 0; i < k; ++i) D[(size_t)i * k + i] = dvec[i];
        lu_inverse(k, D.data(), Di.data());
        for (size_t t = 0; t < kk; ++t) Di[t] = std::sqrt(Di[t]);
        for (int i = 0; i < k; ++i)
            for (int j = 0; j < k; ++j) {
                double s = 0;
                for (int q = 0; q < k; ++q) s += Di[(size_t)i * k + q] * L[(size_t)q * k + j];
                T[(size_t)i * k + j] = s;
            }
        for (int i = 0; i < k; ++i)
            for (int j = 0; j < k; ++j) {
                double s = 0;
                for (int q = 0; q < k; ++q) s += T[(size_t)i * k + q] * Di[(size_t)q * k + j];
                L2[(size_t)i * k + j] = s;
            }
    } else {
        std::vector<double> sv(k);
        for (int i = 0; i < k; ++i) sv[i] = std::sqrt(1.0 / dvec[i]);
        for (int i = 0; i < k; ++i)
            for (int j = 0; j < k; ++j)
                L2[(size_t)i * k + j] = (sv[i] * L[(size_t)i * k + j]) * sv[j];
    }
    if (L2_out) std::memcpy(L2_out, L2.data(), sizeof(double) * kk);

    std::vector<double> ev(k), V(kk);
    cfo_eigh(k, L2.data(), ev.data(), V.data());  // (:164-166), lower triangle

    // sig_min per row, accumulated in float (:169-182)
    float sig_min_max = 0;
    for (int i = 0; i < k; ++i) {
        float sig_min = 0;
        for (int j = 0; j < k; ++j) sig_min += std::pow(L2[(size_t)i * k + j], 2);
        sig_min = std::sqrt(sig_min);  // float overload
        sigs[i] = sig_min + 0.01;
        if (sig_min_max < sig_min) sig_min_max = sig_min;
    }
    sig_min_max += 0.01;

    // lim (:185-191)
    int lim;
    for (lim = 0; lim < k; ++lim)
        if (ev[lim] > sig_min_max) break;
    if (lim < 2) lim = 2;

    for (int j = 0; j < k; ++j) evals[j] = 0.0;
    for (size_t t = 0; t < kk; ++t) evecs[t] = 0.0;
    for (int j = 0; j < lim && j < k; ++j) evals[j] = ev[j];
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < lim; ++j)
            evecs[(size_t)i * lim + j] = (j < k) ? V[(size_t)i * k + j] : 0.0;
    return lim;
}

// Batched precompute_local_threads (precompute_local_threads.cpp:215-317) over a
// dense float item-weight matrix W (n_items x n_items, row-major, directed).
//   item_off[n_users+1], items[] : per-user item indices into W (any order; the
//                                  rows of the user's block follow this order)
//   evec_off[n_users]            : offset of each user's k*k evec slot
//   outputs: m_out[u], sigs/evals at item_off[u], evecs at evec_off[u] (k x m row-major)
// n_threads = std::thread pool size (the reference's boost::threadpool, :300-314).
int cfo_precompute_batch(int n_users, const int64_t* item_off, const int32_t* items,
                         int64_t n_items, const float* W, const int64_t* evec_off,
                         int n_threads, int faithful, int32_t* m_out, double* sigs,
                         double* evals, double* evecs) {
    std::atomic<int> next(0);
    auto worker = [&]() {
        std::vector<double> Wu;
        for (;;) {
            const int u = next.fetch_add(1);
            if (u >= n_users) break;
            const int64_t b = item_off[u];
            const int k = (int)(item_off[u + 1] - b);
            if (k <= 0) {
                m_out[u] = 0;
                continue;
            }
            Wu.assign((size_t)k * k, 0.0);
            for (int i = 0; i < k; ++i) {
                const float* row = W + (size_t)items[b + i] * n_items;
                for (int j = 0; j < k; ++j) Wu[(size_t)i * k + j] = (double)row[items[b + j]];
            }
            m_out[u] = cfo_compute_eigens(k, Wu.data(), faithful, nullptr, sigs + b, evals + b,
                                          evecs + evec_off[u]);
        }
    };
    if (n_threads <= 1) {
        worker();
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < n_threads; ++t) pool.emplace_back(worker);
        for (auto& t : pool) t.join();
    }
    return 0;
}

// a7: neigh_program::apply inner loop for ONE user (local_calc_precomp.cpp:230-360),
// evaluated for every one of the user's k test movies (rows).
//   k, m          : user's item count and stored eigenpair count
//   items[k]      : the user's items as indices into W (row order of the eigen block)
//   ratings[k]    : the user's test ratings of those items (out_test_rat_)
//   evals[m], U   : eigenvalues and k x m row-major eigenvectors (out_eigen_)
//   sigtab[k]     : w_lim per row: the concatenated-sigs table in compat mode
//                   (:414,437,440,271), or the user's own sigs in fixed mode
//   W, n_items    : dense float out_fin_ weights; neighbour iff (double)w > 0.1 (:129-133)
//   rows[n_rows]  : which rows (test movies) to evaluate
// Outputs per evaluated row: mse (float, :358), kk (= c, :359), pred (clamped, double),
// cond-flag bit 0 = Gram matrix had a zero pivot.
int cfo_predict_user(int k, int m, const int32_t* items, const double* ratings,
                     const double* evals, const double* U, const double* sigtab,
                     const float* W, int64_t n_items, int n_rows, const int32_t* rows,
                     float* mse_out, int32_t* kk_out, double* pred_out) {
    std::vector<int> C;
    std::vector<int> keep;
    for (int t = 0; t < n_rows; ++t) {
        const int r = rows[t];
        const double rat_real = ratings[r];
        const float* nrow = W + (size_t)items[r] * n_items;
        // connected movies in the user's row order (:254-265)
        C.clear();
        for (int j = 0; j < k; ++j)
            if ((double)nrow[items[j]] > 0.1) C.push_back(j);
        const int c = (int)C.size();
        // lim from w_lim (:271-279)
        const double w_lim = sigtab[r];
        int lim;
        for (lim = 0; lim < m; ++lim)
            if (evals[lim] > w_lim) break;
        if (lim < 2) lim = 2;
        if (lim > m) lim = m;  // unreachable for m >= 2 (reference would read past the block)
        // zero-column filter (:284-304)
        keep.clear();
        for (int col = 0; col < lim; ++col) {
            int i;
            for (i = 0; i < c; ++i)
                if (U[(size_t)C[i] * m + col] >= 0.0001) break;
            if (i < c) keep.push_back(col);
        }
        const int Lc = (int)keep.size();
        // rating mean and centred ratings (:311-312)
        double sum = 0;
        for (int i = 0; i < c; ++i) sum += ratings[C[i]];
        const double rat_mean = sum / c;
        // t = Uh^T (r - mean); mm = Uh^T Uh; x = inverse(mm) t; pred = vv . x + mean (:308-315)
        std::vector<double> tv(Lc, 0.0), mm((size_t)Lc * Lc, 0.0), inv((size_t)Lc * Lc), x(Lc, 0.0);
        for (int a = 0; a < Lc; ++a) {
            double s = 0;
            for (int i = 0; i < c; ++i) s += U[(size_t)C[i] * m + keep[a]] * (ratings[C[i]] - rat_mean);
            tv[a] = s;
            for (int b2 = 0; b2 < Lc; ++b2) {
                double g = 0;
                for (int i = 0; i < c; ++i)
                    g += U[(size_t)C[i] * m + keep[a]] * U[(size_t)C[i] * m + keep[b2]];
                mm[(size_t)a * Lc + b2] = g;
            }
        }
        if (Lc > 0) lu_inverse(Lc, mm.data(), inv.data());
        for (int a = 0; a < Lc; ++a) {
            double s = 0;
            for (int b2 = 0; b2 < Lc; ++b2) s += inv[(size_t)a * Lc + b2] * tv[b2];
            x[a] = s;
        }
        double pred = 0;
        for (int a = 0; a < Lc; ++a) pred += U[(size_t)r * m + keep[a]] * x[a];
        pred += rat_mean;
        if (pred > 5) pred = 5;  // (:322-325)
        if (pred < 1) pred = 1;
        const double err = std::pow(rat_real - pred, 2);
        mse_out[t] = (float)err;
        kk_out[t] = c;
        if (pred_out) pred_out[t] = pred;
    }
    return 0;
}

// a7 over a batch of users on a std::thread pool: the local_calc_precomp form of the CPU
// baseline (GraphLab runs neigh_program::apply on --ncpus workers, local_calc_precomp.cpp:
// 217-380, 484-583).  Per user u (rows item_off[u]..item_off[u+1]): evals at item_off[u]
// (first m[u] valid), the k x m block at evecs + evec_off[u]; w_lim = sigtab[r] in compat mode
// (the concatenated table, :414,437,440,271) or sigtab[item_off[u] + r] in own mode.
// Outputs mse / kk / pred (pred may be null) at item_off[u] + r.
int cfo_predict_batch(int n_users, const int64_t* item_off, const int32_t* items,
                      const double* ratings, const int32_t* m, const double* evals,
                      const int64_t* evec_off, const double* evecs, const double* sigtab,
                      int compat, const float* W, int64_t n_items, int n_threads,
                      float* mse_out, int32_t* kk_out, double* pred_out) {
    std::atomic<int> next(0);
    auto worker = [&]() {
        std::vector<int32_t> rows;
        for (;;) {
            const int u = next.fetch_add(1);
            if (u >= n_users) break;
            const int64_t b = item_off[u];
            const int k = (int)(item_off[u + 1] - b);
            if (k <= 0 || m[u] <= 0) continue;
            rows.resize(k);
            for (int r = 0; r < k; ++r) rows[r] = r;
            cfo_predict_user(k, m[u], items + b, ratings + b, evals + b, evecs + evec_off[u],
                             compat ? sigtab : sigtab + b, W, n_items, k, rows.data(), mse_out + b,
                             kk_out + b, pred_out ? pred_out + b : nullptr);
        }
    };
    if (n_threads <= 1) {
        worker();
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < n_threads; ++t) pool.emplace_back(worker);
        for (auto& t : pool) t.join();
    }
    return 0;
}

// a8 assembly: the local graph of movie m (local_calc.cpp:268-334).  Row/column 0 is
// the movie, rows 1..deg its out-neighbours nbrs[] (compact ids, w > 0.1, ascending:
// the reference iterates a boost::unordered_map, so its row order is unpinned and the
// results are permutation-equivariant).  Graph edges exist only for w > 0.1
// (graph_loader :113).  W(i, j) = w(nb_i -> nb_j) for i, j >= 1 (:326-330; an
// out-neighbour outside the local graph aliases to column 0 and is overwritten by
// :333), W(0, j) = W(j, 0) = w(m -> nb_j) (:331-333), W(0, 0) = 0.
//   G: n_items x n_items raw weights (float); W: n x n row-major, n = deg + 1.
int cfo_local_graph(int m, int deg, const int32_t* nbrs, const float* G, int64_t n_items, double* W) {
    const int n = deg + 1;
    auto w = [&](int a, int b) {
        const float v = G[(size_t)a * n_items + b];
        return (double)v > 0.1 ? (double)v : 0.0;
    };
    for (int i = 0; i < n * n; ++i) W[i] = 0.0;
    for (int i = 1; i < n; ++i)
        for (int j = 1; j < n; ++j) W[(size_t)i * n + j] = w(nbrs[i - 1], nbrs[j - 1]);
    for (int j = 1; j < n; ++j) {
        W[j] = w(m, nbrs[j - 1]);
        W[(size_t)j * n] = w(m, nbrs[j - 1]);
    }
    return n;
}

// a8: vertex_program::apply for one movie (local_calc.cpp:346-521).
//   W  : n x n local adjacency (cfo_local_graph)
//   R  : n x nu row-major test ratings; column u = one test user of the movie, row 0 its
//        rating of the movie, row i >= 1 its test rating of neighbour i (0 = unrated)
//   out: per user mse (float, :499,519), kk (= #rated rows), pred, w_lim, lim
// D has no 0 -> 1 guard (:354-360); L2 = (s_i L_ij) s_j with s = sqrt(1/d) (:368-374),
// full and unsymmetrised; the eigensolver reads its lower triangle (:378).  Per user:
// row 0 counts as unrated (:405); w_lim = sqrt(lambda_min(L2_h L2_h^T)) over the unrated
// rows h (:417-436); lim = first eigenvalue > w_lim, >= 2 (:444-451); no zero-column
// filter; pred = v^T (mm^-1 (U_C^T (r - mean))) + mean with mm = U_C^T U_C inverted by
// partial-pivot LU (:484-491), clamped to [1, 5] (:494-497).
int cfo_local_calc(int n, const double* W, int nu, const double* R, float* mse_out, int32_t* kk_out,
                   double* pred_out, double* wlim_out, int32_t* lim_out) {
    std::vector<double> d(n), L((size_t)n * n), L2((size_t)n * n), ev(n), V((size_t)n * n);
    for (int i = 0; i < n; ++i) {
        double count = 0;
        for (int j = 0; j < n; ++j) count += W[(size_t)i * n + j];
        d[i] = count;
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) L[(size_t)i * n + j] = (i == j ? d[i] : 0.0) - W[(size_t)i * n + j];
    for (int i = 0; i < n; ++i) {
        const double si = std::sqrt(1.0 / d[i]);
        for (int j = 0; j < n; ++j) L2[(size_t)i * n + j] = (si * L[(size_t)i * n + j]) * std::sqrt(1.0 / d[j]);
    }
    cfo_eigh(n, L2.data(), ev.data(), V.data());
    std::vector<int> hrows, crows;
    for (int u = 0; u < nu; ++u) {
        std::vector<double> r(n);
        for (int i = 0; i < n; ++i) r[i] = R[(size_t)i * nu + u];
        const double rat_real = r[0];
        r[0] = 0;
        hrows.clear();
        crows.clear();
        for (int i = 0; i < n; ++i) (r[i] == 0 ? hrows : crows).push_back(i);
        const int h = (int)hrows.size(), c = (int)crows.size();
        // w_lim = sqrt(lambda_min(L2_h L2_h^T))
        std::vector<double> S((size_t)h * h), sev(h), svec((size_t)h * h);
        for (int a = 0; a < h; ++a)
            for (int b = 0; b < h; ++b) {
                double acc = 0;
                for (int j = 0; j < n; ++j) acc += L2[(size_t)hrows[a] * n + j] * L2[(size_t)hrows[b] * n + j];
                S[(size_t)a * h + b] = acc;
            }
        cfo_eigh(h, S.data(), sev.data(), svec.data());
        double emin = sev[0];
        for (int a = 1; a < h; ++a) emin = std::min(emin, sev[a]);
        const double w_lim = std::sqrt(emin);
        int lim;
        for (lim = 0; lim < n; ++lim)
            if (ev[lim] > w_lim) break;
        if (lim < 2) lim = 2;
        // prediction over the rated rows (:455-491)
        double sum = 0;
        for (int i = 0; i < c; ++i) sum += r[crows[i]];
        const double mean = sum / c;
        std::vector<double> mm((size_t)lim * lim), inv((size_t)lim * lim), tv(lim), x(lim);
        for (int a = 0; a < lim; ++a) {
            double t = 0;
            for (int i = 0; i < c; ++i) t += V[(size_t)crows[i] * n + a] * (r[crows[i]] - mean);
            tv[a] = t;
            for (int b = 0; b < lim; ++b) {
                double g = 0;
                for (int i = 0; i < c; ++i) g += V[(size_t)crows[i] * n + a] * V[(size_t)crows[i] * n + b];
                mm[(size_t)a * lim + b] = g;
            }
        }
        lu_inverse(lim, mm.data(), inv.data());
        for (int a = 0; a < lim; ++a) {
            double t = 0;
            for (int b = 0; b < lim; ++b) t += inv[(size_t)a * lim + b] * tv[b];
            x[a] = t;
        }
        double pred = 0;
        for (int a = 0; a < lim; ++a) pred += V[a] * x[a];   // vv = row 0 of U
        pred += mean;
        if (pred > 5) pred = 5;
        if (pred < 1) pred = 1;
        mse_out[u] = (float)std::pow(rat_real - pred, 2);
        kk_out[u] = c;
        if (pred_out) pred_out[u] = pred;
        if (wlim_out) wlim_out[u] = w_lim;
        if (lim_out) lim_out[u] = lim;
    }
    return 0;
}

// a10: weights_calc for every ordered item pair (knn2.cpp:127-146) + the writer's
// w > 0.01 filter (:157).  Train ratings come per user (CSR); each item's map is
// built in ascending user order (the reference iterates a boost::unordered_map, so
// its order -- and with real-valued ratings the float rounding -- is unpinned).
//   W_out[a*n_items + b] = w if written, else 0.  cnt_out (optional) = common users.
typedef std::vector<std::vector<std::pair<int, double>>> Knn2Maps;

static Knn2Maps knn2_maps(int n_users, const int64_t* user_off, const int32_t* item, const double* rating,
                          int n_items) {
    Knn2Maps maps(n_items);
    for (int u = 0; u < n_users; ++u)
        for (int64_t e = user_off[u]; e < user_off[u + 1]; ++e) maps[item[e]].push_back({u, rating[e]});
    return maps;
}

// weights_calc for one item pair (knn2.cpp:127-146) plus the writer's w > 0.01 (:157).
static float knn2_pair(const std::vector<std::pair<int, double>>& ma, const std::vector<std::pair<int, double>>& mb,
                       int& num_rat) {
    float num = 0, den1 = 0, den2 = 0;
    num_rat = 0;
    size_t j = 0;
    for (size_t i = 0; i < ma.size(); ++i) {  // (:133-140)
        while (j < mb.size() && mb[j].first < ma[i].first) ++j;
        if (j < mb.size() && mb[j].first == ma[i].first) {
            num_rat++;
            num += ma[i].second * mb[j].second;
            den1 += ma[i].second * ma[i].second;
            den2 += mb[j].second * mb[j].second;
        }
    }
    double obs = 0;
    if (num_rat > 5) obs = num / (std::sqrt(den1) * std::sqrt(den2));  // (:142-145)
    return obs > 0.01 ? (float)obs : 0.0f;                              // (:157)
}

int cfo_knn2(int n_users, const int64_t* user_off, const int32_t* item, const double* rating,
             int n_items, float* W_out, int32_t* cnt_out) {
    const Knn2Maps maps = knn2_maps(n_users, user_off, item, rating, n_items);
    for (int a = 0; a < n_items; ++a) {
        for (int b = 0; b < n_items; ++b) {
            float w = 0.0f;
            int num_rat = 0;
            if (a != b) w = knn2_pair(maps[a], maps[b], num_rat);
            W_out[(size_t)a * n_items + b] = w;
            if (cnt_out) cnt_out[(size_t)a * n_items + b] = num_rat;
        }
    }
    return 0;
}

// The same for the rows listed in rows[0..n_rows) only (CPU-baseline sample of bench.py):
// W_out is n_rows x n_items.
// n_threads > 1: rows are handed out to that many std::threads (each row's values are the
// same computation, so the output does not depend on the thread count).
int cfo_knn2_rows_mt(int n_users, const int64_t* user_off, const int32_t* item, const double* rating,
                     int n_items, int n_rows, const int32_t* rows, float* W_out, int n_threads) {
    const Knn2Maps maps = knn2_maps(n_users, user_off, item, rating, n_items);
    std::atomic<int> next{0};
    auto work = [&]() {
        for (int i = next++; i < n_rows; i = next++) {
            const int a = rows[i];
            for (int b = 0; b < n_items; ++b) {
                int num_rat = 0;
                W_out[(size_t)i * n_items + b] = a != b ? knn2_pair(maps[a], maps[b], num_rat) : 0.0f;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < n_threads; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
    return 0;
}

int cfo_knn2_rows(int n_users, const int64_t* user_off, const int32_t* item, const double* rating,
                  int n_items, int n_rows, const int32_t* rows, float* W_out) {
    return cfo_knn2_rows_mt(n_users, user_off, item, rating, n_items, n_rows, rows, W_out, 1);
}

// a11: knn_program gather/apply + error_vertex_data (knn3.cpp:185-256).
//   W: dense out_fin_ weights as parsed floats; edge m -> nb iff (double)w > 0.1 (:91)
//   test ratings per movie (CSR over movies): movie_off, user, rating (out_test_rat_)
//   pred[e]      : ratings_knn[user] of entry e (0 when missing, the operator[] default)
//   movie_mse[m] : error_vertex_data of vertex m (float)
int cfo_knn3(int n_items, const float* W, const int64_t* movie_off, const int32_t* user,
             const double* rating, double* pred, float* movie_mse) {
    std::vector<std::vector<std::pair<int, double>>> test(n_items);
    for (int m = 0; m < n_items; ++m)
        for (int64_t e = movie_off[m]; e < movie_off[m + 1]; ++e) test[m].push_back({user[e], rating[e]});
    std::vector<double> sum_r, sum_w;
    for (int m = 0; m < n_items; ++m) {
        // gather over out-edges (:197-205) and sum (:151-179), keyed by user
        std::vector<std::pair<int, std::pair<double, double>>> acc;  // user -> (sum w*r, sum w)
        for (int nb = 0; nb < n_items; ++nb) {
            const double obs = (double)W[(size_t)m * n_items + nb];
            if (!(obs > 0.1)) continue;
            for (const auto& ur : test[nb]) acc.push_back({ur.first, {obs * ur.second, obs}});
        }
        std::sort(acc.begin(), acc.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        float err = 0, tmp;
        for (int64_t e = movie_off[m]; e < movie_off[m + 1]; ++e) {
            const int u = user[e];
            double sr = 0, sw = 0;
            bool found = false;
            auto it = std::lower_bound(acc.begin(), acc.end(), u,
                                       [](const auto& x, int key) { return x.first < key; });
            for (; it != acc.end() && it->first == u; ++it) {
                sr += it->second.first;
                sw += it->second.second;
                found = true;
            }
            const double p = found ? sr / sw : 0.0;  // (:216); missing key -> 0 (:243)
            pred[e] = p;
            if (p < 0.1)
                tmp = 0;
            else
                tmp = (float)(rating[e] - std::round(p));  // (:246), boost::math::round
            err += tmp * tmp;
        }
        const int64_t sz = movie_off[m + 1] - movie_off[m];
        if (sz > 0)
            movie_mse[m] = std::isnan(err) ? 0.0f : err / (float)sz;  // (:249-253)
        else
            movie_mse[m] = 0.0f;
    }
    return 0;
}

// Graph-signal polynomial filters, restated superstep by superstep as
// the reference's GraphLab sync engines run them, over an explicit directed edge list.
//   graph_loader (cheby.cpp:88-92 / binomials.cpp:77-93): a line with w > 0.1 adds
//     va -> vb and vb -> va (self-edges dropped, as GraphLab's add_edge does);
//   degree_program (cheby.cpp:152-170): d_i = sum of OUT-edge weights;
//   gather (cheby.cpp:188-191, :222-225; binomials.cpp:192-196, :231-235):
//     sum_i = sum_{e = i -> j} w_e / sqrt(d_j * d_i) * x_j;
//   cheby init / step (cheby.cpp:195-206, :228-244), binomials a / b (binomials.cpp:199-205,
//   :238-243) with ind = round index (:357).  kind 0 = cheby, 1 = binomials.
int cfo_graph_filter(int kind, int n, int64_t n_lines, const int32_t* va, const int32_t* vb,
                     const double* w, const double* signal, const double* coeff, int n_coeff,
                     double* out) {
    if (n_coeff < 3) return -1;
    std::vector<int32_t> es, ed;
    std::vector<double> ew;
    for (int64_t l = 0; l < n_lines; ++l) {
        if (!(w[l] > 0.1) || va[l] == vb[l]) continue;
        es.push_back(va[l]); ed.push_back(vb[l]); ew.push_back(w[l]);
        es.push_back(vb[l]); ed.push_back(va[l]); ew.push_back(w[l]);
    }
    const size_t E = es.size();
    std::vector<double> deg(n, 0.0);
    for (size_t e = 0; e < E; ++e) deg[es[e]] += ew[e];
    auto gather = [&](const std::vector<double>& x) {
        std::vector<double> sum(n, 0.0);
        for (size_t e = 0; e < E; ++e)
            sum[es[e]] += ew[e] / std::sqrt(deg[ed[e]] * deg[es[e]]) * x[ed[e]];
        return sum;
    };
    const double a1 = 1.0, a2 = 1.0;   // arange {0, 2} (cheby.cpp:17-19)
    std::vector<double> val(signal, signal + n);
    if (kind == 0) {
        std::vector<double> t_old(n), t_cur(n), t_new(n);
        std::vector<double> sum = gather(val);
        for (int i = 0; i < n; ++i) {
            t_old[i] = val[i];
            t_cur[i] = (val[i] - sum[i] - a2 * val[i]) / a1;
            val[i] = 0.5 * coeff[0] * t_old[i] + coeff[1] * t_cur[i];
        }
        for (int counter = 2; counter < n_coeff; ++counter) {
            sum = gather(t_cur);
            for (int i = 0; i < n; ++i) {
                t_new[i] = (2 / a1) * (t_cur[i] - sum[i] - a2 * t_cur[i]) - t_old[i];
                val[i] = val[i] + coeff[counter] * t_new[i];
                t_old[i] = t_cur[i];
                t_cur[i] = t_new[i];
            }
        }
    } else {
        std::vector<double> part_a(n), tmp(n);
        for (int ind = 0; 3 * ind < n_coeff; ++ind) {
            std::vector<double> sum = gather(val);
            for (int i = 0; i < n; ++i) {
                part_a[i] = (coeff[ind] + coeff[ind + 1]) * val[i] - coeff[ind + 1] * sum[i];
                tmp[i] = val[i] - sum[i];
            }
            sum = gather(tmp);
            for (int i = 0; i < n; ++i) val[i] = part_a[i] + coeff[ind + 2] * (tmp[i] - sum[i]);
        }
    }
    for (int i = 0; i < n; ++i) out[i] = val[i];
    return 0;
}

// knn regroup (knn.cpp:83-111 loader, :160-205 rating maps with the last assignment winning,
// :212-298 co-rated sets of both roles, written sorted by :337-357) with the reference's
// container semantics -- a std::map per movie and role, a sorted unique co-rated list per movie
// -- on n_threads host threads, each owning the movies m % n_threads == t (the CPU baseline of
// bench.py's data-prep leg; the GPU path is cf_knn_regroup).  counts[3] = train entries, test
// entries, co-rated entries.
int cfo_knn_regroup_mt(int64_t n, const uint32_t* user, const uint32_t* movie, const float* rating,
                       const uint8_t* validate, int n_movies, int n_users, int n_threads, uint64_t* counts) {
    n_threads = std::max(1, n_threads);
    // every user's movie set (both roles), built once and shared read-only
    std::vector<std::vector<uint32_t>> sets(n_users);
    for (int64_t i = 0; i < n; ++i) sets[user[i]].push_back(movie[i]);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < n_threads; ++t)
            th.emplace_back([&, t] {
                for (int u = t; u < n_users; u += n_threads) {
                    auto& v = sets[u];
                    std::sort(v.begin(), v.end());
                    v.erase(std::unique(v.begin(), v.end()), v.end());
                }
            });
        for (auto& x : th) x.join();
    }
    std::vector<uint64_t> c_tr(n_threads, 0), c_te(n_threads, 0), c_co(n_threads, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t)
        th.emplace_back([&, t] {
            const int mine = (n_movies - t + n_threads - 1) / n_threads;
            std::vector<std::map<uint32_t, float>> tr(mine), te(mine);
            for (int64_t i = 0; i < n; ++i) {
                const uint32_t m = movie[i];
                if ((int)(m % n_threads) != t) continue;
                auto& mp = (validate && validate[i]) ? te[m / n_threads] : tr[m / n_threads];
                mp[user[i]] = rating[i];   // the last assignment wins
            }
            std::vector<std::vector<uint32_t>> co(mine);
            for (int u = 0; u < n_users; ++u) {
                const auto& v = sets[u];
                for (uint32_t a : v) {
                    if ((int)(a % n_threads) != t) continue;
                    auto& c = co[a / n_threads];
                    for (uint32_t b : v)
                        if (b != a) c.push_back(b);
                }
            }
            for (int j = 0; j < mine; ++j) {
                auto& c = co[j];
                std::sort(c.begin(), c.end());
                c.erase(std::unique(c.begin(), c.end()), c.end());
                c_tr[t] += tr[j].size();
                c_te[t] += te[j].size();
                c_co[t] += c.size();
            }
        });
    for (auto& x : th) x.join();
    counts[0] = counts[1] = counts[2] = 0;
    for (int t = 0; t < n_threads; ++t) {
        counts[0] += c_tr[t];
        counts[1] += c_te[t];
        counts[2] += c_co[t];
    }
    return 0;
}

}  // extern "C"
