// cf_synth.cpp -- counter-based (splitmix64) MovieLens-shaped synthetic data.
//
// Stands in for make_synthetic_als_data.cpp:118-178, whose GraphLab RNG
// (graphlab::random, seed 31413 at :125) is not available here: the same
// generators are re-implemented on a counter-based splitmix64 stream so every
// value depends only on (seed, stream, counter) and any thread can produce it.
//
//   cfh_synth_degrees     per-user item count k: lognormal, clipped  
//   cfh_synth_user_items  k distinct items per user from Zipf(s) popularity, sorted,
//                         integer ratings 1..5 with P = {.06,.11,.26,.35,.22}
//   cfh_synth_als         the make_synthetic_als_data algorithm itself (D latent
//                         Gaussian factors, power-law raters per movie, the
//                         (u + 2654435761) % nusers stepping, movie id offset +nusers)
//   cfh_synth_graph_model expected knn2 output for a Zipf train population (dense)

#include "cf_pyrand.hpp"
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Uniform double in [0,1) from (seed, stream, counter).
inline double u01(uint64_t seed, uint64_t stream, uint64_t ctr) {
    const uint64_t h = splitmix64(seed ^ splitmix64(stream * 0xD1B54A32D192ED03ull + ctr));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

inline double gauss(uint64_t seed, uint64_t stream, uint64_t ctr) {
    double a = u01(seed, stream, 2 * ctr), b = u01(seed, stream, 2 * ctr + 1);
    if (a < 1e-300) a = 1e-300;
    return std::sqrt(-2.0 * std::log(a)) * std::cos(6.283185307179586 * b);
}

template <typename F>
void parallel_for(uint32_t n, int n_threads, F&& f) {
    if (n_threads <= 1 || n < 64) {
        for (uint32_t i = 0; i < n; ++i) f(i, 0);
        return;
    }
    std::atomic<uint32_t> next(0);
    std::vector<std::thread> pool;
    for (int t = 0; t < n_threads; ++t)
        pool.emplace_back([&, t]() {
            for (;;) {
                const uint32_t b = next.fetch_add(256);
                if (b >= n) break;
                const uint32_t e = std::min(n, b + 256);
                for (uint32_t i = b; i < e; ++i) f(i, t);
            }
        });
    for (auto& th : pool) th.join();
}

const double kRatingCdf[5] = {0.06, 0.17, 0.43, 0.78, 1.0};

inline float draw_rating(double x) {
    for (int r = 0; r < 5; ++r)
        if (x < kRatingCdf[r]) return (float)(r + 1);
    return 5.0f;
}

}  // namespace

extern "C" {

void cfh_synth_degrees(uint64_t seed, uint32_t n_users, double k_median, double sigma, uint32_t kmin,
                       uint32_t kmax, uint32_t* k_out) {
    const double mu = std::log(k_median);
    for (uint32_t u = 0; u < n_users; ++u) {
        const double k = std::exp(mu + sigma * gauss(seed, 1, u));
        long v = std::lround(k);
        if (v < (long)kmin) v = kmin;
        if (v > (long)kmax) v = kmax;
        k_out[u] = (uint32_t)v;
    }
}

// Users u_base .. u_base + n_users - 1 of the population: every user's items and ratings depend
// only on (seed, global user index), so a rank can generate just its range of a global set.
int cfh_synth_user_items_at(uint64_t seed, uint32_t u_base, uint32_t n_users, uint32_t n_items,
                            double zipf_s, const uint64_t* item_off, uint32_t* items, float* ratings,
                            int n_threads) {
    if (n_items == 0) return -1;
    std::vector<double> cdf(n_items);
    double acc = 0;
    for (uint32_t i = 0; i < n_items; ++i) {
        acc += std::pow((double)(i + 1), -zipf_s);
        cdf[i] = acc;
    }
    for (auto& c : cdf) c /= acc;
    const int nt = std::max(1, n_threads);
    std::vector<std::vector<uint8_t>> seen(nt, std::vector<uint8_t>(n_items, 0));
    std::atomic<int> err(0);
    parallel_for(n_users, nt, [&](uint32_t u, int t) {
        const uint64_t b = item_off[u];
        const uint32_t k = (uint32_t)(item_off[u + 1] - b);
        if (k > n_items) {
            err = -2;
            return;
        }
        auto& s = seen[t];
        uint64_t ctr = 0;
        uint32_t got = 0;
        const uint64_t stream = 0x1000000ull + u_base + u;
        while (got < k) {
            const double x = u01(seed, stream, ctr++);
            uint32_t it = (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), x) - cdf.begin());
            if (it >= n_items) it = n_items - 1;
            if (ctr > 64ull * k + 4096) {  // pathological: fall back to a linear scan
                for (it = 0; it < n_items && s[it]; ++it) {
                }
            }
            if (s[it]) continue;
            s[it] = 1;
            items[b + got++] = it;
        }
        std::sort(items + b, items + b + k);
        for (uint32_t j = 0; j < k; ++j) {
            s[items[b + j]] = 0;
            ratings[b + j] = draw_rating(u01(seed, 0x2000000ull + u_base + u, j));
        }
    });
    return err.load();
}

int cfh_synth_user_items(uint64_t seed, uint32_t n_users, uint32_t n_items, double zipf_s,
                         const uint64_t* item_off, uint32_t* items, float* ratings, int n_threads) {
    return cfh_synth_user_items_at(seed, 0, n_users, n_items, zipf_s, item_off, items, ratings, n_threads);
}

// make_synthetic_als_data.cpp:118-178 on splitmix64.  Writes up to `cap` train and
// validate triplets (user, movie + nusers, rating) and returns the counts.
int cfh_synth_als(uint64_t seed, uint32_t nusers, uint32_t nmovies, uint32_t D, double stdev,
                  double alpha, uint32_t nvalidate, uint64_t cap, uint32_t* tr_u, uint32_t* tr_m,
                  double* tr_r, uint64_t* n_train, uint32_t* va_u, uint32_t* va_m, double* va_r,
                  uint64_t* n_valid) {
    if (nusers <= nvalidate) return -1;
    std::vector<double> uf((size_t)nusers * D), mf((size_t)nmovies * D);
    uint64_t ctr = 0;
    for (auto& x : uf) x = stdev * gauss(seed, 7, ctr++);   // :127-132
    for (auto& x : mf) x = stdev * gauss(seed, 7, ctr++);   // :135-140
    std::vector<double> prob(nusers - nvalidate);           // :144-148
    double acc = 0;
    for (size_t i = 0; i < prob.size(); ++i) {
        acc += std::pow((double)(i + 1), -alpha);
        prob[i] = acc;
    }
    for (auto& p : prob) p /= acc;
    uint64_t nt = 0, nv = 0, draw = 0;
    uint64_t user_id = 0;
    auto rating = [&](uint64_t uu, uint64_t mm) {
        double s = 0;
        for (uint32_t d = 0; d < D; ++d) s += uf[uu * D + d] * mf[mm * D + d];
        return s;
    };
    for (uint32_t movie = 0; movie < nmovies; ++movie) {
        const double x = u01(seed, 8, draw++);
        const size_t out_degree =
            (size_t)(std::lower_bound(prob.begin(), prob.end(), x) - prob.begin()) + 1;  // :151
        for (size_t i = 0; i < out_degree; ++i) {
            user_id = (user_id + 2654435761ull) % nusers;  // :154
            if (nt < cap) {
                tr_u[nt] = (uint32_t)user_id;
                tr_m[nt] = movie + nusers;  // :159
                tr_r[nt] = rating(user_id, movie);
            }
            ++nt;
        }
        for (uint32_t i = 0; i < nvalidate; ++i) {  // :163-170
            user_id = (user_id + 2654435761ull) % nusers;
            if (nv < cap) {
                va_u[nv] = (uint32_t)user_id;
                va_m[nv] = movie + nusers;
                va_r[nv] = rating(user_id, movie);
            }
            ++nv;
        }
    }
    *n_train = nt;
    *n_valid = nv;
    return (nt > cap || nv > cap) ? 1 : 0;
}

// Expected knn2 output (out_fin_) for `train_users` users whose items follow the
// same Zipf(s) popularity with E[k^2] = k2_mean: items a, b are linked iff the
// expected number of common raters n_ab = train_users * k2_mean * p_a * p_b
// exceeds 5 (knn2.cpp:142); the weight is the cosine of independent 1..5 ratings
// (E[r]^2 / E[r^2] = 0.9088) plus symmetric noise of sd 0.25/sqrt(n_ab).  Integer
// ratings make knn2's two directions identical, so the matrix is symmetric.
int cfh_synth_graph_model(uint64_t seed, uint32_t n_items, double zipf_s, double train_users,
                          double k2_mean, float* W, int n_threads) {
    std::vector<double> p(n_items);
    double acc = 0;
    for (uint32_t i = 0; i < n_items; ++i) {
        p[i] = std::pow((double)(i + 1), -zipf_s);
        acc += p[i];
    }
    for (auto& x : p) x /= acc;
    const double rho = 12.67 / 13.94;
    parallel_for(n_items, std::max(1, n_threads), [&](uint32_t a, int) {
        float* row = W + (size_t)a * n_items;
        for (uint32_t b = 0; b < n_items; ++b) {
            if (a == b) {
                row[b] = 0.0f;
                continue;
            }
            const double nab = train_users * k2_mean * p[a] * p[b];
            if (nab <= 5.0) {
                row[b] = 0.0f;
                continue;
            }
            const uint32_t lo = std::min(a, b), hi = std::max(a, b);
            const double z = gauss(seed, 9, (uint64_t)lo * n_items + hi);
            double w = rho + 0.25 * z / std::sqrt(nab);
            if (w > 1.0) w = 1.0;
            if (w < 0.011) w = 0.011;
            row[b] = (float)w;
        }
    });
    return 0;
}

// random.seed(seed); x = list(range(n)); random.shuffle(x) -> perm (cf_pyrand.hpp)
void cfh_py_shuffle(uint64_t seed, uint32_t n, uint32_t* perm) {
    std::vector<uint32_t> x(n);
    for (uint32_t i = 0; i < n; ++i) x[i] = i;
    pyrand::MT(seed).shuffle(x);
    for (uint32_t i = 0; i < n; ++i) perm[i] = x[i];
}

}  // extern "C"
