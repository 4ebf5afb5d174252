// local_calc_precomp -- drop-in for local_calc_precomp.cpp (a6, a7).
//   :406-482 load_precomputed_data("out_eigen_") incl. the accumulating sigs_min
//            vector (:414,437,440): user n sees the concatenation of every record's
//            sigs up to its own, so w_lim for row r is the r-th sig of the whole file
//   :122-136 out_fin_ edges (out-neighbour iff float weight > 0.1)
//   :138-160 out_test_rat_ vertices
//   :217-380 neigh_program::apply per test rating of the sampled movies (:221)
//            -> cf_predict_precomp_sel (HIP, fp64)
//   :393-404 writer "movie user mse kk" -> out_res_<i>_of_<N>
// Options: --pct P (percent of movie vertices, sampled like rand()%100 < P; default
// 100), --seed S (default: time, as the reference), --compat ref|fixed (fixed = each
// user's own sigs), --verbosity (accepted, ignored), --nshards N, --devices N (users range-split
// over N GPU contexts, cf_predict_precomp_multi; out_res_ identical to one device).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <ctime>
#include <map>
#include <random>

#include "cf_cli.hpp"

int main(int argc, char** argv) {
    int pct = std::stoi(cfcli::opt(argc, argv, "pct", "100"));
    if (argc > 1 && argv[1][0] != '-') pct = std::atoi(argv[1]);   // positional pct (:495)
    const std::string compat = cfcli::opt(argc, argv, "compat", "ref");
    const unsigned seed = (unsigned)std::stoul(cfcli::opt(argc, argv, "seed", std::to_string((unsigned)std::time(nullptr))));
    const int nshards = std::stoi(cfcli::opt(argc, argv, "nshards", "4"));
    const std::string eig_path = cfcli::opt(argc, argv, "eigen", "out_eigen_");

    // text (parsed on --threads threads, default all) or the binary form, detected by its magic,
    // mapped and parsed straight into flat arrays (cfio::load_eigen_flat)
    const cfio::EigenFlat recs = cfio::load_eigen_flat(eig_path, std::stoi(cfcli::opt(argc, argv, "threads", "0")));
    std::printf("Loaded %zu test users\n", recs.size());
    auto edges = cfio::load_edges(".", "out_fin_");
    for (auto& e : edges) e.w = (double)(float)e.w;   // parsed as float (:129)
    cfio::VertexRatings test = cfio::load_vertex_ratings(".", "out_test_rat_", true);

    std::vector<uint32_t> all;
    for (auto& e : edges) {
        all.push_back(e.a);
        all.push_back(e.b);
    }
    for (auto& kv : test) all.push_back(kv.first);
    all.insert(all.end(), recs.movies.begin(), recs.movies.end());
    cfio::IdMap items;
    items.build(all);

    // user -> (movie -> test rating), for the rating vectors of the blocks
    std::unordered_map<uint32_t, std::unordered_map<uint32_t, double>> urat;
    for (auto& kv : test)
        for (auto& ur : kv.second) urat[ur.first][kv.first] = ur.second;

    const uint32_t n_users = (uint32_t)recs.size();
    // the flat record arrays ARE the predictor's inputs: rows at recs.off, blocks at
    // recs.evec_off, and the compat table = every record's sigs in file order (recs.sigs);
    // only the compact ids, ratings and the k-slot eigenvalues are built here
    const std::vector<uint64_t>& off = recs.off;
    std::vector<uint64_t> eoff(recs.evec_off.begin(), recs.evec_off.end() - 1);
    const std::vector<int32_t>& m = recs.m;
    const double* sig_tab = recs.sigs.data();   // own sigs at off[u] == the compat concatenation
    std::vector<uint32_t> its(off.back());
    std::vector<float> rats(off.back());
    std::vector<double> evals(off.back(), 0.0);
    std::unordered_map<uint32_t, uint32_t> rec_of_user;
    for (uint32_t u = 0; u < n_users; ++u) {
        const uint64_t k = off[u + 1] - off[u];
        rec_of_user[recs.user[u]] = u;   // a later record of the same user replaces it (:472)
        auto& ur = urat[recs.user[u]];
        const uint64_t nm = recs.eval_off[u + 1] - recs.eval_off[u];
        for (uint64_t j = 0; j < k; ++j) {
            const uint32_t mv = recs.movies[off[u] + j];
            its[off[u] + j] = items.at[mv];
            auto it = ur.find(mv);
            rats[off[u] + j] = it == ur.end() ? 0.0f : (float)it->second;   // operator[] default 0 (:259)
            evals[off[u] + j] = j < nm ? recs.evals[recs.eval_off[u] + j] : 0.0;
        }
    }
    // text records carry fp64 blocks, the binary form its fp32 blocks as they are (the _f32 entry
    // points: same predictions as the widened values)
    const bool f32 = recs.binary;
    std::vector<double> evecs_pad;
    std::vector<float> evecs_pad32;
    const double* evecs_p = recs.evecs.data();
    const float* evecs_p32 = recs.evecs_f32.data();
    if (recs.evecs.empty()) {
        evecs_pad.assign(1, 0.0);
        evecs_p = evecs_pad.data();
    }
    if (recs.evecs_f32.empty()) {
        evecs_pad32.assign(1, 0.0f);
        evecs_p32 = evecs_pad32.data();
    }
    // movie vertices sampled like rand() % 100 < pct in apply (:221), BEFORE prediction:
    // only the rows of sampled movies are predicted (cf_predict_precomp_sel)
    std::mt19937 rng(seed);
    std::map<uint32_t, std::vector<std::pair<uint32_t, double>>> movies(test.begin(), test.end());
    std::unordered_map<uint32_t, bool> sampled;
    for (auto& kv : movies) sampled[kv.first] = (unsigned)(rng() % 100) < (unsigned)pct;
    std::vector<uint8_t> sel(its.size(), 0);
    {
        size_t e = 0;
        for (uint32_t u = 0; u < n_users; ++u)
            for (uint64_t j = off[u]; j < off[u + 1]; ++j) {
                const uint32_t mv = recs.movies[j];
                auto it = sampled.find(mv);
                sel[e++] = it != sampled.end() && it->second;
            }
    }
    const bool ref = compat != "fixed";
    std::vector<float> mse(its.size(), std::numeric_limits<float>::quiet_NaN());
    std::vector<int32_t> kk(its.size(), 0);
    // --devices N (or CF_DEVICES): the users range-split by k^3 over N contexts, GPU (i % visible)
    // each -- the reference's ranks each hold the whole out_eigen_ (:485-486, 509) -- with the
    // global compat table on every context, so out_res_ is identical to the one-device run's
    const char* env_dev = std::getenv("CF_DEVICES");
    const int n_dev = std::max(1, std::atoi(cfcli::opt(argc, argv, "devices", env_dev ? env_dev : "1").c_str()));
    const double* tab = sig_tab;          // both modes read the same flat array (CF_SIGS_COMPAT by row,
    const uint64_t tab_len = off.back();  // CF_SIGS_OWN at off[u] + row)
    const int mode = ref ? CF_SIGS_COMPAT : CF_SIGS_OWN;
    const uint8_t* rsel = pct >= 100 ? nullptr : sel.data();
    if (n_dev == 1) {
        cf_ctx* ctx = cfcli::open_device();
        cfcli::upload_edges(ctx, items, edges);
        if (n_users && f32)
            cfcli::check(ctx, cf_predict_precomp_sel_f32(ctx, n_users, off.data(), its.data(), rats.data(), m.data(),
                                                         evals.data(), eoff.data(), evecs_p32, tab, tab_len, mode,
                                                         rsel, mse.data(), kk.data(), nullptr),
                         "cf_predict_precomp_sel_f32");
        else if (n_users)
            cfcli::check(ctx, cf_predict_precomp_sel(ctx, n_users, off.data(), its.data(), rats.data(), m.data(),
                                                     evals.data(), eoff.data(), evecs_p, tab, tab_len, mode,
                                                     rsel, mse.data(), kk.data(), nullptr),
                         "cf_predict_precomp_sel");
        cf_destroy(ctx);
    } else {
        const int visible = cf_device_count();
        if (visible <= 0) cfcli::die("no usable MI355X device");
        const char* dev0 = std::getenv("CF_DEVICE");
        const int base = dev0 ? std::atoi(dev0) : 0;
        std::vector<cf_ctx*> ctxs(n_dev, nullptr);
        for (int d = 0; d < n_dev; ++d) {
            if (cf_create((base + d) % visible, &ctxs[d]) != CF_OK) cfcli::die("cf_create failed");
            cfcli::upload_edges(ctxs[d], items, edges);
        }
        std::vector<uint32_t> split(n_dev + 1);
        if (n_users && f32)
            cfcli::check(ctxs[0], cf_predict_precomp_multi_f32(ctxs.data(), n_dev, n_users, off.data(), its.data(),
                                                               rats.data(), m.data(), evals.data(), eoff.data(),
                                                               evecs_p32, tab, tab_len, mode, rsel, mse.data(),
                                                               kk.data(), nullptr, split.data()),
                         "cf_predict_precomp_multi_f32");
        else if (n_users)
            cfcli::check(ctxs[0], cf_predict_precomp_multi(ctxs.data(), n_dev, n_users, off.data(), its.data(),
                                                           rats.data(), m.data(), evals.data(), eoff.data(),
                                                           evecs_p, tab, tab_len, mode, rsel, mse.data(),
                                                           kk.data(), nullptr, split.data()),
                         "cf_predict_precomp_multi");
        for (int d = 0; d < n_dev; ++d)
            std::printf("device part %d: users %u..%u on GPU %d\n", d, split[d], split[d + 1], (base + d) % visible);
        for (auto* c : ctxs) cf_destroy(c);
    }

    // rows per test movie vertex (:230-361), sampled per vertex (:221)
    cfio::ShardWriter res(".", "out_res", nshards);
    size_t rows = 0, missing = 0;
    for (auto& kv : movies) {
        if (!sampled[kv.first]) continue;
        const uint32_t movie = kv.first;
        std::string& out = res.shard(movie);
        for (auto& ur : kv.second) {
            float e = std::numeric_limits<float>::quiet_NaN();
            int32_t c = 0;
            auto ri = rec_of_user.find(ur.first);
            if (ri != rec_of_user.end()) {
                const uint32_t r = ri->second;
                for (uint64_t j = off[r]; j < off[r + 1]; ++j)
                    if (recs.movies[j] == movie) {
                        e = mse[j];
                        c = kk[j];
                        break;
                    }
            }
            if (c == 0 && std::isnan(e)) ++missing;
            cfio::append_u(out, movie);   // "movie user mse kk" (:397-399)
            out += ' ';
            cfio::append_u(out, ur.first);
            out += ' ';
            cfio::append_g(out, (double)e);
            out += ' ';
            cfio::append_u(out, (uint32_t)c);
            out += '\n';
            ++rows;
        }
    }
    res.flush();
    std::printf("Wrote %zu predictions (%zu without a connected item) to out_res_*\n", rows, missing);
    return 0;
}
