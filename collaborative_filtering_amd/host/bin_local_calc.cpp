// local_calc -- drop-in for local_calc.cpp (a8).
//   :103-117  out_fin_ edges, kept iff the float weight > 0.1 (graph_loader)
//   :119-141  out_test_rat_ vertices with at least one rating
//   :180-208  neigh_program: each vertex's out-neighbour map (a repeated edge keeps the
//             last weight, like the dense upload)
//   :262-526  vertex_program::apply per movie vertex -> cf_local_calc (HIP)
//   :548-558  writer "movie user mse kk" -> out_res_<i>_of_<N>
// Options: --pct P / positional P (percent of vertices, sampled like rand()%100 < P,
// :266; default 100), --seed S (default: time, as the reference :566), --verbosity
// (accepted, ignored), --nshards N.  Movies with up to 191 out-neighbours run on the LDS
// kernels, more on the fp64 spill kernels: no neighbourhood cap, as the reference (a unit's
// n x n blocks and its solver workspace must fit in HBM; CF_ENOMEM otherwise).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <map>
#include <random>

#include "cf_cli.hpp"

int main(int argc, char** argv) {
    int pct = std::stoi(cfcli::opt(argc, argv, "pct", "100"));
    if (argc > 1 && argv[1][0] != '-') pct = std::atoi(argv[1]);   // positional pct (:570)
    const unsigned seed = (unsigned)std::stoul(cfcli::opt(argc, argv, "seed", std::to_string((unsigned)std::time(nullptr))));
    const int nshards = std::stoi(cfcli::opt(argc, argv, "nshards", "4"));

    auto edges = cfio::load_edges(".", "out_fin_");
    for (auto& e : edges) e.w = (double)(float)e.w;   // parsed as float (:110-112)
    cfio::VertexRatings test = cfio::load_vertex_ratings(".", "out_test_rat_", true);

    std::vector<uint32_t> all;
    for (auto& e : edges) {
        all.push_back(e.a);
        all.push_back(e.b);
    }
    for (auto& kv : test) all.push_back(kv.first);
    cfio::IdMap items;
    items.build(all);
    const uint32_t n_items = items.size();

    // out-neighbours (w > 0.1, :113), last duplicate wins, ascending compact id
    std::vector<std::map<uint32_t, double>> nb(n_items);
    for (auto& e : edges) {
        if (!(e.w > 0.1) || e.a == e.b) continue;   // knn output has no self-pairs (knn.cpp:344)
        nb[items.at.at(e.a)][items.at.at(e.b)] = e.w;
    }
    // test ratings CSR over compact ids, users ascending
    std::vector<uint64_t> toff(n_items + 1, 0);
    std::vector<uint32_t> tuser;
    std::vector<float> trat;
    std::vector<std::vector<std::pair<uint32_t, double>>> per(n_items);
    for (auto& kv : test) {
        auto v = kv.second;
        std::sort(v.begin(), v.end());
        per[items.at.at(kv.first)] = std::move(v);
    }
    for (uint32_t i = 0; i < n_items; ++i) {
        for (auto& ur : per[i]) {
            tuser.push_back(ur.first);
            trat.push_back((float)ur.second);
        }
        toff[i + 1] = tuser.size();
    }

    // vertices in ascending id order, sampled like rand() % 100 < pct (:266)
    std::mt19937 rng(seed);
    std::vector<uint32_t> order(n_items);
    for (uint32_t i = 0; i < n_items; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return items.ids[x] < items.ids[y]; });
    std::vector<uint64_t> moff{0};
    std::vector<uint32_t> mitems, units;
    for (uint32_t v : order) {
        if ((unsigned)(rng() % 100) >= (unsigned)pct) continue;
        if (nb[v].size() + 1 < 3 || toff[v + 1] == toff[v]) continue;   // no rows written (:271, :394)
        units.push_back(v);
        mitems.push_back(v);
        for (auto& kv : nb[v]) mitems.push_back(kv.first);
        moff.push_back(mitems.size());
    }

    const uint64_t n_test = toff[n_items];
    std::vector<float> mse(n_test, 0.0f);
    std::vector<int32_t> kk(n_test, 0);
    cf_ctx* ctx = cfcli::open_device();
    cfcli::upload_edges(ctx, items, edges);
    if (!units.empty())
        cfcli::check(ctx, cf_local_calc(ctx, (uint32_t)units.size(), moff.data(), mitems.data(), toff.data(),
                                        tuser.data(), trat.data(), mse.data(), kk.data(), nullptr, nullptr, nullptr),
                     "cf_local_calc");
    cf_destroy(ctx);

    cfio::ShardWriter res(".", "out_res", nshards);
    size_t rows = 0;
    for (uint32_t v : units) {
        const uint32_t movie = items.ids[v];
        std::string& out = res.shard(movie);
        for (uint64_t t = toff[v]; t < toff[v + 1]; ++t) {   // "movie user mse kk" (:552-555)
            cfio::append_u(out, movie);
            out += ' ';
            cfio::append_u(out, tuser[t]);
            out += ' ';
            cfio::append_g(out, (double)mse[t]);
            out += ' ';
            cfio::append_u(out, (uint32_t)kk[t]);
            out += '\n';
            ++rows;
        }
    }
    res.flush();
    std::printf("Processed %zu movie vertices, wrote %zu predictions to out_res_*\n", units.size(), rows);
    return 0;
}
